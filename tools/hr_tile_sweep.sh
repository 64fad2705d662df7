# conv_hr tile sweep at the mid-resolution conv shapes (GPU box): PG_HR_TILE = 0..8
S="${HR_SPECS:-c:256:64:128:22 c:256:128:64:8 c:256:64:64:6 c:128:256:128:8 c:128:128:256:22 c:128:128:128:6 c:64:512:256:8 c:64:256:512:22 c:64:256:256:6}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/hrtile.log
: > $out
echo "== default" >> $out
timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || exit 1
for t in ${HR_TILES:-3 6}; do
  echo "== tile $t" >> $out
  PG_HR_TILE=$t timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || echo "fail $t" >> $out
done
echo done
