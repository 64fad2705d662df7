# A/B of the double-buffered wide conv tile (PG_HR_TILE=12) against the default tiles
# at the 64^2-256^2 wide conv shapes (GPU box); writes gpurun_out/hrdb.log
S="${HR_SPECS:-c:256:64:128:22 c:256:128:64:8 c:256:64:64:6 c:128:256:128:8 c:128:128:256:22 c:128:128:128:6 c:64:512:256:8 c:64:256:512:22 c:64:256:256:6 c:32:512:512:6}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/hrdb.log
: > $out
for r in 1 2; do
  echo "== default" >> $out
  timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || exit 1
  for t in ${HR_TILES:-12 6}; do
    echo "== tile $t" >> $out
    PG_HR_TILE=$t timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || { echo "fail $t" >> $out; exit 1; }
  done
done
echo done
