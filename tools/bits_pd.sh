# GPU box: the sign-bit / PixelNorm persistent variants at ring depth 1 vs 2 (kbench)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:1024:32:16:521 c:1024:16:32:150 c:1024:16:32:280 c:1024:16:16:70 c:1024:32:16:71 c:1024:16:16:2048 c:512:32:32:2048 c:512:32:32:70 c:512:64:32:521 c:512:32:64:150"
for v in "PG_HR_EF_PD=1" "PG_HR_EF_PD=2" "PG_HR_EF=0"; do
  echo "== $v" >> gpurun_out/bpd.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/bpd.txt 2>&1 || exit 1
done
