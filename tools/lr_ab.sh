# A/B of the low-resolution conv kernel (conv_lr.inc) against the split-K conv3x3 path
# (PG_CONV_LR=0) at the 4^2-16^2 shapes of the step; writes gpurun_out/lr_ab.log
S="${LR_SPECS:-c:16:512:512:6 c:16:512:512:8 c:16:512:512:0 c:16:512:512:22 c:8:512:512:6 c:8:512:512:8 c:8:512:512:22 c:8:512:512:16 c:4:512:512:6 c:4:512:512:0 c:4:513:512:6 c:16:512:512:7}"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/lr_ab.log
: > $out
for r in 1 2; do
  echo "== conv_lr (PG_CONV_LR=2: 4^2-16^2)" >> $out
  PG_CONV_LR=2 timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || exit 1
  echo "== split-K (PG_CONV_LR=0)" >> $out
  PG_CONV_LR=0 timeout -k 10 120 python tools/kbench.py $S >> $out 2>&1 || exit 1
done
echo done
