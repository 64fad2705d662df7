#!/bin/bash
# GPU box: the k-loop probe + the live wide conv tiles in kbench with and without their
# staging / epilogue (PG_HR_DIAG), for the round-4 wide-conv work.  Logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kloop_probe > gpurun_out/kloop_probe.log 2>&1; rc=$?
echo "kloop_probe rc=$rc"; cat gpurun_out/kloop_probe.log; [ $rc -eq 0 ] || exit $rc
S="c:128:128:128:0 c:64:256:256:0 c:256:64:64:0 c:32:512:512:0 c:64:512:256:1"
for dg in 0 7 4; do
  echo "== PG_HR_DIAG=$dg"
  PG_HR_DIAG=$dg timeout -k 10 120 python tools/kbench.py --iters 20 $S; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
