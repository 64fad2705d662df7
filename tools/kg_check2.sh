#!/bin/bash
# GPU box: conv_kg op tests, then kbench PG_KG=0 (conv_hr) / 1 (default choice) / 2 (every
# eligible shape) at 64^2-512^2.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  -k "conv_kg or conv3x3_fwd" > gpurun_out/kg_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/kg_tests.log; [ $rc -eq 0 ] || exit $rc
S="c:64:256:256:0 c:64:256:512:22 c:256:64:64:0 c:256:64:64:6 c:256:64:128:22 c:256:64:64:8 c:256:64:64:70 \
   c:256:64:128:8 c:512:32:64:22 c:512:32:64:0 c:128:128:128:0"
for kg in 0 1 2; do
  echo "== PG_KG=$kg"
  PG_KG=$kg timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
done
