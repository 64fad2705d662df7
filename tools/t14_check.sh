#!/bin/bash
# GPU box: tile 14 EF for the 512^2 32 -> 64 sign-bit convs: op tests + kbench A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  -k "sign_bit" > gpurun_out/t14_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 3 gpurun_out/t14_tests.log; [ $rc -eq 0 ] || exit $rc
for on in 0 1 0 1; do
  echo "== PG_HR_T14EF=$on"
  PG_HR_T14EF=$on timeout -k 10 120 python tools/kbench.py --iters 30 c:512:32:64:150 c:512:32:64:280 || exit $?
done
