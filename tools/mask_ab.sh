#!/bin/bash
# Branch-free lrelu' bit mask (lrelu_mask_bf16x8): sign-bit op tests, then kbench A/B of the
# X_BITS convs and GZ_BITS weight gradients (ab/lib_A.so old, ab/lib_B.so new)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "sign_bit or wgrad" --timeout 300 --timeout-method thread > gpurun_out/ops.log 2>&1; rc=$?; tail -3 gpurun_out/ops.log; [ $rc -eq 0 ] || exit $rc
LAB_SPECS="c:1024:32:16:521 c:512:64:32:521 w:1024:16:32:2 w:512:32:64:2" timeout -k 10 600 bash tools/lib_ab.sh 3
