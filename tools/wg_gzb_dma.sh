#!/bin/bash
# Sign-bit (GZ_BITS) weight gradients on the LDS-DMA kernel: the sign-bit op test, kbench A/B
# against the register kernel (PG_WG_DMA_GZB=0), whole-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "sign_bit or wgrad" --timeout 300 --timeout-method thread > gpurun_out/ops.log 2>&1; rc=$?; tail -3 gpurun_out/ops.log; [ $rc -eq 0 ] || exit $rc
ENV_AB=PG_WG_DMA_GZB AB_VALS="0 1" AB_SPECS="w:1024:16:32:2 w:512:32:64:2 w:256:16:32:2" timeout -k 10 600 bash tools/env_ab.sh 2 || exit 1
timeout -k 10 900 bash tools/ab_env.sh 2 "d:PG_WG_DMA_GZB=0" "d:PG_WG_DMA_GZB=1"
