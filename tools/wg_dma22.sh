#!/bin/bash
# (2,2) / (1,1) narrow weight gradients on the DMA kernel with their own split targets:
# op tests, kbench A/B against the wide-only DMA routing, whole-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k wgrad --timeout 300 --timeout-method thread > gpurun_out/ops.log 2>&1; rc=$?; tail -3 gpurun_out/ops.log; [ $rc -eq 0 ] || exit $rc
ENV_AB=PG_WG_DMA AB_VALS="1 2" AB_SPECS="w:512:32:32:0 w:512:64:32:1 w:1024:16:16:0 w:1024:16:32:0 w:1024:32:16:1 w:256:64:64:0" timeout -k 10 600 bash tools/env_ab.sh 2 || exit 1
timeout -k 10 900 bash tools/ab_env.sh 2 "c:PG_WG_DMA=1" "c:PG_WG_DMA=2"
