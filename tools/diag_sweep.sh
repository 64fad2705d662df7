#!/bin/bash
# conv_hr LDS-DMA timing diagnostics (wrong results): PG_HR_DIAG 1 = no halo DMA, 2 = no weight
# DMA, 4 = no epilogue; GPU box.   DG_VALS="0 1 2 4" DG_SPECS="c:128:128:128:0 ..." bash tools/diag_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${DG_VALS:-0 1 2 3 4}; do
  echo "== diag $v"
  PG_HR_DIAG=$v timeout -k 10 120 python tools/kbench.py --iters 20 $DG_SPECS 2>&1 | grep -v amdgpu || exit 1
done
