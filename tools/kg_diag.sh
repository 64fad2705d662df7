#!/bin/bash
# GPU box: conv_kg with parts switched off (PG_KG_DIAG: 1 no staging DMA, 4 no epilogue; timing
# only) next to conv_hr's (PG_HR_DIAG: 3 no DMA, 4 no epilogue), at the wide shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="c:32:512:512:0 c:64:256:256:0 c:128:128:128:0 c:256:64:64:0 c:256:128:64:8"
for dg in 0 1 4 5; do
  echo "== conv_kg PG_KG_DIAG=$dg"
  PG_KG_DIAG=$dg timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
done
for dg in 0 3 4 7; do
  echo "== conv_hr PG_HR_DIAG=$dg"
  PG_KG=0 PG_HR_DIAG=$dg timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
done
