#!/bin/bash
# GPU box: the wide LDS-DMA conv tiles with parts of their work switched off (PG_HR_DIAG:
# 1 no halo DMA, 2 no weight DMA, 4 no epilogue; wrong results, timing only) and with the
# XCD remap off, at the 32^2 / 64^2 / 128^2 / 256^2 shapes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="c:32:512:512:0 c:32:512:512:8 c:64:256:256:0 c:64:512:256:8 c:128:128:128:0 c:256:64:64:0 c:256:128:64:8"
for dg in 0 1 2 3 4 7; do
  echo "== PG_HR_DIAG=$dg"
  PG_HR_DIAG=$dg timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
done
echo "== PG_HR_XCD=0"
PG_HR_XCD=0 timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
