#!/bin/bash
# GPU box: conv_hr tile choices for the 512^2 / 1024^2 sign-bit and one-chunk convs
# (PG_HR_TILE / PG_HR_TILE_XB overrides; kbench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
K="timeout -k 10 120 python tools/kbench.py --iters 20"
echo "== 512^2 32->64 pool (one chunk): tiles 3 6 12 14"
for t in 3 6 12 14; do PG_KG=0 PG_HR_TILE=$t $K c:512:32:64:22 c:512:32:64:16 || exit $?; done
echo "== default"
PG_KG=0 $K c:512:32:64:150 c:512:32:64:280 c:512:64:32:521 c:1024:32:16:521 c:1024:16:32:150 c:1024:16:32:280 c:512:32:32:0 c:512:32:32:8 || exit $?
echo "== XB tile 16 / 5"
for t in 16 5; do PG_KG=0 PG_HR_TILE_XB=$t $K c:512:64:32:521 || exit $?; done
