#!/bin/bash
# X_BITS input-gradient conv at 512^2 (64 -> 32, UPS_IN | MASK): tile 8 (default) vs 16 vs 5;
# ring depth of the persistent forms
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "PG_HR_TILE_XB=-1" "PG_HR_TILE_XB=16" "PG_HR_TILE_XB=16 PG_HR_PD=2" "PG_HR_TILE_XB=-1 PG_HR_EF_PD=2"; do
  echo "== $v"
  env $v timeout -k 10 120 python tools/kbench.py --iters 30 c:512:64:32:521 c:1024:32:16:521 c:512:64:32:9 2>&1 | grep -v amdgpu || exit 1
done
