#!/bin/bash
# kbench of conv specs under forced conv_hr tiles (PG_HR_TILE), GPU box:
#   SW_TILES="3 6 13" SW_SPECS="c:512:32:64:16 ..." bash tools/tile_sweep.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for t in ${SW_TILES:-3 6 13}; do
  echo "== tile $t"
  PG_HR_TILE=$t timeout -k 10 120 python tools/kbench.py --iters 20 $SW_SPECS 2>&1 | grep -v amdgpu || exit 1
done
