#!/bin/bash
# Interleaved A/B of one environment switch on kbench specs, in one GPU call:
#   ENV_AB="PG_HR_DMA" AB_SPECS="c:128:128:128:6 ..." bash tools/env_ab.sh [rounds]
# (value 0 vs 1; min over rounds).  Log: gpurun_out/env_ab.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
r=${1:-2}
for i in $(seq "$r"); do
  for v in 0 1; do
    env $ENV_AB=$v timeout -k 10 120 python tools/kbench.py $AB_SPECS 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done > gpurun_out/env_ab.log
python - <<'PY'
import collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/env_ab.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        d[f[1]][f[0]].append(float(f[2]))
for spec, v in d.items():
    a, b = min(v["0"]), min(v["1"])
    print(f"{spec:24s} 0: {a:8.1f}  1: {b:8.1f}  1/0 {b / a:6.3f}")
PY
