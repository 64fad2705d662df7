#!/bin/bash
# Interleaved A/B of one environment switch on kbench specs, in one GPU call:
#   ENV_AB="PG_HR_DMA" [AB_VALS="0 1"] AB_SPECS="c:128:128:128:6 ..." bash tools/env_ab.sh [rounds]
# (value A vs B, default 0 vs 1; min over rounds).  Log: gpurun_out/env_ab.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
r=${1:-2}
for i in $(seq "$r"); do
  for v in ${AB_VALS:-0 1}; do
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
    (ka, a), (kb, b) = [(k, min(x)) for k, x in v.items()][:2]
    print(f"{spec:24s} {ka}: {a:8.1f}  {kb}: {b:8.1f}  {kb}/{ka} {b / a:6.3f}")
PY
