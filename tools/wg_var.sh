#!/bin/bash
# Wide weight-gradient variants (prefetch depth, waves/SIMD, target workgroups), interleaved
# in one GPU call: min over rounds per (variant, spec).  Log: gpurun_out/wg_var.log
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S=${WG_SPECS:-"w:256:64:128:0 w:128:128:256:0 w:64:256:512:0 w:128:128:128:0 w:64:256:256:0 w:32:512:512:0 w:256:64:64:0"}
for i in 1 2; do
  for v in "4,1:256" "2,1:256" "2,2:512" "1,2:512" "2,2:256"; do
    PG_WG_VARIANT=${v%%:*} PG_WG_TARGET=${v##*:} timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done > gpurun_out/wg_var.log
python - <<'PY'
import collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/wg_var.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        d[f[1]][f[0]].append(float(f[2]))
for spec, v in d.items():
    print(f"{spec:22s} " + "  ".join(f"{k} {min(x):6.1f}" for k, x in v.items()))
PY
