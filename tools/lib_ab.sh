#!/bin/bash
# kbench A/B of two library builds (ab/lib_A.so vs ab/lib_B.so), interleaved rounds; GPU box.
#   LAB_SPECS="c:128:128:128:0 ..." bash tools/lib_ab.sh [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
r=${1:-2}
for i in $(seq "$r"); do
  for v in A B; do
    timeout -k 10 120 python tools/kbench.py --lib ab/lib_$v.so $LAB_SPECS 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done > gpurun_out/lib_ab.log
python - <<'PY'
import collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/lib_ab.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        d[f[1]][f[0]].append(float(f[2]))
for spec, v in d.items():
    a, b = min(v["A"]), min(v["B"])
    print(f"{spec:24s} A: {a:8.1f}  B: {b:8.1f}  B/A {b / a:6.3f}")
PY
