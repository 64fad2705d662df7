#!/bin/bash
# A/B kernel timing of ab/lib_A.so vs ab/lib_B.so in one GPU call, interleaved rounds.
#   AB_SPECS="w:256:64:128:0 ..." tools/ab_run.sh [rounds]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
r=${1:-3}
for i in $(seq "$r"); do
  for v in A B; do
    timeout -k 10 120 python tools/kbench.py --lib ab/lib_$v.so $AB_SPECS 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done > gpurun_out/ab.log
python - <<'PY'
import collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/ab.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        d[f[1]][f[0]].append(float(f[2]))
for spec, v in d.items():
    a, b = min(v["A"]), min(v["B"])
    print(f"{spec:24s} A {a:8.1f}  B {b:8.1f}  B/A {b / a:6.3f}")
PY
