#!/bin/bash
# A/B of the XCD-aware workgroup order (PG_WG_XCD / PG_CONV_XCD = 0 vs 1) on the bench's
# wide weight-gradient and low-resolution conv shapes, interleaved in one GPU call, plus
# FETCH_SIZE of one wgrad launch each way.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
S="w:256:64:128:0 w:128:128:256:0 w:64:256:512:0 w:128:128:128:0 w:64:256:256:0 w:32:512:512:0 w:16:512:512:0 w:8:512:512:0 c:32:512:512:8 c:16:512:512:8 c:8:512:512:8 c:4:512:512:6 c:64:512:256:8"
for i in 1 2; do
  for v in 0 1; do
    PG_WG_XCD=$v PG_CONV_XCD=$v timeout -k 10 120 python tools/kbench.py $S 2>&1 | grep -v amdgpu | sed "s/^/$v /" || exit 1
  done
done > gpurun_out/xcd_ab.log
python - <<'PY'
import collections
d = collections.defaultdict(lambda: collections.defaultdict(list))
for l in open("gpurun_out/xcd_ab.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        d[f[1]][f[0]].append(float(f[2]))
for spec, v in d.items():
    a, b = min(v["0"]), min(v["1"])
    print(f"{spec:24s} off {a:8.1f}  on {b:8.1f}  on/off {b / a:6.3f}")
PY
ROOT=$(pwd); export TMPDIR=/tmp
for v in 0 1; do
  ( cd /tmp && PG_WG_XCD=$v PG_CONV_XCD=$v timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d "$ROOT/gpurun_out/xcd_pmc_$v" -o run -- python "$ROOT/tools/kbench.py" --iters 2 w:128:128:256:0 c:32:512:512:8 ) \
      > gpurun_out/xcd_pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo xcd_ab done
