#!/bin/bash
# GPU box: the K-grouped wide conv (conv_kg.hip): op tests, then kbench with it on and off
# (PG_KG), then a short whole-step bench A/B.  Stops at the first step that fails.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 120 --timeout-method thread \
  -k "conv_kg or conv3x3_fwd" > gpurun_out/kg_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -n 5 gpurun_out/kg_tests.log; [ $rc -eq 0 ] || exit $rc
S="c:32:512:512:0 c:32:512:512:6 c:32:512:512:8 c:64:256:256:0 c:64:512:256:8 c:64:256:512:22 \
   c:128:128:128:0 c:128:256:128:8 c:128:128:256:22 c:256:64:64:0 c:256:128:64:8 c:256:64:128:22 c:256:128:64:71"
for kg in 0 1; do
  echo "== PG_KG=$kg"
  PG_KG=$kg timeout -k 10 120 python tools/kbench.py --iters 30 $S || exit $?
done
for kg in 0 1 0 1; do
  PG_KG=$kg timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-baseline off > gpurun_out/kg_bench_$kg.log 2>&1 || exit $?
  echo "bench PG_KG=$kg: $(tail -n 1 gpurun_out/kg_bench_$kg.log | cut -c1-220)"
done
