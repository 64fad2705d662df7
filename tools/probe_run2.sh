#!/bin/bash
# GPU box: k-loop probe (small wave tiles) + per-shape isolated conv / wgrad times of the
# current build (bench.py PG_BENCH_SHAPES).  Logs under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kloop_probe > gpurun_out/kloop_probe2.log 2>&1; rc=$?
echo "kloop_probe rc=$rc"; cat gpurun_out/kloop_probe2.log; [ $rc -eq 0 ] || exit $rc
PG_BENCH_SHAPES=gpurun_out/shapes_r4.json timeout -k 10 300 python bench.py --steps 3 --warmup 2 \
  --cpu-baseline off > gpurun_out/shapes_r4.log 2>&1; rc=$?
echo "shapes rc=$rc"; tail -n 2 gpurun_out/shapes_r4.log | cut -c1-300
