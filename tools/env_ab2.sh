#!/bin/bash
# Interleaved whole-step A/B of one environment switch (GPU box):
#   AB_VAR=PG_SIDE_WGRAD AB_A=0 AB_B=1 bash tools/env_ab2.sh [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 ${1:-2}); do
  for v in "$AB_A" "$AB_B"; do
    env "$AB_VAR=$v" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > gpurun_out/ab_${v}_$r.json 2> gpurun_out/ab_${v}_$r.err || { echo "bench $v failed"; tail -5 gpurun_out/ab_${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$r.json').read().strip().splitlines()[-1]); print('$AB_VAR=$v round $r', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'])"
  done
done
