#!/bin/bash
# Interleaved whole-step comparison of several environments (GPU box):
#   bash tools/env_multi.sh ROUNDS "A=1" "A=2 B=3" ...   ("-" = the defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  k=0
  for v in "$@"; do
    k=$((k+1))
    e=$v; [ "$v" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off \
      > gpurun_out/em_${k}_$r.json 2> gpurun_out/em_${k}_$r.err || { echo "bench [$v] failed"; tail -5 gpurun_out/em_${k}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/em_${k}_$r.json').read().strip().splitlines()[-1]); print('[$v] round $r', d['value'], d['ms_per_step'])"
  done
done
