#!/bin/bash
# Interleaved whole-step comparison of several bench.py argument sets (GPU box):
#   bash tools/args_multi.sh ROUNDS "" "--dp-exchange" ...   ("-" = no extra arguments)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R=$1; shift
for r in $(seq 1 $R); do
  k=0
  for v in "$@"; do
    k=$((k+1))
    a=$v; [ "$v" = "-" ] && a=""
    # leading VAR=value words go to the environment
    e=""; while [[ "$a" =~ ^([A-Z_0-9]+=[^ ]*)\ ?(.*)$ ]]; do e="$e ${BASH_REMATCH[1]}"; a="${BASH_REMATCH[2]}"; done
    env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off $a \
      > gpurun_out/am_${k}_$r.json 2> gpurun_out/am_${k}_$r.err || { echo "bench [$v] failed"; tail -5 gpurun_out/am_${k}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/am_${k}_$r.json').read().strip().splitlines()[-1]); print('[$v] round $r', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('dp_exchange'))"
  done
done
