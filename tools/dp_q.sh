#!/bin/bash
# Hardware-queue count vs the DP bookkeeping at one rank, C++ replay (GPU box), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in plain_q4 plain_q16 dpx_q16 dpx_q8; do
    case $v in
      plain_q4) args=""; q=4 ;;
      plain_q16) args=""; q=16 ;;
      dpx_q16) args="--dp-exchange"; q=16 ;;
      dpx_q8) args="--dp-exchange"; q=8 ;;
    esac
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off \
      --no-kernel-events $args > gpurun_out/dpq.json 2> gpurun_out/dpq.err \
      || { echo "$v failed"; tail -3 gpurun_out/dpq.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/dpq.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
  done
done
