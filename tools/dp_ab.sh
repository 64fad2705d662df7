#!/bin/bash
# Interleaved whole-step A/B of the DP bookkeeping at one rank (GPU box):
#   plain    the default step (C++ replay), 4 hardware queues
#   dpx      --dp-exchange: the bucketed exchange over a one-rank RCCL group, 16 queues, C++
#            replay with the collectives recorded between launch segments
#   dpx_sync --dp-exchange, the G exchange waited for before the next step (no B2 reorder)
#   dpx_eager --dp-exchange enqueued from Python every step
#   dpx_b64  --dp-exchange with 64 MiB buckets
# 10 timed steps after 3 warm-up, ROUNDS rounds.  Log: gpurun_out/dp_ab.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=${ROUNDS:-2}
: > gpurun_out/dp_ab.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events \
    $ARGS > gpurun_out/dp_ab.json 2> gpurun_out/dp_ab.err
  local rc=$?
  [ $rc -eq 0 ] || { echo "bench $name failed"; tail -5 gpurun_out/dp_ab.err; exit $rc; }
  python -c "import json; d=json.loads(open('gpurun_out/dp_ab.json').read().strip().splitlines()[-1]); print('$name', d['value'], 'img/s', d['ms_per_step'], 'ms/step host', d.get('host_enqueue_ms_per_step'), d.get('launch_path'))" | tee -a gpurun_out/dp_ab.log
}
for i in $(seq "$rounds"); do
  ARGS="" run plain GPU_MAX_HW_QUEUES=4
  ARGS="--dp-exchange" run dpx GPU_MAX_HW_QUEUES=16
  ARGS="--dp-exchange" run dpx_sync GPU_MAX_HW_QUEUES=16 PG_ENGINE=overlap_g_exchange=0
  ARGS="--dp-exchange --dp-bucket-mb 64" run dpx_b64 GPU_MAX_HW_QUEUES=16
done
