#!/bin/bash
# The committed --dp-exchange lines (GPU box): plain step, the DP bookkeeping at one rank with the
# default schedule (at one rank: the G exchange waited at the step start), and with the G
# exchange overlapped into the next step (the default across ranks); interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in plain dpx dpx_ovl; do
    case $v in
      plain) args=""; envs="" ;;
      dpx) args="--dp-exchange"; envs="" ;;
      dpx_ovl) args="--dp-exchange"; envs="PG_ENGINE=overlap_g_exchange=1" ;;
    esac
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off \
      --no-kernel-events $args > gpurun_out/dpl_${v}_$i.json 2> gpurun_out/dpl_${v}_$i.err \
      || { echo "$v failed"; tail -3 gpurun_out/dpl_${v}_$i.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/dpl_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], 'host', d.get('host_enqueue_ms_per_step'), d.get('launch_path'), d.get('dp_exchange'))"
  done
done
