set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
for v in "plain4::4" "plain16::16" "dpx16:--dp-exchange:16" "dpx8:--dp-exchange:8"; do
  name=${v%%:*}; rest=${v#*:}; a=${rest%%:*}; q=${rest#*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events $a > gpurun_out/q.json 2> gpurun_out/q.err || { echo "$name failed"; tail -3 gpurun_out/q.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/q.json').read().strip().splitlines()[-1]); print('$name', d['value'], d['ms_per_step'], 'host', d.get('host_enqueue_ms_per_step'))"
done; done
