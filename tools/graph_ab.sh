# A/B in one GPU call: graph-replayed vs eager steps (PG_GRAPH) and the CLR graph knobs
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off --no-kernel-events > gpurun_out/gab_$n.json 2> gpurun_out/gab_$n.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/gab_$n.json')); print('$n', d['value'], d['ms_per_step'], 'host', d['host_enqueue_ms_per_step'], 'replays', d['graph_replayed_steps'])"
}
run eager PG_GRAPH=0
run graph PG_GRAPH=1
run graph_nopkt PG_GRAPH=1 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run graph_q2 PG_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2
run graph_q8 PG_GRAPH=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=8
run eager2 PG_GRAPH=0
run graph2 PG_GRAPH=1
