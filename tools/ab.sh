#!/bin/bash
# Interleaved A/B timing in one GPU call (GPU box).
#
#   tools/ab.sh [-r ROUNDS] [-k "KBENCH SPECS"] VARIANT [VARIANT ...]
#   VARIANT = "name:ENV=a ENV2=b"       environment switches (the library's PG_* knobs)
#           | "name:lib=ab/lib_X.so"    a library built by tools/ab_build.sh
#
# With -k every variant runs tools/kbench.py on the specs (printed: the minimum over rounds per
# spec and variant); without it a whole-step bench.py (10 timed steps after 3 warm-up, no CPU
# baseline, extra bench arguments from $AB_ARGS; printed: img/s and ms/step per round).
# Variants alternate within each round.
# Logs: gpurun_out/ab.log.  Replaces the round-2/3 one-off wrappers (*_ab.sh, *_sweep.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=2; specs=""
while getopts "r:k:" o; do
  case $o in r) rounds=$OPTARG ;; k) specs=$OPTARG ;; *) exit 2 ;; esac
done
shift $((OPTIND - 1))
: > gpurun_out/ab.log
for i in $(seq "$rounds"); do
  for v in "$@"; do
    name=${v%%:*}; rest=${v#*:}; lib=""; envs=""
    case $rest in lib=*) lib=${rest#lib=} ;; *) envs=$rest ;; esac
    if [ -n "$specs" ]; then
      env $envs timeout -k 10 180 python tools/kbench.py ${lib:+--lib $lib} $specs 2>&1 \
        | grep -v amdgpu.ids | sed "s/^/$name /" >> gpurun_out/ab.log || { echo "kbench $name failed"; exit 1; }
    else
      [ -n "$lib" ] && { cp pggan_amd/libpggan_hip.so /tmp/ab_lib_cur.so; cp "$lib" pggan_amd/libpggan_hip.so; }
      env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events \
        ${AB_ARGS:-} > gpurun_out/ab_bench.json 2> gpurun_out/ab_bench.err
      rc=$?
      [ -n "$lib" ] && cp /tmp/ab_lib_cur.so pggan_amd/libpggan_hip.so
      [ $rc -eq 0 ] || { echo "bench $name failed"; tail -5 gpurun_out/ab_bench.err; exit $rc; }
      python -c "import json; d=json.loads(open('gpurun_out/ab_bench.json').read().strip().splitlines()[-1]); print('$name round $i', d['value'], 'img/s', d['ms_per_step'], 'ms/step')" | tee -a gpurun_out/ab.log
    fi
  done
done
if [ -n "$specs" ]; then
  python - <<'PY'
import collections
d = collections.defaultdict(dict)
for l in open("gpurun_out/ab.log"):
    f = l.split()
    if len(f) > 3 and f[3] == "us":
        t = float(f[2])
        d[f[1]][f[0]] = min(t, d[f[1]].get(f[0], 1e30))
for spec, v in d.items():
    print(f"{spec:24s} " + "  ".join(f"{k}: {t:8.1f}" for k, t in v.items()))
PY
fi
