#!/bin/bash
# Whole-step A/B with per-variant environment: tools/ab_env.sh ROUNDS "A:ENV=.." "B:ENV=.." ...
# (variant letter = ab/lib_<letter>.so swapped in as the in-tree library; GPU box copy only)
cd "$(dirname "$0")/.."
r=$1; shift
cp pggan_amd/libpggan_hip.so /tmp/lib_cur.so
for i in $(seq "$r"); do
  for spec in "$@"; do
    v=${spec%%:*}; envs=${spec#*:}
    cp ab/lib_$v.so pggan_amd/libpggan_hip.so
    echo -n "$spec "
    env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events 2>&1 \
      | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
cp /tmp/lib_cur.so pggan_amd/libpggan_hip.so
