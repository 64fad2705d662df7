#!/bin/bash
# Whole-step A/B: bench.py with ab/lib_A.so and ab/lib_B.so swapped in as the in-tree
# library (GPU box copy only), interleaved rounds.   tools/ab_bench.sh [rounds]
cd "$(dirname "$0")/.."
r=${1:-2}
cp pggan_amd/libpggan_hip.so /tmp/lib_cur.so
for i in $(seq "$r"); do
  for v in A B; do
    cp ab/lib_$v.so pggan_amd/libpggan_hip.so
    echo -n "$v "
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off --no-kernel-events 2>&1 \
      | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
cp /tmp/lib_cur.so pggan_amd/libpggan_hip.so
