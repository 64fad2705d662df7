#!/bin/bash
# Kernel trace of the bench with and without the world-1 DP exchange (GPU box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); export TMPDIR=/tmp
for v in plain dp; do
  a=""; [ $v = dp ] && a="--dp-exchange"
  rm -rf gpurun_out/prof_$v
  ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/gpurun_out/prof_$v" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 1 \
      --cpu-baseline off --no-kernel-events $a ) > gpurun_out/prof_$v.log 2>&1
  rc=$?; echo "prof $v rc=$rc"; tail -n 1 gpurun_out/prof_$v.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
