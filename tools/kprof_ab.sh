#!/bin/bash
# Kernel-trace A/B of library builds on kbench specs (GPU box): true per-launch GPU durations
# (kbench's event timing is host-bound below ~12 us per launch).
#   tools/kprof_ab.sh "KBENCH ARGS" NAME=LIB [NAME=LIB ...]    -> gpurun_out/kprof_<NAME>/
# then: python tools/kprof_table.py gpurun_out/kprof_<NAME> ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd); export TMPDIR=/tmp
args=$1; shift
for v in "$@"; do
  name=${v%%=*}; lib=${v#*=}
  rm -rf "gpurun_out/kprof_$name"
  ( cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv \
      -d "$ROOT/gpurun_out/kprof_$name" -o run -- python "$ROOT/tools/kbench.py" --lib "$ROOT/$lib" \
      --iters 10 $args ) > "gpurun_out/kprof_$name.log" 2>&1
  rc=$?; echo "kprof $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/kprof_$name.log"; exit $rc; fi
done
