#!/bin/bash
# Round-3 iteration check (GPU box): op tests of the changed kernels, a wgrad slab-reduction
# A/B on kbench and the per-op profile of one step.  Each GPU step time-limited; stops at the
# first step that ends other than pass / test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
t() { local n=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 gpurun_out/$n.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
t ops 600 python -u -m pytest tests/test_gpu_ops.py -x -q -m gpu -k "${ITER_K:-wgrad or rgb}" --timeout 300 --timeout-method thread
if [ -n "$ITER_AB" ]; then
  ENV_AB=$ITER_AB AB_SPECS="$ITER_SPECS" timeout -k 10 600 bash tools/env_ab.sh 2 > gpurun_out/ab.txt 2>&1; echo "ab rc=$?"; cat gpurun_out/ab.txt
fi
t opprof 300 python tools/op_profile.py --json gpurun_out/opprof.json
