set -o pipefail
cd $GRAFT_REPO_ROOT
( while sleep 50; do date +%T >> gpurun_out/heartbeat.log; done ) & hb=$!
timeout -k 10 1100 python -u -m pytest tests -v -m gpu --ignore=tests/test_gpu_baseline_parity.py --ignore=tests/test_gpu_dp.py --timeout 600 --timeout-method thread > gpurun_out/gpuA.log 2>&1; rc=$?
kill $hb; echo "gpuA rc=$rc"; tail -n 3 gpurun_out/gpuA.log
