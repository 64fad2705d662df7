set -o pipefail
cd $GRAFT_REPO_ROOT
( while sleep 50; do date +%T >> gpurun_out/heartbeat.log; done ) & hb=$!
PG_PARITY_OUT=gpurun_out/parity_r6v6 timeout -k 10 1000 python -u -m pytest tests/test_gpu_baseline_parity.py tests/test_gpu_dp.py -v -m gpu --timeout 900 --timeout-method thread -s > gpurun_out/gpuB.log 2>&1; rc=$?
kill $hb; echo "gpuB rc=$rc"; tail -n 3 gpurun_out/gpuB.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -n 2 gpurun_out/smoke.log
