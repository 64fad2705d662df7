set -o pipefail
cd $GRAFT_REPO_ROOT
( while sleep 50; do date +%T >> gpurun_out/heartbeat.log; done ) & hb=$!
timeout -k 10 1100 python -u -m pytest tests -v -m gpu --ignore=tests/test_gpu_baseline_parity.py --ignore=tests/test_gpu_dp.py --timeout 600 --timeout-method thread > gpurun_out/gpuA.log 2>&1; rc=$?
echo "gpuA rc=$rc"; tail -n 2 gpurun_out/gpuA.log
[ $rc -eq 0 ] || { kill $hb; exit $rc; }
PG_PARITY_OUT=gpurun_out/parity_r6v5 timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_parity.py -v -m gpu -k bf16 --timeout 500 --timeout-method thread -s > gpurun_out/gpuC5.log 2>&1; rc=$?
echo "gpuC5 rc=$rc"; tail -n 2 gpurun_out/gpuC5.log
[ $rc -eq 0 ] || { kill $hb; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -n 1 gpurun_out/smoke.log
kill $hb
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -n 1 gpurun_out/bench.log | cut -c1-300
