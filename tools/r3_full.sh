# whole GPU suite, then the bench (each step time-limited; stops at a fault/timeout)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -n 15 gpurun_out/gpu_all.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_r3.json 2> gpurun_out/bench_r3.err
rc=$?; echo "bench rc=$rc"; tail -n 2 gpurun_out/bench_r3.err
