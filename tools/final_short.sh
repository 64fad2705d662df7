# Short end-of-session check (GPU box): smoke(), the bench line, the rocprofv3 kernel trace and
# the two PMC passes (full_check.sh without the -m gpu suite)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/bench.log; exit $rc; fi
tail -n 1 gpurun_out/bench.log | cut -c1-200
bash tools/gpu_check.sh prof pmc
