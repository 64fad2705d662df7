# Whole GPU check of one build (GPU box): the -m gpu suite, smoke(), the bench line, a
# rocprofv3 kernel trace and the two PMC passes.  Stops at the first GPU step that ends
# other than pass (0) / test failures (1).  Logs and outputs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PG_PARITY_OUT=gpurun_out/parity timeout -k 10 780 python -u -m pytest tests -m gpu -q \
  --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -n 3 gpurun_out/gpu_all.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; if [ $rc -ne 0 ]; then tail -n 5 gpurun_out/bench.log; exit $rc; fi
bash tools/gpu_check.sh prof pmc
