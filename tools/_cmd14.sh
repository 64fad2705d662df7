set -o pipefail
cd $GRAFT_REPO_ROOT
ROOT=$(pwd); export TMPDIR=/tmp; rm -rf gpurun_out/htrace
( cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --output-format csv \
   -d "$ROOT/gpurun_out/htrace" -o run -- python "$ROOT/bench.py" --steps 3 --warmup 1 \
   --cpu-baseline off --no-kernel-events ) > gpurun_out/htrace.log 2>&1; echo "htrace rc=$?"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_dp.py -v -k paper --timeout 1000 --timeout-method thread -s > gpurun_out/t_dp_paper.log 2>&1; echo "dp rc=$?"; tail -4 gpurun_out/t_dp_paper.log
