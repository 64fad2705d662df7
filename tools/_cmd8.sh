set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "linear" --timeout 200 --timeout-method thread > gpurun_out/t_lin.log 2>&1; echo "lin rc=$?"; tail -3 gpurun_out/t_lin.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_graph.log 2>&1; echo "graph rc=$?"; tail -3 gpurun_out/t_graph.log
bash tools/gpu_check.sh prof
python /root/repo/tools/trace_streams.py gpurun_out/prof/run_kernel_trace.csv --steps 3 --top 40 > gpurun_out/streams.txt 2>&1 || true
