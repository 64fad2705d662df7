set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "rgbd or rgbw or from_rgb or linear" --timeout 200 --timeout-method thread > gpurun_out/t_rgbd.log 2>&1; echo "ops rc=$?"; tail -3 gpurun_out/t_rgbd.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fusion.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_graph.log 2>&1; echo "graph rc=$?"; tail -3 gpurun_out/t_graph.log
PG_PARITY_OUT=gpurun_out/parity_r6 timeout -k 10 600 python -u -m pytest tests/test_gpu_baseline_parity.py -x -q -k "bf16 or C2" --timeout 500 --timeout-method thread > gpurun_out/t_bf16.log 2>&1; echo "bf16 rc=$?"; tail -3 gpurun_out/t_bf16.log
bash tools/ab.sh -r 3 "rgbd:" "head:lib=ab/lib_head.so"
