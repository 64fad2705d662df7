set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or dgrad_pack or fwd" --timeout 200 --timeout-method thread > gpurun_out/t_wide.log 2>&1; echo "ops rc=$?"; tail -2 gpurun_out/t_wide.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -2 gpurun_out/t_par.log
bash tools/ab.sh -r 4 "t16:" "head:lib=ab/lib_head.so"; grep round gpurun_out/ab.log
