set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wgrad or unpool" --timeout 200 --timeout-method thread > gpurun_out/t_wg.log 2>&1; echo "ops rc=$?"; tail -n 2 gpurun_out/t_wg.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -n 2 gpurun_out/t_par.log
bash tools/ab.sh -r 4 "mix:" "all4:lib=ab/lib_wg4.so" "all3:lib=ab/lib_wg3.so"; grep round gpurun_out/ab.log
