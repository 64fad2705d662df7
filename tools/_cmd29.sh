set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "rgbo or wide or rgb" --timeout 200 --timeout-method thread > gpurun_out/t_rgbo.log 2>&1; echo "ops rc=$?"; tail -n 3 gpurun_out/t_rgbo.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -n 2 gpurun_out/t_par.log
bash tools/ab.sh -r 4 "rgbo:" "norgbo:PG_ENGINE=fuse_rgbo=0"; grep round gpurun_out/ab.log
