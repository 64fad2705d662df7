set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "rgb" --timeout 200 --timeout-method thread > gpurun_out/t_rgb.log 2>&1; echo "ops rc=$?"; tail -3 gpurun_out/t_rgb.log
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_graph.log 2>&1; echo "graph rc=$?"; tail -3 gpurun_out/t_graph.log
bash tools/ab.sh -r 4 "wg:" "nowg:PG_ENGINE=fuse_torgb_wg=0"
