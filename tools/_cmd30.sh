set -o pipefail
cd $GRAFT_REPO_ROOT
PG_ENGINE=tail_sync=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -n 2 gpurun_out/t_par.log
bash tools/ab.sh -r 4 "base:" "tsync:PG_ENGINE=tail_sync=1" "tsync2:PG_ENGINE=tail_sync=1,tail_levels=2"; grep round gpurun_out/ab.log
