# round-3 GPU check: the changed paths' tests, then the graph A/B (each step time-limited)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
t() { local n=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$n.log 2>&1; local rc=$?; echo "$n rc=$rc"; tail -n 3 gpurun_out/$n.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
t graphaug 400 python -u -m pytest tests/test_gpu_graph.py tests/test_augment.py -x -v -m gpu --timeout 300 --timeout-method thread
t parity 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_fusion.py -x -q -m gpu --timeout 300 --timeout-method thread
t c2gp 600 python -u -m pytest tests/test_gpu_baseline_parity.py -x -v -k wgan --timeout 500 --timeout-method thread -s
bash tools/graph_ab.sh
