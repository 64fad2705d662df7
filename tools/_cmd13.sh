set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/wait_probe.py > gpurun_out/wait_probe.txt 2>&1; echo "probe rc=$?"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_dp.py -v -k paper --timeout 1000 --timeout-method thread -s > gpurun_out/t_dp_paper.log 2>&1; echo "dp rc=$?"; tail -5 gpurun_out/t_dp_paper.log
