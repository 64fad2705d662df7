# GPU box: A/B of the concurrent fake-image pass, then the GPU suite
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
AB_VAR=PG_FAKE_STREAM AB_A=0 AB_B=1 bash tools/env_ab2.sh 2 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_all.log; exit $rc
