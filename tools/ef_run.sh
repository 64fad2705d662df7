cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:1024:16:16:8 c:1024:16:16:6 c:1024:16:16:0 c:1024:16:32:16 c:1024:16:16:70 c:1024:32:16:71 c:512:32:32:6 c:512:32:32:8 c:512:32:32:0 c:512:32:32:70"
PG_HR_EF=0 timeout -k 10 200 python tools/kbench.py $S > gpurun_out/kef0.txt 2>&1 || exit 1
timeout -k 10 200 python tools/kbench.py $S > gpurun_out/kef1.txt 2>&1 || exit 1
PG_HR_EF_PD=1 timeout -k 10 200 python tools/kbench.py $S > gpurun_out/kef1pd1.txt 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusion.py tests/test_gpu_baseline_parity.py -k "not fp32_step" -x -q --timeout 600 --timeout-method thread > gpurun_out/eft.log 2>&1; rc=$?; tail -3 gpurun_out/eft.log; [ $rc -le 1 ] || exit $rc
AB_VAR=PG_HR_EF AB_A=0 AB_B=1 bash tools/env_ab2.sh 2
