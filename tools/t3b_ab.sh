cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:512:32:64:150 c:512:32:64:280 c:128:128:128:6"
for v in "PG_HR_T3_ASM=0" "PG_HR_T3_ASM=1"; do
  echo "== $v" >> gpurun_out/t3b.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/t3b.txt 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusion.py tests/test_gpu_baseline_parity.py -k "not fp32_step" -x -q --timeout 600 --timeout-method thread > gpurun_out/t3b_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t3b_tests.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=PG_HR_T3_ASM AB_A=0 AB_B=1 bash tools/env_ab2.sh 2
