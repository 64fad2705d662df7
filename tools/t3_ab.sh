cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:128:128:128:6 c:128:128:128:0 c:256:128:64:8 c:128:256:128:8 c:256:64:128:22 c:128:128:256:22"
for v in "PG_HR_T3_ASM=0" "PG_HR_T3_ASM=1"; do
  echo "== $v" >> gpurun_out/t3.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/t3.txt 2>&1 || exit 1
done
PG_HR_T3_ASM=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t3_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t3_tests.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=PG_HR_T3_ASM AB_A=0 AB_B=1 bash tools/env_ab2.sh 2
