# GPU box: tile 13 (8-row LDS-DMA conv_hr tile) for the 32^2 wide convs vs conv3x3_kernel
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:32:512:512:8 c:32:512:512:6 c:32:512:512:0 c:32:512:512:22 c:32:256:512:22 c:32:512:256:8"
for v in "PG_HR_T13=0" "PG_HR_T13=1"; do
  echo "== $v" >> gpurun_out/t13.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/t13.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t13_tests.log 2>&1; rc=$?; tail -2 gpurun_out/t13_tests.log; [ $rc -eq 0 ] || exit $rc
AB_VAR=PG_HR_T13 AB_A=0 AB_B=1 bash tools/env_ab2.sh 2
