cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
S="c:128:128:128:6 c:64:256:256:6 c:256:64:64:6 c:256:128:64:8 c:128:256:128:8 c:64:512:256:8 c:32:512:512:8 c:32:512:512:0 c:32:256:512:22"
for v in "PG_HR_DMA=1" "PG_HR_DMA=0"; do
  echo "== $v" >> gpurun_out/dma2.txt
  env $v timeout -k 10 120 python tools/kbench.py $S >> gpurun_out/dma2.txt 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_fusion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/dma_tests.log 2>&1; rc=$?; tail -2 gpurun_out/dma_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/env_multi.sh 2 - PG_HR_DMA=0 PG_HR_T13=0
