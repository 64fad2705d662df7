set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repro_probe.py bf16 6 4 2 3 1 > gpurun_out/repro_det_bf16.log 2>&1 && \
timeout -k 10 300 python -u tools/repro_probe.py f32 6 4 2 2 1 > gpurun_out/repro_det_f32.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -k "elision or reproducible" --timeout 300 --timeout-method thread > gpurun_out/det_tests.log 2>&1 ; \
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ops_det.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/ops_det.log
grep -E "PASS|FAIL|Error|assert" gpurun_out/det_tests.log | head -20
