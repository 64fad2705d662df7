set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/repro_probe.py bf16 6 4 2 3 1 > gpurun_out/repro_det_bf16.log 2>&1 && \
timeout -k 10 300 python -u tools/repro_probe.py f32 6 4 2 2 1 > gpurun_out/repro_det_f32.log 2>&1 && \
timeout -k 10 1200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_augment.py tests/test_gpu_graph.py -v -k "elision or reproducible or dp or loader or graph or replay" --timeout 300 --timeout-method thread > gpurun_out/det_tests.log 2>&1 ; \
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread > gpurun_out/ops_det.log 2>&1 ; \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err && \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --replay > gpurun_out/bench_replay.json 2> gpurun_out/bench_replay.err ; \
timeout -k 10 600 python -u tools/loader_bench.py --out gpurun_out/loader.json > gpurun_out/loader.log 2>&1
echo "rc=$?"
tail -3 gpurun_out/ops_det.log
grep -E "PASS|FAIL|Error|assert" gpurun_out/det_tests.log | head -40
cut -c1-300 gpurun_out/bench_eager.json gpurun_out/bench_replay.json
cat gpurun_out/loader.log | cut -c1-200
