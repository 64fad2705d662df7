set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dp.py tests/test_gpu_graph.py -v -k "elision_on_hip or two_steps or cpp_replay" --timeout 300 --timeout-method thread > gpurun_out/det_tests2.log 2>&1 ; \
timeout -k 10 600 python -u tools/loader_bench.py --out gpurun_out/loader.json > gpurun_out/loader.log 2>&1 ; \
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --cpu-baseline off --dp-exchange > gpurun_out/bench_dpx.json 2> gpurun_out/bench_dpx.err
echo "rc=$?"
grep -E "PASS|FAIL|Error|assert" gpurun_out/det_tests2.log | head -40
cut -c1-300 gpurun_out/bench_dpx.json
