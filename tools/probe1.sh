set -o pipefail
mkdir -p gpurun_out
W="w:64:256:256:0 w:64:256:256:4 w:32:512:512:0 w:32:512:512:4 w:128:128:128:0 w:128:128:128:4 w:256:64:64:0 w:256:64:64:4 w:512:32:64:0 w:512:32:64:4 w:128:128:256:0 w:128:128:256:4 w:512:32:64:2 w:512:32:64:6"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -q -x -k "wgrad" --timeout 300 --timeout-method thread > gpurun_out/wg_tests.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --iters 30 --rounds 2 $W > gpurun_out/kb_comb.log 2>&1 && \
timeout -k 10 300 python tools/kbench.py --B 8 --iters 30 $W > gpurun_out/kb_comb8.log 2>&1 && \
timeout -k 10 300 python -u tools/repro_probe.py bf16 6 4 2 2 1 > gpurun_out/repro_comb.log 2>&1 && \
for r in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/ab_comb_$r.json 2>/dev/null && \
PG_ENGINE=wgrad_reduce_launch=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/ab_launch_$r.json 2>/dev/null || exit 1
done
echo rc=$?
tail -n 3 gpurun_out/wg_tests.log; cat gpurun_out/kb_comb.log gpurun_out/kb_comb8.log | grep -v amdgpu; tail -n 2 gpurun_out/repro_comb.log
for f in gpurun_out/ab_*_?.json; do python3 -c "import json,sys; b=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', b['value'], b['ms_per_step'], b.get('launch_path'))"; done
