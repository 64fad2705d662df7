#!/bin/bash
# GPU-box runner: `bash tools/gpu_check.sh STEP [STEP ...]`, each GPU step under its own time
# limit; stops at the first step that ends other than pass (0) / test failures (1).  Logs under
# gpurun_out/<step>.log.  The steps are the measurement recipes DESIGN.md cites (suite, smoke,
# bench, kernel trace + PMC passes, kbench shape lists, probes, loader, configs, DP rehearsal);
# interleaved A/B runs of library knobs or builds: tools/ab.sh.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1; shift
  local t=$1; shift
  # heartbeat: the CPU oracle of the largest parity cases runs for minutes without output
  ( while sleep 50; do date +%T >> gpurun_out/heartbeat.log; done ) &
  local hb=$!
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  kill $hb 2>/dev/null; wait $hb 2>/dev/null
  echo "$name rc=$rc"
  tail -n 3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    ops) run ops 900 python -m pytest tests/test_gpu_ops.py -q -x ;;
    parity) run parity 1200 python -m pytest tests/test_gpu_parity.py -q ;;
    gpu) run gpu 1500 python -u -m pytest tests -v -m gpu --timeout 600 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps 20 --warmup 5 ;;
    benchq) run benchq 600 python bench.py --steps 3 --warmup 1 --cpu-baseline off ;;
    prof)
      ROOT=$(pwd)
      rm -rf gpurun_out/prof
      export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$ROOT/gpurun_out/prof" -o run -- python "$ROOT/bench.py" --steps ${PROF_STEPS:-3} --warmup 1 \
          --cpu-baseline off --no-kernel-events ) > gpurun_out/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -n 3 gpurun_out/prof.log
      if [ $rc -ne 0 ]; then exit $rc; fi ;;
    pmc)
      ROOT=$(pwd)
      export TMPDIR=/tmp
      for c in FETCH_SIZE WRITE_SIZE; do
        rm -rf "gpurun_out/pmc_$c"
        ( cd /tmp && PG_BENCH_LAUNCHES="$ROOT/gpurun_out/launches_$c.json" timeout -k 10 900 \
            rocprofv3 --pmc $c --output-format csv \
            -d "$ROOT/gpurun_out/pmc_$c" -o run -- python "$ROOT/bench.py" --steps 1 --warmup 1 \
            --cpu-baseline off ) > gpurun_out/pmc_$c.log 2>&1
        rc=$?; echo "pmc $c rc=$rc"; tail -n 3 gpurun_out/pmc_$c.log
        if [ $rc -ne 0 ]; then exit $rc; fi
      done
      python tools/prof_summary.py gpurun_out/prof --fetch gpurun_out/pmc_FETCH_SIZE \
        --write gpurun_out/pmc_WRITE_SIZE --launches gpurun_out/launches_FETCH_SIZE.json \
        -o gpurun_out/prof_summary.json > /dev/null ;;
    shapes) PG_BENCH_SHAPES=gpurun_out/shapes.json run shapes 600 python bench.py --steps 3 --warmup 1 --cpu-baseline off ;;
    wg) run wg 600 python -m pytest tests/test_gpu_ops.py -q -x -k wgrad ;;
    kbw) run kbw 300 python tools/kbench.py w:1024:16:32:0 w:1024:16:16:0 w:1024:32:16:1 \
           w:512:32:64:0 w:512:32:32:0 w:256:64:128:0 w:256:64:64:0 w:128:128:256:0 \
           w:128:128:128:0 w:64:256:512:0 w:64:256:256:0 w:32:512:512:0 w:16:512:512:0 \
           w:8:512:512:0 w:4:512:512:0 w:4:513:512:0 ;;
    conv) run conv 600 python -m pytest tests/test_gpu_ops.py -q -x -k "conv3x3_fwd or dgrad" ;;
    kbc) run kbc 300 python tools/kbench.py c:1024:32:16:8 c:1024:16:16:8 c:1024:16:32:22 \
           c:1024:16:16:6 c:512:64:32:8 c:512:32:64:22 c:512:32:32:6 c:512:32:32:0 \
           c:256:128:64:8 c:256:64:128:22 c:256:64:64:6 c:128:256:128:8 c:128:128:128:6 \
           c:64:512:256:8 c:64:256:256:6 c:32:512:512:8 c:1024:32:16:7 c:1024:16:32:8 ;;
    pmcq)   # counters of one kbench spec: PMC_SPEC, PMC_COUNTERS (one pass)
      ROOT=$(pwd); export TMPDIR=/tmp
      ( cd /tmp && timeout -k 10 300 rocprofv3 --pmc ${PMC_COUNTERS} --output-format csv \
          -d "$ROOT/gpurun_out/pmcq" -o run -- python "$ROOT/tools/kbench.py" --iters 3 ${PMC_SPEC} ) \
          > gpurun_out/pmcq.log 2>&1
      rc=$?; echo "pmcq rc=$rc"; tail -n 3 gpurun_out/pmcq.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    listc) ( rocprofv3 -L > gpurun_out/counters.txt 2>&1 ); echo "listc rc=$?" ;;
    kbl) run kbl 300 python tools/kbench.py c:32:512:512:8 c:32:512:512:6 c:32:512:512:0 \
           c:64:256:512:22 c:64:512:256:8 c:64:256:256:6 c:16:512:512:6 c:16:512:512:8 \
           c:8:512:512:6 c:4:512:512:6 c:128:128:256:22 c:128:256:128:8 c:128:128:128:6 \
           w:32:512:512:0 w:64:256:512:0 w:64:256:256:0 w:16:512:512:0 w:128:128:256:0 ;;
    kprof)   # kernel trace of the kbench specs in KPROF_SPECS
      ROOT=$(pwd); export TMPDIR=/tmp; rm -rf gpurun_out/kprof
      ( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$ROOT/gpurun_out/kprof" -o run -- python "$ROOT/tools/kbench.py" --iters 5 ${KPROF_SPECS} ) \
          > gpurun_out/kprof.log 2>&1
      rc=$?; echo "kprof rc=$rc"; tail -n 3 gpurun_out/kprof.log; if [ $rc -ne 0 ]; then exit $rc; fi ;;
    opprof) run opprof 300 python tools/op_profile.py --json gpurun_out/opprof.json ;;
    dbg4) run dbg4 600 python tools/debug_buffers.py 4 1.0 ;;
    kloop) run kloop 120 ./tools/kloop_probe ;;   # build: hipcc --offload-arch=gfx950 -O3 -o tools/kloop_probe tools/kloop_probe.hip
    dp) run dp 600 python -u -m pytest tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread ;;
    graph) run graph 600 python -u -m pytest tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread ;;
    loader) run loader 600 python tools/loader_bench.py --out gpurun_out/loader.json ;;
    configs) run configs 1500 bash tools/configs_bench.sh ;;
    rehearsal) run rehearsal 900 bash tools/dp_rehearsal.sh ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
