cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_augment.py tests/test_abi.py -v --timeout 120 --timeout-method thread > gpurun_out/aug.log 2>&1; rc=$?; tail -12 gpurun_out/aug.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > gpurun_out/b9.json 2> gpurun_out/b9.err; rc=$?; tail -2 gpurun_out/b9.err; exit $rc
