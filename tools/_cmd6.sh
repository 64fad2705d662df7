set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "splitk_combine or conv3x3_fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_sk.log 2>&1; echo "ops rc=$?"; tail -3 gpurun_out/t_sk.log
rm -rf gpurun_out/skprof
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/skprof -o run -- python $GRAFT_REPO_ROOT/tools/sk_probe.py > $GRAFT_REPO_ROOT/gpurun_out/sk_probe.txt 2>&1 ); echo "prof rc=$?"
python tools/sk_report.py $(ls gpurun_out/skprof/*/*kernel_trace.csv gpurun_out/skprof/*kernel_trace.csv 2>/dev/null | head -1) gpurun_out/sk_probe.txt
