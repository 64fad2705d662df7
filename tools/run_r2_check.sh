cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -n 3 gpurun_out/bench.err; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_check.sh prof pmc || exit $?
AB_SPECS="c:256:64:128:22 c:256:128:64:8 c:256:64:64:6 c:128:256:128:8 c:128:128:256:22 c:128:128:128:6 c:64:512:256:8 c:64:256:512:22 c:64:256:256:6" bash tools/ab_run.sh 2 > gpurun_out/ab_BA.txt 2>&1
cp ab/lib_C.so ab/lib_B.so
AB_SPECS="c:256:64:128:22 c:256:128:64:8 c:256:64:64:6 c:128:256:128:8 c:128:128:256:22 c:128:128:128:6 c:64:512:256:8 c:64:256:512:22 c:64:256:256:6" bash tools/ab_run.sh 2 > gpurun_out/ab_CA.txt 2>&1
echo done
