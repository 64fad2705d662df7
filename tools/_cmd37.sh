set -o pipefail
cd $GRAFT_REPO_ROOT
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_t3b16.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_t3b.log 2>&1; echo "t3b16 ops rc=$?"; tail -n 1 gpurun_out/t_t3b.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
S="c:256:64:128:150 c:128:128:256:150 c:64:256:512:150 c:256:64:128:280 c:128:128:256:280"
bash tools/kprof_ab.sh "--B 4 $S" c8=pggan_amd/libpggan_hip.so c16=ab/lib_t3b16.so || exit 1
python tools/kprof_table.py $S -- gpurun_out/kprof_c8 gpurun_out/kprof_c16 | cut -c1-110
bash tools/ab.sh -r 3 "b8:" "b16:lib=ab/lib_t3b16.so"; grep round gpurun_out/ab.log
