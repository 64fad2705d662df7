set -o pipefail
cd $GRAFT_REPO_ROOT
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_t6w8.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_t6.log 2>&1; echo "t6w8 ops rc=$?"; tail -n 1 gpurun_out/t_t6.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B c:32:512:512:6 c:32:512:512:8 c:64:256:256:6 c:64:512:256:8 c:64:256:512:22" a4_$B=pggan_amd/libpggan_hip.so a8_$B=ab/lib_t6w8.so || exit 1
done
python tools/kprof_table.py c:32:512:512:6 c:32:512:512:8 c:64:256:256:6 c:64:512:256:8 c:64:256:512:22 -- gpurun_out/kprof_a4_4 gpurun_out/kprof_a8_4 gpurun_out/kprof_a4_8 gpurun_out/kprof_a8_8 | cut -c1-110
bash tools/ab.sh -r 3 "t6w4:" "t6w8:lib=ab/lib_t6w8.so"; grep round gpurun_out/ab.log
