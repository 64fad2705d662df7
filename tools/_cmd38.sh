set -o pipefail
cd $GRAFT_REPO_ROOT
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_not13.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_13.log 2>&1; echo "not13 ops rc=$?"; tail -n 1 gpurun_out/t_13.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
S="c:32:512:512:6 c:32:512:512:8 c:32:512:512:0 c:32:512:512:22"
bash tools/kprof_ab.sh "--B 4 $S" t13=pggan_amd/libpggan_hip.so t6=ab/lib_not13.so || exit 1
python tools/kprof_table.py $S -- gpurun_out/kprof_t13 gpurun_out/kprof_t6 | cut -c1-110
bash tools/ab.sh -r 3 "t13:" "not13:lib=ab/lib_not13.so"; grep round gpurun_out/ab.log
