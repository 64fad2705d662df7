set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:128:128:128:0 c:128:128:128:6 c:64:256:256:0 c:128:256:128:8 c:256:128:64:8 c:64:512:256:8 c:128:128:256:22"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" t3_$B=pggan_amd/libpggan_hip.so alt_$B=ab/lib_t3alt.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_t3_4 gpurun_out/kprof_alt_4 gpurun_out/kprof_t3_8 gpurun_out/kprof_alt_8 | cut -c1-110
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_t3alt.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_alt.log 2>&1; echo "alt ops rc=$?"; tail -n 2 gpurun_out/t_alt.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
bash tools/ab.sh -r 3 "t3:" "alt:lib=ab/lib_t3alt.so"; grep round gpurun_out/ab.log
