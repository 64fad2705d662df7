set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:128:128:128:0 c:128:128:128:6 c:64:256:256:0 c:128:256:128:8 c:256:128:64:8 c:64:512:256:8 c:128:128:256:22"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" w8_$B=pggan_amd/libpggan_hip.so w4_$B=ab/lib_t3w4.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_w8_4 gpurun_out/kprof_w4_4 gpurun_out/kprof_w8_8 gpurun_out/kprof_w4_8 | cut -c1-100
python - <<'PY'
import csv
for n in ('w8_4','w4_4'):
    seen=set()
    for r in csv.DictReader(open(f'gpurun_out/kprof_{n}/run_kernel_trace.csv')):
        k=r['Kernel_Name']
        if 'conv_hr' in k and k not in seen:
            seen.add(k); print(n, 'vgpr', r['VGPR_Count'], 'agpr', r['Accum_VGPR_Count'], 'scratch', r['Scratch_Size'], 'lds', r['LDS_Block_Size'])
PY
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_t3w4.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_alt.log 2>&1; echo "w4 ops rc=$?"; tail -n 2 gpurun_out/t_alt.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
