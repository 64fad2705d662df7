set -o pipefail
cd $GRAFT_REPO_ROOT
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_t3w16.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wide or fwd or dgrad_pack" --timeout 200 --timeout-method thread > gpurun_out/t_t3.log 2>&1; echo "t3w16 ops rc=$?"; tail -n 1 gpurun_out/t_t3.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
S="c:128:128:128:0 c:128:128:128:6 c:128:256:128:8 c:256:128:64:8 c:64:512:256:8 c:128:128:256:22"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" b8_$B=pggan_amd/libpggan_hip.so b16_$B=ab/lib_t3w16.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_b8_4 gpurun_out/kprof_b16_4 gpurun_out/kprof_b8_8 gpurun_out/kprof_b16_8 | cut -c1-110
python - <<'PY'
import csv
for n in ('b8_4','b16_4'):
    seen=set()
    for r in csv.DictReader(open(f'gpurun_out/kprof_{n}/run_kernel_trace.csv')):
        k=r['Kernel_Name']
        if 'conv_hr' in k and k not in seen:
            seen.add(k); print(n, k.split('(')[0][-50:], 'vgpr', r['VGPR_Count'], 'scratch', r['Scratch_Size'])
PY
bash tools/ab.sh -r 3 "w8:" "w16:lib=ab/lib_t3w16.so"; grep round gpurun_out/ab.log
