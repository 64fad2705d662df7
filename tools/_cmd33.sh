set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:512:32:64:150 c:512:32:64:280"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" w4_$B=pggan_amd/libpggan_hip.so w8_$B=ab/lib_t14w8.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_w4_4 gpurun_out/kprof_w8_4 gpurun_out/kprof_w4_8 gpurun_out/kprof_w8_8 | cut -c1-110
python - <<'PY'
import csv
for n in ('w4_4','w8_4'):
    seen=set()
    for r in csv.DictReader(open(f'gpurun_out/kprof_{n}/run_kernel_trace.csv')):
        k=r['Kernel_Name']
        if 'conv_hr' in k and k not in seen:
            seen.add(k); print(n, 'vgpr', r['VGPR_Count'], 'scratch', r['Scratch_Size'])
PY
