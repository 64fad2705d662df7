set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:512:32:64:150 c:512:64:32:521 c:1024:16:16:6 c:1024:16:16:70 c:1024:16:16:264 c:512:32:32:0 c:512:32:32:6 c:256:64:64:0"
bash tools/kprof_ab.sh "--B 4 $S" pd2=pggan_amd/libpggan_hip.so pd4=ab/lib_pd4.so || exit 1
python tools/kprof_table.py $S -- gpurun_out/kprof_pd2 gpurun_out/kprof_pd4 | cut -c1-120
python - <<'PY'
import csv
for n in ('pd2','pd4'):
    seen=set()
    for r in csv.DictReader(open(f'gpurun_out/kprof_{n}/run_kernel_trace.csv')):
        k=r['Kernel_Name']
        if 'conv_hr' in k and k not in seen:
            seen.add(k); print(n, k.split('(')[0][-60:], 'vgpr', r['VGPR_Count'], 'agpr', r['Accum_VGPR_Count'], 'scratch', r['Scratch_Size'])
PY
