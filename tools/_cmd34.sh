set -o pipefail
cd $GRAFT_REPO_ROOT
# 1. tile 14 at 8 waves (in-tree default now): ops + parity/graph + step A/B vs the EF-8 build and HEAD~
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ops.log 2>&1; echo "ops rc=$?"; tail -n 1 gpurun_out/t_ops.log
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_ef8.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_ops8.log 2>&1; echo "ef8 ops rc=$?"; tail -n 1 gpurun_out/t_ops8.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
S="c:1024:16:16:6 c:1024:16:16:70 c:1024:16:16:264 c:1024:16:32:150 c:1024:32:16:521 c:1024:32:16:71 c:512:32:32:0 c:512:32:32:6"
bash tools/kprof_ab.sh "--B 4 $S" n4=pggan_amd/libpggan_hip.so n8=ab/lib_ef8.so || exit 1
python tools/kprof_table.py $S -- gpurun_out/kprof_n4 gpurun_out/kprof_n8 | cut -c1-110
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -n 1 gpurun_out/t_par.log
bash tools/ab.sh -r 3 "t14w8:" "ef8:lib=ab/lib_ef8.so"; grep round gpurun_out/ab.log
