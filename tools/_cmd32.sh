set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > gpurun_out/t_wg.log 2>&1; echo "ops rc=$?"; tail -n 2 gpurun_out/t_wg.log
[ -n "$(grep -c passed gpurun_out/t_wg.log)" ] || exit 1
S="w:1024:16:32:2 w:512:32:64:2"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" go_$B=pggan_amd/libpggan_hip.so ng_$B=ab/lib_nogonce.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_go_4 gpurun_out/kprof_ng_4 gpurun_out/kprof_go_8 gpurun_out/kprof_ng_8 | cut -c1-110
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_graph.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_par.log 2>&1; echo "par rc=$?"; tail -n 2 gpurun_out/t_par.log
bash tools/ab.sh -r 4 "gonce:" "nogonce:lib=ab/lib_nogonce.so"; grep round gpurun_out/ab.log
