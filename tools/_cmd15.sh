set -o pipefail
cd $GRAFT_REPO_ROOT
S="c:256:64:64:0 c:256:64:64:6 c:256:64:64:8 c:256:64:64:70"
for B in 4 8; do
bash tools/kprof_ab.sh "--B $B $S" head$B=ab/lib_head.so th8_$B=ab/lib_t16th8.so nw8_$B=ab/lib_th16nw8.so || exit 1
done
python tools/kprof_table.py $S -- gpurun_out/kprof_head4 gpurun_out/kprof_th8_4 gpurun_out/kprof_nw8_4 gpurun_out/kprof_head8 gpurun_out/kprof_th8_8 gpurun_out/kprof_nw8_8 > gpurun_out/t16_kprof.txt 2>&1; cut -c1-110 gpurun_out/t16_kprof.txt
