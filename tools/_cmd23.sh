set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/_cmd22.sh || exit 1
S="w:1024:16:32:2 w:512:32:64:2 w:1024:16:16:0 w:512:32:32:0 w:256:64:128:0 w:128:128:256:0"
bash tools/kprof_ab.sh "--B 4 $S" s3=pggan_amd/libpggan_hip.so s4=ab/lib_wg4.so || exit 1
python tools/kprof_table.py $S -- gpurun_out/kprof_s3 gpurun_out/kprof_s4 | cut -c1-120
bash tools/ab.sh -r 3 "cur:" "wg4:lib=ab/lib_wg4.so" "oldunpool:lib=ab/lib_unpoolv.so"; grep round gpurun_out/ab.log
