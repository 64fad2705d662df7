set -o pipefail
cd $GRAFT_REPO_ROOT
cp pggan_amd/libpggan_hip.so /tmp/cur.so && cp ab/lib_wnc2.so pggan_amd/libpggan_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -k "wgrad" --timeout 200 --timeout-method thread > gpurun_out/t_wn.log 2>&1; echo "wnc2 ops rc=$?"; tail -n 2 gpurun_out/t_wn.log
cp /tmp/cur.so pggan_amd/libpggan_hip.so
bash tools/ab.sh -r 4 "cur:" "wnc2:lib=ab/lib_wnc2.so"; grep round gpurun_out/ab.log
