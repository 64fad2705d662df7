# Rehearsal of the driver's N>1 bench command on a one-GPU box (GPU box): the same
# torch.distributed.run launch, with the gloo backend (RCCL does not run two ranks on one
# GPU) and every rank on cuda:0.  Output: gpurun_out/dp<N>.log (the JSON line is rank 0's).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for n in ${DP_RANKS:-2}; do
  PG_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py \
    --gpus $n --steps ${DP_STEPS:-3} --warmup 1 > gpurun_out/dp$n.log 2>&1
  rc=$?
  echo "dp$n rc=$rc"
  tail -n 1 gpurun_out/dp$n.log | cut -c1-300
  if [ $rc -ne 0 ]; then tail -n 20 gpurun_out/dp$n.log; exit $rc; fi
done
