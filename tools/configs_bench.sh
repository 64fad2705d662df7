# Bench lines for the other BASELINE configs on one GPU (GPU box): C2 (128^2, B=16,
# alpha 1, WGAN-GP and R1), C3 (256^2, B=8, alpha 0.5), C4's per-GPU shard (512^2, B=8) and
# C5 with WGAN-GP.  One JSON line each under gpurun_out/cfg_<name>.json; stops at the first
# run that fails.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline off "$@" \
    > "gpurun_out/cfg_$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/cfg_$name.log"; exit $rc; fi
  tail -n 1 "gpurun_out/cfg_$name.log" > "gpurun_out/cfg_$name.json"
}
run C2_wgangp --stage 5 --batch 16 --alpha 1.0 --gp-mode wgan-gp
run C2_r1 --stage 5 --batch 16 --alpha 1.0
run C3 --stage 6 --batch 8 --alpha 0.5
run C4shard --stage 7 --batch 8 --alpha 1.0
run C5_wgangp --stage 8 --batch 4 --alpha 1.0 --gp-mode wgan-gp
