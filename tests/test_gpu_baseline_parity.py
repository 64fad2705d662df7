"""Step parity at the BASELINE configurations, on the GPU, through the C ABI.

BASELINE.json configs[1..4] at paper widths
[512,512,512,512,256,128,64,32,16], one full train_step each (pggan/model.py:206-255:
D half with R1 double-backward + Adam_D, G half + Adam_G), compared with the CPU
oracle replayed from the same parameters and inputs in float64 with the HIP forward's
leaky-ReLU region choices injected (tests/kink_parity.py explains why and bounds the
injected flips to rounding):

* fp32 mode (the north star's parity bar): EVERY live D and G gradient tensor, all
  three images, the losses and R1 within 1e-3 relative L2; parameters after both Adam
  steps within 1e-5; injected region flips only at |pre-activation| <= 2e-4 RMS.
  C4 runs its per-GPU shard (B=8 at 512^2: the DP contract makes each rank's step the
  single-process step on its shard, tests/test_dp_gloo.py).
* bf16 mode (the benchmarked path, C5 = the bench workload), the oracle fed our fake
  images so each network sees identical inputs: images within 3% relative L2, losses
  and R1 within 2e-3 relative, every live gradient tensor at cosine >= 0.999 with the
  oracle, injected flips on <= 1% of pre-activations and only at |x| <= 0.3 RMS (bf16
  storage and weights round to 2^-9 and the error compounds over 18 layers; measured in
  round 2: images 2%, losses <= 5e-4, worst cosine 0.99986, 0.15% flips, worst at 0.16
  RMS; the bars sit near what the kernels achieve so a regression shows, round-6 reports:
  profiles/r6_parity_*.json).

Inputs: numpy PCG64 seeds (tests/golden/gen_inputs.py): weights N(0,1) like the
reference init (lib/layers.py:51-56), biases 0.1*N(0,1) so the bias*c path is live,
reals U[-1,1), latents N(0,1).  If PG_PARITY_OUT names a directory, a JSON report per
config is written there (profiles/r6_parity_*.json are copies).
"""
import json
import os
import time

import pytest
import torch

import kink_parity as K
from gen_inputs import make_inputs, make_params
from oracle import pggan_oracle as O

pytestmark = pytest.mark.gpu

CONFIGS = [  # (name, stage, batch per GPU, alpha, steps)
    ("C2", 5, 16, 1.0, 2),
    ("C3", 6, 8, 0.5, 1),
    ("C4shard", 7, 8, 1.0, 1),
    ("C5", 8, 4, 1.0, 1),
]
THREADS = min(16, os.cpu_count() or 1)


def build(s, B, dtype, seed):
    from pggan_amd import _lib
    from pggan_amd import engine as E
    depths = O.PAPER_DEPTHS
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = {k: torch.from_numpy(v) for k, v in make_params(gsh, seed=seed).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(dsh, seed=seed + 1).items()}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), "cuda", PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", s), "cuda", PD)
    eng = E.StepEngine(_lib.HipOps(dtype), depths, s, B, "cuda")
    eng.bind(fpG, fpD, E.Hyper())
    return eng, fpG, fpD


def _report(name, rep, extra):
    out = os.environ.get("PG_PARITY_OUT")
    if not out:
        return
    os.makedirs(out, exist_ok=True)
    d = dict(extra)
    d["flips"] = {k: list(v) for k, v in rep["flips"].items()}
    for k in ("errs", "cos", "rel"):
        if k in rep:
            d[k] = {kk: float(f"{vv:.4e}") for kk, vv in rep[k].items()}
    for k in ("L_real", "L_fake", "reg", "L_G", "img_real", "img_fake_D", "img_fake_G"):
        if k in rep:
            d[f"{k}_rel_err"] = rep[k]
    with open(os.path.join(out, f"{name}.json"), "w") as f:
        json.dump(d, f, indent=1)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name,s,B,alpha,steps", CONFIGS, ids=[c[0] for c in CONFIGS])
def test_fp32_step_matches_oracle_at_baseline_config(name, s, B, alpha, steps):
    eng, fpG, fpD = build(s, B, torch.float32, seed=500 + s)
    inputs = make_inputs(B, 4 * 2 ** s, seed=600 + s, n_steps=steps)
    for t, st in enumerate(inputs):
        real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
        t0 = time.time()
        ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, threads=THREADS)
        rep = K.compare(ours, ref, fpG, fpD, kinks, tol=1e-3,
                        flip_bound=K.FLIP_BOUND[torch.float32], ptol=1e-5,
                        what=f"{name} step {t}: ")
        msg = K.summarize(rep)
        print(f"\n{name} fp32 step {t} ({time.time() - t0:.0f}s incl. oracle): {msg}", flush=True)
        _report(f"{name}_fp32_step{t}", rep, dict(config=name, stage=s, batch=B, alpha=alpha,
                                                  mode="f32", oracle="float64 + injected kinks",
                                                  tol=1e-3, summary=msg))


@pytest.mark.timeout(900)
def test_fp32_wgan_gp_step_matches_oracle_at_c2():
    """C2 in the mode BASELINE.json names for it ("WGAN-GP on"): 128^2, B=16, alpha 1, the
    optional WGAN-GP loss (pggan/loss.py:54-100: BCE + W_gp * sum_b (|grad D(x_hat_b)| - 1)^2
    + W_drift_D * sum pred_real^2, configs.yaml:31-32), the interpolation / per-sample norm
    and its double-backward on the HIP kernels; every tensor at the strict fp32 bar."""
    from pggan_amd import engine as E
    s, B, alpha = 5, 16, 1.0
    eng, fpG, fpD = build(s, B, torch.float32, seed=705)
    eng.hyper = E.Hyper(gp_mode="wgan-gp", W_gp=10.0, W_drift=0.001)
    eng.bind(fpG, fpD, eng.hyper)
    st = make_inputs(B, 4 * 2 ** s, seed=805, n_steps=1)[0]
    real, z1, z2, eps = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2", "gp_eps"))
    ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, gp_eps=eps, threads=THREADS)
    rep = K.compare(ours, ref, fpG, fpD, kinks, tol=1e-3, flip_bound=K.FLIP_BOUND[torch.float32],
                    ptol=1e-5, what="C2 WGAN-GP: ")
    assert ours["reg"] > 0.0 and ours["drift"] > 0.0
    msg = K.summarize(rep)
    print(f"\nC2 WGAN-GP fp32: {msg}", flush=True)
    _report("C2_wgangp_fp32", rep, dict(config="C2", stage=s, batch=B, alpha=alpha, mode="f32",
                                        loss="wgan-gp", oracle="float64 + injected kinks",
                                        tol=1e-3, summary=msg))


@pytest.mark.timeout(900)
def test_bf16_bench_path_matches_oracle_at_c5():
    """The benchmarked configuration itself (bench.py: 1024^2, B=4, alpha 1, bf16)."""
    s, B, alpha = 8, 4, 1.0
    eng, fpG, fpD = build(s, B, torch.bfloat16, seed=508)
    st = make_inputs(B, 4 * 2 ** s, seed=608, n_steps=1)[0]
    real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
    ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, threads=THREADS,
                                  feed_images=True)
    rep = K.compare_bf16(ours, ref, fpG, fpD, kinks, loss_rtol=2e-3, min_cos=0.999,
                         flip_bound=K.FLIP_BOUND[torch.bfloat16], img_rtol=3e-2,
                         what="C5 bf16: ")
    msg = K.summarize(rep)
    print(f"\nC5 bf16: {msg}", flush=True)
    _report("C5_bf16", rep, dict(config="C5", stage=s, batch=B, alpha=alpha, mode="bf16",
                                 oracle="float64 + injected kinks", loss_rtol=2e-3,
                                 min_cos=0.999, img_rtol=3e-2, summary=msg))
