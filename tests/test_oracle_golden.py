"""Pin the CPU oracle (oracle/pggan_oracle.py) to the reference's own outputs.

The fixtures in tests/golden/*.npz were produced by running the reference's
ProgressiveGAN.train_step (pggan/model.py:206-255) in the build container
(tests/golden/make_golden.py).  Here the oracle restatement must reproduce
them: images, logits, R1, losses, every D/G gradient (incl. which are None)
and the post-Adam parameters, over 1-2 consecutive steps.
"""
import numpy as np
import pytest
import torch

from gen_inputs import GOLDEN_CONFIGS, make_inputs, make_params
from golden_utils import check_tensor, load
from oracle import pggan_oracle as O

NAMES = [c[0] for c in GOLDEN_CONFIGS]


def run_oracle(meta, step_cb):
    depths, s, B, alpha = meta["depths"], meta["s"], meta["B"], meta["alpha"]
    PG = {k: torch.from_numpy(v) for k, v in
          make_params(O.g_param_shapes(depths, s), seed=1000 + 10 * s + B).items()}
    PD = {k: torch.from_numpy(v) for k, v in
          make_params(O.d_param_shapes(depths, s), seed=2000 + 10 * s + B).items()}
    optG, optD = O.AdamState(lr=1e-4), O.AdamState(lr=1e-5)
    steps = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B, n_steps=meta["n_steps"])
    for t, st in enumerate(steps):
        out = O.train_step(PG, PD, optG, optD, torch.from_numpy(st["real"]),
                           torch.from_numpy(st["z1"]), torch.from_numpy(st["z2"]),
                           s, alpha, alpha)
        step_cb(t, out, PG, PD)


@pytest.mark.parametrize("name", NAMES)
def test_oracle_matches_reference(name):
    torch.set_num_threads(4)
    meta, z = load(name)
    tol = 2e-5

    def cb(t, out, PG, PD):
        pre = f"s{t}/"
        for k in ("img_real", "img_fake_D", "img_fake_G", "pred_real", "pred_fake",
                  "pred_fake_G"):
            check_tensor(z, pre + k, getattr(out, k).numpy(), tol)
        L = z[pre + "losses"]
        assert abs(out.R1 - L[2]) <= 1e-5 * abs(L[2]) + 1e-12
        # loss_dict values are rounded to 4 d.p. by the reference (pggan/loss.py:12,23-25)
        for got, ref in ((out.L_D_real, L[0]), (out.L_D_fake, L[1]), (out.L_D, L[3]),
                         (out.L_G, L[4])):
            assert abs(round(got, 4) - ref) <= 1.01e-4
        for net, grads, P in (("D", out.grads_D, PD), ("G", out.grads_G, PG)):
            for k, g in grads.items():
                key = f"{pre}grad_{net}/{k}"
                if g is None:
                    assert key + "#none" in z.files, f"{key} is None in oracle only"
                    continue
                assert key + "#none" not in z.files, f"{key} is None in reference only"
                check_tensor(z, key, g.numpy(), tol)
            for k, p in P.items():
                check_tensor(z, f"{pre}param_{net}/{k}", p.numpy(), 1e-6)

    run_oracle(meta, cb)


GP_NAMES = ["gp_tiny_s2_b8_a03", "gp_tiny_s1_b4_a05"]


@pytest.mark.parametrize("name", GP_NAMES)
def test_oracle_wgan_gp_matches_reference(name):
    """The optional WGAN-GP mode: the oracle's penalty and drift against the reference's
    own get_gradient_penalty / get_drift_loss (pggan/loss.py:54-100; fixture made by
    tests/golden/make_golden.py with the SURVEY §8(c) get_device patch): the penalty
    value, its gradient w.r.t. every D parameter (backward=True), and the drift value."""
    torch.set_num_threads(4)
    meta, z = load(name)
    depths, s, B, alpha = meta["depths"], meta["s"], meta["B"], meta["alpha"]
    PD = {k: torch.from_numpy(v).requires_grad_() for k, v in
          make_params(O.d_param_shapes(depths, s), seed=2000 + 10 * s + B).items()}
    st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B)[0]
    xr, xf = torch.from_numpy(z["img_real"]), torch.from_numpy(z["img_fake"])
    pred_real = O.discriminator_forward(PD, xr, s, alpha)
    check_tensor(z, "pred_real", pred_real.detach().numpy(), 2e-5)
    gp = O.wgan_gp(lambda t: O.discriminator_forward(PD, t, s, alpha), xr, xf,
                   torch.from_numpy(st["gp_eps"]), float(z["W_gp"][0]))
    assert abs(float(gp) - z["gp"][0]) <= 1e-5 * abs(z["gp"][0])
    names = list(PD)
    grads = torch.autograd.grad(gp, [PD[k] for k in names], allow_unused=True)
    for k, g in zip(names, grads):
        key = f"grad_D/{k}"
        if g is None:
            assert key + "#none" in z.files, k
            continue
        check_tensor(z, key, g.numpy(), 1e-4)
    drift = O.drift_loss(pred_real, float(z["W_drift_D"][0]))
    assert abs(float(drift) - z["drift"][0]) <= 1e-5 * abs(z["drift"][0]) + 1e-12
