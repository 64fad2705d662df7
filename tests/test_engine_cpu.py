"""Host-logic test: the hand-scheduled step of pggan_amd/engine.py (explicit
forward / input-gradient / tangent / second backward for the R1 double-backward)
reproduces the reference's autograd step (golden fixtures), with the CPU test
double standing in for the HIP ops.  GPU parity of the kernels themselves is in
test_gpu_parity.py."""
import pytest
import torch

from cpu_ops import CpuOps
from gen_inputs import GOLDEN_CONFIGS, make_inputs, make_params
import kink_parity as K
from golden_utils import load
from oracle import pggan_oracle as O
from pggan_amd import engine as E

NAMES = [c[0] for c in GOLDEN_CONFIGS]


def build(meta, ops, device="cpu", **opts):
    depths, s, B = meta["depths"], meta["s"], meta["B"]
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = make_params(gsh, seed=1000 + 10 * s + B)
    PD = make_params(dsh, seed=2000 + 10 * s + B)
    fpG = E.FlatParams(gsh, E.dead_params("G", s), device,
                       {k: torch.from_numpy(v) for k, v in PG.items()})
    fpD = E.FlatParams(dsh, E.dead_params("D", s), device,
                       {k: torch.from_numpy(v) for k, v in PD.items()})
    eng = E.StepEngine(ops, depths, s, B, device, **opts)
    if device == "cpu":
        # exercise both sign-bit schedules at the fixture sizes: 8^2 keeps the conv-b bits for
        # the unpool pass (_ubits), >= 16^2 the full sign-bit path (_dbits)
        eng.dbits_min_res = 16
    eng.bind(fpG, fpD, E.Hyper())
    eng.keep_fake_D = True
    return eng, fpG, fpD


def run_and_check(meta, z, eng, fpG, fpD, tol, flip_bound=1e-4, ptol=1e-5, fixture_tol=1e-3):
    """Every step of a golden configuration, twice anchored:
      * strict: the oracle replayed (float64) from our state with our leaky-ReLU region
        choices injected; EVERY live D and G gradient, every image and loss within `tol`,
        parameters after both Adam steps within `ptol` (tests/kink_parity.py);
      * the reference's own outputs (fixture): within fixture_tol plus what the kink
        choice alone explains (kink_parity.check_fixture).
    Each step starts from our own state, so step 2 is checked as strictly as step 1."""
    s, B, alpha = meta["s"], meta["B"], meta["alpha"]
    steps = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B, n_steps=meta["n_steps"])
    reps = []
    for t, st in enumerate(steps):
        real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
        ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha)
        rep = K.compare(ours, ref, fpG, fpD, kinks, tol=tol, flip_bound=flip_bound, ptol=ptol,
                        what=f"step {t}: ")
        K.check_fixture(z, f"s{t}/", ours, ref, fpG, fpD, fixture_tol, what=f"step {t}: ")
        reps.append(rep)
    return reps


@pytest.mark.parametrize("name", NAMES)
def test_engine_schedule_matches_reference(name):
    torch.set_num_threads(4)
    meta, z = load(name)
    eng, fpG, fpD = build(meta, CpuOps())
    run_and_check(meta, z, eng, fpG, fpD, tol=1e-3)


def test_engine_schedule_unfused_pixelnorm():
    """The unfused generator path (conv -> u, separate PixelNorm kernel, backward from u)
    that the engine takes where the conv tile cannot hold every output channel."""
    torch.set_num_threads(4)
    name = [n for n in NAMES if n.startswith("tiny")][-1]
    meta, z = load(name)
    eng, fpG, fpD = build(meta, CpuOps(fused=False))
    run_and_check(meta, z, eng, fpG, fpD, tol=1e-3)


@pytest.mark.parametrize("name", ["tiny_s3_b4_a1", "tiny_s1_b4_a05"])
def test_engine_schedule_separate_generator_forwards(name):
    """Merged D passes with the G half's own generator forward (merge_g=False: the schedule
    the engine falls back to under a bucketed DP exchange) against the golden fixtures; the
    default (both generator forwards merged at batch 2B) is test_engine_schedule_matches_reference."""
    torch.set_num_threads(4)
    meta, z = load(name)
    eng, fpG, fpD = build(meta, CpuOps(), merge_g=False)
    assert eng.g2 is None and eng.dd2 is not None
    run_and_check(meta, z, eng, fpG, fpD, tol=1e-3)


def test_engine_options_env(monkeypatch):
    """PG_ENGINE (A/B runs) overrides the schedule defaults; unknown names raise."""
    monkeypatch.setenv("PG_ENGINE", "merge_g=0,dbits_min_res=64")
    o = E.engine_options()
    assert o["merge_g"] is False and o["dbits_min_res"] == 64 and o["merge_d"] is True
    monkeypatch.setenv("PG_ENGINE", "no_such_option=1")
    with pytest.raises(ValueError):
        E.engine_options()


GP_NAMES = ["gp_tiny_s2_b8_a03", "gp_tiny_s1_b4_a05"]


def build_gp(meta, ops, device="cpu"):
    """Engine in the optional WGAN-GP mode with the fixture's parameters (same seeds as
    make_golden.run_gp) and the reference configuration's W_gp / W_drift_D."""
    m = dict(meta, n_steps=1)
    eng, fpG, fpD = build(m, ops, device)
    eng.hyper = E.Hyper(gp_mode="wgan-gp", W_gp=10.0, W_drift=0.001)
    eng.bind(fpG, fpD, eng.hyper)
    return eng, fpG, fpD


def run_gp_and_check(name, ops, device="cpu", tol=1e-3, bf16=False):
    """The WGAN-GP step (BCE + penalty + drift in the D gradient, pggan/loss.py:54-100)
    against the kink-injected oracle replay, and the penalty / drift values against the
    reference's own functions on the same inputs (fixture)."""
    meta, z = load(name)
    eng, fpG, fpD = build_gp(meta, ops, device)
    s, B, alpha = meta["s"], meta["B"], meta["alpha"]
    st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B)[0]
    real, z1, z2, eps = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2", "gp_eps"))
    ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, gp_eps=eps,
                                  feed_images=bf16)
    if bf16:
        rep = K.compare_bf16(ours, ref, fpG, fpD, kinks, loss_rtol=2e-2, min_cos=0.99,
                             flip_bound=K.FLIP_BOUND[torch.bfloat16], img_rtol=5e-2)
    else:
        rep = K.compare(ours, ref, fpG, fpD, kinks, tol=tol, flip_bound=1e-4, ptol=1e-5)
        # the penalty and the drift against the reference's own get_gradient_penalty /
        # get_drift_loss, evaluated on the reference's images (our images match them)
        assert abs(ours["reg"] - z["gp"][0]) <= 2e-3 * abs(z["gp"][0]) + 1.05 * abs(ref["reg"] - z["gp"][0])
        assert abs(ours["drift"] - z["drift"][0]) <= 2e-3 * abs(z["drift"][0]) + 1e-9
    assert ours["drift"] > 0.0 and ours["reg"] > 0.0
    return rep


@pytest.mark.parametrize("name", GP_NAMES)
def test_engine_wgan_gp_step(name):
    torch.set_num_threads(4)
    run_gp_and_check(name, CpuOps())


def run_steps(ops_factory, device, depths, s, B, steps=2, elide=True):
    """`steps` training steps at alpha = 1 from fixed parameters and inputs: per step the
    three images, the loss vector, both flat gradients and both flat parameter buffers."""
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = {k: torch.from_numpy(v) for k, v in make_params(gsh, seed=61).items()}
    PD = {k: torch.from_numpy(v) for k, v in make_params(dsh, seed=62).items()}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), device, PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", s), device, PD)
    eng = E.StepEngine(ops_factory(), depths, s, B, device)
    eng.elide_zero_blend = elide
    eng.bind(fpG, fpD, E.Hyper())
    eng.keep_fake_D = True
    res = []
    for t, st in enumerate(make_inputs(B, 4 * 2 ** s, seed=63, n_steps=steps)):
        r, z1, z2 = (torch.from_numpy(st[k]).to(device) for k in ("real", "z1", "z2"))
        ims = eng.train_step(r, z1, z2, 1.0, 1.0)
        eng.flush()
        res.append([x.detach().cpu().clone() for x in ims] +
                   [eng.loss.cpu().clone(), fpD.grad.cpu().clone(), fpG.grad.cpu().clone(),
                    fpD.flat.cpu().clone(), fpG.flat.cpu().clone()])
    return res


STEP_TENSORS = ["img_real", "img_fake_D", "img_fake_G", "loss", "grad_D", "grad_G", "param_D",
                "param_G"]


def assert_runs_equal(out_a, out_b, rtol=0.0):
    """Per step and tensor: bitwise equal (rtol 0) or within rtol relative L2."""
    for t, (a, b) in enumerate(zip(out_a, out_b)):
        for name, x, y in zip(STEP_TENSORS, a, b):
            if rtol == 0.0:
                assert torch.equal(x, y), (f"step {t} {name}: {int((x != y).sum())} elements differ, "
                                           f"max {float((x - y).abs().max())}")
            else:
                e = float((x.double() - y.double()).norm() / max(float(y.double().norm()), 1e-30))
                assert e <= rtol, (t, name, e)


def elision_bitwise(ops_factory, device, depths, s, B, dtype=torch.float32, steps=2, rtol=0.0):
    """alpha = 1: eliding the fade-in's exactly-zero low-resolution branches (engine
    .elide_zero_blend) must leave every image, loss, gradient and parameter bit-identical
    to computing them (the reference computes them, pggan/nets.py:155-156,263-265).
    rtol > 0: where the elided schedule runs different (fused) kernels than the computed
    one -- bf16 storage, whose roundings then differ -- the two are held to rtol per tensor."""
    out = [run_steps(ops_factory, device, depths, s, B, steps, elide) for elide in (False, True)]
    assert_runs_equal(out[0], out[1], rtol)


def test_alpha_one_elision_is_bitwise():
    torch.set_num_threads(4)
    from gen_inputs import TINY_DEPTHS
    elision_bitwise(CpuOps, "cpu", TINY_DEPTHS, 3, 4)
