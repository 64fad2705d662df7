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


def build(meta, ops, device="cpu"):
    depths, s, B = meta["depths"], meta["s"], meta["B"]
    gsh, dsh = E.g_param_shapes(depths, s), E.d_param_shapes(depths, s)
    PG = make_params(gsh, seed=1000 + 10 * s + B)
    PD = make_params(dsh, seed=2000 + 10 * s + B)
    fpG = E.FlatParams(gsh, E.dead_params("G", s), device,
                       {k: torch.from_numpy(v) for k, v in PG.items()})
    fpD = E.FlatParams(dsh, E.dead_params("D", s), device,
                       {k: torch.from_numpy(v) for k, v in PD.items()})
    eng = E.StepEngine(ops, depths, s, B, device)
    if device == "cpu":
        eng.dbits_min_res = 8      # exercise the sign-bit schedule at the fixture sizes
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
