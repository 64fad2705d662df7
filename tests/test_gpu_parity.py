"""Step-level parity on the GPU: the HIP training step against the reference's golden
vectors and the CPU oracle, through the C ABI.

* golden configs (tests/golden), fp32 mode, every step: the oracle replayed in float64
  from our state with our leaky-ReLU region choices injected -- EVERY live D and G
  gradient, the images, losses and R1 within 1e-3 relative, parameters after both Adam
  steps within 1e-5 -- and the reference's own outputs within 1e-3 plus what the region
  choice alone explains (tests/kink_parity.py, test_engine_cpu.run_and_check).
* full-width stages 32^2 / 64^2: the same strict replay check.
* bf16 perf mode at the golden configs: losses / R1 within 2%, every gradient tensor at
  cosine >= 0.99 with the replay.  The BASELINE-size configs are in
  test_gpu_baseline_parity.py.
"""
import pytest
import torch

import kink_parity as K
from gen_inputs import GOLDEN_CONFIGS, make_inputs
from golden_utils import load
from oracle import pggan_oracle as O
from test_engine_cpu import run_and_check

pytestmark = pytest.mark.gpu

NAMES = [c[0] for c in GOLDEN_CONFIGS]


def gpu_build(meta, dtype):
    from pggan_amd import _lib
    from test_engine_cpu import build
    return build(meta, _lib.HipOps(dtype), device="cuda")


@pytest.mark.parametrize("name", NAMES)
def test_hip_step_matches_reference_fp32(name):
    meta, z = load(name)
    eng, fpG, fpD = gpu_build(meta, torch.float32)
    reps = run_and_check(meta, z, eng, fpG, fpD, tol=1e-3)
    print(name, [K.summarize(r) for r in reps])


@pytest.mark.parametrize("s,B,alpha", [(3, 4, 0.5), (4, 4, 1.0)])
def test_hip_step_full_width_vs_oracle(s, B, alpha):
    meta = dict(depths=O.PAPER_DEPTHS, s=s, B=B, alpha=alpha, n_steps=1)
    eng, fpG, fpD = gpu_build(meta, torch.float32)
    st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B, n_steps=1)[0]
    real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
    ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, threads=8)
    rep = K.compare(ours, ref, fpG, fpD, kinks, tol=1e-3, flip_bound=K.FLIP_BOUND[torch.float32],
                    ptol=1e-5)
    print(K.summarize(rep))


@pytest.mark.parametrize("name", ["tiny_s2_b8_a03", "tiny_s5_b4_a1", "full_s2_b4_a05"])
def test_hip_step_bf16_vs_oracle(name):
    """bf16 storage / fp32 accumulate against the replay of the oracle with the bf16
    forward's own region choices."""
    meta, _ = load(name)
    eng, fpG, fpD = gpu_build(meta, torch.bfloat16)
    s, B, alpha = meta["s"], meta["B"], meta["alpha"]
    st = make_inputs(B, 4 * 2 ** s, seed=3000 + 10 * s + B, n_steps=1)[0]
    real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
    ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, alpha, threads=8,
                                   feed_images=True)
    rep = K.compare_bf16(ours, ref, fpG, fpD, kinks, loss_rtol=2e-2, min_cos=0.99,
                         flip_bound=K.FLIP_BOUND[torch.bfloat16], img_rtol=5e-2)
    print(K.summarize(rep))


@pytest.mark.parametrize("name", ["gp_tiny_s2_b8_a03", "gp_tiny_s1_b4_a05"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_hip_wgan_gp_step(name, dtype):
    """The optional WGAN-GP mode on the HIP kernels (interpolate -> D -> per-sample gradient
    norm -> double-backward, plus the drift term): kink-resolved against the oracle, and the
    penalty / drift against the reference's own get_gradient_penalty / get_drift_loss."""
    from pggan_amd import _lib
    from test_engine_cpu import run_gp_and_check
    rep = run_gp_and_check(name, _lib.HipOps(dtype), device="cuda",
                           bf16=dtype == torch.bfloat16)
    print(K.summarize(rep))


@pytest.mark.parametrize("dtype,s,rtol", [(torch.float32, 3, 1e-6), (torch.bfloat16, 6, 1e-3)],
                         ids=["f32", "bf16"])
def test_alpha_one_elision_on_hip(dtype, s, rtol):
    """The benchmark runs at alpha = 1 with the exactly-zero fade-in branches elided; the
    HIP step must equal computing them, over two steps.  Bitwise on the CPU double
    (test_engine_cpu); here the two schedules run different kernels where the branch is
    computed -- the toRGB output with the fade-in term sums its channels in another order
    (fp32: last-bit differences of the image, 1e-6), the elided generator backward runs the
    toRGB input gradient fused with the top PixelNorm backward (fp32 in registers) where the
    computed branch stores dL/dy in bf16 (bf16 at paper widths, 256^2: 1e-3).  Each run is
    itself bitwise reproducible (test_step_bitwise_reproducible)."""
    from pggan_amd import _lib
    from gen_inputs import TINY_DEPTHS
    from test_engine_cpu import elision_bitwise
    depths = TINY_DEPTHS if dtype == torch.float32 else O.PAPER_DEPTHS
    elision_bitwise(lambda: _lib.HipOps(dtype), "cuda", depths, s, 4, dtype, rtol=rtol, steps=2)


@pytest.mark.parametrize("dtype,s,B", [(torch.bfloat16, 6, 4), (torch.bfloat16, 8, 4),
                                       (torch.float32, 5, 4)], ids=["bf16-256", "bf16-1024", "f32-128"])
def test_step_bitwise_reproducible(dtype, s, B):
    """Two runs of the default schedule (the benchmarked one: merged passes, side stream,
    sign-bit tiles, alpha = 1 elision) from the same parameters and inputs are BITWISE equal
    over two steps -- images, losses, every gradient and parameter.  Every reduction over
    workgroups sums in a fixed order (det_commit, the slab reductions), so nothing depends on
    the order the workgroups or the two streams finish (pggan/model.py:206-255 is a
    deterministic CPU step)."""
    from pggan_amd import _lib
    from test_engine_cpu import assert_runs_equal, run_steps
    runs = [run_steps(lambda: _lib.HipOps(dtype), "cuda", O.PAPER_DEPTHS, s, B, steps=2)
            for _ in range(2)]
    assert_runs_equal(runs[0], runs[1], rtol=0.0)
