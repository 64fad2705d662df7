"""Deterministic synthetic parameters and inputs for parity tests (numpy PCG64).

Shared by ``make_golden.py`` (which feeds them to the imported reference) and
by the tests (which feed them to the oracle and to the HIP path), so no weight
tensors need to be committed.  Raw weights are N(0,1) like the reference init
(lib/layers.py:51-56); biases are small and nonzero (scaled N(0,1)) so the
equalized-LR bias scaling path (lib/layers.py:58-63) is exercised.
"""
import numpy as np

TINY_DEPTHS = [32, 32, 32, 32, 16, 16, 8, 8, 8]


def make_params(shapes, seed, bias_scale=0.1):
    rng = np.random.default_rng(seed)
    out = {}
    for name, shp in shapes:
        a = rng.standard_normal(shp, dtype=np.float32)
        if name.endswith("bias"):
            a = (a * np.float32(bias_scale)).astype(np.float32)
        out[name] = a
    return out


def make_inputs(B, res, seed, n_steps=1, latent_dim=512):
    """Per step: real images U[-1,1) [B,3,res,res] and two latents z ~ N(0,1) [B,latent]."""
    rng = np.random.default_rng(seed)
    steps = []
    for _ in range(n_steps):
        real = rng.uniform(-1.0, 1.0, size=(B, 3, res, res)).astype(np.float32)
        z1 = rng.standard_normal((B, latent_dim), dtype=np.float32)
        z2 = rng.standard_normal((B, latent_dim), dtype=np.float32)
        eps = rng.uniform(0.0, 1.0, size=(B, 1)).astype(np.float32)
        steps.append(dict(real=real, z1=z1, z2=z2, gp_eps=eps))
    return steps


# Golden configurations: (name, depths, stage s, batch B, alpha, n_steps, full tensors?)
GOLDEN_CONFIGS = [
    ("tiny_s0_b4", TINY_DEPTHS, 0, 4, 0.0, 2, True),
    ("tiny_s1_b4_a05", TINY_DEPTHS, 1, 4, 0.5, 2, True),
    ("tiny_s2_b8_a03", TINY_DEPTHS, 2, 8, 0.3, 2, True),
    ("tiny_s2_b6_a07", TINY_DEPTHS, 2, 6, 0.7, 1, True),     # 6 % 4 != 0 -> one group of 6
    ("tiny_s3_b4_a1", TINY_DEPTHS, 3, 4, 1.0, 2, True),
    ("tiny_s4_b2_a06", TINY_DEPTHS, 4, 2, 0.6, 1, True),
    ("tiny_s5_b4_a1", TINY_DEPTHS, 5, 4, 1.0, 1, True),
    ("tiny_s1_b1_a02", TINY_DEPTHS, 1, 1, 0.2, 1, True),     # group size 1 -> zero stddev channel
    ("full_s0_b16", None, 0, 16, 0.0, 1, False),              # C1 (paper depths)
    ("full_s2_b4_a05", None, 2, 4, 0.5, 1, False),
]
