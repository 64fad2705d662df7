"""Helpers to load golden fixtures and compare results (test infrastructure)."""
import ast
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = ast.literal_eval(bytes(z["meta"]).decode())
    return meta, z


def rel_l2(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    den = max(np.linalg.norm(b), 1e-30)
    return float(np.linalg.norm(a - b) / den)


def check_tensor(z, key, got, rtol, what=""):
    """Compare `got` (full array) with a fixture entry stored full or as samples+norm."""
    got = np.asarray(got, np.float32)
    if key in z.files:
        ref = z[key]
        assert ref.shape == got.shape, f"{what}{key}: shape {got.shape} vs {ref.shape}"
        err = rel_l2(got, ref)
        assert err <= rtol, f"{what}{key}: rel L2 err {err:.3e} > {rtol:.1e}"
        return err
    idx, val, nrm = z[key + "#idx"], z[key + "#val"], z[key + "#norm"][0]
    flat = got.reshape(-1)
    gn = float(np.linalg.norm(flat.astype(np.float64)))
    assert abs(gn - nrm) <= rtol * max(nrm, 1e-30) + 1e-30, \
        f"{what}{key}: norm {gn:.6e} vs {nrm:.6e}"
    err = rel_l2(flat[idx], val)
    assert err <= max(rtol, 1e-6) * 10, f"{what}{key}: sampled rel err {err:.3e}"
    return err
