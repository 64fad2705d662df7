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


def rms(a, b):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    return float(np.sqrt(np.mean((a - b) ** 2))) if a.size else 0.0


def check_tensor(z, key, got, rtol, what="", atol=0.0):
    """Compare `got` (full array) with a fixture entry stored full or as samples+norm.
    Passes when the relative L2 error <= rtol OR the RMS error <= atol (atol guards
    tensors whose value is a near-cancelling sum, e.g. a bias gradient ~1e-5)."""
    got = np.asarray(got, np.float32)
    if key in z.files:
        ref = z[key]
        assert ref.shape == got.shape, f"{what}{key}: shape {got.shape} vs {ref.shape}"
        err = rel_l2(got, ref)
        assert err <= rtol or rms(got, ref) <= atol, \
            f"{what}{key}: rel L2 err {err:.3e} > {rtol:.1e} (rms {rms(got, ref):.3e})"
        return err
    idx, val, nrm = z[key + "#idx"], z[key + "#val"], z[key + "#norm"][0]
    flat = got.reshape(-1)
    gn = float(np.linalg.norm(flat.astype(np.float64)))
    assert abs(gn - nrm) <= rtol * max(nrm, 1e-30) + atol * np.sqrt(flat.size) + 1e-30, \
        f"{what}{key}: norm {gn:.6e} vs {nrm:.6e}"
    err = rel_l2(flat[idx], val)
    assert err <= max(rtol, 1e-6) * 10 or rms(flat[idx], val) <= atol, \
        f"{what}{key}: sampled rel err {err:.3e}"
    return err


def kink_robust_err(got, ref, frac=1e-3):
    """Relative L2 error after dropping the `frac` largest |differences|.

    A leaky-relu kink whose pre-activation is ~1e-7 from zero flips sign under any
    change of summation order; with 1e5-1e6 pre-activations per layer a few flips are
    expected, and each perturbs a small neighbourhood of the gradient (measured: 70 of
    196608 elements of dL/dimg in the 128^2 tiny config).  This metric checks the other
    99.9% strictly; callers also bound the plain relative error."""
    a = np.asarray(got, np.float64).ravel()
    b = np.asarray(ref, np.float64).ravel()
    d = np.abs(a - b)
    k = int(d.size * frac)
    if k:
        keep = np.argsort(d)[:d.size - k]
        a, b = a[keep], b[keep]
    return rel_l2(a, b)


def assert_close(got, ref, tol, what="", cap=1e-2, atol=0.0):
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float32)
    assert got.shape == ref.shape, f"{what}: shape {got.shape} vs {ref.shape}"
    e = rel_l2(got, ref)
    if e <= tol or rms(got, ref) <= atol:
        return e
    er = kink_robust_err(got, ref)
    assert er <= tol and e <= cap, f"{what}: rel err {e:.3e}, kink-robust {er:.3e} (tol {tol:.1e})"
    return e
