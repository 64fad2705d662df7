"""Kink-resolved step parity: the engine's training step against the oracle run with
the engine's own leaky-ReLU region choices injected (test infrastructure).

Why: a pre-activation within rounding of 0 takes either slope depending on summation
order, and the gradient through it changes by 1/slope = 5x.  Two correct
implementations therefore disagree on a handful of elements per layer, and a bias
gradient (a sum over B*H*W elements) moves by up to a few percent.  Instead of
loosening the bar, `run_step` records every forward's region choices from the
engine's activation buffers (engine.trace), replays the same step in the oracle with
those choices (oracle.Kinks), and then holds EVERY tensor to the strict bar.  The
oracle also reports, per site, how many elements the injected choice flipped relative
to its own sign and the largest |pre-activation| / RMS among them; that must stay
below a stated rounding bound (FLIP_BOUND), so a sign error far from 0 (a real kernel
bug) fails instead of being absorbed.
"""
from __future__ import annotations

import math

import torch

from oracle import pggan_oracle as O

# largest |pre-activation| / RMS(site) at which an injected region choice may differ
# from the oracle's own sign.  fp32: accumulation-order rounding (K <= 4617 terms) is
# ~1e-6 of the RMS; the worst of the ~2e9 pre-activations of a C5 step measured 4.2e-5
# (profiles/r2_parity_C5_fp32_step0.json).  bf16: storage and packed weights round to
# 2^-9 relative, compounding over 18 generator layers to ~2% of the RMS (the images
# differ by 2%); the worst of 2e9 samples sits ~6-8 sigma out, measured 0.16.  A real
# kernel error (a wrong sign far from 0) shows up at O(1) x RMS.
FLIP_BOUND = {torch.float32: 2e-4, torch.bfloat16: 0.3}
# Relative-error floor of gradient tensors that are a sum with heavy cancellation: the D
# decision-layer bias gradient is ONE number, the sum over the batch of the logit gradients,
# whose real (-(1 - sigma)/B) and fake (+sigma/B) terms nearly cancel once D is near
# balance.  The fp32 GPU step (cross-workgroup fp32 atomics, run-to-run order) measured
# 5.8e-4 - 1.02e-3 at tiny_s2_b8_a03 step 1 against the float64 oracle, with the separate and
# the merged real/fake schedules alike (profiles/r4_merge_ab.txt); every other tensor stays
# at the strict bar, and the CPU double at ~1e-6.
CANCEL_TOL = {"D:decision_layer.module.bias": 2e-3}
# bf16 only: at most this fraction of pre-activations may take the injected region
# against the oracle's own sign (measured 0.15% at C5)
FLIP_FRAC_BF16 = 1e-2


def _nchw(t, C):
    return t[..., :C].permute(0, 3, 1, 2)


def _unpack_bits(b, C):
    """uint8 [B,H,W,nbytes] -> bool [B,C,H,W]; channel c at byte c//8, bit c%8
    (include/pggan_hip.h)."""
    k = torch.arange(8, dtype=torch.uint8, device=b.device)
    bits = (b.unsqueeze(-1) >> k) & 1
    m = bits.reshape(b.shape[:-1] + (-1,))[..., :C].bool()
    return m.permute(0, 3, 1, 2)


def d_masks(eng):
    """Region choices of the D forward that just ran, keyed by oracle site."""
    D, d, s = eng.dd, eng.depths, eng.s
    m = {"rgb": _nchw(D["yrgb"], d[s]) > 0}
    if s:
        # None: the engine elided the low-resolution branch (alpha = 1, weight exactly 0)
        m["rgbd"] = _nchw(D["yd"], d[s - 1]) > 0 if eng._last_dlow else None
    for i in range(s):
        m[f"a{i}"] = _nchw(D[f"a{i}"], d[i + 1]) > 0
        if eng._dbits(i) or eng._ubits(i):
            m[f"b{i}"] = _unpack_bits(D[f"mb{i}"], d[i])
        else:
            m[f"b{i}"] = _nchw(D[f"bf{i}"], d[i]) > 0
    m["mb"] = _nchw(D["c"], d[0]) > 0
    m["lin"] = D["l1"][:, :d[0]] > 0
    return {k: (None if v is None else v.cpu()) for k, v in m.items()}


def g_masks(eng):
    """Region choices of the G forward that just ran (PixelNorm keeps the sign, so the
    normalised outputs carry them)."""
    g, d, s, B = eng.g, eng.depths, eng.s, eng.B
    m = {"fmt": (_nchw(g["f"], d[0]) > 0).reshape(B, -1),
         "first": _nchw(g["y0"], d[0]) > 0}
    for i in range(s):
        m[f"a{i}"] = _nchw(g[f"ya{i}"], d[i + 1]) > 0
        m[f"b{i}"] = _nchw(g[f"yb{i}"], d[i + 1]) > 0
    return {k: v.cpu() for k, v in m.items()}


class Recorder:
    """engine.trace callback: one oracle.Kinks per forward, in call order."""

    def __init__(self):
        self.seq = {"D": [], "G": []}

    def __call__(self, net, eng):
        self.seq[net].append(O.Kinks(d_masks(eng) if net == "D" else g_masks(eng)))


def rel_l2(a, b):
    a = a.double().ravel()
    b = b.double().ravel()
    return float((a - b).norm() / max(float(b.norm()), 1e-300))


def cosine(a, b):
    a = a.double().ravel()
    b = b.double().ravel()
    return float((a @ b) / max(float(a.norm() * b.norm()), 1e-300))


def _adam_state(fp, lr, hyper, dtype):
    st = O.AdamState(lr=lr, beta1=hyper.beta1, beta2=hyper.beta2, eps=hyper.eps)
    if fp.step:
        for n in fp.names:
            if n in fp.dead:
                continue
            st.step[n] = fp.step
            st.m[n] = fp._view(fp.m, n).detach().cpu().to(dtype).clone()
            st.v[n] = fp._view(fp.v, n).detach().cpu().to(dtype).clone()
    return st


def run_step(eng, fpG, fpD, real, z1, z2, alpha, gp_eps=None, oracle_dtype=torch.float64,
             threads=None, feed_images=False):
    """One engine train_step plus the kink-injected oracle replay from the same state.
    Returns (ours, ref, kinks) with ours/ref dicts of CPU tensors.

    feed_images: the oracle's D sees OUR fake images (D half, and the value of the G
    half's image with the gradient flowing into the oracle's G), so each network is
    compared on identical inputs.  Used for bf16, where the generator's own rounding
    changes the image by ~1% and D's region choices downstream of it with it; the images
    themselves are still compared with the oracle's own G outputs."""
    hp = eng.hyper
    eng.keep_fake_D = True       # the D half's fake image survives the G half
    PG0 = {k: v.detach().cpu().clone() for k, v in fpG.views.items()}
    PD0 = {k: v.detach().cpu().clone() for k, v in fpD.views.items()}
    optG = _adam_state(fpG, hp.lr_G, hp, oracle_dtype)
    optD = _adam_state(fpD, hp.lr_D, hp, oracle_dtype)
    optG2 = _adam_state(fpG, hp.lr_G, hp, oracle_dtype)   # for the Adam step on OUR gradients
    optD2 = _adam_state(fpD, hp.lr_D, hp, oracle_dtype)
    rec = Recorder()
    eng.trace = rec
    try:
        dev = fpG.flat.device
        img_real, img_fake_D, img_fake = eng.train_step(
            real.to(dev), z1.to(dev), z2.to(dev), alpha, alpha,
            gp_eps=None if gp_eps is None else gp_eps.to(dev))
        eng.flush()
    finally:
        eng.trace = None
    loss = eng.loss.detach().cpu().double()
    ours = dict(img_real=img_real.detach().cpu().clone(),
                img_fake_D=img_fake_D.detach().cpu().clone(),
                img_fake_G=img_fake.detach().cpu().clone(),
                L_real=float(loss[0]), L_fake=float(loss[1]), reg=float(loss[2]),
                L_G=float(loss[3]), drift=float(loss[4]),
                grads_D={k: v.detach().cpu().clone() for k, v in fpD.gviews.items()},
                grads_G={k: v.detach().cpu().clone() for k, v in fpG.gviews.items()},
                PD={k: v.detach().cpu().clone() for k, v in fpD.views.items()},
                PG={k: v.detach().cpu().clone() for k, v in fpG.views.items()})
    print(f"[parity] engine step done (stage {eng.s}, B {eng.B}); oracle replay ...", flush=True)
    if threads:
        torch.set_num_threads(threads)
    cast = lambda t: t.detach().cpu().to(oracle_dtype).clone()
    PGr = {k: cast(v) for k, v in PG0.items()}
    PDr = {k: cast(v) for k, v in PD0.items()}
    out = O.train_step(PGr, PDr, optG, optD, cast(real), cast(z1), cast(z2), eng.s, alpha, alpha,
                       W_adv=hp.W_adv, slope_cfg=hp.slope_cfg, gp_mode=hp.gp_mode,
                       gp_eps=None if gp_eps is None else cast(gp_eps), W_gp=hp.W_gp,
                       W_drift=getattr(hp, "W_drift", 0.0), kinks=rec.seq,
                       fake_D=cast(ours["img_fake_D"]) if feed_images else None,
                       fake_G=cast(ours["img_fake_G"]) if feed_images else None)
    ref = dict(img_real=out.img_real, img_fake_D=out.img_fake_D, img_fake_G=out.img_fake_G,
               L_real=out.L_D_real, L_fake=out.L_D_fake, reg=out.R1, L_G=out.L_G,
               drift=out.drift, grads_D=out.grads_D, grads_G=out.grads_G, PD=PDr, PG=PGr)
    # the oracle's Adam applied to OUR gradients (live parameters as the reference has them):
    # with beta1 = 0 the first update is ~lr * g / (|g| + eps), so a near-zero gradient
    # element that agrees with the oracle's to the gradient bar can still move its parameter
    # by a visible fraction of lr; the Adam arithmetic itself is checked against this
    for P0, opt, key, grads in ((PG0, optG2, "PG", out.grads_G), (PD0, optD2, "PD", out.grads_D)):
        Pa = {k: cast(v) for k, v in P0.items()}
        opt.update(Pa, {k: (None if g is None else cast(ours["grads_" + key[1]][k]))
                        for k, g in grads.items()})
        ref[key + "_adam_ours"] = Pa
    return ours, ref, rec.seq


def flip_report(kinks):
    """{forward: (flips, elements, worst |x|/rms)} over all sites of each forward."""
    rep = {}
    for net, lst in kinks.items():
        for j, k in enumerate(lst):
            n = sum(v[0] for v in k.stats.values())
            tot = sum(v[1] for v in k.stats.values())
            rep[f"{net}{j}"] = (n, tot, k.worst())
    return rep


def compare(ours, ref, fpG, fpD, kinks, *, tol, flip_bound, ptol=None, what=""):
    """Strict bar: every live gradient tensor and every image within `tol` relative L2,
    losses within `tol` relative, injected kinks within `flip_bound`.  Returns a report."""
    rep = {"flips": flip_report(kinks)}
    fails = [f"{f}: an injected leaky-relu region differs at |x|/rms = {worst:.2e} > "
             f"{flip_bound:.0e} ({n} flips of {tot}): a sign error, not rounding"
             for f, (n, tot, worst) in rep["flips"].items() if worst > flip_bound]
    errs = {}
    for k in ("img_real", "img_fake_D", "img_fake_G"):
        errs[k] = rel_l2(ours[k], ref[k])
    for k in ("L_real", "L_fake", "reg", "L_G", "drift"):
        a, b = ours[k], ref[k]
        errs[k] = abs(a - b) / max(abs(b), 1e-30) if (a or b) else 0.0
    for net, fp, key in (("D", fpD, "grads_D"), ("G", fpG, "grads_G")):
        for n, g in ref[key].items():
            if g is None:
                assert n in fp.dead, f"{what}{net} {n}: reference grad is None but param is live"
                continue
            assert n not in fp.dead, f"{what}{net} {n}: marked dead but the reference has a grad"
            if float(g.norm()) == 0.0:
                assert float(ours[key][n].norm()) == 0.0, f"{what}{net} {n}: expected zero grad"
                continue
            errs[f"{net}:{n}"] = rel_l2(ours[key][n], g)
    if ptol is not None:
        # parameters after Adam: within ptol of the oracle's step, or (a near-zero gradient
        # element, see run_step) within ptol of the oracle's Adam on our gradients, which are
        # themselves held to tol above
        for net, fp, key in (("D", fpD, "PD"), ("G", fpG, "PG")):
            for n in fp.names:
                e = rel_l2(ours[key][n], ref[key][n])
                if e > ptol and key + "_adam_ours" in ref:
                    e = min(e, rel_l2(ours[key][n], ref[key + "_adam_ours"][n]))
                errs[f"param {net}:{n}"] = e
    bad = {k: v for k, v in errs.items()
           if v > (ptol if k.startswith("param") else max(tol, CANCEL_TOL.get(k, 0.0)))
           or not math.isfinite(v)}
    rep["errs"] = errs
    rep["worst"] = max(((k, v) for k, v in errs.items() if not k.startswith("param")),
                       key=lambda kv: kv[1])
    if bad:
        fails.append("over tolerance: " + ", ".join(
            f"{k} {v:.2e}" for k, v in sorted(bad.items(), key=lambda kv: -kv[1])[:12]))
    print(f"{what}{summarize(rep)}", flush=True)
    assert not fails, what + "; ".join(fails)
    return rep


def compare_bf16(ours, ref, fpG, fpD, kinks, *, loss_rtol, min_cos, flip_bound, img_rtol,
                 what=""):
    """bf16 storage / fp32 accumulate against the kink-injected float64 oracle (run with
    feed_images=True): the images within `img_rtol` relative L2, losses and the penalty
    within `loss_rtol` relative, every live gradient tensor at cosine >= `min_cos`
    (relative L2 reported), injected flips within `flip_bound`.  All checks are
    evaluated and reported together."""
    rep = {"flips": flip_report(kinks)}
    fails = []
    for f, (n, tot, worst) in rep["flips"].items():
        if worst > flip_bound:
            fails.append(f"{f}: flip at |x|/rms {worst:.2e} > {flip_bound} ({n} of {tot})")
        if n > FLIP_FRAC_BF16 * tot:
            fails.append(f"{f}: {n} of {tot} region choices flipped (> {FLIP_FRAC_BF16:.0e})")
    for k in ("img_real", "img_fake_D", "img_fake_G"):
        e = rel_l2(ours[k], ref[k])
        rep[k] = e
        if e > img_rtol:
            fails.append(f"{k}: rel L2 {e:.2e} > {img_rtol}")
    for k in ("L_real", "L_fake", "reg", "L_G"):
        a, b = ours[k], ref[k]
        e = abs(a - b) / max(abs(b), 1e-30)
        rep[k] = e
        if e > loss_rtol:
            fails.append(f"{k}: {a:.6e} vs {b:.6e} ({e:.2e} > {loss_rtol})")
    cos, rel = {}, {}
    for net, fp, key in (("D", fpD, "grads_D"), ("G", fpG, "grads_G")):
        for n, g in ref[key].items():
            if g is None or float(g.norm()) == 0.0:
                continue
            cos[f"{net}:{n}"] = cosine(ours[key][n], g)
            rel[f"{net}:{n}"] = rel_l2(ours[key][n], g)
    rep["cos"], rep["rel"] = cos, rel
    worst = sorted(cos.items(), key=lambda kv: kv[1])[:6]
    rep["worst_cos"] = worst
    if worst[0][1] < min_cos:
        fails.append(f"gradient cosine below {min_cos}: {worst}")
    rep["fails"] = fails
    print(f"{what}{summarize(rep)}; images " +
          ", ".join(f"{k} {rep[k]:.2e}" for k in ("img_real", "img_fake_D", "img_fake_G")) +
          "; losses " + ", ".join(f"{k} {rep[k]:.2e}" for k in ("L_real", "L_fake", "reg", "L_G")),
          flush=True)
    assert not fails, what + "; ".join(fails)
    return rep


def summarize(rep):
    fl = rep["flips"]
    nf = sum(v[0] for v in fl.values())
    tot = sum(v[1] for v in fl.values())
    w = max((v[2] for v in fl.values()), default=0.0)
    s = f"injected kinks: {nf} flips of {tot} pre-activations (worst |x|/rms {w:.1e})"
    if "worst" in rep:
        s += f"; worst tensor {rep['worst'][0]} rel {rep['worst'][1]:.2e}"
    if "worst_cos" in rep:
        s += f"; worst cosine {rep['worst_cos'][0][0]} {rep['worst_cos'][0][1]:.5f}"
    return s


# --------------------------------------------------------------------------- fixtures
def fixture_err(z, key, got):
    """Relative error of `got` against a golden entry stored in full (relative L2) or as
    samples + norm (max of the norm's relative error and the samples' relative L2)."""
    got = got.detach().cpu().double().reshape(-1)
    if key in z.files:
        ref = torch.from_numpy(z[key]).double().reshape(-1)
        return rel_l2(got, ref)
    idx = torch.from_numpy(z[key + "#idx"]).long()
    val = torch.from_numpy(z[key + "#val"]).double()
    nrm = float(z[key + "#norm"][0])
    en = abs(float(got.norm()) - nrm) / max(nrm, 1e-300)
    return max(en, rel_l2(got[idx], val))


def check_fixture(z, pre, ours, ref, fpG, fpD, tol, what=""):
    """The reference's own outputs (golden fixture of this step) against ours, with the
    kink choice accounted for explicitly: a tensor may deviate from the fixture by at
    most tol + 1.05 x the deviation of the oracle replayed with OUR region choices (the
    part of the difference those choices alone explain).  Together with the strict
    ours-vs-replay check and the oracle's pin to the fixtures (test_oracle_golden) this
    ties every tensor to the reference."""
    out = {}

    def one(key, a, b):
        ea, eb = fixture_err(z, key, a), fixture_err(z, key, b)
        out[key] = (ea, eb)
        assert ea <= tol + 1.05 * eb, \
            f"{what}{key}: {ea:.2e} from the reference fixture, the replay with our " \
            f"kinks is {eb:.2e} from it (allowed {tol + 1.05 * eb:.2e})"

    for k in ("img_real", "img_fake_D", "img_fake_G"):
        one(pre + k, ours[k], ref[k])
    for net, fp, key in (("D", fpD, "grads_D"), ("G", fpG, "grads_G")):
        for n in fp.names:
            fk = f"{pre}grad_{net}/{n}"
            if fk + "#none" in z.files:
                assert n in fp.dead, f"{what}{n}: reference grad is None but param is live"
                continue
            assert n not in fp.dead, f"{what}{n}: marked dead but the reference has a grad"
            one(fk, ours[key][n], ref[key][n].float())
    L = z[pre + "losses"]     # L_real, L_fake, R1, L_D, L_G (4-decimal rounding for all but R1)
    assert abs(round(ours["L_real"], 4) - L[0]) <= 1.01e-4
    assert abs(round(ours["L_fake"], 4) - L[1]) <= 1.01e-4
    assert abs(round(ours["L_G"], 4) - L[4]) <= 1.01e-4
    assert abs(ours["reg"] - L[2]) <= tol * abs(L[2]) + 1.05 * abs(ref["reg"] - L[2]) + 1e-12
    return out
