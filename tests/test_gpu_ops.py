"""Kernel-level parity: every HIP entry point (via pggan_amd._lib.HipOps) against the
CPU test double on identical random inputs.  fp32 mode must agree to ~1e-5
(exact-fp32 MFMA, different summation order); bf16 mode to bf16 rounding."""
import itertools

import pytest
import torch

from cpu_ops import CpuOps, cinp, r16
from cpu_ops import packbits as cpu_packbits
from golden_utils import rel_l2

pytestmark = pytest.mark.gpu

L = None


def lib():
    global L
    if L is None:
        from pggan_amd import _lib
        L = _lib
    return L


def rnd(*shape, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return torch.randn(*shape, generator=g) * scale


def ops_pair(dtype):
    return lib().HipOps(dtype), CpuOps()


def cmp(a_gpu, b_cpu, tol, what):
    a = a_gpu.float().cpu().numpy()
    b = b_cpu.float().numpy()
    e = rel_l2(a, b)
    assert e <= tol, f"{what}: rel err {e:.3e} > {tol:.1e}"


def tol_for(dtype, base=2e-5):
    return base if dtype == torch.float32 else 2e-2


def q(t, dtype):
    """round a CPU fp32 tensor through the storage dtype (so both sides see the same data)"""
    return t.to(dtype).float()


CONV_CASES = [
    # (B, H, cin, cout, flags)
    (2, 8, 32, 32, ("bias", "lrelu")),
    (3, 4, 64, 64, ("bias", "lrelu")),          # tiny images, several per tile, ragged B
    (2, 16, 16, 16, ("ups", "bias", "lrelu")),
    (1, 32, 8, 8, ("bias", "lrelu")),
    (2, 16, 32, 64, ("bias", "lrelu", "pool")),
    (2, 32, 64, 32, ("mask",)),
    (2, 8, 128, 48, ("accum",)),
    (1, 64, 16, 32, ("pool", "accum")),
    (4, 4, 33, 32, ("bias", "lrelu")),          # mbstd-style padded cin (33 -> 64)
    (2, 8, 32, 20, ("bias",)),                  # cout not a multiple of 16
    # H, W >= 16: the compile-time-geometry kernel (conv_hr.inc), persistent when cin <= 32
    (2, 32, 16, 16, ("bias", "lrelu")),
    (2, 32, 16, 32, ("ups", "bias", "lrelu")),
    (2, 32, 32, 16, ("mask",)),
    (2, 32, 16, 32, ("bias", "lrelu", "pool")),
    (1, 64, 32, 64, ("bias", "lrelu", "pool")),
    (2, 64, 64, 32, ("mask", "accum")),
    (1, 32, 128, 64, ("bias", "lrelu")),
    (2, 16, 16, 16, ("mask", "accum")),
    (4, 512, 16, 16, ("bias", "lrelu")),        # > 2048 tiles: several tiles per workgroup
    (4, 512, 32, 16, ("mask",)),
    (4, 512, 16, 32, ("ups", "bias", "lrelu", "pool")),
    # wide 8-wave tile (conv_hr tile 3, LDS-DMA double-buffered staging): >= 256 tiles
    (4, 128, 64, 128, ("bias", "lrelu")),
    (8, 128, 64, 64, ("ups", "bias", "lrelu", "pool")),
    (4, 128, 128, 128, ("mask", "accum")),
    # tile 3 with more tiles than one round of workgroups (one tile per workgroup): one chunk
    # with the pre-pool copy, two chunks x two output-channel blocks, two chunks with bias
    (4, 256, 32, 64, ("bias", "lrelu", "pool")),
    (2, 256, 64, 128, ("mask", "accum")),
    (4, 256, 64, 64, ("bias", "lrelu")),
    # the generator's input gradient through its 512^2 conv a (32 -> 64, pooled)
    (2, 256, 32, 64, ("pool",)),
]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3x3_fwd(case, dtype):
    B, H, cin, cout, fl = case
    _L = lib()
    hip, cpu = ops_pair(dtype)
    flags = 0
    for f, v in (("ups", _L.CONV_UPS_IN), ("bias", _L.CONV_BIAS), ("lrelu", _L.CONV_LRELU),
                 ("mask", _L.CONV_MASK), ("pool", _L.CONV_POOL), ("accum", _L.CONV_ACCUM)):
        if f in fl:
            flags |= v
    Hin = H // 2 if "ups" in fl else H
    xcs = cinp(cin)
    x = q(rnd(B, Hin, Hin, xcs, seed=1), dtype)
    x[..., cin:] = 0
    w = rnd(cout, cin, 3, 3, seed=2)
    bias = rnd(cout, seed=3) * 0.1
    Ho = H // 2 if "pool" in fl else H
    ycs = cout + 4
    y0 = q(rnd(B, Ho, Ho, ycs, seed=4), dtype)
    aux = q(rnd(B, H, H, cout, seed=5), dtype)
    scale = 0.05
    outs = []
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        wp = torch.zeros(ops.packed_elems(0, cout, cin), dtype=dtype if dev == "cuda" else torch.float32,
                         device=dev)
        ops.conv_pack(0, w.to(dev), scale, wp)
        y = y0.to(dev).to(wp.dtype).clone()
        y2 = torch.zeros(B, H, H, cout, dtype=wp.dtype, device=dev) if "pool" in fl else None
        ops.conv3x3(x.to(dev).to(wp.dtype), wp, y, B=B, H=H, W=H, cin=cin, cout=cout, flags=flags,
                    slope=0.2, out_scale=0.25 if "pool" in fl else 1.0,
                    bias=(bias * scale).to(dev), aux=aux.to(dev).to(wp.dtype), y2=y2)
        outs.append((y, y2))
    cmp(outs[0][0], outs[1][0], tol_for(dtype), "conv y")
    if outs[0][1] is not None:
        cmp(outs[0][1], outs[1][1], tol_for(dtype), "conv y2")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(2, 8, 32, 48), (2, 16, 16, 16), (3, 4, 513, 512), (1, 32, 8, 8)])
def test_conv3x3_dgrad_pack(case, dtype):
    """dgrad = conv with the PACK_DGRAD layout (flipped / transposed weights)."""
    B, H, cin, cout = case
    hip, cpu = ops_pair(dtype)
    w = rnd(cout, cin, 3, 3, seed=7)
    gz = q(rnd(B, H, H, cinp(cout), seed=8), dtype)
    gz[..., cout:] = 0
    outs = []
    cout_d = (cin + 3) // 4 * 4
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        wp = torch.zeros(ops.packed_elems(1, cout, cin), dtype=dt, device=dev)
        ops.conv_pack(1, w.to(dev), 0.1, wp)
        y = torch.zeros(B, H, H, cinp(cin), dtype=dt, device=dev)
        ops.conv3x3(gz.to(dev).to(dt), wp, y, B=B, H=H, W=H, cin=cout, cout=cout_d, flags=0)
        outs.append(y)
    cmp(outs[0], outs[1], tol_for(dtype), "dgrad")


WGRAD_CASES = [(2, 8, 32, 48, False), (2, 16, 16, 16, True), (4, 4, 513, 512, False),
               (1, 64, 8, 8, False), (2, 32, 64, 32, True),
               # bench-like: many pixel splits (slabs), direct single split, ups + cin 32
               (4, 128, 16, 32, False), (4, 32, 512, 512, False), (2, 64, 32, 16, True),
               (4, 64, 64, 128, False),
               # the 16^2 wide layer (the register-staged kernel) and the LDS-DMA kernel with ups
               (4, 16, 512, 512, False), (2, 64, 256, 128, True)]


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("use_ws", [True, False])
@pytest.mark.parametrize("case", WGRAD_CASES)
def test_conv3x3_wgrad(case, dtype, use_ws):
    """Weight + fused bias gradient.  With a workspace the pixel splits write fp32 slabs
    summed in split order by the reduction launch; without one the plan runs one split.  Both
    are deterministic."""
    B, H, cin, cout, ups = case
    hip, cpu = ops_pair(dtype)
    Hin = H // 2 if ups else H
    x = q(rnd(B, Hin, Hin, cinp(cin), seed=11), dtype)
    gz = q(rnd(B, H, H, cout, seed=12), dtype)
    outs = []
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        dw = torch.full((cout, cin, 3, 3), 0.5, device=dev)
        db = torch.full((cout,), 0.25, device=dev)
        ws = None
        if use_ws and dev == "cuda":
            nb = ops.wgrad_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout, ups=ups)
            ws = torch.full((max(nb // 4, 1),), float("nan"), device=dev)
        ops.conv_wgrad(x.to(dev).to(dt), gz.to(dev).to(dt), dw, B=B, H=H, W=H, cin=cin, cout=cout,
                       ups=ups, scale=0.3, db=db, ws=ws)
        outs.append((dw, db))
    tol = 2e-5 if dtype == torch.float32 else 1e-4
    cmp(outs[0][0], outs[1][0], tol, "wgrad")
    cmp(outs[0][1], outs[1][1], tol, "wgrad bias")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_elementwise_ops(dtype):
    hip, cpu = ops_pair(dtype)
    B, H, C = 2, 8, 32
    x = q(rnd(B, H, H, C, seed=21), dtype)
    g = q(rnd(B, H // 2, H // 2, C, seed=22), dtype)
    y = q(rnd(B, H, H, C, seed=23), dtype)
    tol = tol_for(dtype, 1e-6)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        X, G, Y = x.to(dev).to(dt), g.to(dev).to(dt), y.to(dev).to(dt)
        r = {}
        r["pn"] = torch.zeros_like(X); ops.pixnorm(X, r["pn"], C)
        r["pnb"] = torch.zeros_like(X); ops.pixnorm_lrelu_bwd(X, Y, r["pnb"], C, 0.2)
        r["um"] = torch.zeros_like(X)
        ops.unpool_mask(G, Y, r["um"], B=B, H=H, W=H, C=C, scale=0.25, slope=0.2, ups=True)
        r["ap"] = torch.zeros_like(G); ops.avgpool2(X, r["ap"], B=B, H=H, W=H, C=C)
        r["bl"] = torch.zeros_like(X); ops.blend(0.3, X, 0.7, Y, r["bl"])
        db = torch.zeros(C, device=dev); ops.bias_grad(X, db, C, 0.5); r["db"] = db
        res[dev] = r
    for k in res["cpu"]:
        cmp(res["cuda"][k], res["cpu"][k], tol if k != "db" else 1e-5, k)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("s", [0, 2])
def test_rgb_ops(dtype, s):
    hip, cpu = ops_pair(dtype)
    B, R, C, Cp = 2, 4 * 2 ** s, 16, 32
    x = q(rnd(B, R, R, C, seed=31), dtype)
    xp = q(rnd(B, R // 2, R // 2, Cp, seed=32), dtype)
    w, b = rnd(3, C, 1, 1, seed=33), rnd(3, seed=34)
    wp, bp = rnd(3, Cp, 1, 1, seed=35), rnd(3, seed=36)
    gimg = rnd(B, 3, R, R, seed=37)
    img = rnd(B, 3, R, R, seed=38)
    fw, fb = rnd(C, 3, 1, 1, seed=39), rnd(C, seed=40)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        X, XP = x.to(dev).to(dt), xp.to(dev).to(dt)
        kw = dict(xp=XP, wp=wp.to(dev), bp=bp.to(dev), cp=0.2, Cp=Cp, alpha=0.3) if s else {}
        r = {"img": torch.zeros(B, 3, R, R, device=dev)}
        ops.rgb_out(X, w.to(dev), b.to(dev), 0.35, r["img"], B=B, R=R, C=C, **kw)
        r["gx"] = torch.zeros_like(X)
        r["dw"] = torch.zeros(3, C, 1, 1, device=dev)
        r["db"] = torch.zeros(3, device=dev)
        kwb = {}
        if s:
            r["gxp"] = torch.zeros_like(XP)
            r["dwp"] = torch.zeros(3, Cp, 1, 1, device=dev)
            r["dbp"] = torch.zeros(3, device=dev)
            kwb = dict(xp=XP, wp=wp.to(dev), cp=0.2, Cp=Cp, alpha=0.3, gxp=r["gxp"], dwp=r["dwp"],
                       dbp=r["dbp"])
        ops.rgb_out_bwd(X, w.to(dev), 0.35, gimg.to(dev), r["gx"], r["dw"], r["db"], B=B, R=R, C=C,
                        **kwb)
        for down in ((False, True) if s else (False,)):
            Ro = R // 2 if down else R
            yy = torch.zeros(B, Ro, Ro, C, dtype=dt, device=dev)
            ops.from_rgb(img.to(dev), fw.to(dev), fb.to(dev), 0.8, yy, B=B, R=Ro, C=C, down=down)
            r[f"fr{down}"] = yy
            ty = torch.zeros_like(yy)
            ops.from_rgb(img.to(dev), fw.to(dev), None, 0.8, ty, B=B, R=Ro, C=C, down=down,
                         mask_y=yy)
            r[f"ft{down}"] = ty
            gi = torch.zeros(B, 3, R, R, device=dev)
            dw_ = torch.zeros(C, 3, 1, 1, device=dev)
            db_ = torch.zeros(C, device=dev)
            ops.from_rgb_bwd(yy, fw.to(dev), 0.8, B=B, R=Ro, C=C, down=down, img=img.to(dev),
                             gimg=gi, dw=dw_, db=db_)
            r[f"fgi{down}"], r[f"fdw{down}"], r[f"fdb{down}"] = gi, dw_, db_
        fo = torch.zeros_like(img.to(dev))
        if s:
            ops.img_fade(img.to(dev), 0.4, fo)
        r["fade"] = fo
        res[dev] = r
    for k in res["cpu"]:
        cmp(res["cuda"][k], res["cpu"][k], tol_for(dtype, 2e-5), k)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [1, 4, 6, 16])
def test_linear_mbstd_loss(dtype, B):
    _L = lib()
    hip, cpu = ops_pair(dtype)
    C = 32
    mcs = cinp(C + 1)
    x = q(rnd(B, 4, 4, C, seed=51), dtype)
    w = rnd(C, 16 * C, seed=52)
    bb = rnd(C, seed=53)
    wdec = rnd(1, C, seed=54)
    aux = q(rnd(B, 4, 4, C, seed=55), dtype)
    gy = q(rnd(B, 4, 4, mcs, seed=56), dtype)
    a = q(rnd(B, 4, 4, C, seed=57), dtype)
    z = rnd(B, 64, seed=58)
    wf = rnd(16 * C, 64, seed=59)
    logits = rnd(B, 1, seed=60)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        X, AUX, GY, A = (t.to(dev).to(dt) for t in (x, aux, gy, a))
        r = {}
        r["l1"] = torch.zeros(B, C, dtype=dt, device=dev)
        ops.linear(X, w.to(dev), bb.to(dev), r["l1"], B=B,
                   flags=_L.LIN_BIAS | _L.LIN_LRELU | _L.LIN_IN_CHW, scale=0.1)
        r["out"] = torch.zeros(B, 1, device=dev)
        ops.linear(r["l1"], wdec.to(dev), torch.zeros(1, device=dev), r["out"], B=B, flags=_L.LIN_BIAS,
                   scale=0.2)
        r["gl1"] = torch.zeros(B, C, dtype=dt, device=dev)
        ops.linear_dgrad(r["out"], wdec.to(dev), r["gl1"], B=B, flags=_L.LIN_MASK, scale=0.2,
                         aux=r["l1"])
        r["gx"] = torch.zeros_like(X)
        ops.linear_dgrad(r["gl1"], w.to(dev), r["gx"], B=B, flags=_L.LIN_IN_CHW | _L.LIN_MASK,
                         scale=0.1, aux=AUX)
        r["dw"] = torch.zeros_like(w.to(dev))
        r["db"] = torch.zeros(C, device=dev)
        ops.linear_wgrad(X, r["gl1"], r["dw"], r["db"], B=B, flags=_L.LIN_IN_CHW, scale=0.1)
        r["f"] = torch.zeros(B, 4, 4, C, dtype=dt, device=dev)
        ops.linear(z.to(dev), wf.to(dev), torch.zeros(16 * C, device=dev), r["f"], B=B,
                   flags=_L.LIN_BIAS | _L.LIN_LRELU | _L.LIN_OUT_CHW, scale=0.3)
        r["dwf"] = torch.zeros(16 * C, 64, device=dev)
        ops.linear_wgrad(z.to(dev), r["f"], r["dwf"], None, B=B, flags=_L.LIN_OUT_CHW, scale=0.3)
        r["m"] = torch.zeros(B, 4, 4, mcs, dtype=dt, device=dev)
        ops.mbstd_fwd(X, r["m"], B=B, HW=16, C=C)
        r["gm"] = torch.zeros_like(X)
        ops.mbstd_bwd(X, GY, r["gm"], B=B, HW=16, C=C)
        r["tout"] = torch.zeros(B, 4, 4, mcs, dtype=dt, device=dev)
        r["inj"] = torch.zeros_like(X)
        ops.mbstd_r1(X, A, GY, r["tout"], r["inj"], B=B, HW=16, C=C)
        for tgt in (True, False):
            lo = torch.zeros(1, device=dev)
            u = torch.zeros(B, device=dev)
            h = torch.zeros(B, device=dev)
            ops.bce(logits.to(dev), tgt, 0.7, lo, u, h)
            r[f"bce{tgt}"], r[f"u{tgt}"], r[f"h{tgt}"] = lo, u, h
        gimg = logits.to(dev).view(B, 1, 1, 1).expand(B, 3, 4, 4).contiguous() * 1e-3
        r1 = torch.zeros(1, device=dev)
        gbar = torch.zeros_like(gimg)
        ops.r1_penalty(gimg, B, r1, gbar)
        r["r1"], r["gbar"] = r1, gbar
        gp = torch.zeros(1, device=dev)
        nrm = torch.zeros(B, device=dev)
        gb2 = torch.zeros_like(gimg)
        ops.gp_penalty(gimg, 10.0, gp, nrm, gb2)
        r["gp"], r["gpbar"] = gp, gb2
        res[dev] = r
    for k in res["cpu"]:
        tol = tol_for(dtype, 3e-5)
        if k in ("inj", "tout") and dtype == torch.float32:
            tol = 2e-4   # closed form vs autograd; includes 1/sigma^3 terms
        cmp(res["cuda"][k], res["cpu"][k], tol, k)


def test_adam_matches_torch():
    hip, cpu = ops_pair(torch.float32)
    n = 10000
    p0, g1, g2 = rnd(n, seed=71), rnd(n, seed=72) * 1e-3, rnd(n, seed=73)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        p = p0.clone().to(dev)
        m = torch.zeros(n, device=dev)
        v = torch.zeros(n, device=dev)
        for t, g in enumerate((g1, g2), start=1):
            ops.adam(p, g.to(dev), m, v, lr=1e-4, beta1=0.0, beta2=0.99, eps=1e-8, step=t)
        res[dev] = p
    ref = p0.clone().requires_grad_()
    opt = torch.optim.Adam([ref], lr=1e-4, betas=(0.0, 0.99), eps=1e-8)
    for g in (g1, g2):
        ref.grad = g.clone()
        opt.step()
    cmp(res["cuda"], ref.detach(), 1e-7, "adam vs torch.optim.Adam")
    cmp(res["cpu"], ref.detach(), 1e-7, "cpu double vs torch.optim.Adam")


def test_randn_moments():
    hip = lib().HipOps(torch.float32)
    z = torch.empty(1 << 20, device="cuda")
    hip.randn(z, 1234, 0)
    assert abs(z.mean().item()) < 5e-3 and abs(z.std().item() - 1) < 5e-3
    z2 = torch.empty(1 << 20, device="cuda")
    hip.randn(z2, 1234, 0)
    assert torch.equal(z, z2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", [(4, 8, 512, 512, ("bias", "lrelu")),
                                  (4, 16, 512, 512, ("bias", "lrelu", "pool")),
                                  (4, 4, 513, 512, ("bias", "lrelu")),
                                  (4, 4, 512, 516, ()),
                                  (4, 8, 512, 512, ("mask", "accum")),
                                  (3, 8, 256, 64, ("ups", "bias", "lrelu")),
                                  (4, 8, 512, 512, ("ups", "bias", "lrelu", "pixnorm")),
                                  (4, 4, 512, 512, ("bias", "lrelu", "pixnorm"))])
def test_conv3x3_splitk(case, dtype):
    """Small-spatial wide convs take the split-K path (fp32 partial slabs + epilogue; the
    generator's PixelNorm runs in that epilogue, y2 = the per-pixel factor)."""
    B, H, cin, cout, fl = case
    _L = lib()
    hip, cpu = ops_pair(dtype)
    flags = 0
    for f, v in (("ups", _L.CONV_UPS_IN), ("bias", _L.CONV_BIAS), ("lrelu", _L.CONV_LRELU),
                 ("mask", _L.CONV_MASK), ("pool", _L.CONV_POOL), ("accum", _L.CONV_ACCUM),
                 ("pixnorm", _L.CONV_PIXNORM)):
        if f in fl:
            flags |= v
    need = hip.conv_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout)
    assert need > 0, "expected the split-K path for this shape"
    Hin = H // 2 if "ups" in fl else H
    x = q(rnd(B, Hin, Hin, cinp(cin), seed=81), dtype)
    x[..., cin:] = 0
    w = rnd(cout, cin, 3, 3, seed=82)
    bias = rnd(cout, seed=83) * 0.1
    Ho = H // 2 if "pool" in fl else H
    y0 = q(rnd(B, Ho, Ho, cout, seed=84), dtype)
    aux = q(rnd(B, H, H, cout, seed=85), dtype)
    outs = []
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        wp = torch.zeros(ops.packed_elems(0, cout, cin), dtype=dt, device=dev)
        ops.conv_pack(0, w.to(dev), 0.02, wp)
        y = y0.to(dev).to(dt).clone()
        y2 = torch.zeros(B, H, H, cout, dtype=dt, device=dev) if "pool" in fl else None
        if "pixnorm" in fl:
            if dtype != torch.bfloat16:
                pytest.skip("split-K PixelNorm is a bf16-step fusion")
            y2 = torch.zeros(B, H, H, dtype=torch.float32, device=dev)
            assert ops.conv_supported(B=B, H=H, W=H, cin=cin, cout=cout, flags=flags,
                                      ws_bytes=need), "split-K PixelNorm expected"
        ws = torch.empty(need // 4, device=dev) if dev == "cuda" else None
        ops.conv3x3(x.to(dev).to(dt), wp, y, B=B, H=H, W=H, cin=cin, cout=cout, flags=flags,
                    out_scale=0.25 if "pool" in fl else 1.0, bias=(bias * 0.02).to(dev),
                    aux=aux.to(dev).to(dt), y2=y2, ws=ws)
        outs.append((y, y2))
    cmp(outs[0][0], outs[1][0], tol_for(dtype), "splitk y")
    if outs[0][1] is not None:
        cmp(outs[0][1], outs[1][1], tol_for(dtype), "splitk y2")


WIDE_CASES = [
    # wide bf16 convs at 32^2-512^2 through the default dispatch (tiles 13 / 6 / 3 / 14 and the
    # persistent narrow tiles) with every epilogue they take
    (4, 32, 512, 512, ("bias", "lrelu")),
    (4, 32, 512, 512, ("mask", "accum")),
    (4, 32, 512, 512, ("bias", "lrelu", "pool")),
    (4, 64, 256, 256, ()),
    (4, 64, 256, 512, ("bias", "lrelu", "pool")),
    (4, 64, 512, 256, ("ups", "bias", "lrelu")),
    (4, 64, 256, 256, ("pool", "accum")),
    (4, 128, 128, 128, ("mask",)),
    (4, 128, 256, 128, ("ups", "bias", "lrelu")),
    (2, 256, 64, 128, ("bias", "lrelu", "pool")),
    (4, 256, 128, 64, ("ups", "bias", "lrelu", "pixnorm")),
    (4, 256, 64, 64, ("bias", "lrelu", "pixnorm")),
    (2, 256, 64, 64, ("mask", "accum")),
    # one-slot form (two workgroups per CU): one- and two-chunk layers at >= 256^2
    (4, 256, 64, 64, ("bias", "lrelu")),
    (4, 256, 64, 128, ("mask",)),
    (2, 512, 32, 64, ("bias", "lrelu", "pool")),
    (2, 512, 32, 64, ()),
    # tile 15 (64 -> 32, CK = 64, persistent, compile-time flags): the G conv a at 512^2
    (2, 512, 64, 32, ("ups", "bias", "lrelu", "pixnorm")),
    # the 32^2 wide convs of the merged passes (B = 8) on the 16-row tile
    (8, 32, 512, 512, ("bias", "lrelu")),
    # tile 16 (64 -> 64, CK = 64, persistent, compile-time flags): the 256^2 level
    (4, 256, 64, 64, ()),
    (8, 256, 64, 64, ("mask",)),
    (8, 256, 64, 64, ("bias", "lrelu")),
    (2, 128, 64, 64, ("bias", "lrelu", "pixnorm")),
]


@pytest.mark.parametrize("case", WIDE_CASES)
def test_conv_wide(case):
    """bf16 wide convs against the CPU double: output, the pre-pool copy (y2 with POOL) and
    the PixelNorm factor (y2 with PIXNORM)."""
    B, H, cin, cout, fl = case
    _L = lib()
    dtype = torch.bfloat16
    hip, cpu = ops_pair(dtype)
    flags = 0
    for f, v in (("ups", _L.CONV_UPS_IN), ("bias", _L.CONV_BIAS), ("lrelu", _L.CONV_LRELU),
                 ("mask", _L.CONV_MASK), ("pool", _L.CONV_POOL), ("accum", _L.CONV_ACCUM),
                 ("pixnorm", _L.CONV_PIXNORM)):
        if f in fl:
            flags |= v
    Hin = H // 2 if "ups" in fl else H
    x = q(rnd(B, Hin, Hin, cinp(cin), seed=91), dtype)
    w = rnd(cout, cin, 3, 3, seed=92)
    bias = rnd(cout, seed=93) * 0.1
    Ho = H // 2 if "pool" in fl else H
    y0 = q(rnd(B, Ho, Ho, cout, seed=94), dtype)
    aux = q(rnd(B, H, H, cout, seed=95), dtype)
    scale = 1.0 / (9 * cin) ** 0.5
    outs = []
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        wp = torch.zeros(ops.packed_elems(0, cout, cin), dtype=dt, device=dev)
        ops.conv_pack(0, w.to(dev), scale, wp)
        y = y0.to(dev).to(dt).clone()
        y2 = None
        if "pool" in fl:
            y2 = torch.zeros(B, H, H, cout, dtype=dt, device=dev)
        if "pixnorm" in fl:
            y2 = torch.zeros(B, H, H, dtype=torch.float32, device=dev)
        ops.conv3x3(x.to(dev).to(dt), wp, y, B=B, H=H, W=H, cin=cin, cout=cout, flags=flags,
                    slope=0.2, out_scale=0.25 if "pool" in fl else 1.0,
                    bias=(bias * scale).to(dev), aux=aux.to(dev).to(dt), y2=y2)
        outs.append((y, y2))
    cmp(outs[0][0], outs[1][0], 2e-2, "wide y")
    if outs[0][1] is not None:
        cmp(outs[0][1], outs[1][1], 2e-2, "wide y2")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_pack_batch(dtype):
    """One batched launch == the per-layer fwd / dgrad packs and scaled biases, bit-exact."""
    hip = lib().HipOps(dtype)
    shapes = [(16, 16), (32, 16), (16, 32), (64, 32), (512, 513), (20, 33), (512, 512)]
    ents, refs = [], []
    for i, (co, ci) in enumerate(shapes):
        w = rnd(co, ci, 3, 3, seed=40 + i).cuda()
        b = rnd(co, seed=60 + i).cuda()
        sc = 0.1 + 0.01 * i
        pf = torch.full((hip.packed_elems(0, co, ci),), 7.0, device="cuda").to(dtype)
        pd = torch.full((hip.packed_elems(1, co, ci),), 7.0, device="cuda").to(dtype)
        bs = torch.zeros(co, device="cuda")
        ents.append((w, b, pf, pd, bs, sc))
        rf, rd = torch.zeros_like(pf), torch.zeros_like(pd)
        hip.conv_pack(0, w, sc, rf)
        hip.conv_pack(1, w, sc, rd)
        refs.append((rf, rd, b * sc))
    hip.conv_pack_batch(hip.pack_table(ents))
    torch.cuda.synchronize()
    for (w, b, pf, pd, bs, sc), (rf, rd, rb) in zip(ents, refs):
        assert torch.equal(pf, rf) and torch.equal(pd, rd)
        assert torch.allclose(bs, rb, rtol=1e-6, atol=0)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B", [4, 11, 20])
def test_linear_paper_sizes(dtype, B):
    """The mbstd linear (K = 16*512 CHW gather -> 512) and the latent layer (512 -> 16*512
    CHW scatter) at the paper width, forward and input gradient."""
    _L = lib()
    hip, cpu = ops_pair(dtype)
    C = 512
    x = q(rnd(B, 4, 4, C, seed=71), dtype)
    w = rnd(C, 16 * C, seed=72) * 0.05
    bb = rnd(C, seed=73)
    aux = q(rnd(B, 4, 4, C, seed=74), dtype)
    gy = rnd(B, C, seed=75)
    z = rnd(B, C, seed=76)
    wf = rnd(16 * C, C, seed=77) * 0.05
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        r = {}
        r["l1"] = torch.zeros(B, C, dtype=dt, device=dev)
        ops.linear(x.to(dev).to(dt), w.to(dev), bb.to(dev), r["l1"], B=B,
                   flags=_L.LIN_BIAS | _L.LIN_LRELU | _L.LIN_IN_CHW, scale=0.1)
        r["gx"] = torch.zeros(B, 4, 4, C, dtype=dt, device=dev)
        ops.linear_dgrad(gy.to(dev).to(dt), w.to(dev), r["gx"], B=B,
                         flags=_L.LIN_IN_CHW | _L.LIN_MASK, scale=0.1, aux=aux.to(dev).to(dt))
        r["f"] = torch.zeros(B, 4, 4, C, dtype=dt, device=dev)
        ops.linear(z.to(dev), wf.to(dev), bb.repeat(16).to(dev), r["f"], B=B,
                   flags=_L.LIN_BIAS | _L.LIN_LRELU | _L.LIN_OUT_CHW, scale=0.3)
        res[dev] = r
    for k in res["cpu"]:
        cmp(res["cuda"][k], res["cpu"][k], tol_for(dtype, 2e-5), k)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,H", [(16, 512), (32, 256), (64, 64), (512, 4), (24, 8)])
def test_elementwise_vector_shapes(dtype, C, H):
    """The vectorised row-grid kernels (ew.inc) at stage shapes: rows wider than one
    256-thread block, 16..512 channels, and a non-power-of-two count (generic fallback)."""
    hip, cpu = ops_pair(dtype)
    B = 2
    x = q(rnd(B, H, H, C, seed=51), dtype)
    g = q(rnd(B, H // 2, H // 2, C, seed=52), dtype)
    y = q(rnd(B, H, H, C, seed=53), dtype)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        X, G, Y = x.to(dev).to(dt), g.to(dev).to(dt), y.to(dev).to(dt)
        r = {}
        r["pn"] = torch.zeros_like(X); ops.pixnorm(X, r["pn"], C)
        r["pnb"] = torch.zeros_like(X); ops.pixnorm_lrelu_bwd(X, Y, r["pnb"], C, 0.2)
        r["um"] = torch.zeros_like(X)
        ops.unpool_mask(G, Y, r["um"], B=B, H=H, W=H, C=C, scale=0.25, slope=0.2, ups=True)
        r["um0"] = torch.zeros_like(X)
        ops.unpool_mask(X, Y, r["um0"], B=B, H=H, W=H, C=C, scale=0.5, slope=0.2, ups=False)
        r["ap"] = torch.zeros_like(G); ops.avgpool2(X, r["ap"], B=B, H=H, W=H, C=C)
        r["bl"] = torch.zeros_like(X); ops.blend(0.3, X, 0.7, Y, r["bl"])
        res[dev] = r
    for k in res["cpu"]:
        cmp(res["cuda"][k], res["cpu"][k], tol_for(dtype, 1e-6), f"{k} C={C} H={H}")


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,Cp,R", [(32, 64, 512), (16, 32, 1024), (64, 128, 64)])
def test_rgb_vector_shapes(dtype, C, Cp, R):
    """to/fromRGB kernels at the 512^2/1024^2 stage widths (row grids wider than a block)."""
    hip, cpu = ops_pair(dtype)
    B = 1
    x = q(rnd(B, R, R, C, seed=61), dtype)
    xp = q(rnd(B, R // 2, R // 2, Cp, seed=62), dtype)
    w, b = rnd(3, C, 1, 1, seed=63), rnd(3, seed=64)
    wp, bp = rnd(3, Cp, 1, 1, seed=65), rnd(3, seed=66)
    gimg = rnd(B, 3, R, R, seed=67)
    img = rnd(B, 3, R, R, seed=68)
    fw, fb = rnd(C, 3, 1, 1, seed=69), rnd(C, seed=70)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        X, XP = x.to(dev).to(dt), xp.to(dev).to(dt)
        r = {"img": torch.zeros(B, 3, R, R, device=dev)}
        ops.rgb_out(X, w.to(dev), b.to(dev), 0.35, r["img"], B=B, R=R, C=C, xp=XP, wp=wp.to(dev),
                    bp=bp.to(dev), cp=0.2, Cp=Cp, alpha=0.3)
        r["gx"] = torch.zeros_like(X)
        r["dw"] = torch.zeros(3, C, 1, 1, device=dev)
        r["db"] = torch.zeros(3, device=dev)
        r["gxp"] = torch.zeros_like(XP)
        r["dwp"] = torch.zeros(3, Cp, 1, 1, device=dev)
        r["dbp"] = torch.zeros(3, device=dev)
        ops.rgb_out_bwd(X, w.to(dev), 0.35, gimg.to(dev), r["gx"], r["dw"], r["db"], B=B, R=R, C=C,
                        xp=XP, wp=wp.to(dev), cp=0.2, Cp=Cp, alpha=0.3, gxp=r["gxp"], dwp=r["dwp"],
                        dbp=r["dbp"])
        for down in (False, True):
            Ro = R // 2 if down else R
            yy = torch.zeros(B, Ro, Ro, C, dtype=dt, device=dev)
            ops.from_rgb(img.to(dev), fw.to(dev), fb.to(dev), 0.8, yy, B=B, R=Ro, C=C, down=down)
            r[f"fr{down}"] = yy
            gi = torch.zeros(B, 3, R, R, device=dev)
            dw_ = torch.zeros(C, 3, 1, 1, device=dev)
            db_ = torch.zeros(C, device=dev)
            ops.from_rgb_bwd(yy, fw.to(dev), 0.8, B=B, R=Ro, C=C, down=down, img=img.to(dev),
                             gimg=gi, dw=dw_, db=db_)
            r[f"fgi{down}"], r[f"fdw{down}"], r[f"fdb{down}"] = gi, dw_, db_
        fo = torch.zeros_like(img.to(dev))
        ops.img_fade(img.to(dev), 0.4, fo)
        r["fade"] = fo
        res[dev] = r
    for k in res["cpu"]:
        # fp32 weight gradients sum ~1M pixel terms in a different order: 3e-4
        cmp(res["cuda"][k], res["cpu"][k], tol_for(dtype, 3e-4), f"{k} C={C} R={R}")


@pytest.mark.parametrize("B,H,c1,c2", [(1, 256, 16, 32), (1, 512, 32, 64), (1, 1024, 16, 32)])
def test_sign_bit_conv_paths(B, H, c1, c2):
    """bf16 sign-bit variants of the D conv-b chain (include/pggan_hip.h PG_CONV_*_BITS):
    forward with Y2_BITS (bits of the pre-pool activation), the R1 tangent with
    AUX_BITS|MASK|POOL, the input gradient with X_BITS|UPS_IN|MASK and the weight gradient
    with GZ_BITS, each against the CPU double on the same bf16 data; the bits themselves
    must match exactly where the activation is not within rounding of 0."""
    from cpu_ops import (CONV_AUX_BITS, CONV_BIAS, CONV_GZ_BITS, CONV_LRELU, CONV_MASK,
                         CONV_POOL, CONV_UPS_IN, CONV_X_BITS, CONV_Y2_BITS)
    hip, cpu = ops_pair(torch.bfloat16)
    dt = torch.bfloat16
    for fl, ci, co in ((CONV_BIAS | CONV_LRELU | CONV_POOL | CONV_Y2_BITS, c1, c2),
                       (CONV_MASK | CONV_AUX_BITS | CONV_POOL, c1, c2),
                       (CONV_MASK | CONV_UPS_IN | CONV_X_BITS, c2, c1)):
        assert hip.conv_supported(B=B, H=H, W=H, cin=ci, cout=co, flags=fl), (fl, ci, co)
    a = q(rnd(B, H, H, c1, seed=81), dt)                    # conv-b input (cin = c1)
    wf = q(rnd(r16(c2) * 9 * cinp(c1), seed=82, scale=0.05), dt)
    wd = q(rnd(r16(c1) * 9 * cinp(c2), seed=83, scale=0.05), dt)
    bias = rnd(c2, seed=84, scale=0.1)
    g = q(rnd(B, H // 2, H // 2, c2, seed=85), dt)           # pooled-resolution gradient
    amask = q(rnd(B, H, H, c1, seed=86), dt)                 # lrelu' operand of the dgrad
    res = {}
    shared_bits = None
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        d_ = dt if dev == "cuda" else torch.float32
        A, G, AM = a.to(dev).to(d_), g.to(dev).to(d_), amask.to(dev).to(d_)
        WF, WD, BS = wf.to(dev).to(d_), wd.to(dev).to(d_), bias.to(dev)
        r = {}
        p = torch.zeros(B, H // 2, H // 2, c2, dtype=d_, device=dev)
        bits = torch.zeros(B, H, H, c2 // 8, dtype=torch.uint8, device=dev)
        ops.conv3x3(A, WF, p, B=B, H=H, W=H, cin=c1, cout=c2,
                    flags=CONV_BIAS | CONV_LRELU | CONV_POOL | CONV_Y2_BITS, bias=BS, y2=bits,
                    out_scale=0.25)
        r["p"], r["bits"] = p, bits.clone()
        if shared_bits is None:
            shared_bits = bits.cpu()
        bits = shared_bits.to(dev)      # consumers: identical bits on both sides
        tp = torch.zeros_like(p)
        ops.conv3x3(A, WF, tp, B=B, H=H, W=H, cin=c1, cout=c2,
                    flags=CONV_MASK | CONV_AUX_BITS | CONV_POOL, aux=bits, out_scale=0.25)
        r["tp"] = tp
        gza = torch.zeros(B, H, H, c1, dtype=d_, device=dev)
        ops.conv3x3(G, WD, gza, B=B, H=H, W=H, cin=c2, cout=c1,
                    flags=CONV_MASK | CONV_UPS_IN | CONV_X_BITS, aux=AM, xbits=bits,
                    out_scale=0.25)
        r["gza"] = gza
        dw = torch.zeros(c2, c1, 3, 3, device=dev)
        db = torch.zeros(c2, device=dev)
        ops.conv_wgrad(A, G, dw, B=B, H=H, W=H, cin=c1, cout=c2, ups=False, scale=0.5, db=db,
                       gzbits=bits)
        r["dw"], r["db"] = dw, db
        res[dev] = r
    hb, cb = res["cuda"]["bits"].cpu(), res["cpu"]["bits"]
    diff = (hb ^ cb).count_nonzero().item()
    assert diff <= max(2, hb.numel() // 2000), f"{diff} bit bytes differ"
    for k in ("p", "tp", "gza", "dw", "db"):
        cmp(res["cuda"][k], res["cpu"][k], 2e-2, f"{k} H={H} {c1}->{c2}")


@pytest.mark.parametrize("B,H,c1,c2", [(2, 128, 128, 256), (4, 64, 256, 512), (1, 256, 64, 128)])
def test_sign_bit_unpool_paths(B, H, c1, c2):
    """The conv-b sign bits below the full sign-bit resolution (engine._ubits, the wide LDS-DMA
    tile): forward with Y2_BITS|POOL, the R1 tangent with AUX_BITS|MASK|POOL against the CPU
    double, and the unpool pass reading the bits (pg_unpool_mask_bits) bitwise equal to the
    same pass reading the bf16 activation whose signs they are."""
    from cpu_ops import CONV_AUX_BITS, CONV_BIAS, CONV_LRELU, CONV_MASK, CONV_POOL, CONV_Y2_BITS
    hip, cpu = ops_pair(torch.bfloat16)
    dt = torch.bfloat16
    for fl in (CONV_BIAS | CONV_LRELU | CONV_POOL | CONV_Y2_BITS, CONV_MASK | CONV_AUX_BITS | CONV_POOL):
        assert hip.conv_supported(B=B, H=H, W=H, cin=c1, cout=c2, flags=fl), fl
    a = q(rnd(B, H, H, c1, seed=101), dt)
    wf = q(rnd(r16(c2) * 9 * cinp(c1), seed=102, scale=0.05), dt)
    bias = rnd(c2, seed=103, scale=0.1)
    g = q(rnd(B, H // 2, H // 2, c2, seed=104), dt)
    res, shared = {}, None
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        d_ = dt if dev == "cuda" else torch.float32
        A, WF, BS, G = a.to(dev).to(d_), wf.to(dev).to(d_), bias.to(dev), g.to(dev).to(d_)
        r = {}
        p = torch.zeros(B, H // 2, H // 2, c2, dtype=d_, device=dev)
        bits = torch.zeros(B, H, H, c2 // 8, dtype=torch.uint8, device=dev)
        ops.conv3x3(A, WF, p, B=B, H=H, W=H, cin=c1, cout=c2,
                    flags=CONV_BIAS | CONV_LRELU | CONV_POOL | CONV_Y2_BITS, bias=BS, y2=bits,
                    out_scale=0.25)
        r["p"], r["bits"] = p, bits.clone()
        if shared is None:
            shared = bits.cpu()
        bits = shared.to(dev)
        tp = torch.zeros_like(p)
        ops.conv3x3(A, WF, tp, B=B, H=H, W=H, cin=c1, cout=c2,
                    flags=CONV_MASK | CONV_AUX_BITS | CONV_POOL, aux=bits, out_scale=0.25)
        r["tp"] = tp
        gz = torch.zeros(B, H, H, c2, dtype=d_, device=dev)
        ops.unpool_mask(G, None, gz, B=B, H=H, W=H, C=c2, scale=0.25, slope=0.2, ups=True,
                        bits=bits)
        r["gz"] = gz
        if dev == "cuda":
            # the bf16 pre-pool activation with exactly these signs -> the same unpool result
            y2 = torch.zeros(B, H, H, c2, dtype=d_, device=dev)
            ops.conv3x3(A, WF, torch.zeros_like(p), B=B, H=H, W=H, cin=c1, cout=c2,
                        flags=CONV_BIAS | CONV_LRELU | CONV_POOL, bias=BS, y2=y2, out_scale=0.25)
            if torch.equal(cpu_packbits(y2.float().cpu() > 0), shared):
                gz2 = torch.zeros_like(gz)
                ops.unpool_mask(G, y2, gz2, B=B, H=H, W=H, C=c2, scale=0.25, slope=0.2, ups=True)
                assert torch.equal(gz2, gz)
        res[dev] = r
    hb, cb = res["cuda"]["bits"].cpu(), res["cpu"]["bits"]
    diff = (hb ^ cb).count_nonzero().item()
    assert diff <= max(2, hb.numel() // 2000), f"{diff} bit bytes differ"
    for k in ("p", "tp", "gz"):
        cmp(res["cuda"][k], res["cpu"][k], 2e-2, f"{k} H={H} {c1}->{c2}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,R", [(16, 1024), (32, 128)])
def test_rgb_out_bwd_pn(dtype, C, R):
    """pg_rgb_out_bwd_pn: the toRGB input gradient with the PixelNorm + LReLU backward of its
    input fused in, against the CPU double and against the unfused HIP pair (rgb_out_bwd ->
    gy in the storage dtype -> pixnorm_lrelu_bwd_y)."""
    hip, cpu = ops_pair(dtype)
    B = 2
    y = q(rnd(B, R, R, C, seed=111), dtype)
    r = rnd(B * R * R, seed=112).abs() + 0.5
    w = rnd(3, C, 1, 1, seed=113)
    gimg = rnd(B, 3, R, R, seed=114)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = dtype if dev == "cuda" else torch.float32
        Y, Rr, Wd, G = y.to(dev).to(dt), r.to(dev), w.to(dev), gimg.to(dev)
        gz = torch.zeros(B, R, R, C, dtype=dt, device=dev)
        ops.rgb_out_bwd_pn(Y, Rr, Wd, 0.35, G, gz, B=B, R=R, C=C, slope=0.2)
        res[dev] = gz
        if dev == "cuda":
            gy = torch.zeros_like(gz)
            ops.rgb_out_bwd(Y, Wd, 0.35, G, gy, None, None, B=B, R=R, C=C)
            gz2 = torch.zeros_like(gz)
            ops.pixnorm_lrelu_bwd_y(Y, Rr, gy, gz2, C, 0.2)
            cmp(gz, gz2.cpu(), tol_for(dtype, 1e-6), "fused vs unfused")
            # with the toRGB weight / bias gradients in the same pass (_wg): the same gz, and the
            # gradients of the separate pass (accumulated onto existing values)
            dw0, db0 = rnd(3 * C, seed=115).to(dev), rnd(3, seed=116).to(dev)
            gz3, dw, db = torch.zeros_like(gz), dw0.clone(), db0.clone()
            ops.rgb_out_bwd_pn(Y, Rr, Wd, 0.35, G, gz3, B=B, R=R, C=C, slope=0.2, dw=dw, db=db)
            assert torch.equal(gz3, gz)
            dw2, db2 = dw0.clone(), db0.clone()
            ops.rgb_out_bwd(Y, Wd, 0.35, G, None, dw2, db2, B=B, R=R, C=C)
            cmp(dw, (dw2 - dw0).cpu() + dw0.cpu(), 1e-5, "toRGB dw fused")
            cmp(db, (db2 - db0).cpu() + db0.cpu(), 1e-5, "toRGB db fused")
    cmp(res["cuda"], res["cpu"], tol_for(dtype, 1e-6), f"gz C={C} R={R}")


@pytest.mark.parametrize("C,R", [(16, 256), (32, 128), (16, 1024)])
def test_from_rgb_sign_bits(C, R):
    """pg_from_rgb_bits (bf16): the forward writes the lrelu sign bits of its output with the
    same y as pg_from_rgb, and the tangent masked by those bits equals the tangent masked by
    the bf16 activation (mask_y) bit for bit, and the CPU double."""
    hip, cpu = ops_pair(torch.bfloat16)
    B = 2
    img = rnd(B, 3, R, R, seed=71)
    tin = rnd(B, 3, R, R, seed=72)
    fw, fb = rnd(C, 3, 1, 1, seed=73), rnd(C, seed=74)
    res = {}
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        dt = torch.bfloat16 if dev == "cuda" else torch.float32
        r = {}
        y = torch.zeros(B, R, R, C, dtype=dt, device=dev)
        yb = torch.zeros(B, R, R, C // 8, dtype=torch.uint8, device=dev)
        ops.from_rgb(img.to(dev), fw.to(dev), fb.to(dev), 0.8, y, B=B, R=R, C=C, down=False,
                     ybits=yb)
        r["y"], r["yb"] = y, yb
        t = torch.zeros_like(y)
        ops.from_rgb(tin.to(dev), fw.to(dev), None, 0.8, t, B=B, R=R, C=C, down=False,
                     mask_bits=yb)
        r["t"] = t
        if dev == "cuda":
            y0 = torch.zeros_like(y)
            ops.from_rgb(img.to(dev), fw.to(dev), fb.to(dev), 0.8, y0, B=B, R=R, C=C, down=False)
            assert torch.equal(y0, y)
            assert torch.equal(yb.cpu(), cpu_packbits(y.float().cpu() > 0))
            t0 = torch.zeros_like(y)
            ops.from_rgb(tin.to(dev), fw.to(dev), None, 0.8, t0, B=B, R=R, C=C, down=False,
                         mask_y=y)
            assert torch.equal(t0, t)
        res[dev] = r
    cmp(res["cuda"]["y"], res["cpu"]["y"], 2e-2, "y")
    cmp(res["cuda"]["t"], res["cpu"]["t"], 2e-2, "t")


@pytest.mark.parametrize("B,H,c1,c2", [(1, 256, 16, 32), (1, 512, 32, 64), (1, 1024, 16, 32)])
def test_sign_bit_mask_paths(B, H, c1, c2):
    """bf16 lrelu' masks from sign bits (include/pggan_hip.h PG_CONV_*_BITS) for the D conv a
    chain: the forward writes the bits of its activation (Y2_BITS, no pool), the R1 tangent
    masks with them (AUX_BITS|MASK) and the conv-b input gradient masks its result with them
    while reading its input through X_BITS (X_BITS|AUX_BITS|UPS_IN|MASK), against the CPU
    double on the same bf16 data and bits, and against the bf16-activation mask on the GPU."""
    from cpu_ops import (CONV_AUX_BITS, CONV_BIAS, CONV_LRELU, CONV_MASK, CONV_UPS_IN,
                         CONV_X_BITS, CONV_Y2_BITS)
    hip, cpu = ops_pair(torch.bfloat16)
    dt = torch.bfloat16
    for fl, ci, co in ((CONV_BIAS | CONV_LRELU | CONV_Y2_BITS, c1, c1),
                       (CONV_MASK | CONV_AUX_BITS, c1, c1),
                       (CONV_MASK | CONV_UPS_IN | CONV_X_BITS | CONV_AUX_BITS, c2, c1)):
        assert hip.conv_supported(B=B, H=H, W=H, cin=ci, cout=co, flags=fl), (fl, ci, co)
    x = q(rnd(B, H, H, c1, seed=91), dt)
    wa = q(rnd(r16(c1) * 9 * cinp(c1), seed=92, scale=0.05), dt)
    wd = q(rnd(r16(c1) * 9 * cinp(c2), seed=93, scale=0.05), dt)
    bias = rnd(c1, seed=94, scale=0.1)
    g = q(rnd(B, H // 2, H // 2, c2, seed=95), dt)
    bb = torch.randint(0, 256, (B, H, H, c2 // 8), dtype=torch.uint8,
                       generator=torch.Generator().manual_seed(96))
    res = {}
    shared = None
    for ops, dev in ((hip, "cuda"), (cpu, "cpu")):
        d_ = dt if dev == "cuda" else torch.float32
        X, WA, WD, BS, G = (x.to(dev).to(d_), wa.to(dev).to(d_), wd.to(dev).to(d_),
                            bias.to(dev), g.to(dev).to(d_))
        r = {}
        a = torch.zeros(B, H, H, c1, dtype=d_, device=dev)
        ab = torch.zeros(B, H, H, c1 // 8, dtype=torch.uint8, device=dev)
        ops.conv3x3(X, WA, a, B=B, H=H, W=H, cin=c1, cout=c1,
                    flags=CONV_BIAS | CONV_LRELU | CONV_Y2_BITS, bias=BS, y2=ab)
        r["a"], r["ab"] = a, ab.clone()
        if shared is None:
            shared = (ab.cpu(), a.cpu())
        ab, am = shared[0].to(dev), shared[1].to(dev).to(d_)     # identical operands both sides
        ta = torch.zeros_like(a)
        ops.conv3x3(X, WA, ta, B=B, H=H, W=H, cin=c1, cout=c1, flags=CONV_MASK | CONV_AUX_BITS,
                    aux=ab)
        r["ta"] = ta
        gza = torch.zeros_like(a)
        ops.conv3x3(G, WD, gza, B=B, H=H, W=H, cin=c2, cout=c1,
                    flags=CONV_MASK | CONV_UPS_IN | CONV_X_BITS | CONV_AUX_BITS, aux=ab,
                    xbits=bb.to(dev), out_scale=0.25)
        r["gza"] = gza
        if dev == "cuda":
            # the same launches with the bf16 activation as the mask operand
            ta2, gza2 = torch.zeros_like(a), torch.zeros_like(a)
            ops.conv3x3(X, WA, ta2, B=B, H=H, W=H, cin=c1, cout=c1, flags=CONV_MASK, aux=am)
            ops.conv3x3(G, WD, gza2, B=B, H=H, W=H, cin=c2, cout=c1,
                        flags=CONV_MASK | CONV_UPS_IN | CONV_X_BITS, aux=am, xbits=bb.to(dev),
                        out_scale=0.25)
            same = (ab.cpu() == cpu_packbits(am.float().cpu() > 0)).all().item()
            r["eq_ta"] = (ta2, same)
            r["eq_gza"] = (gza2, same)
        res[dev] = r
    hb, cb = res["cuda"]["ab"].cpu(), res["cpu"]["ab"]
    diff = (hb ^ cb).count_nonzero().item()
    assert diff <= max(2, hb.numel() // 2000), f"{diff} bit bytes differ"
    for k in ("a", "ta", "gza"):
        cmp(res["cuda"][k], res["cpu"][k], 2e-2, f"{k} H={H} {c1}->{c2}")
    for k in ("ta", "gza"):
        alt, same = res["cuda"]["eq_" + k]
        if same:    # bits == sign of the stored bf16 activation: bitwise the same result
            assert torch.equal(alt.cpu(), res["cuda"][k].cpu()), k


@pytest.mark.parametrize("B,H,cin", [(2, 64, 16), (1, 1024, 16), (2, 256, 16)])
def test_pixnorm_bwd_after_pool(B, H, cin):
    """PG_CONV_PNBWD | PG_CONV_POOL (bf16, 32 output channels): the generator's upsampling
    conv-a input gradient (2x2 sum) followed by the previous block's PixelNorm + LReLU
    backward at the pooled resolution, in one launch, against an fp32 restatement on the CPU
    double and the unfused HIP pair (pooled conv -> gy in bf16 -> pg_pixnorm_lrelu_bwd_y)."""
    from cpu_ops import CONV_PNBWD, CONV_POOL
    C = 32
    hip, cpu = ops_pair(torch.bfloat16)
    dt = torch.bfloat16
    fl = CONV_POOL | CONV_PNBWD
    assert hip.conv_supported(B=B, H=H, W=H, cin=cin, cout=C, flags=fl)
    Hp = H // 2
    gz = q(rnd(B, H, H, cin, seed=121), dt)
    wd = q(rnd(r16(C) * 9 * cinp(cin), seed=122, scale=0.05), dt)
    u = rnd(B, Hp, Hp, C, seed=123)
    r = torch.rsqrt((u * u).mean(-1) + 1e-8)
    y = q(u * r[..., None], dt)
    v = torch.zeros(B, Hp, Hp, C)
    cpu.conv3x3(gz, wd, v, B=B, H=H, W=H, cin=cin, cout=C, flags=CONV_POOL, out_scale=1.0)
    ref = r[..., None] * (v - y * (y * v).mean(-1, keepdim=True)) * torch.where(y > 0, 1.0, 0.2)
    G, WD, Y, Rr = gz.cuda().to(dt), wd.cuda().to(dt), y.cuda().to(dt), r.cuda().contiguous()
    out = torch.zeros(B, Hp, Hp, C, dtype=dt, device="cuda")
    hip.conv3x3(G, WD, out, B=B, H=H, W=H, cin=cin, cout=C, flags=fl, aux=Y, y2=Rr, out_scale=1.0)
    gy = torch.zeros(B, Hp, Hp, C, dtype=dt, device="cuda")
    hip.conv3x3(G, WD, gy, B=B, H=H, W=H, cin=cin, cout=C, flags=CONV_POOL, out_scale=1.0)
    unf = torch.zeros_like(gy)
    hip.pixnorm_lrelu_bwd_y(Y, Rr, gy, unf, C, 0.2)
    out2 = torch.zeros(B, Hp, Hp, C)
    cpu.conv3x3(gz, wd, out2, B=B, H=H, W=H, cin=cin, cout=C, flags=fl, aux=y, y2=r, out_scale=1.0)
    torch.cuda.synchronize()
    cmp(out, ref, 1e-2, f"pooled PNBWD H={H}")
    cmp(out, out2, 1e-2, f"pooled PNBWD vs CPU double H={H}")
    cmp(out, unf.float().cpu(), 2e-2, f"fused vs unfused H={H}")


@pytest.mark.parametrize("B,H,C", [(2, 32, 16), (2, 64, 32), (2, 256, 16), (1, 512, 32)])
def test_pixnorm_bwd_fused_dgrad(B, H, C):
    """PG_CONV_PNBWD (bf16, include/pggan_hip.h): the input-gradient conv writes the
    PixelNorm + LReLU backward of its result, r * (v - y * mean_c(y v)) * lrelu'(y), against
    an fp32 restatement on the CPU double's conv, and against the unfused HIP pair
    (conv -> gy in bf16 -> pg_pixnorm_lrelu_bwd_y)."""
    from cpu_ops import CONV_PNBWD
    hip, cpu = ops_pair(torch.bfloat16)
    dt = torch.bfloat16
    assert hip.conv_supported(B=B, H=H, W=H, cin=C, cout=C, flags=CONV_PNBWD)
    gz = q(rnd(B, H, H, C, seed=91), dt)
    wd = q(rnd(r16(C) * 9 * cinp(C), seed=92, scale=0.05), dt)
    u = rnd(B, H, H, C, seed=93)
    r = torch.rsqrt((u * u).mean(-1) + 1e-8)
    y = q(u * r[..., None], dt)
    v = torch.zeros(B, H, H, C)
    cpu.conv3x3(gz, wd, v, B=B, H=H, W=H, cin=C, cout=C, flags=0)
    ref = r[..., None] * (v - y * (y * v).mean(-1, keepdim=True)) * torch.where(y > 0, 1.0, 0.2)
    G, WD, Y, Rr = gz.cuda().to(dt), wd.cuda().to(dt), y.cuda().to(dt), r.cuda().contiguous()
    out = torch.zeros(B, H, H, C, dtype=dt, device="cuda")
    hip.conv3x3(G, WD, out, B=B, H=H, W=H, cin=C, cout=C, flags=CONV_PNBWD, aux=Y, y2=Rr)
    gy = torch.zeros(B, H, H, C, dtype=dt, device="cuda")
    hip.conv3x3(G, WD, gy, B=B, H=H, W=H, cin=C, cout=C, flags=0)
    unf = torch.zeros_like(gy)
    hip.pixnorm_lrelu_bwd_y(Y, Rr, gy, unf, C, 0.2)
    torch.cuda.synchronize()
    cmp(out, ref, 1e-2, f"fused PNBWD H={H} C={C}")
    cmp(out, unf.float().cpu(), 2e-2, f"fused vs unfused H={H} C={C}")


@pytest.mark.parametrize("B,H,C", [(2, 1024, 16), (2, 512, 32), (1, 512, 32)])
def test_conv_rgbw_epilogue(B, H, C):
    """PG_CONV_RGBW (bf16): the top conv a's input gradient with the fromRGB weight / bias
    gradients in its epilogue (dw[n*3+i] += s sum gz[n] img[i], db[n] += s sum gz[n]; the
    result gz is not stored) against the same conv on the CPU double (fp32 on the same bf16
    operands and sign bits) followed by the float64 sums, accumulated onto existing values
    (the tangent's term is already in the gradient); and bitwise reproducible."""
    from cpu_ops import CONV_AUX_BITS, CONV_MASK
    hip, cpu = ops_pair(torch.bfloat16)
    fl = CONV_MASK | CONV_AUX_BITS
    assert hip.conv_supported(B=B, H=H, W=H, cin=C, cout=C, flags=fl | _lib_flag("CONV_RGBW"))
    dt = torch.bfloat16
    x = q(rnd(B, H, H, C, seed=131), dt)
    wd = q(rnd(r16(C) * 9 * cinp(C), seed=132, scale=0.05), dt)
    bits = torch.randint(0, 256, (B, H, H, C // 8), dtype=torch.uint8,
                         generator=torch.Generator().manual_seed(133))
    img = rnd(B, 3, H, H, seed=134)
    dw0, db0 = rnd(C * 3, seed=135), rnd(C, seed=136)
    s = 0.8165
    gz = torch.zeros(B, H, H, C)
    cpu.conv3x3(x.float(), wd.float(), gz, B=B, H=H, W=H, cin=C, cout=C, flags=fl, aux=bits)
    g64, i64 = gz.double(), img.double()
    dw_ref = dw0.double().view(C, 3) + s * torch.einsum("bhwn,bihw->ni", g64, i64)
    db_ref = db0.double() + s * g64.sum(dim=(0, 1, 2))
    outs = []
    for _ in range(2):
        dw, db = dw0.clone().cuda(), db0.clone().cuda()
        hip.conv3x3_rgbw(x.to(dt).cuda(), wd.to(dt).cuda(), B=B, H=H, W=H, cin=C, cout=C, flags=fl,
                         aux=bits.cuda(), img=img.cuda(), s=s, dw=dw, db=db)
        outs.append((dw.cpu(), db.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1]), \
        "RGBW sums not bitwise reproducible"
    for got, ref, what in ((outs[0][0].view(C, 3), dw_ref, "dw"), (outs[0][1], db_ref, "db")):
        err = float((got.double() - ref).norm() / ref.norm())
        assert err <= 1e-4, (what, err)


def _lib_flag(name):
    from pggan_amd import _lib
    return getattr(_lib, name)


@pytest.mark.parametrize("B,H,C", [(4, 1024, 16), (2, 512, 32), (3, 512, 32)])
def test_conv_rgbd_epilogue(B, H, C):
    """PG_CONV_RGBD (bf16): the top conv a's input gradient with the fromRGB input gradient
    gimg = f W^T gz (written), its per-sample squared norms (accumulated) and the R1 tangent's
    fromRGB weight term s sum gz (x) gimg (accumulated) in its epilogue, against the same conv
    on the CPU double followed by float64 arithmetic; bitwise reproducible."""
    from cpu_ops import CONV_AUX_BITS, CONV_MASK
    hip, cpu = ops_pair(torch.bfloat16)
    fl = CONV_MASK | CONV_AUX_BITS
    assert hip.conv_supported(B=B, H=H, W=H, cin=C, cout=C, flags=fl | _lib_flag("CONV_RGBD"))
    dt = torch.bfloat16
    x = q(rnd(B, H, H, C, seed=151), dt)
    wd = q(rnd(r16(C) * 9 * cinp(C), seed=152, scale=0.05), dt)
    bits = torch.randint(0, 256, (B, H, H, C // 8), dtype=torch.uint8,
                         generator=torch.Generator().manual_seed(153))
    wr = rnd(C, 3, seed=154)
    f, s = 0.8165, 0.8165 / B
    n0, dw0 = rnd(B, seed=155).abs(), rnd(C * 3, seed=156)
    gz = torch.zeros(B, H, H, C)
    cpu.conv3x3(x.float(), wd.float(), gz, B=B, H=H, W=H, cin=C, cout=C, flags=fl, aux=bits)
    g64 = gz.double()
    gimg_ref = f * torch.einsum("bhwn,ni->bihw", g64, wr.double())
    norms_ref = n0.double() + (gimg_ref ** 2).sum(dim=(1, 2, 3))
    dw_ref = dw0.double().view(C, 3) + s * torch.einsum("bhwn,bihw->ni", g64, gimg_ref)
    outs = []
    for _ in range(2):
        gimg = torch.full((B, 3, H, H), float("nan"), device="cuda")
        norms, dw = n0.clone().cuda(), dw0.clone().cuda()
        hip.conv3x3_rgbd(x.to(dt).cuda(), wd.to(dt).cuda(), B=B, H=H, W=H, cin=C, cout=C, flags=fl,
                         aux=bits.cuda(), w_rgb=wr.cuda(), f=f, gimg=gimg, norms=norms, dw=dw, s=s)
        outs.append((gimg.cpu(), norms.cpu(), dw.cpu()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b), "RGBD outputs not bitwise reproducible"
    for got, ref, what in ((outs[0][0], gimg_ref, "gimg"), (outs[0][1], norms_ref, "norms"),
                           (outs[0][2].view(C, 3), dw_ref, "dw")):
        err = float((got.double() - ref).norm() / ref.norm())
        assert err <= 1e-4, (what, err)


@pytest.mark.parametrize("B,H,C,keep", [(4, 1024, 16, True), (8, 1024, 16, False), (2, 512, 32, True)])
def test_conv_rgbo_epilogue(B, H, C, keep):
    """PG_CONV_RGBO (bf16): the generator's top conv b forward with PixelNorm and the toRGB output
    img = c (W y + b) in its epilogue, against the unfused pair (the same conv, then
    pg_rgb_out on the stored y): y and the PixelNorm factor bitwise equal, img within fp32
    summation-order rounding (1e-5 relative L2; the epilogue sums the 16 / 32 channels as
    per-lane partials, the toRGB pass in channel order)."""
    from cpu_ops import CONV_BIAS, CONV_LRELU, CONV_PIXNORM
    hip, _ = ops_pair(torch.bfloat16)
    fl = CONV_PIXNORM | CONV_LRELU | CONV_BIAS
    assert hip.conv_supported(B=B, H=H, W=H, cin=C, cout=C, flags=fl | _lib_flag("CONV_RGBO"))
    dt = torch.bfloat16
    x = q(rnd(B, H, H, C, seed=141), dt).to(dt).cuda()
    w = rnd(C, C, 3, 3, seed=142)
    scale = 1.0 / (9 * C) ** 0.5
    wp = torch.zeros(hip.packed_elems(0, C, C), dtype=dt, device="cuda")
    hip.conv_pack(0, w.cuda(), scale, wp)
    bias = (rnd(C, seed=143) * 0.1 * scale).cuda()
    w_rgb, b_rgb = rnd(3, C, seed=144).cuda(), (rnd(3, seed=145) * 0.1).cuda()
    c = (1.0 / C) ** 0.5
    outs = []
    for fused in (True, False):
        y = torch.zeros(B, H, H, C, dtype=dt, device="cuda")
        r = torch.zeros(B, H, H, dtype=torch.float32, device="cuda") if keep else None
        img = torch.zeros(B, 3, H, H, dtype=torch.float32, device="cuda")
        if fused:
            hip.conv3x3_rgbo(x, wp, y, B=B, H=H, W=H, cin=C, cout=C, flags=fl, bias=bias, y2=r,
                             w_rgb=w_rgb, b_rgb=b_rgb, c=c, img=img)
        else:
            hip.conv3x3(x, wp, y, B=B, H=H, W=H, cin=C, cout=C, flags=fl, bias=bias, y2=r)
            hip.rgb_out(y, w_rgb, b_rgb, c, img, B=B, R=H, C=C)
        torch.cuda.synchronize()
        outs.append((y.cpu(), None if r is None else r.cpu(), img.cpu()))
    (yf, rf, imf), (yu, ru, imu) = outs
    assert torch.equal(yf, yu), "fused y differs"
    if keep:
        assert torch.equal(rf, ru), "fused PixelNorm factor differs"
    err = float((imf.double() - imu.double()).norm() / imu.double().norm())
    assert err <= 1e-5, err
