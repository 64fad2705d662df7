"""CPU oracle for the PGGAN G+D+R1 training step — TEST INFRASTRUCTURE ONLY.

This module is a plain-PyTorch (CPU, fp32, NCHW) restatement of the reference
training step of yukyeongleee/pggan.  It is the *checker* used by ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``.
The product path (``pggan_amd``) never imports it: the product runs only the
hand-written HIP kernels in ``pggan_amd/csrc`` and fails loudly without them.

Parity pinning: the restatement is checked in ``tests/test_oracle_golden.py``
against golden vectors produced by importing the reference itself in the build
container (``tests/golden/make_golden.py``); see DESIGN.md "Oracle".

Every function cites the reference file:line it restates (paths relative to the
reference root).  Parameters are a flat ``dict[name -> Tensor]`` keyed by the
reference ``state_dict`` names (``blocks.{i}.block.{0,3}.module.weight`` ...).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch
import torch.nn.functional as F

PAPER_DEPTHS = [512, 512, 512, 512, 256, 128, 64, 32, 16]


# --------------------------------------------------------------------------
# L1 ops
# --------------------------------------------------------------------------
def pixel_norm(x, eps=1e-8):
    """lib/layers.py:13-14  x * rsqrt(mean_c x^2 + eps)."""
    return x * (((x ** 2).mean(dim=1, keepdim=True) + eps).rsqrt())


def he_const(w):
    """lib/layers.py:17-25  sqrt(2 / prod(weight.shape[1:]))."""
    fan_in = 1
    for s in w.shape[1:]:
        fan_in *= int(s)
    return math.sqrt(2.0 / fan_in)


def eq_conv(x, w, b, padding):
    """lib/layers.py:58-63 via EqualizedConv2d :66-89 — (conv(x,W)+b)*c (bias scaled too)."""
    y = F.conv2d(x, w, b, padding=padding)
    return y * he_const(w)


def eq_linear(x, w, b):
    """lib/layers.py:58-63 via EqualizedLinear :92-108."""
    return F.linear(x, w, b) * he_const(w)


def lrelu(x, slope=0.2):
    return F.leaky_relu(x, slope)


class Kinks:
    """Leaky-ReLU region choices injected from another implementation's forward pass.

    Parity tests only.  A pre-activation within rounding of 0 can take the other slope
    under any change of summation order, and its gradient then changes by 1/slope; with
    10^5-10^7 pre-activations per layer such flips are expected between two correct
    implementations.  Injecting the region choice of the implementation under test makes
    both compute the same piecewise-linear function, so the remaining difference is pure
    rounding and every tensor can be held to the strict bar.  Each site records how many
    elements the injected choice flips relative to this forward's own sign, and the
    largest |pre-activation| among them relative to the site's RMS: the tests assert that
    bound, so a real kernel error (a wrong sign far from 0) cannot hide behind a mask.

    masks: {site: bool tensor shaped like the pre-activation (NCHW / [B, N])}, True =
    slope 1.  Every site the forward reaches must be present; None marks a branch the
    implementation elided because its weight is exactly 0 (its own sign is used)."""

    def __init__(self, masks):
        self.masks = masks
        self.stats = {}

    def act(self, x, site, slope):
        if self.masks[site] is None:   # a branch the implementation elided (zero weight)
            return lrelu(x, slope)
        m = self.masks[site].to(x.device)
        assert m.shape == x.shape, (site, tuple(m.shape), tuple(x.shape))
        with torch.no_grad():
            own = x > 0
            flip = own != m
            n = int(flip.sum())
            rms = float(x.detach().double().pow(2).mean().sqrt()) or 1.0
            worst = float(x.detach()[flip].abs().max()) / rms if n else 0.0
            self.stats[site] = (n, x.numel(), worst)
        k = torch.where(m, torch.ones((), dtype=x.dtype), torch.full((), slope, dtype=x.dtype))
        return x * k

    def flips(self):
        return sum(v[0] for v in self.stats.values())

    def worst(self):
        return max((v[2] for v in self.stats.values()), default=0.0)


def _act(kinks):
    if kinks is None:
        return lambda x, site, slope: lrelu(x, slope)
    return kinks.act


def upscale2d(x):
    """lib/utils.py:106-118 nearest x2 via view/expand."""
    s = x.shape
    x = x.view(-1, s[1], s[2], 1, s[3], 1).expand(-1, s[1], s[2], 2, s[3], 2)
    return x.contiguous().view(-1, s[1], s[2] * 2, s[3] * 2)


def downscale2d(x):
    """lib/utils.py:120-124 avg_pool2d 2x2."""
    return F.avg_pool2d(x, (2, 2))


def mbstd(x, subgroup_size=4):
    """lib/blocks.py:204-233 concatenate_stddev_channel (contiguous groups, unbiased var)."""
    size = x.shape
    g = min(size[0], subgroup_size)
    if size[0] % g != 0:
        g = size[0]
    n_groups = size[0] // g
    if g > 1:
        y = x.view(-1, g, size[1], size[2], size[3])
        y = torch.var(y, 1)
        y = torch.sqrt(y + 1e-8)
        y = y.view(n_groups, -1)
        y = torch.mean(y, 1).view(n_groups, 1)
        y = y.expand(n_groups, size[2] * size[3]).view((n_groups, 1, 1, size[2], size[3]))
        y = y.expand(n_groups, g, -1, -1, -1)
        y = y.contiguous().view((-1, 1, size[2], size[3]))
    else:
        y = torch.zeros(x.size(0), 1, x.size(2), x.size(3), dtype=x.dtype)
    return torch.cat([x, y], dim=1)


# --------------------------------------------------------------------------
# Networks
# --------------------------------------------------------------------------
def g_param_shapes(depths, s, latent_dim=512, out_dim=3):
    """Generator parameters at stage s in reference registration order
    (pggan/nets.py:53-71, add_block :102-119, lib/blocks.py:113-170)."""
    d0 = depths[0]
    shapes = []
    for i in range(s):
        prev, new = depths[i], depths[i + 1]
        shapes += [(f"blocks.{i}.block.0.module.weight", (new, prev, 3, 3)),
                   (f"blocks.{i}.block.0.module.bias", (new,)),
                   (f"blocks.{i}.block.3.module.weight", (new, new, 3, 3)),
                   (f"blocks.{i}.block.3.module.bias", (new,))]
    for i in range(s + 1):
        shapes += [(f"toRGB_blocks.{i}.toRGB.module.weight", (out_dim, depths[i], 1, 1)),
                   (f"toRGB_blocks.{i}.toRGB.module.bias", (out_dim,))]
    shapes += [("latent_format_layer.module.weight", (16 * d0, latent_dim)),
               ("latent_format_layer.module.bias", (16 * d0,)),
               ("first_block.block.0.module.weight", (d0, d0, 3, 3)),
               ("first_block.block.0.module.bias", (d0,))]
    return shapes


def d_param_shapes(depths, s, in_dim=3):
    """Discriminator parameters at stage s (pggan/nets.py:164-246, lib/blocks.py:173-292)."""
    d0 = depths[0]
    shapes = []
    for i in range(s):
        new, prev = depths[i + 1], depths[i]
        shapes += [(f"blocks.{i}.block.0.module.weight", (new, new, 3, 3)),
                   (f"blocks.{i}.block.0.module.bias", (new,)),
                   (f"blocks.{i}.block.2.module.weight", (prev, new, 3, 3)),
                   (f"blocks.{i}.block.2.module.bias", (prev,))]
    for i in range(s + 1):
        shapes += [(f"fromRGB_blocks.{i}.fromRGB.module.weight", (depths[i], in_dim, 1, 1)),
                   (f"fromRGB_blocks.{i}.fromRGB.module.bias", (depths[i],))]
    shapes += [("decision_layer.module.weight", (1, d0)),
               ("decision_layer.module.bias", (1,)),
               ("minibatch_normalization_block.conv.module.weight", (d0, d0 + 1, 3, 3)),
               ("minibatch_normalization_block.conv.module.bias", (d0,)),
               ("minibatch_normalization_block.linear.module.weight", (d0, 16 * d0)),
               ("minibatch_normalization_block.linear.module.bias", (d0,))]
    return shapes


def generator_forward(P, z, s, alpha, slope_cfg=0.2, kinks=None):
    """pggan/nets.py:121-161 Generator.forward.  kinks: optional Kinks (parity tests)
    with sites fmt, first, a{i}, b{i}."""
    act = _act(kinks)
    x = pixel_norm(z)                                              # :124-125
    x = x.view(-1, x[0].numel())                                   # :126
    x = act(eq_linear(x, P["latent_format_layer.module.weight"],
                      P["latent_format_layer.module.bias"]), "fmt", slope_cfg)   # :129
    x = x.view(x.shape[0], -1, 4, 4)                               # :130
    x = pixel_norm(x)                                              # :132-133
    x = pixel_norm(act(eq_conv(x, P["first_block.block.0.module.weight"],
                               P["first_block.block.0.module.bias"], 1), "first", 0.2))
    # :136, blocks.py:131-139

    def to_rgb(i, h, up):                                          # blocks.py:153-170
        y = eq_conv(h, P[f"toRGB_blocks.{i}.toRGB.module.weight"],
                    P[f"toRGB_blocks.{i}.toRGB.module.bias"], 0)
        return upscale2d(y) if up else y

    x_up = None
    if s == 1:
        x_up = to_rgb(s - 1, x, True)                              # :140-141
    for i in range(s):                                             # :144-149
        x = upscale2d(x)
        x = pixel_norm(act(eq_conv(x, P[f"blocks.{i}.block.0.module.weight"],
                                   P[f"blocks.{i}.block.0.module.bias"], 1), f"a{i}", 0.2))
        x = pixel_norm(act(eq_conv(x, P[f"blocks.{i}.block.3.module.weight"],
                                   P[f"blocks.{i}.block.3.module.bias"], 1), f"b{i}", 0.2))
        if i == s - 2:
            x_up = to_rgb(s - 1, x, True)
    x = to_rgb(s, x, False)                                        # :152
    if s:
        x = (1.0 - alpha) * x_up + alpha * x                       # :155-156
    return x


def discriminator_forward(P, x, s, alpha, get_feature=False, kinks=None):
    """pggan/nets.py:248-276 Discriminator.forward.  kinks: optional Kinks (parity tests)
    with sites rgb, rgbd, a{i}, b{i}, mb, lin."""
    act = _act(kinks)

    def from_rgb(i, h, down, site):                                # blocks.py:271-292
        if down:
            h = downscale2d(h)
        return act(eq_conv(h, P[f"fromRGB_blocks.{i}.fromRGB.module.weight"],
                           P[f"fromRGB_blocks.{i}.fromRGB.module.bias"], 0), site, 0.2)

    x_down = from_rgb(s - 1, x, True, "rgbd") if s else None       # :251-252
    x = from_rgb(s, x, False, "rgb")                               # :255
    merge = s > 0
    for i in reversed(range(s)):                                   # :260-265, blocks.py:179-199
        x = act(eq_conv(x, P[f"blocks.{i}.block.0.module.weight"],
                        P[f"blocks.{i}.block.0.module.bias"], 1), f"a{i}", 0.2)
        x = act(eq_conv(x, P[f"blocks.{i}.block.2.module.weight"],
                        P[f"blocks.{i}.block.2.module.bias"], 1), f"b{i}", 0.2)
        x = F.avg_pool2d(x, (2, 2))
        if merge:
            merge = False
            x = (1 - alpha) * x_down + alpha * x
    x = mbstd(x)                                                   # blocks.py:261
    x = act(eq_conv(x, P["minibatch_normalization_block.conv.module.weight"],
                    P["minibatch_normalization_block.conv.module.bias"], 1), "mb", 0.2)
    x = x.view(-1, x[0].numel())
    x = act(eq_linear(x, P["minibatch_normalization_block.linear.module.weight"],
                      P["minibatch_normalization_block.linear.module.bias"]), "lin", 0.2)
    out = eq_linear(x, P["decision_layer.module.weight"], P["decision_layer.module.bias"])
    return (out, x) if get_feature else out


# --------------------------------------------------------------------------
# Losses
# --------------------------------------------------------------------------
def bce_logits(logits, target):
    """lib/loss.py:119-123 BCE-with-logits mean vs constant target."""
    return F.binary_cross_entropy_with_logits(logits, torch.full_like(logits, float(target)))


def r1_reg(d_out, x_in):
    """lib/loss.py:125-135: 0.5 * mean_b sum (dL/dx)^2 (create_graph)."""
    g = torch.autograd.grad(d_out.sum(), x_in, create_graph=True, retain_graph=True,
                            only_inputs=True)[0]
    return 0.5 * g.pow(2).view(x_in.shape[0], -1).sum(1).mean(0)


def wgan_gp(Dfn, img_real, img_fake, eps, w_gp):
    """pggan/loss.py:54-92 get_gradient_penalty (dead in the reference; optional mode).
    eps: [B,1] uniform (:71-73); x^ = eps*x_r + (1-eps)*x_f (:75); d = sum_b D(x^)[:,0]
    (:78-79); per-sample L2 norm of dd/dx^ (:81-86); W_gp * sum_b (|g|-1)^2 (:87)."""
    B = img_real.shape[0]
    e = eps.expand(B, img_real[0].numel()).contiguous().view(img_real.shape)
    interp = (e * img_real + (1 - e) * img_fake).detach().requires_grad_()
    d = Dfn(interp)[:, 0].sum()
    g = torch.autograd.grad(d, interp, create_graph=True, retain_graph=True)[0]
    g = g.view(B, -1)
    g = (g * g).sum(dim=1).sqrt()
    return ((g - 1.0) ** 2).sum() * w_gp


def drift_loss(pred_real, w_drift):
    """pggan/loss.py:94-100 get_drift_loss: W_drift_D * sum_b D(x_real)^2."""
    return (pred_real ** 2).sum() * w_drift


# --------------------------------------------------------------------------
# Adam (torch.optim.Adam, single-tensor, lib/model.py:95-97)
# --------------------------------------------------------------------------
@dataclass
class AdamState:
    lr: float
    beta1: float = 0.0
    beta2: float = 0.99
    eps: float = 1e-8
    step: dict = field(default_factory=dict)
    m: dict = field(default_factory=dict)
    v: dict = field(default_factory=dict)

    def update(self, P, grads):
        """Params whose grad is None are skipped (as torch does)."""
        for k, g in grads.items():
            if g is None:
                continue
            if k not in self.step:
                self.step[k] = 0
                self.m[k] = torch.zeros_like(P[k])
                self.v[k] = torch.zeros_like(P[k])
            self.step[k] += 1
            t = self.step[k]
            self.m[k].lerp_(g, 1 - self.beta1)
            self.v[k].mul_(self.beta2).addcmul_(g, g, value=1 - self.beta2)
            bc1 = 1 - self.beta1 ** t
            bc2 = 1 - self.beta2 ** t
            step_size = self.lr / bc1
            denom = (self.v[k].sqrt() / math.sqrt(bc2)).add_(self.eps)
            P[k].addcdiv_(self.m[k], denom, value=-step_size)


# --------------------------------------------------------------------------
# The training step (pggan/model.py:206-255)
# --------------------------------------------------------------------------
@dataclass
class StepOut:
    img_real: torch.Tensor
    img_fake_D: torch.Tensor
    img_fake_G: torch.Tensor
    pred_real: torch.Tensor
    pred_fake: torch.Tensor
    pred_fake_G: torch.Tensor
    L_D_real: float
    L_D_fake: float
    R1: float
    L_D: float
    L_G: float
    grads_D: dict
    grads_G: dict
    drift: float = 0.0


def train_step(PG, PD, optG, optD, img_real, z1, z2, s, alpha_G, alpha_D,
               W_adv=1.0, slope_cfg=0.2, gp_mode="r1", gp_eps=None, W_gp=10.0, W_drift=0.0,
               kinks=None, fake_D=None, fake_G=None, grads_D_update=None):
    """pggan/model.py:206-255 ProgressiveGAN.train_step on CPU; updates PG/PD in place.

    gp_mode="r1" is the live reference path (pggan/loss.py:16-27).
    gp_mode="wgan-gp" is the optional mode the north star names: L_D = BCE(real,1) +
    BCE(fake,0) + get_gradient_penalty (pggan/loss.py:54-92) + get_drift_loss
    (:94-100), both terms differentiated into D's gradient (the paper's meaning; the
    reference's code for them is never called).

    kinks: optional {"D": [Kinks...], "G": [Kinks...]} consumed in forward-call order
    (D: real, fake, [interpolate], fake of the G half; G: z1, z2) -- parity tests only.
    fake_D / fake_G: optional fake images of the implementation under test, fed to D in
    place of this G's output (parity tests, to compare each network on identical inputs;
    the G half keeps this G's gradient path: the value is fake_G, the gradient flows
    into this G).  The returned img_fake_* are always this G's own outputs.
    grads_D_update: optional D gradient that Adam_D applies instead of this step's own (the
    data-parallel contract: every rank's G half runs with D updated by the mean over ranks;
    tests/test_gpu_dp.py); the returned grads_D are still this step's own.
    Works in any floating dtype (the tests run it in float64)."""
    kD = list(kinks["D"]) if kinks else []
    kG = list(kinks["G"]) if kinks else []

    def D(P, x, get_feature=False):
        return discriminator_forward(P, x, s, alpha_D, get_feature, kD.pop(0) if kinks else None)

    def G(P, z):
        return generator_forward(P, z, s, alpha_G, slope_cfg, kG.pop(0) if kinks else None)

    for P in (PG, PD):
        for k in P:
            P[k].requires_grad_(True)
    if s:                                                           # :217-221
        low = F.interpolate(F.avg_pool2d(img_real, (2, 2)), scale_factor=2, mode="nearest")
        img_real = (1 - alpha_D) * low + alpha_D * img_real
    img_real = img_real.detach().clone().requires_grad_()          # :223
    pred_real = D(PD, img_real)                                     # :224
    img_fake = G(PG, z1).detach()                                   # :226-227
    img_fake_own = img_fake
    if fake_D is not None:
        img_fake = fake_D.detach().to(img_fake.dtype)
    pred_fake = D(PD, img_fake)                                     # :228
    L_real = bce_logits(pred_real, 1)                               # pggan/loss.py:18-21
    L_fake = bce_logits(pred_fake, 0)
    drift = None
    if gp_mode == "r1":
        reg = r1_reg(L_real, img_real)
    else:
        reg = wgan_gp(lambda t: D(PD, t), img_real.detach(), img_fake, gp_eps, W_gp)
        drift = drift_loss(pred_real, W_drift)
    L_D = L_real + L_fake + reg + (drift if drift is not None else 0.0)
    dkeys = list(PD.keys())
    gd = torch.autograd.grad(L_D, [PD[k] for k in dkeys], allow_unused=True)
    grads_D = dict(zip(dkeys, gd))
    with torch.no_grad():
        optD.update(PD, grads_D if grads_D_update is None else grads_D_update)   # lib/utils.py:72-75

    img_fake_G = G(PG, z2)                                          # :244-245
    img_fake_G_own = img_fake_G
    if fake_G is not None:
        img_fake_G = img_fake_G + (fake_G.to(img_fake_G.dtype) - img_fake_G).detach()
    pred_fake_G = D(PD, img_fake_G)                                 # :246
    L_G = W_adv * bce_logits(pred_fake_G, 1)                        # pggan/loss.py:5-14
    gkeys = list(PG.keys())
    gg = torch.autograd.grad(L_G, [PG[k] for k in gkeys], allow_unused=True)
    grads_G = dict(zip(gkeys, gg))
    with torch.no_grad():
        optG.update(PG, grads_G)
    for P in (PG, PD):
        for k in P:
            P[k].requires_grad_(False)
    return StepOut(img_real.detach(), img_fake_own, img_fake_G_own.detach(), pred_real.detach(),
                   pred_fake.detach(), pred_fake_G.detach(), L_real.item(), L_fake.item(),
                   float(reg.detach()) if torch.is_tensor(reg) else float(reg), L_D.item(), L_G.item(),
                   {k: (None if v is None else v.detach()) for k, v in grads_D.items()},
                   {k: (None if v is None else v.detach()) for k, v in grads_G.items()},
                   float(drift.detach()) if drift is not None else 0.0)
