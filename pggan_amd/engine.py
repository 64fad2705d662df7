"""Hand-scheduled PGGAN training step (G + D + R1) on the HIP kernels.

The reference step (pggan/model.py:206-255) relies on autograd, including a
double-backward for the R1 penalty (lib/loss.py:125-135).  Here every pass is
an explicit kernel sequence and the R1 double-backward is derived by hand:

  F   forward of D on the real image, keeping every activation
  B1  input-gradient pass from u = dL_real/dlogit, keeping the gradient at
      every pre-activation (gz) and producing g = dL_real/dx
  R1  r1 = 0.5 mean_b |g_b|^2 ;  gbar = dR1/dg = g / B
  T   tangent pass: gbar pushed forward through D (the transpose of B1):
      conv -> *lrelu'(z) -> pool -> blend ...; at every weight layer the R1
      weight term  dW += c * gz (x) t_in  (the B1 gz paired with the tangent at
      the layer input) is accumulated.  Two second-order injections appear at
      the non-piecewise-linear ops: at minibatch-stddev (d/dx <t, J^T gy>) and
      at the logit (t_out * sigma(l)sigma(-l)/B through the BCE derivative).
  B2  full backward from u + t_out*h with the mbstd injection added: the weight
      gradient of L_real plus the indirect part of dR1/dtheta.
then the fake-image forward/backward (L_fake) and Adam; the G half runs G fwd,
D fwd, D input-gradient (no D weight gradient: the reference computes and then
discards it), G backward and Adam.

Activations are NHWC in the engine's storage dtype (fp32 parity mode or bf16),
images NCHW fp32, parameters/gradients/Adam state fp32 in flat buffers.
"""
from __future__ import annotations

import contextlib
import math
import os
from dataclasses import dataclass

import torch

from . import _lib as L

SLOPE = 0.2  # blocks hard-code LeakyReLU(0.2) (lib/blocks.py:127,137,185,192,254,283)


def cinp(c):
    """Channel padding the conv kernels expect for their input."""
    return ((c + 7) // 8) * 8 if c <= 16 else ((c + 31) // 32) * 32


def r4(c):
    return (c + 3) // 4 * 4


def he(fan_in):
    return math.sqrt(2.0 / fan_in)


# ---------------------------------------------------------------------------
# Parameter naming (reference state_dict order, see oracle / SURVEY §8(b))
# ---------------------------------------------------------------------------
def g_param_shapes(depths, s, latent_dim=512, out_dim=3):
    d0 = depths[0]
    sh = []
    for i in range(s):
        p, n = depths[i], depths[i + 1]
        sh += [(f"blocks.{i}.block.0.module.weight", (n, p, 3, 3)),
               (f"blocks.{i}.block.0.module.bias", (n,)),
               (f"blocks.{i}.block.3.module.weight", (n, n, 3, 3)),
               (f"blocks.{i}.block.3.module.bias", (n,))]
    for i in range(s + 1):
        sh += [(f"toRGB_blocks.{i}.toRGB.module.weight", (out_dim, depths[i], 1, 1)),
               (f"toRGB_blocks.{i}.toRGB.module.bias", (out_dim,))]
    sh += [("latent_format_layer.module.weight", (16 * d0, latent_dim)),
           ("latent_format_layer.module.bias", (16 * d0,)),
           ("first_block.block.0.module.weight", (d0, d0, 3, 3)),
           ("first_block.block.0.module.bias", (d0,))]
    return sh


def d_param_shapes(depths, s, in_dim=3):
    d0 = depths[0]
    sh = []
    for i in range(s):
        n, p = depths[i + 1], depths[i]
        sh += [(f"blocks.{i}.block.0.module.weight", (n, n, 3, 3)),
               (f"blocks.{i}.block.0.module.bias", (n,)),
               (f"blocks.{i}.block.2.module.weight", (p, n, 3, 3)),
               (f"blocks.{i}.block.2.module.bias", (p,))]
    for i in range(s + 1):
        sh += [(f"fromRGB_blocks.{i}.fromRGB.module.weight", (depths[i], in_dim, 1, 1)),
               (f"fromRGB_blocks.{i}.fromRGB.module.bias", (depths[i],))]
    sh += [("decision_layer.module.weight", (1, d0)),
           ("decision_layer.module.bias", (1,)),
           ("minibatch_normalization_block.conv.module.weight", (d0, d0 + 1, 3, 3)),
           ("minibatch_normalization_block.conv.module.bias", (d0,)),
           ("minibatch_normalization_block.linear.module.weight", (d0, 16 * d0)),
           ("minibatch_normalization_block.linear.module.bias", (d0,))]
    return sh


def dead_params(net, s):
    """Parameters the forward never touches at stage s (their grad stays None in the
    reference and Adam skips them): toRGB / fromRGB blocks below s-1."""
    pre = "toRGB_blocks" if net == "G" else "fromRGB_blocks"
    return {f"{pre}.{j}.{'toRGB' if net == 'G' else 'fromRGB'}.module.{k}"
            for j in range(max(0, s - 1)) for k in ("weight", "bias")}


class FlatParams:
    """fp32 parameters of one net in one flat buffer (live parameters first) plus
    flat gradient / Adam-moment buffers; `views[name]` are reference-shaped views."""

    def __init__(self, shapes, dead, device, init=None):
        order = [n for n, _ in shapes if n not in dead] + [n for n, _ in shapes if n in dead]
        shp = dict(shapes)
        self.names = [n for n, _ in shapes]          # reference order
        # every tensor starts on a 64-byte boundary (vector loads in the kernels); the
        # padding slots stay zero (zero gradient -> Adam leaves them at zero)
        self.offsets, self.spans, off = {}, {}, 0
        self.n_live = 0
        for n in order:
            self.offsets[n] = off
            padded = (int(math.prod(shp[n])) + 15) // 16 * 16
            self.spans[n] = (off, off + padded)     # incl. the zero padding slots
            off += padded
            if n not in dead:
                self.n_live = off
        self.numel = off
        self.flat = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros_like(self.flat)
        self.m = torch.zeros_like(self.flat)
        self.v = torch.zeros_like(self.flat)
        self.step = 0
        # the step count Adam reads on the device (pg_adam_dev: graph replay); _step_dev_host
        # is the value it is known to hold (None: unknown, rewritten before the next update)
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=device)
        self._step_dev_host = 0
        self.shapes = shp
        self.dead = set(dead)
        self.views = {n: self._view(self.flat, n) for n in self.names}
        self.gviews = {n: self._view(self.grad, n) for n in self.names}
        if init is not None:
            for n in self.names:
                self.views[n].copy_(init[n])

    def _view(self, buf, n):
        o = self.offsets[n]
        return buf[o:o + int(math.prod(self.shapes[n]))].view(self.shapes[n])

    def live_grad(self):
        return self.grad[:self.n_live]

    def reset_optimizer(self):
        self.m.zero_()
        self.v.zero_()
        self.step = 0


# ---------------------------------------------------------------------------
@dataclass
class Hyper:
    lr_G: float = 1e-4
    lr_D: float = 1e-5
    beta1: float = 0.0
    beta2: float = 0.99
    eps: float = 1e-8
    W_adv: float = 1.0
    slope_cfg: float = 0.2      # LReLU_slope (G format layer only, pggan/nets.py:45,129)
    gp_mode: str = "r1"         # "r1" (live reference path) | "wgan-gp" (optional mode)
    W_gp: float = 10.0
    W_drift: float = 0.0        # W_drift_D (wgan-gp mode only, pggan/loss.py:94-100)


# measurement only (bench.py's isolated instrumented step): run the side-stream launches
# inline on the current stream so per-launch HIP event durations exclude overlap
FORCE_SERIAL = False

# Schedule options: attributes of StepEngine, set by keyword (tests) or, for A/B runs, by ONE
# environment string PG_ENGINE="name=value,..." (tools/ab.sh).  Every default is the measured
# faster choice (DESIGN.md performance log); the alternatives stay because the engine needs them
# anyway (batch sizes that are not a multiple of 4, the bucketed DP exchange, the fp32 parity
# mode, the CPU test double).
ENGINE_DEFAULTS = dict(
    merge_d=True,          # the D half's real / fake forward and second backward at batch 2B
    merge_g=True,          # both generator forwards of a step at batch 2B
    side_stream=True,      # weight gradients on a least-priority side stream
    elide_zero_blend=True,  # alpha = 1: skip the exactly-zero fade-in branches
    fuse_pixnorm=True,     # PixelNorm in the G conv epilogues
    fuse_pnbwd=True,       # G PixelNorm backward in the input-gradient conv epilogue
    fuse_pn_pool=True,     # ... also after the pool of the next level's conv-a input gradient
    fuse_rgb_pnbwd=True,   # the toRGB input gradient with the top PixelNorm backward
    fuse_dbits=True,       # D conv+lrelu+pool outputs as sign bits (see _dbits)
    dbits_min_res=512,     # ... from this resolution; below it the unpool-pass bits (_ubits)
    fuse_ubits=True,
    fuse_rgbbits=True,     # the top fromRGB output's sign bits (see _rgbbits)
    # DP: the G all-reduce behind the next step's real-image part (-1: only where the exchange
    # spans more than one rank -- at one rank (bench.py --dp-exchange) there is no transfer to
    # hide and the reorder's bookkeeping measured slower, profiles/r6_dp_lines.txt)
    overlap_g_exchange=-1,
    tail_main=True,        # the last weight gradients of a final pass on the main stream
    sep_b2=True,           # the merged second backward writes its own gradient buffers
    fuse_rgbw=True,        # the final pass's fromRGB weight gradient in the top conv's epilogue
    fuse_rgbd=True,        # the fromRGB input gradient (+ norms, + R1 tangent term) there too
    fuse_torgb_wg=True,    # the toRGB weight gradient in the toRGB input-gradient pass
    tail_b=True,           # ... with tail_main: the top level's conv-b weight gradient too
    tail_levels=1,         # ... and both weight gradients of this many top levels
    fuse_rgbo=False,       # the toRGB output in the epilogue of the top conv b: measured -1 % (opt-in)
)


def engine_options(overrides=None):
    """ENGINE_DEFAULTS with the PG_ENGINE environment string and then `overrides` applied."""
    opts = dict(ENGINE_DEFAULTS)
    for item in filter(None, os.environ.get("PG_ENGINE", "").split(",")):
        k, _, v = item.partition("=")
        k = k.strip()
        if k not in opts:
            raise ValueError(f"PG_ENGINE: unknown option {k!r} (known: {sorted(opts)})")
        opts[k] = type(opts[k])(int(v)) if isinstance(opts[k], (bool, int)) else type(opts[k])(v)
    for k, v in (overrides or {}).items():
        if k not in opts:
            raise ValueError(f"unknown engine option {k!r}")
        opts[k] = v
    return opts


class StepEngine:
    """All device buffers and kernel schedules for one (stage, batch, dtype)."""

    def __init__(self, ops, depths, s, B, device, latent_dim=512, forward_only=None, **options):
        """forward_only: "G" or "D" allocates just that net's forward activations (the
        inference / sampling path of nets.Generator / nets.Discriminator.forward).
        options: schedule options (ENGINE_DEFAULTS)."""
        self.ops, self.depths, self.s, self.B = ops, list(depths), s, B
        self.forward_only = forward_only
        self.dev = device
        self.dt = ops.tdtype
        self.latent = latent_dim
        self.R = 4 * 2 ** s
        d = self.depths
        self.d0 = d[0]
        self.mcs = cinp(d[0] + 1)
        self.keep_fake_D = False
        for k, v in engine_options(options).items():
            setattr(self, k, v)
        self.ws = None          # split-K workspace (fp32), grown on first use
        self._ws_cache = {}
        self.plan = None        # pg_step_plan description (HIP library)
        if forward_only is None and hasattr(ops, "step_plan"):
            # the step's split-reduction workspace at once (pg_step_plan_workspace_size), so
            # no launch of the step allocates
            need, self.plan = ops.step_plan(self.depths, s, B)
            if need:
                self.ws = torch.empty((need + 3) // 4, dtype=torch.float32, device=device)
        # alpha == 1 (elide_zero_blend): the low-resolution branches of the fade-in (toRGB /
        # fromRGB of the previous level, the real-image fade) are multiplied by exactly 0 in the
        # reference (pggan/nets.py:155-156,263-265, pggan/model.py:217-221) and contribute exactly
        # 0 to every output and gradient; elide them.  Their parameters
        # still get a zero gradient and the Adam step, as in the reference.
        self._last_dlow = True
        # trace(net, engine) after every G / D forward, or None: parity tests read the
        # leaky-ReLU region choices of each forward from the activation buffers
        self.trace = None
        # grad_ready(net, names) right after the last kernel writing those gradients in the
        # final backward pass of a half-step, or None (DP bucketing, pggan_amd.dp)
        self.grad_ready = None
        # weight gradients on a second stream (HIP device, training step): every conv wgrad
        # of a backward pass is off the pass's critical path (the input-gradient chain), so it
        # runs beside the next levels' convs -- at 4^2-32^2 neither launch fills the 256 CUs.
        # One side stream serialises the wgrads among themselves, so every dW accumulates in
        # the same order as on one stream.  _side_join() orders the side stream back into the
        # main one before anything overwrites a wgrad input or reads a gradient.  The stream is
        # the library's least-priority stream (pg_stream_create, one per device and process):
        # its own hardware-queue pool, so it never shares the main stream's queue (with a torch
        # pool stream the two landed on one queue in DP runs and serialised: 301 vs 351 img/s,
        # profiles/r4_side_queue_ab.txt).
        self.side = None
        self._side_ev = {}      # buffer-set key -> last side-stream event reading it
        self.ws_side = None
        if (forward_only is None and str(device).startswith("cuda") and self.side_stream and
                hasattr(ops, "side_stream")):
            self.side = ops.side_stream()
        # the cross-stream events: the library's device-scope-release events (pg_event_create).
        # torch's events release to system scope (each record writes back and invalidates every
        # XCD's L2).  Two rings: records on the side stream (the joins wait on those) and records
        # on the main stream (the side stream's waits): a slot is re-recorded only on its own
        # stream after 256 more records there, so a join that meets a re-recorded slot waits for
        # a later point of the same stream -- more ordering, never less.
        self._ev_side = self._ev_main = None
        self._ev_si = self._ev_mi = 0
        if self.side is not None and hasattr(ops, "event"):
            self._ev_side = [ops.event() for _ in range(256)]
            self._ev_main = [ops.event() for _ in range(256)]
        self._alloc()

    def _event(self, side):
        """The next event of the side-stream ring (side) or of the main-stream ring."""
        ring = self._ev_side if side else self._ev_main
        if ring is None:
            return None
        if side:
            ev, self._ev_si = ring[self._ev_si], (self._ev_si + 1) % len(ring)
        else:
            ev, self._ev_mi = ring[self._ev_mi], (self._ev_mi + 1) % len(ring)
        return ev

    # ------------------------------------------------------------------ buffers
    def _zero(self, t):
        """t.zero_() through the op set where it offers it (recordable, pg_fill_zero)."""
        if hasattr(self.ops, "zero_") and t.is_contiguous():
            self.ops.zero_(t)
        else:
            t.zero_()

    def _copy(self, dst, src):
        """dst.copy_(src) through the op set where possible (recordable, pg_copy)."""
        if (hasattr(self.ops, "copy_") and dst.is_contiguous() and src.is_contiguous() and
                dst.dtype == src.dtype and src.is_cuda and dst.numel() == src.numel()):
            self.ops.copy_(dst, src)
        else:
            dst.copy_(src)

    def _t(self, *shape, f32=False):
        return torch.zeros(*shape, dtype=torch.float32 if f32 else self.dt, device=self.dev)

    def _alloc(self):
        B, s, d, R = self.B, self.s, self.depths, self.R
        t = self._t
        fo = self.forward_only
        # forward_only: None (the training step), "G" / "D" (that net's forward), "Gtrain" /
        # "Dtrain" (that net's forward + first-order backward: the autograd modules)
        need_G, need_D = fo in (None, "G", "Gtrain"), fo in (None, "D", "Dtrain")
        train = fo in (None, "Gtrain", "Dtrain")
        merge_d = fo is None and B % 4 == 0 and self.merge_d
        # the D half's generator forward (the fake image) and the G half's use the same G
        # parameters (Adam_G runs after the G half): with merge_g they run as ONE forward at
        # batch 2B ([fake for D; fake for G], see _d_step_merged); the G buffers are
        # allocated at 2B, self.g holds first-half views and g_hi the G half's.
        # +1.5 % at C5 (profiles/r4_merge_g_ab.txt).
        merge_g = merge_d and self.merge_g
        GB = 2 * B if merge_g else B
        self._GBs = (B, 2 * B) if merge_g else (B,)
        self._g_done = False
        self._z_g = None
        # ---- G
        self.g = g = {}
        B0, B = B, GB
        if need_G:
            g["z"] = t(B, self.latent, f32=True)
            g["zn"] = t(B, self.latent, f32=True)
            g["f"] = t(B, 4, 4, d[0])
            g["h0"] = t(B, 4, 4, d[0])
            g["u0"] = t(B, 4, 4, d[0])
            g["y0"] = t(B, 4, 4, d[0])
            g["r0"] = t(B, 4, 4, 1, f32=True)
            for i in range(s):
                Ri = 8 * 2 ** i
                for k in ("ua", "ya", "ub", "yb") + (("gzb", "gya", "gza") if train else ()):
                    g[f"{k}{i}"] = t(B, Ri, Ri, d[i + 1])
                # per-pixel PixelNorm factors of the fused conv epilogues (G-half backward)
                g[f"ra{i}"] = t(B, Ri, Ri, 1, f32=True)
                g[f"rb{i}"] = t(B, Ri, Ri, 1, f32=True)
            g["img"] = t(B, 3, R, R, f32=True)
        if need_G and train:
            # gradient wrt level outputs: lvl 0 = y0 (4x4), lvl i+1 = yb_i
            for j in range(s + 1):
                Rj = 4 * 2 ** j
                g[f"gy{j}"] = t(B, Rj, Rj, d[j])
            g["gz0"] = t(B, 4, 4, d[0])
            g["gh0"] = t(B, 4, 4, d[0])
            g["gzf"] = t(B, 4, 4, d[0])
        B = B0
        self.g2 = self.g_hi = None
        if merge_g and need_G:
            self.g2 = g
            self.g = g = {k: v[:B] for k, v in self.g2.items()}
            self.g_hi = {k: v[B:] for k, v in self.g2.items()}
        self.g_lo = g
        # ---- D
        # the D half's real and fake passes share one forward and one second backward at
        # batch 2B (see _merged): the D buffers are allocated at 2B ([real; fake] along the
        # batch), self.dd holds first-half views (every batch-B pass: B1, the tangent, the G
        # half) and the generator's image is the second half of the merged input.  Needs
        # B % 4 == 0 so the minibatch-stddev groups (4 contiguous samples) stay within a half.
        self.dd2 = self.dd2b = None
        self._Bs = (B,)
        if merge_d:
            self._Bs = (B, 2 * B)
            self.dd2 = self._alloc_D(need_D, train, 2 * B)
            # the images [real; fake for D; fake for G]: D's merged input is the first two
            # thirds, the generator writes the last two
            x3 = t(3 * B, 3, R, R, f32=True)
            self.dd2["xin"] = x3[:2 * B]
            self.dd = {k: v[:B] for k, v in self.dd2.items()}
            self.dd_hi = {k: v[B:] for k, v in self.dd2.items()}
            # the merged second backward's gradient buffers: its own set, not the first-half
            # views B1 wrote, so it does not wait for the tangent pass's weight terms (side
            # stream) that still read B1's gradients (d_backward(join=False))
            self.dd2b = dict(self.dd2)
            if train and self.sep_b2:
                for k in self._dgrad_keys():
                    self.dd2b[k] = torch.zeros_like(self.dd2[k])
            g["img"] = x3[B:2 * B]
            if self.g2 is not None:
                self.g2["img"] = x3[B:]
                self.g_hi["img"] = x3[2 * B:]
        else:
            self.dd = self._alloc_D(need_D, train)
        # losses: 0 L_real, 1 L_fake, 2 reg (R1 or GP), 3 L_G, 4 drift (wgan-gp mode)
        self.loss = torch.zeros(8, dtype=torch.float32, device=self.dev)

    def _dgrad_keys(self):
        """The D buffers a backward pass writes (d_backward)."""
        ks = ["gzl1", "gzc", "gm", "gh", "gzrgb"] + (["gzd"] if self.s >= 1 else [])
        for i in range(self.s):
            ks += [f"gzb{i}", f"gza{i}", f"ghin{i}"]
        return ks

    def _alloc_D(self, need_D, train, B=None):
        B = self.B if B is None else B
        s, d, R = self.s, self.depths, self.R
        t = self._t
        D = {}
        if need_D:
            D["yrgb"] = t(B, R, R, d[s])
            # lrelu sign bits of the fromRGB output (see _rgbbits)
            D["rgbb"] = torch.zeros(B, R, R, (d[s] + 7) // 8, dtype=torch.uint8, device=self.dev)
            if s >= 1:
                D["yd"] = t(B, R // 2, R // 2, d[s - 1])
                D["hblend"] = t(B, R // 2, R // 2, d[s - 1])
            for i in range(s):
                Ri = 8 * 2 ** i
                # lrelu sign bits of the pre-pool conv-b output (used instead of bf{i} where
                # the kernels support it, see _dbits)
                D[f"mb{i}"] = torch.zeros(B, Ri, Ri, (d[i] + 7) // 8, dtype=torch.uint8,
                                          device=self.dev)
                D[f"a{i}"] = t(B, Ri, Ri, d[i + 1])
                D[f"bf{i}"] = t(B, Ri, Ri, d[i])
                D[f"p{i}"] = t(B, Ri // 2, Ri // 2, d[i])
            D["m"] = t(B, 4, 4, self.mcs)
            D["c"] = t(B, 4, 4, d[0])
            D["l1"] = t(B, d[0])
            D["logit"] = t(B, 1, f32=True)
        if need_D and train:
            D["gzrgb"] = t(B, R, R, d[s])
            D["trgb"] = t(B, R, R, d[s])
            if s >= 1:
                D["gzd"] = t(B, R // 2, R // 2, d[s - 1])
                D["td"] = t(B, R // 2, R // 2, d[s - 1])
                D["tblend"] = t(B, R // 2, R // 2, d[s - 1])
            for i in range(s):
                Ri = 8 * 2 ** i
                D[f"gzb{i}"] = t(B, Ri, Ri, d[i])
                D[f"gza{i}"] = t(B, Ri, Ri, d[i + 1])
                D[f"ghin{i}"] = t(B, Ri, Ri, d[i + 1])
                D[f"ta{i}"] = t(B, Ri, Ri, d[i + 1])
                D[f"tbf{i}"] = t(B, Ri, Ri, d[i])
                D[f"tp{i}"] = t(B, Ri // 2, Ri // 2, d[i])
            D["gzl1"] = t(B, d[0])
            D["gzc"] = t(B, 4, 4, d[0])
            D["gm"] = t(B, 4, 4, self.mcs)
            D["gh"] = t(B, 4, 4, d[0])
            D["tm"] = t(B, 4, 4, self.mcs)
            D["inj"] = t(B, 4, 4, d[0])
            D["tc"] = t(B, 4, 4, d[0])
            D["tl1"] = t(B, d[0])
            D["tout"] = t(B, 1, f32=True)
            D["u"] = t(B, f32=True)
            D["u2"] = t(B, f32=True)
            D["hl"] = t(B, f32=True)
            D["gimg"] = t(B, 3, R, R, f32=True)
            D["gbar"] = t(B, 3, R, R, f32=True)
            D["real"] = t(B, 3, R, R, f32=True)
            if s >= 1:
                D["real_in"] = t(B, 3, R, R, f32=True)
            # WGAN-GP optional mode
            D["interp"] = t(B, 3, R, R, f32=True)
            D["gp_eps"] = t(B, 1, f32=True)
            D["gp_c"] = t(B, 1, f32=True)         # 1 - eps
            # per-sample squared norms of dD/dx (kept at zero between uses: pg_penalty_scale
            # resets them) and the tangent pass's per-sample scale of dD/dx
            D["gp_norms"] = t(B, f32=True)
            D["gp_scale"] = t(B, f32=True)
            D["ones"] = torch.full((B,), 1.0, dtype=torch.float32, device=self.dev)
            D["zeros"] = torch.zeros((B,), dtype=torch.float32, device=self.dev)
        return D

    # ------------------------------------------------------------------ weights
    def _conv_list(self, net):
        """(key, weight name, cout, cin) of every 3x3 conv of a net at this stage."""
        d, s = self.depths, self.s
        out = []
        if net == "G":
            out.append(("first", "first_block.block.0.module", d[0], d[0]))
            for i in range(s):
                out.append((f"a{i}", f"blocks.{i}.block.0.module", d[i + 1], d[i]))
                out.append((f"b{i}", f"blocks.{i}.block.3.module", d[i + 1], d[i + 1]))
        else:
            out.append(("mb", "minibatch_normalization_block.conv.module", d[0], d[0] + 1))
            for i in range(s):
                out.append((f"a{i}", f"blocks.{i}.block.0.module", d[i + 1], d[i + 1]))
                out.append((f"b{i}", f"blocks.{i}.block.2.module", d[i], d[i + 1]))
        return out

    def alloc_packs(self):
        ops = self.ops
        self.packs = {}
        for net in (("G", "D") if self.forward_only is None else (self.forward_only[0],)):
            for key, _, cout, cin in self._conv_list(net):
                nf = ops.packed_elems(L.PACK_FWD, cout, cin)
                nd = ops.packed_elems(L.PACK_DGRAD, cout, cin)
                self.packs[(net, key)] = (
                    torch.empty(nf, dtype=self.dt, device=self.dev),
                    torch.empty(nd, dtype=self.dt, device=self.dev),
                    torch.empty(cout, dtype=torch.float32, device=self.dev),
                    he(cin * 9))

    def pack(self, net, P):
        """Fold the He constant into packed fwd/dgrad weights and scaled biases: one batched
        launch per net (table of pointers built once, rebuilt if a tensor moves)."""
        if not hasattr(self, "packs"):
            self.alloc_packs()
        if hasattr(self, "_packed"):
            self._packed[net] = True
        ops = self.ops
        if hasattr(ops, "pack_table"):
            ents = []
            for key, wname, cout, cin in self._conv_list(net):
                pf, pd, bs, c = self.packs[(net, key)]
                ents.append((P[wname + ".weight"], P[wname + ".bias"], pf, pd, bs, c))
            sig = tuple(t.data_ptr() for e in ents for t in (e[0], e[1]))
            tabs = self.__dict__.setdefault("_pack_tables", {})
            if net not in tabs or tabs[net][0] != sig:
                tabs[net] = (sig, ops.pack_table(ents))
            ops.conv_pack_batch(tabs[net][1])
            return
        for key, wname, cout, cin in self._conv_list(net):
            pf, pd, bs, c = self.packs[(net, key)]
            w = P[wname + ".weight"]
            ops.conv_pack(L.PACK_FWD, w, c, pf)
            ops.conv_pack(L.PACK_DGRAD, w, c, pd)
            ops.blend(c, P[wname + ".bias"], 0.0, None, bs)

    # ------------------------------------------------------------------ conv helpers
    def _conv(self, net, key, x, y, H, cin, cout, flags, aux=None, y2=None, out_scale=1.0,
              dgrad=False, bias=True, xbits=None):
        pf, pd, bs, _ = self.packs[(net, key)]
        if not dgrad and bias:
            flags |= L.CONV_BIAS
        need = self._ws_need("c", H, cin, cout, False)
        kw = dict(xbits=xbits) if xbits is not None else {}
        self.ops.conv3x3(x, pd if dgrad else pf, y, B=self.B, H=H, W=H, cin=cin, cout=cout,
                         flags=flags, slope=SLOPE, out_scale=out_scale,
                         bias=bs if (flags & L.CONV_BIAS) else None, aux=aux, y2=y2,
                         ws=self.ws if need else None, **kw)

    def _ws_bytes(self, kind, H, cin, cout, ups, B=None):
        """Split-reduction workspace bytes of a conv / wgrad launch (cached per shape)."""
        B = self.B if B is None else B
        key = (kind, H, cin, cout, ups, B)
        need = self._ws_cache.get(key)
        if need is None:
            if kind == "c":
                need = self.ops.conv_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout)
            else:
                need = self.ops.wgrad_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout,
                                                      ups=ups)
            self._ws_cache[key] = need
        return need

    def _ws_need(self, kind, H, cin, cout, ups, B=None):
        """_ws_bytes, growing the main stream's shared workspace to the largest need
        (launches on one stream are ordered)."""
        need = self._ws_bytes(kind, H, cin, cout, ups, B)
        if need and (self.ws is None or self.ws.numel() * 4 < need):
            self.ws = torch.empty((need + 3) // 4, dtype=torch.float32, device=self.dev)
        return need

    def _wgrad(self, net, key, x, gz, dW, H, cin, cout, ups=False, db=None, gzbits=None,
               gscale=1.0, main=False):
        """gzbits: gz is the pooled-resolution gradient g and the conv's output gradient is
        gscale * up2(g) * lrelu'(gzbits) (never materialised).  main: on the current stream
        even with a side stream (the end of a final pass, _tail_main_on)."""
        c = self.packs[(net, key)][3]
        kw = dict(gzbits=gzbits, slope=SLOPE) if gzbits is not None else {}
        if self.side is None or FORCE_SERIAL or main:
            need = self._ws_need("w", H, cin, cout, ups)
            self.ops.conv_wgrad(x, gz, dW, B=self.B, H=H, W=H, cin=cin, cout=cout, ups=ups,
                                scale=c * gscale, db=db, ws=self.ws if need else None, **kw)
            return
        need = self._ws_bytes("w", H, cin, cout, ups)
        if need and (self.ws_side is None or self.ws_side.numel() * 4 < need):
            # the side stream may still read the old workspace
            self.side.synchronize()
            self.ws_side = torch.empty((need + 3) // 4, dtype=torch.float32, device=self.dev)
        self._side_call((net,), self.ops.conv_wgrad, x, gz, dW, B=self.B, H=H, W=H, cin=cin,
                        cout=cout, ups=ups, scale=c * gscale, db=db,
                        ws=self.ws_side if need else None, **kw)

    def _side_call(self, nets, fn, *a, **kw):
        """Run a weight-gradient launch `fn` on the side stream (or inline without one).
        nets: whose buffers it reads (joins before those are overwritten).  Its inputs were
        written on the main stream, so the side stream first waits for it."""
        if self.side is None or FORCE_SERIAL:
            return fn(*a, **kw)
        self._side_wait_main()
        with torch.cuda.stream(self.side):
            fn(*a, **kw)
        ev = self._event(True) or torch.cuda.Event()
        ev.record(self.side)
        for n in nets:
            self._side_ev[n] = ev

    def _side_wait_main(self):
        """The side stream waits for everything enqueued on the current stream so far."""
        ev = self._event(False)
        if ev is None:
            self.side.wait_stream(torch.cuda.current_stream())
        else:
            ev.record(torch.cuda.current_stream())
            ev.wait(self.side)

    def _side_join(self, net=None):
        """Order the side-stream launches that read `net`'s buffers (all of them when None)
        before whatever the current stream enqueues next: called before a pass overwrites a
        net's activation / gradient buffers, before Adam reads the gradients and at the end of
        each half-step (so callers reading gradients need no stream handling).  Events, not
        stream waits: a join never waits for side work of the other net's buffers."""
        if not self._side_ev:
            return
        keys = list(self._side_ev) if net is None else [net]
        cur = torch.cuda.current_stream()
        for k in keys:
            ev = self._side_ev.pop(k, None)
            if ev is not None:
                if isinstance(ev, torch.cuda.Event):
                    cur.wait_event(ev)
                else:
                    ev.wait(cur)

    def _tail_main_on(self):
        """Whether the final pass's last weight gradients run on the main stream."""
        return self.side is not None and not FORCE_SERIAL and self.tail_main

    def _tail_wait(self):
        """Before a main-stream weight gradient of the final pass: the side-stream launches
        issued before this pass (the tangent's weight terms it accumulates onto) are done."""
        ev, self._tail_ev = getattr(self, "_tail_ev", None), None
        if ev is not None:
            cur = torch.cuda.current_stream()
            if isinstance(ev, torch.cuda.Event):
                cur.wait_event(ev)
            else:
                ev.wait(cur)

    def _ready_main(self, net, *prefixes):
        """grad_ready for gradients written on the main stream: the callbacks run on the
        side stream (_ready), which first waits for the main one."""
        if self.grad_ready is None:
            return
        if self.side is not None:
            self._side_wait_main()
        self._ready(net, *prefixes)

    def _conv_sup(self):
        """ops.conv_supported at every batch size the D passes run (B, and 2B when the D
        half's passes are merged): a sign-bit layout decided once serves both."""
        f = getattr(self.ops, "conv_supported", None)
        if f is None:
            return None
        Bs = self._Bs
        return lambda B, **kw: all(f(B=b, **kw) for b in Bs)

    def _dbits(self, i):
        """Whether D level i keeps its conv-b (conv + lrelu + pool) output as sign bits only:
        the forward writes bits instead of the full-resolution activation, and every consumer
        of its lrelu' mask (input-gradient conv, weight gradient, R1 tangent) reads the bits
        and the pooled-resolution gradient directly (no unpool_mask pass)."""
        key = ("dbits", i, 0, 0, 0)
        if key not in self._ws_cache:
            f = self._conv_sup()
            d, Ri = self.depths, 8 * 2 ** i
            # below 512^2 the saved bytes no longer pay for the masking work in the staging
            ok = bool(self.fuse_dbits and f is not None and d[i] % 16 == 0 and
                      Ri >= self.dbits_min_res)
            if ok:
                B = self.B
                ok = (f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i],
                        flags=L.CONV_BIAS | L.CONV_LRELU | L.CONV_POOL | L.CONV_Y2_BITS)
                      and f(B=B, H=Ri, W=Ri, cin=d[i], cout=d[i + 1],
                            flags=L.CONV_UPS_IN | L.CONV_X_BITS | L.CONV_MASK)
                      and f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i],
                            flags=L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_POOL)
                      and f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i], flags=L.CONV_GZ_BITS))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _ubits(self, i):
        """Below the sign-bit resolution (_dbits false): D level i's conv b still keeps its
        pre-pool lrelu sign as bits instead of the bf16 activation where the pooled conv
        supports it (the wide LDS-DMA tile at 64^2-256^2): the input-gradient pass forms
        gzb = up2(g) * lrelu'(bits) in the unpool pass (pg_unpool_mask_bits), the R1 tangent
        masks and pools in its conv (no avgpool launch); gzb itself stays materialised for the
        input-gradient conv and the weight gradient."""
        key = ("ubits", i, 0, 0, 0)
        if key not in self._ws_cache:
            f = self._conv_sup()
            d, Ri, B = self.depths, 8 * 2 ** i, self.B
            ok = bool(f is not None and self.fuse_dbits and self.fuse_ubits and
                      not self._dbits(i) and d[i] % 16 == 0)
            if ok:
                ok = (f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i],
                        flags=L.CONV_BIAS | L.CONV_LRELU | L.CONV_POOL | L.CONV_Y2_BITS)
                      and f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i],
                            flags=L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_POOL))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _rgbbits(self):
        """Whether the top fromRGB layer also writes the sign bits of its output and its two
        lrelu' consumers -- the input gradient of the top conv a and the fromRGB tangent --
        mask from those bits instead of the bf16 activation (at >= the sign-bit resolution)."""
        key = ("rgbbits", 0, 0, 0, 0)
        if key not in self._ws_cache:
            f = self._conv_sup()
            d, s, R, B = self.depths, self.s, self.R, self.B
            ok = bool(f is not None and self.fuse_dbits and self.fuse_rgbbits and s >= 1 and
                      d[s] % 8 == 0 and
                      d[s] <= 64 and R >= self.dbits_min_res and
                      f(B=B, H=R, W=R, cin=d[s], cout=d[s], flags=L.CONV_MASK | L.CONV_AUX_BITS))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _rgbw(self):
        """Whether the final backward pass computes the top fromRGB weight / bias gradients in
        the epilogue of the top conv a's input gradient (PG_CONV_RGBW: that gradient, which only
        the fromRGB weight gradient reads in this pass, is never written)."""
        key = ("rgbw", 0, 0, 0, 0)
        if key not in self._ws_cache:
            f = self._conv_sup()
            d, s, R, B = self.depths, self.s, self.R, self.B
            ok = bool(self.fuse_rgbw and self._rgbbits() and hasattr(self.ops, "conv3x3_rgbw") and
                      f(B=B, H=R, W=R, cin=d[s], cout=d[s],
                        flags=L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_RGBW))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _rgbd(self):
        """Whether the input-gradient passes (the penalty's B1, the G half's) compute the top
        fromRGB input gradient, its squared norms and (R1) the tangent's fromRGB weight term in
        the epilogue of the top conv a's input gradient (PG_CONV_RGBD: that gradient is never
        written)."""
        key = ("rgbd", 0, 0, 0, 0)
        if key not in self._ws_cache:
            f = self._conv_sup()
            d, s, R, B = self.depths, self.s, self.R, self.B
            ok = bool(self.fuse_rgbd and self._rgbbits() and hasattr(self.ops, "conv3x3_rgbd") and
                      B <= 16 and
                      f(B=B, H=R, W=R, cin=d[s], cout=d[s],
                        flags=L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_RGBD))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _pn_pool(self, i):
        """Whether level i's conv-a input gradient (pooled to level i-1) also applies level
        i-1's conv-b PixelNorm + LReLU backward (PG_CONV_POOL | PG_CONV_PNBWD): level i-1's
        forward kept y and r (fused PixelNorm) and the kernel supports it (32 channels)."""
        key = ("pnpool", i, 0, 0, 0)
        if key not in self._ws_cache:
            f = getattr(self.ops, "conv_supported", None)
            d, Ri, B = self.depths, 8 * 2 ** i, self.B
            ok = bool(i >= 1 and f is not None and self.fuse_pn_pool and
                      self._pn_fused(Ri // 2, d[i], d[i], L.CONV_LRELU) and
                      f(B=B, H=Ri, W=Ri, cin=d[i + 1], cout=d[i],
                        flags=L.CONV_POOL | L.CONV_PNBWD))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _pn_fused(self, H, cin, cout, flags):
        """Whether this generator conv can run PixelNorm in its epilogue (all output
        channels in one tile of the kernel the library picks for the shape)."""
        key = ("pn", H, cin, cout, flags)
        if key not in self._ws_cache:
            f = getattr(self.ops, "conv_supported", None)
            ok = bool(self.fuse_pixnorm and f is not None)
            for b in self._GBs:   # the generator forward runs at B and, merged, at 2B
                need = self._ws_need("c", H, cin, cout, False, b)
                ok = ok and bool(f(B=b, H=H, W=H, cin=cin, cout=cout,
                                   flags=flags | L.CONV_PIXNORM | L.CONV_BIAS, ws_bytes=need))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _pnb_fused(self, H, cin, cout):
        """Whether conv a (cin -> cout, up2 input) of a generator block has its PixelNorm
        backward fused into the input-gradient conv of conv b (cout -> cout) that produces
        its upstream gradient: needs the fused forward (y and r stored) and a tile holding
        every channel."""
        key = ("pnb", H, cin, cout)
        if key not in self._ws_cache:
            f = getattr(self.ops, "conv_supported", None)
            ok = bool(self.fuse_pixnorm and self.fuse_pnbwd and f is not None and
                      self._pn_fused(H, cin, cout, L.CONV_UPS_IN | L.CONV_LRELU))
            if ok:
                need = self._ws_need("c", H, cout, cout, False)
                ok = bool(f(B=self.B, H=H, W=H, cin=cout, cout=cout, flags=L.CONV_PNBWD,
                            ws_bytes=need))
            self._ws_cache[key] = ok
        return self._ws_cache[key]

    def _g_conv_pn(self, key, x, u, y, r, H, cin, cout, flags, keep):
        """conv + lrelu + PixelNorm of a generator block (lib/blocks.py:126-139): fused
        (y and, for the backward, the per-pixel factor r) or conv -> u then pixnorm -> y."""
        if self._pn_fused(H, cin, cout, flags):
            self._conv("G", key, x, y, H, cin, cout, flags | L.CONV_PIXNORM, y2=r if keep else None)
        else:
            self._conv("G", key, x, u, H, cin, cout, flags)
            self.ops.pixnorm(u, y, cout)

    def _g_pn_bwd(self, key, u, y, r, gy, gz, H, cin, cout, flags):
        if self._pn_fused(H, cin, cout, flags):
            self.ops.pixnorm_lrelu_bwd_y(y, r, gy, gz, cout, SLOPE)
        else:
            self.ops.pixnorm_lrelu_bwd(u, gy, gz, cout, SLOPE)

    # ================================================================== G
    def g_forward(self, P, z, alpha, keep=True):
        """keep: store what g_backward needs (the G half); the D half only needs the image."""
        ops, g, d, s, B = self.ops, self.g, self.depths, self.s, self.B
        self._side_join("G")
        if z is not g["z"]:
            self._copy(g["z"], z)
        ops.pixnorm(g["z"], g["zn"], self.latent)                            # nets.py:124-125
        Wf = P["latent_format_layer.module.weight"]
        ops.linear(g["zn"], Wf, P["latent_format_layer.module.bias"], g["f"], B=B,
                   flags=L.LIN_BIAS | L.LIN_LRELU | L.LIN_OUT_CHW, scale=he(self.latent),
                   slope=self.hyper.slope_cfg)                                # :129-130
        ops.pixnorm(g["f"], g["h0"], d[0])                                   # :132-133
        self._g_conv_pn("first", g["h0"], g["u0"], g["y0"], g["r0"], 4, d[0], d[0], L.CONV_LRELU,
                        keep)                                                # blocks.py:131-139
        prev = g["y0"]
        rgbo = s >= 1 and not self._low(alpha) and self._rgbo()
        for i in range(s):                                                   # nets.py:144-149
            Ri = 8 * 2 ** i
            self._g_conv_pn(f"a{i}", prev, g[f"ua{i}"], g[f"ya{i}"], g[f"ra{i}"], Ri, d[i],
                            d[i + 1], L.CONV_UPS_IN | L.CONV_LRELU, keep)
            if i == s - 1 and rgbo:
                # the top conv b with the toRGB output in its epilogue (PG_CONV_RGBO: the top
                # activation is not read back by a separate toRGB pass)
                pf, _, bs, _ = self.packs[("G", f"b{i}")]
                pre = f"toRGB_blocks.{s}.toRGB.module."
                ops.conv3x3_rgbo(g[f"ya{i}"], pf, g[f"yb{i}"], B=B, H=Ri, W=Ri, cin=d[i + 1],
                                 cout=d[i + 1], flags=L.CONV_PIXNORM | L.CONV_LRELU | L.CONV_BIAS,
                                 bias=bs, y2=g[f"rb{i}"] if keep else None,
                                 w_rgb=P[pre + "weight"], b_rgb=P[pre + "bias"], c=he(d[s]),
                                 img=g["img"], slope=SLOPE)                   # nets.py:140-156
            else:
                self._g_conv_pn(f"b{i}", g[f"ya{i}"], g[f"ub{i}"], g[f"yb{i}"], g[f"rb{i}"], Ri,
                                d[i + 1], d[i + 1], L.CONV_LRELU, keep)
            prev = g[f"yb{i}"]
        if not rgbo:
            self._rgb_out(P, alpha)
        if self.trace is not None:
            self.trace("G", self)
        return g["img"]

    def _rgbo(self):
        """Whether the top conv b can write the toRGB output in its epilogue (PG_CONV_RGBO): the
        fused PixelNorm forward on a tile holding every channel, at every batch the G forward
        runs (B, and 2B merged)."""
        if "rgbo" not in self._ws_cache:
            s, d = self.s, self.depths
            f = getattr(self.ops, "conv_supported", None)
            ok = bool(self.fuse_rgbo and self.fuse_pixnorm and f is not None and
                      hasattr(self.ops, "conv3x3_rgbo") and
                      self._pn_fused(self.R, d[s], d[s], L.CONV_LRELU))
            if ok:
                flags = L.CONV_PIXNORM | L.CONV_LRELU | L.CONV_BIAS | L.CONV_RGBO
                ok = all(f(B=b, H=self.R, W=self.R, cin=d[s], cout=d[s], flags=flags, ws_bytes=0)
                         for b in (self.B, 2 * self.B))
            self._ws_cache["rgbo"] = ok
        return self._ws_cache["rgbo"]

    def _ylvl(self, j):
        return self.g["y0"] if j == 0 else self.g[f"yb{j - 1}"]

    def _low(self, alpha):
        """Whether the fade-in's low-resolution branch contributes (alpha < 1 at s >= 1)."""
        return self.s >= 1 and not (self.elide_zero_blend and alpha == 1.0)

    def _top_out(self, alpha):
        """D's output of the top block after the fade-in blend."""
        return self.dd["hblend"] if self._low(alpha) else self.dd[f"p{self.s - 1}"]

    def _rgb_out(self, P, alpha):
        s, d, g = self.s, self.depths, self.g
        w = P[f"toRGB_blocks.{s}.toRGB.module.weight"]
        kw = {}
        if self._low(alpha):
            kw = dict(xp=self._ylvl(s - 1), wp=P[f"toRGB_blocks.{s - 1}.toRGB.module.weight"],
                      bp=P[f"toRGB_blocks.{s - 1}.toRGB.module.bias"], cp=he(d[s - 1]), Cp=d[s - 1],
                      alpha=alpha)
        self.ops.rgb_out(self._ylvl(s), w, P[f"toRGB_blocks.{s}.toRGB.module.bias"], he(d[s]),
                         g["img"], B=self.B, R=self.R, C=d[s], **kw)   # nets.py:140-156

    def g_backward(self, P, GR, gimg, alpha):
        ops, g, d, s, B = self.ops, self.g, self.depths, self.s, self.B
        self._side_join("G")
        kw = {}
        low = self._low(alpha)
        if low:
            pre = f"toRGB_blocks.{s - 1}.toRGB.module."
            kw = dict(xp=self._ylvl(s - 1), wp=P[pre + "weight"], cp=he(d[s - 1]), Cp=d[s - 1],
                      alpha=alpha, gxp=g[f"gy{s - 1}"], dwp=GR[pre + "weight"],
                      dbp=GR[pre + "bias"])
        pre = f"toRGB_blocks.{s}.toRGB.module."
        # the toRGB input gradient with the top block's PixelNorm backward fused in
        # (pg_rgb_out_bwd_pn: the 16-channel 1024^2 dL/dy never goes through HBM); its weight
        # gradient on the side stream
        top_pn = (s >= 1 and not low and hasattr(ops, "rgb_out_bwd_pn") and d[s] in (16, 32) and
                  self.fuse_rgb_pnbwd and
                  self._pn_fused(self.R, d[s], d[s], L.CONV_LRELU))
        w_rgb = P[pre + "weight"]
        # the toRGB weight gradient in the same pass as the input gradient where the fused form
        # runs (y and gimg streamed once, on the main stream: rgb_dgrad_pn_wg_v)
        wg_fused = top_pn and self.fuse_torgb_wg
        if top_pn:
            ops.rgb_out_bwd_pn(self._ylvl(s), g[f"rb{s - 1}"], w_rgb, he(d[s]), gimg,
                               g[f"gzb{s - 1}"], B=B, R=self.R, C=d[s], slope=SLOPE,
                               **(dict(dw=GR[pre + "weight"], db=GR[pre + "bias"]) if wg_fused else {}))
        else:
            ops.rgb_out_bwd(self._ylvl(s), w_rgb, he(d[s]), gimg, g[f"gy{s}"], None, None,
                            B=B, R=self.R, C=d[s],
                            **{k: (None if k in ("dwp", "dbp") else v) for k, v in kw.items()})
        if wg_fused:
            self._ready_main("G", pre)
        else:
            # img / the fade-in branch's operands are D / G buffers: pending for both nets
            self._side_call(("G", "D"), ops.rgb_out_bwd, self._ylvl(s), w_rgb, he(d[s]), gimg, None,
                            GR[pre + "weight"], GR[pre + "bias"], B=B, R=self.R, C=d[s],
                            **{k: (None if k == "gxp" else v) for k, v in kw.items()})
            self._ready("G", pre, *([f"toRGB_blocks.{s - 1}.toRGB.module."] if s >= 1 else []))
        pn_done = s - 1 if top_pn else None   # level whose conv-b PixelNorm backward is done
        for i in reversed(range(s)):
            Ri = 8 * 2 ** i
            a, b = f"blocks.{i}.block.0.module.", f"blocks.{i}.block.3.module."
            if pn_done != i:
                self._g_pn_bwd(f"b{i}", g[f"ub{i}"], g[f"yb{i}"], g[f"rb{i}"], g[f"gy{i + 1}"],
                               g[f"gzb{i}"], Ri, d[i + 1], d[i + 1], L.CONV_LRELU)
            self._wgrad("G", f"b{i}", g[f"ya{i}"], g[f"gzb{i}"], GR[b + "weight"], Ri, d[i + 1],
                        d[i + 1],
                        db=GR[b + "bias"])
            self._ready("G", b)
            if self._pnb_fused(Ri, d[i], d[i + 1]):
                # conv b's input gradient with conv a's PixelNorm + LReLU backward in its
                # epilogue (the gradient w.r.t. ya never goes through HBM)
                self._conv("G", f"b{i}", g[f"gzb{i}"], g[f"gza{i}"], Ri, d[i + 1], d[i + 1],
                           L.CONV_PNBWD, dgrad=True, aux=g[f"ya{i}"], y2=g[f"ra{i}"])
            else:
                self._conv("G", f"b{i}", g[f"gzb{i}"], g[f"gya{i}"], Ri, d[i + 1], d[i + 1], 0,
                           dgrad=True)
                self._g_pn_bwd(f"a{i}", g[f"ua{i}"], g[f"ya{i}"], g[f"ra{i}"], g[f"gya{i}"],
                               g[f"gza{i}"], Ri, d[i], d[i + 1], L.CONV_UPS_IN | L.CONV_LRELU)
            self._wgrad("G", f"a{i}", self._ylvl(i), g[f"gza{i}"], GR[a + "weight"], Ri, d[i],
                        d[i + 1], ups=True,
                        db=GR[a + "bias"])
            self._ready("G", a)
            # level s-1 also received the toRGB fade-in branch's gradient: accumulate
            flags = L.CONV_POOL | (L.CONV_ACCUM if (i == s - 1 and low) else 0)
            if not (flags & L.CONV_ACCUM) and self._pn_pool(i):
                # the level below's conv-b PixelNorm backward after the pool, in this launch
                self._conv("G", f"a{i}", g[f"gza{i}"], g[f"gzb{i - 1}"], Ri, d[i + 1], d[i],
                           L.CONV_POOL | L.CONV_PNBWD, dgrad=True, out_scale=1.0,
                           aux=g[f"yb{i - 1}"], y2=g[f"rb{i - 1}"])
                pn_done = i - 1
            else:
                self._conv("G", f"a{i}", g[f"gza{i}"], g[f"gy{i}"], Ri, d[i + 1], d[i], flags,
                           dgrad=True, out_scale=1.0)                 # up2 backward = 2x2 sum
        fb = "first_block.block.0.module."
        self._g_pn_bwd("first", g["u0"], g["y0"], g["r0"], g["gy0"], g["gz0"], 4, d[0], d[0],
                       L.CONV_LRELU)
        # the input-gradient chain ends at the latent: with tail_main the last two weight
        # gradients run on the main stream after it while the side stream drains its queue
        tail = self._tail_main_on()
        if not tail:
            self._wgrad("G", "first", g["h0"], g["gz0"], GR[fb + "weight"], 4, d[0], d[0],
                        db=GR[fb + "bias"])
            self._ready("G", fb)
        self._conv("G", "first", g["gz0"], g["gh0"], 4, d[0], d[0], 0, dgrad=True)
        ops.pixnorm_lrelu_bwd(g["f"], g["gh0"], g["gzf"], d[0], self.hyper.slope_cfg)
        lin = (g["zn"], g["gzf"], GR["latent_format_layer.module.weight"],
               GR["latent_format_layer.module.bias"])
        lkw = dict(B=B, flags=L.LIN_OUT_CHW, scale=he(self.latent))
        if tail:
            self._wgrad("G", "first", g["h0"], g["gz0"], GR[fb + "weight"], 4, d[0], d[0],
                        db=GR[fb + "bias"], main=True)
            ops.linear_wgrad(*lin, **lkw)
            self._ready_main("G", fb, "latent_format_layer.module.")
        else:
            self._side_call(("G",), ops.linear_wgrad, *lin, **lkw)
            self._ready("G", "latent_format_layer.module.")

    # ================================================================== D
    def d_forward(self, P, img, alpha, join=True):
        ops, D, d, s, B, R = self.ops, self.dd, self.depths, self.s, self.B, self.R
        if join:
            self._side_join("D")
        fr = "fromRGB_blocks.{}.fromRGB.module."
        ops.from_rgb(img, P[fr.format(s) + "weight"], P[fr.format(s) + "bias"], he(3), D["yrgb"],
                     B=B, R=R, C=d[s], down=False, slope=SLOPE,            # nets.py:255
                     **(dict(ybits=D["rgbb"]) if self._rgbbits() else {}))
        low = self._low(alpha)
        self._last_dlow = low
        if low:
            ops.from_rgb(img, P[fr.format(s - 1) + "weight"], P[fr.format(s - 1) + "bias"], he(3),
                         D["yd"], B=B, R=R // 2, C=d[s - 1], down=True, slope=SLOPE)  # :251-252
        h = D["yrgb"]
        for i in reversed(range(s)):                                           # :260-265
            Ri = 8 * 2 ** i
            self._conv("D", f"a{i}", h, D[f"a{i}"], Ri, d[i + 1], d[i + 1], L.CONV_LRELU)
            if self._dbits(i):
                self._conv("D", f"b{i}", D[f"a{i}"], D[f"p{i}"], Ri, d[i + 1], d[i],
                           L.CONV_LRELU | L.CONV_POOL | L.CONV_Y2_BITS, y2=D[f"mb{i}"],
                           out_scale=0.25)
            elif self._ubits(i):
                self._conv("D", f"b{i}", D[f"a{i}"], D[f"p{i}"], Ri, d[i + 1], d[i],
                           L.CONV_LRELU | L.CONV_POOL | L.CONV_Y2_BITS, y2=D[f"mb{i}"],
                           out_scale=0.25)
            else:
                self._conv("D", f"b{i}", D[f"a{i}"], D[f"p{i}"], Ri, d[i + 1], d[i],
                           L.CONV_LRELU | L.CONV_POOL, y2=D[f"bf{i}"], out_scale=0.25)
            if i == s - 1 and low:
                ops.blend(1.0 - alpha, D["yd"], alpha, D[f"p{i}"], D["hblend"])
                h = D["hblend"]
            else:
                h = D[f"p{i}"]
        self.h_mb = h
        # the D-buffer key of the mbstd input (the merged second backward needs its 2B view)
        self.h_mb_key = "yrgb" if s == 0 else ("hblend" if (s == 1 and low) else "p0")
        ops.mbstd_fwd(h, D["m"], B=B, HW=16, C=d[0])                           # blocks.py:261
        self._conv("D", "mb", D["m"], D["c"], 4, d[0] + 1, d[0], L.CONV_LRELU)
        mb = "minibatch_normalization_block.linear.module."
        ops.linear(D["c"], P[mb + "weight"], P[mb + "bias"], D["l1"], B=B,
                   flags=L.LIN_BIAS | L.LIN_LRELU | L.LIN_IN_CHW, scale=he(16 * d[0]), slope=SLOPE)
        ops.linear(D["l1"], P["decision_layer.module.weight"], P["decision_layer.module.bias"],
                   D["logit"], B=B, flags=L.LIN_BIAS, scale=he(d[0]))          # nets.py:271
        if self.trace is not None:
            self.trace("D", self)
        return D["logit"]

    def _ready(self, net, *prefixes):
        if self.grad_ready is None:
            return
        names = [p + k for p in prefixes for k in ("weight", "bias")]
        if self.side is None:
            self.grad_ready(net, names)
            return
        # every parameter gradient is written on the side stream (_side_call / _wgrad: the
        # conv, linear, to/fromRGB weight and bias gradients; the zero fill before the step is
        # ordered ahead of them by the side stream's wait for the main one at each launch), so
        # the callback runs on the side stream and a collective it starts sees the finished
        # gradients in stream order -- no main-stream event record (each costs the main
        # stream's next kernel ~6.5 us; round 4 recorded one per bucket launch)
        with torch.cuda.stream(self.side):
            self.grad_ready(net, names)

    def d_backward(self, P, GR, u, alpha, img=None, gimg=None, inj_mbstd=None, final=False,
                   gimg_overwrite=False, norms=None, join=True, t_dw=None):
        """Backward from u = dL/dlogit.  GR: grad views (None -> input-gradient only);
        gimg: accumulate dL/dimg (zeroed by the caller unless gimg_overwrite: the first
        fromRGB input gradient then writes it); norms: += per-sample sum of dL/dimg^2, fused
        into the last pass writing gimg; keeps every gz.  img: the D input (a tensor or an
        _lib.ImgMix) for the fromRGB weight gradients.
        final: the last pass writing D's gradients this half-step (grad_ready calls); its top
        level's conv-a and fromRGB weight gradients run on the main stream (_tail_main).
        join=False: the pass writes buffers no pending side-stream launch reads (the merged
        second backward's own set, dd2b)."""
        ops, D, d, s, B, R = self.ops, self.dd, self.depths, self.s, self.B, self.R
        if join:
            self._side_join("D")
        # the side-stream point after every weight term issued so far (the tangent's): a
        # main-stream weight gradient accumulating onto one of them waits for it
        self._tail_ev = self._side_ev.get("D")
        tail = final and GR is not None and self._tail_main_on()
        fr = "fromRGB_blocks.{}.fromRGB.module."
        rgbw = (tail and gimg is None and s >= 1 and isinstance(img, torch.Tensor) and
                self._rgbw())
        # the input-gradient passes: gimg (+ norms, + the R1 tangent's fromRGB weight term
        # t_dw, s / B) from the top conv a's epilogue (t_dw only without the fade-in branch,
        # whose gradient joins gimg afterwards)
        rgbd = (GR is None and gimg is not None and gimg_overwrite and s >= 1 and self._rgbd())
        low_a = self._low(alpha)
        self._t_rgb_done = bool(rgbd and t_dw is not None and not low_a)
        ready = (lambda *p: self._ready("D", *p)) if final else (lambda *p: None)
        dec = "decision_layer.module."
        lin = "minibatch_normalization_block.linear.module."
        if GR is not None:
            self._side_call(("D",), ops.linear_wgrad,
                            D["l1"], u, GR[dec + "weight"], GR[dec + "bias"], B=B, flags=0,
                            scale=he(d[0]))
            ready(dec)
        ops.linear_dgrad(u, P[dec + "weight"], D["gzl1"], B=B, flags=L.LIN_MASK, scale=he(d[0]),
                         slope=SLOPE, aux=D["l1"])
        if GR is not None:
            self._side_call(("D",), ops.linear_wgrad,
                            D["c"], D["gzl1"], GR[lin + "weight"], GR[lin + "bias"], B=B,
                            flags=L.LIN_IN_CHW, scale=he(16 * d[0]))
            ready(lin)
        ops.linear_dgrad(D["gzl1"], P[lin + "weight"], D["gzc"], B=B,
                         flags=L.LIN_IN_CHW | L.LIN_MASK, scale=he(16 * d[0]), slope=SLOPE,
                         aux=D["c"])
        if GR is not None:
            cv = "minibatch_normalization_block.conv.module."
            self._wgrad("D", "mb", D["m"], D["gzc"], GR[cv + "weight"], 4, d[0] + 1, d[0],
                        db=GR[cv + "bias"])
            ready(cv)
        self._conv("D", "mb", D["gzc"], D["gm"], 4, d[0], r4(d[0] + 1), 0, dgrad=True)
        ops.mbstd_bwd(self.h_mb, D["gm"], D["gh"], B=B, HW=16, C=d[0])
        if inj_mbstd is not None:
            ops.blend(1.0, D["gh"], 1.0, inj_mbstd, D["gh"])
        g = D["gh"]
        low = self._low(alpha)
        tail_jobs = []   # (order, _wgrad args, kwargs, grad_ready prefix) run at the tail
        for i in range(s):
            Ri = 8 * 2 ** i
            a, b = f"blocks.{i}.block.0.module.", f"blocks.{i}.block.2.module."
            if i == s - 1 and low:
                # blend backward: the low-res branch gets (1-alpha) g (nets.py:263-265)
                ops.unpool_mask(g, D["yd"], D["gzd"], B=B, H=Ri // 2, W=Ri // 2, C=d[i],
                                scale=1.0 - alpha, slope=SLOPE, ups=False)
            sc = 0.25 * (alpha if i == s - 1 else 1.0)
            # the final pass's top-level weight gradients on the main stream after its
            # input-gradient chain (tail_main / tail_b / tail_levels): the side stream's queue
            # is the step's critical path at this point
            in_tail = tail and i >= s - max(1, self.tail_levels)
            tail_b = in_tail and (i < s - 1 or self.tail_b)
            if self._dbits(i):
                # gzb = sc * up2(g) * lrelu'(bits): read by the kernels from g and the bits
                wgb = dict(db=GR[b + "bias"], gzbits=D[f"mb{i}"], gscale=sc) if GR is not None else None
                if GR is not None and not tail_b:
                    self._wgrad("D", f"b{i}", D[f"a{i}"], g, GR[b + "weight"], Ri, d[i + 1], d[i],
                                **wgb)
                    ready(b)
                elif tail_b:
                    tail_jobs.append(((-i, 1), (f"b{i}", D[f"a{i}"], g, GR[b + "weight"], Ri,
                                                d[i + 1], d[i]), wgb, b))
                self._conv("D", f"b{i}", g, D[f"gza{i}"], Ri, d[i], d[i + 1],
                           L.CONV_MASK | L.CONV_UPS_IN | L.CONV_X_BITS, aux=D[f"a{i}"],
                           dgrad=True, out_scale=sc, xbits=D[f"mb{i}"])
            else:
                if self._ubits(i):
                    ops.unpool_mask(g, None, D[f"gzb{i}"], B=B, H=Ri, W=Ri, C=d[i], scale=sc,
                                    slope=SLOPE, ups=True, bits=D[f"mb{i}"])
                else:
                    ops.unpool_mask(g, D[f"bf{i}"], D[f"gzb{i}"], B=B, H=Ri, W=Ri, C=d[i], scale=sc,
                                    slope=SLOPE, ups=True)
                wgb = dict(db=GR[b + "bias"]) if GR is not None else None
                if GR is not None and not tail_b:
                    self._wgrad("D", f"b{i}", D[f"a{i}"], D[f"gzb{i}"], GR[b + "weight"], Ri,
                                d[i + 1], d[i], **wgb)
                    ready(b)
                elif tail_b:
                    tail_jobs.append(((-i, 1), (f"b{i}", D[f"a{i}"], D[f"gzb{i}"], GR[b + "weight"],
                                                Ri, d[i + 1], d[i]), wgb, b))
                self._conv("D", f"b{i}", D[f"gzb{i}"], D[f"gza{i}"], Ri, d[i], d[i + 1],
                           L.CONV_MASK, aux=D[f"a{i}"], dgrad=True)
            hin = D["yrgb"] if i == s - 1 else (self._top_out(alpha) if i == s - 2 else D[f"p{i + 1}"])
            top_tail = tail and i == s - 1
            if GR is not None and not in_tail:
                self._wgrad("D", f"a{i}", hin, D[f"gza{i}"], GR[a + "weight"], Ri, d[i + 1],
                            d[i + 1],
                            db=GR[a + "bias"])
                ready(a)
            elif in_tail:
                tail_jobs.append(((-i, 0), (f"a{i}", hin, D[f"gza{i}"], GR[a + "weight"], Ri,
                                            d[i + 1], d[i + 1]), dict(db=GR[a + "bias"]), a))
            if i == s - 1 and rgbd:
                fw = fr.format(s) + "weight"
                ops.conv3x3_rgbd(D[f"gza{i}"], self.packs[("D", f"a{i}")][1], B=B, H=Ri, W=Ri,
                                 cin=d[i + 1], cout=d[i + 1], flags=L.CONV_MASK | L.CONV_AUX_BITS,
                                 slope=SLOPE, aux=D["rgbb"], w_rgb=P[fw], f=he(3), gimg=gimg,
                                 norms=None if low_a else norms,
                                 dw=t_dw if self._t_rgb_done else None, s=he(3) / B)
            elif i == s - 1 and rgbw:
                # the fromRGB weight gradient in this conv's epilogue: its result is not stored
                self._tail_wait()   # after the tangent's fromRGB weight term (side stream)
                fw = fr.format(s)
                ops.conv3x3_rgbw(D[f"gza{i}"], self.packs[("D", f"a{i}")][1], B=B, H=Ri, W=Ri,
                                 cin=d[i + 1], cout=d[i + 1], flags=L.CONV_MASK | L.CONV_AUX_BITS,
                                 slope=SLOPE, aux=D["rgbb"], img=img, s=he(3),
                                 dw=GR[fw + "weight"], db=GR[fw + "bias"])
            elif i == s - 1 and self._rgbbits():
                self._conv("D", f"a{i}", D[f"gza{i}"], D["gzrgb"], Ri, d[i + 1], d[i + 1],
                           L.CONV_MASK | L.CONV_AUX_BITS, aux=D["rgbb"], dgrad=True)
            elif i == s - 1:
                self._conv("D", f"a{i}", D[f"gza{i}"], D["gzrgb"], Ri, d[i + 1], d[i + 1],
                           L.CONV_MASK, aux=D["yrgb"], dgrad=True)
            else:
                self._conv("D", f"a{i}", D[f"gza{i}"], D[f"ghin{i}"], Ri, d[i + 1], d[i + 1], 0,
                           dgrad=True)
                g = D[f"ghin{i}"]
            if top_tail:
                # the input-gradient chain ends here: the deferred weight gradients on the main
                # stream (idle otherwise) while the side stream drains its queue, the top
                # level's first, conv a before conv b
                self._tail_wait()
                for _, args, kw, pre in sorted(tail_jobs, key=lambda j: j[0]):
                    self._wgrad("D", *args, main=True, **kw)
                    self._ready_main("D", pre)
        if s == 0:
            ops.unpool_mask(D["gh"], D["yrgb"], D["gzrgb"], B=B, H=4, W=4, C=d[0], scale=1.0,
                            slope=SLOPE, ups=False)
        fr = "fromRGB_blocks.{}.fromRGB.module."
        w = P[fr.format(s) + "weight"]
        if rgbw:
            self._ready_main("D", fr.format(s))
        elif GR is not None and tail and gimg is None:
            self._tail_wait()
            ops.from_rgb_bwd(D["gzrgb"], w, he(3), B=B, R=R, C=d[s], down=False, img=img,
                             dw=GR[fr.format(s) + "weight"], db=GR[fr.format(s) + "bias"])
            self._ready_main("D", fr.format(s))
        elif GR is not None:
            # img may be the generator's output buffer (fake pass): pending for both nets
            self._side_call(("D", "G"), ops.from_rgb_bwd,
                            D["gzrgb"], w, he(3), B=B, R=R, C=d[s], down=False, img=img,
                            dw=GR[fr.format(s) + "weight"], db=GR[fr.format(s) + "bias"])
            ready(fr.format(s))
        if gimg is not None and not rgbd:
            ops.from_rgb_bwd(D["gzrgb"], w, he(3), B=B, R=R, C=d[s], down=False, gimg=gimg,
                             **self._gimg_kw(gimg_overwrite, None if low else norms))
        if low:
            w1 = P[fr.format(s - 1) + "weight"]
            if GR is not None:
                self._side_call(("D", "G"), ops.from_rgb_bwd,
                                D["gzd"], w1, he(3), B=B, R=R // 2, C=d[s - 1], down=True, img=img,
                                dw=GR[fr.format(s - 1) + "weight"],
                                db=GR[fr.format(s - 1) + "bias"])
                ready(fr.format(s - 1))
            if gimg is not None:
                ops.from_rgb_bwd(D["gzd"], w1, he(3), B=B, R=R // 2, C=d[s - 1], down=True,
                                 gimg=gimg, **self._gimg_kw(False, norms))

    @staticmethod
    def _gimg_kw(overwrite, norms):
        kw = {}
        if overwrite:
            kw["gimg_overwrite"] = True
        if norms is not None:
            kw["norms"] = norms
        return kw

    def _fused_penalty(self):
        """The penalties' squared norms fused into the input-gradient pass and their weighted
        gradient read by the tangent pass through an image mix (the ops support it)."""
        return hasattr(self.ops, "penalty_scale")

    def _input_grad(self, P, u, alpha, mode, w=0.0, GR=None):
        """B1 of a penalty: dD/dx into D["gimg"] from the upstream u, the penalty into
        loss[2] and the tangent pass's input gbar (R1: g / B; WGAN-GP: the weighted g).
        GR (R1): the D gradients, so the tangent's fromRGB weight term can be taken in this
        pass (PG_CONV_RGBD; d_tangent then skips it)."""
        ops, D, B = self.ops, self.dd, self.B
        if self._fused_penalty():
            fw = f"fromRGB_blocks.{self.s}.fromRGB.module.weight"
            self.d_backward(P, None, u, alpha, gimg=D["gimg"], gimg_overwrite=True,
                            norms=D["gp_norms"],
                            t_dw=GR[fw] if (GR is not None and mode == "r1") else None)
            ops.penalty_scale(mode, D["gp_norms"], w, self.loss[2:3], D["gp_scale"])
            return L.ImgMix(D["gimg"], a=D["gp_scale"])
        D["gimg"].zero_()
        self.d_backward(P, None, u, alpha, gimg=D["gimg"])
        if mode == "r1":
            ops.r1_penalty(D["gimg"], B, self.loss[2:3], D["gbar"])   # lib/loss.py:125-135
        else:
            ops.gp_penalty(D["gimg"], w, self.loss[2:3], D["gp_norms"], D["gbar"])
        return D["gbar"]

    def d_tangent(self, P, GR, gbar, u, alpha):
        """Push gbar (= dR1/dx-gradient) forward through D with the B1 masks, adding the R1
        weight terms; returns (tangent logit, mbstd injection) for the B2 pass."""
        ops, D, d, s, B, R = self.ops, self.dd, self.depths, self.s, self.B, self.R
        self._side_join("D")
        fr = "fromRGB_blocks.{}.fromRGB.module."
        mk = dict(mask_bits=D["rgbb"]) if self._rgbbits() else dict(mask_y=D["yrgb"])
        ops.from_rgb(gbar, P[fr.format(s) + "weight"], None, he(3), D["trgb"], B=B, R=R, C=d[s],
                     down=False, slope=SLOPE, **mk)
        if not getattr(self, "_t_rgb_done", False):   # else B1's RGBD epilogue added it
            self._side_call(("D",), ops.from_rgb_bwd,
                            D["gzrgb"], P[fr.format(s) + "weight"], he(3), B=B, R=R, C=d[s],
                            down=False, img=gbar, dw=GR[fr.format(s) + "weight"])
        self._t_rgb_done = False
        low = self._low(alpha)
        if low:
            ops.from_rgb(gbar, P[fr.format(s - 1) + "weight"], None, he(3), D["td"], B=B, R=R // 2,
                         C=d[s - 1], down=True, slope=SLOPE, mask_y=D["yd"])
            self._side_call(("D",), ops.from_rgb_bwd,
                            D["gzd"], P[fr.format(s - 1) + "weight"], he(3), B=B, R=R // 2,
                            C=d[s - 1], down=True, img=gbar, dw=GR[fr.format(s - 1) + "weight"])
        t = D["trgb"]
        for i in reversed(range(s)):
            Ri = 8 * 2 ** i
            a, b = f"blocks.{i}.block.0.module.", f"blocks.{i}.block.2.module."
            self._conv("D", f"a{i}", t, D[f"ta{i}"], Ri, d[i + 1], d[i + 1], L.CONV_MASK,
                       aux=D[f"a{i}"], bias=False)
            self._wgrad("D", f"a{i}", t, D[f"gza{i}"], GR[a + "weight"], Ri, d[i + 1], d[i + 1])
            if self._dbits(i):
                # tangent through conv b, lrelu' (bits) and the avg pool in one launch; the
                # weight term pairs the tangent with B1's gradient at this level
                self._conv("D", f"b{i}", D[f"ta{i}"], D[f"tp{i}"], Ri, d[i + 1], d[i],
                           L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_POOL, aux=D[f"mb{i}"],
                           bias=False, out_scale=0.25)
                gb1 = D["gh"] if i == 0 else D[f"ghin{i - 1}"]
                self._wgrad("D", f"b{i}", D[f"ta{i}"], gb1, GR[b + "weight"], Ri, d[i + 1], d[i],
                            gzbits=D[f"mb{i}"], gscale=0.25 * (alpha if i == s - 1 else 1.0))
            elif self._ubits(i):
                # mask (bits) and pool in the conv; the weight term reads B1's materialised gzb
                self._conv("D", f"b{i}", D[f"ta{i}"], D[f"tp{i}"], Ri, d[i + 1], d[i],
                           L.CONV_MASK | L.CONV_AUX_BITS | L.CONV_POOL, aux=D[f"mb{i}"],
                           bias=False, out_scale=0.25)
                self._wgrad("D", f"b{i}", D[f"ta{i}"], D[f"gzb{i}"], GR[b + "weight"], Ri,
                            d[i + 1], d[i])
            else:
                self._conv("D", f"b{i}", D[f"ta{i}"], D[f"tbf{i}"], Ri, d[i + 1], d[i],
                           L.CONV_MASK, aux=D[f"bf{i}"], bias=False)
                self._wgrad("D", f"b{i}", D[f"ta{i}"], D[f"gzb{i}"], GR[b + "weight"], Ri,
                            d[i + 1], d[i])
                ops.avgpool2(D[f"tbf{i}"], D[f"tp{i}"], B=B, H=Ri, W=Ri, C=d[i])
            if i == s - 1 and low:
                ops.blend(1.0 - alpha, D["td"], alpha, D[f"tp{i}"], D["tblend"])
                t = D["tblend"]
            else:
                t = D[f"tp{i}"]
        ops.mbstd_r1(self.h_mb, t, D["gm"], D["tm"], D["inj"], B=B, HW=16, C=d[0])
        cv = "minibatch_normalization_block.conv.module."
        self._conv("D", "mb", D["tm"], D["tc"], 4, d[0] + 1, d[0], L.CONV_MASK, aux=D["c"],
                   bias=False)
        self._wgrad("D", "mb", D["tm"], D["gzc"], GR[cv + "weight"], 4, d[0] + 1, d[0])
        lin = "minibatch_normalization_block.linear.module."
        ops.linear(D["tc"], P[lin + "weight"], None, D["tl1"], B=B,
                   flags=L.LIN_IN_CHW | L.LIN_MASK, scale=he(16 * d[0]), slope=SLOPE, aux=D["l1"])
        self._side_call(("D",), ops.linear_wgrad,
                        D["tc"], D["gzl1"], GR[lin + "weight"], None, B=B, flags=L.LIN_IN_CHW,
                        scale=he(16 * d[0]))
        dec = "decision_layer.module."
        ops.linear(D["tl1"], P[dec + "weight"], None, D["tout"], B=B, flags=0, scale=he(d[0]))
        self._side_call(("D",), ops.linear_wgrad,
                        D["tl1"], u, GR[dec + "weight"], None, B=B, flags=0, scale=he(d[0]))
        return D["tout"], D["inj"]

    # ================================================================== step
    def d_step(self, PG, PD, GD, real, z, alpha_G, alpha_D, gp_eps=None, before_fake=None):
        """D half of train_step (pggan/model.py:211-238).  Returns the faded real image and
        the fake image.  Gradients are written to GD (zeroed here).  before_fake() runs
        between the real-image part (which does not read G) and the fake image."""
        ops, D, B, hp = self.ops, self.dd, self.B, self.hyper
        GD_flat = self._GD_flat
        self._zero(GD_flat)
        self._zero(self.loss[:3])
        self._zero(self.loss[4:5])
        if self._merged():
            return self._d_step_merged(PG, PD, GD, real, z, alpha_G, alpha_D, before_fake, gp_eps)
        if self._low(alpha_D):
            ops.img_fade(real, alpha_D, D["real_in"])                       # :217-221
            xr = D["real_in"]
        else:
            xr = real   # s = 0, or alpha = 1: (1 - 1) * up2(avgpool2(x)) + 1 * x == x exactly
        if hp.gp_mode == "r1":
            # ---- real: F, B1, R1, T, B2
            self.d_forward(PD, xr, alpha_D)
            ops.bce(D["logit"], True, 1.0, self.loss[0:1], D["u"], D["hl"])   # lib/loss.py:119-123
            gbar = self._input_grad(PD, D["u"], alpha_D, "r1", GR=GD)          # lib/loss.py:125-135
            tout, inj = self.d_tangent(PD, GD, gbar, D["u"], alpha_D)
            ops.mul_add(D["u"], tout.view(-1), D["hl"], D["u2"])
            self.d_backward(PD, GD, D["u2"], alpha_D, img=xr, inj_mbstd=inj)
        else:
            self.d_forward(PD, xr, alpha_D)
            ops.bce(D["logit"], True, 1.0, self.loss[0:1], D["u"], None)
            if hp.W_drift:
                ops.drift(D["logit"], hp.W_drift, self.loss[4:5], D["u"])   # pggan/loss.py:94-100
            self.d_backward(PD, GD, D["u"], alpha_D, img=xr)
        if before_fake is not None:
            before_fake()
        # ---- fake
        img_fake = self.g_forward(PG, z, alpha_G, keep=False)                   # :226-227
        if self.keep_fake_D:
            img_fake = img_fake.clone()
        self.d_forward(PD, img_fake, alpha_D)                                   # :228
        ops.bce(D["logit"], False, 1.0, self.loss[1:2], D["u"], None)
        self.d_backward(PD, GD, D["u"], alpha_D, img=img_fake, final=hp.gp_mode == "r1")
        if hp.gp_mode != "r1":
            self._wgan_gp(PD, GD, xr, img_fake, gp_eps, alpha_D)
        self._side_join()
        return xr, img_fake

    def _merged(self):
        """Whether this D half runs its real and fake passes merged (batch 2B buffers
        allocated).  With a generator update still waiting for its DP exchange the R1 mode
        keeps the second backward merged but runs the two forwards separately, the real
        image's first (see _d_step_merged_b2); the WGAN-GP mode then keeps the separate
        schedule."""
        if self.dd2 is None or self.hyper.gp_mode not in ("r1", "wgan-gp"):
            return False
        return self.hyper.gp_mode == "r1" or not hasattr(self._pending_G, "wait")

    @contextlib.contextmanager
    def _pair(self, b2=False):
        """Run the enclosed passes at batch 2B on the merged buffers (b2: the second
        backward's own gradient buffers)."""
        saved = (self.dd, self.B)
        self.dd, self.B = (self.dd2b if b2 else self.dd2), 2 * saved[1]
        try:
            yield
        finally:
            self.dd, self.B = saved

    def _d_step_merged(self, PG, PD, GD, real, z, alpha_G, alpha_D, before_fake, gp_eps=None):
        """The R1 D half with the fake image's passes merged into the real image's
        (pggan/model.py:211-238; the same terms, batch [real; fake] = 2B):
          G forward (the fake image straight into the second half of the merged input),
          F over both images, the two BCE terms (each over its own half, so each is the
          reference's mean over B), B1 + R1 + T on the real half at batch B, then ONE
          second backward over both halves -- upstream u2 = u + tout * hl for the real
          samples and the fake BCE gradient for the fake ones -- whose weight gradients are
          the sum of the two passes'.  Every per-sample quantity is the separate schedule's
          (convs and mbstd groups never mix samples of the two halves); only the order in
          which the weight gradients sum over samples differs.  Half the D forward and
          second-backward launches, at twice the work each: the 4^2-32^2 levels are latency
          bound and the wide levels amortise each launch's ramp and epilogue."""
        ops, hp = self.ops, self.hyper
        B = self.B
        D1, D2 = self.dd, self.dd2
        X = D2["xin"]
        if hasattr(self._pending_G, "wait") and hp.gp_mode == "r1":
            return self._d_step_merged_b2(PG, PD, GD, real, z, alpha_G, alpha_D, before_fake)
        if before_fake is not None:
            before_fake()
        img_fake = self._g_forward_d_half(PG, z, alpha_G)                       # :226-227
        trace, self.trace = self.trace, None
        try:
            if self._low(alpha_D):
                ops.img_fade(real, alpha_D, X[:B])                               # :217-221
            else:
                self._copy(X[:B], real)
            with self._pair():
                self.d_forward(PD, X, alpha_D)                                  # :216, :228
        finally:
            self.trace = trace
        h2 = self.h_mb
        self.h_mb = h2[:B]
        if trace is not None:   # one record per image, in the separate schedule's order
            trace("D", self)
            self.dd = self.dd_hi
            try:
                trace("D", self)
            finally:
                self.dd = D1
        if hp.gp_mode != "r1":
            # WGAN-GP mode: one backward over both halves from the two BCE terms (+ drift on
            # the real half), then the penalty pass on the interpolation at batch B
            ops.bce(D1["logit"], True, 1.0, self.loss[0:1], D1["u"], None)
            if hp.W_drift:
                ops.drift(D1["logit"], hp.W_drift, self.loss[4:5], D1["u"])   # pggan/loss.py:94-100
            ops.bce(D2["logit"][B:], False, 1.0, self.loss[1:2], D2["u"][B:], None)
            self.h_mb = h2
            try:
                with self._pair(b2=True):
                    self.d_backward(PD, GD, D2["u"], alpha_D, img=X)
            finally:
                self.h_mb = h2[:B]
            self._wgan_gp(PD, GD, X[:B], X[B:], gp_eps, alpha_D)
            self._side_join()
            return X[:B], (img_fake.clone() if self.keep_fake_D else img_fake)
        ops.bce(D1["logit"], True, 1.0, self.loss[0:1], D1["u"], D1["hl"])    # lib/loss.py:119-123
        ops.bce(D2["logit"][B:], False, 1.0, self.loss[1:2], D2["u2"][B:], None)
        gbar = self._input_grad(PD, D1["u"], alpha_D, "r1", GR=GD)              # lib/loss.py:125-135
        tout, inj = self.d_tangent(PD, GD, gbar, D1["u"], alpha_D)
        ops.mul_add(D1["u"], tout.view(-1), D1["hl"], D1["u2"])
        self.h_mb = h2
        try:
            with self._pair(b2=True):
                # D2["inj"]: the tangent wrote the real half; the fake half stays zero
                self.d_backward(PD, GD, D2["u2"], alpha_D, img=X, inj_mbstd=D2["inj"], final=True,
                                join=not self.sep_b2)
        finally:
            self.h_mb = h2[:B]
        self._side_join()
        return X[:B], (img_fake.clone() if self.keep_fake_D else img_fake)

    def _g_forward_d_half(self, PG, z, alpha_G):
        """The D half's generator forward (the fake image).  With a merged generator forward
        pending (self._z_g, see train_step) both generator forwards of the step run as one
        (G is not updated in between): latents [z; z_g], images [fake for D; fake for G] into
        the merged input's X[B:3B], activations kept for the G half (its g_step then skips
        its own forward)."""
        z_g = self._z_g
        self._z_g = None
        if z_g is None:
            return self.g_forward(PG, z, alpha_G, keep=False)                 # :226-227
        B, g2 = self.B, self.g2
        self._copy(g2["z"][:B], z)
        self._copy(g2["z"][B:], z_g)
        trace, self.trace = self.trace, None
        saved = self.g, self.B
        self.g, self.B = g2, 2 * B
        try:
            self.g_forward(PG, g2["z"], alpha_G, keep=True)                     # :226-227, :244-245
        finally:
            self.g, self.B = saved
            self.trace = trace
        self._g_done = True
        if trace is not None:
            trace("G", self)            # the D half's generator forward, then the G half's
            self.g = self.g_hi
            try:
                trace("G", self)
            finally:
                self.g = self.g_lo
        return self.g["img"]

    def _d_step_merged_b2(self, PG, PD, GD, real, z, alpha_G, alpha_D, before_fake):
        """The merged R1 D half while the previous step's G gradient is still in its DP
        exchange (lib/model.py:74-79 is the reference's collective site): the real image's
        forward, B1, R1 and tangent at batch B first -- none of them reads G, so the exchange
        completes behind them -- then before_fake (the exchange's wait, Adam_G, the G packing),
        the generator forward, the fake image's forward at batch B into the second half of
        the merged buffers, and ONE second backward over [real; fake] at 2B as in
        _d_step_merged.  Every per-sample quantity is the separate schedule's."""
        ops = self.ops
        B = self.B
        D1, D2 = self.dd, self.dd2
        X = D2["xin"]
        if self._low(alpha_D):
            ops.img_fade(real, alpha_D, X[:B])                                   # :217-221
        else:
            self._copy(X[:B], real)
        self.d_forward(PD, X[:B], alpha_D)                                       # :216
        ops.bce(D1["logit"], True, 1.0, self.loss[0:1], D1["u"], D1["hl"])    # lib/loss.py:119-123
        gbar = self._input_grad(PD, D1["u"], alpha_D, "r1", GR=GD)              # lib/loss.py:125-135
        tout, inj = self.d_tangent(PD, GD, gbar, D1["u"], alpha_D)
        ops.mul_add(D1["u"], tout.view(-1), D1["hl"], D1["u2"])
        if before_fake is not None:
            before_fake()
        img_fake = self._g_forward_d_half(PG, z, alpha_G)                       # :226-227
        self.dd = self.dd_hi
        try:
            # writes second-half activations only: the tangent's weight terms still running
            # on the side stream read first-half buffers, so no join
            self.d_forward(PD, X[B:], alpha_D, join=not self.sep_b2)             # :228
        finally:
            self.dd = D1
        ops.bce(D2["logit"][B:], False, 1.0, self.loss[1:2], D2["u2"][B:], None)
        self.h_mb = D2[self.h_mb_key]
        try:
            with self._pair(b2=True):
                # D2["inj"]: the tangent wrote the real half; the fake half stays zero
                self.d_backward(PD, GD, D2["u2"], alpha_D, img=X, inj_mbstd=D2["inj"], final=True,
                                join=not self.sep_b2)
        finally:
            self.h_mb = D1[self.h_mb_key]
        self._side_join()
        return X[:B], (img_fake.clone() if self.keep_fake_D else img_fake)

    def _wgan_gp(self, PD, GD, xr, xf, eps, alpha):
        """Optional WGAN-GP mode (pggan/loss.py:54-92): interp -> D -> per-sample grad norm.
        Fused form: the interpolation eps x_r + (1 - eps) x_f is read by the fromRGB layers
        from x_r, x_f and eps (never written), the per-sample squared norm is summed by the
        pass writing dD/dx, and the tangent pass reads dD/dx with the per-sample weight
        2 W_gp (|g| - 1) / |g| applied on load."""
        ops, D, B = self.ops, self.dd, self.B
        D["gp_eps"].copy_(eps)
        if self._fused_penalty():
            torch.sub(D["ones"].view(-1, 1), D["gp_eps"], out=D["gp_c"])
            interp = L.ImgMix(xr, xf, D["gp_eps"], D["gp_c"])
        else:
            ops.gp_interp(xr, xf, D["gp_eps"], D["interp"])
            interp = D["interp"]
        self.d_forward(PD, interp, alpha)
        gbar = self._input_grad(PD, D["ones"], alpha, "wgan-gp", self.hyper.W_gp)  # d(sum D)/dx
        tout, inj = self.d_tangent(PD, GD, gbar, D["ones"], alpha)
        # upstream of the second backward: no BCE here, so no logit injection
        self.d_backward(PD, GD, D["zeros"], alpha, img=interp, inj_mbstd=inj, final=True)

    def g_step(self, PG, PD, GG, z, alpha_G, alpha_D, before_d=None):
        """G half of train_step (pggan/model.py:244-253).  before_d() runs after the
        generator forward (which does not read D) and before D is evaluated."""
        ops, D, hp = self.ops, self.dd, self.hyper
        self._zero(self._GG_flat)
        self._zero(self.loss[3:4])
        if self._g_done:
            # the D half ran this half's generator forward (merged): its activations and
            # image are the second half of the 2B generator buffers
            self._g_done = False
            self.g = self.g_hi
            try:
                return self._g_step_rest(PG, PD, GG, self.g["img"], alpha_G, alpha_D, before_d)
            finally:
                self.g = self.g_lo
        img = self.g_forward(PG, z, alpha_G)
        return self._g_step_rest(PG, PD, GG, img, alpha_G, alpha_D, before_d)

    def _g_step_rest(self, PG, PD, GG, img, alpha_G, alpha_D, before_d):
        ops, D, hp = self.ops, self.dd, self.hyper
        if before_d is not None:
            before_d()
        self.d_forward(PD, img, alpha_D)
        ops.bce(D["logit"], True, hp.W_adv, self.loss[3:4], D["u"], None)   # pggan/loss.py:5-14
        if self._fused_penalty():
            self.d_backward(PD, None, D["u"], alpha_D, gimg=D["gimg"], gimg_overwrite=True)
        else:
            D["gimg"].zero_()
            self.d_backward(PD, None, D["u"], alpha_D, gimg=D["gimg"])
        self.g_backward(PG, GG, D["gimg"], alpha_G)
        self._side_join()
        return img

    def bind(self, fpG: FlatParams, fpD: FlatParams, hyper: Hyper):
        """Attach parameter / optimizer buffers.  Re-binding the same objects is a no-op (the
        packed weights stay valid); binding new ones first completes a deferred G update."""
        if getattr(self, "fpG", None) is fpG and self.fpD is fpD and self.hyper is hyper:
            return
        if getattr(self, "_pending_G", None) is not None:
            self._finish_G()
        self.fpG, self.fpD, self.hyper = fpG, fpD, hyper
        self._GD_flat, self._GG_flat = fpD.grad, fpG.grad
        self._pending_G = None     # deferred Adam_G (overlapped DP mode)
        self._packed = {"G": False, "D": False}   # packed weights match the parameters

    def adam(self, fp: FlatParams, lr):
        hp = self.hyper
        if fp is self.fpG:
            self._side_join("G")   # only G's pending side work (D's may still be running)
        else:
            self._side_join()
        n = fp.n_live
        if hasattr(self.ops, "adam_dev"):
            if fp._step_dev_host != fp.step:   # a reset / checkpoint load changed the count
                fp.step_dev.fill_(fp.step)
            fp.step += 1
            fp._step_dev_host = fp.step
            self.ops.adam_dev(fp.flat[:n], fp.grad[:n], fp.m[:n], fp.v[:n], lr=lr, beta1=hp.beta1,
                              beta2=hp.beta2, eps=hp.eps, step_dev=fp.step_dev)
            return
        fp.step += 1
        self.ops.adam(fp.flat[:n], fp.grad[:n], fp.m[:n], fp.v[:n], lr=lr, beta1=hp.beta1,
                      beta2=hp.beta2, eps=hp.eps, step=fp.step)

    def train_step(self, real, z1, z2, alpha_G, alpha_D, grad_hook=None, gp_eps=None):
        """One full step: D half (R1) + Adam_D, G half + Adam_G (pggan/model.py:206-255).

        grad_hook(net, flat_live_grad) runs before each Adam (DP all-reduce).  If it returns
        an object with .wait() (an async collective, e.g. torch.distributed work), the
        engine overlaps the exchange with work that does not depend on it:
          D gradients  -> the G half's generator forward (G is not changed by Adam_D);
          G gradients  -> the next step's real-image part of the D half (which never
                          reads G); Adam_G and the G weight packing then run just before
                          that step's fake image.  flush() completes a pending G update.
        The arithmetic and its order per parameter are the reference's either way."""
        fpG, fpD, hp = self.fpG, self.fpD, self.hyper
        PG, PD = fpG.views, fpD.views
        ov = self.overlap_g_exchange
        if ov < 0:
            # a bound GradExchange.hook carries the exchange's world size
            ov = int(getattr(getattr(grad_hook, "__self__", None), "world", 2) > 1)
        if not ov:
            self._finish_G()   # the previous step's G exchange completes first (no B2 reorder)
        if self._pending_G is None and not self._packed["G"]:
            self.pack("G", PG)
        if not self._packed["D"]:
            self.pack("D", PD)
        # z2 for a merged generator forward (_d_step_merged).  Also under a bucketed DP
        # exchange: the D gradients go out layer by layer during the last backward (the
        # 512-channel bulk first), so at its end only the last bucket is in flight, and the
        # separate G-half generator forward that would hide it costs more than it hides
        # (one rank, interleaved: profiles/r5_dp_ab.txt)
        self._z_g = z2 if self.g2 is not None else None
        img_real, img_fake_D = self.d_step(PG, PD, fpD.gviews, real, z1, alpha_G, alpha_D,
                                           gp_eps=gp_eps, before_fake=self._finish_G)
        if self._z_g is not None:   # d_step did not merge: the G half runs its own forward
            self._z_g = None
        hD = grad_hook("D", fpD.live_grad()) if grad_hook is not None else None

        def finish_D():
            if hD is not None and hasattr(hD, "wait"):
                hD.wait()
            self.adam(fpD, hp.lr_D)
            self.pack("D", PD)

        if hD is not None and hasattr(hD, "wait"):
            img_fake = self.g_step(PG, PD, fpG.gviews, z2, alpha_G, alpha_D, before_d=finish_D)
        else:
            finish_D()
            img_fake = self.g_step(PG, PD, fpG.gviews, z2, alpha_G, alpha_D)
        hG = grad_hook("G", fpG.live_grad()) if grad_hook is not None else None
        self._pending_G = hG if hG is not None else True
        if not (hG is not None and hasattr(hG, "wait")):
            self._finish_G()
        return img_real, img_fake_D, img_fake

    def _finish_G(self):
        """Adam_G (after the pending G all-reduce, if any) and the G weight packing."""
        h = self._pending_G
        if h is None:
            return
        self._pending_G = None
        if hasattr(h, "wait"):
            h.wait()
        self.adam(self.fpG, self.hyper.lr_G)
        self.pack("G", self.fpG.views)

    def flush(self):
        """Complete a deferred G update (overlapped DP mode); no-op otherwise."""
        self._finish_G()

    def host_state(self):
        """The Python-side schedule state a step leaves behind (ProgressiveGAN's C++ replay
        runs no Python, so it restores this after re-issuing a recorded step)."""
        return (self._pending_G, self._g_done, self._z_g, dict(self._packed))

    def set_host_state(self, st):
        self._pending_G, self._g_done, self._z_g, packed = st
        self._packed = dict(packed)

    def params_changed(self):
        """Parameters were modified outside the engine (checkpoint load, broadcast):
        repack both nets at the next step."""
        self.flush()
        self._packed = {"G": False, "D": False}
