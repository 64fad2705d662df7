"""Generator / Discriminator modules with the reference's Python surface
(pggan/nets.py:10-276): constructor arguments, `add_block(depth)`, float
attribute `alpha`, `forward(z)` / `forward(x, get_feature=False)`, and the exact
`state_dict` keys of the reference (``blocks.{i}.block.{0,3}.module.weight`` ...),
so reference checkpoints load unchanged.

Compute goes through the HIP kernels (pggan_amd.engine).  forward() is differentiable
once (first-order backward on the HIP kernels, torch.autograd.Function) when grad is
enabled, and a forward-only sampling path otherwise; the training step, with its R1
double backward, is the hand-scheduled ProgressiveGAN.train_step.  Non-default architecture switches that the
reference exposes but never uses (equalized_lr=False, apply_pixel_norm=False,
last_activation, LReLU_slope on blocks) raise NotImplementedError.
"""
from __future__ import annotations

import torch
from torch import nn

from . import engine as E


class _Param(nn.Module):
    """Stands in for ConstrainedLayer.module (lib/layers.py:48): holds weight/bias.

    Init as the reference: W ~ N(0,1) (lib/layers.py:54); b = 0 when init_bias_to_zero
    (:51-52), else the wrapped nn.Conv2d / nn.Linear default it keeps,
    U(-1/sqrt(fan_in), 1/sqrt(fan_in)) with fan_in = prod(weight.shape[1:])."""

    def __init__(self, wshape, bshape, init_bias_to_zero=True):
        super().__init__()
        self.weight = nn.Parameter(torch.randn(*wshape))            # lib/layers.py:54
        if init_bias_to_zero:
            b = torch.zeros(*bshape)                                 # lib/layers.py:51-52
        else:
            fan_in = 1
            for d in wshape[1:]:
                fan_in *= int(d)
            bound = 1.0 / fan_in ** 0.5
            b = torch.empty(*bshape).uniform_(-bound, bound)
        self.bias = nn.Parameter(b)


class _Eq(nn.Module):
    def __init__(self, wshape, bshape, init_bias_to_zero=True):
        super().__init__()
        self.module = _Param(wshape, bshape, init_bias_to_zero)


class _Seq(nn.Module):
    """A parameter container whose children are indexed like nn.Sequential."""

    def __init__(self, entries):
        super().__init__()
        for i, m in entries:
            self.add_module(str(i), m)


class _GBlock(nn.Module):
    def __init__(self, prev, new, is_first, ibz):
        super().__init__()
        if is_first:
            self.block = _Seq([(0, _Eq((new, new, 3, 3), (new,), ibz))])
        else:
            self.block = _Seq([(0, _Eq((new, prev, 3, 3), (new,), ibz)),
                               (3, _Eq((new, new, 3, 3), (new,), ibz))])


class _DBlock(nn.Module):
    def __init__(self, new, prev, ibz):
        super().__init__()
        self.block = _Seq([(0, _Eq((new, new, 3, 3), (new,), ibz)),
                           (2, _Eq((prev, new, 3, 3), (prev,), ibz))])


class _ToRGB(nn.Module):
    def __init__(self, depth, out_dim, ibz):
        super().__init__()
        self.toRGB = _Eq((out_dim, depth, 1, 1), (out_dim,), ibz)


class _FromRGB(nn.Module):
    def __init__(self, in_dim, depth, ibz):
        super().__init__()
        self.fromRGB = _Eq((depth, in_dim, 1, 1), (depth,), ibz)


class _MBBlock(nn.Module):
    def __init__(self, depth, ibz):
        super().__init__()
        self.conv = _Eq((depth, depth + 1, 3, 3), (depth,), ibz)
        self.linear = _Eq((depth, depth * 16), (depth,), ibz)


_ENGINES = {}
OPS_FACTORY = None   # tests may substitute a CPU double; default: the HIP library


def _engine(net, ops_dtype, depths, s, B, device):
    """The engine of one net: "G" / "D" hold the forward activations only (sampling),
    "Gtrain" / "Dtrain" also that net's backward buffers (the autograd path); at most one
    cached per kind (a new shape, dtype or stage replaces it), so sampling at 1024^2 does
    not keep a training-sized buffer set alive."""
    from . import _lib
    key = (ops_dtype, tuple(depths), s, B, str(device))
    cur = _ENGINES.get(net)
    if cur is None or cur[0] != key:
        _ENGINES.pop(net, None)
        factory = OPS_FACTORY or _lib.HipOps
        eng = E.StepEngine(factory(ops_dtype), depths, s, B, device, forward_only=net)
        eng.hyper = E.Hyper()
        eng.fwd_version = 0
        _ENGINES[net] = (key, eng)
    return _ENGINES[net][1]


def _wants_grad(x, module):
    return torch.is_grad_enabled() and (x.requires_grad or
                                        any(p.requires_grad for p in module.parameters()))


def _no_double_backward():
    if torch.is_grad_enabled():
        raise NotImplementedError(
            "pggan_amd modules are differentiable once (first-order backward on the HIP "
            "kernels); the R1 double backward runs hand-scheduled in ProgressiveGAN.train_step")


def _check_version(ctx):
    if ctx.eng.fwd_version != ctx.version:
        raise RuntimeError("pggan_amd: a later forward of this module overwrote the activations "
                           "this backward needs; call backward before the next forward")


class _GFn(torch.autograd.Function):
    """Generator forward / first-order backward on the HIP kernels (pggan/nets.py:121-161;
    the gradient w.r.t. every parameter; the latent receives none, as in the reference
    where z never requires grad)."""

    @staticmethod
    def forward(ctx, module, z, *params):
        names = [n for n, _ in module.named_parameters()]
        P = dict(zip(names, params))
        eng = _engine("Gtrain", module.compute_dtype, module.block_depths, module.scale_index,
                      z.shape[0], z.device)
        eng.hyper.slope_cfg = module.LReLU_slope
        eng.fwd_version += 1
        ctx.eng, ctx.version, ctx.names, ctx.alpha = eng, eng.fwd_version, names, float(module.alpha)
        ctx.P = P
        eng.pack("G", P)
        return eng.g_forward(P, z.reshape(z.shape[0], -1).float(), ctx.alpha).clone()

    @staticmethod
    def backward(ctx, gimg):
        _no_double_backward()
        _check_version(ctx)
        GR = {n: torch.zeros_like(p) for n, p in ctx.P.items()}
        ctx.eng.g_backward(ctx.P, GR, gimg.float().contiguous(), ctx.alpha)
        dead = E.dead_params("G", ctx.eng.s)     # unused at this stage: grad None, as in torch
        return (None, None) + tuple(None if n in dead else GR[n] for n in ctx.names)


class _DFn(torch.autograd.Function):
    """Discriminator forward / first-order backward (pggan/nets.py:248-276): gradients
    w.r.t. every parameter and the input image, from the logit's gradient."""

    @staticmethod
    def forward(ctx, module, x, *params):
        names = [n for n, _ in module.named_parameters()]
        P = dict(zip(names, params))
        eng = _engine("Dtrain", module.compute_dtype, module.depths, module.scale_index,
                      x.shape[0], x.device)
        eng.fwd_version += 1
        ctx.eng, ctx.version, ctx.names, ctx.alpha = eng, eng.fwd_version, names, float(module.alpha)
        ctx.P = P
        ctx.set_materialize_grads(False)
        eng.pack("D", P)
        ctx.x = x.float().contiguous()
        out = eng.d_forward(P, ctx.x, ctx.alpha).clone()
        return out, eng.dd["l1"].float().clone()

    @staticmethod
    def backward(ctx, gout, gfeat):
        _no_double_backward()
        _check_version(ctx)
        if gfeat is not None and bool(gfeat.ne(0).any()):
            raise NotImplementedError("pggan_amd: gradient through the D feature output")
        GR = {n: torch.zeros_like(p) for n, p in ctx.P.items()}
        eng = ctx.eng
        gx = torch.zeros_like(ctx.x)
        u = torch.zeros(ctx.x.shape[0], dtype=torch.float32, device=ctx.x.device)
        if gout is not None:
            u.copy_(gout.reshape(-1))
        eng.d_backward(ctx.P, GR, u, ctx.alpha, img=ctx.x, gimg=gx)
        dead = E.dead_params("D", eng.s)
        return (None, gx) + tuple(None if n in dead else GR[n] for n in ctx.names)


class Generator(nn.Module):
    """pggan/nets.py:10-161."""

    def __init__(self, latent_dim, first_depth, init_bias_to_zero=True, LReLU_slope=0.2,
                 apply_pixel_norm=True, last_activation=None, output_dim=3, equalized_lr=True):
        super().__init__()
        if not equalized_lr or not apply_pixel_norm or last_activation is not None:
            raise NotImplementedError("pggan_amd implements the reference's default G "
                                      "(equalized_lr, pixel norm, no last activation)")
        if output_dim != 3:
            raise NotImplementedError("pggan_amd kernels produce RGB output")
        self.latent_dim = latent_dim
        self.first_depth = first_depth
        self.init_bias_to_zero = init_bias_to_zero
        self.LReLU_slope = LReLU_slope
        self.output_dim = output_dim
        self.block_depths = [first_depth]
        self.blocks = nn.ModuleList()
        self.toRGB_blocks = nn.ModuleList()
        self.latent_format_layer = _Eq((16 * first_depth, latent_dim), (16 * first_depth,),
                                       init_bias_to_zero)
        self.first_block = _GBlock(first_depth, first_depth, True, init_bias_to_zero)
        self.toRGB_blocks.append(_ToRGB(first_depth, output_dim, init_bias_to_zero))
        self.alpha = 0
        self.compute_dtype = torch.float32

    def add_block(self, new_depth):
        """pggan/nets.py:102-119."""
        _ENGINES.pop("G", None)
        _ENGINES.pop("Gtrain", None)
        prev = self.block_depths[-1]
        self.block_depths.append(new_depth)
        dev = self.latent_format_layer.module.weight.device
        self.blocks.append(_GBlock(prev, new_depth, False, self.init_bias_to_zero).to(dev))
        self.toRGB_blocks.append(_ToRGB(new_depth, self.output_dim, self.init_bias_to_zero).to(dev))

    @property
    def scale_index(self):
        return len(self.blocks)

    def forward(self, x):
        """pggan/nets.py:121-161 on the HIP kernels.  Differentiable once when grad is
        enabled and a parameter requires it (_GFn); a forward-only engine otherwise."""
        if _wants_grad(x, self):
            return _GFn.apply(self, x, *self.parameters())
        s = self.scale_index
        B = x.shape[0]
        eng = _engine("G", self.compute_dtype, self.block_depths, s, B, x.device)
        eng.hyper.slope_cfg = self.LReLU_slope
        P = dict(self.named_parameters())
        with torch.no_grad():
            eng.pack("G", P)
            img = eng.g_forward(P, x.reshape(B, -1).float(), float(self.alpha))
        return img.clone()


class Discriminator(nn.Module):
    """pggan/nets.py:164-276."""

    def __init__(self, last_depth, init_bias_to_zero=True, LReLU_slope=0.2, decision_layer_size=1,
                 apply_minibatch_norm=False, input_dim=3, equalized_lr=True):
        super().__init__()
        if not equalized_lr or not apply_minibatch_norm or decision_layer_size != 1:
            raise NotImplementedError("pggan_amd implements the reference's configured D "
                                      "(equalized_lr, minibatch stddev, one logit)")
        if input_dim != 3:
            raise NotImplementedError("pggan_amd kernels consume RGB input")
        self.init_bias_to_zero = init_bias_to_zero
        self.input_dim = input_dim
        self.depths = [last_depth]
        self.blocks = nn.ModuleList()
        self.fromRGB_blocks = nn.ModuleList()
        self.mergeLayers = nn.ModuleList()
        self.decision_layer = _Eq((decision_layer_size, last_depth), (decision_layer_size,),
                                  init_bias_to_zero)
        self.minibatch_normalization_block = _MBBlock(last_depth, init_bias_to_zero)
        self.fromRGB_blocks.append(_FromRGB(input_dim, last_depth, init_bias_to_zero))
        self.alpha = 0
        self.compute_dtype = torch.float32

    def add_block(self, new_depth):
        """pggan/nets.py:227-239."""
        _ENGINES.pop("D", None)
        _ENGINES.pop("Dtrain", None)
        prev = self.depths[-1]
        self.depths.append(new_depth)
        dev = self.decision_layer.module.weight.device
        self.blocks.append(_DBlock(new_depth, prev, self.init_bias_to_zero).to(dev))
        self.fromRGB_blocks.append(_FromRGB(self.input_dim, new_depth, self.init_bias_to_zero).to(dev))

    @property
    def scale_index(self):
        return len(self.blocks)

    def forward(self, x, get_feature=False):
        """pggan/nets.py:248-276 on the HIP kernels.  Differentiable once when grad is
        enabled and the input or a parameter requires it (_DFn); forward-only otherwise."""
        if _wants_grad(x, self):
            out, feat = _DFn.apply(self, x, *self.parameters())
            return (out, feat) if get_feature else out
        s = self.scale_index
        B = x.shape[0]
        eng = _engine("D", self.compute_dtype, self.depths, s, B, x.device)
        P = dict(self.named_parameters())
        with torch.no_grad():
            eng.pack("D", P)
            out = eng.d_forward(P, x.float().contiguous(), float(self.alpha)).clone()
        if not get_feature:
            return out
        return out, eng.dd["l1"].float().clone()
