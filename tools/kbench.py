"""Micro-benchmark of single conv / wgrad launches at bench shapes (GPU only).

    python tools/kbench.py [--B 4] [--iters 20] SPEC [SPEC ...]
    SPEC = c:H:cin:cout:flags   conv3x3 (flags as in include/pggan_hip.h; H = output size
                                 before pooling)
           w:H:cin:cout:ups     conv3x3 weight gradient (with fused bias grad)
Prints one line per spec: avg us per launch, TFLOP/s and the GB/s of the minimal bytes.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pggan_amd import _lib  # noqa: E402
from pggan_amd.engine import cinp  # noqa: E402


def r8(c):
    return (c + 7) // 8 * 8


def run(ops, spec, B, iters):
    kind, H, cin, cout, fl = spec.split(":")
    H, cin, cout, fl = int(H), int(cin), int(cout), int(fl)
    dev, bf = "cuda", torch.bfloat16
    cp = cinp(cin)
    g = torch.Generator(device=dev).manual_seed(0)
    if kind == "c":
        Hin = H // 2 if fl & 1 else H
        x = torch.randn(B, Hin, Hin, cp, device=dev, generator=g).to(bf)
        wpk = torch.randn(ops.packed_elems(0, cout, cin), device=dev, generator=g).to(bf) * 0.05
        Ho = H // 2 if fl & 16 else H
        y = torch.empty(B, Ho, Ho, cinp(cout), device=dev, dtype=bf)
        aux = torch.randn(B, H, H, r8(cout), device=dev, generator=g).to(bf) if fl & (8 | 2048) else None
        u8 = lambda C: torch.randint(0, 256, (B, H, H, (C + 7) // 8), device=dev, generator=g,
                                     dtype=torch.uint8)
        if fl & 256:                       # AUX_BITS: the mask operand is sign bits
            aux = u8(cout)
        xbits = u8(cp) if fl & 512 else None
        y2 = None
        if fl & 128:                       # Y2_BITS (with POOL): pre-pool sign bits
            y2 = u8(cout)
        elif fl & (64 | 2048):             # PIXNORM (keep) / PNBWD: the per-pixel factor
            y2 = torch.rand(B, H, H, 1, device=dev, generator=g) + 0.5
        bias = torch.zeros(cout, device=dev) if fl & 2 else None
        nb = ops.conv_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout)
        ws = torch.empty(max(nb // 4, 1), device=dev) if nb else None

        def f():
            ops.conv3x3(x, wpk, y, B=B, H=H, W=H, cin=cin, cout=cout, flags=fl, bias=bias,
                        aux=aux, ws=ws, out_scale=0.25 if fl & 16 else 1.0, y2=y2, xbits=xbits)
        byts = sum(t.numel() * t.element_size() for t in (x, y, aux, y2, xbits) if t is not None)
    else:
        # w flags: 1 = UPS_IN (x at half resolution), 2 = GZ_BITS (g at half resolution,
        # masked by lrelu' sign bits at full resolution: the D conv-b weight gradient)
        ups, gzb = bool(fl & 1), bool(fl & 2)
        Hin = H // 2 if ups else H
        x = torch.randn(B, Hin, Hin, cp, device=dev, generator=g).to(bf)
        Hg = H // 2 if gzb else H
        gz = torch.randn(B, Hg, Hg, r8(cout), device=dev, generator=g).to(bf)
        bits = (torch.randint(0, 256, (B, H, H, r8(cout) // 8), device=dev, generator=g,
                              dtype=torch.uint8) if gzb else None)
        dw = torch.zeros(cout, cin, 3, 3, device=dev)
        db = torch.zeros(cout, device=dev)

        # the split-partial workspace the engine passes (WG_SLABS); without one the plan
        # falls back to one split
        nbw = ops.wgrad_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout, ups=ups)
        wsw = torch.empty(max(nbw // 4, 1), device=dev) if nbw else None

        def f():
            ops.conv_wgrad(x, gz, dw, B=B, H=H, W=H, cin=cin, cout=cout, ups=ups, scale=1.0,
                           db=db, ws=wsw, gzbits=bits)
        byts = x.numel() * 2 + gz.numel() * 2 + (bits.numel() if gzb else 0)
    for _ in range(3):
        f()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(iters):
        f()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / iters
    flops = 2.0 * B * H * H * 9 * cin * cout
    print(f"{spec:24s} {us:9.1f} us  {flops / us / 1e6:8.1f} TF/s  {byts / us / 1e3:8.1f} GB/s",
          flush=True)
    return us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib", default=None, help="library to load instead of the in-tree build")
    ap.add_argument("--rounds", type=int, default=1, help="repeat the spec list (A/B interleaving)")
    ap.add_argument("specs", nargs="+")
    a = ap.parse_args()
    if a.lib:
        _lib.load_library(a.lib)
    ops = _lib.HipOps(torch.bfloat16)
    for s in a.specs * a.rounds:
        try:
            run(ops, s, a.B, a.iters)
        except RuntimeError as e:   # e.g. a tuning override with no kernel for the plan
            print(f"{s:24s} skipped: {str(e).splitlines()[0][:80]}", flush=True)


if __name__ == "__main__":
    main()
