"""Low-resolution conv launches, split-K in-launch combine (conv_sk) vs the round-5 paths
(conv_lr / conv3x3 split-K + conv_splitk_epilogue), for a rocprofv3 kernel trace (GPU box):

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/sk_probe.py
    python tools/kprof_table.py OUT/run_kernel_trace.csv     (per kernel name and grid)

The shapes are the step's 4^2-16^2 convs at B = 4 and at the merged passes' B = 8."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pggan_amd import _lib  # noqa: E402

SPECS = [(4, 512, 512, 6), (4, 544, 512, 6), (4, 512, 512, 0), (8, 512, 512, 22), (8, 512, 512, 8),
         (8, 512, 512, 0), (16, 512, 512, 22), (16, 512, 512, 8), (16, 512, 512, 0)]


def main():
    ops = _lib.HipOps(torch.bfloat16)
    dev, bf = "cuda", torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    for nosk in (False, True):
        if nosk:
            ops._scr = lambda: None     # no scratch: the round-5 launch paths
        for B in (4, 8):
            for H, cin, cout, fl in SPECS:
                x = torch.randn(B, H, H, cin, device=dev, generator=g).to(bf)
                wpk = torch.randn(ops.packed_elems(0, cout, cin), device=dev, generator=g).to(bf) * 0.05
                Ho = H // 2 if fl & 16 else H
                y = torch.empty(B, Ho, Ho, cout, device=dev, dtype=bf)
                aux = torch.randn(B, H, H, cout, device=dev, generator=g).to(bf) if fl & 8 else None
                y2 = torch.empty(B, H, H, cout, device=dev, dtype=bf) if fl & 16 else None
                bias = torch.zeros(cout, device=dev) if fl & 2 else None
                nb = ops.conv_workspace_bytes(B=B, H=H, W=H, cin=cin, cout=cout)
                ws = torch.empty(max(nb // 4, 1), device=dev) if nb else None
                for _ in range(10):
                    ops.conv3x3(x, wpk, y, B=B, H=H, W=H, cin=cin, cout=cout, flags=fl, bias=bias,
                                aux=aux, ws=ws, out_scale=0.25 if fl & 16 else 1.0, y2=y2)
                torch.cuda.synchronize()
                print(f"{'old' if nosk else 'sk '} B={B} H={H} {cin}->{cout} flags {fl}", flush=True)


if __name__ == "__main__":
    main()
