"""Launch loop over the step's elementwise (glue) passes at bench shapes, for kernel-trace A/B
of library builds (GPU only; time them with rocprofv3 --kernel-trace, see tools/kprof_ab.sh).

    python tools/glue_bench.py [--lib ab/lib_X.so] [--iters 10] [SPEC ...]
    SPEC = u:B:H:C     unpool_mask with sign bits (g at H/2 x C, output H x C)
           uy:B:H:C    unpool_mask with the bf16 activation as the lrelu' operand
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pggan_amd import _lib  # noqa: E402

DEFAULT = ["u:4:256:128", "u:8:256:128", "u:4:128:256", "u:8:128:256", "u:4:64:512",
           "u:8:32:512", "uy:4:256:128", "uy:8:128:256"]


def run(ops, spec, iters):
    kind, B, H, C = spec.split(":")
    B, H, C = int(B), int(H), int(C)
    dev, bf = "cuda", torch.bfloat16
    torch.manual_seed(B * 100003 + H * 101 + C)
    g = torch.randn(B, H // 2, H // 2, C, device=dev).to(bf)
    out = torch.empty(B, H, H, C, device=dev, dtype=bf)
    bits = torch.randint(0, 256, (B, H, H, C // 8), device=dev, dtype=torch.uint8)
    y = torch.randn(B, H, H, C, device=dev).to(bf)
    for _ in range(iters):
        if kind == "u":
            ops.unpool_mask(g, None, out, B=B, H=H, W=H, C=C, scale=0.25, slope=0.2, ups=True,
                            bits=bits)
        else:
            ops.unpool_mask(g, y, out, B=B, H=H, W=H, C=C, scale=0.25, slope=0.2, ups=True)
    torch.cuda.synchronize()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--check", default=None, help="second library: outputs must be bitwise equal")
    ap.add_argument("specs", nargs="*")
    a = ap.parse_args()
    if a.lib:
        _lib.load_library(a.lib)
    ops = _lib.HipOps(torch.bfloat16)
    outs = [run(ops, s, a.iters) for s in (a.specs or DEFAULT)]
    print("glue_bench done", flush=True)
    if a.check:
        # reference outputs from the other build in a child process (one library per process)
        import subprocess
        import tempfile
        with tempfile.TemporaryDirectory() as d:
            ref = os.path.join(d, "ref.pt")
            subprocess.run([sys.executable, __file__, "--lib", a.check, "--iters", "1", "--dump", ref]
                           + (a.specs or DEFAULT), check=True)
            r = torch.load(ref, weights_only=True)
        for s, o, ro in zip(a.specs or DEFAULT, outs, r):
            assert torch.equal(o.cpu(), ro), s
        print("bitwise equal to", a.check, flush=True)


if __name__ == "__main__":
    if "--dump" in sys.argv:
        i = sys.argv.index("--dump")
        path = sys.argv[i + 1]
        del sys.argv[i:i + 2]
        ap = argparse.ArgumentParser()
        ap.add_argument("--lib", default=None)
        ap.add_argument("--iters", type=int, default=1)
        ap.add_argument("specs", nargs="*")
        a = ap.parse_args()
        if a.lib:
            _lib.load_library(a.lib)
        ops = _lib.HipOps(torch.bfloat16)
        torch.save([run(ops, s, 1).cpu() for s in (a.specs or DEFAULT)], path)
    else:
        main()
