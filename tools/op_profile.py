"""Per-op timing of one C5 training step: every HipOps entry point is wrapped with HIP events
(on the launching stream) and keyed by (op, resolution, channels, flags); prints a table sorted
by time per step.  Usage (GPU box): python tools/op_profile.py [--stage 8 --batch 4 --steps 3]"""
import argparse
import collections
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from pggan_amd import _lib  # noqa: E402
from pggan_amd import engine as E  # noqa: E402

PAPER = [512, 512, 512, 512, 256, 128, 64, 32, 16]


def key_of(name, args, kw):
    if name in ("conv3x3", "conv_wgrad"):
        return (name, kw["H"], kw["cin"], kw["cout"], kw.get("flags", int(kw.get("ups", 0))))
    ts = [a for a in list(args) + list(kw.values()) if isinstance(a, torch.Tensor)]
    big = max(ts, key=lambda t: t.numel()) if ts else None
    shape = tuple(big.shape) if big is not None else ()
    return (name, shape)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=8)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = _lib.HipOps(torch.bfloat16)
    rec = []
    on = [False]
    for name in [n for n in dir(ops) if not n.startswith("_")]:
        f = getattr(ops, name)
        if not callable(f) or name in ("packed_elems", "pack_table", "conv_workspace_bytes",
                                       "wgrad_workspace_bytes"):
            continue

        def wrap(f=f, name=name):
            def g(*args, **kw):
                if not on[0]:
                    return f(*args, **kw)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r = f(*args, **kw)
                e1.record()
                rec.append((key_of(name, args, kw), e0, e1))
                return r
            return g
        setattr(ops, name, wrap())
    s, B = a.stage, a.batch
    R = 4 * 2 ** s
    gen = torch.Generator().manual_seed(1234)
    gsh, dsh = E.g_param_shapes(PAPER, s), E.d_param_shapes(PAPER, s)
    init = lambda sh: {k: (torch.randn(v, generator=gen) if k.endswith("weight") else torch.zeros(v))
                       for k, v in sh}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), dev, init(gsh))
    fpD = E.FlatParams(dsh, E.dead_params("D", s), dev, init(dsh))
    eng = E.StepEngine(ops, PAPER, s, B, dev)
    eng.bind(fpG, fpD, E.Hyper())
    real = torch.rand(B, 3, R, R, device=dev) * 2 - 1
    z = torch.randn(2, B, 512, device=dev)
    for _ in range(2):
        eng.train_step(real, z[0], z[1], 1.0, 1.0)
    torch.cuda.synchronize()
    on[0] = True
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    for _ in range(a.steps):
        eng.train_step(real, z[0], z[1], 1.0, 1.0)
    s1.record()
    torch.cuda.synchronize()
    on[0] = False
    agg = collections.defaultdict(lambda: [0.0, 0])
    for k, e0, e1 in rec:
        agg[k][0] += e0.elapsed_time(e1)
        agg[k][1] += 1
    step_ms = s0.elapsed_time(s1) / a.steps
    tot = sum(v[0] for v in agg.values()) / a.steps
    print(f"step {step_ms:.3f} ms, op time {tot:.3f} ms")
    byop = collections.defaultdict(float)
    for k, v in agg.items():
        byop[k[0]] += v[0] / a.steps
    for k, v in sorted(byop.items(), key=lambda kv: -kv[1]):
        print(f"  {k:22s} {v:7.3f} ms")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][0])
    out = []
    for k, (ms, n) in rows:
        out.append(dict(key=[str(x) for x in k], ms_per_step=round(ms / a.steps, 4),
                        calls_per_step=n // a.steps, us_per_call=round(1e3 * ms / n, 1)))
        print(f"{ms / a.steps:7.3f} ms {n // a.steps:3d}x {1e3 * ms / n:7.1f} us  {k}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(dict(step_ms=step_ms, rows=out), f, indent=1)


if __name__ == "__main__":
    main()
