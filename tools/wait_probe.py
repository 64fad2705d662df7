"""Where the main stream waits on the side stream (GPU only; diagnostic).

    python tools/wait_probe.py [--stage 8] [--B 4]

Runs two eager C5-shaped training steps of the engine (paper widths, bf16, random
parameters) and logs, for the second, every op call and every cross-stream event
operation with the stream it is enqueued on (main / side) and the engine line that issued
it.  A 'WAIT main' line is a point where the main (input-gradient) stream waits for the
side (weight-gradient) stream.
"""
import argparse
import os
import sys
import traceback

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from pggan_amd import _lib  # noqa: E402
from pggan_amd import engine as E  # noqa: E402

PAPER = [512, 512, 512, 512, 256, 128, 64, 32, 16]
LOG = []
ON = [False]


def where():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if fr.filename.endswith("engine.py"):
            return f"{fr.name}:{fr.lineno}"
    return "?"


def sname(eng, s):
    s = s if s is not None else torch.cuda.current_stream()
    if eng.side is not None and s.cuda_stream == eng.side.cuda_stream:
        return "side"
    return "main"


class Proxy:
    def __init__(self, ops, eng_ref):
        self._ops, self._eng = ops, eng_ref

    def __getattr__(self, n):
        a = getattr(self._ops, n)
        if not callable(a) or n.startswith("_"):
            return a

        def f(*x, **k):
            if ON[0]:
                LOG.append(f"  {sname(self._eng[0], None):4s} {n:22s} {where()}")
            return a(*x, **k)
        return f


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=8)
    ap.add_argument("--B", type=int, default=4)
    a = ap.parse_args()
    s, B = a.stage, a.B
    gsh, dsh = E.g_param_shapes(PAPER, s), E.d_param_shapes(PAPER, s)
    g = torch.Generator().manual_seed(0)
    PG = {k: torch.randn(v, generator=g) for k, v in gsh}
    PD = {k: torch.randn(v, generator=g) for k, v in dsh}
    fpG = E.FlatParams(gsh, E.dead_params("G", s), "cuda:0", PG)
    fpD = E.FlatParams(dsh, E.dead_params("D", s), "cuda:0", PD)
    ref = [None]
    ops = Proxy(_lib.HipOps(torch.bfloat16), ref)
    eng = E.StepEngine(ops, PAPER, s, B, "cuda:0")
    ref[0] = eng
    eng.bind(fpG, fpD, E.Hyper())

    orig_rec, orig_wait = _lib.HipEvent.record, _lib.HipEvent.wait

    def rec(self, stream=None):
        if ON[0]:
            LOG.append(f"  {sname(eng, stream):4s} record ev{id(self) % 997:<16d} {where()}")
        return orig_rec(self, stream)

    def wait(self, stream=None):
        if ON[0]:
            w = sname(eng, stream)
            LOG.append(f"{'WAIT' if w == 'main' else '    '} {w:4s} wait   ev{id(self) % 997:<16d} {where()}")
        return orig_wait(self, stream)
    _lib.HipEvent.record, _lib.HipEvent.wait = rec, wait
    ows = torch.cuda.Stream.wait_event

    def tw(self, ev):
        if ON[0]:
            w = sname(eng, self)
            LOG.append(f"{'WAIT' if w == 'main' else '    '} {w:4s} torch-wait {where()}")
        return ows(self, ev)
    torch.cuda.Stream.wait_event = tw

    real = torch.randn(B, 3, 4 * 2 ** s, 4 * 2 ** s, device="cuda")
    for step in range(2):
        ON[0] = step == 1
        z1, z2 = torch.randn(B, PAPER[0], device="cuda"), torch.randn(B, PAPER[0], device="cuda")
        eng.train_step(real, z1, z2, 1.0, 1.0)
        torch.cuda.synchronize()
    print("\n".join(LOG))


if __name__ == "__main__":
    main()
