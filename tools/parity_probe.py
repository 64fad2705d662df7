"""bf16 step parity over consecutive steps, single process (GPU only; diagnostic).

    python tools/parity_probe.py [--stage 7] [--B 4] [--steps 2]

Each step is checked by kink_parity.run_step against the float64 oracle replayed from the
state before that step (our fake images fed to D); prints the loss / image errors and the
worst gradient cosines per step without asserting.
"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")):
    sys.path.insert(0, p)
import kink_parity as K  # noqa: E402
from gen_inputs import make_inputs  # noqa: E402
from test_gpu_baseline_parity import build  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stage", type=int, default=7)
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--steps", type=int, default=2)
    a = ap.parse_args()
    eng, fpG, fpD = build(a.stage, a.B, torch.bfloat16, seed=708)
    for t in range(a.steps):
        st = make_inputs(a.B, 4 * 2 ** a.stage, seed=808 + t, n_steps=1)[0]
        real, z1, z2 = (torch.from_numpy(st[k]) for k in ("real", "z1", "z2"))
        ours, ref, kinks = K.run_step(eng, fpG, fpD, real, z1, z2, 1.0, threads=16,
                                      feed_images=True)
        try:
            K.compare_bf16(ours, ref, fpG, fpD, kinks, loss_rtol=2e-3, min_cos=0.999,
                           flip_bound=K.FLIP_BOUND[torch.bfloat16], img_rtol=3e-2,
                           what=f"step {t}: ")
        except AssertionError as e:
            print(f"step {t} FAILS: {e}", flush=True)


if __name__ == "__main__":
    main()
