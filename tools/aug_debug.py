"""GPU: pg_augment_u8 vs the PIL path on the all-orders batch; prints the mismatching pixels."""
import itertools
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import augment_oracle as A  # noqa: E402
from pggan_amd import data as PD  # noqa: E402
from test_augment import _images, _run_gpu  # noqa: E402

perms = list(itertools.permutations(range(4)))
u8 = _images(len(perms), 32, 9)
p = PD.draw_params(len(perms), torch.Generator().manual_seed(9))
p[:, 5:9] = np.float32(perms)
got = _run_gpu(u8, p)
ref = A.augment_pil(u8, p)
bad = np.argwhere(got != ref)
print("mismatches", len(bad))
for b, c, y, x in bad[:40]:
    sx = 31 - x if p[b, 0] else x
    print(f"img {b} ch {c} y {y} x {x} src {u8[b, y, sx].tolist()} order {p[b, 5:9].astype(int).tolist()} "
          f"f {p[b, 1:5].tolist()} got {got[b, c, y, x] * 127.5 + 127.5:.1f} ref {ref[b, c, y, x] * 127.5 + 127.5:.1f}")
