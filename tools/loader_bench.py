"""Input-pipeline throughput (GPU box): pggan_amd.data.BatchLoader on image
files written at run time, at every stage a BASELINE config trains (128^2 .. 1024^2 targets from
1024^2 sources: the host decodes the full image and resizes, lib/dataset.py:101-107), with the
decode threads the box's CPU share allows (16), next to the training step's rate.

    python tools/loader_bench.py [--n 64] [--workers 16] [--out FILE]

Images: smooth synthetic RGB content (colour gradients + low-amplitude noise; pure noise
compresses like no photograph does) saved as 1024^2 PNG (the format of the reference's own sample
assets, assets/k-celeb).  Per target size, two epochs over the n images in the config's batch
size through `next(idx, prefetch)` exactly as ProgressiveGAN.load_next_batch chains them:
  cold -- the first epoch: every image decoded + resized on the host (the HBM cache fills);
  warm -- the second epoch: every batch gathered from the HBM cache (HbmImageCache).
img/s = images delivered on the GPU / wall time, synchronised per epoch.  One JSON line each.
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (stage, batch per GPU) of the BASELINE configs: C2 128^2 B16, C3 256^2 B8, C4 512^2 B8, C5 1024^2 B4
STAGES = [(5, 16), (6, 8), (7, 8), (8, 4)]


def synth(rng, size):
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / size
    base = np.stack([x, y, 1.0 - 0.5 * (x + y)], axis=-1)
    a = rng.uniform(0.3, 1.0, size=3).astype(np.float32)
    img = base * a * 200 + rng.normal(0, 6, size=(size, size, 3)).astype(np.float32) + 20
    return np.clip(img, 0, 255).astype(np.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--workers", type=int, default=16)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from PIL import Image

    from pggan_amd import _lib
    from pggan_amd.data import BatchLoader, ImageFolderDataset

    ops = _lib.HipOps(torch.bfloat16)
    rng = np.random.default_rng(0)
    lines = []
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        for i in range(a.n):
            Image.fromarray(synth(rng, 1024)).save(os.path.join(tmp, f"{i:04d}.png"))
        write_s = time.perf_counter() - t0
        mb = sum(os.path.getsize(os.path.join(tmp, f)) for f in os.listdir(tmp)) / a.n / 1e6
        # untimed warm-up: the thread pool, the pinned-memory pool and the first launches of
        # the gather / augmentation kernels (~50 ms once per process)
        ds = ImageFolderDataset([tmp], scale_index=STAGES[0][0])
        ld = BatchLoader(ds, "cuda", ops, seed=0, workers=a.workers, cache_bytes=1 << 30)
        for _ in range(2):
            ld.next(list(range(STAGES[0][1])))
        torch.cuda.synchronize()
        ld.close()
        for stage, B in STAGES:
            ds = ImageFolderDataset([tmp], scale_index=stage)
            S = ds.size
            assert len(ds) == a.n and a.n % B == 0
            ld = BatchLoader(ds, "cuda", ops, seed=0, workers=a.workers, cache_bytes=8 << 30)
            nb = a.n // B
            idx = lambda k: list(range((k % nb) * B, (k % nb) * B + B))
            for epoch in ("cold", "warm"):
                base = 0 if epoch == "cold" else nb
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for k in range(base, base + nb):
                    out = ld.next(idx(k), prefetch=idx(k + 1))
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                assert out.shape == (B, 3, S, S)
                line = dict(epoch=epoch, format="png", source_px=1024, target_px=S, stage=stage,
                            batch=B, workers=a.workers, host_cpu_count=os.cpu_count(),
                            omp_num_threads=os.environ.get("OMP_NUM_THREADS"), images=nb * B,
                            seconds=round(dt, 4), img_per_s=round(nb * B / dt, 1),
                            decoded=ld.decoded, cached=ld.cache.used, mean_file_mb=round(mb, 2),
                            write_s=round(write_s, 1))
                print(json.dumps(line), flush=True)
                lines.append(line)
            ld.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
