"""Input-pipeline throughput (GPU box): pggan_amd.data.BatchLoader on image
files written at run time, at the C5 stage (1024^2, batch 4), with the decode threads the box's
CPU share allows (16), next to the training step's rate.

    python tools/loader_bench.py [--n 48] [--batches 24] [--workers 16] [--out FILE]

Images: smooth synthetic RGB content (colour gradients + low-amplitude noise; pure noise
compresses like no photograph does) saved as PNG (the reference's own sample assets are
1024^2 PNGs, assets/k-celeb) and as JPEG (quality 95), once at 1024^2 (decode only; the
Resize is a same-size resample) and once at 1280^2 (decode + a real bilinear downscale).
Each configuration: one warm-up batch, then `batches` batches through `next(idx, prefetch)`
exactly as ProgressiveGAN.load_next_batch chains them, synchronised at the end; img/s = images
delivered on the GPU / wall time.  One JSON line per configuration.
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


def synth(rng, size):
    y, x = np.mgrid[0:size, 0:size].astype(np.float32) / size
    base = np.stack([x, y, 1.0 - 0.5 * (x + y)], axis=-1)
    a = rng.uniform(0.3, 1.0, size=3).astype(np.float32)
    img = base * a * 200 + rng.normal(0, 6, size=(size, size, 3)).astype(np.float32) + 20
    return np.clip(img, 0, 255).astype(np.uint8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=48)
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--batch", type=int, default=4)
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
        for fmt, src in (("png", 1024), ("jpg", 1024), ("png", 1280), ("jpg", 1280)):
            d = os.path.join(tmp, f"{fmt}{src}")
            os.makedirs(d)
            t0 = time.perf_counter()
            for i in range(a.n):
                im = Image.fromarray(synth(rng, src))
                if fmt == "png":
                    im.save(os.path.join(d, f"{i:04d}.png"))
                else:
                    im.save(os.path.join(d, f"{i:04d}.jpg"), quality=95)
            write_s = time.perf_counter() - t0
            ds = ImageFolderDataset([d], scale_index=8)
            assert len(ds) == a.n and ds.size == 1024
            ld = BatchLoader(ds, "cuda", ops, seed=0, workers=a.workers)
            order = np.arange(a.n)
            B = a.batch

            def idx(k):
                j = (k * B) % (a.n - B + 1)
                return order[j:j + B]

            ld.next(idx(0), prefetch=idx(1))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(1, a.batches + 1):
                out = ld.next(idx(k), prefetch=idx(k + 1))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ld.close()
            assert out.shape == (B, 3, 1024, 1024)
            mb = sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)) / a.n / 1e6
            line = dict(format=fmt, source_px=src, target_px=1024, batch=B, workers=a.workers,
                        host_cpu_count=os.cpu_count(), omp_num_threads=os.environ.get("OMP_NUM_THREADS"),
                        images=a.batches * B, seconds=round(dt, 3),
                        img_per_s=round(a.batches * B / dt, 1), mean_file_mb=round(mb, 2),
                        write_s=round(write_s, 1))
            print(json.dumps(line), flush=True)
            lines.append(line)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
