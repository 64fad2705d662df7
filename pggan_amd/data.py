"""Training-image input pipeline: UnsupervisedDataset (lib/dataset.py:86-127)
with the per-image augmentation on the GPU.

Host: glob the roots like the reference (`*.*g` at every depth), decode + Resize with PIL
(torchvision's Resize on a PIL image is PIL's bilinear resize, so this step is the
reference's own code path) in a thread pool that prefetches the next batch while the
current step runs; the uint8 HWC batch goes to HBM from pinned memory.

GPU (`pg_augment_u8`, pggan_amd/csrc/augment.hip): RandomHorizontalFlip(0.5),
ColorJitter(0.2, 0.2, 0.2, 0.01), ToTensor, Normalize(0.5, 0.5) in one pass over the
batch (three launches).  The random parameters are drawn on the host with a torch CPU
generator in torchvision's call order per image -- `torch.rand(1) < p` for the flip, then
ColorJitter.get_params: `torch.randperm(4)`, brightness, contrast, saturation, hue
`torch.empty(1).uniform_(lo, hi)` -- so a generator in the same state draws the same
parameters as the reference's transform.  The jitter is the reference's PIL path
(ImageEnhance blends and PIL's uint8 HSV hue shift, uint8 after every op) in Pillow's own
arithmetic: the output equals the reference transform byte for byte (tests/test_augment.py).

HBM cache (`HbmImageCache`): decode + Resize is deterministic and runs before every random
op (lib/dataset.py:102-112), so the resized uint8 image of a dataset index is the same in
every epoch.  The loader keeps it in HBM after its first decode (per stage: the target size
changes with the stage) and gathers later batches from there, so after the first epoch the
host decode -- 344 img/s from 1024^2 PNG on the box's 16 threads, below the step's rate at
every stage (profiles/r4_loader.json) -- no longer bounds training.  The bytes the augmentation
reads are the ones it would have decoded, so the output stays byte-exact.  Sizes: 3 S^2 bytes
per image (3 MiB at 1024^2, 192 KiB at 256^2); a DP rank caches only its own shard.
"""
from __future__ import annotations

import glob
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

# ColorJitter(0.2, 0.2, 0.2, 0.01) ranges (lib/dataset.py:110), flip probability (:108)
JITTER = dict(brightness=(0.8, 1.2), contrast=(0.8, 1.2), saturation=(0.8, 1.2), hue=(-0.01, 0.01))
FLIP_P = 0.5
PSTRIDE = 12   # floats per image in the pg_augment_u8 parameter table


def image_paths(roots):
    """lib/dataset.py:89-99: `*.*g` directly under each root and in every subdirectory."""
    paths = []
    for r in roots or []:
        paths += glob.glob(f"{r}/*.*g")
        for root, dirs, _ in os.walk(r):
            for d in dirs:
                paths += glob.glob(f"{root}/{d}/*.*g")
    return paths


def load_u8(path, size):
    """Decode + Resize((size, size)) (lib/dataset.py:107) -> uint8 [size, size, 3]."""
    from PIL import Image
    im = Image.open(path).convert("RGB").resize((size, size), Image.BILINEAR)
    return np.asarray(im, dtype=np.uint8)


def draw_params(B, gen):
    """Per-image flip / ColorJitter parameters in torchvision's draw order -> fp32 [B, 12]:
    {flip, brightness, contrast, saturation, hue, fn_idx[4], 1 - contrast, 1 - saturation, 0}
    (the last three are not read by the PIL-path kernel; the table layout is the ABI's)."""
    p = np.zeros((B, PSTRIDE), np.float32)
    for b in range(B):
        flip = bool(torch.rand(1, generator=gen) < FLIP_P)
        fn_idx = torch.randperm(4, generator=gen)
        f = [float(torch.empty(1).uniform_(*JITTER[k], generator=gen))
             for k in ("brightness", "contrast", "saturation", "hue")]
        p[b, 0] = 1.0 if flip else 0.0
        p[b, 1:5] = f
        p[b, 5:9] = fn_idx.numpy()
        p[b, 9] = 1.0 - f[1]
        p[b, 10] = 1.0 - f[2]
    return p


class ImageFolderDataset:
    """The image list of UnsupervisedDataset; `load(i)` decodes + resizes one image."""

    def __init__(self, roots, scale_index=0):
        self.paths = image_paths(roots)
        self.size = 2 ** (scale_index + 2)

    def __len__(self):
        return len(self.paths)

    def load(self, i):
        return load_u8(self.paths[i], self.size)


class HbmImageCache:
    """The decoded + resized uint8 images of one dataset at one size, in HBM: slot table
    (dataset index -> row of `buf`, -1 = not cached) and rows filled in first-decode order
    until `budget_bytes` is used (the rest is decoded on the host every time)."""

    def __init__(self, n, size, device, budget_bytes):
        per = 3 * size * size
        self.cap = int(max(0, min(n, budget_bytes // per)))
        self.size = size
        self.slot = np.full(n, -1, dtype=np.int64)
        self.used = 0
        self.buf = (torch.empty(self.cap, size, size, 3, dtype=torch.uint8, device=device)
                    if self.cap else None)

    def slots(self, idx):
        return [int(self.slot[i]) for i in idx]

    def insert(self, idx, dev_imgs):
        """Store rows dev_imgs[k] (uint8 [m, S, S, 3] on the device) for dataset indices idx
        while there is room; returns how many were stored."""
        k = 0
        for j, i in enumerate(idx):
            if self.slot[i] >= 0 or self.used >= self.cap:
                continue
            self.buf[self.used].copy_(dev_imgs[j])
            self.slot[i] = self.used
            self.used += 1
            k += 1
        return k


def default_cache_bytes(device, fraction=0.4):
    """HBM for the image cache: `fraction` of the device's free memory now."""
    dev = torch.device(device)
    if dev.type != "cuda":
        return 0
    free, _ = torch.cuda.mem_get_info(dev)
    return int(free * fraction)


class BatchLoader:
    """Decode/resize in `workers` host threads (PIL releases the GIL), one batch ahead;
    flip + jitter + normalize on the GPU.  `next(indices, prefetch=None)` returns the fp32
    NCHW [-1, 1] batch on `device` and starts decoding `prefetch` (the next indices).
    cache_bytes > 0: decoded images are kept in an HbmImageCache and later batches gather
    them there (no decode, no host-to-device copy); None: default_cache_bytes."""

    def __init__(self, dataset, device, ops, seed=0, workers=None, gen=None, cache_bytes=None):
        """gen: the torch CPU generator the augmentation parameters are drawn from (shared
        across the loaders of successive stages); default a new one seeded with `seed`."""
        self.ds, self.dev, self.ops = dataset, torch.device(device), ops
        if not hasattr(ops, "augment_u8"):
            raise RuntimeError("pggan_amd: the input pipeline needs the HIP library (augment_u8)")
        self.pool = ThreadPoolExecutor(max_workers=workers or min(16, os.cpu_count() or 1))
        self.gen = gen if gen is not None else torch.Generator().manual_seed(seed)
        self._pending = {}       # dataset index -> future of its decoded image
        self._ws = None
        # the cache is allocated at the SECOND batch: the first one is drawn before the stage's
        # training step has allocated its buffers (ProgressiveGAN.train_step builds the engine
        # after load_next_batch), so a default budget sized from free memory then would take
        # memory the step needs.  cache_bytes=0 turns it off (opt-out).
        self._cache_bytes = cache_bytes
        self._calls = 0
        self.cache = None
        self.decoded = 0         # images decoded on the host so far

    def _make_cache(self):
        b = self._cache_bytes
        if b is None:
            b = default_cache_bytes(self.dev)
        if b > 0:
            self.cache = HbmImageCache(len(self.ds), self.ds.size, self.dev, b)

    def _cached(self, i):
        return self.cache is not None and self.cache.slot[i] >= 0

    def _submit(self, idx):
        for i in idx:
            i = int(i)
            if i not in self._pending and not self._cached(i):
                self._pending[i] = self.pool.submit(self.ds.load, i)

    def next(self, idx, prefetch=None):
        if self._calls == 1:
            self._make_cache()
        self._calls += 1
        idx = [int(i) for i in idx]
        self._submit(idx)
        B, S = len(idx), self.ds.size
        miss = [k for k, i in enumerate(idx) if not self._cached(i)]
        src = torch.empty(B, S, S, 3, dtype=torch.uint8, device=self.dev)
        if miss:
            imgs = [self._pending.pop(idx[k]).result() for k in miss]
            self.decoded += len(imgs)
            host = torch.from_numpy(np.stack(imgs)).pin_memory()
            dev_miss = host.to(self.dev, non_blocking=True)
            src[torch.tensor(miss, device=self.dev)] = dev_miss
            if self.cache is not None:
                self.cache.insert([idx[k] for k in miss], dev_miss)
        hit = [k for k in range(B) if k not in miss]
        if hit:
            rows = torch.tensor([int(self.cache.slot[idx[k]]) for k in hit], device=self.dev)
            if len(hit) == B:
                torch.index_select(self.cache.buf, 0, rows, out=src)
            else:
                src[torch.tensor(hit, device=self.dev)] = self.cache.buf.index_select(0, rows)
        if prefetch is not None:
            self._submit(prefetch)
        params = torch.from_numpy(draw_params(B, self.gen)).to(self.dev, non_blocking=True)
        out = torch.empty(B, 3, S, S, dtype=torch.float32, device=self.dev)
        self._ws = self.ops.augment_u8(src, params, out, ws=self._ws)
        return out

    def close(self):
        """Stop the decode threads; pending prefetches are cancelled; the cache is freed."""
        self._pending = {}
        self.cache = None
        self.pool.shutdown(wait=False, cancel_futures=True)
