"""GPU input pipeline: flip + ColorJitter + ToTensor + Normalize of
lib/dataset.py:106-117 on the GPU (pg_augment_u8), byte-exact against the reference's own
path: ColorJitter on the PIL image (oracle/augment_oracle.py:augment_pil, real PIL calls).

* CPU: the parameter draw follows torchvision's call order (a generator in the same state
  gives the same draws as RandomHorizontalFlip + ColorJitter.get_params); the numpy
  restatement of Pillow's C arithmetic (what the kernel computes) equals PIL exhaustively
  per op -- L and RGB->HSV over all 2^24 colours, HSV->RGB over all 2^24 triples, blend over
  every byte pair at 400 factors -- and the whole chain equals augment_pil byte for byte
  over random images and all 24 op orders.
* GPU: the kernel's output equals augment_pil exactly (fp32 values of (u8/255 - .5)/.5,
  compared with ==) at 64^2 with edge-case images (flat gray, saturated primaries, hue wrap,
  negative and positive hue shifts, factors past 1), at 1024^2 (the C5 size), for all 24
  op orders, and through the threaded loader end to end on PNG files.
"""
import itertools
import os

import numpy as np
import pytest
import torch

from oracle import augment_oracle as A
from pggan_amd import data as PD


def _images(B, S, seed):
    rng = np.random.default_rng(seed)
    # smooth random images (natural-image-like) plus a few hard pixels
    base = rng.integers(0, 256, size=(B, S // 8 + 1, S // 8 + 1, 3)).astype(np.float32)
    big = np.repeat(np.repeat(base, 8, axis=1), 8, axis=2)[:, :S, :S]
    noise = rng.normal(0, 12, size=big.shape)
    u8 = np.clip(big + noise, 0, 255).astype(np.uint8)
    u8[0, :4, :4] = 128                              # flat gray (max == min)
    u8[0, 4:8, :4] = (255, 0, 0)                     # primaries (hue sectors)
    u8[0, 8:12, :4] = (0, 255, 0)
    u8[0, 12:16, :4] = (0, 0, 255)
    u8[0, 16:20, :4] = (255, 0, 1)                   # hue just below 1.0 (wraps with +hue)
    u8[0, 20:24, :4] = (0, 0, 0)
    u8[0, 24:28, :4] = (255, 255, 255)
    return u8


def _torchvision_draws(B, seed):
    """The torch RNG calls of RandomHorizontalFlip(0.5).forward + ColorJitter.get_params, in
    the order torchvision makes them per image."""
    g = torch.Generator().manual_seed(seed)
    out = []
    for _ in range(B):
        flip = torch.rand(1, generator=g) < 0.5
        perm = torch.randperm(4, generator=g)
        b = float(torch.empty(1).uniform_(0.8, 1.2, generator=g))
        c = float(torch.empty(1).uniform_(0.8, 1.2, generator=g))
        s = float(torch.empty(1).uniform_(0.8, 1.2, generator=g))
        h = float(torch.empty(1).uniform_(-0.01, 0.01, generator=g))
        out.append((bool(flip), perm.tolist(), b, c, s, h))
    return out


def test_param_draw_follows_torchvision_order():
    p = PD.draw_params(6, torch.Generator().manual_seed(7))
    for row, (flip, perm, b, c, s, h) in zip(p, _torchvision_draws(6, 7)):
        assert bool(row[0]) == flip
        assert row[5:9].astype(int).tolist() == perm
        np.testing.assert_allclose(row[1:5], np.float32([b, c, s, h]), rtol=0, atol=0)
    assert ((p[:, 1:4] >= 0.8) & (p[:, 1:4] <= 1.2)).all() and (np.abs(p[:, 4]) <= 0.01).all()


def _all_colours():
    idx = np.arange(1 << 24, dtype=np.uint32)
    rgb = np.stack([(idx >> 16) & 255, (idx >> 8) & 255, idx & 255], -1).astype(np.uint8)
    return rgb


def test_luma_and_hsv_exhaustive():
    """Convert.c restated: RGB->L and RGB->HSV over every colour, HSV->RGB over every
    triple, equal to PIL's conversions."""
    from PIL import Image
    rgb = _all_colours()
    im = Image.fromarray(rgb.reshape(4096, 4096, 3), "RGB")
    r, g, b = (rgb[:, c].astype(np.int64) for c in range(3))
    assert np.array_equal(np.asarray(im.convert("L")).ravel(), A.luma_u8(r, g, b))
    hsv = np.asarray(im.convert("HSV")).reshape(-1, 3).astype(np.int64)
    h, s, v = A.rgb2hsv_u8(r, g, b)
    assert np.array_equal(hsv, np.stack([h, s, v], -1))
    back = np.asarray(Image.frombytes("HSV", (4096, 4096), rgb.tobytes()).convert("RGB"))
    R, G, B = A.hsv2rgb_u8(r, g, b)     # the same bytes read as (h, s, v)
    assert np.array_equal(back.reshape(-1, 3).astype(np.int64), np.stack([R, G, B], -1))


def test_blend_every_byte_pair():
    """Blend.c restated: every (in1, in2) byte pair at 400 factors in and past [0, 1]."""
    from PIL import Image
    a = np.repeat(np.arange(256, dtype=np.uint8), 256)
    b = np.tile(np.arange(256, dtype=np.uint8), 256)
    A1 = np.stack([a, b, a], -1).reshape(256, 256, 3)
    A2 = np.stack([b, a, b], -1).reshape(256, 256, 3)
    i1, i2 = Image.fromarray(A1, "RGB"), Image.fromarray(A2, "RGB")
    rng = np.random.default_rng(0)
    alphas = list(rng.uniform(0.8, 1.2, 392)) + [0.8, 1.2, 1.0, 0.0, 0.99999994, 1.0000001, 1.5,
                                                 -0.25]
    for al in alphas:
        ref = np.asarray(Image.blend(i1, i2, float(al))).astype(np.int64)
        assert np.array_equal(ref, A.blend_u8(A1, A2, np.float32(al))), al


@pytest.mark.parametrize("S,seed", [(48, 3), (64, 4)])
def test_restatement_equals_pil_chain(S, seed):
    """The whole chain (flip, the 4 ops in every order, contrast's integer mean taken after
    the ops before it, ToTensor, Normalize) equals the PIL calls byte for byte."""
    perms = list(itertools.permutations(range(4)))
    u8 = _images(len(perms), S, seed)
    p = PD.draw_params(len(perms), torch.Generator().manual_seed(seed))
    p[:, 5:9] = np.float32(perms)
    p[0, 4], p[1, 4] = 0.01, -0.01
    assert np.array_equal(A.augment_pil_np(u8, p), A.augment_pil(u8, p))


def _run_gpu(u8, p):
    from pggan_amd import _lib
    ops = _lib.HipOps(torch.bfloat16)
    B, H, W, _ = u8.shape
    src = torch.from_numpy(u8).cuda()
    prm = torch.from_numpy(p).cuda()
    out = torch.empty(B, 3, H, W, device="cuda")
    ops.augment_u8(src, prm, out)
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _assert_bytes_equal(got, ref):
    bad = got != ref
    assert not bad.any(), (int(bad.sum()), float(np.abs(got - ref).max()) * 127.5)


@pytest.mark.gpu
@pytest.mark.parametrize("B,S,seed", [(4, 64, 5), (2, 1024, 6)], ids=["64", "1024"])
def test_augment_kernel_equals_pil(B, S, seed):
    u8 = _images(B, S, seed)
    p = PD.draw_params(B, torch.Generator().manual_seed(seed))
    p[0, 0] = 1.0                       # at least one flipped and one unflipped image
    p[-1, 0] = 0.0
    p[0, 4] = 0.01                      # hue wrap, both shift signs
    p[-1, 4] = -0.01
    _assert_bytes_equal(_run_gpu(u8, p), A.augment_pil(u8, p))


@pytest.mark.gpu
def test_every_op_order():
    """All 24 fn_idx orders (contrast at every position: its mean is taken after the ops
    before it)."""
    perms = list(itertools.permutations(range(4)))
    u8 = _images(len(perms), 32, 9)
    p = PD.draw_params(len(perms), torch.Generator().manual_seed(9))
    p[:, 5:9] = np.float32(perms)
    _assert_bytes_equal(_run_gpu(u8, p), A.augment_pil(u8, p))


@pytest.mark.gpu
def test_batch_loader_end_to_end(tmp_path):
    from PIL import Image
    from pggan_amd import _lib
    rng = np.random.default_rng(2)
    os.makedirs(tmp_path / "sub")
    for k in range(6):
        im = rng.integers(0, 256, size=(40 + k, 50, 3), dtype=np.uint8)
        Image.fromarray(im).save(tmp_path / ("sub" if k % 2 else "") / f"im{k}.png")
    ds = PD.ImageFolderDataset([str(tmp_path)], scale_index=3)      # 32 x 32
    assert len(ds) == 6
    batches = [[0, 1, 2, 3], [4, 5, 0, 1], [2, 3, 4, 5], [0, 1, 2, 3]]
    # cache_bytes: room for 5 of the 6 images, then no cache; 0: no cache.  Every batch is
    # byte-exact either way.  The cache is allocated at the second batch (after the stage's
    # step has its buffers): batch 0 decodes 4, batch 1 decodes and caches 4, 5, 0, 1,
    # batch 2 decodes 2 (cached, the fifth row) and 3 (no room), batch 3 decodes 3 again.
    for cache in (5 * 32 * 32 * 3, 0):
        ld = PD.BatchLoader(ds, "cuda", _lib.HipOps(torch.bfloat16), seed=4, workers=3,
                            cache_bytes=cache)
        outs = [ld.next(b, prefetch=batches[(k + 1) % len(batches)]).cpu().numpy()
                for k, b in enumerate(batches)]
        decoded = ld.decoded
        ld.close()
        assert decoded == (4 + 4 + 2 + 1 if cache else 16), decoded
        g = torch.Generator().manual_seed(4)
        for idx, out in zip(batches, outs):
            u8 = np.stack([ds.load(i) for i in idx])
            _assert_bytes_equal(out, A.augment_pil(u8, PD.draw_params(4, g)))
