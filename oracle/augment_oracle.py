"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): CPU statements of the
reference's training-image transform after the resize, lib/dataset.py:106-117

    RandomHorizontalFlip(p=0.5) -> ColorJitter(0.2, 0.2, 0.2, 0.01) -> ToTensor
    -> Normalize((0.5, 0.5, 0.5), (0.5, 0.5, 0.5)),

which the reference applies to a PIL image, so ColorJitter runs torchvision's PIL path
(torchvision/transforms/functional_pil.py, torchvision 0.12 as pinned with torch 1.11):
ImageEnhance.Brightness / Contrast / Color and adjust_hue (the H band of PIL's HSV mode
shifted by np.uint8(hue_factor * 255), wrapping).

* `augment_pil`: that path itself -- the same PIL calls (PIL is installed here; torchvision
  is not, so its four adjust_* wrappers are restated line for line).
* `augment_pil_np`: a numpy restatement of the C arithmetic under those calls (Pillow's
  libImaging: Blend.c ImagingBlend, Convert.c rgb2l / rgb2hsv_row / hsv2rgb, ImageStat's
  mean), i.e. exactly what pg_augment_u8 computes.  Each piece is checked against PIL
  exhaustively where the domain allows (every RGB colour for L and HSV, every HSV triple
  for the way back, every byte pair for blend over many factors: tests/test_augment.py),
  and the whole chain against `augment_pil` byte for byte.

Parameters: per image {flip, brightness, contrast, saturation, hue, fn_idx[4]} as drawn by
pggan_amd.data.draw_params (torchvision's RandomHorizontalFlip + ColorJitter.get_params
call order).  The hue shift np.uint8(hue_factor * 255) of a negative factor is taken as
truncation toward zero, then wrapping (the x86 behaviour numpy had for that cast).
"""
from __future__ import annotations

import numpy as np

F32, F64 = np.float32, np.float64


def hue_shift_u8(hf):
    """np.uint8(hue_factor * 255): the product in double, truncated, wrapped to a byte."""
    return int(np.array(float(hf) * 255.0).astype(np.int64)) & 255


def augment_pil(u8, params):
    """The reference's path: flip + the four ops on the PIL image (functional_pil), then
    ToTensor (uint8 / 255 in fp32) + Normalize."""
    from PIL import Image, ImageEnhance
    out = []
    for im, prm in zip(u8, params):
        img = Image.fromarray(im, "RGB")
        if prm[0]:
            img = img.transpose(Image.FLIP_LEFT_RIGHT)
        bf, cf, sf, hf = (float(x) for x in prm[1:5])
        for fn in prm[5:9].astype(int):
            if fn == 0:
                img = ImageEnhance.Brightness(img).enhance(bf)
            elif fn == 1:
                img = ImageEnhance.Contrast(img).enhance(cf)
            elif fn == 2:
                img = ImageEnhance.Color(img).enhance(sf)
            else:
                h, s, v = img.convert("HSV").split()
                np_h = np.array(h, dtype=np.uint8)
                with np.errstate(over="ignore"):
                    np_h += np.uint8(hue_shift_u8(hf))
                img = Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert("RGB")
        x = np.asarray(img, F32).transpose(2, 0, 1) / F32(255.0)
        out.append((x - F32(0.5)) / F32(0.5))
    return np.stack(out)


# ---- numpy restatement of Pillow's C arithmetic (libImaging) --------------------------
def blend_u8(a, b, alpha):
    """ImagingBlend (Blend.c): out = in1 + alpha * (in2 - in1) in float (alpha is the C
    float of the factor), truncated to uint8; outside 0 <= alpha <= 1 clipped to [0, 255]."""
    al = F32(alpha)
    t = (np.asarray(a).astype(F32) + al * (np.asarray(b).astype(F32) - np.asarray(a).astype(F32))
         ).astype(F32)
    if F32(0) <= al <= F32(1):
        return t.astype(np.int64)
    return np.where(t <= 0, 0, np.where(t >= 255, 255, np.trunc(t))).astype(np.int64)


def luma_u8(r, g, b):
    """rgb2l (Convert.c): ITU-R 601-2 luma in 16.16 fixed point, rounded."""
    return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16


def rgb2hsv_u8(r, g, b):
    """rgb2hsv_row (Convert.c): float ratios, the sector offsets and the wrap in double,
    truncation to uint8; max == min gives h = s = 0."""
    mx = np.maximum(r, np.maximum(g, b))
    mn = np.minimum(r, np.minimum(g, b))
    eq = mx == mn
    cr = np.where(eq, 1, mx - mn).astype(F32)
    s = cr / np.where(mx == 0, 1, mx).astype(F32)
    rc = (mx - r).astype(F32) / cr
    gc = (mx - g).astype(F32) / cr
    bc = (mx - b).astype(F32) / cr
    h = np.where(r == mx, (bc - gc).astype(F64),
                 np.where(g == mx, (2.0 + rc.astype(F64)) - bc.astype(F64),
                          (4.0 + gc.astype(F64)) - rc.astype(F64))).astype(F32)
    h = np.fmod(h.astype(F64) / 6.0 + 1.0, 1.0).astype(F32)
    uh = np.clip((h.astype(F64) * 255.0).astype(np.int64), 0, 255)
    us = np.clip((s.astype(F64) * 255.0).astype(np.int64), 0, 255)
    return np.where(eq, 0, uh), np.where(eq, 0, us), mx


def hsv2rgb_u8(h, s, v):
    """hsv2rgb (Convert.c): sector and remainder in double, fs and f stored as float, C
    round() (half away from zero) of v * (1 - ...), clipped; s == 0 gives (v, v, v)."""
    hd = h.astype(F32).astype(F64) * 6.0 / 255.0
    i = np.floor(hd).astype(np.int64)
    f = (hd - i.astype(F32).astype(F64)).astype(F32)
    fs = (s.astype(F32).astype(F64) / 255.0).astype(F32)
    vf = v.astype(F32).astype(F64)

    def c8(x):
        return np.clip(np.floor(x + 0.5), 0, 255).astype(np.int64)
    p = c8(vf * (1.0 - fs.astype(F64)))
    q = c8(vf * (1.0 - (fs * f).astype(F32).astype(F64)))
    t = c8(vf * (1.0 - fs.astype(F64) * (1.0 - f.astype(F64))))
    k = i % 6
    R = np.choose(k, (v, q, p, p, t, v))
    G = np.choose(k, (t, v, v, q, p, p))
    B = np.choose(k, (p, p, t, v, v, q))
    z = s == 0
    return np.where(z, v, R), np.where(z, v, G), np.where(z, v, B)


def contrast_mean(r, g, b):
    """ImageEnhance.Contrast's degenerate level: int(ImageStat.Stat(L).mean[0] + 0.5), the
    mean = (exact integer sum of L) / count in double."""
    L = luma_u8(r, g, b)
    return int(float(L.sum()) / float(L.size) + 0.5)


def augment_pil_np(u8, params):
    """augment_pil with every op restated (what pg_augment_u8 computes)."""
    out = []
    for im, prm in zip(u8, params):
        x = im[:, ::-1] if prm[0] else im
        r, g, b = (x[..., c].astype(np.int64) for c in range(3))
        bf, cf, sf = F32(prm[1]), F32(prm[2]), F32(prm[3])
        dh = hue_shift_u8(prm[4])
        for fn in prm[5:9].astype(int):
            if fn == 0:
                r, g, b = blend_u8(0, r, bf), blend_u8(0, g, bf), blend_u8(0, b, bf)
            elif fn == 1:
                m = contrast_mean(r, g, b)
                r, g, b = blend_u8(m, r, cf), blend_u8(m, g, cf), blend_u8(m, b, cf)
            elif fn == 2:
                L = luma_u8(r, g, b)
                r, g, b = blend_u8(L, r, sf), blend_u8(L, g, sf), blend_u8(L, b, sf)
            else:
                h, s, v = rgb2hsv_u8(r, g, b)
                r, g, b = hsv2rgb_u8((h + dh) & 255, s, v)
        y = np.stack([r, g, b]).astype(F32) / F32(255.0)
        out.append((y - F32(0.5)) / F32(0.5))
    return np.stack(out)
