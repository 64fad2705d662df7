"""TEST INFRASTRUCTURE ONLY (the checker, never the product path): CPU restatement of the
reference's training-image transform after the resize, lib/dataset.py:106-117

    RandomHorizontalFlip(p=0.5) -> ColorJitter(0.2, 0.2, 0.2, 0.01) -> ToTensor
    -> Normalize((0.5, 0.5, 0.5), (0.5, 0.5, 0.5)),

in two forms:

* `augment_tensor`: torchvision's tensor formulation (torchvision/transforms/
  functional_tensor.py: _blend, rgb_to_grayscale, adjust_brightness / contrast /
  saturation / hue, _rgb2hsv, _hsv2rgb) in numpy float32 -- what pg_augment_u8 computes;
* `augment_pil`: the reference's own path, the ops applied to the PIL image
  (torchvision/transforms/functional_pil.py: ImageEnhance.Brightness / Contrast / Color,
  hue through PIL's HSV mode with a uint8 shift of the H band), then ToTensor + Normalize.

torchvision is not installed in this image (the reference's dataset module cannot be
imported here), so neither form is checked against the reference's own run: the tensor
form is a restatement of torchvision's published algorithm (parity unpinned against a
torchvision run), and the PIL form calls the same PIL functions torchvision's PIL path calls.
Parameters: per image {flip, brightness, contrast, saturation, hue, fn_idx[4]} as drawn by
pggan_amd.data.draw_params (torchvision's ColorJitter.get_params order).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _gray(img):
    # rgb_to_grayscale (float input): 0.2989 r + 0.587 g + 0.114 b
    r, g, b = img[0], img[1], img[2]
    return (F32(0.2989) * r + F32(0.587) * g + F32(0.114) * b).astype(F32)


def _blend(img1, img2, ratio, one_minus):
    return np.clip(F32(ratio) * img1 + F32(one_minus) * img2, F32(0), F32(1)).astype(F32)


def _rgb2hsv(img):
    r, g, b = img[0], img[1], img[2]
    maxc = img.max(axis=0)
    minc = img.min(axis=0)
    eqc = maxc == minc
    cr = maxc - minc
    ones = np.ones_like(maxc)
    s = cr / np.where(eqc, ones, maxc)
    crd = np.where(eqc, ones, cr)
    rc = (maxc - r) / crd
    gc = (maxc - g) / crd
    bc = (maxc - b) / crd
    hr = (maxc == r) * (bc - gc)
    hg = ((maxc == g) & (maxc != r)) * (F32(2.0) + rc - bc)
    hb = ((maxc != g) & (maxc != r)) * (F32(4.0) + gc - rc)
    h = (hr + hg + hb).astype(F32)
    h = np.fmod(h / F32(6.0) + F32(1.0), F32(1.0)).astype(F32)
    return np.stack((h, s.astype(F32), maxc))


def _hsv2rgb(img):
    h, s, v = img[0], img[1], img[2]
    i = np.floor(h * F32(6.0))
    f = (h * F32(6.0) - i).astype(F32)
    i = i.astype(np.int32) % 6
    p = np.clip(v * (F32(1.0) - s), 0, 1).astype(F32)
    q = np.clip(v * (F32(1.0) - s * f), 0, 1).astype(F32)
    t = np.clip(v * (F32(1.0) - s * (F32(1.0) - f)), 0, 1).astype(F32)
    r = np.choose(i, (v, q, p, p, t, v))
    g = np.choose(i, (t, v, v, q, p, p))
    b = np.choose(i, (p, p, t, v, v, q))
    return np.stack((r, g, b)).astype(F32)


def jitter_tensor(img, prm):
    """ColorJitter.forward on a float32 [3, H, W] image in [0, 1] (functional_tensor)."""
    bf, cf, sf, hf = (float(x) for x in prm[1:5])
    c1, s1 = (float(x) for x in prm[9:11])
    for fn in prm[5:9].astype(int):
        if fn == 0:
            img = _blend(img, np.zeros_like(img), bf, 1.0 - bf)
        elif fn == 1:
            m = F32(_gray(img).mean(dtype=np.float64))
            img = _blend(img, m, cf, c1)
        elif fn == 2:
            img = _blend(img, _gray(img)[None], sf, s1)
        else:
            hsv = _rgb2hsv(img)
            h = (hsv[0] + F32(hf)).astype(F32)
            hsv[0] = h - np.floor(h)
            img = _hsv2rgb(hsv)
    return img


def augment_tensor(u8, params):
    """u8 [B, H, W, 3] uint8, params [B, 12] -> float32 [B, 3, H, W] in [-1, 1]."""
    out = []
    for im, prm in zip(u8, params):
        x = im.transpose(2, 0, 1).astype(F32) / F32(255.0)      # ToTensor (div by 255)
        if prm[0]:
            x = x[:, :, ::-1]                                     # hflip
        x = jitter_tensor(np.ascontiguousarray(x), prm)
        out.append(((x - F32(0.5)) / F32(0.5)).astype(F32))       # Normalize
    return np.stack(out)


def augment_pil(u8, params):
    """The reference's path: flip + the four ops on the PIL image, then ToTensor +
    Normalize (functional_pil.adjust_* as torchvision applies them)."""
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
                    np_h += np.array(hf * 255).astype(np.int64).astype(np.uint8)
                img = Image.merge("HSV", (Image.fromarray(np_h, "L"), s, v)).convert("RGB")
        x = np.asarray(img, F32).transpose(2, 0, 1) / F32(255.0)
        out.append((x - F32(0.5)) / F32(0.5))
    return np.stack(out)
