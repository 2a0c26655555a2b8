"""TEST INFRASTRUCTURE ONLY (the parity checker, never the product path): CPU restatement of the
reference's image transform, Resize((224, 224)) -> ToTensor -> Normalize(mean, std)
(models/attention.py:296-301, applied per image at dataset.py:55-59).

torchvision's Resize on a PIL image calls Image.resize(size, BILINEAR); the arithmetic is
Pillow's (src/libImaging/Resample.c; Pillow is present in this image, torchvision is not): per
output index, precompute_coeffs (antialiasing triangle filter, support max(1, in/out), weights
normalised in double), normalize_coeffs_8bpc (22-bit fixed point), a horizontal pass rounded to
uint8, then a vertical pass rounded to uint8. Pinned bit-exactly to the installed Pillow by
tests/test_image_cpu.py; the GPU kernel (csrc/image.hip) is compared to both.
"""
import math

import numpy as np

PREC = 22
MEAN = (0.485, 0.456, 0.406)
STD = (0.229, 0.224, 0.225)


def coeffs(in_size, out_size):
    """(xmin[out], taps[out], k[out][ksize] int) as Pillow's precompute + normalize_coeffs_8bpc."""
    scale = float(np.float32(in_size)) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xmins, ns, ks = [], [], np.zeros((out_size, ksize), np.int64)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            v = 1.0 - t if t < 1.0 else 0.0
            w.append(v)
            ww += v
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            ks[xx, x] = int(-0.5 + v * (1 << PREC)) if v < 0 else int(0.5 + v * (1 << PREC))
        xmins.append(xmin)
        ns.append(xmax)
    return np.array(xmins), np.array(ns), ks


def _pass(img, axis, out_size):
    """One separable pass along `axis` (1 = width, 0 = height) of an (H, W, 3) uint8 image."""
    xmin, n, k = coeffs(img.shape[axis], out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)          # (in, other, 3)
    out = np.empty((out_size,) + src.shape[1:], np.int64)
    for o in range(out_size):
        acc = np.full(src.shape[1:], 1 << (PREC - 1), np.int64)
        for i in range(n[o]):
            acc += src[xmin[o] + i] * k[o, i]
        out[o] = np.clip(acc >> PREC, 0, 255)
    return np.moveaxis(out, 0, axis).astype(np.uint8)


def resize_bilinear(img, size):
    """Image.resize((W, H), BILINEAR) of an (H, W, 3) uint8 array -> (H', W', 3) uint8."""
    oh, ow = size
    return _pass(_pass(img, 1, ow), 0, oh)


def transform(img, size=(224, 224)):
    """The reference transform -> (3, H', W') float32 (ToTensor: u8 / 255, Normalize in fp32)."""
    r = resize_bilinear(img, size).astype(np.float32) / np.float32(255)
    m = np.array(MEAN, np.float32).reshape(1, 1, 3)
    s = np.array(STD, np.float32).reshape(1, 1, 3)
    return ((r - m) / s).transpose(2, 0, 1).copy()
