"""TEST INFRASTRUCTURE ONLY — integer restatement of the preprocess.

The reference preprocess is `processor(images=image, return_tensors="pt")`
(serve.py:98) → RTDetrImageProcessorPil._preprocess: resize to 640×640 with
PIL BILINEAR (IPP:451-459 → IT:367 `image.resize((w, h), resample,
reducing_gap=None)`), then `rescale` = f32(f64(u8) * (1/255)) (IT:118-122),
HWC→CHW, no normalize, no pad (IPP:129-143). Pillow (pinned 11.1.0,
uv.lock:582-583; 12.2.0 here) resamples in libImaging/Resample.c: separable
triangle filter with support max(in/out, 1), horizontal pass first over only
the source rows the vertical pass uses, 22-bit fixed-point coefficients,
`clip8(2^21 + Σ px·k) >> 22` after each pass. Restated here in numpy; pinned
bit-exactly against Pillow by tests/test_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np

PRECISION_BITS = 32 - 8 - 2


def precompute_coeffs(in_size: int, out_size: int):
    """(bounds [out,2] = (xmin, n), int32 coeffs [out, ksize]) — Resample.c precompute_coeffs."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = int(center - support + 0.5)
        if xmin < 0:
            xmin = 0
        xmax = int(center + support + 0.5)
        if xmax > in_size:
            xmax = in_size
        n = xmax - xmin
        ws = []
        for x in range(n):
            t = abs((x + xmin - center + 0.5) * ss)
            ws.append(1.0 - t if t < 1.0 else 0.0)
        tot = sum(ws)
        for x in range(n):
            w = ws[x] / tot if tot != 0.0 else ws[x]
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS))
        bounds[xx] = (xmin, n)
    return bounds, kk


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def resize_bilinear_u8(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """img uint8 [H,W,C] → uint8 [out_h,out_w,C], bit-exact with PIL Image.resize(BILINEAR)."""
    h, w, c = img.shape
    if (h, w) == (out_h, out_w):
        return img.copy()  # Image.resize returns a copy when the size is unchanged
    hb, hk = precompute_coeffs(w, out_w)
    vb, vk = precompute_coeffs(h, out_h)
    need_h = w != out_w
    need_v = h != out_h
    src = img.astype(np.int64)
    if need_h:
        y0 = int(vb[0, 0])
        y1 = int(vb[-1, 0] + vb[-1, 1])
        rows = src[y0:y1]
        acc = np.full((y1 - y0, out_w, c), 1 << (PRECISION_BITS - 1), np.int64)
        for j in range(hk.shape[1]):
            xi = np.minimum(hb[:, 0] + j, w - 1)
            kj = np.where(j < hb[:, 1], hk[:, j], 0).astype(np.int64)
            acc += rows[:, xi, :] * kj[None, :, None]
        tmp = _clip8(acc).astype(np.int64)
        vb = vb.copy()
        vb[:, 0] -= y0
    else:
        tmp = src
    if not need_v:
        return tmp.astype(np.uint8)
    acc = np.full((out_h, tmp.shape[1], c), 1 << (PRECISION_BITS - 1), np.int64)
    for j in range(vk.shape[1]):
        yi = np.minimum(vb[:, 0] + j, tmp.shape[0] - 1)
        kj = np.where(j < vb[:, 1], vk[:, j], 0).astype(np.int64)
        acc += tmp[yi, :, :] * kj[:, None, None]
    return _clip8(acc)


RESCALE_LUT = (np.arange(256, dtype=np.float64) * (1 / 255)).astype(np.float32)


def preprocess(img: np.ndarray, size=(640, 640)) -> np.ndarray:
    """uint8 HWC → f32 [3, H, W] exactly as the HF PIL processor's pixel_values[0]."""
    r = resize_bilinear_u8(img, size[0], size[1])
    return np.ascontiguousarray(RESCALE_LUT[r].transpose(2, 0, 1))
