"""Seeded synthetic uint8 RGB images.

Low-frequency colour fields + flat rectangles + mild noise: spatial structure
keeps the synthetic-weight network's queries distinct (an i.i.d.-noise input
makes every position statistically identical). numpy only, so the same pixels
come out on the GPU box.
"""
from __future__ import annotations

import numpy as np


def _bilinear_up(low: np.ndarray, h: int, w: int) -> np.ndarray:
    lh, lw, _ = low.shape
    ys = (np.arange(h) + 0.5) * lh / h - 0.5
    xs = (np.arange(w) + 0.5) * lw / w - 0.5
    y0 = np.clip(np.floor(ys).astype(int), 0, lh - 1)
    x0 = np.clip(np.floor(xs).astype(int), 0, lw - 1)
    y1 = np.clip(y0 + 1, 0, lh - 1)
    x1 = np.clip(x0 + 1, 0, lw - 1)
    fy = np.clip(ys - y0, 0, 1)[:, None, None]
    fx = np.clip(xs - x0, 0, 1)[None, :, None]
    a = low[y0][:, x0]
    b = low[y0][:, x1]
    c = low[y1][:, x0]
    d = low[y1][:, x1]
    return (a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy


def synthetic_image(seed: int, h: int = 640, w: int = 640, flat: bool = False) -> np.ndarray:
    """uint8 HWC RGB image."""
    rng = np.random.default_rng(seed)
    if flat:
        return np.full((h, w, 3), int(rng.integers(0, 256)), dtype=np.uint8)
    low = rng.uniform(0, 255, (6, 6, 3))
    img = _bilinear_up(low, h, w)
    for _ in range(12):
        x0, y0 = int(rng.integers(0, max(1, w - 40))), int(rng.integers(0, max(1, h - 40)))
        ww, hh = int(rng.integers(20, max(21, w // 3))), int(rng.integers(20, max(21, h // 3)))
        img[y0:y0 + hh, x0:x0 + ww] = rng.uniform(0, 255, 3)
    img = img + rng.normal(0, 8, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


TEST_PIC_SEED = -1  # the reference's own fixture, tests/golden/test_pic.jpg
FLAT_GRAY_SEED = -2  # a constant mid-gray frame (SURVEY.md §8 D1.3 parity set)


def golden_source(seed: int, h: int, w: int, pic_path: str) -> np.ndarray:
    """The uint8 HWC source image a golden record names by (seed, h, w)."""
    if seed == TEST_PIC_SEED:
        from PIL import Image

        with Image.open(pic_path) as im:
            return np.asarray(im.convert("RGB"))
    if seed == FLAT_GRAY_SEED:
        return np.full((h, w, 3), 128, dtype=np.uint8)
    return synthetic_image(seed, h, w)


def synthetic_batch(n: int, h: int = 640, w: int = 640, seed0: int = 1234) -> np.ndarray:
    return np.stack([synthetic_image(seed0 + i, h, w) for i in range(n)])
