"""CPU: the JPEG encode step behind serve.py:139-142 (`image.save(buffer, format="JPEG")`, Pillow's libjpeg-turbo).

1. The numpy restatement (oracle/jpeg_enc_np.py) writes Pillow's bytes, byte for byte: odd and tiny sizes (MCU
   padding and dummy blocks), every Pillow subsampling, qualities 1..100, smooth and noise content, a comment,
   the reference's own test_pic.jpg decoded. That pins the oracle.
2. The library's host half (sp_jpeg_enc_plan + sp_jpeg_enc_finish: layout, quantisation tables, reciprocals,
   markers, 0xFF stuffing, padding), fed the oracle's raw code stream, writes the same bytes. The GPU half
   (the kernels) is checked against Pillow in tests/test_gpu_jpeg.py.
3. The rule that decides which save() calls take the GPU encoder.
"""
import ctypes as C
import io
import os

import numpy as np
import pytest
from PIL import Image

from oracle.jpeg_enc_np import coefficient_blocks, encode, entropy_bits
from spotter_amd.synthetic import synthetic_image

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg")


def pillow(img, comment=None, quality=-1, subsampling=-1):
    im = Image.fromarray(img)
    if comment:
        im.info["comment"] = comment
    kw = {}
    if quality != -1:
        kw["quality"] = quality
    if subsampling != -1:
        kw["subsampling"] = subsampling
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def _img(h, w, kind, seed):
    if kind == "noise" or min(h, w) < 2:
        return np.random.default_rng(seed).integers(0, 256, (h, w, 3), dtype=np.uint8)
    return synthetic_image(seed, h, w)


SIZES = [(1, 1), (2, 3), (8, 8), (9, 17), (16, 16), (17, 33), (24, 40), (31, 2), (40, 72), (123, 77)]


@pytest.mark.parametrize("hw", SIZES)
@pytest.mark.parametrize("sub", [-1, 0, 1, 2])
def test_oracle_writes_pillows_bytes(hw, sub):
    h, w = hw
    for kind in ("smooth", "noise"):
        img = _img(h, w, kind, h * 100 + w)
        for q in (-1, 1, 50, 95, 100):
            assert encode(img, q, sub) == pillow(img, quality=q, subsampling=sub), (hw, kind, q, sub)


def test_oracle_comment_and_reference_fixture():
    img = synthetic_image(3, 50, 60)
    assert encode(img, comment=b"spotter") == pillow(img, comment=b"spotter")
    ref = np.asarray(Image.open(GOLDEN).convert("RGB"))  # serve.py re-encodes exactly such a decoded image
    assert encode(ref) == pillow(ref)


def _finish(img, q=-1, sub=-1, comment=None):
    from spotter_amd._lib import SpJpegEncLayout, load

    L = load()
    comps, _ = coefficient_blocks(img, q, sub)
    raw, nbits = entropy_bits(comps, stuff=False)
    lay = SpJpegEncLayout()
    h, w, _ = img.shape
    assert L.sp_jpeg_enc_plan(w, h, q, sub, C.byref(lay)) == 0
    com = comment or b""
    cap = L.sp_jpeg_enc_max_bytes(C.byref(lay), nbits, len(com))
    out = C.create_string_buffer(cap)
    n = C.c_int64()
    assert L.sp_jpeg_enc_finish(C.byref(lay), raw, nbits, com, len(com), out, cap, C.byref(n)) == 0
    assert L.sp_jpeg_enc_finish(C.byref(lay), raw, nbits, com, len(com), out, 10, C.byref(n)) == -1  # too small
    return out.raw[:n.value], lay


@pytest.mark.parametrize("case", [((17, 33), -1, -1, None), ((64, 48), 90, 0, b"hi"), ((40, 72), 30, 1, None),
                                  ((1, 1), -1, -1, None), ((123, 77), 100, 2, b"x" * 300), ((9, 17), 1, 0, None)])
def test_host_half_writes_pillows_bytes(case):
    (h, w), q, sub, com = case
    img = _img(h, w, "smooth", 7)
    got, lay = _finish(img, q, sub, com)
    assert got == pillow(img, com, q, sub)
    assert lay.bpm == lay.h0 * lay.v0 + 2 and lay.total_blocks == lay.mcux * lay.mcuy * lay.bpm


def test_plan_refuses_what_it_does_not_encode():
    from spotter_amd._lib import SpJpegEncLayout, load

    L = load()
    lay = SpJpegEncLayout()
    for args in ((0, 10, -1, -1), (10, 70000, -1, -1), (10, 10, 0, -1), (10, 10, 101, -1), (10, 10, -1, 3),
                 (65501, 8, -1, -1), (8, 65501, -1, -1), (65535, 1, -1, -1)):
        assert L.sp_jpeg_enc_plan(*args, C.byref(lay)) == -1, args  # 65501+: libjpeg's JERR_IMAGE_TOO_BIG
    for args in ((65500, 8, -1, -1), (8, 65500, -1, -1)):  # JPEG_MAX_DIMENSION itself is encodable
        assert L.sp_jpeg_enc_plan(*args, C.byref(lay)) == 0, args


def test_which_saves_take_the_gpu_encoder():
    """DeviceRGBImage.save → GPU only where Pillow's JpegImagePlugin._save would write exactly those bytes."""
    from spotter_amd.jpeg import _gpu_jpeg_options

    im = Image.new("RGB", (8, 8))
    buf = io.BytesIO()
    assert _gpu_jpeg_options(im, buf, "JPEG", {}) == (-1, -1, None)
    assert _gpu_jpeg_options(im, buf, "jpeg", {"quality": 90, "subsampling": "4:4:4"}) == (90, 0, None)
    im.info["comment"] = b"c"
    assert _gpu_jpeg_options(im, buf, "JPEG", {}) == (-1, -1, b"c")
    for fmt, params in (("PNG", {}), (None, {}), ("JPEG", {"optimize": True}), ("JPEG", {"progressive": True}),
                        ("JPEG", {"dpi": (72, 72)}), ("JPEG", {"quality": "web_high"}), ("JPEG", {"quality": 0}),
                        ("JPEG", {"exif": b"Exif"}), ("JPEG", {"subsampling": "keep"})):
        assert _gpu_jpeg_options(im, buf, fmt, params) is None, (fmt, params)
    assert _gpu_jpeg_options(im, "out.jpg", "JPEG", {}) is None  # file names: Pillow's save
    assert _gpu_jpeg_options(Image.new("L", (8, 8)), buf, "JPEG", {}) is None
    # above libjpeg's JPEG_MAX_DIMENSION Pillow's save raises JERR_IMAGE_TOO_BIG: that save stays Pillow's
    assert _gpu_jpeg_options(Image.new("RGB", (65500, 1)), buf, "JPEG", {}) == (-1, -1, None)
    for size in ((65501, 1), (1, 65501)):
        assert _gpu_jpeg_options(Image.new("RGB", size), buf, "JPEG", {}) is None
