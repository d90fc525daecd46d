"""CPU: the JPEG decode step in front of A1 (serve.py:96-97, Pillow's libjpeg-turbo decode).

The library's host entropy decoder (sp_jpeg_decode_coefs: baseline + progressive Huffman, restart markers)
feeds the numpy restatement of libjpeg-turbo's pixel pipeline (oracle/jpeg_np.py: ISLOW IDCT, fancy
upsampling, YCbCr→RGB); the result must equal Pillow's own `Image.open(..).convert("RGB")` bit for bit.
That pins both halves against the reference's decoder here; tests/test_gpu_kernels.py then checks the GPU
kernels (sp_jpeg_to_rgb) against Pillow directly. No device call: sp_jpeg_decode_coefs is host code.
"""
import io

import numpy as np
import pytest
from PIL import Image

from oracle.jpeg_np import to_rgb
from spotter_amd.synthetic import synthetic_image

GOLDEN = __import__("os").path.join(__import__("os").path.dirname(__file__), "golden", "test_pic.jpg")


def _jpeg(img, mode="RGB", **kw):
    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, "JPEG", **kw)
    return b.getvalue()


def _check(data):
    from spotter_amd.jpeg import decode_coefs, layout_dict

    lay, co = decode_coefs(data)
    got = to_rgb(co, layout_dict(lay))
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
    assert got.shape == ref.shape
    bad = np.argwhere(got != ref)
    assert bad.size == 0, f"{len(bad)} samples differ, first at {bad[:3].tolist()}"
    return layout_dict(lay)


def test_reference_fixture_progressive():
    """The reference's own test image (apps/spotter/tests/spotter/test_data/test_pic.jpg): a progressive
    (spectral-selection) 4:4:4 JPEG, 1200×717."""
    lay = _check(open(GOLDEN, "rb").read())
    assert lay["progressive"] == 1 and (lay["width"], lay["height"]) == (1200, 717)


SIZES = [(1, 1), (2, 3), (8, 8), (9, 17), (17, 33), (31, 2), (64, 48), (233, 177)]


@pytest.mark.parametrize("hw", SIZES)
@pytest.mark.parametrize("sub", [0, 1, 2])  # Pillow's 4:4:4, 4:2:2, 4:2:0
@pytest.mark.parametrize("prog", [False, True])
def test_decode_matches_pillow(hw, sub, prog):
    """Baseline and progressive (Pillow's default script: spectral selection + successive approximation,
    i.e. DC / AC first and refinement scans), every Pillow subsampling, odd and tiny sizes (the box
    upsampling of downsampled widths <= 2 and the edge-row replication), two qualities."""
    h, w = hw
    img = synthetic_image(h * 1000 + w, h, w) if min(h, w) >= 2 else np.random.default_rng(h).integers(
        0, 256, (h, w, 3), dtype=np.uint8)
    for q in (50, 95):
        lay = _check(_jpeg(img, quality=q, subsampling=sub, progressive=prog))
        assert lay["progressive"] == int(prog)
        if sub == 2 and min(h, w) > 1:
            assert (lay["max_h"], lay["max_v"]) == (2, 2)


@pytest.mark.parametrize("prog", [False, True])
def test_grayscale(prog):
    img = synthetic_image(3, 45, 61)
    lay = _check(_jpeg(img, mode="L", quality=85, progressive=prog))
    assert lay["ncomp"] == 1 and lay["color"] == 0


@pytest.mark.parametrize("kw", [dict(restart_marker_blocks=3), dict(restart_marker_rows=1),
                                dict(restart_marker_blocks=1, progressive=True),
                                dict(restart_marker_rows=2, subsampling=2, progressive=True)])
def test_restart_markers(kw):
    _check(_jpeg(synthetic_image(5, 123, 77), quality=80, **kw))


def test_flat_and_extreme_content():
    """A constant frame and saturated noise (IDCT range-limit wrap and clamps)."""
    _check(_jpeg(np.full((40, 56, 3), 128, np.uint8), quality=90))
    rng = np.random.default_rng(7)
    noise = np.where(rng.random((48, 64, 3)) < 0.5, 0, 255).astype(np.uint8)
    for q in (10, 100):
        _check(_jpeg(noise, quality=q, subsampling=2))


def test_unsupported_forms_raise():
    """Forms outside the decoder (CMYK, PNG bytes, truncated headers) raise UnsupportedJpeg / RuntimeError
    instead of producing pixels; open_image keeps the reference's Image.open for them."""
    from spotter_amd.jpeg import UnsupportedJpeg, decode_coefs

    b = io.BytesIO()
    Image.fromarray(synthetic_image(1, 16, 16)).convert("CMYK").save(b, "JPEG")
    with pytest.raises(UnsupportedJpeg):
        decode_coefs(b.getvalue())
    p = io.BytesIO()
    Image.fromarray(synthetic_image(1, 16, 16)).save(p, "PNG")
    with pytest.raises(UnsupportedJpeg):
        decode_coefs(p.getvalue())
    data = open(GOLDEN, "rb").read()
    with pytest.raises((UnsupportedJpeg, RuntimeError)):
        decode_coefs(data[:100])


def _with_frame_size(data: bytes, w: int, h: int) -> bytes:
    """The JPEG with its SOF0 header's height / width fields rewritten."""
    i = data.index(b"\xff\xc0")
    b = bytearray(data)
    b[i + 5:i + 9] = bytes([h >> 8, h & 255, w >> 8, w & 255])
    return bytes(b)


@pytest.mark.parametrize("w,h", [(65501, 8), (8, 65501), (65535, 65535)])
def test_frames_above_libjpegs_max_dimension_are_left_to_pillow(w, h):
    """libjpeg's JPEG_MAX_DIMENSION (65500, jmorecfg.h): jdinput.c raises JERR_IMAGE_TOO_BIG above it, so the
    strict parser refuses such frames at the header and the file goes to Pillow, which raises as
    the reference does. 65500 itself passes the header check (this file then fails later: its data is 8×8)."""
    from spotter_amd.jpeg import UnsupportedJpeg, decode_coefs

    data = _jpeg(synthetic_image(4, 8, 8), quality=90)
    with pytest.raises(UnsupportedJpeg, match="wider or higher than 65500"):
        decode_coefs(_with_frame_size(data, w, h))
    with pytest.raises((UnsupportedJpeg, RuntimeError)) as e:
        decode_coefs(_with_frame_size(data, min(w, 65500), min(h, 65500)))
    assert "wider or higher" not in str(e.value)


def test_truncated_or_corrupt_data_is_left_to_pillow():
    """Entropy-coded data cut short, or a file without its EOI: Pillow raises ("image file is truncated")
    or applies its own LOAD_TRUNCATED_IMAGES policy, which is not libjpeg arithmetic — the decoder reports
    UnsupportedJpeg for these, so open_image gives the file to the reference's own Image.open."""
    from spotter_amd.jpeg import UnsupportedJpeg, decode_coefs

    for kw in (dict(), dict(subsampling=2), dict(progressive=True), dict(restart_marker_rows=1)):
        data = _jpeg(synthetic_image(9, 64, 64), quality=90, **kw)
        for frac in (0.5, 0.8, 0.999):
            with pytest.raises(UnsupportedJpeg):
                decode_coefs(data[: int(len(data) * frac)])
        with pytest.raises(UnsupportedJpeg):
            decode_coefs(data[:-2])  # no EOI
        _check(data)
