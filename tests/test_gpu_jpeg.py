"""GPU: the JPEG decode step (sp_jpeg_to_rgb + the host entropy decoder) against Pillow's own decode, bit for
bit, and the serve.py drop-in around it (spotter_amd.jpeg.open_image → SpotterImageProcessor)."""
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
from PIL import Image, ImageDraw  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg")


def _jpeg(img, mode="RGB", **kw):
    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, "JPEG", **kw)
    return b.getvalue()


def _cases():
    from spotter_amd.synthetic import synthetic_image

    yield "test_pic", open(GOLDEN, "rb").read()
    for (h, w) in [(1, 1), (2, 3), (17, 33), (233, 177), (480, 640), (720, 1280)]:
        img = synthetic_image(h * 7 + w, h, w) if min(h, w) >= 2 else np.full((h, w, 3), 77, np.uint8)
        for sub in (0, 1, 2):
            for prog in (False, True):
                yield f"{h}x{w} sub{sub} prog{int(prog)}", _jpeg(img, quality=90, subsampling=sub, progressive=prog)
    yield "gray", _jpeg(synthetic_image(3, 45, 61), mode="L", quality=85)
    yield "restart", _jpeg(synthetic_image(5, 123, 77), quality=80, restart_marker_rows=1, subsampling=2)


@pytest.fixture(scope="module")
def dev():
    from spotter_amd._lib import lib

    assert lib().sp_device_init(0) == 0, lib().sp_last_error()
    return torch.device("cuda", 0)


def test_gpu_decode_matches_pillow(dev):
    from spotter_amd.jpeg import JpegDecoder

    d = JpegDecoder(dev)
    n = 0
    for name, data in _cases():
        got = d.decode(data).cpu().numpy()
        ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
        assert got.shape == ref.shape, name
        bad = np.argwhere(got != ref)
        assert bad.size == 0, f"{name}: {len(bad)} samples differ, first at {bad[:3].tolist()}"
        n += 1
    assert n > 30


def test_open_image_is_a_lazy_pil_image(dev):
    """open_image(bytes) → DeviceRGBImage: size / mode without a sync, convert("RGB") stays lazy, the host
    pixels (np.asarray, ImageDraw, JPEG save — serve.py's draw / encode tail) equal Pillow's decode; PNG
    bytes take the reference's Image.open."""
    from spotter_amd.jpeg import DeviceRGBImage, open_image

    data = open(GOLDEN, "rb").read()
    ref = Image.open(io.BytesIO(data)).convert("RGB")
    with open_image(data) as raw:
        assert isinstance(raw, DeviceRGBImage)
        im = raw.convert("RGB")
        assert isinstance(im, DeviceRGBImage) and im.size == ref.size and im.mode == "RGB"
        assert np.array_equal(np.asarray(im), np.asarray(ref))
        d1, d2 = ImageDraw.Draw(im), ImageDraw.Draw(ref)
        for d in (d1, d2):
            d.rectangle([10, 10, 200, 100], outline="red", width=3)
        assert np.array_equal(np.asarray(im), np.asarray(ref))
        b, b2 = io.BytesIO(), io.BytesIO()
        im.save(b, format="JPEG")  # drawn on: the host pixels go up to the GPU encoder
        ref.save(b2, format="JPEG")
        assert b.getvalue() == b2.getvalue()
    p = io.BytesIO()
    ref.save(p, "PNG")
    other = open_image(p.getvalue())
    assert not isinstance(other, DeviceRGBImage) and other.convert("RGB").size == ref.size


def test_processor_reads_the_device_image_in_place(dev):
    """processor(images=open_image(bytes)) gives the same pixel_values as processor(images=Pillow's decode),
    bit for bit, for the reference fixture and a 4:2:0 progressive JPEG, alone and batched with a PIL image."""
    from spotter_amd import SpotterImageProcessor
    from spotter_amd.jpeg import open_image
    from spotter_amd.synthetic import synthetic_image

    proc = SpotterImageProcessor()
    datas = [open(GOLDEN, "rb").read(), _jpeg(synthetic_image(11, 480, 800), quality=88, subsampling=2,
                                             progressive=True)]
    for data in datas:
        with open_image(data) as raw:
            im = raw.convert("RGB")
            a = proc(images=im)["pixel_values"]
            assert getattr(im, "_im", None) is None  # the processor never pulled the host pixels
        b = proc(images=Image.open(io.BytesIO(data)).convert("RGB"))["pixel_values"]
        assert torch.equal(a, b)
    mix = proc(images=[open_image(datas[0]).convert("RGB"), Image.open(io.BytesIO(datas[1])).convert("RGB")])
    ref = proc(images=[Image.open(io.BytesIO(x)).convert("RGB") for x in datas])
    assert torch.equal(mix["pixel_values"], ref["pixel_values"])


def test_gpu_path_on_the_corrupt_corpus(dev):
    """The ~1700 malformed files of tests/jpeg_corpus.py through the drop-in Image.open: each one either comes
    back GPU-decoded with exactly Pillow's pixels, or is Pillow's own image (the GPU path declined: parser
    rejection, or the IDCT kernel's status flag for coefficients outside the range shared with libjpeg-turbo's
    SIMD code), or raises what Pillow's Image.open raises. The flag must fire on the files the oracle puts
    outside that range."""
    import sys
    import warnings

    sys.path.insert(0, os.path.dirname(__file__))
    from jpeg_corpus import corpus

    from oracle.jpeg_np import simd_envelope_ok
    from spotter_amd.jpeg import DeviceRGBImage, JpegDecoder, UnsupportedJpeg, decode_coefs, image_module, layout_dict

    shim = image_module(dev)
    d = JpegDecoder(dev)
    gpu = flagged = 0
    for lab, data in corpus():
        try:
            lay, co = decode_coefs(data)
            inside = simd_envelope_ok(co, layout_dict(lay))
        except UnsupportedJpeg:
            lay = None
        if lay is not None:
            try:
                d.decode(data)
                assert inside, lab
            except UnsupportedJpeg:
                assert not inside, lab
                flagged += 1
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            try:
                ref_im = Image.open(io.BytesIO(data))
            except Exception as e:  # noqa: BLE001 - whatever Pillow raises, the shim raises too
                with pytest.raises(type(e)):
                    shim.open(io.BytesIO(data))
                continue
            im = shim.open(io.BytesIO(data))
            if isinstance(im, DeviceRGBImage):
                gpu += 1
                ref = np.asarray(ref_im.convert("RGB"))
                assert np.array_equal(np.asarray(im.convert("RGB")), ref), lab
            else:
                assert type(im) is type(ref_im), lab
    assert gpu >= 100 and flagged >= 5, (gpu, flagged)


def _pillow_jpeg(img, comment=None, **kw):
    im = Image.fromarray(img)
    if comment:
        im.info["comment"] = comment
    b = io.BytesIO()
    im.save(b, "JPEG", **kw)
    return b.getvalue()


def test_gpu_encode_writes_pillows_bytes(dev):
    """sp_jpeg_enc_rgb + the host finish against Pillow's own save, byte for byte: the reference fixture decoded
    (what serve.py re-encodes), synthetic 640², 720p and 1080p frames, odd sizes (dummy blocks), noise, every
    subsampling, qualities 1..100, a comment; from a device tensor (RGB) and from host pixels (RGBX / RGB)."""
    from spotter_amd.jpeg import JpegEncoder
    from spotter_amd.synthetic import synthetic_image

    enc = JpegEncoder(dev)
    ref_img = np.asarray(Image.open(GOLDEN).convert("RGB"))
    cases = [("test_pic", ref_img, {}), ("640", synthetic_image(1, 640, 640), {}),
             ("720p", synthetic_image(2, 720, 1280), {}), ("1080p", synthetic_image(3, 1080, 1920), {})]
    rng = np.random.default_rng(0)
    for (h, w) in [(1, 1), (2, 3), (9, 17), (17, 33), (31, 2), (123, 77), (233, 177)]:
        img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8) if min(h, w) < 4 else synthetic_image(h + w, h, w)
        for q in (-1, 1, 50, 100):
            for sub in (-1, 0, 1, 2):
                cases.append((f"{h}x{w} q{q} s{sub}", img, {"quality": q, "subsampling": sub}))
    noise = rng.integers(0, 256, (96, 80, 3), dtype=np.uint8)
    cases += [("noise q100", noise, {"quality": 100}), ("noise q1", noise, {"quality": 1})]
    for name, img, kw in cases:
        pkw = {k: v for k, v in kw.items() if v != -1}
        want = _pillow_jpeg(img, **pkw)
        t = torch.from_numpy(np.ascontiguousarray(img)).to(dev)
        got = enc.encode(t, kw.get("quality", -1), kw.get("subsampling", -1))
        assert got == want, f"{name}: {len(got)} vs {len(want)} bytes"
        if name in ("test_pic", "640") or "q-1 s-1" in name:
            assert enc.encode(Image.fromarray(img)) == want, name  # host pixels (Arrow RGBX or packed RGB)
    img = synthetic_image(9, 50, 60)
    t = torch.from_numpy(img).to(dev)
    assert enc.encode(t, comment=b"spotter") == _pillow_jpeg(img, comment=b"spotter")
    big = Image.fromarray(synthetic_image(5, 2160, 3840))  # several Pillow memory blocks: packed-RGB upload
    assert enc.encode(big) == _pillow_jpeg(np.asarray(big))


def test_serve_tail_with_the_drop_in_image_module(dev):
    """serve.py:96-142 as the unchanged class runs it after the drop-in: Image.open (module shim) → convert →
    draw → save(format="JPEG") → base64 gives the reference's exact base64 string; without a draw the encoder
    reads the device copy (no host pixels pulled)."""
    import base64

    from spotter_amd.jpeg import DeviceRGBImage, image_module

    Img = image_module(dev)
    data = open(GOLDEN, "rb").read()
    for draw in (True, False):
        with Img.open(io.BytesIO(data)) as raw, Image.open(io.BytesIO(data)) as raw_ref:
            image, ref = raw.convert("RGB"), raw_ref.convert("RGB")
            assert isinstance(image, DeviceRGBImage)
            if draw:
                for im in (image, ref):
                    d = ImageDraw.Draw(im)
                    d.rectangle([100.5, 80.25, 400.75, 300.0], outline="red", width=3)
                    d.text(xy=(105.5, 85.25), text="dining area", fill="white", stroke_width=1, stroke_fill="black")
            outs = []
            for im in (image, ref):
                b = io.BytesIO()
                im.save(b, format="JPEG")
                outs.append(base64.b64encode(b.getvalue()).decode("utf-8"))
            assert outs[0] == outs[1]
            assert (getattr(image, "_im", None) is None) == (not draw)
