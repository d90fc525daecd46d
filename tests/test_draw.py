"""CPU: the label drawing of serve.py:119-137 through the drop-in's ImageDraw (spotter_amd/draw.py) draws exactly
Pillow's pixels: the memoised glyph masks of the default font equal fresh renders for every amenity string
(serve.py:31-59) over dense grids of fractional start positions, class boundaries included, and whole
images with many labels drawn both ways are identical."""
import numpy as np
import pytest
from PIL import Image, ImageDraw, ImageFont

AMENITY_TEXTS = sorted({"refrigerator", "oven", "microwave", "sink", "dining area", "toaster", "kitchen", "TV",
                        "sofa", "chair", "bed", "bathroom", "hair dryer", "workspace", "parking"})


def _sig(m):
    mask, off = m
    return bytes(mask), mask.size, tuple(off)


def test_memoised_masks_equal_fresh_renders():
    from spotter_amd.draw import _UPPER_X, _UPPER_Y, memo_default_font

    memo = memo_default_font()
    fresh = ImageFont.load_default()
    rng = np.random.default_rng(0)
    fr = list(rng.random(60)) + [0.0, 1e-9, 1e-6, 2e-5, 0.25, 0.5, 0.999999]
    for u in (_UPPER_X, _UPPER_Y):
        fr += [u - 1e-4, u - 2e-5, u - 2e-6, u, u + 2e-6, u + 2e-5, u + 1e-4]
    for text in AMENITY_TEXTS:
        for sw in (0, 1):
            for fx in fr:
                fy = float(rng.choice(fr))
                for start in ((fx, fy), (fy, fx)):
                    kw = dict(direction=None, features=None, language=None, stroke_width=sw, stroke_filled=True,
                              anchor="la", ink=255 if sw == 0 else 0, start=start)
                    assert _sig(memo.getmask2(text, "L", **kw)) == _sig(fresh.getmask2(text, "L", **kw)), \
                        (text, sw, start)
    assert memo.memo_stats["hits"] > 1000 and not memo._no_memo


def test_draw_shim_draws_pillows_pixels():
    """The serve.py draw loop (rectangle width 3 + text with a 1-px black stroke) with 40 labels at random float
    boxes, some partly outside the image and at negative coordinates, via both ImageDraw modules."""
    from spotter_amd.draw import draw_module

    import os

    golden = os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg")
    base = Image.open(golden).convert("RGB")
    rng = np.random.default_rng(1)
    shim = draw_module()
    for rep in range(3):  # the memo warms up over the repetitions
        a, b = base.copy(), base.copy()
        da, db = ImageDraw.Draw(a), shim.Draw(b)
        for _ in range(40):
            x0, y0 = rng.uniform(-50, 1150), rng.uniform(-50, 680)
            box = [x0, y0, x0 + rng.uniform(5, 400), y0 + rng.uniform(5, 300)]
            text = str(rng.choice(AMENITY_TEXTS))
            for d in (da, db):
                d.rectangle(box, outline="red", width=3)
                d.text(xy=(box[0] + 5, box[1] + 5), text=text, fill="white", stroke_width=1, stroke_fill="black")
        assert np.array_equal(np.asarray(a), np.asarray(b)), rep
    assert shim.Draw(b).font.memo_stats["hits"] > 50


def test_draw_module_is_pillows_otherwise():
    from spotter_amd.draw import draw_module

    shim = draw_module()
    assert shim.ImageDraw is ImageDraw.ImageDraw and shim.floodfill is ImageDraw.floodfill
    im = Image.new("RGB", (20, 20))
    d = shim.Draw(im)
    assert isinstance(d, ImageDraw.ImageDraw)
    own = ImageFont.load_default()
    d2 = shim.Draw(im)
    d2.font = own  # a caller's own font is used as is
    d2.text((1, 1), "x", font=own)
    with pytest.raises(TypeError):
        shim.Draw()


def test_exact_repeats_are_cached_and_bounded():
    """A render at exactly the same (string, options, start) is served again from the bounded exact cache, also
    for starts the class memo does not use (a fraction next to a class boundary); the cache keeps at most
    EXACT_CAP entries."""
    from spotter_amd.draw import _UPPER_X, _MemoFont

    f = ImageFont.load_default()
    f.__class__ = _MemoFont
    f._memo_init()
    f.EXACT_CAP = 8
    fresh = ImageFont.load_default()
    kw = dict(direction=None, features=None, language=None, stroke_width=1, stroke_filled=True, anchor="la", ink=0)
    for start in ((3.25, 7.5), (2.0 + _UPPER_X, 1e-9)):  # a class-memo key, then a bypassed start
        a = f.getmask2("sofa", "L", start=start, **kw)
        b = f.getmask2("sofa", "L", start=start, **kw)
        assert b is a and _sig(a) == _sig(fresh.getmask2("sofa", "L", start=start, **kw))
    assert f.memo_stats["exact_hits"] == 2
    for i in range(20):  # distinct strings: no class-memo hits, every render enters the exact cache
        f.getmask2(f"bed {i}", "L", start=(0.3, 0.3), **kw)
    assert len(f._exact) == 8 and ("bed 19", "L", 0.3, 0.3) == next(reversed(f._exact))[:4]


def test_embedded_color_text_is_never_served_from_the_memo():
    """ImageDraw.text(embedded_color=True) on an RGBA image asks for an "RGBA" mask and Pillow then writes the
    ink alpha into that mask in place (color.fillband): a cached mask would be changed under the memo. Such
    renders bypass both caches, so repeated and differently coloured labels draw Pillow's pixels."""
    from spotter_amd.draw import draw_module

    shim = draw_module()
    a, b = Image.new("RGBA", (160, 60), (10, 20, 30, 255)), Image.new("RGBA", (160, 60), (10, 20, 30, 255))
    da, db = ImageDraw.Draw(a), shim.Draw(b)
    for i, fill in enumerate(("white", (255, 0, 0, 128), "white", (0, 255, 0, 40))):
        for d in (da, db):
            d.text(xy=(5.25, 5 + 12 * i), text="sofa", fill=fill, embedded_color=True)
            d.text(xy=(5.25, 5 + 12 * i), text="sofa", fill=fill, embedded_color=True, stroke_width=1,
                   stroke_fill="black")
        assert np.array_equal(np.asarray(a), np.asarray(b)), i
    assert not any(k[1] == "RGBA" for k in shim.Draw(b).font._exact)
