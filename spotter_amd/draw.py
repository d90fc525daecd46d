"""The label drawing of serve.py:119-137 (`ImageDraw.Draw(image)`, `draw.rectangle`, `draw.text`), kept on the
host in Pillow's own code, with one change: the default font's glyph masks are memoised.

Measured on the MI355X box's EPYC host (tools/detect_path.py, profiles/r5/jpeg/): drawing the 16 labels of a
/detect response takes 6.3 ms, nearly all of it FreeType rendering the same few strings (the amenity names of
serve.py:31-59) again and again: `ImageDraw.text` with `stroke_width=1` renders each label twice through
`FreeTypeFont.getmask2` (stroke, then fill), ~0.2 ms each, and the result depends on the string, the stroke,
the ink and — through the hinted 26.6 fixed-point origin — only on which of three classes each fractional
start coordinate falls in: exactly 0, (0, u), [u, 1) with u = 31.5/64 for x and 32.5/64 for y. `Draw(im)`
here is Pillow's ImageDraw with its default font replaced by the same font whose getmask2 keeps the masks per
(string, options, start class).

Exactness: a key is served from the memo only after two renders at *different* start fractions of its class
gave identical masks (a key whose masks differ is never memoised again); fractions within 1e-5 of a class
boundary, negative fractions and every non-default option are rendered by Pillow as before. A render at
exactly the same start (string, options and both start coordinates equal) is also served again from a bounded
cache (`EXACT_CAP` entries, least recently used out): the same inputs, so the same mask. The masks are pure
functions of those inputs, and draw_bitmap then composites them exactly as Pillow does, so the drawn pixels
are Pillow's (tests/test_draw.py: all amenity strings over dense start grids; the whole serve.py tail
byte-identical on the GPU box).
"""
from __future__ import annotations

import threading
import types
from collections import OrderedDict

from PIL import ImageDraw as _PILDraw
from PIL import ImageFont as _PILFont

# the hinted origin moves to the next pixel from these fractions on (26.6 fixed point; y points down in the
# image and up in FreeType, hence the different half-way point)
_UPPER_X = 31.5 / 64
_UPPER_Y = 32.5 / 64
_EPS = 1e-5


def start_class(f: float, upper: float):
    """The start-offset class of a fractional coordinate, or None where the memo is not used."""
    if f == 0.0:
        return 0
    if f < _EPS or f >= 1.0 or abs(f - upper) < _EPS:
        return None
    return 1 if f < upper else 2


class _MemoFont(_PILFont.FreeTypeFont):
    """Pillow's default FreeType font (ImageFont.load_default()) with memoised getmask2."""

    EXACT_CAP = 4096  # renders kept for an exact repeat of (string, options, start)

    def _memo_init(self):
        self._memo_lock = threading.Lock()
        self._memo: dict = {}        # key -> (mask, offset) once verified
        self._pending: dict = {}     # key -> (start pair, mask signature) of its first render
        self._no_memo: set = set()
        self._exact: OrderedDict = OrderedDict()  # (string, options, exact start) -> (mask, offset)
        self.memo_stats = {"hits": 0, "exact_hits": 0, "renders": 0, "bypass": 0}

    def _exact_put(self, ekey, val):
        with self._memo_lock:
            self._exact[ekey] = val
            if len(self._exact) > self.EXACT_CAP:
                self._exact.popitem(last=False)

    def getmask2(self, text, mode="", *args, start=None, **kwargs):
        if mode not in ("", "L", "1"):
            # "RGBA" (ImageDraw.text(embedded_color=True)): Pillow fills the returned mask's alpha band in place
            # (color.fillband), so a shared cached mask would be overwritten; these renders are never cached
            self.memo_stats["bypass"] += 1
            return super().getmask2(text, mode, *args, start=start, **kwargs)
        key = ekey = None
        if not args and isinstance(text, str) and start is not None:
            try:
                opts = tuple(sorted((k, tuple(v) if isinstance(v, list) else v) for k, v in kwargs.items()))
                sx, sy = float(start[0]), float(start[1])
                ekey = (text, mode, sx, sy, opts)
                hash(ekey)
            except (TypeError, ValueError, IndexError):
                ekey = None
            if ekey is not None:
                cx, cy = start_class(sx, _UPPER_X), start_class(sy, _UPPER_Y)
                if cx is not None and cy is not None:
                    key = (text, mode, cx, cy, opts)
        if ekey is not None:
            with self._memo_lock:
                hit = self._exact.get(ekey)
                if hit is not None:
                    self._exact.move_to_end(ekey)
            if hit is not None:
                self.memo_stats["exact_hits"] += 1
                return hit
        if key is None or key in self._no_memo:
            self.memo_stats["bypass"] += 1
            out = super().getmask2(text, mode, *args, start=start, **kwargs)
            if ekey is not None:
                self._exact_put(ekey, out)
            return out
        hit = self._memo.get(key)
        if hit is not None:
            self.memo_stats["hits"] += 1
            return hit
        mask, offset = super().getmask2(text, mode, start=start, **kwargs)
        self._exact_put(ekey, (mask, offset))
        self.memo_stats["renders"] += 1
        sig = (bytes(mask), mask.size, tuple(offset))
        with self._memo_lock:
            first = self._pending.get(key)
            if first is None:
                self._pending[key] = (tuple(start), sig)
            elif first[0] != tuple(start):  # a second fraction of the class: verify before memoising
                if first[1] == sig:
                    self._memo[key] = (mask, offset)
                else:
                    self._no_memo.add(key)
                del self._pending[key]
        return mask, offset


_font = None
_font_lock = threading.Lock()


def memo_default_font() -> _MemoFont:
    global _font
    with _font_lock:
        if _font is None:
            f = _PILFont.load_default()
            if not isinstance(f, _PILFont.FreeTypeFont):  # Pillow without FreeType: its bitmap font, as is
                return f
            f.__class__ = _MemoFont
            f._memo_init()
            _font = f
        return _font


class _DrawModule(types.ModuleType):
    """`PIL.ImageDraw` as serve.py sees it after the drop-in (module scope): every attribute is
    Pillow's; `Draw(im)` is Pillow's ImageDraw on `im` whose default font memoises its glyph masks."""

    def __init__(self):
        super().__init__("PIL.ImageDraw", _PILDraw.__doc__)

    def __getattr__(self, name):
        return getattr(_PILDraw, name)

    def Draw(self, im, mode=None):  # noqa: N802 - Pillow's name
        d = _PILDraw.Draw(im, mode)
        if d.font is None:
            d.font = memo_default_font()
        return d


def draw_module() -> types.ModuleType:
    """The `ImageDraw` global the drop-in binds in serve.py (spotter_amd/dropin.py)."""
    return _DrawModule()
