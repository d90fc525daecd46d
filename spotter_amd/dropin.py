"""The serve.py change of INTEGRATION.md §2, as code: applied by deploy/Dockerfile.rocm at image build
time and by tests/test_dropin_reference.py in memory, so the image and the test run the same edit.

    python -m spotter_amd.dropin <path to apps/spotter/src/spotter/serve.py>

Only module-scope lines change; the Ray Serve deployment class AmenitiesDetector (serve.py:64-196) stays the
reference's text byte for byte (tests/test_dropin_reference.py compares it). The model and processor built
at import (serve.py:203-204) become the spotter_amd objects (the model's operand precision from the
SPOTTER_PRECISION environment variable, default "fp32"; an unknown value fails the import; serve.py already
imports os, :5), and serve.py's module-global `Image` (bound by
`from PIL import Image, ImageDraw`, serve.py:10) is rebound to spotter_amd.jpeg.image_module(): Pillow's
module with a GPU `open` (JPEGs decoded on the GPU, pixels identical to Pillow's; Pillow parses the header
first, so every file Pillow refuses raises exactly as before) whose decoded images also encode on the GPU
in `save(..., format="JPEG")` (bytes identical to Pillow's); `ImageDraw` is rebound to
spotter_amd.draw.draw_module() (Pillow's ImageDraw, the default font's glyph masks memoised: Pillow's
pixels). Assert-then-replace: each reference line must
occur exactly once, else the build stops instead of shipping an image that still runs the CPU HuggingFace
model.
"""
from __future__ import annotations

import sys

OLD_MODEL = "model = AutoModelForObjectDetection.from_pretrained(model_name).to(device)  # type: ignore"
OLD_PROC = "processor = AutoImageProcessor.from_pretrained(model_name)"
NEW_MODEL = ("from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor\n"
             "from spotter_amd.draw import draw_module\n"
             "from spotter_amd.jpeg import image_module\n"
             "Image = image_module()  # PIL.Image with the GPU JPEG decode / encode (AmenitiesDetector unchanged)\n"
             "ImageDraw = draw_module()  # PIL.ImageDraw whose default font memoises its glyph masks\n"
             "model = SpotterForObjectDetection.from_pretrained(\n"
             "    model_name, precision=os.environ.get(\"SPOTTER_PRECISION\", \"fp32\")  # fp32 (parity) or bf16 (C4)\n"
             ").to(device)")
NEW_PROC = "processor = SpotterImageProcessor.from_pretrained(model_name)"
MARK = "from spotter_amd import SpotterForObjectDetection"
PRECISION_ARG = 'precision=os.environ.get("SPOTTER_PRECISION", "fp32")'
REPLACEMENTS = ((OLD_MODEL, NEW_MODEL), (OLD_PROC, NEW_PROC))


def patch_source(src: str) -> str:
    """serve.py text → the drop-in text. Raises ValueError unless each line occurs exactly once."""
    for old, _ in REPLACEMENTS:
        n = src.count(old)
        if n != 1:
            raise ValueError(f"reference serve.py: expected exactly one {old!r}, found {n}; "
                             "update spotter_amd/dropin.py and INTEGRATION.md")
    out = src
    for old, new in REPLACEMENTS:
        out = out.replace(old, new)
    check(out)
    return out


def check(src: str) -> None:
    """The patched file builds the model and processor from spotter_amd and rebinds Image at module scope."""
    if (MARK not in src or NEW_PROC not in src or "Image = image_module()" not in src
            or "ImageDraw = draw_module()" not in src or PRECISION_ARG not in src
            or any(old in src for old, _ in REPLACEMENTS)):
        raise ValueError("serve.py is not the spotter_amd drop-in")


def main(argv) -> int:
    if len(argv) != 2:
        print(__doc__, file=sys.stderr)
        return 2
    path = argv[1]
    with open(path) as f:
        src = f.read()
    if MARK in src:
        check(src)  # already applied (idempotent rebuilds)
        return 0
    with open(path, "w") as f:
        f.write(patch_source(src))
    print(f"spotter_amd drop-in applied to {path}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
