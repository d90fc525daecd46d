"""The serve.py change of INTEGRATION.md §2, as code: applied by deploy/Dockerfile.rocm at image build
time and by tests/test_dropin_reference.py in memory, so the image and the test run the same edit.

    python -m spotter_amd.dropin <path to apps/spotter/src/spotter/serve.py>

Three reference lines change: the model and processor built at import (serve.py:203-204) and the
image open of _process_single_image (serve.py:96, `Image.open(BytesIO(image_bytes))` →
`open_image(image_bytes)`: JPEGs decoded on the GPU, bit-identical to Pillow's pixels; other formats
still go through Image.open). Assert-then-replace: each reference line must occur exactly once, else
the build stops instead of shipping an image that still runs the CPU HuggingFace model.
"""
from __future__ import annotations

import sys

OLD_MODEL = "model = AutoModelForObjectDetection.from_pretrained(model_name).to(device)  # type: ignore"
OLD_PROC = "processor = AutoImageProcessor.from_pretrained(model_name)"
OLD_OPEN = "with Image.open(BytesIO(image_bytes)) as img_raw:"
NEW_MODEL = ("from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor\n"
             "from spotter_amd.jpeg import open_image\n"
             "model = SpotterForObjectDetection.from_pretrained(model_name).to(device)")
NEW_PROC = "processor = SpotterImageProcessor.from_pretrained(model_name)"
NEW_OPEN = "with open_image(image_bytes) as img_raw:"
MARK = "from spotter_amd import SpotterForObjectDetection"
REPLACEMENTS = ((OLD_MODEL, NEW_MODEL), (OLD_PROC, NEW_PROC), (OLD_OPEN, NEW_OPEN))


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
    """The patched file builds the model and processor from spotter_amd and opens images with open_image."""
    if (MARK not in src or NEW_PROC not in src or NEW_OPEN not in src
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
