"""The two-line serve.py change of INTEGRATION.md §2, as code: applied by deploy/Dockerfile.rocm at
image build time and by tests/test_dropin_reference.py in memory, so the image and the test run
the same edit.

    python -m spotter_amd.dropin <path to apps/spotter/src/spotter/serve.py>

Assert-then-replace: each reference line (serve.py:203-204) must occur exactly once, else the
build stops instead of shipping an image that still runs the CPU HuggingFace model.
"""
from __future__ import annotations

import sys

OLD_MODEL = "model = AutoModelForObjectDetection.from_pretrained(model_name).to(device)  # type: ignore"
OLD_PROC = "processor = AutoImageProcessor.from_pretrained(model_name)"
NEW_MODEL = ("from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor\n"
             "model = SpotterForObjectDetection.from_pretrained(model_name).to(device)")
NEW_PROC = "processor = SpotterImageProcessor.from_pretrained(model_name)"
MARK = "from spotter_amd import SpotterForObjectDetection"


def patch_source(src: str) -> str:
    """serve.py text → the drop-in text. Raises ValueError unless both lines occur exactly once."""
    for old in (OLD_MODEL, OLD_PROC):
        n = src.count(old)
        if n != 1:
            raise ValueError(f"reference serve.py: expected exactly one {old!r}, found {n}; "
                             "update spotter_amd/dropin.py and INTEGRATION.md")
    out = src.replace(OLD_MODEL, NEW_MODEL).replace(OLD_PROC, NEW_PROC)
    check(out)
    return out


def check(src: str) -> None:
    """The patched file builds the model and processor from spotter_amd, not from transformers."""
    if MARK not in src or NEW_PROC not in src or OLD_MODEL in src or OLD_PROC in src:
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
