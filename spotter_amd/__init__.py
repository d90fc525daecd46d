"""spotter_amd — MI355X-native RT-DETRv2 `/detect` hot path for chilir/spotter.

Drop-in replacement for the HuggingFace processor/model pair that
`AmenitiesDetector` (reference: apps/spotter/src/spotter/serve.py:64-205)
consumes through its duck-typed interface (serve.py:98-117). Every stage of the
path runs as a hand-written CDNA4 HIP kernel in ``libspotter_hip.so`` (C-ABI,
see include/spotter_hip.h) loaded with ctypes; PyTorch-ROCm only allocates
device memory and provides the stream.
"""
from .config import SpotterConfig, PRESETS, COCO_ID2LABEL  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy imports keep `import spotter_amd` cheap and GPU-free.
    if name in ("SpotterImageProcessor",):
        from .processor import SpotterImageProcessor
        return SpotterImageProcessor
    if name in ("SpotterForObjectDetection",):
        from .model import SpotterForObjectDetection
        return SpotterForObjectDetection
    raise AttributeError(name)
