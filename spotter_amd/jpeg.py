"""JPEG decode in front of the processor: serve.py:96-97 decodes every image on the host with
Pillow (`Image.open(BytesIO(resp.content)).convert("RGB")`); here the Huffman entropy decode runs in the
library's host code (sp_jpeg_decode_coefs, a serial bit stream) and the per-pixel part — dequantisation,
ISLOW IDCT, fancy upsampling, YCbCr→RGB — on the GPU (sp_jpeg_to_rgb), producing the same pixels as
Pillow's libjpeg-turbo, bit for bit (tests/test_jpeg.py, tests/test_gpu_kernels.py).

`JpegDecoder.decode(data)` returns the uint8 [H, W, 3] image on the device, ready for sp_preprocess_u8;
`open_image(data)` is the drop-in for serve.py:96's `Image.open(BytesIO(image_bytes))`: a PIL RGB image (what the unchanged draw / encode tail
needs) that also carries its device copy, which SpotterImageProcessor then uses instead of uploading it
again. JPEG forms the library does not decode (CMYK, 12-bit, arithmetic coding, ...) and other image formats
keep the reference's host decode: UnsupportedJpeg is raised and open_image falls back to Pillow's Image.open for that image.
"""
from __future__ import annotations

import ctypes as C
import threading

import numpy as np
import torch

from ._lib import SP_JPEG_UNSUPPORTED, SpJpegLayout, lib


class UnsupportedJpeg(ValueError):
    """A JPEG form (or another format) the GPU decoder does not implement."""


def _buf(data):
    if isinstance(data, (bytes, bytearray)):
        b = bytes(data)
        return C.cast(C.c_char_p(b), C.c_void_p), len(b), b
    a = np.ascontiguousarray(np.frombuffer(data, dtype=np.uint8))
    return a.ctypes.data, a.size, a


def decode_coefs(data, out: np.ndarray | None = None):
    """Host entropy decode: (layout, int16 coefficients [total_blocks, 64] natural order). out: reuse this
    int16 buffer (e.g. a pinned one) when it is large enough."""
    ptr, n, keep = _buf(data)
    lay = SpJpegLayout()
    L = lib()
    rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), None, 0)
    if rc == SP_JPEG_UNSUPPORTED:
        raise UnsupportedJpeg(L.sp_last_error().decode(errors="replace"))
    if rc:
        raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
    need = lay.total_blocks * 64
    if out is None or out.size < need:
        out = np.empty(need, dtype=np.int16)
    rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), out.ctypes.data, out.size)
    del keep
    if rc == SP_JPEG_UNSUPPORTED:
        raise UnsupportedJpeg(L.sp_last_error().decode(errors="replace"))
    if rc:
        raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
    return lay, out[:need].reshape(-1, 64)


def layout_dict(lay: SpJpegLayout) -> dict:
    d = {k: getattr(lay, k) for k in ("width", "height", "ncomp", "color", "progressive", "max_h", "max_v",
                                      "total_blocks", "plane_bytes")}
    for k in ("h", "v", "bw", "bh", "block_off", "plane_off"):
        d[k] = list(getattr(lay, k))
    d["quant"] = [list(lay.quant[c]) for c in range(3)]
    return d


class JpegDecoder:
    """Per-device decoder state: a pinned host coefficient buffer and device buffers, grown as needed and
    reused (one decode at a time per decoder; the lock serialises concurrent callers)."""

    def __init__(self, device):
        self.dev = torch.device(device)
        self._lock = threading.Lock()
        self._host = None  # pinned int16
        self._coefs = None  # device int16
        self._work = None  # device uint8 planes
        self._copied = None  # event: the last H2D copy out of the pinned buffer is done
        self._done = None  # event: the last decode's kernels are done with the device buffers

    def _grow(self, n_coef, n_work):
        if self._host is None or self._host.numel() < n_coef:
            self._host = torch.empty(max(n_coef, 1 << 20), dtype=torch.int16, pin_memory=True)
            self._coefs = torch.empty(self._host.numel(), dtype=torch.int16, device=self.dev)
        if self._work is None or self._work.numel() < n_work:
            self._work = torch.empty(max(n_work, 1 << 20), dtype=torch.uint8, device=self.dev)

    def decode(self, data, out: torch.Tensor | None = None) -> torch.Tensor:
        """JPEG bytes → uint8 [H, W, 3] on the device (on torch's current stream)."""
        ptr, n, keep = _buf(data)
        lay = SpJpegLayout()
        L = lib()
        with self._lock:
            rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), None, 0)
            if rc == SP_JPEG_UNSUPPORTED:
                raise UnsupportedJpeg(L.sp_last_error().decode(errors="replace"))
            if rc:
                raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
            ncoef = lay.total_blocks * 64
            self._grow(ncoef, lay.plane_bytes)
            if self._copied is not None:
                self._copied.synchronize()  # the pinned buffer is free again
            rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), self._host.data_ptr(), self._host.numel())
            del keep
            if rc:
                raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
            cur = torch.cuda.current_stream(self.dev)
            if self._done is not None:
                cur.wait_event(self._done)  # another stream's previous decode may still read the buffers
            self._coefs[:ncoef].copy_(self._host[:ncoef], non_blocking=True)
            self._copied = torch.cuda.Event()
            self._copied.record()
            H, W = lay.height, lay.width
            if out is None:
                out = torch.empty((H, W, 3), dtype=torch.uint8, device=self.dev)
            assert out.dtype == torch.uint8 and out.is_cuda and out.shape == (H, W, 3) and out.is_contiguous()
            rc = L.sp_jpeg_to_rgb(self._coefs.data_ptr(), C.byref(lay), self._work.data_ptr(), self._work.numel(),
                                  out.data_ptr(), W * 3, cur.cuda_stream)
            if rc:
                raise RuntimeError(f"sp_jpeg_to_rgb: {L.sp_last_error().decode(errors='replace')}")
            self._done = torch.cuda.Event()
            self._done.record(cur)
            return out


_decoders: dict = {}
_dec_lock = threading.Lock()


def decoder(device=None) -> JpegDecoder:
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    with _dec_lock:
        d = _decoders.get(dev)
        if d is None:
            d = _decoders[dev] = JpegDecoder(dev)
        return d


try:
    from PIL import Image as _PILImage
except Exception:  # pragma: no cover - Pillow is a dependency of the reference app
    _PILImage = None


class DeviceRGBImage(_PILImage.Image if _PILImage is not None else object):
    """A PIL RGB image decoded on the GPU. `spotter_device_rgb` holds the uint8 [H, W, 3] device tensor that
    SpotterImageProcessor reads in place; the host pixels (what the unchanged draw / JPEG-encode tail of
    serve.py:119-142 needs) arrive by an async D2H copy on a side stream and are materialised only when
    Pillow first needs them (load()). convert("RGB") / copy() of a not-yet-loaded image stay lazy."""

    def __init__(self, rgb_dev: torch.Tensor, host=None, done=None):
        super().__init__()
        H, W, _ = rgb_dev.shape
        self._mode = "RGB"
        self._size = (int(W), int(H))
        self.spotter_device_rgb = rgb_dev
        if host is None:
            dev = rgb_dev.device
            host = torch.empty(rgb_dev.shape, dtype=torch.uint8, pin_memory=True)
            side = _side_stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                host.copy_(rgb_dev, non_blocking=True)
                done = torch.cuda.Event()
                done.record(side)
            rgb_dev.record_stream(side)
        self._pending = (host, done)

    def _lazy_copy(self):
        return DeviceRGBImage(self.spotter_device_rgb, *self._pending)

    def load(self):
        if self._im is None and getattr(self, "_pending", None) is not None:
            host, done = self._pending
            done.synchronize()
            self.im = _PILImage.frombytes("RGB", self._size, host.numpy().tobytes()).im
        return super().load()

    def convert(self, mode=None, *args, **kwargs):
        if mode in (None, "RGB") and not args and not kwargs and self._im is None:
            return self._lazy_copy()
        return super().convert(mode, *args, **kwargs)

    def copy(self):
        if self._im is None:
            return self._lazy_copy()
        return super().copy()


_sides: dict = {}


def _side_stream(dev):
    s = _sides.get(dev)
    if s is None:
        s = _sides[dev] = torch.cuda.Stream(dev)
    return s


def open_image(data, device=None):
    """The drop-in for serve.py:96 `Image.open(BytesIO(image_bytes))`: JPEG bytes the library decodes →
    a DeviceRGBImage (decoded on the GPU, pixels identical to Pillow's); anything else (PNG, CMYK JPEG, ...)
    → the reference's own Image.open. Either way the caller's `.convert("RGB")` follows unchanged."""
    import io

    b = bytes(data)
    if len(b) >= 3 and b[:3] == b"\xff\xd8\xff":
        try:
            return DeviceRGBImage(decoder(device).decode(b))
        except UnsupportedJpeg:
            pass
    return _PILImage.open(io.BytesIO(b))
