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
import types

import numpy as np
import torch

from ._lib import SP_JPEG_UNSUPPORTED, SpJpegLayout, lib


class UnsupportedJpeg(ValueError):
    """A JPEG form (or another format) the GPU decoder does not implement, or a malformed file: either way the
    bytes go to Pillow, i.e. to the reference's own decoder and its own errors and warnings."""


def _check_pixels(lay) -> None:
    """Pillow's decompression-bomb rule (Image._decompression_bomb_check): above Image.MAX_IMAGE_PIXELS Pillow
    warns, above twice that it raises DecompressionBombError. The GPU path takes neither: such a frame is left
    to Pillow (which then warns or raises exactly as the reference does), and nothing is allocated for it."""
    from PIL import Image

    limit = Image.MAX_IMAGE_PIXELS
    if limit is not None and max(1, lay.width) * max(1, lay.height) > limit:
        raise UnsupportedJpeg(f"{lay.width}x{lay.height} exceeds Image.MAX_IMAGE_PIXELS: left to Pillow")


# decode buffers a JpegDecoder keeps between calls; a larger image gets buffers of its own for that call only
KEEP_COEFS = 1 << 25  # int16 coefficients (64 MiB pinned + 64 MiB device): a 4K 4:4:4 frame fits
KEEP_WORK = 1 << 26   # bytes of component planes


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
    _check_pixels(lay)
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
    """Per-device decoder state: a pinned host coefficient buffer and device buffers, grown as needed up to
    KEEP_COEFS / KEEP_WORK and reused (one decode at a time per decoder; the lock serialises concurrent
    callers). A larger image decodes through buffers allocated for that call and released after it."""

    def __init__(self, device):
        self.dev = torch.device(device)
        self._lock = threading.Lock()
        self._host = None  # pinned int16
        self._coefs = None  # device int16
        self._work = None  # device uint8 planes
        self._copied = None  # event: the last H2D copy out of the pinned buffer is done
        self._done = None  # event: the last decode's kernels are done with the device buffers
        self._status = torch.zeros(1, dtype=torch.int32, device=self.dev)  # sp_jpeg_to_rgb's envelope flag
        self._status_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)

    def _buffers(self, n_coef, n_work):
        """(pinned host coefficients, device coefficients, device planes, kept?) for one decode."""
        if n_coef > KEEP_COEFS or n_work > KEEP_WORK:
            if self._copied is not None:
                self._copied.synchronize()
            return (torch.empty(n_coef, dtype=torch.int16, pin_memory=True),
                    torch.empty(n_coef, dtype=torch.int16, device=self.dev),
                    torch.empty(n_work, dtype=torch.uint8, device=self.dev), False)
        grow_c = self._host is None or self._host.numel() < n_coef
        grow_w = self._work is None or self._work.numel() < n_work
        if (grow_c or grow_w) and self._done is not None:
            # the old buffers may still be read by the previous decode on another stream: let it finish
            # before they go back to the caching allocator
            self._done.synchronize()
        if grow_c:
            n = min(KEEP_COEFS, max(n_coef, 1 << 20))
            self._host = torch.empty(n, dtype=torch.int16, pin_memory=True)
            self._coefs = torch.empty(n, dtype=torch.int16, device=self.dev)
        if grow_w:
            self._work = torch.empty(min(KEEP_WORK, max(n_work, 1 << 20)), dtype=torch.uint8, device=self.dev)
        return self._host, self._coefs, self._work, True

    def decode(self, data, out: torch.Tensor | None = None) -> torch.Tensor:
        """JPEG bytes → uint8 [H, W, 3] on the device (on torch's current stream). Returns once the kernels
        have run (the IDCT's envelope flag is read back: a file outside it raises UnsupportedJpeg, for Pillow)."""
        ptr, n, keep = _buf(data)
        lay = SpJpegLayout()
        L = lib()
        with self._lock:
            rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), None, 0)
            if rc == SP_JPEG_UNSUPPORTED:
                raise UnsupportedJpeg(L.sp_last_error().decode(errors="replace"))
            if rc:
                raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
            _check_pixels(lay)
            ncoef = lay.total_blocks * 64
            host, coefs, work, kept = self._buffers(ncoef, lay.plane_bytes)
            if kept and self._copied is not None:
                self._copied.synchronize()  # the pinned buffer is free again
            rc = L.sp_jpeg_decode_coefs(ptr, n, C.byref(lay), host.data_ptr(), host.numel())
            del keep
            if rc == SP_JPEG_UNSUPPORTED:
                raise UnsupportedJpeg(L.sp_last_error().decode(errors="replace"))
            if rc:
                raise RuntimeError(f"sp_jpeg_decode_coefs: {L.sp_last_error().decode(errors='replace')}")
            cur = torch.cuda.current_stream(self.dev)
            if kept and self._done is not None:
                cur.wait_event(self._done)  # another stream's previous decode may still read the buffers
            coefs[:ncoef].copy_(host[:ncoef], non_blocking=True)
            copied = torch.cuda.Event()
            copied.record()
            H, W = lay.height, lay.width
            if out is None:
                out = torch.empty((H, W, 3), dtype=torch.uint8, device=self.dev)
            assert out.dtype == torch.uint8 and out.is_cuda and out.shape == (H, W, 3) and out.is_contiguous()
            self._status.zero_()
            rc = L.sp_jpeg_to_rgb(coefs.data_ptr(), C.byref(lay), work.data_ptr(), work.numel(),
                                  out.data_ptr(), W * 3, self._status.data_ptr(), cur.cuda_stream)
            if rc:
                raise RuntimeError(f"sp_jpeg_to_rgb: {L.sp_last_error().decode(errors='replace')}")
            self._status_host.copy_(self._status, non_blocking=True)
            done = torch.cuda.Event()
            done.record(cur)
            done.synchronize()
            if kept:
                self._copied, self._done = copied, done
            if int(self._status_host[0]):
                raise UnsupportedJpeg("coefficients outside the IDCT range shared with libjpeg-turbo's SIMD "
                                      "code (corrupt or crafted data): left to Pillow")
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


from PIL import Image as _PILImage  # noqa: E402  (Pillow is a dependency of the reference app)
from PIL import JpegImagePlugin as _JpegPlugin  # noqa: E402


class DeviceRGBImage(_PILImage.Image):
    """A PIL RGB image decoded on the GPU. `spotter_device_rgb` holds the uint8 [H, W, 3] device tensor that
    SpotterImageProcessor reads in place; the host pixels (what the unchanged draw / JPEG-encode tail of
    serve.py:119-142 needs) arrive by an async D2H copy on a side stream and are materialised only when
    Pillow first needs them (load()). convert("RGB") / copy() of a not-yet-loaded image stay lazy. `info` is
    the source file's, as Pillow's JpegImageFile would carry it (its "comment" is written back by save)."""

    def __init__(self, rgb_dev: torch.Tensor, host=None, done=None, info=None):
        super().__init__()
        H, W, _ = rgb_dev.shape
        self._mode = "RGB"
        self._size = (int(W), int(H))
        self.spotter_device_rgb = rgb_dev
        if info:
            self.info = dict(info)
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
        return DeviceRGBImage(self.spotter_device_rgb, *self._pending, info=self.info)

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


def _device_image(im, data, device=None):
    """A file Pillow has opened (its header parse, identification rules and decompression-bomb check have run,
    raising whatever the reference raises) → its GPU-decoded DeviceRGBImage, or None to keep Pillow's image:
    other formats and modes, MPO, and every JPEG the library leaves to the host decoder."""
    if type(im) is not _JpegPlugin.JpegImageFile or im.mode != "RGB":
        return None
    try:
        return DeviceRGBImage(decoder(device).decode(data), info=im.info)
    except UnsupportedJpeg:
        return None


def open_image(data, device=None):
    """serve.py:96's `Image.open(BytesIO(image_bytes))` for raw bytes: a DeviceRGBImage for the JPEGs the
    library decodes (pixels identical to Pillow's), Pillow's own image otherwise. Pillow parses the header
    first, so a file Pillow refuses raises exactly what the reference raises."""
    import io

    b = bytes(data)
    im = _PILImage.open(io.BytesIO(b))
    dev = _device_image(im, b, device)
    if dev is None:
        return im
    im.close()
    return dev


class _ImageModule(types.ModuleType):
    """`PIL.Image` as serve.py sees it after the drop-in: every attribute is Pillow's,
    except `open`, which decodes JPEGs on the GPU (open_image's rule) when handed an in-memory file, as
    serve.py:96 does. Bound at module scope, so AmenitiesDetector's body stays the reference's, byte for byte."""

    def __init__(self, device=None):
        super().__init__("PIL.Image", _PILImage.__doc__)
        self._spotter_device = device

    def __getattr__(self, name):
        return getattr(_PILImage, name)

    def open(self, fp, mode="r", formats=None):
        import io

        im = _PILImage.open(fp, mode, formats)
        if mode == "r" and isinstance(fp, io.BytesIO):
            dev = _device_image(im, fp.getvalue(), self._spotter_device)
            if dev is not None:
                im.close()
                return dev
        return im


def image_module(device=None) -> types.ModuleType:
    """The `Image` global the drop-in binds in serve.py (spotter_amd/dropin.py)."""
    return _ImageModule(device)
