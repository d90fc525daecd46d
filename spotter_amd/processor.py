"""SpotterImageProcessor — drop-in for the HF RT-DETR image processor on MI355X.

Implements the part of `RTDetrImageProcessorPil` that AmenitiesDetector uses
(reference serve.py:67-68, 98, 103-109):

* ``processor(images=PIL.Image, return_tensors="pt")`` (or a GPU-decoded image from
  ``spotter_amd.jpeg.open_image``, read in place) → mapping with
  ``pixel_values`` f32 ``[n, 3, 640, 640]`` (IPP:129-143 defaults: resize
  640×640 BILINEAR, rescale 1/255, no normalize, no pad), computed by the
  fused HIP kernel ``sp_preprocess_u8`` (bit-exact with Pillow).
* ``processor.post_process_object_detection(outputs, threshold, target_sizes)``
  (IPP:508-578, use_focal_loss=True) by ``sp_postprocess`` → list of dicts of
  CPU tensors ``scores`` f32, ``labels`` int64, ``boxes`` f32 xyxy.

Device placement belongs to the processor: the reference moves inputs to
``device`` = cpu/mps (serve.py:61, 98); here ``.to(cpu|mps)`` on the returned
batch keeps ``pixel_values`` on the MI355X so the model reads it in place.
The object holds no device state, so Ray can pickle it into each replica.
"""
from __future__ import annotations

import json
import os
import threading

import numpy as np
import torch

from . import ops


class SpotterBatchFeature(dict):
    """Minimal BatchFeature: a dict whose `.to()` never pulls device tensors to the host."""

    def to(self, device=None, *args, **kwargs):
        dev = torch.device(device) if device is not None else None
        if dev is None or dev.type in ("cpu", "mps"):
            return self  # placement is owned by the engine: stay in HBM
        return SpotterBatchFeature({k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in self.items()})

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e


def _device_rgb(img, dev):
    """A uint8 [H, W, 3] device tensor already holding the image (a GPU-decoded DeviceRGBImage, or a CUDA
    tensor given directly), else None."""
    t = getattr(img, "spotter_device_rgb", None)
    if t is None and torch.is_tensor(img) and img.is_cuda:
        t = img
    if t is None:
        return None
    if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
        raise ValueError("device images must be uint8 [H, W, 3]")
    return t.to(dev).contiguous()


def _as_uint8_rgb(img) -> np.ndarray:
    try:
        from PIL import Image
    except Exception:  # pragma: no cover
        Image = None
    if Image is not None and isinstance(img, Image.Image):
        if img.mode != "RGB":
            img = img.convert("RGB")
        return np.asarray(img)
    a = np.asarray(img)
    if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
        raise ValueError("images must be RGB PIL images or uint8 HWC arrays with 3 channels")
    return a


class SpotterImageProcessor:
    model_input_names = ["pixel_values"]

    def __init__(self, size=None, device=None, **kwargs):
        self.size = dict(size) if size else {"height": 640, "width": 640}
        self.do_resize = kwargs.get("do_resize", True)
        self.do_rescale = kwargs.get("do_rescale", True)
        self.do_normalize = kwargs.get("do_normalize", False)
        self.do_pad = kwargs.get("do_pad", False)
        self.rescale_factor = kwargs.get("rescale_factor", 1 / 255)
        if not (self.do_resize and self.do_rescale) or self.do_normalize or self.do_pad:
            raise NotImplementedError("only the RT-DETR defaults (resize, rescale 1/255, no normalize/pad) are on the HIP path")
        if abs(self.rescale_factor - 1 / 255) > 1e-12:
            raise NotImplementedError("rescale_factor must be 1/255")
        # PIL.Image.BILINEAR == 2 (IPP:129-143 default); the kernel is Pillow's bilinear resample only
        self.resample = kwargs.get("resample", 2)
        if self.resample not in (2, "bilinear", "BILINEAR"):
            raise NotImplementedError(f"resample={self.resample!r}: the HIP preprocess implements PIL BILINEAR (2) only")
        if not {"height", "width"} <= set(self.size):
            raise NotImplementedError(f"size={self.size!r}: only an explicit {{height, width}} resize is on the HIP path")
        self.device = device
        self._stage = None  # pinned host staging buffer, reused across calls
        self._stage_done = None  # event after the last H2D copy out of it
        self._stage_lock = threading.Lock()  # request threads may share one processor

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_stage"] = None
        st["_stage_done"] = None
        st["_stage_lock"] = None
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._stage_lock = threading.Lock()

    @classmethod
    def from_pretrained(cls, path_or_name, **kwargs):
        """A local directory or a hub repo id cached locally (checkpoint.resolve_pretrained: the
        reference's download.py:29-30 pre-fetches the processor config under the same name);
        preprocessor_config.json fields that change the arithmetic are honoured or refused.
        "synthetic:<preset>" → the RT-DETR defaults (explicit opt-in, as for the model)."""
        cfg = {}
        if not str(path_or_name).startswith("synthetic:"):
            from .checkpoint import resolve_pretrained

            d = resolve_pretrained(path_or_name, need="preprocessor_config.json") if not os.path.isdir(
                path_or_name) else path_or_name
            p = os.path.join(d, "preprocessor_config.json")
            if os.path.exists(p):
                with open(p) as f:
                    cfg = json.load(f)
        cfg.update(kwargs)
        keep = {k: cfg[k] for k in ("size", "do_resize", "do_rescale", "do_normalize", "do_pad",
                                     "rescale_factor", "resample") if k in cfg}
        return cls(**keep)

    def _upload(self, arrs, dev):
        """Decoded uint8 images → device, through one reused pinned staging buffer (no per-request
        pinned allocation): wait for the previous copy out of it, fill it, one async H2D per image."""
        sizes = [a.size for a in arrs]
        offs, total = [], 0
        for n in sizes:  # 256-B aligned slots (the same-size kernel reads 4-byte words)
            offs.append(total)
            total += (n + 255) & ~255
        dst = torch.empty((total,), dtype=torch.uint8, device=dev)
        with self._stage_lock:  # fill → async copy → event, one caller at a time
            if self._stage_done is not None:
                self._stage_done.synchronize()
            if self._stage is None or self._stage.numel() < total:
                self._stage = torch.empty((max(total, 1 << 20),), dtype=torch.uint8, pin_memory=True)
            host = self._stage.numpy()
            ups = []
            for a, n, off in zip(arrs, sizes, offs):
                host[off:off + n] = a.reshape(-1)
                ups.append(dst[off:off + n].view(a.shape))
            dst.copy_(self._stage[:total], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(dev))
            self._stage_done = ev
        return ups

    def _dev(self):
        if self.device is not None:
            return torch.device(self.device)
        return torch.device("cuda", torch.cuda.current_device())

    def __call__(self, images=None, return_tensors="pt", **kwargs):
        if images is None:
            raise ValueError("images is required")
        if not isinstance(images, (list, tuple)):
            images = [images]
        dev = self._dev()
        # GPU-decoded images (spotter_amd.jpeg.open_image) are read in place; the rest go up once, pinned
        dimgs = [_device_rgb(im, dev) for im in images]
        arrs = [_as_uint8_rgb(im) for im, d in zip(images, dimgs) if d is None]
        oh, ow = int(self.size["height"]), int(self.size["width"])
        with torch.cuda.device(dev):
            ups = iter(self._upload(arrs, dev) if arrs else [])
            srcs = [d if d is not None else next(ups) for d in dimgs]
            out = torch.empty((len(srcs), 3, oh, ow), dtype=torch.float32, device=dev)
            ops.preprocess_u8(srcs, out, oh, ow)
        if return_tensors not in ("pt", None):
            raise ValueError("only return_tensors='pt' is supported")
        return SpotterBatchFeature(pixel_values=out)

    def post_process_object_detection(self, outputs, threshold: float = 0.5, target_sizes=None,
                                      use_focal_loss: bool = True):
        if not use_focal_loss:
            raise NotImplementedError("RT-DETRv2 uses focal-loss (sigmoid) scores")
        logits, boxes = outputs.logits, outputs.pred_boxes
        b, q, c = logits.shape
        dev = logits.device
        if target_sizes is not None:
            if len(target_sizes) != b:
                raise ValueError("Make sure that you pass in as many target sizes as the batch dimension of the logits")
            ts = torch.as_tensor(np.asarray([[int(h), int(w)] for h, w in (
                target_sizes.tolist() if torch.is_tensor(target_sizes) else target_sizes)]), dtype=torch.int32)
        else:
            ts = torch.ones((b, 2), dtype=torch.int32)
        k = q  # num_top_queries = logits.shape[1] (IPP:551-556)
        with torch.cuda.device(dev):
            tsd = ts.to(dev, non_blocking=True)
            scores = torch.empty((b, k), dtype=torch.float32, device=dev)
            labels = torch.empty((b, k), dtype=torch.int64, device=dev)
            bx = torch.empty((b, k, 4), dtype=torch.float32, device=dev)
            counts = torch.empty((b,), dtype=torch.int32, device=dev)
            work = torch.empty((b, k), dtype=torch.int32, device=dev)
            ops.postprocess(logits.contiguous().float(), boxes.contiguous().float(), tsd, k, float(threshold),
                            scores, labels, bx, counts, work)
            # four async copies into pinned host memory, one wait (not four synchronous round trips)
            host = [t.to("cpu", non_blocking=True) for t in (scores, labels, bx, counts)]
            torch.cuda.current_stream(dev).synchronize()
        s_h, l_h, b_h, c_h = host
        res = []
        for i in range(b):
            n = int(c_h[i])
            res.append({"scores": s_h[i, :n], "labels": l_h[i, :n], "boxes": b_h[i, :n]})
        return res
