"""SpotterForObjectDetection — drop-in for HF RTDetrV2ForObjectDetection on MI355X.

The interface AmenitiesDetector relies on (reference serve.py:99-100, 111-114,
199-205): ``model(**inputs)`` (under ``torch.no_grad()``) returning an object
with ``.logits [B,300,80]`` and ``.pred_boxes [B,300,4]``; ``model.config.id2label``;
``.to(device)``; and cheap pickling, because ``AmenitiesDetector.bind(model,
processor)`` ships the bound model into every Serve replica.
The device engine is therefore created lazily inside the replica, on its
first call, from the host-side weight dictionary.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass

import torch

from .config import PRESETS, SpotterConfig, check_precision


@dataclass
class SpotterDetectionOutput:
    logits: torch.Tensor
    pred_boxes: torch.Tensor

    def __getitem__(self, k):
        return getattr(self, k)


class _Config:
    """The bits of HF's config the caller reads (`id2label`, `num_labels`)."""

    def __init__(self, cfg: SpotterConfig):
        self.id2label = dict(cfg.id2label)
        self.label2id = {v: k for k, v in self.id2label.items()}
        self.num_labels = cfg.num_labels
        self.num_queries = cfg.num_queries
        self.model_type = "rt_detr_v2"
        self.spotter = cfg


def _preset_for(name: str) -> SpotterConfig:
    n = name.lower()
    if "r18" in n:
        return PRESETS["r18vd"]
    return PRESETS["r101vd"]


class SpotterForObjectDetection:
    main_input_name = "pixel_values"

    def __init__(self, cfg: SpotterConfig, weights: dict | None = None, seed: int = 0,
                 use_graphs: bool = True, precision: str = "fp32", batching: bool = False,
                 max_batch: int = 32, max_wait_ms: float = 2.0):
        """batching: coalesce concurrent calls (several request threads) into one engine forward
        (spotter_amd.batching.MicroBatcher, up to max_batch images within max_wait_ms)."""
        self.cfg = cfg
        self.batching = batching
        self.max_batch = max_batch
        self.max_wait_ms = max_wait_ms
        self._batcher = None
        self.use_graphs = use_graphs
        # config.PRECISIONS key; "fp32" = the fp32-accurate parity path, "bf16" = the C4 variant. Checked here, at
        # construction (serve.py import time), so a bad SPOTTER_PRECISION fails the deployment, not the first request.
        self.precision = check_precision(precision)
        self._graphs = {}
        self._seen = set()
        self.config = _Config(cfg)
        self._weights = weights
        self._seed = seed
        self._engine = None
        self._device = None
        self._lock = threading.Lock()

    # -- construction -------------------------------------------------------------
    @classmethod
    def from_pretrained(cls, name_or_path: str = "PekingU/rtdetr_v2_r101vd", synthetic: bool = False,
                        revision: str = "main", precision: str = "fp32", **kw):
        """What HF `from_pretrained` loads, offline: a local checkpoint directory, or a hub repo id
        resolved to its snapshot in the local HF cache (the reference image pre-fetches MODEL_NAME
        there: apps/spotter/Dockerfile:17 → download.py:23-27). A name that resolves to nothing
        raises OSError, as HF does offline. Deterministic synthetic weights only on explicit opt-in:
        `synthetic=True`, or a name of the form "synthetic:<preset>" (e.g. via MODEL_NAME).
        precision: the engine's operand precision (config.PRECISIONS); the drop-in serve.py passes
        os.environ.get("SPOTTER_PRECISION", "fp32") (deploy/rayservice-template.yaml sets "bf16" for C4).
        HF's own from_pretrained has no such input; the weights loaded are the same either way."""
        check_precision(precision)
        kw["precision"] = precision
        if name_or_path.startswith("synthetic:"):
            synthetic, name_or_path = True, name_or_path[len("synthetic:"):]
        if synthetic:
            preset = name_or_path if name_or_path in PRESETS else _preset_for(name_or_path).name
            return cls(PRESETS[preset], None, **kw)
        from .checkpoint import load_local, resolve_pretrained

        cfg, weights = load_local(resolve_pretrained(name_or_path, revision=revision))
        return cls(cfg, weights, **{k: v for k, v in kw.items() if k != "seed"})

    def _host_weights(self):
        if self._weights is None:
            from .weights import generate

            self._weights = generate(self.cfg, seed=self._seed)
        return self._weights

    # -- nn.Module-ish surface ----------------------------------------------------
    def to(self, device=None, *a, **k):
        dev = torch.device(device) if device is not None else None
        if dev is not None and dev.type == "cuda":
            self._device = dev
        return self  # cpu/mps requests (serve.py:61) keep the engine on the MI355X

    def eval(self):
        return self

    def __getstate__(self):
        st = self.__dict__.copy()
        st["_engine"] = None
        st["_batcher"] = None
        st["_lock"] = None
        st["_graphs"] = {}
        st["_seen"] = set()
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._lock = threading.Lock()

    @property
    def engine(self):
        if self._engine is None:
            with self._lock:
                if self._engine is None:
                    from .engine import Engine

                    dev = self._device or torch.device("cuda", torch.cuda.current_device())
                    self._engine = Engine(self.cfg, self._host_weights(), dev,
                                          precision=getattr(self, "precision", "fp32"))
        return self._engine

    # -- forward ------------------------------------------------------------------
    def __call__(self, pixel_values=None, pixel_mask=None, **kwargs):
        if pixel_values is None:
            raise ValueError("You have to specify either pixel_values or inputs_embeds")
        eng = self.engine
        if torch.is_tensor(pixel_values) and pixel_values.device != eng.dev:
            pixel_values = pixel_values.to(eng.dev)
        if getattr(self, "batching", False):
            if self._batcher is None:
                with self._lock:
                    if self._batcher is None:
                        from .batching import MicroBatcher

                        self._batcher = MicroBatcher(self._run, eng.dev, self.max_batch, self.max_wait_ms)
            logits, boxes = self._batcher(pixel_values.float())  # the batcher hands out owned rows
            return SpotterDetectionOutput(logits=logits, pred_boxes=boxes)
        logits, boxes = self._run(pixel_values)
        # own copies: the engine reuses its workspace on the next call
        return SpotterDetectionOutput(logits=logits.clone(), pred_boxes=boxes.clone())

    def _run(self, pixel_values):
        """One forward on the engine's stream; outputs live in engine / graph buffers until the next call."""
        eng = self.engine
        key = tuple(pixel_values.shape)
        if self.use_graphs and key[0] <= 4:
            # small batches are launch-bound: replay a captured hipGraph of the whole forward
            # (first call for a shape runs eager; the second captures)
            g = self._graphs.get(key)
            if g is None and key in self._seen:
                from .graph import GraphRunner

                g = self._graphs[key] = GraphRunner(eng, *key[:1], *key[2:])
            self._seen.add(key)
            if g is not None:
                return g(pixel_values.float())
        return eng.forward(pixel_values)

    forward = __call__
