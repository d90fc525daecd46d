"""TEST INFRASTRUCTURE ONLY — the reference's own CPU path, built with our weights.

The reference (apps/spotter/src/spotter/serve.py:199-204) runs
`AutoModelForObjectDetection.from_pretrained("PekingU/rtdetr_v2_r101vd")` and
`AutoImageProcessor` from HF transformers (pinned 4.50.3 at
apps/spotter/uv.lock:1235-1236; 5.15.0 is what this image ships — same math,
renamed modules). Real weights are unreachable offline, so
this builds the same HF classes from a local config and loads the synthetic
weights of spotter_amd.weights.generate(). Used to make golden fixtures
(oracle/make_goldens.py) and as bench.py's cpu_baseline ("reference" kind).
"""
from __future__ import annotations

import numpy as np
import torch


def build_hf_model(cfg, weights: dict):
    from transformers import RTDetrResNetConfig, RTDetrV2Config, RTDetrV2ForObjectDetection

    kw = cfg.to_hf_kwargs()
    bb = RTDetrResNetConfig(**kw["backbone"])
    hcfg = RTDetrV2Config(backbone_config=bb, **kw["model"])
    model = RTDetrV2ForObjectDetection(hcfg).eval()
    sd = model.state_dict()
    new = {}
    for k, v in sd.items():
        if k.endswith("num_batches_tracked"):
            new[k] = v
            continue
        src = k
        if k.startswith("class_embed.") or k.startswith("bbox_embed."):
            src = "model.decoder." + k  # tied alias of model.decoder.{class,bbox}_embed
        arr = weights[src]
        if tuple(arr.shape) != tuple(v.shape):
            raise ValueError(f"shape mismatch {k}: {arr.shape} vs {tuple(v.shape)}")
        new[k] = torch.from_numpy(np.array(arr, copy=True))
    extra = set(weights) - {("model.decoder." + k if k.startswith(("class_embed.", "bbox_embed.")) else k) for k in sd}
    if extra:
        raise ValueError(f"generator keys unknown to HF: {sorted(extra)[:5]}")
    model.load_state_dict(new, strict=True)
    return model


def build_hf_processor():
    from transformers.models.rt_detr.image_processing_pil_rt_detr import RTDetrImageProcessorPil

    return RTDetrImageProcessorPil()
