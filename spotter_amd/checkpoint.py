"""Real-weight loader from a LOCAL directory: config.json +
model.safetensors in HF layout. 4.x key names are mapped to the 5.x names the
engine uses (transformers/conversion_mapping.py:1042-1047: out_proj→o_proj,
layers.N.fc1/fc2→layers.N.mlp.fc1/fc2, encoder.encoder.N.layers→encoder.aifi.N.layers).
Nothing is fetched; a hub name never reaches this module.
"""
from __future__ import annotations

import json
import os
import re

import numpy as np

from .config import COCO_ID2LABEL, SpotterConfig

_RENAMES = [
    (re.compile(r"\.out_proj\."), ".o_proj."),
    (re.compile(r"(layers\.\d+)\.fc([12])\."), r"\1.mlp.fc\2."),
    (re.compile(r"encoder\.encoder\.(\d+)\.layers\."), r"encoder.aifi.\1.layers."),
]


def rename_key(k: str) -> str:
    for pat, rep in _RENAMES:
        k = pat.sub(rep, k)
    return k


def config_from_hf(js: dict) -> SpotterConfig:
    bb = js.get("backbone_config") or {}
    id2label = {int(k): v for k, v in (js.get("id2label") or COCO_ID2LABEL).items()}
    return SpotterConfig(
        name=js.get("_name_or_path", "local"),
        depths=list(bb.get("depths", [3, 4, 23, 3])),
        hidden_sizes=list(bb.get("hidden_sizes", [256, 512, 1024, 2048])),
        layer_type=bb.get("layer_type", "bottleneck"),
        embedding_size=bb.get("embedding_size", 64),
        encoder_hidden_dim=js.get("encoder_hidden_dim", 256),
        encoder_ffn_dim=js.get("encoder_ffn_dim", 1024),
        encoder_attention_heads=js.get("encoder_attention_heads", 8),
        encoder_in_channels=list(js.get("encoder_in_channels", [512, 1024, 2048])),
        hidden_expansion=js.get("hidden_expansion", 1.0),
        d_model=js.get("d_model", 256),
        decoder_in_channels=list(js.get("decoder_in_channels", [256, 256, 256])),
        decoder_ffn_dim=js.get("decoder_ffn_dim", 1024),
        decoder_layers=js.get("decoder_layers", 6),
        decoder_attention_heads=js.get("decoder_attention_heads", 8),
        decoder_n_points=js.get("decoder_n_points", 4),
        decoder_offset_scale=js.get("decoder_offset_scale", 0.5),
        num_queries=js.get("num_queries", 300),
        num_labels=len(id2label),
        id2label=id2label,
    )


def load_local(path: str):
    from safetensors.numpy import load_file

    with open(os.path.join(path, "config.json")) as f:
        cfg = config_from_hf(json.load(f))
    raw = {}
    for fn in sorted(os.listdir(path)):
        if fn.endswith(".safetensors"):
            raw.update(load_file(os.path.join(path, fn)))
    w = {}
    for k, v in raw.items():
        k2 = rename_key(k)
        if k2.startswith(("class_embed.", "bbox_embed.")):
            k2 = "model.decoder." + k2
        w[k2] = np.ascontiguousarray(v, dtype=np.float32)
    return cfg, w
