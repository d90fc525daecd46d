"""Parameter inventory, deterministic synthetic weights, and device-layout packing.

The canonical weight dictionary is keyed by HF transformers 5.x
`RTDetrV2ForObjectDetection.state_dict()` names (fp32 numpy arrays), so the
same dictionary feeds (a) the HF model on CPU (oracle/hf_ref.py, goldens and
CPU baseline) and (b) the MI355X engine after `pack_for_device`.

Architecture restated from:
  * backbone  transformers/models/rt_detr/modeling_rt_detr_resnet.py:38-310
    (conv layer :38-68, stem :71-114, shortcut :117-132, basic :135-175,
     bottleneck :179-231, stage :234-268, encoder :272-310)
  * encoder/decoder transformers/models/rt_detr_v2/modeling_rt_detr_v2.py
    (input proj :1350-1360, AIFI :1041-1095, CCFM :1113-1209, enc heads
     :1376-1381, decoder input proj :1389-1407, decoder :555-661, heads
     :1777-1787)

No real checkpoint is reachable offline, so parity runs on
synthetic weights from `generate()`: per-tensor numpy PCG64 streams seeded from
crc32(name) — identical on any host with numpy ≥ 1.17.
"""
from __future__ import annotations

import math
import zlib
from collections import OrderedDict

import numpy as np

from .config import SpotterConfig

# kinds: conv | bn | linear_w | linear_b | ln_w | ln_b | misc
_BN = ("weight", "bias", "running_mean", "running_var")


def _conv_bn(specs, prefix, cin, cout, k, conv_name="convolution", bn_name="normalization",
             role="plain"):
    specs.append((f"{prefix}.{conv_name}.weight", (cout, cin, k, k), ("conv", role)))
    for f in _BN:
        specs.append((f"{prefix}.{bn_name}.{f}", (cout,), ("bn_" + f, role)))


def _linear(specs, prefix, fin, fout, role="plain"):
    specs.append((f"{prefix}.weight", (fout, fin), ("linear_w", role)))
    specs.append((f"{prefix}.bias", (fout,), ("linear_b", role)))


def _ln(specs, prefix, n):
    specs.append((f"{prefix}.weight", (n,), ("ln_w", "plain")))
    specs.append((f"{prefix}.bias", (n,), ("ln_b", "plain")))


def backbone_plan(cfg: SpotterConfig):
    """Yields (stage, layer, kind, cin, cout, stride, shortcut) per residual block.

    shortcut ∈ {"identity", "conv", "avgconv"} (RN:135-231; "avgconv" is the vd
    AvgPool2d(2,2,ceil_mode=True) + 1×1 conv, RN:199-207 / RN:150-158).
    """
    plan = []
    cin = cfg.embedding_size
    for s, (cout, depth) in enumerate(zip(cfg.hidden_sizes, cfg.depths)):
        stride = 1 if s == 0 else 2  # downsample_in_first_stage=False (RN:277-285)
        for i in range(depth):
            bin_ = cin if i == 0 else cout
            bst = stride if i == 0 else 1
            if cfg.layer_type == "bottleneck":
                apply = (bin_ != cout) or bst != 1
                if bst == 2:
                    sc = "avgconv" if apply else "avgonly"
                else:
                    sc = "conv" if apply else "identity"
            else:  # basic: only the first layer of a stage has a shortcut (RN:253-256)
                if i == 0:
                    sc = "avgconv" if bin_ != cout else "conv"
                else:
                    sc = "identity"
            plan.append((s, i, cfg.layer_type, bin_, cout, bst, sc))
        cin = cout
    return plan


def param_specs(cfg: SpotterConfig):
    """Ordered (key, shape, (kind, role)) for every tensor in the HF state dict."""
    sp = []
    bb = "model.backbone.model"
    e = cfg.embedding_size
    # stem (RN:78-103)
    _conv_bn(sp, f"{bb}.embedder.embedder.0", 3, e // 2, 3)
    _conv_bn(sp, f"{bb}.embedder.embedder.1", e // 2, e // 2, 3)
    _conv_bn(sp, f"{bb}.embedder.embedder.2", e // 2, e, 3)
    for (s, i, lt, cin, cout, st, sc) in backbone_plan(cfg):
        p = f"{bb}.encoder.stages.{s}.layers.{i}"
        if sc == "conv":
            _conv_bn(sp, f"{p}.shortcut", cin, cout, 1)
        elif sc == "avgconv":
            _conv_bn(sp, f"{p}.shortcut.1", cin, cout, 1)
        if lt == "bottleneck":
            red = cout // 4
            _conv_bn(sp, f"{p}.layer.0", cin, red, 1)
            _conv_bn(sp, f"{p}.layer.1", red, red, 3)
            _conv_bn(sp, f"{p}.layer.2", red, cout, 1, role="resid_last")
        else:
            _conv_bn(sp, f"{p}.layer.0", cin, cout, 3)
            _conv_bn(sp, f"{p}.layer.1", cout, cout, 3, role="resid_last")
    H = cfg.encoder_hidden_dim
    for l, c in enumerate(cfg.encoder_in_channels):
        _conv_bn(sp, f"model.encoder_input_proj.{l}", c, H, 1, conv_name="0", bn_name="1")
    a = "model.encoder.aifi.0.layers.0"
    for n in ("k_proj", "v_proj", "q_proj", "o_proj"):
        _linear(sp, f"{a}.self_attn.{n}", H, H)
    _ln(sp, f"{a}.self_attn_layer_norm", H)
    _linear(sp, f"{a}.mlp.fc1", H, cfg.encoder_ffn_dim)
    _linear(sp, f"{a}.mlp.fc2", cfg.encoder_ffn_dim, H)
    _ln(sp, f"{a}.final_layer_norm", H)
    hid = int(H * cfg.hidden_expansion)

    def csp(prefix):
        _conv_bn(sp, f"{prefix}.conv1", 2 * H, hid, 1, conv_name="conv", bn_name="norm")
        _conv_bn(sp, f"{prefix}.conv2", 2 * H, hid, 1, conv_name="conv", bn_name="norm")
        for b in range(3):
            _conv_bn(sp, f"{prefix}.bottlenecks.{b}.conv1", hid, hid, 3, conv_name="conv",
                     bn_name="norm")
            _conv_bn(sp, f"{prefix}.bottlenecks.{b}.conv2", hid, hid, 1, conv_name="conv",
                     bn_name="norm")
        if hid != H:
            _conv_bn(sp, f"{prefix}.conv3", hid, H, 1, conv_name="conv", bn_name="norm")

    nl = len(cfg.encoder_in_channels)
    for i in range(nl - 1):
        _conv_bn(sp, f"model.encoder.lateral_convs.{i}", H, H, 1, conv_name="conv", bn_name="norm")
        csp(f"model.encoder.fpn_blocks.{i}")
    for i in range(nl - 1):
        _conv_bn(sp, f"model.encoder.downsample_convs.{i}", H, H, 3, conv_name="conv",
                 bn_name="norm")
        csp(f"model.encoder.pan_blocks.{i}")
    D = cfg.d_model
    sp.append(("model.denoising_class_embed.weight", (cfg.num_labels + 1, D), ("misc", "dn")))
    _linear(sp, "model.enc_output.0", D, D)
    _ln(sp, "model.enc_output.1", D)
    _linear(sp, "model.enc_score_head", D, cfg.num_labels, role="cls")
    _linear(sp, "model.enc_bbox_head.layers.0", D, D)
    _linear(sp, "model.enc_bbox_head.layers.1", D, D)
    _linear(sp, "model.enc_bbox_head.layers.2", D, 4, role="box_last")
    for l, c in enumerate(cfg.decoder_in_channels):
        _conv_bn(sp, f"model.decoder_input_proj.{l}", c, D, 1, conv_name="0", bn_name="1")
    nH, nL, nP = cfg.decoder_attention_heads, cfg.decoder_n_levels, cfg.decoder_n_points
    for j in range(cfg.decoder_layers):
        p = f"model.decoder.layers.{j}"
        for n in ("k_proj", "v_proj", "q_proj"):
            _linear(sp, f"{p}.self_attn.{n}", D, D)
        _linear(sp, f"{p}.self_attn.o_proj", D, D, role="resid_out")
        _ln(sp, f"{p}.self_attn_layer_norm", D)
        sp.append((f"{p}.encoder_attn.n_points_scale", (nL * nP,), ("misc", "npscale")))
        _linear(sp, f"{p}.encoder_attn.sampling_offsets", D, nH * nL * nP * 2, role="msda_off")
        _linear(sp, f"{p}.encoder_attn.attention_weights", D, nH * nL * nP, role="msda_aw")
        _linear(sp, f"{p}.encoder_attn.value_proj", D, D)
        _linear(sp, f"{p}.encoder_attn.output_proj", D, D, role="resid_out")
        _ln(sp, f"{p}.encoder_attn_layer_norm", D)
        _linear(sp, f"{p}.mlp.fc1", D, cfg.decoder_ffn_dim)
        _linear(sp, f"{p}.mlp.fc2", cfg.decoder_ffn_dim, D, role="resid_out")
        _ln(sp, f"{p}.final_layer_norm", D)
    _linear(sp, "model.decoder.query_pos_head.layers.0", 4, 2 * D)
    _linear(sp, "model.decoder.query_pos_head.layers.1", 2 * D, D)
    for j in range(cfg.decoder_layers):
        _linear(sp, f"model.decoder.class_embed.{j}", D, cfg.num_labels, role="cls")
    for j in range(cfg.decoder_layers):
        _linear(sp, f"model.decoder.bbox_embed.{j}.layers.0", D, D)
        _linear(sp, f"model.decoder.bbox_embed.{j}.layers.1", D, D)
        _linear(sp, f"model.decoder.bbox_embed.{j}.layers.2", D, 4, role="box_last")
    return sp


# Class heads: logits = CLS_GAIN·w·h + CLS_BIAS with unit-variance LayerNorm'd h, so a
# few per mille of the 24,000 (query, class) pairs clear the 0.5 threshold with a
# spread of scores up to ~0.95 (SURVEY.md §7 "No real weights").
# RESID_GAIN scales the decoder's residual-branch outputs (self-attn o_proj, MSDA
# output_proj, FFN fc2), the usual scaled-residual init: at 1.0 each decoder layer
# pulls the 300 queries towards one vector (uniform random attention averages them),
# so logits vary by class only and the detections are all-or-nothing per class.
CLS_BIAS = -8.0
# Per-preset shift of the class-head biases: R101vd at -8 left its goldens with 0-8 detections per
# image, too few to pin the threshold behaviour; -7 gives 32-259 per 640² golden image with 11-32
# scores within 0.05 of the 0.5 threshold ("parity margins"). A uniform shift of every
# class bias moves all logits alike, so the encoder's top-300 query selection is unchanged.
CLS_BIAS_BY_PRESET = {"r101vd": -7.0}
CLS_GAIN = 3.0
RESID_GAIN = 0.3


def _msda_grid_bias(nH, nL, nP):
    # Same sampling-offset pattern HF initialises (modeling_rt_detr_v2.py:464-478).
    thetas = np.arange(nH, dtype=np.float64) * (2.0 * math.pi / nH)
    g = np.stack([np.cos(thetas), np.sin(thetas)], -1)
    g = g / np.abs(g).max(-1, keepdims=True)
    g = np.tile(g.reshape(nH, 1, 1, 2), (1, nL, nP, 1))
    for i in range(nP):
        g[:, :, i, :] *= i + 1
    return g.reshape(-1).astype(np.float32)


def generate(cfg: SpotterConfig, seed: int = 0) -> "OrderedDict[str, np.ndarray]":
    """Deterministic, well-conditioned synthetic weights (HF key names, fp32)."""
    cls_bias = CLS_BIAS_BY_PRESET.get(cfg.name, CLS_BIAS)
    out = OrderedDict()
    for key, shape, (kind, role) in param_specs(cfg):
        rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
        if kind == "conv":
            fan_in = shape[1] * shape[2] * shape[3]
            w = rng.standard_normal(shape, dtype=np.float32)
            # Zero-mean filters reject the DC of the previous activation, so the
            # synthetic net keeps spatial contrast instead of collapsing every
            # position (and hence every decoder query) onto one vector.
            w = w - w.reshape(shape[0], -1).mean(1).reshape(-1, 1, 1, 1)
            w = w * np.float32(math.sqrt(2.0 / fan_in))
        elif kind == "bn_weight":
            lo, hi = (0.1, 0.3) if role == "resid_last" else (1.0, 1.6)
            if key.startswith("model.encoder."):
                # CCFM: RepVGG sums two branches and CSP adds two paths per block, so unit-gain
                # BN would grow activations ~1000x over FPN+PAN and make the net chaotic.
                lo, hi = (0.3, 0.6)
            w = rng.uniform(lo, hi, shape).astype(np.float32)
        elif kind == "bn_bias":
            w = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        elif kind == "bn_running_mean":
            w = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        elif kind == "bn_running_var":
            w = rng.uniform(0.5, 2.0, shape).astype(np.float32)
        elif kind == "linear_w":
            std = 1.0 / math.sqrt(shape[1])
            if role in ("box_last",):
                std *= 0.05
            elif role == "cls":
                std *= CLS_GAIN
            elif role == "resid_out":
                std *= RESID_GAIN
            elif role == "msda_off":
                std *= 0.02
            w = (rng.standard_normal(shape) * std).astype(np.float32)
        elif kind == "linear_b":
            if role == "cls":
                w = (cls_bias + rng.standard_normal(shape) * 0.2).astype(np.float32)
            elif role == "msda_off":
                nH, nL, nP = cfg.decoder_attention_heads, cfg.decoder_n_levels, cfg.decoder_n_points
                w = _msda_grid_bias(nH, nL, nP)
            elif role == "box_last":
                w = (rng.standard_normal(shape) * 0.05).astype(np.float32)
            else:
                w = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        elif kind == "ln_w":
            w = rng.uniform(0.8, 1.2, shape).astype(np.float32)
        elif kind == "ln_b":
            w = (rng.standard_normal(shape) * 0.05).astype(np.float32)
        elif role == "npscale":
            w = np.array([1.0 / cfg.decoder_n_points] * shape[0], dtype=np.float32)
        else:  # denoising embedding: training only
            w = (rng.standard_normal(shape) * 0.02).astype(np.float32)
        out[key] = np.ascontiguousarray(w, dtype=np.float32)
    return out


def num_params(cfg: SpotterConfig) -> int:
    """Parameter count as HF reports it (tied head aliases counted once)."""
    n = 0
    for key, shape, (kind, role) in param_specs(cfg):
        if kind.startswith("bn_running") or role == "npscale":
            continue
        n += int(np.prod(shape))
    return n


def shift_class_bias(weights: dict, delta: float) -> dict:
    """A copy of `weights` with every class-head bias (enc_score_head and each decoder class_embed) moved by
    `delta`: all class logits shift alike, so the encoder's top-300 query selection is unchanged and only
    how many scores clear the 0.5 threshold moves (used by the 1280² goldens, whose score distribution sits
    lower than at 640²: tests/golden/r101vd_1280.npz stores the shift it was made with)."""
    out = dict(weights)
    for k in weights:
        if k.endswith(".bias") and (k.startswith("model.enc_score_head") or ".class_embed." in k):
            out[k] = (weights[k] + np.float32(delta)).astype(np.float32)
    return out
