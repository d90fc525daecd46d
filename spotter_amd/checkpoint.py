"""Real-weight loader: config.json + model.safetensors in HF layout,
from a local directory or from the local HF hub cache. 4.x key names are mapped to the
5.x names the engine uses (transformers/conversion_mapping.py:1042-1047: out_proj→o_proj,
layers.N.fc1/fc2→layers.N.mlp.fc1/fc2, encoder.encoder.N.layers→encoder.aifi.N.layers).

Hub names resolve the way `from_pretrained` resolves them offline: the reference image
pre-downloads MODEL_NAME into the HF cache at build time (reference
apps/spotter/Dockerfile:17 → src/spotter/download.py:23-27) and serve.py:203-204 loads
it by the same name. `resolve_pretrained` finds that snapshot
(<cache>/models--{org}--{name}/snapshots/<refs/main>/); nothing is fetched, and a name
that is not in the cache raises instead of running other weights.
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


_V4 = [
    (re.compile(r"\.o_proj\."), ".out_proj."),
    (re.compile(r"(layers\.\d+)\.mlp\.fc([12])\."), r"\1.fc\2."),
    (re.compile(r"encoder\.aifi\.(\d+)\.layers\."), r"encoder.encoder.\1.layers."),
]


def v4_key(k: str) -> str:
    """5.x module name → the 4.x checkpoint key (the inverse of rename_key; CM:1042-1047)."""
    for pat, rep in _V4:
        k = pat.sub(rep, k)
    return k


# Activation names the fused GEMM epilogue implements (transformers ACT2FN keys → sp_act).
SUPPORTED_ACTS = {"relu": "relu", "silu": "silu", "swish": "silu", "gelu": "gelu"}

# Inference-relevant RTDetrV2Config fields (configuration_rt_detr_v2.py:136-189) that the engine has ONE
# implementation of: a checkpoint with another value would compute something else, so it is refused.
_FIXED = {
    "encoder_layers": 1, "encode_proj_layers": [2], "normalize_before": False, "learn_initial_query": False,
    "with_box_refine": True, "decoder_method": "default", "use_focal_loss": True,
}
_FIXED_BACKBONE = {"num_channels": 3, "downsample_in_first_stage": False, "downsample_in_bottleneck": False}
# Fields that do not touch the inference arithmetic (losses, matcher, denoising, init, dropout in eval).
_IGNORED = {
    "initializer_range", "initializer_bias_prior_prob", "freeze_backbone_batch_norms", "dropout",
    "activation_dropout", "attention_dropout", "num_denoising", "label_noise_ratio", "box_noise_scale",
    "is_encoder_decoder", "matcher_alpha", "matcher_gamma", "matcher_class_cost", "matcher_bbox_cost",
    "matcher_giou_cost", "auxiliary_loss", "focal_loss_alpha", "focal_loss_gamma", "weight_loss_vfl",
    "weight_loss_bbox", "weight_loss_giou", "eos_coefficient", "tie_word_embeddings", "disable_custom_kernels",
    "model_type", "architectures", "transformers_version", "torch_dtype", "dtype", "id2label", "label2id",
    "_name_or_path", "backbone_config", "backbone", "use_timm_backbone", "use_pretrained_backbone",
    "backbone_kwargs", "return_dict", "output_hidden_states", "output_attentions", "use_return_dict",
    "pruned_heads", "chunk_size_feed_forward", "problem_type", "tokenizer_class", "num_labels",
}


# Generic PretrainedConfig attributes (generation / bookkeeping; configuration_utils.py) that some
# transformers versions write on save_pretrained. Underscore-prefixed bookkeeping keys
# (_attn_implementation_autoset, _commit_hash, …) are skipped by prefix.
_GENERIC = {
    "add_cross_attention", "bad_words_ids", "begin_suppress_tokens", "bos_token_id", "cross_attention_hidden_size",
    "decoder_start_token_id", "diversity_penalty", "do_sample", "early_stopping", "encoder_no_repeat_ngram_size",
    "eos_token_id", "exponential_decay_length_penalty", "finetuning_task", "forced_bos_token_id",
    "forced_eos_token_id", "is_decoder", "length_penalty", "max_length", "min_length", "no_repeat_ngram_size",
    "num_beam_groups", "num_beams", "num_return_sequences", "output_scores", "pad_token_id", "prefix",
    "remove_invalid_values", "repetition_penalty", "return_dict_in_generate", "sep_token_id", "suppress_tokens",
    "task_specific_params", "temperature", "tf_legacy_loss", "tie_encoder_decoder", "top_k", "top_p",
    "torchscript", "typical_p", "use_bfloat16", "label_smoothing", "use_cache",
}


class UnsupportedConfig(ValueError):
    """The checkpoint's config asks for arithmetic the MI355X path does not implement."""


def _act(js, key, default):
    name = js.get(key, default)
    if name not in SUPPORTED_ACTS:
        raise UnsupportedConfig(f"{key}={name!r}: the fused epilogue implements {sorted(SUPPORTED_ACTS)}")
    return SUPPORTED_ACTS[name]


def _size2(v):
    if v is None:
        return None
    if isinstance(v, int):
        return (v, v)
    return tuple(int(x) for x in v)


def config_from_hf(js: dict) -> SpotterConfig:
    """HF config.json (RTDetrV2Config with an rt_detr_resnet backbone_config) → SpotterConfig.
    Every field that changes inference is read; values the engine does not implement raise
    UnsupportedConfig instead of running a different model silently."""
    bb = dict(js.get("backbone_config") or {})
    if bb.get("model_type", "rt_detr_resnet") != "rt_detr_resnet" or js.get("use_timm_backbone"):
        raise UnsupportedConfig(f"backbone {bb.get('model_type')!r}: only the HF rt_detr_resnet backbone is implemented")
    for key, want in _FIXED.items():
        if key in js and js[key] != want:
            raise UnsupportedConfig(f"{key}={js[key]!r}: only {want!r} is implemented")
    for key, want in _FIXED_BACKBONE.items():
        if key in bb and bb[key] != want:
            raise UnsupportedConfig(f"backbone_config.{key}={bb[key]!r}: only {want!r} is implemented")
    out_idx = bb.get("out_indices")
    out_feat = bb.get("out_features")
    if out_idx is not None and list(out_idx) != [2, 3, 4] or (out_feat is not None and list(out_feat) != ["stage2", "stage3", "stage4"]):
        raise UnsupportedConfig(f"backbone out_indices {out_idx} / out_features {out_feat}: the encoder reads stages 2-4")
    depths = list(bb.get("depths", [3, 4, 6, 3]))  # RTDetrResNetConfig defaults (configuration_rt_detr_resnet.py:58-67)
    n_in = len(js.get("encoder_in_channels", [512, 1024, 2048]))
    dec_in = list(js.get("decoder_in_channels", [256, 256, 256]))
    for key in ("num_feature_levels", "decoder_n_levels"):
        if js.get(key, len(dec_in)) != len(dec_in):
            raise UnsupportedConfig(f"{key}={js[key]}: must equal len(decoder_in_channels)={len(dec_in)}")
    if n_in != 3 or len(dec_in) != 3:
        raise UnsupportedConfig("the hybrid encoder / decoder are implemented for 3 feature levels")
    n_points = js.get("decoder_n_points", 4)
    if not isinstance(n_points, int):
        raise UnsupportedConfig(f"decoder_n_points={n_points!r}: one point count for every level")
    id2label = {int(k): v for k, v in (js.get("id2label") or COCO_ID2LABEL).items()}
    return SpotterConfig(
        name=js.get("_name_or_path", "local"),
        depths=depths,
        hidden_sizes=list(bb.get("hidden_sizes", [256, 512, 1024, 2048])),
        layer_type=bb.get("layer_type", "bottleneck"),
        embedding_size=bb.get("embedding_size", 64),
        hidden_act=_act(bb, "hidden_act", "relu"),
        encoder_hidden_dim=js.get("encoder_hidden_dim", 256),
        encoder_ffn_dim=js.get("encoder_ffn_dim", 1024),
        encoder_attention_heads=js.get("encoder_attention_heads", 8),
        encoder_in_channels=list(js.get("encoder_in_channels", [512, 1024, 2048])),
        feat_strides=list(js.get("feat_strides", [8, 16, 32])),
        hidden_expansion=js.get("hidden_expansion", 1.0),
        positional_encoding_temperature=int(js.get("positional_encoding_temperature", 10000)),
        encoder_activation_function=_act(js, "encoder_activation_function", "gelu"),
        activation_function=_act(js, "activation_function", "silu"),
        eval_size=_size2(js.get("eval_size")),
        d_model=js.get("d_model", 256),
        decoder_in_channels=dec_in,
        decoder_ffn_dim=js.get("decoder_ffn_dim", 1024),
        decoder_activation_function=_act(js, "decoder_activation_function", "relu"),
        decoder_layers=js.get("decoder_layers", 6),
        decoder_attention_heads=js.get("decoder_attention_heads", 8),
        decoder_n_levels=len(dec_in),
        decoder_n_points=n_points,
        decoder_offset_scale=float(js.get("decoder_offset_scale", 0.5)),
        num_queries=js.get("num_queries", 300),
        anchor_image_size=_size2(js.get("anchor_image_size")),
        num_labels=len(id2label),
        layer_norm_eps=float(js.get("layer_norm_eps", 1e-5)),
        batch_norm_eps=float(js.get("batch_norm_eps", 1e-5)),
        id2label=id2label,
    )


def unknown_fields(js: dict) -> list:
    """config.json keys this loader neither reads nor knows to be inference-irrelevant."""
    read = {"encoder_hidden_dim", "encoder_ffn_dim", "encoder_attention_heads", "encoder_in_channels",
            "feat_strides", "hidden_expansion", "positional_encoding_temperature", "encoder_activation_function",
            "activation_function", "eval_size", "d_model", "decoder_in_channels", "decoder_ffn_dim",
            "decoder_activation_function", "decoder_layers", "decoder_attention_heads", "decoder_n_levels",
            "num_feature_levels", "decoder_n_points", "decoder_offset_scale", "num_queries", "anchor_image_size",
            "layer_norm_eps", "batch_norm_eps", "hidden_size", "num_attention_heads"}
    return sorted(k for k in js if k not in read and k not in _FIXED and k not in _IGNORED
                  and k not in _GENERIC and not k.startswith("_"))


def hub_cache_dirs() -> list:
    """The HF hub cache directories `from_pretrained` would look in, in huggingface_hub's order
    (constants.py: HF_HUB_CACHE, else HF_HOME/hub, else ~/.cache/huggingface/hub; the
    deprecated TRANSFORMERS_CACHE / HUGGINGFACE_HUB_CACHE names too)."""
    out = []
    for var in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE", "TRANSFORMERS_CACHE"):
        if os.environ.get(var):
            out.append(os.path.expanduser(os.environ[var]))
    home = os.environ.get("HF_HOME") or os.path.join(
        os.environ.get("XDG_CACHE_HOME") or os.path.join(os.path.expanduser("~"), ".cache"), "huggingface")
    out.append(os.path.join(os.path.expanduser(home), "hub"))
    seen = []
    for d in out:
        if d not in seen:
            seen.append(d)
    return seen


def resolve_pretrained(name_or_path: str, revision: str = "main", need: str = "config.json") -> str:
    """A local directory → itself; a hub repo id ("PekingU/rtdetr_v2_r101vd") → its snapshot
    directory in the local HF cache (refs/<revision> → snapshots/<commit>, or a commit hash given
    as revision). Raises OSError naming the searched paths when no snapshot holding `need` exists:
    there is no network and no silent substitute."""
    if os.path.isdir(name_or_path):
        if need and not os.path.isfile(os.path.join(name_or_path, need)):
            # an existing but empty directory (e.g. an image built without its checkpoint context) is
            # not a checkpoint: refuse here rather than fail later in every replica
            raise OSError(f"{name_or_path!r} is a directory without {need}: not a checkpoint")
        return name_or_path
    repo = name_or_path.strip("/")
    if repo.count("/") > 1 or not repo:
        raise OSError(f"{name_or_path!r} is neither a local directory nor a hub repo id")
    folder = "models--" + repo.replace("/", "--")
    tried = []
    for cache in hub_cache_dirs():
        base = os.path.join(cache, folder)
        tried.append(base)
        if not os.path.isdir(base):
            continue
        commit = revision
        ref = os.path.join(base, "refs", revision)
        if os.path.isfile(ref):
            with open(ref) as f:
                commit = f.read().strip()
        snap = os.path.join(base, "snapshots", commit)
        if os.path.isfile(os.path.join(snap, need)):
            return snap
    raise OSError(f"{name_or_path!r}: no local directory and no cached snapshot with {need} "
                  f"(searched {tried}; nothing is downloaded — pre-fetch it as the reference's "
                  f"download.py does, or pass a checkpoint directory)")


# Unknown keys named like RTDetrV2Config model fields (configuration_rt_detr_v2.py:136-189 uses these
# prefixes for every architecture field): a later transformers version adding one would change the
# arithmetic, so it is refused rather than ignored.
_MODEL_FIELD_PREFIXES = ("encoder", "decoder", "backbone", "anchor", "num_", "d_model", "feat_", "with_", "layer_")


def check_fields(js: dict, strict: bool = False) -> None:
    """Refuse unknown config.json keys that look like model fields (always) or any unknown key
    (strict=True, what the image build uses); other unknown keys only warn."""
    unk = unknown_fields(js)
    model_like = [k for k in unk if k.startswith(_MODEL_FIELD_PREFIXES)]
    if model_like or (strict and unk):
        raise UnsupportedConfig(f"config.json fields this loader does not implement: {model_like or unk}")
    if unk:
        import warnings

        warnings.warn(f"config.json fields this loader does not read (assumed not to change inference): {unk}",
                      stacklevel=3)


def load_local(path: str, strict: bool = False):
    from safetensors.numpy import load_file

    with open(os.path.join(path, "config.json")) as f:
        js = json.load(f)
    check_fields(js, strict)
    cfg = config_from_hf(js)
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


def hf_config_dict(cfg: SpotterConfig) -> dict:
    """The config.json HF writes for this model (RTDetrV2Config + rt_detr_resnet backbone_config), as
    far as inference reads it; tests/test_host.py checks it against HF's own save_pretrained."""
    kw = cfg.to_hf_kwargs()
    js = dict(kw["model"])
    js["id2label"] = {str(i): n for i, n in cfg.id2label.items()}
    js["label2id"] = {n: i for i, n in cfg.id2label.items()}
    js["eval_size"] = list(cfg.eval_size) if cfg.eval_size else None
    js["anchor_image_size"] = list(cfg.anchor_image_size) if cfg.anchor_image_size else None
    js.update(model_type="rt_detr_v2", architectures=["RTDetrV2ForObjectDetection"], d_model=cfg.d_model,
              decoder_n_levels=cfg.decoder_n_levels, num_feature_levels=cfg.decoder_n_levels,
              encoder_layers=1, encode_proj_layers=[2], normalize_before=False, with_box_refine=True,
              learn_initial_query=False, decoder_method="default", use_focal_loss=True)
    bb = dict(kw["backbone"], model_type="rt_detr_resnet", num_channels=3, downsample_in_first_stage=False,
              downsample_in_bottleneck=False, out_features=["stage2", "stage3", "stage4"])
    js["backbone_config"] = bb
    return js


def save_local(path: str, cfg: SpotterConfig, weights: dict) -> None:
    """Write a local checkpoint directory the way a 4.x HF checkpoint looks (config.json +
    model.safetensors with 4.x key names): what load_local / from_pretrained(dir) read."""
    from safetensors.numpy import save_file

    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(hf_config_dict(cfg), f, indent=1)
    save_file({v4_key(k): np.ascontiguousarray(v, dtype=np.float32) for k, v in weights.items()},
              os.path.join(path, "model.safetensors"))


def check_image_model(name: str) -> str:
    """What the image build runs on its ENV MODEL_NAME (deploy/Dockerfile.rocm): a synthetic: name is
    accepted as is; anything else must resolve to a directory holding config.json whose every field
    the loader implements (strict). Returns the resolved directory; raises otherwise."""
    if name.startswith("synthetic:"):
        return name
    d = resolve_pretrained(name)
    with open(os.path.join(d, "config.json")) as f:
        js = json.load(f)
    check_fields(js, strict=True)
    config_from_hf(js)
    return d


if __name__ == "__main__":
    import sys

    if len(sys.argv) != 3 or sys.argv[1] != "--check":
        sys.exit("usage: python -m spotter_amd.checkpoint --check <MODEL_NAME>")
    print("weights:", check_image_model(sys.argv[2]))
