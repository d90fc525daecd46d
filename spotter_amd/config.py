"""Model hyper-parameters for the RT-DETRv2 presets the bench and tests use.

Mirrors the fields of HF `RTDetrV2Config` (transformers/models/rt_detr_v2/
configuration_rt_detr_v2.py:136-189) and `RTDetrResNetConfig`
(transformers/models/rt_detr/configuration_rt_detr_resnet.py:58-67) that the
inference path reads. Presets reproduce the published parameter counts
(R101vd 76,556,268; R18vd 20,174,608 — SURVEY.md §6, §8 D1.2).
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field

# HF COCO label names in RT-DETR's contiguous 0..79 order (the names that
# AMENITIES_MAPPING keys use, reference serve.py:31-59: "tv", "couch",
# "dining table", "hair drier" …).
COCO_NAMES = [
    "person", "bicycle", "car", "motorcycle", "airplane", "bus", "train", "truck", "boat",
    "traffic light", "fire hydrant", "stop sign", "parking meter", "bench", "bird", "cat",
    "dog", "horse", "sheep", "cow", "elephant", "bear", "zebra", "giraffe", "backpack",
    "umbrella", "handbag", "tie", "suitcase", "frisbee", "skis", "snowboard", "sports ball",
    "kite", "baseball bat", "baseball glove", "skateboard", "surfboard", "tennis racket",
    "bottle", "wine glass", "cup", "fork", "knife", "spoon", "bowl", "banana", "apple",
    "sandwich", "orange", "broccoli", "carrot", "hot dog", "pizza", "donut", "cake", "chair",
    "couch", "potted plant", "bed", "dining table", "toilet", "tv", "laptop", "mouse",
    "remote", "keyboard", "cell phone", "microwave", "oven", "toaster", "sink",
    "refrigerator", "book", "clock", "vase", "scissors", "teddy bear", "hair drier",
    "toothbrush",
]
COCO_ID2LABEL = {i: n for i, n in enumerate(COCO_NAMES)}


@dataclass
class SpotterConfig:
    name: str = "r101vd"
    # backbone (RTDetrResNetConfig)
    depths: list = field(default_factory=lambda: [3, 4, 23, 3])
    hidden_sizes: list = field(default_factory=lambda: [256, 512, 1024, 2048])
    layer_type: str = "bottleneck"
    embedding_size: int = 64
    hidden_act: str = "relu"  # backbone convs (RN:85-99, 168, 223)
    # hybrid encoder
    encoder_hidden_dim: int = 384
    encoder_ffn_dim: int = 2048
    encoder_attention_heads: int = 8
    encoder_in_channels: list = field(default_factory=lambda: [512, 1024, 2048])
    feat_strides: list = field(default_factory=lambda: [8, 16, 32])
    hidden_expansion: float = 1.0
    positional_encoding_temperature: int = 10000
    encoder_activation_function: str = "gelu"  # AIFI FFN (M2:853)
    activation_function: str = "silu"  # CCFM conv-norm layers (M2:915, 937, 1140, 1156)
    eval_size: tuple | None = None  # set: AIFI runs without the sine position embedding (M2:1073-1081)
    # decoder
    d_model: int = 256
    decoder_in_channels: list = field(default_factory=lambda: [384, 384, 384])
    decoder_ffn_dim: int = 1024
    decoder_activation_function: str = "relu"  # decoder FFN (M2:358)
    decoder_layers: int = 6
    decoder_attention_heads: int = 8
    decoder_n_levels: int = 3
    decoder_n_points: int = 4
    decoder_offset_scale: float = 0.5
    num_queries: int = 300
    anchor_image_size: tuple | None = None  # set: anchors from this size / feat_strides (M2:1384, 1451-1456)
    num_labels: int = 80
    layer_norm_eps: float = 1e-5
    batch_norm_eps: float = 1e-5
    image_size: int = 640
    id2label: dict = field(default_factory=lambda: dict(COCO_ID2LABEL))

    @property
    def label2id(self):
        return {v: k for k, v in self.id2label.items()}

    def replace(self, **kw) -> "SpotterConfig":
        return dataclasses.replace(self, **kw)

    def to_hf_kwargs(self) -> dict:
        """Keyword arguments for HF RTDetrV2Config / RTDetrResNetConfig (oracle side)."""
        return dict(
            backbone=dict(depths=list(self.depths), hidden_sizes=list(self.hidden_sizes),
                          layer_type=self.layer_type, embedding_size=self.embedding_size,
                          hidden_act=self.hidden_act, out_indices=[2, 3, 4]),
            model=dict(encoder_hidden_dim=self.encoder_hidden_dim,
                       encoder_ffn_dim=self.encoder_ffn_dim,
                       encoder_in_channels=list(self.encoder_in_channels),
                       decoder_in_channels=list(self.decoder_in_channels),
                       hidden_expansion=self.hidden_expansion,
                       decoder_layers=self.decoder_layers, d_model=self.d_model,
                       decoder_ffn_dim=self.decoder_ffn_dim, num_queries=self.num_queries,
                       num_labels=self.num_labels, id2label=dict(self.id2label),
                       encoder_attention_heads=self.encoder_attention_heads,
                       decoder_attention_heads=self.decoder_attention_heads,
                       decoder_n_points=self.decoder_n_points, decoder_offset_scale=self.decoder_offset_scale,
                       feat_strides=list(self.feat_strides),
                       positional_encoding_temperature=int(self.positional_encoding_temperature),
                       layer_norm_eps=self.layer_norm_eps, batch_norm_eps=self.batch_norm_eps,
                       encoder_activation_function=self.encoder_activation_function,
                       activation_function=self.activation_function,
                       decoder_activation_function=self.decoder_activation_function,
                       eval_size=list(self.eval_size) if self.eval_size else None,
                       anchor_image_size=list(self.anchor_image_size) if self.anchor_image_size else None),
        )

    def to_json(self) -> str:
        return json.dumps(dataclasses.asdict(self))


R101VD = SpotterConfig()
R18VD = SpotterConfig(
    name="r18vd", depths=[2, 2, 2, 2], hidden_sizes=[64, 128, 256, 512], layer_type="basic",
    encoder_hidden_dim=256, encoder_ffn_dim=1024, encoder_in_channels=[128, 256, 512],
    decoder_in_channels=[256, 256, 256], decoder_layers=3, hidden_expansion=0.5,
)
PRESETS = {"r101vd": R101VD, "r18vd": R18VD}

# Engine precision names → (conv GEMM operand mode, linear GEMM operand mode); engine.py documents the modes.
# Here (no GPU import) so the drop-in can refuse an unknown SPOTTER_PRECISION at serve.py import time.
PRECISIONS = {
    "fp32": ("x3", "x3"),
    "fp32-mfma": ("f32", "f32"),
    "bf16": ("bf16", "bf16"),
    "bf16-convs": ("bf16", "x3"),
    "bf16-all": ("bf16", "bf16"),  # round-2 name of "bf16"
}
PRECISION_ENV = "SPOTTER_PRECISION"


def check_precision(precision: str) -> str:
    """A PRECISIONS key, else ValueError naming the accepted values (and the env variable that set it)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision {precision!r} (e.g. from {PRECISION_ENV}) must be one of {sorted(PRECISIONS)}")
    return precision
