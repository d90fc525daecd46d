"""The RT-DETRv2 forward on MI355X: weight packing + launch orchestration.

Data layout in HBM (all fp32): activations NHWC (`[B, H, W, C]` = `[B·H·W, C]`
rows), conv weights `[Cout][KH][KW][Cin]`, linear weights `[N][K]` (PyTorch's
own), BatchNorm folded to per-channel (scale, shift) applied in the GEMM
epilogue. Buffers are allocated once per (batch, size) and reused, so a
forward allocates nothing (hipGraph-capturable). Fusions relative to the HF
graph (transformers/models/rt_detr_v2/modeling_rt_detr_v2.py = M2,
models/rt_detr/modeling_rt_detr_resnet.py = RN):

* conv + BN + activation + residual in one GEMM epilogue (RN:225-231, M2:921-923)
* CSPRep conv1 ‖ conv2 as one GEMM (same input, M2:949-951); the CSP sum
  h1 + h2 as the last RepVGG block's post-activation residual (M2:952)
* encoder_input_proj / lateral / downsample convs write straight into the
  concat buffers (M2:1193, M2:1205); decoder_input_proj writes straight into
  source_flatten (M2:1553-1555) through the grouped output row map
* query selection's valid-mask multiply as a GEMM row scale (M2:1592)
* q_proj ‖ k_proj as one GEMM with the +pos addend fused in the A loader
  (M2:313-317); sampling_offsets ‖ attention_weights as one GEMM (M2:196-203)
* all six decoder value_proj GEMMs as one N = 6·256 GEMM over source_flatten
* enc_bbox_head evaluated only on the 300 selected rows (its other rows are
  never read, M2:1601-1603) and class_embed only for the last decoder layer
  (the only logits the output uses, M2:1880); both are dead-code elimination
  with identical per-row math.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import ops
from .config import PRECISIONS, SpotterConfig, check_precision
from .ops import V, view
from .weights import backbone_plan


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


bf16_bits = ops.bf16_bits  # fp32 → bf16 bit patterns, RNE (host, weight-pack time)


# precision → (conv GEMM operand mode, linear GEMM operand mode):
#   "f32"  fp32 MFMA (v_mfma_f32_32x32x2_f32, an exact fmaf chain),
#   "x3"   fp32 operands as hi/mid/lo bf16 splits on bf16 MFMA (SP_PREC_F32X3; fp32-accurate),
#   "bf16" bf16 operands, fp32 accumulate (the separately reported bf16 variant).
# (Cout, K, small_m) layers inside the thin / small-M rule above where the split kernel measured faster
# than the fp32 MFMA at bs32 (tools/tune_conv.py --cross, profiles/r2/tune_bs32_r101vd_cross_r2.json; each
# side with its best tile): the stage-0 1×1 expand (0.374 vs 0.401 ms) and the decoder's 9600-row
# FFN / value / query-pos / box-head linears (1.04-1.26×). Both modes are fp32-accurate.
ATTN_BF16 = True  # the bf16 variant's AIFI / decoder self-attention on sp_attention_bf16

_X3_FASTER = {(256, 64, False), (256, 1024, True), (1024, 256, True), (512, 256, True), (256, 512, True),
              (288, 256, True), (4, 256, False)}

# The bf16 variant ("bf16") runs every conv and linear on bf16 operands; the stem's first conv stays on
# the direct fp32 kernel (_direct_stem). Measured against the HF fp32 goldens (profiles/r3/bf16/, R101vd
# bs32): recall 0.971, p95 |dscore| 0.012, AP 0.958 — closer than round 2's bf16 mode with x3 linears and
# a bf16 stem (0.906 / 0.052 / 0.916: the bf16-rounded raw pixels of the stem conv were most of the error),
# at 1.07x (C2) / 1.10x (C3) its speed. "bf16-convs" keeps the linears on the fp32-accurate split.
# The precision names and their (conv, linear) operand modes: config.PRECISIONS.


def _wkw(wq):
    """ops.conv2d keyword for a packed GEMM weight form (see Engine._wq)."""
    if wq is None:
        return {}
    if wq.dim() == 2 and wq.shape[0] == 3:
        return {"wt_planes": wq}
    return {"wt16": wq}


class ConvW:
    __slots__ = ("w", "cin", "cout", "k", "scale", "shift", "w16", "host", "wino", "mode")

    def __init__(self, w, cin, cout, k, scale, shift, w16=None, host=None, mode="f32"):
        self.w, self.cin, self.cout, self.k, self.scale, self.shift = w, cin, cout, k, scale, shift
        self.w16 = w16
        self.mode = mode  # operand mode of w16: "f32" (none: fp32 MFMA), "bf16" (one plane), "x3" (three)
        self.host = host  # the packed fp32 [Cout, K] weights on the host (pack-time fusions read them)
        self.wino = None  # Winograd F(2x2, 3x3) weight planes when this stride-1 3x3 runs that way


class LinW:
    __slots__ = ("w", "b", "k", "n", "w16", "mode")

    def __init__(self, w, b, k, n, w16=None, mode="f32"):
        self.w, self.b, self.k, self.n = w, b, k, n
        self.w16 = w16
        self.mode = mode  # as ConvW.mode


def frozen_bn_affine(p, pre):
    # RTDetrV2FrozenBatchNorm2d.forward M2:751-757
    scale = p[pre + ".weight"] * (p[pre + ".running_var"] + np.float32(1e-5)) ** np.float32(-0.5)
    shift = p[pre + ".bias"] - p[pre + ".running_mean"] * scale
    return scale.astype(np.float32), shift.astype(np.float32)


def eval_bn_affine(p, pre, eps=1e-5):
    # nn.BatchNorm2d eval: (x - mean) / sqrt(var + eps) * w + b
    inv = (p[pre + ".running_var"] + np.float32(eps)) ** np.float32(-0.5)
    scale = p[pre + ".weight"] * inv
    shift = p[pre + ".bias"] - p[pre + ".running_mean"] * scale
    return scale.astype(np.float32), shift.astype(np.float32)


def conv_khwc(w):
    co, ci, k, _ = w.shape
    return np.ascontiguousarray(w.transpose(0, 2, 3, 1).reshape(co, k * k * ci))


def sine_pos_embed(h, w, dim, temperature):
    """build_2d_sinusoidal_position_embedding M2:955-1000 (f64 on host, cast to f32; constant)."""
    pd = dim // 4
    omega = 1.0 / temperature ** (np.arange(pd, dtype=np.float64) / pd)
    gh, gw = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    eh = np.outer(gh.reshape(-1), omega)
    ew = np.outer(gw.reshape(-1), omega)
    return np.concatenate([np.sin(eh), np.cos(eh), np.sin(ew), np.cos(ew)], 1).astype(np.float32)


def anchors_for(shapes, grid_size=0.05):
    """_cached_generate_anchors M2:1421-1449 (constant table, built once per shape set)."""
    out = []
    f = np.float32
    for lvl, (h, w) in enumerate(shapes):
        gy, gx = np.meshgrid(np.arange(h, dtype=f), np.arange(w, dtype=f), indexing="ij")
        xy = np.stack([gx, gy], -1) + f(0.5)
        xy[..., 0] /= f(w)
        xy[..., 1] /= f(h)
        wh = np.ones_like(xy) * f(grid_size * 2.0 ** lvl)
        out.append(np.concatenate([xy, wh], -1).reshape(h * w, 4))
    a = np.concatenate(out, 0).astype(f)
    valid = ((a > f(1e-2)) & (a < f(1 - 1e-2))).all(-1)
    lg = np.log(a / (f(1) - a)).astype(f)
    lg[~valid] = np.finfo(f).max
    return lg, valid.astype(f)


class Engine:
    """Owns the packed device weights and the per-shape workspaces of one GPU."""

    def __init__(self, cfg: SpotterConfig, weights: dict, device: str | torch.device = "cuda",
                 fold_repvgg: bool = True, precision: str = "fp32", fuse_shortcut: bool = True,
                 fuse_ln: bool = False, winograd: str | bool = "auto", wino_m: int = 4,
                 bf16_store: bool | None = None, direct_c32: bool = True,
                 direct_c64_bf16: bool = True, splitk_combine: bool = False):
        from ._lib import SP_BUILD_FUSED_LN, lib

        check_precision(precision)
        self.cfg = cfg
        self.fold_repvgg = fold_repvgg
        self.fuse_shortcut = fuse_shortcut  # bottleneck tail + projection shortcut as one GEMM (_fused_tail)
        # post-norm LayerNorms in the preceding GEMM's epilogue (_lin_op ln=). Off by default: the fused
        # kernel needs whole rows per workgroup (32-row fp32-MFMA tiles), which at bs32 ran the 21 GEMMs at
        # 42 TF/s (2.47 ms/step) against 1.4 ms/step for the unfused GEMMs + 21 sp_layernorm launches
        # (profiles/r2/fused_ln_ab.json); it stays selectable, in diagnostic library builds (SP_DIAG_KERNELS).
        self.fuse_ln = fuse_ln  # the fused-LN epilogue is compiled into diagnostic library builds only
        if fuse_ln and PRECISIONS.get(precision, ("", ""))[1] == "bf16":
            # the fused-LN tile runs fp32 weights: it would silently raise the bf16 linears' operand precision
            raise ValueError(f"fuse_ln=True runs the linears on fp32 weights: not available with precision={precision!r}")
        if fuse_ln and not (lib().sp_build_flags() & SP_BUILD_FUSED_LN):
            # refuse here, not at the first fused GEMM in the middle of a forward
            raise ValueError("fuse_ln=True needs a diagnostic library with the fused-LayerNorm tiles "
                             "(UNIT=conv_gemm tools/build_diag.sh <name> -DSP_DIAG_KERNELS=1; SPOTTER_HIP_LIB)")
        # stride-1 3x3 convs as Winograd F(m x m, 3x3) on the split GEMM (sp_winograd_f{2,4}3_*): "auto"
        # (default) = those on the split operand mode with Cin >= 128 for F(4x4) (1.4-2.6x faster than the
        # implicit GEMM at bs32, profiles/r2/tune_wino_f43_x3.json) or Cin >= 256 for F(2x2) (1.25-1.8x,
        # profiles/r2/tune_wino_x3.json; below that the transforms cost more than the multiply saving; on
        # bf16 operands it is always slower, profiles/r2/tune_wino_bf16.json), on maps of >= WINO_MIN_PIXELS
        # pixels; "repvgg" = only the encoder's folded RepVGG convs; "all" = every stride-1 3x3 on a
        # bf16-operand mode; False = none. wino_m = 4 (default, 1/4 of the direct multiply-adds, fp32 error
        # 3-5x the direct conv's) or 2 (4/9, error on par with the direct conv).
        if winograd is True:
            winograd = "auto"
        if winograd not in (False, None, "auto", "repvgg", "all"):
            raise ValueError("winograd must be False, 'auto', 'repvgg' or 'all'")
        self.winograd = winograd or False
        if wino_m not in (2, 4):
            raise ValueError("wino_m must be 2 (F(2x2,3x3)) or 4 (F(4x4,3x3))")
        self.wino_m = wino_m
        self.precision = precision
        # activations by config (the fused epilogue implements relu / silu / gelu; checkpoint.py refuses others)
        self.act_bb = cfg.hidden_act
        self.act_enc = cfg.activation_function
        self.act_aifi = cfg.encoder_activation_function
        self.act_dec = cfg.decoder_activation_function
        self._conv_mode, self._lin_mode = PRECISIONS[precision]
        # the attention core on bf16 operands where the linears around it are bf16 (sp_attention_bf16)
        self._attn_bf16 = self._lin_mode == "bf16" and ATTN_BF16
        # bf16 conv operands: keep the backbone's activation maps in HBM as bf16 rows (half the bytes of every
        # producer write and consumer read; the GEMMs stage them as their bf16 A plane, the epilogues round
        # once at the store) instead of fp32 maps rounded per GEMM fragment. Default on for the bf16 modes.
        self.bf16_store = (self._conv_mode == "bf16") if bf16_store is None else bool(bf16_store)
        if self.bf16_store and self._conv_mode != "bf16":
            raise ValueError("bf16_store needs a bf16 conv operand mode")
        # the Cin-32 stem 3x3s on fp32-MFMA weights as the direct LDS-halo kernel (sp_conv3x3_c32) instead of
        # the fp32-MFMA implicit GEMM
        self.direct_c32 = direct_c32
        self.direct_c64_bf16 = direct_c64_bf16  # the stage-0 3x3 (Cin 64 -> 64) on bf16 rows (sp_conv3x3_c64_bf16)
        # split-K GEMMs (the small-batch path) combine their partial sums inside the GEMM launch (per-context
        # arrival counters, sp_conv_desc.splitk_counters) instead of a second reduce launch: bit-identical, 303
        # instead of 438 launches per bs1 forward, but 4.786 against 4.714 ms per graph replay (the write-through
        # partial stores and the last workgroup's combine cost more than the reduce launch they replace,
        # profiles/r5/bs1/bs1_ab_splitk_combine.json), so off by default
        self.splitk_combine = splitk_combine
        # linears over at most this many rows never split K (the bs1 decoder's 300-row GEMMs: one launch instead
        # of partial + reduce); 0 = every launch may split (tools/bs1_ab.py "nosk<rows>" variants)
        self.splitk_min_rows = 0
        # the h + pos attention inputs materialised for the LDS-DMA tiles (_lin_plus); False = the A2 addend (A/B)
        self.add_rows = True
        # the bf16 variant's encoder head LayerNorm written as bf16 rows for the score projection (decode); False =
        # the fp32 normalised map (A/B)
        self.enc_head_bf16 = True
        # with it, the score head and its per-anchor class max fused (sp_linear_rowmax_bf16); False = GEMM + rowmax
        self.enc_rowmax_fused = True
        self.dev = torch.device(device)
        if self.dev.type != "cuda":
            raise RuntimeError("spotter_amd runs on an MI355X (gfx950) device only")
        idx = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
        self.dev = torch.device("cuda", idx)
        rc = lib().sp_device_init(idx)
        if rc != 0:
            raise RuntimeError(f"sp_device_init: {lib().sp_last_error().decode()}")
        with torch.cuda.device(self.dev):
            self._pack(weights)
        self._ws = {}
        self._consts = {}
        self._ctxs = {}
        self._outs = {}
        # None = the default split (micro_batches_for: one stream). Two streams measured +1.7 % at bs32
        # (640 vs 629 img/s, events off; profiles/r2/microbatch_ab_r2.json) but make every kernel share
        # the chip with the other stream's, so per-kernel durations (the roofline, rocprof) stop
        # describing the kernels; k > 1 stays available (Engine.forward(microbatches=k) / bench.py
        # --microbatches k)
        self.microbatches = None
        self.stagger = 1  # residual blocks of offset between consecutive micro-batch streams

    # ------------------------------------------------------------------ weights
    def _wq(self, w: np.ndarray, mode: str):
        """GEMM operand form of host fp32 weights w [Cout, K], uploaded: None (fp32 MFMA), bf16 bit
        patterns (RNE), or the hi / mid / lo bf16 planes of the fp32-accurate split path. The
        rounding runs in numpy at pack time; the device only receives bit patterns."""
        if mode == "f32":
            return None
        if mode == "bf16":
            return torch.from_numpy(bf16_bits(w).view(np.int16)).to(self.dev)
        return torch.from_numpy(ops.split_bf16x3_host(w)).to(self.dev)

    def _add_wino(self, cw: ConvW):
        """Attach the F(2x2, 3x3) transformed weight planes (host fp64 transform, then the conv's own
        operand form: three split planes or one bf16 plane) to a stride-1 3x3 conv the Winograd policy
        (self.winograd) selects."""
        if cw.k != 3 or cw.mode == "f32" or cw.cin % 32 or cw.cout % 4 or not self.winograd:
            return cw
        if self.winograd == "auto" and (cw.cin < (self.WINO43_MIN_CIN if self.wino_m == 4 else 256) or cw.mode != "x3"):
            return cw
        u = ops.winograd_weights_host(cw.host.reshape(cw.cout, 3, 3, cw.cin), self.wino_m)
        if cw.mode == "x3":
            cw.wino = torch.from_numpy(ops.split_bf16x3_host(u)).to(self.dev)
        else:
            cw.wino = torch.from_numpy(bf16_bits(u).reshape(1, -1).view(np.int16)).to(self.dev)
        return cw

    def _pick(self, mode: str, cout: int, kdim: int, small_m: bool = False) -> str:
        """Per-layer GEMM mode. Under precision "fp32" both operand modes are fp32-accurate, so layers
        where the plain fp32 MFMA measured faster than the 6-MFMA split (tools/conv_bench.py,
        profiles/r1/conv_detail_*.json) take it: thin outputs (Cout <= 64: stem, stage-1), thin
        reductions (K <= 64) and the decoder's M = B·300 linears."""
        if mode == "x3" and self.precision == "fp32" and (cout <= 64 or kdim <= 64 or small_m):
            if cout == 64 and kdim >= 576 and not small_m:
                return mode  # 3×3 64→64 (stage 1): the split kernel's 256×64 tile, 1.09× (conv_bench_thin_x3)
            if (cout, kdim, small_m) in _X3_FASTER:
                return mode
            return "f32"
        return mode

    def _mk_conv(self, wk, ci, co, k, sc, sh):
        wk = np.ascontiguousarray(wk, dtype=np.float32)
        mode = self._pick(self._conv_mode, co, ci * k * k)
        return ConvW(_t(wk, self.dev), ci, co, k, _t(sc, self.dev), _t(sh, self.dev), self._wq(wk, mode), host=wk,
                     mode=mode)

    def _conv(self, p, conv_key, bn_pre, frozen):
        w = p[conv_key]
        co, ci, k, _ = w.shape
        # FrozenBN's eps is fixed at 1e-5 (M2:755); the encoder's nn.BatchNorm2d uses config.batch_norm_eps
        sc, sh = frozen_bn_affine(p, bn_pre) if frozen else eval_bn_affine(p, bn_pre, self.cfg.batch_norm_eps)
        return self._mk_conv(conv_khwc(w), ci, co, k, sc, sh)

    def _lin(self, p, pre, *more, per_query: bool = False):
        """per_query: a decoder-side linear over the B·Q selected queries (small M)."""
        ws = [p[pre + ".weight"]] + [p[m + ".weight"] for m in more]
        bs = [p[pre + ".bias"]] + [p[m + ".bias"] for m in more]
        w = np.ascontiguousarray(np.concatenate(ws, 0))
        b = np.concatenate(bs, 0)
        wd = _t(w, self.dev)
        mode = self._pick(self._lin_mode, w.shape[0], w.shape[1], small_m=per_query and w.shape[0] > 128)
        return LinW(wd, _t(b, self.dev), w.shape[1], w.shape[0], self._wq(w.astype(np.float32), mode), mode=mode)

    def _ln(self, p, pre):
        return (_t(p[pre + ".weight"], self.dev), _t(p[pre + ".bias"], self.dev))

    def _pack(self, p):
        cfg = self.cfg
        bb = "model.backbone.model"
        self.stem = [self._conv(p, f"{bb}.embedder.embedder.{i}.convolution.weight",
                                f"{bb}.embedder.embedder.{i}.normalization", True) for i in range(3)]
        self.blocks = []
        for (s, i, lt, cin, cout, st, sc) in backbone_plan(cfg):
            pre = f"{bb}.encoder.stages.{s}.layers.{i}"
            blk = {"s": s, "i": i, "type": lt, "cin": cin, "cout": cout, "stride": st, "sc": sc}
            if sc == "conv":
                blk["short"] = self._conv(p, pre + ".shortcut.convolution.weight", pre + ".shortcut.normalization", True)
            elif sc == "avgconv":
                blk["short"] = self._conv(p, pre + ".shortcut.1.convolution.weight", pre + ".shortcut.1.normalization", True)
            nl = 3 if lt == "bottleneck" else 2
            blk["layers"] = [self._conv(p, f"{pre}.layer.{j}.convolution.weight", f"{pre}.layer.{j}.normalization", True)
                             for j in range(nl)]
            if self.winograd in ("auto", "all"):
                # the stride-1 3x3s: bottleneck conv2 (RN:225-231) when the block keeps the resolution,
                # basic-block conv2 always (RN:170-180)
                for j, c in enumerate(blk["layers"]):
                    if c.k == 3 and (st == 1 or (lt != "bottleneck" and j == 1)):
                        self._add_wino(c)
            if self.fuse_shortcut and lt == "bottleneck" and (sc == "avgconv" or (sc == "conv" and st == 1)):
                sk = pre + (".shortcut.1" if sc == "avgconv" else ".shortcut")
                blk["fused"] = self._fused_tail(p, f"{pre}.layer.2", sk, cin)
            self.blocks.append(blk)
        self.in_proj = [self._conv(p, f"model.encoder_input_proj.{l}.0.weight", f"model.encoder_input_proj.{l}.1", False)
                        for l in range(len(cfg.encoder_in_channels))]
        a = "model.encoder.aifi.0.layers.0"
        self.aifi = {
            "qk": self._lin(p, a + ".self_attn.q_proj", a + ".self_attn.k_proj"),
            "v": self._lin(p, a + ".self_attn.v_proj"),
            "o": self._lin(p, a + ".self_attn.o_proj"),
            "ln1": self._ln(p, a + ".self_attn_layer_norm"),
            "fc1": self._lin(p, a + ".mlp.fc1"),
            "fc2": self._lin(p, a + ".mlp.fc2"),
            "ln2": self._ln(p, a + ".final_layer_norm"),
        }
        E = "model.encoder"
        nl = len(cfg.encoder_in_channels)
        self.lateral = [self._conv(p, f"{E}.lateral_convs.{i}.conv.weight", f"{E}.lateral_convs.{i}.norm", False)
                        for i in range(nl - 1)]
        self.down = [self._conv(p, f"{E}.downsample_convs.{i}.conv.weight", f"{E}.downsample_convs.{i}.norm", False)
                     for i in range(nl - 1)]
        self.fpn = [self._csp(p, f"{E}.fpn_blocks.{i}") for i in range(nl - 1)]
        self.pan = [self._csp(p, f"{E}.pan_blocks.{i}") for i in range(nl - 1)]
        self.dec_proj = [self._conv(p, f"model.decoder_input_proj.{l}.0.weight", f"model.decoder_input_proj.{l}.1", False)
                         for l in range(len(cfg.decoder_in_channels))]
        self.enc_output = self._lin(p, "model.enc_output.0")
        self.enc_ln = self._ln(p, "model.enc_output.1")
        self.enc_score = self._lin(p, "model.enc_score_head")
        self.enc_bbox = [self._lin(p, f"model.enc_bbox_head.layers.{i}", per_query=True) for i in range(3)]
        self.qpos = [self._lin(p, f"model.decoder.query_pos_head.layers.{i}", per_query=True) for i in range(2)]
        D = "model.decoder.layers"
        L = cfg.decoder_layers
        self.value_all = self._lin(p, f"{D}.0.encoder_attn.value_proj",
                                   *[f"{D}.{j}.encoder_attn.value_proj" for j in range(1, L)])
        self.dec = []
        for j in range(L):
            q = f"{D}.{j}"
            pq = {"per_query": True}
            self.dec.append({
                "qk": self._lin(p, q + ".self_attn.q_proj", q + ".self_attn.k_proj", **pq),
                "v": self._lin(p, q + ".self_attn.v_proj", **pq),
                "o": self._lin(p, q + ".self_attn.o_proj", **pq),
                "ln1": self._ln(p, q + ".self_attn_layer_norm"),
                "offaw": self._lin(p, q + ".encoder_attn.sampling_offsets", q + ".encoder_attn.attention_weights", **pq),
                "out": self._lin(p, q + ".encoder_attn.output_proj", **pq),
                "ln2": self._ln(p, q + ".encoder_attn_layer_norm"),
                "fc1": self._lin(p, q + ".mlp.fc1", **pq),
                "fc2": self._lin(p, q + ".mlp.fc2", **pq),
                "ln3": self._ln(p, q + ".final_layer_norm"),
                "bbox": [self._lin(p, f"model.decoder.bbox_embed.{j}.layers.{i}", **pq) for i in range(3)],
            })
        self.cls_last = self._lin(p, f"model.decoder.class_embed.{L - 1}")

    def _fused_tail(self, p, conv3, short, cin):
        """Bottleneck tail + projection shortcut as one 1×1 GEMM over K = red + cin (RN:199-207, 225-231):
        relu(BN3(W3·t2) + BNsc(Wsc·x)) = relu([s3·W3 | ssc·Wsc]·[t2 | x] + (b3 + bsc)). The producers write
        t2 and the (pooled) block input side by side in one NHWC buffer, so the shortcut's Cout-wide
        output never goes through HBM. BN scales fold into the weights in f64, rounded once to f32."""
        w3 = conv_khwc(p[conv3 + ".convolution.weight"]).astype(np.float64)
        wsc = conv_khwc(p[short + ".convolution.weight"]).astype(np.float64)
        s3, b3 = frozen_bn_affine(p, conv3 + ".normalization")
        ss, bs = frozen_bn_affine(p, short + ".normalization")
        wf = np.concatenate([w3 * s3.astype(np.float64)[:, None], wsc * ss.astype(np.float64)[:, None]], 1)
        co, kc = wf.shape
        assert kc == w3.shape[1] + cin
        shift = b3.astype(np.float64) + bs.astype(np.float64)
        return self._mk_conv(wf.astype(np.float32), kc, co, 1, np.ones(co, np.float32), shift.astype(np.float32))

    def _csp(self, p, pre):
        # conv1 ‖ conv2: one GEMM over the same input (M2:949-951), concatenated on the host
        w1 = p[pre + ".conv1.conv.weight"]
        w2 = p[pre + ".conv2.conv.weight"]
        s1, b1 = eval_bn_affine(p, pre + ".conv1.norm", self.cfg.batch_norm_eps)
        s2, b2 = eval_bn_affine(p, pre + ".conv2.norm", self.cfg.batch_norm_eps)
        w12 = np.concatenate([conv_khwc(w1), conv_khwc(w2)], 0)
        c12 = ConvW(_t(w12, self.dev), w1.shape[1], w1.shape[0] + w2.shape[0], 1,
                    _t(np.concatenate([s1, s2]), self.dev), _t(np.concatenate([b1, b2]), self.dev),
                    self._wq(w12, self._conv_mode), host=w12, mode=self._conv_mode)
        reps = []
        for b in range(3):
            q = f"{pre}.bottlenecks.{b}"
            if self.fold_repvgg:
                # RepVGG re-parameterisation (M2:921-923): BN1(conv3x3(x)) + BN2(conv1x1(x)) is one 3×3
                # conv whose weights are s1·W3 with s2·W1 added to the centre tap, shift b1 + b2.
                w3, w1 = p[q + ".conv1.conv.weight"], p[q + ".conv2.conv.weight"]
                s1, b1 = eval_bn_affine(p, q + ".conv1.norm", self.cfg.batch_norm_eps)
                s2, b2 = eval_bn_affine(p, q + ".conv2.norm", self.cfg.batch_norm_eps)
                wf = (w3.astype(np.float64) * s1[:, None, None, None]).copy()
                wf[:, :, 1, 1] += w1[:, :, 0, 0].astype(np.float64) * s2[:, None]
                co, ci = w3.shape[:2]
                cw = self._mk_conv(conv_khwc(wf.astype(np.float32)), ci, co, 3, np.ones(co, np.float32),
                                   (b1.astype(np.float64) + b2).astype(np.float32))
                reps.append(("fold", self._add_wino(cw) if self.winograd else cw))
            else:
                reps.append((self._conv(p, q + ".conv1.conv.weight", q + ".conv1.norm", False),
                             self._conv(p, q + ".conv2.conv.weight", q + ".conv2.norm", False)))
        c3 = None
        if (pre + ".conv3.conv.weight") in p:
            c3 = self._conv(p, pre + ".conv3.conv.weight", pre + ".conv3.norm", False)
        return {"c12": c12, "hid": w1.shape[0], "reps": reps, "c3": c3}

    # ------------------------------------------------------------------ workspace
    def _buf(self, key, *shape, dtype=torch.float32):
        ws = self._ws
        t = ws.get(key)
        n = int(np.prod(shape))
        if t is None or t.numel() < n or t.dtype != dtype:
            t = torch.empty(n, dtype=dtype, device=self.dev)
            ws[key] = t
        return t[:n]

    SPLITK_COUNTERS = 4096  # arrival counters per context: one per output tile of a split-K launch

    def _splitk(self) -> dict:
        """The split-K scratch of this context's GEMM launches: the partial-sum workspace and, with
        splitk_combine, the arrival counters (zeroed once here; every launch leaves them zero)."""
        kw = {"workspace": self._buf("splitk", self.SPLITK_ELEMS)}
        if self.splitk_combine:
            c = self._ws.get("splitk_cnt")
            if c is None:
                c = torch.zeros(self.SPLITK_COUNTERS, dtype=torch.int32, device=self.dev)
                self._ws["splitk_cnt"] = c
            kw["counters"] = c
        return kw

    def _const(self, key, fn):
        c = self._consts.get(key)
        if c is None:
            c = fn()
            self._consts[key] = c
        return c

    # ------------------------------------------------------------------ layers
    SPLITK_ELEMS = 16 << 20  # 64 MB fp32 split-K scratch per context
    # F(4x4) Winograd from Cin 128. Round 5 measured Cin 64 (the stage-1 160²×64 3x3s): 0.50 against 0.65 ms
    # for the implicit GEMM in isolation (profiles/r5/wino/tune_wino_c64.json), but no change in the C2 step
    # (772-774 img/s either way, same box, alternating) and 0.2 % slower at bs1 (profiles/r5/wino/ab_cin64.json)
    WINO43_MIN_CIN = 128
    WINO_MIN_PIXELS = 8192
    WINO43_MIN_WORK = 1 << 19

    def _wino_pays(self, pixels: int, cin: int) -> bool:
        """Size gate of the Winograd path. F(2x2): maps of >= 8192 output pixels (2048 tiles): at bs1 the
        40² / 20² convs measured 0.69-1.07x of the split-K implicit GEMM, from bs8 up 1.2-1.8x
        (profiles/r2/tune_wino_x3_bs8_bs1.json). F(4x4): pixels x Cin >= 2^19: at bs1 the 80²x384 /
        40²x384 / 80²x128 convs measured 2.6x / 1.45x / 1.09x, 40²x256 1.04x, 20²x384 / 20²x512 0.85-0.95x
        (profiles/r2/tune_wino_f43_bs1.json); every bs8 / bs32 map clears it."""
        if self.wino_m == 4:
            # the Cin gate belongs to the "auto" policy only (as in _add_wino): a forced winograd=True / "all"
            # has built the transformed weights for the thin convs too and runs them
            return pixels * cin >= self.WINO43_MIN_WORK and (cin >= self.WINO43_MIN_CIN or self.winograd != "auto")
        return pixels >= self.WINO_MIN_PIXELS

    def _cv(self, x: V, n, h, w, cw: ConvW, stride, out: V, act=None, res1=None, res2=None, **kw):
        pad = cw.k // 2
        if (cw.cin == 64 and cw.cout == 64 and cw.k == 3 and stride == 1 and not kw and res2 is None
                and act in ("relu", None) and n * h * w >= self.C64_MIN_PIXELS):
            rows16 = lambda v: v.ld % 8 == 0 and v.off % 8 == 0  # noqa: E731 (16-byte aligned bf16 rows)
            if (self.direct_c64_bf16 and x.is_bf16 and out.is_bf16 and cw.mode == "bf16" and rows16(x)
                    and rows16(out) and (res1 is None or (res1.is_bf16 and rows16(res1)))):
                # the bf16 variant's stage-0 3x3: direct LDS-halo kernel, bit-identical to the implicit GEMM and
                # 1.53x it at bs32 / bs256 (814 TF at C3; profiles/r3/bf16/ab_conv3x3_c64_bf16.jsonl)
                return ops.conv3x3_c64_bf16(x, cw.w16, cw.scale, cw.shift, out, n, h, w, act=act, res1=res1)
        if cw.wino is not None and stride == 1 and not kw and not x.is_bf16 and self._wino_pays(n * h * w, cw.cin):
            wm = self.wino_m
            tiles = n * ((h + wm - 1) // wm) * ((w + wm - 1) // wm)
            work = self._buf("wino_work", ops.wino_work_elems(wm, tiles, cw.cin, cw.cout))
            return ops.conv2d(x, n, h, w, cw.cin, cw.w, cw.cout, 3, 1, 1, out, scale=cw.scale, shift=cw.shift,
                              act=act, res1=res1, res2=res2, wino=(cw.wino, work, wm))
        return ops.conv2d(x, n, h, w, cw.cin, cw.w, cw.cout, cw.k, stride, pad, out, scale=cw.scale,
                          shift=cw.shift, act=act, res1=res1, res2=res2,
                          **self._splitk(), **_wkw(cw.w16), **kw)

    def _lin_op(self, x: V, rows, lw: LinW, out: V, act=None, res1=None, res2=None, a2=None, row_scale=None,
                ln=None):
        """ln = (gamma, beta): the post-norm LayerNorm of the output row fused into the GEMM epilogue
        (fp32-MFMA tile holding whole rows; sp_conv_desc.ln_gamma)."""
        if ln is not None and self.fuse_ln:
            # the fused-LN tile runs on the fp32 weights (fp32 MFMA): exact for the fp32-accurate modes,
            # but it would silently raise a bf16 layer's operand precision, and its epilogue has no act /
            # post-act residual: refuse rather than drop either
            if act is not None or res2 is not None:
                raise ValueError("fused LayerNorm epilogue: act / res2 are not implemented")
            if lw.mode == "bf16":
                raise ValueError("fuse_ln runs fp32 weights: not available on a bf16-operand layer")
            return ops.linear(x, rows, lw.k, lw.w, lw.n, out, bias=lw.b, res1=res1, a2=a2, row_scale=row_scale,
                              ln=(ln[0], ln[1], self.cfg.layer_norm_eps))
        if ln is not None:  # unfused: GEMM into a scratch row block, then sp_layernorm into `out`
            tmp = view(self._buf("ln_tmp", rows, lw.n), lw.n)
            ops.linear(x, rows, lw.k, lw.w, lw.n, tmp, bias=lw.b, act=act, res1=res1, res2=res2, a2=a2,
                       row_scale=row_scale, **self._splitk(), **_wkw(lw.w16))
            return ops.layernorm(tmp, *ln, out, rows, lw.n, self.cfg.layer_norm_eps)
        sk = self._splitk() if rows > self.splitk_min_rows else {}
        return ops.linear(x, rows, lw.k, lw.w, lw.n, out, bias=lw.b, act=act, res1=res1, res2=res2, a2=a2,
                          row_scale=row_scale, **sk, **_wkw(lw.w16))

    def _lin_plus(self, x: V, addend: V | None, rows, lw: LinW, out: V, key: str):
        """out = (x + addend) @ W + b: the attention projections whose input is h + pos (M2:395-404, 409-423; AIFI
        M2:873-880). On the bf16 / split kernels the sum is materialised once (sp_add_rows; bf16 rows in the bf16
        mode, the operand that kernel's loader would have rounded) so the GEMM loads it by LDS-DMA; their A2
        addend exists only in the register-staged tiles, 2.7x slower on C3's decoder projections
        (profiles/r6/c3tail/). The fp32 MFMA kernel keeps its in-loader add."""
        if addend is None:
            return self._lin_op(x, rows, lw, out)
        if not self.add_rows or lw.mode == "f32":
            return self._lin_op(x, rows, lw, out, a2=addend)
        hp = view(self._buf(key, rows, lw.k, dtype=torch.int16 if lw.mode == "bf16" else torch.float32), lw.k)
        ops.add_rows(x, addend, hp, rows, lw.k)
        return self._lin_op(hp, rows, lw, out)

    C64_MIN_PIXELS = 1 << 18
    C32_MIN_PIXELS = 1 << 19  # sp_conv3x3_c32 from about 4 tiles per CU up (bs8 at 320²: 1.08-1.17x)

    def _direct_stem(self) -> bool:
        """The stem's first conv (Cin 3, K = 27) runs on the direct NCHW kernel (sp_stem_conv3x3s2_nchw, fp32
        weights, exact fmaf chains) in every precision mode: K = 27 gives a GEMM nothing to tile (the bf16
        GEMM ran it at 20 TF/s, 2.3 ms of a C3 step, profiles/r3/bf16/), and fp32 here is only more exact."""
        c = self.stem[0]
        return c.cin == 3 and c.k == 3 and c.cout in (32, 64) and self.act_bb in ("relu", None)

    def backbone(self, pixel_values: torch.Tensor, B, H, W):
        """RTDetrResNetBackbone.forward RN:365-422 → [stage2, stage3, stage4] outputs (NHWC).
        pixel_values is the processor's NCHW batch (IPP:461-462)."""
        e = self.cfg.embedding_size
        h1, w1 = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        dt = torch.int16 if self.bf16_store else torch.float32  # bf16 maps: bit patterns in int16 buffers

        def buf(key, *shape):
            return self._buf(key, *shape, dtype=dt)

        s0 = buf("stem0", B, h1, w1, e // 2)
        s1 = buf("stem1", B, h1, w1, e // 2)
        s2 = buf("stem2", B, h1, w1, e)
        c0 = self.stem[0]
        if self._direct_stem():
            ops.stem_conv_nchw(pixel_values, c0.w, c0.scale, c0.shift, view(s0, e // 2), c0.cout, act=self.act_bb)
        else:
            px = self._buf("px_nhwc", B, H, W, 3)
            ops.nchw_to_nhwc(pixel_values, px)
            self._cv(view(px, 3), B, H, W, c0, 2, view(s0, e // 2), act=self.act_bb)
        for src, cw, dst in ((s0, self.stem[1], s1), (s1, self.stem[2], s2)):
            c32 = cw.cin == 32 and cw.k == 3 and cw.cout in (32, 64) and self.act_bb in ("relu", None)
            if c32 and self.bf16_store:
                # the bf16 variant's Cin-32 stem 3×3s: direct LDS-halo kernel (the implicit GEMM re-fetched every
                # A row per tap and wasted half a 64-wide tile on Cout 32)
                ops.conv3x3_c32_bf16(view(src, cw.cin), cw.w16, cw.scale, cw.shift, view(dst, cw.cout), B, h1, w1,
                                     cw.cout, act=self.act_bb)
            elif (c32 and self.direct_c32 and cw.mode == "f32" and not self.bf16_store
                  and B * h1 * w1 >= self.C32_MIN_PIXELS):
                # the fp32 modes: the same direct kernel on fp32 rows with fp32 MFMAs (exact products): 1.24-1.29x
                # the fp32-MFMA GEMM at bs32 (113 / 128 TF), 1.08-1.17x at bs8 of 320²
                # (profiles/r3/x3/ab_stem_c32_f32.jsonl); smaller maps (a few tiles per CU at most for its
                # one-workgroup-per-CU grid) keep the GEMM
                ops.conv3x3_c32(view(src, cw.cin), cw.w, cw.scale, cw.shift, view(dst, cw.cout), B, h1, w1, cw.cout,
                                act=self.act_bb)
            else:
                self._cv(view(src, cw.cin), B, h1, w1, cw, 1, view(dst, cw.cout), act=self.act_bb)
        h, w = (h1 - 1) // 2 + 1, (w1 - 1) // 2 + 1
        b0 = self.blocks[0]
        if "fused" in b0 and b0["sc"] == "conv":
            # the first block's fused tail reads the pooled stem next to its conv2 output: pool into that slice
            kc = b0["layers"][0].cout + e
            curv = V(buf(f"s{b0['s']}_cat", B, h, w, kc), kc - e, kc)
        else:
            curv = view(buf("pool", B, h, w, e), e)
        ops.maxpool3x3s2(s2, curv, B, h1, w1, e)
        c = e
        feats = []
        nstage = len(self.cfg.depths)
        for blk in self.blocks:
            s, i, st, cout = blk["s"], blk["i"], blk["stride"], blk["cout"]
            cur = curv.t
            if i == 0 and s > 0:
                assert curv.off == 0 and curv.ld == c
                feats.append((cur, h, w, c))
            ho, wo = (h - 1) // st + 1, (w - 1) // st + 1
            L = blk["layers"]
            if "fused" in blk:
                red = L[0].cout
                kc = red + c
                if blk["sc"] == "avgconv":
                    assert curv.off == 0 and curv.ld == c
                    cat = buf(f"s{s}_cat", B, ho, wo, kc)
                    ops.avgpool2x2_ceil(cur, V(cat, red, kc), B, h, w, c)
                else:  # stride-1 projection: the block input already sits in the slice (see above)
                    assert curv.off == red and curv.ld == kc and st == 1
                    cat = cur
                t1 = buf(f"s{s}_t1", B, h, w, red)
                out = buf(f"s{s}_out{i % 2}", B, ho, wo, cout)
                self._cv(curv, B, h, w, L[0], 1, view(t1, red), act=self.act_bb)
                self._cv(view(t1, red), B, h, w, L[1], st, V(cat, 0, kc), act=self.act_bb)
                self._cv(V(cat, 0, kc), B, ho, wo, blk["fused"], 1, view(out, cout), act=self.act_bb)
                curv, h, w, c = view(out, cout), ho, wo, cout
                yield
                continue
            # shortcut (RN:199-207)
            if blk["sc"] == "identity":
                res = view(cur, c)
            else:
                src, sh_, sw_ = cur, h, w
                if blk["sc"] == "avgconv":
                    pooled = buf(f"s{s}_pool", B, (h + 1) // 2, (w + 1) // 2, c)
                    ops.avgpool2x2_ceil(cur, pooled, B, h, w, c)
                    src, sh_, sw_ = pooled, (h + 1) // 2, (w + 1) // 2
                sbuf = buf(f"s{s}_sc", B, ho, wo, cout)
                self._cv(view(src, c), B, sh_, sw_, blk["short"], 1 if blk["sc"] == "avgconv" else st, view(sbuf, cout))
                res = view(sbuf, cout)
            out = buf(f"s{s}_out{i % 2}", B, ho, wo, cout)
            if blk["type"] == "bottleneck":
                red = L[0].cout
                t1 = buf(f"s{s}_t1", B, h, w, red)
                t2 = buf(f"s{s}_t2", B, ho, wo, red)
                self._cv(view(cur, c), B, h, w, L[0], 1, view(t1, red), act=self.act_bb)
                self._cv(view(t1, red), B, h, w, L[1], st, view(t2, red), act=self.act_bb)
                self._cv(view(t2, red), B, ho, wo, L[2], 1, view(out, cout), act=self.act_bb, res1=res)
            else:
                t1 = buf(f"s{s}_t1", B, ho, wo, cout)
                self._cv(view(cur, c), B, h, w, L[0], st, view(t1, cout), act=self.act_bb)
                self._cv(view(t1, cout), B, ho, wo, L[1], 1, view(out, cout), act=self.act_bb, res1=res)
            curv, h, w, c = view(out, cout), ho, wo, cout
            yield
        feats.append((curv.t, h, w, c))
        return feats[-3:] if nstage >= 3 else feats

    def _csp_fwd(self, cs, x: V, B, h, w, out: V, tag):
        """RTDetrV2CSPRepLayer.forward M2:948-952 on a 2·H-channel NHWC input."""
        hid = cs["hid"]
        dt = torch.int16 if self.bf16_store else torch.float32  # the bf16 variant keeps the CCFM maps in bf16
        c12 = self._buf(f"{tag}_c12", B, h, w, 2 * hid, dtype=dt)
        self._cv(x, B, h, w, cs["c12"], 1, view(c12, 2 * hid), act=self.act_enc)
        h2 = V(c12, hid, 2 * hid)
        cur = V(c12, 0, 2 * hid)
        t = None if self.fold_repvgg else self._buf(f"{tag}_t", B, h, w, hid, dtype=dt)
        final_to_out = cs["c3"] is None
        for b, (k3, k1) in enumerate(cs["reps"]):
            last = b == len(cs["reps"]) - 1
            if last and final_to_out:
                dst = out
            else:
                dst = view(self._buf(f"{tag}_r{b % 2}", B, h, w, hid, dtype=dt), hid)
            if k3 == "fold":
                self._cv(cur, B, h, w, k1, 1, dst, act=self.act_enc, res2=h2 if last else None)
            else:
                self._cv(cur, B, h, w, k3, 1, view(t, hid))
                self._cv(cur, B, h, w, k1, 1, dst, act=self.act_enc, res1=view(t, hid), res2=h2 if last else None)
            cur = dst
        if cs["c3"] is not None:
            self._cv(cur, B, h, w, cs["c3"], 1, out, act=self.act_enc)

    def encoder(self, feats, B):
        """encoder_input_proj (M2:1512) + RTDetrV2HybridEncoder.forward (M2:1164-1209)."""
        cfg = self.cfg
        Hd = cfg.encoder_hidden_dim
        (f0, h0, w0, c0), (f1, h1, w1, c1), (f2, h2, w2, c2) = feats
        # bf16 variant: the CCFM maps (concat buffers, CSPRep internals and outputs) in bf16 like the backbone's;
        # AIFI (p5 → p5a) and everything from source_flatten on stay fp32
        dt = torch.int16 if self.bf16_store else torch.float32
        cat3 = self._buf("cat3", B, h0, w0, 2 * Hd, dtype=dt)   # [up(lat1) | proj0]
        cat4 = self._buf("cat4", B, h1, w1, 2 * Hd, dtype=dt)   # [up(lat0) | proj1]
        catn4 = self._buf("catn4", B, h1, w1, 2 * Hd, dtype=dt)  # [down0 | lat1]
        catn5 = self._buf("catn5", B, h2, w2, 2 * Hd, dtype=dt)  # [down1 | lat0]
        p5 = self._buf("p5", B, h2, w2, Hd)
        self._cv(view(f0, c0), B, h0, w0, self.in_proj[0], 1, V(cat3, Hd, 2 * Hd))
        self._cv(view(f1, c1), B, h1, w1, self.in_proj[1], 1, V(cat4, Hd, 2 * Hd))
        self._cv(view(f2, c2), B, h2, w2, self.in_proj[2], 1, view(p5, Hd))
        # AIFI on level 2 (M2:1058-1095; encoder layer M2:856-904, post-norm)
        n = h2 * w2
        rows = B * n
        A = self.aifi
        pos = self._const(("pos", B, h2, w2), lambda: _t(np.tile(
            sine_pos_embed(h2, w2, Hd, cfg.positional_encoding_temperature), (B, 1)), self.dev))
        qk = self._buf("aifi_qk", rows, 2 * Hd)
        vv = self._buf("aifi_v", rows, Hd)
        at = self._buf("aifi_at", rows, Hd)
        y1 = self._buf("aifi_y1", rows, Hd)
        ff = self._buf("aifi_ff", rows, cfg.encoder_ffn_dim)
        p5a = self._buf("p5a", rows, Hd)
        # with config.eval_size set HF runs AIFI without the position embedding (M2:1073-1081)
        self._lin_plus(view(p5, Hd), None if cfg.eval_size else view(pos, Hd), rows, A["qk"], view(qk, 2 * Hd),
                       "aifi_hp")
        self._lin_op(view(p5, Hd), rows, A["v"], view(vv, Hd))
        heads = cfg.encoder_attention_heads
        ops.attention(V(qk, 0, 2 * Hd), V(qk, Hd, 2 * Hd), view(vv, Hd), view(at, Hd), B, n, heads, Hd // heads,
                      (Hd // heads) ** -0.5, bf16=self._attn_bf16)
        self._lin_op(view(at, Hd), rows, A["o"], view(y1, Hd), res1=view(p5, Hd), ln=A["ln1"])
        self._lin_op(view(y1, Hd), rows, A["fc1"], view(ff, cfg.encoder_ffn_dim), act=self.act_aifi)
        self._lin_op(view(ff, cfg.encoder_ffn_dim), rows, A["fc2"], view(p5a, Hd), res1=view(y1, Hd), ln=A["ln2"])
        yield
        # FPN (M2:1183-1197)
        self._cv(view(p5a, Hd), B, h2, w2, self.lateral[0], 1, V(catn5, Hd, 2 * Hd), act=self.act_enc)
        ops.upsample2x(V(catn5, Hd, 2 * Hd), V(cat4, 0, 2 * Hd), B, h2, w2, Hd)
        F4 = self._buf("F4", B, h1, w1, Hd, dtype=dt)
        self._csp_fwd(self.fpn[0], view(cat4, 2 * Hd), B, h1, w1, view(F4, Hd), "fpn0")
        yield
        self._cv(view(F4, Hd), B, h1, w1, self.lateral[1], 1, V(catn4, Hd, 2 * Hd), act=self.act_enc)
        ops.upsample2x(V(catn4, Hd, 2 * Hd), V(cat3, 0, 2 * Hd), B, h1, w1, Hd)
        F3 = self._buf("F3", B, h0, w0, Hd, dtype=dt)
        self._csp_fwd(self.fpn[1], view(cat3, 2 * Hd), B, h0, w0, view(F3, Hd), "fpn1")
        yield
        # PAN (M2:1199-1207)
        self._cv(view(F3, Hd), B, h0, w0, self.down[0], 2, V(catn4, 0, 2 * Hd), act=self.act_enc)
        N4 = self._buf("N4", B, h1, w1, Hd, dtype=dt)
        self._csp_fwd(self.pan[0], view(catn4, 2 * Hd), B, h1, w1, view(N4, Hd), "pan0")
        yield
        self._cv(view(N4, Hd), B, h1, w1, self.down[1], 2, V(catn5, 0, 2 * Hd), act=self.act_enc)
        N5 = self._buf("N5", B, h2, w2, Hd, dtype=dt)
        self._csp_fwd(self.pan[1], view(catn5, 2 * Hd), B, h2, w2, view(N5, Hd), "pan1")
        return [(F3, h0, w0), (N4, h1, w1), (N5, h2, w2)]

    def decoder_inputs(self, enc, B):
        """decoder_input_proj + flatten/concat (M2:1533-1556) → source_flatten [B, S, d]."""
        D = self.cfg.d_model
        shapes = [(h, w) for (_, h, w) in enc]
        S = sum(h * w for h, w in shapes)
        starts = [0]
        for h, w in shapes[:-1]:
            starts.append(starts[-1] + h * w)
        # bf16 variant: source_flatten in bf16 — its two consumers are bf16-operand GEMMs (enc_output, the value
        # projection) that round it to bf16 anyway, so this changes no result ("bf16-convs" keeps it fp32: its
        # linears run the fp32-accurate split)
        src = self._buf("src_flat", B, S, D, dtype=torch.int16 if self.bf16_store and self._lin_mode == "bf16"
                        else torch.float32)
        Hd = self.cfg.encoder_hidden_dim
        for l, (t, h, w) in enumerate(enc):
            self._cv(view(t, Hd), B, h, w, self.dec_proj[l], 1, V(src, starts[l] * D, D),
                     rows_per_group=h * w, group_stride=S * D)
        return src, shapes, starts, S

    def forward(self, pixel_values: torch.Tensor, microbatches: int | None = None):
        """pixel_values [B,3,H,W] fp32 (device) → (logits [B,Q,C], pred_boxes [B,Q,4]) (M2:1864-1881).

        The batch is split into `microbatches` independent slices (images never interact), each
        with its own workspace and HIP stream; their launches are interleaved block by block so
        one slice's GEMMs fill the other's wave-quantisation tails. The returned tensors are
        engine-owned and overwritten by the next call.
        """
        cfg = self.cfg
        if pixel_values.device != self.dev:
            pixel_values = pixel_values.to(self.dev, non_blocking=True)
        pixel_values = pixel_values.contiguous()
        if pixel_values.dtype != torch.float32:
            raise TypeError("pixel_values must be float32")
        B, C, H, W = pixel_values.shape
        if C != 3:
            raise ValueError("Make sure that the channel dimension of the pixel values match with the one set in the configuration.")
        nmb = self.micro_batches_for(B) if microbatches is None else microbatches
        nmb = max(1, min(nmb, B))
        Q, NC = cfg.num_queries, cfg.num_labels
        with torch.cuda.device(self.dev):
            out_logits = self._out("logits", B * Q * NC).view(B, Q, NC)
            out_boxes = self._out("boxes", B * Q * 4).view(B, Q, 4)
            if nmb == 1:
                for _ in self._run(pixel_values, out_logits, out_boxes):
                    pass
                return out_logits, out_boxes
            main = torch.cuda.current_stream()
            bounds = [B * i // nmb for i in range(nmb + 1)]
            jobs = []
            for i in range(nmb):
                ctx = self._ctx(i)
                ctx["stream"].wait_stream(main)
                b0, b1 = bounds[i], bounds[i + 1]
                jobs.append([ctx, self._run(pixel_values[b0:b1], out_logits[b0:b1], out_boxes[b0:b1])])
            saved = self._ws
            # job i starts on the GPU only after job i-1 has issued `stagger` residual blocks
            # (stream event), so the slices' GEMM tails do not line up.
            steps = [0] * nmb
            gate = [None] * nmb
            try:
                while any(j is not None for j in jobs):
                    for ji, job in enumerate(jobs):
                        if job is None:
                            continue
                        ctx, g = job
                        if ji > 0 and steps[ji] == 0:
                            if gate[ji - 1] is None and jobs[ji - 1] is not None:
                                continue
                            if gate[ji - 1] is not None:
                                ctx["stream"].wait_event(gate[ji - 1])
                        self._ws = ctx["ws"]
                        with torch.cuda.stream(ctx["stream"]):
                            try:
                                next(g)
                            except StopIteration:
                                jobs[ji] = None
                            steps[ji] += 1
                            if steps[ji] == max(1, self.stagger) and gate[ji] is None:
                                gate[ji] = torch.cuda.Event()
                                gate[ji].record(ctx["stream"])
            finally:
                self._ws = saved
            for i in range(nmb):
                main.wait_stream(self._ctx(i)["stream"])
            return out_logits, out_boxes

    def micro_batches_for(self, B: int) -> int:
        """Streams a batch of B images is split over (the served path and bench.py share this)."""
        if self.microbatches is not None:
            return self.microbatches
        return 1

    def _ctx(self, i):
        c = self._ctxs.get(i)
        if c is None:
            c = {"ws": {}, "stream": torch.cuda.Stream(self.dev)}
            self._ctxs[i] = c
        return c

    def _out(self, key, n):
        t = self._outs.get(key)
        if t is None or t.numel() < n:
            t = torch.empty(n, dtype=torch.float32, device=self.dev)
            self._outs[key] = t
        return t[:n]

    def _run(self, pixel_values, out_logits, out_boxes):
        B, C, H, W = pixel_values.shape
        feats = yield from self.backbone(pixel_values.contiguous(), B, H, W)
        enc = yield from self.encoder(feats, B)
        src, shapes, starts, S = self.decoder_inputs(enc, B)
        yield
        yield from self.decode(src, shapes, starts, S, B, out_logits, out_boxes)

    def decode(self, src, shapes, starts, S, B, out_logits, out_boxes):
        cfg = self.cfg
        D, Q, NC = cfg.d_model, cfg.num_queries, cfg.num_labels
        # query selection (M2:1582-1623)
        if cfg.anchor_image_size:
            # fixed anchors from config.anchor_image_size (M2:1384, 1451-1456); HF cannot combine them with
            # feature maps of another size either
            ashapes = [(int(cfg.anchor_image_size[0] / s), int(cfg.anchor_image_size[1] / s)) for s in cfg.feat_strides]
            if [tuple(s) for s in ashapes] != [tuple(s) for s in shapes]:
                raise ValueError(f"anchor_image_size {cfg.anchor_image_size} gives levels {ashapes}, input has {shapes}")
        anchors, valid = self._const(("anchors", tuple(shapes)), lambda: tuple(
            _t(a, self.dev) for a in anchors_for(shapes)))
        rows = B * S
        cmax = self._buf("enc_cls_max", rows)
        lw = self.enc_output
        # the bf16 variant's score projection rounds its operand to bf16 anyway: the encoder head's LayerNorm
        # writes bf16 rows for it (half the write and the read of the normalised map), and the Q selected rows
        # per image are normalised again from the pre-norm rows for the decoder (LayerNorm is row-local: the
        # same kernel on the same row gives the same bits as gathering the fp32 normalised map)
        bf16_head = self.enc_head_bf16 and self.enc_score.mode == "bf16" and not self.fuse_ln and D == 256
        if bf16_head:
            pre = view(self._buf("ln_tmp", rows, lw.n), lw.n)
            ops.linear(view(src, D), rows, lw.k, lw.w, lw.n, pre, bias=lw.b, row_scale=valid, **self._splitk(),
                       **_wkw(lw.w16))
            om16 = self._buf("om16", rows, D, dtype=torch.int16)
            ops.layernorm(pre, *self.enc_ln, view(om16, D), rows, D, cfg.layer_norm_eps)
            sw = self.enc_score
            if self.enc_rowmax_fused and NC <= 96 and sw.k == 256:
                # the score head and its class max in one pass, bit-identical to the GEMM + sp_rowmax below
                ops.linear_rowmax_bf16(view(om16, D), rows, sw.k, sw.w16, NC, sw.b, cmax)
            else:
                cls = self._buf("enc_cls", rows, NC)
                self._lin_op(view(om16, D), rows, sw, view(cls, NC))
                ops.rowmax(view(cls, NC), rows, NC, cmax)
        else:
            om = self._buf("om", rows, D)
            cls = self._buf("enc_cls", rows, NC)
            self._lin_op(view(src, D), rows, lw, view(om, D), row_scale=valid, ln=self.enc_ln)
            self._lin_op(view(om, D), rows, self.enc_score, view(cls, NC))
            ops.rowmax(view(cls, NC), rows, NC, cmax)
        topk = self._buf("topk", B, Q, dtype=torch.int32)
        ops.topk_rows(V(cmax, 0, S), B, S, Q, topk)
        Bq = B * Q
        h = self._buf("dec_h", Bq, D)
        if bf16_head:
            hraw = self._buf("dec_hraw", Bq, D)
            ops.gather_rows(pre, S, topk, Q, B, D, view(hraw, D))
            ops.layernorm(view(hraw, D), *self.enc_ln, view(h, D), Bq, D, cfg.layer_norm_eps)
        else:
            ops.gather_rows(view(om, D), S, topk, Q, B, D, view(h, D))
        t_a = self._buf("dec_ta", Bq, D)
        t_b = self._buf("dec_tb", Bq, D)
        delta = self._buf("dec_delta", Bq, 4)
        self._lin_op(view(h, D), Bq, self.enc_bbox[0], view(t_a, D), act="relu")
        self._lin_op(view(t_a, D), Bq, self.enc_bbox[1], view(t_b, D), act="relu")
        self._lin_op(view(t_b, D), Bq, self.enc_bbox[2], view(delta, 4))
        ref = out_boxes.reshape(-1)  # refined in place, layer by layer
        ops.ref_init(view(delta, 4), anchors, topk, B, Q, ref)
        # all six value projections at once (M2:190)
        L = cfg.decoder_layers
        # bf16 variant: the value projections stored as bf16 rows (sp_msda samples them in fp32)
        vall = self._buf("value_all", rows, L * D, dtype=torch.int16 if self.bf16_store and self._lin_mode == "bf16"
                         else torch.float32)
        self._lin_op(view(src, D), rows, self.value_all, view(vall, L * D))
        # decoder (M2:578-661)
        nH, nL, nP = cfg.decoder_attention_heads, cfg.decoder_n_levels, cfg.decoder_n_points
        qp = self._buf("dec_qp", Bq, 2 * D)
        pos = self._buf("dec_pos", Bq, D)
        qk = self._buf("dec_qk", Bq, 2 * D)
        vv = self._buf("dec_v", Bq, D)
        at = self._buf("dec_at", Bq, D)
        offaw = self._buf("dec_offaw", Bq, nH * nL * nP * 3)
        ff = self._buf("dec_ff", Bq, cfg.decoder_ffn_dim)
        for j, P in enumerate(self.dec):
            self._lin_op(view(ref, 4), Bq, self.qpos[0], view(qp, 2 * D), act="relu")
            self._lin_op(view(qp, 2 * D), Bq, self.qpos[1], view(pos, D))
            # self-attention, q = k = h + pos, v = h (M2:395-404)
            self._lin_plus(view(h, D), view(pos, D), Bq, P["qk"], view(qk, 2 * D), "dec_hp")
            self._lin_op(view(h, D), Bq, P["v"], view(vv, D))
            ops.attention(V(qk, 0, 2 * D), V(qk, D, 2 * D), view(vv, D), view(at, D), B, Q, nH, D // nH,
                          (D // nH) ** -0.5, bf16=self._attn_bf16)
            self._lin_op(view(at, D), Bq, P["o"], view(h, D), res1=view(h, D), ln=P["ln1"])  # in place: row-local
            # deformable cross-attention (M2:409-423)
            self._lin_plus(view(h, D), view(pos, D), Bq, P["offaw"], view(offaw, nH * nL * nP * 3), "dec_hp")
            ops.msda(V(vall, 0, L * D), j * D, view(offaw, nH * nL * nP * 3), ref, view(at, D), B, S, Q, nH,
                     D // nH, shapes, starts, nP, cfg.decoder_offset_scale)
            self._lin_op(view(at, D), Bq, P["out"], view(h, D), res1=view(h, D), ln=P["ln2"])
            # FFN (M2:426-429)
            self._lin_op(view(h, D), Bq, P["fc1"], view(ff, cfg.decoder_ffn_dim), act=self.act_dec)
            self._lin_op(view(ff, cfg.decoder_ffn_dim), Bq, P["fc2"], view(h, D), res1=view(h, D), ln=P["ln3"])
            # iterative box refinement (M2:636-639)
            b0, b1, b2 = P["bbox"]
            self._lin_op(view(h, D), Bq, b0, view(t_a, D), act="relu")
            self._lin_op(view(t_a, D), Bq, b1, view(t_b, D), act="relu")
            self._lin_op(view(t_b, D), Bq, b2, view(delta, 4))
            ops.box_refine(view(delta, 4), ref, Bq)
            yield
        self._lin_op(view(h, D), Bq, self.cls_last, view(out_logits.reshape(-1), NC))
