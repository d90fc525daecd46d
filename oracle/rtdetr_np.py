"""TEST INFRASTRUCTURE ONLY — numpy restatement of the RT-DETRv2 /detect forward.

This is the CPU oracle the HIP path is checked against. It restates, in plain
numpy (fp32 storage, fp32 matmuls; im2col convolutions), the algorithm that
the reference runs through HF transformers: `processor(...)` →
`model(**inputs)` → `processor.post_process_object_detection(...)`
(reference apps/spotter/src/spotter/serve.py:98-109). The HF code is a
third-party dependency that is *not* vendored under /root/reference: pinned
transformers==4.50.3 (apps/spotter/uv.lock:1235-1236); this image ships 5.15.0,
whose source the citations below use (prefix M2 = models/rt_detr_v2/
modeling_rt_detr_v2.py, RN = models/rt_detr/modeling_rt_detr_resnet.py,
IPP = models/rt_detr/image_processing_pil_rt_detr.py, IT = image_transforms.py).
Pinned by tests/golden/*.npz, which oracle/make_goldens.py produced with the
HF classes themselves (oracle/hf_ref.py) on the same synthetic weights.

Known 4.50.3 ↔ 5.15.0 differences on this path, all value-preserving at the
square feature maps used here: sdpa vs eager attention (same math); the AIFI
sine embedding is built in f64 then cast (5.15) vs f32 (4.50) with a
W-outer meshgrid that equals 5.15's H-outer layout when H == W.
"""
from __future__ import annotations

import math

import numpy as np
from numpy.lib.stride_tricks import as_strided

try:
    from scipy.special import erf as _erf
except Exception:  # pragma: no cover - scipy ships in the image
    _erf = np.vectorize(math.erf)

F32 = np.float32


# ----------------------------------------------------------------------------- primitives
def conv2d_nhwc(x, w, stride=1, pad=None):
    """x [N,H,W,C] f32, w [Cout,Cin,k,k] (PyTorch layout). Zero padding k//2."""
    n, h, wd, c = x.shape
    co, ci, k, _ = w.shape
    assert ci == c, (ci, c)
    p = k // 2 if pad is None else pad
    if p:
        x = np.pad(x, ((0, 0), (p, p), (p, p), (0, 0)))
    ho = (h + 2 * p - k) // stride + 1
    wo = (wd + 2 * p - k) // stride + 1
    s0, s1, s2, s3 = x.strides
    cols = as_strided(x, (n, ho, wo, k, k, c), (s0, s1 * stride, s2 * stride, s1, s2, s3))
    cols = cols.reshape(n * ho * wo, k * k * c)
    wm = np.ascontiguousarray(w.transpose(2, 3, 1, 0).reshape(k * k * c, co))
    return (cols @ wm).astype(F32).reshape(n, ho, wo, co)


def frozen_bn(x, p, pre):
    # RTDetrV2FrozenBatchNorm2d.forward M2:748-758 (eps 1e-5 hard-coded M2:755)
    scale = p[pre + ".weight"] * (p[pre + ".running_var"] + F32(1e-5)) ** F32(-0.5)
    bias = p[pre + ".bias"] - p[pre + ".running_mean"] * scale
    return (x * scale + bias).astype(F32)


def bn_eval(x, p, pre, eps=1e-5):
    # nn.BatchNorm2d in eval mode (RTDetrV2ConvNormLayer M2:828, input proj M2:1357/1396)
    inv = (p[pre + ".running_var"] + F32(eps)) ** F32(-0.5)
    return ((x - p[pre + ".running_mean"]) * inv * p[pre + ".weight"] + p[pre + ".bias"]).astype(F32)


def relu(x):
    return np.maximum(x, F32(0))


def silu(x):
    return (x / (F32(1) + np.exp(-x))).astype(F32)


def gelu(x):  # erf GELU (ACT2FN["gelu"])
    return (F32(0.5) * x * (F32(1) + _erf(x / F32(math.sqrt(2.0))).astype(F32))).astype(F32)


def sigmoid(x):
    return (F32(1) / (F32(1) + np.exp(-x))).astype(F32)


def linear(x, p, pre):
    return (x @ p[pre + ".weight"].T + p[pre + ".bias"]).astype(F32)


def layer_norm(x, p, pre, eps=1e-5):
    mu = x.mean(-1, keepdims=True)
    var = ((x - mu) ** 2).mean(-1, keepdims=True)
    return ((x - mu) / np.sqrt(var + F32(eps)) * p[pre + ".weight"] + p[pre + ".bias"]).astype(F32)


def maxpool3s2(x):
    # nn.MaxPool2d(3, 2, 1) RN:88
    n, h, w, c = x.shape
    xp = np.pad(x, ((0, 0), (1, 1), (1, 1), (0, 0)), constant_values=-np.inf)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    out = np.full((n, ho, wo, c), -np.inf, F32)
    for dy in range(3):
        for dx in range(3):
            out = np.maximum(out, xp[:, dy:dy + 2 * ho:2, dx:dx + 2 * wo:2, :])
    return out


def avgpool2_ceil(x):
    # nn.AvgPool2d(2, 2, 0, ceil_mode=True) RN:150,202: windows clipped to the input
    n, h, w, c = x.shape
    ho, wo = (h + 1) // 2, (w + 1) // 2
    xp = np.zeros((n, ho * 2, wo * 2, c), F32)
    cnt = np.zeros((ho * 2, wo * 2), F32)
    xp[:, :h, :w] = x
    cnt[:h, :w] = 1
    s = xp.reshape(n, ho, 2, wo, 2, c).sum((2, 4))
    k = cnt.reshape(ho, 2, wo, 2).sum((1, 3))
    return (s / k[None, :, :, None]).astype(F32)


def upsample2(x):
    # F.interpolate(scale_factor=2, mode="nearest") M2:1192
    return np.repeat(np.repeat(x, 2, axis=1), 2, axis=2)


def mha(xq, xk, xv, p, pre, heads):
    # RTDetrV2SelfAttention M2:300-336 (q=k=x+pos, v=x), eager_attention_forward M2:245-270
    b, n, d = xq.shape
    dh = d // heads
    q = linear(xq, p, pre + ".q_proj").reshape(b, n, heads, dh).transpose(0, 2, 1, 3)
    k = linear(xk, p, pre + ".k_proj").reshape(b, n, heads, dh).transpose(0, 2, 1, 3)
    v = linear(xv, p, pre + ".v_proj").reshape(b, n, heads, dh).transpose(0, 2, 1, 3)
    s = (q @ k.transpose(0, 1, 3, 2)) * F32(dh ** -0.5)
    s = s - s.max(-1, keepdims=True)
    e = np.exp(s)
    a = (e / e.sum(-1, keepdims=True)).astype(F32)
    o = (a @ v).transpose(0, 2, 1, 3).reshape(b, n, d)
    return linear(o, p, pre + ".o_proj")


def sine_pos_embed(h, w, dim, temperature):
    # build_2d_sinusoidal_position_embedding M2:955-1000 (f64, [sin_h|cos_h|sin_w|cos_w], H-outer)
    pd = dim // 4
    omega = 1.0 / temperature ** (np.arange(pd, dtype=np.float64) / pd)
    gh, gw = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
    eh = np.outer(gh.reshape(-1), omega)
    ew = np.outer(gw.reshape(-1), omega)
    return np.concatenate([np.sin(eh), np.cos(eh), np.sin(ew), np.cos(ew)], 1).astype(F32)


def anchors_for(shapes, grid_size=0.05):
    # _cached_generate_anchors M2:1421-1449
    anchors = []
    for lvl, (h, w) in enumerate(shapes):
        gy, gx = np.meshgrid(np.arange(h, dtype=F32), np.arange(w, dtype=F32), indexing="ij")
        xy = np.stack([gx, gy], -1) + F32(0.5)
        xy[..., 0] /= F32(w)
        xy[..., 1] /= F32(h)
        wh = np.ones_like(xy) * F32(grid_size * 2.0 ** lvl)
        anchors.append(np.concatenate([xy, wh], -1).reshape(h * w, 4))
    a = np.concatenate(anchors, 0).astype(F32)
    valid = ((a > F32(1e-2)) & (a < F32(1 - 1e-2))).all(-1, keepdims=True)
    lg = np.log(a / (F32(1) - a)).astype(F32)
    lg = np.where(valid, lg, np.finfo(F32).max).astype(F32)
    return lg, valid


def grid_sample_bilinear(value, loc):
    """grid_sample(bilinear, zeros, align_corners=False) with loc in [0,1] (M2:79-81).

    value [BH, Hl, Wl, Dh]; loc [BH, Q, P, 2] (x, y) → [BH, Q, P, Dh].
    """
    bh, hl, wl, dh = value.shape
    x = loc[..., 0] * F32(wl) - F32(0.5)
    y = loc[..., 1] * F32(hl) - F32(0.5)
    x0 = np.floor(x)
    y0 = np.floor(y)
    out = np.zeros(loc.shape[:-1] + (dh,), F32)
    bidx = np.arange(bh)[:, None, None]
    for dy in (0, 1):
        for dx in (0, 1):
            xi = x0 + dx
            yi = y0 + dy
            wgt = (F32(1) - np.abs(x - xi)) * (F32(1) - np.abs(y - yi))
            ok = (xi >= 0) & (xi < wl) & (yi >= 0) & (yi < hl)
            xc = np.clip(xi, 0, wl - 1).astype(np.int64)
            yc = np.clip(yi, 0, hl - 1).astype(np.int64)
            v = value[bidx, yc, xc]
            out += (v * (wgt * ok)[..., None]).astype(F32)
    return out


def msda(h, pos, src, ref, p, pre, cfg, shapes, starts):
    # RTDetrV2MultiscaleDeformableAttention.forward M2:166-225 + core M2:44-115
    b, nq, d = h.shape
    nH, nL, nP = cfg.decoder_attention_heads, cfg.decoder_n_levels, cfg.decoder_n_points
    dh = d // nH
    hs = h + pos
    value = linear(src, p, pre + ".value_proj").reshape(b, -1, nH, dh)
    off = linear(hs, p, pre + ".sampling_offsets").reshape(b, nq, nH, nL * nP, 2)
    aw = linear(hs, p, pre + ".attention_weights").reshape(b, nq, nH, nL * nP)
    aw = aw - aw.max(-1, keepdims=True)
    aw = np.exp(aw)
    aw = (aw / aw.sum(-1, keepdims=True)).astype(F32)
    nps = p[pre + ".n_points_scale"].reshape(1, 1, 1, nL * nP, 1)
    # M2:212-215: loc = ref_xy + off * (1/P) * ref_wh * offset_scale
    offs = off * nps * ref[:, :, None, None, 2:] * F32(cfg.decoder_offset_scale)
    loc = (ref[:, :, None, None, :2] + offs).astype(F32)
    out = np.zeros((b, nH, nq, dh), F32)
    for l, (hl, wl) in enumerate(shapes):
        v = value[:, starts[l]:starts[l] + hl * wl].reshape(b, hl, wl, nH, dh)
        v = v.transpose(0, 3, 1, 2, 4).reshape(b * nH, hl, wl, dh)
        lc = loc[:, :, :, l * nP:(l + 1) * nP].transpose(0, 2, 1, 3, 4).reshape(b * nH, nq, nP, 2)
        sv = grid_sample_bilinear(v, lc).reshape(b, nH, nq, nP, dh)
        a = aw[:, :, :, l * nP:(l + 1) * nP].transpose(0, 2, 1, 3)[..., None]
        out += (sv * a).sum(3)
    out = out.transpose(0, 2, 1, 3).reshape(b, nq, d)
    return linear(out, p, pre + ".output_proj")


def inverse_sigmoid(x, eps=1e-5):
    # M2:548-552
    x = np.clip(x, 0, 1)
    return np.log(np.clip(x, eps, None) / np.clip(1 - x, eps, None)).astype(F32)


def topk_desc(vals, k):
    """Indices of the k largest along the last axis; ties → lower index first."""
    idx = np.argsort(-vals, axis=-1, kind="stable")[..., :k]
    return idx


# ----------------------------------------------------------------------------- model
def backbone(x, p, cfg, feats=None):
    from spotter_amd.weights import backbone_plan

    bb = "model.backbone.model"
    h = x
    for i, st in enumerate((2, 1, 1)):  # stem RN:78-103
        pre = f"{bb}.embedder.embedder.{i}"
        h = relu(frozen_bn(conv2d_nhwc(h, p[pre + ".convolution.weight"], st), p, pre + ".normalization"))
    h = maxpool3s2(h)
    outs = []
    cur_stage = 0
    for (s, i, lt, cin, cout, st, sc) in backbone_plan(cfg):
        if s != cur_stage:
            outs.append(h)
            cur_stage = s
        pre = f"{bb}.encoder.stages.{s}.layers.{i}"
        res = h
        if sc == "conv":
            res = frozen_bn(conv2d_nhwc(res, p[pre + ".shortcut.convolution.weight"], st), p,
                            pre + ".shortcut.normalization")
        elif sc == "avgconv":
            res = avgpool2_ceil(res)
            res = frozen_bn(conv2d_nhwc(res, p[pre + ".shortcut.1.convolution.weight"], 1), p,
                            pre + ".shortcut.1.normalization")
        if lt == "bottleneck":  # RN:179-231, stride on the 3×3 (RN:215-220)
            t = relu(frozen_bn(conv2d_nhwc(h, p[pre + ".layer.0.convolution.weight"], 1), p, pre + ".layer.0.normalization"))
            t = relu(frozen_bn(conv2d_nhwc(t, p[pre + ".layer.1.convolution.weight"], st), p, pre + ".layer.1.normalization"))
            t = frozen_bn(conv2d_nhwc(t, p[pre + ".layer.2.convolution.weight"], 1), p, pre + ".layer.2.normalization")
        else:  # RN:135-175
            t = relu(frozen_bn(conv2d_nhwc(h, p[pre + ".layer.0.convolution.weight"], st), p, pre + ".layer.0.normalization"))
            t = frozen_bn(conv2d_nhwc(t, p[pre + ".layer.1.convolution.weight"], 1), p, pre + ".layer.1.normalization")
        h = relu(t + res)
    outs.append(h)
    return outs[1:]  # out_indices [2,3,4] → stage2..stage4 outputs (RN:405-408)


def conv_norm(x, p, pre, stride=1, act=None):
    # RTDetrV2ConvNormLayer M2:817-835
    y = bn_eval(conv2d_nhwc(x, p[pre + ".conv.weight"], stride), p, pre + ".norm")
    return silu(y) if act == "silu" else y


def csp(x, p, pre, cfg):
    # RTDetrV2CSPRepLayer M2:926-952 with RepVGG blocks M2:907-923
    h1 = conv_norm(x, p, pre + ".conv1", act="silu")
    for b in range(3):
        q = f"{pre}.bottlenecks.{b}"
        h1 = silu(conv_norm(h1, p, q + ".conv1") + conv_norm(h1, p, q + ".conv2"))
    h2 = conv_norm(x, p, pre + ".conv2", act="silu")
    s = h1 + h2
    if int(cfg.encoder_hidden_dim * cfg.hidden_expansion) != cfg.encoder_hidden_dim:
        s = conv_norm(s, p, pre + ".conv3", act="silu")
    return s


def hybrid_encoder(feats, p, cfg):
    # RTDetrV2HybridEncoder.forward M2:1164-1209; AIFI M2:1058-1095
    H = cfg.encoder_hidden_dim
    fm = list(feats)
    x = fm[2]
    b, hh, ww, _ = x.shape
    t = x.reshape(b, hh * ww, H)
    pos = sine_pos_embed(hh, ww, H, cfg.positional_encoding_temperature)[None]
    a = "model.encoder.aifi.0.layers.0"
    # RTDetrV2EncoderLayer M2:856-904 (post-norm)
    r = t
    t = mha(t + pos, t + pos, t, p, a + ".self_attn", cfg.encoder_attention_heads)
    t = layer_norm(r + t, p, a + ".self_attn_layer_norm")
    r = t
    t = linear(gelu(linear(t, p, a + ".mlp.fc1")), p, a + ".mlp.fc2")
    t = layer_norm(r + t, p, a + ".final_layer_norm")
    fm[2] = t.reshape(b, hh, ww, H)
    # FPN M2:1183-1197
    fpn = [fm[-1]]
    for idx in range(len(fm) - 1):
        bbm = fm[len(fm) - 2 - idx]
        top = conv_norm(fpn[-1], p, f"model.encoder.lateral_convs.{idx}", act="silu")
        fpn[-1] = top
        fused = np.concatenate([upsample2(top), bbm], -1)
        fpn.append(csp(fused, p, f"model.encoder.fpn_blocks.{idx}", cfg))
    fpn.reverse()
    # PAN M2:1199-1207
    pan = [fpn[0]]
    for idx in range(len(fm) - 1):
        d = conv_norm(pan[-1], p, f"model.encoder.downsample_convs.{idx}", stride=2, act="silu")
        fused = np.concatenate([d, fpn[idx + 1]], -1)
        pan.append(csp(fused, p, f"model.encoder.pan_blocks.{idx}", cfg))
    return pan


def forward(pixel_values, p, cfg, want=None):
    """pixel_values [B,3,H,W] f32 → dict(logits [B,Q,C], pred_boxes [B,Q,4], + intermediates)."""
    st = {}
    x = np.ascontiguousarray(pixel_values.transpose(0, 2, 3, 1)).astype(F32)
    feats = backbone(x, p, cfg)
    st["backbone"] = feats
    # encoder_input_proj M2:1512
    proj = [bn_eval(conv2d_nhwc(f, p[f"model.encoder_input_proj.{l}.0.weight"], 1), p,
                    f"model.encoder_input_proj.{l}.1") for l, f in enumerate(feats)]
    st["proj"] = proj
    enc = hybrid_encoder(proj, p, cfg)
    st["encoder"] = enc
    # decoder_input_proj + flatten M2:1533-1556
    srcs, shapes = [], []
    for l, e in enumerate(enc):
        s = bn_eval(conv2d_nhwc(e, p[f"model.decoder_input_proj.{l}.0.weight"], 1), p,
                    f"model.decoder_input_proj.{l}.1")
        b, hh, ww, d = s.shape
        shapes.append((hh, ww))
        srcs.append(s.reshape(b, hh * ww, d))
    src = np.concatenate(srcs, 1)
    starts = np.concatenate([[0], np.cumsum([h * w for h, w in shapes])[:-1]]).astype(int)
    st["source_flatten"] = src
    # query selection M2:1582-1623
    anchors, valid = anchors_for(shapes)
    memory = (valid.astype(F32)[None] * src).astype(F32)
    om = layer_norm(linear(memory, p, "model.enc_output.0"), p, "model.enc_output.1")
    cls = linear(om, p, "model.enc_score_head")
    topk = topk_desc(cls.max(-1), cfg.num_queries)
    st["enc_topk_ind"] = topk
    st["enc_outputs_class"] = cls
    bsel = np.take_along_axis(om, topk[..., None], 1)
    t = relu(linear(bsel, p, "model.enc_bbox_head.layers.0"))
    t = relu(linear(t, p, "model.enc_bbox_head.layers.1"))
    ref_unact = (linear(t, p, "model.enc_bbox_head.layers.2") + anchors[topk]).astype(F32)
    target = bsel
    # decoder M2:578-661
    ref = sigmoid(ref_unact)
    h = target
    D = cfg.d_model
    logits = None
    for j in range(cfg.decoder_layers):
        pre = f"model.decoder.layers.{j}"
        qp = relu(linear(ref, p, "model.decoder.query_pos_head.layers.0"))
        pos = linear(qp, p, "model.decoder.query_pos_head.layers.1")
        r = h
        t = mha(h + pos, h + pos, h, p, pre + ".self_attn", cfg.decoder_attention_heads)
        h = layer_norm(r + t, p, pre + ".self_attn_layer_norm")
        r = h
        t = msda(h, pos, src, ref, p, pre + ".encoder_attn", cfg, shapes, starts)
        h = layer_norm(r + t, p, pre + ".encoder_attn_layer_norm")
        r = h
        t = linear(relu(linear(h, p, pre + ".mlp.fc1")), p, pre + ".mlp.fc2")
        h = layer_norm(r + t, p, pre + ".final_layer_norm")
        q = f"model.decoder.bbox_embed.{j}"
        t = relu(linear(h, p, q + ".layers.0"))
        t = relu(linear(t, p, q + ".layers.1"))
        delta = linear(t, p, q + ".layers.2")
        ref = sigmoid(delta + inverse_sigmoid(ref))
        st[f"dec{j}"] = h
        if j == cfg.decoder_layers - 1:
            logits = linear(h, p, f"model.decoder.class_embed.{j}")
    st["logits"] = logits
    st["pred_boxes"] = ref
    return st


# ----------------------------------------------------------------------------- post-process
def post_process(logits, boxes, target_sizes, threshold=0.5):
    """post_process_object_detection (use_focal_loss=True) IPP:508-578 / IT:529-536."""
    cx, cy, w, h = [boxes[..., i] for i in range(4)]
    xyxy = np.stack([cx - F32(0.5) * w, cy - F32(0.5) * h, cx + F32(0.5) * w, cy + F32(0.5) * h], -1)
    res = []
    b, q, c = logits.shape
    for i in range(b):
        ih, iw = target_sizes[i]
        sc = np.array([iw, ih, iw, ih], F32)
        bx = (xyxy[i] * sc).astype(F32)
        s = sigmoid(logits[i]).reshape(-1)
        idx = topk_desc(s, q)
        ss = s[idx]
        lab = idx % c
        qi = idx // c
        keep = ss > threshold
        res.append({"scores": ss[keep], "labels": lab[keep].astype(np.int64), "boxes": bx[qi][keep]})
    return res
