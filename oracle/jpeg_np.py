"""TEST INFRASTRUCTURE ONLY (never imported by spotter_amd): numpy restatement of the pixel half of the JPEG
decode that serve.py:96-97 runs through Pillow (`Image.open(BytesIO(..)).convert("RGB")`).

Pillow 12.2.0 (this image; the reference pins 11.1.0, apps/spotter/uv.lock:582-583) decodes JPEG with its
bundled libjpeg-turbo, a dependency absent from /root/reference. Its published algorithms, restated:
  * jidctint.c jpeg_idct_islow — the ISLOW integer IDCT (CONST_BITS 13, PASS1_BITS 2, the 12 FIX_ constants,
    DESCALE rounding, IDCT_range_limit's & RANGE_MASK wrap + clamp from jdmaster.c prepare_range_limit_table);
  * jdsample.c h2v1 / h2v2 / h1v2_fancy_upsample (+ the box forms for downsampled widths <= 2), with the edge
    rows jdmainct.c's context pointers replicate;
  * jdcolor.c build_ycc_rgb_table / ycc_rgb_convert (SCALEBITS 16).
The input is the quantised coefficient array sp_jpeg_decode_coefs (the library's host entropy decoder)
returns; tests/test_jpeg.py checks this restatement, fed by that decoder, against Pillow's own decode bit for
bit (progressive and baseline, 4:4:4 / 4:2:2 / 4:2:0, gray, odd sizes, restart markers) — that pins both —
and the GPU kernels (csrc/jpeg.hip) against Pillow directly.
"""
from __future__ import annotations

import numpy as np

CB, P1 = 13, 2
F = dict(F0_298=2446, F0_390=3196, F0_541=4433, F0_765=6270, F0_899=7373, F1_175=9633, F1_501=12299, F1_847=15137,
         F1_961=16069, F2_053=16819, F2_562=20995, F3_072=25172)


def _islow_1d(v, shift):
    """jidctint.c's butterfly along axis -1 of int64 v [..., 8]; returns DESCALE(·, shift)."""
    z2, z3 = v[..., 2], v[..., 6]
    z1 = (z2 + z3) * F["F0_541"]
    tmp2 = z1 + z3 * -F["F1_847"]
    tmp3 = z1 + z2 * F["F0_765"]
    t0 = (v[..., 0] + v[..., 4]) << CB
    t1 = (v[..., 0] - v[..., 4]) << CB
    tmp10, tmp13, tmp11, tmp12 = t0 + tmp3, t0 - tmp3, t1 + tmp2, t1 - tmp2
    o0, o1, o2, o3 = v[..., 7], v[..., 5], v[..., 3], v[..., 1]
    z1, z2, z3, z4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
    z5 = (z3 + z4) * F["F1_175"]
    o0, o1, o2, o3 = o0 * F["F0_298"], o1 * F["F2_053"], o2 * F["F3_072"], o3 * F["F1_501"]
    z1, z2, z3, z4 = z1 * -F["F0_899"], z2 * -F["F2_562"], z3 * -F["F1_961"] + z5, z4 * -F["F0_390"] + z5
    o0, o1, o2, o3 = o0 + z1 + z3, o1 + z2 + z4, o2 + z2 + z3, o3 + z1 + z4
    r = 1 << (shift - 1)
    out = [tmp10 + o3, tmp11 + o2, tmp12 + o1, tmp13 + o0, tmp13 - o0, tmp12 - o1, tmp11 - o2, tmp10 - o3]
    return np.stack([(x + r) >> shift for x in out], -1)


def idct_islow(blocks, quant):
    """blocks int16 [n, 64] natural order, quant [64] → uint8 [n, 8, 8] (jpeg_idct_islow)."""
    c = blocks.astype(np.int64).reshape(-1, 8, 8) * quant.astype(np.int64).reshape(8, 8)
    ws = _islow_1d(np.swapaxes(c, 1, 2), CB - P1)       # pass 1 on columns: ws[n, col, row]
    ws = np.swapaxes(ws.astype(np.int32).astype(np.int64), 1, 2)  # (int) workspace → [n, row, col]
    out = _islow_1d(ws, CB + P1 + 3)                    # pass 2 on rows
    v = out & 1023
    v = np.where(v >= 512, v - 1024, v) + 128
    return np.clip(v, 0, 255).astype(np.uint8)


def simd_envelope_ok(coefs, lay) -> bool:
    """Mirror of the GPU IDCT's status flag (csrc/jpeg.hip kEnv16): True when every block stays where this
    C-semantics IDCT and libjpeg-turbo's SIMD IDCT (Pillow on x86) agree — dequantised and pass-1 values within
    +-(2^14 - 1), pass-2 values within [-512, 511]. Files outside it are left to Pillow (tests/test_jpeg_corpus.py
    found every divergent corrupt file outside it and no well-formed one)."""
    env = (1 << 14) - 1
    for c in range(lay["ncomp"]):
        nb, off = lay["bw"][c] * lay["bh"][c], lay["block_off"][c]
        b = coefs[off:off + nb].astype(np.int64).reshape(-1, 8, 8) * np.asarray(lay["quant"][c], np.int64).reshape(8, 8)
        ws = _islow_1d(np.swapaxes(b, 1, 2), CB - P1)
        out = _islow_1d(np.swapaxes(ws, 1, 2), CB + P1 + 3)
        if np.abs(b).max() > env or np.abs(ws).max() > env or out.max() > 511 or out.min() < -512:
            return False
    return True


def planes(coefs, lay):
    """Component sample planes [bh*8, bw*8] from the coefficient array and layout (dict of lists)."""
    out = []
    for c in range(lay["ncomp"]):
        nb = lay["bw"][c] * lay["bh"][c]
        o = lay["block_off"][c]
        px = idct_islow(coefs[o:o + nb], np.asarray(lay["quant"][c]))
        out.append(px.reshape(lay["bh"][c], lay["bw"][c], 8, 8).transpose(0, 2, 1, 3)
                   .reshape(lay["bh"][c] * 8, lay["bw"][c] * 8))
    return out


def _upsample(pl, rh, rv, dw, dh, W, H):
    """jdsample.c fancy upsampling of one component to [H, W] (int)."""
    p = pl[:dh, :dw].astype(np.int64)
    if rh == 1 and rv == 1:
        return p[:H, :W]
    if rv == 2:  # vertical neighbours: the row above for even output rows, below for odd; edges replicated
        up = np.concatenate([p[:1], p[:-1]], 0)
        dn = np.concatenate([p[1:], p[-1:]], 0)
    if rh == 2 and dw <= 2:  # box replication (h2v1_upsample / h2v2_upsample)
        return np.repeat(np.repeat(p, 2, 1), rv, 0)[:H, :W]
    if rh == 2 and rv == 1:  # h2v1_fancy_upsample
        left = np.concatenate([p[:, :1], p[:, :-1]], 1)
        right = np.concatenate([p[:, 1:], p[:, -1:]], 1)
        even = (p * 3 + left + 1) >> 2
        odd = (p * 3 + right + 2) >> 2
        even[:, 0] = p[:, 0]
        odd[:, -1] = p[:, -1]
        o = np.stack([even, odd], 2).reshape(dh, 2 * dw)
        return o[:H, :W]
    if rh == 1:  # h1v2_fancy_upsample
        o = np.stack([(p * 3 + up + 1) >> 2, (p * 3 + dn + 2) >> 2], 1).reshape(2 * dh, dw)
        return o[:H, :W]
    rows = []
    for nb in (up, dn):  # h2v2_fancy_upsample: even output rows pair with the row above, odd with below
        cs = p * 3 + nb
        left = np.concatenate([cs[:, :1], cs[:, :-1]], 1)
        right = np.concatenate([cs[:, 1:], cs[:, -1:]], 1)
        even = (cs * 3 + left + 8) >> 4
        odd = (cs * 3 + right + 7) >> 4
        even[:, 0] = (cs[:, 0] * 4 + 8) >> 4
        odd[:, -1] = (cs[:, -1] * 4 + 7) >> 4
        rows.append(np.stack([even, odd], 2).reshape(dh, 2 * dw))
    o = np.stack(rows, 1).reshape(2 * dh, 2 * dw)
    return o[:H, :W]


def to_rgb(coefs, lay):
    """Pillow's convert("RGB") pixels, uint8 [H, W, 3], from the coefficient array + layout."""
    W, H = lay["width"], lay["height"]
    pl = planes(coefs, lay)
    y = pl[0][:H, :W].astype(np.int64)
    if lay["ncomp"] == 1:
        return np.repeat(y[..., None], 3, 2).astype(np.uint8)
    cc = []
    for k in (1, 2):
        rh, rv = lay["max_h"] // lay["h"][k], lay["max_v"] // lay["v"][k]
        dw = -(-W * lay["h"][k] // lay["max_h"])
        dh = -(-H * lay["v"][k] // lay["max_v"])
        cc.append(_upsample(pl[k], rh, rv, dw, dh, W, H))
    if lay["color"] == 2:
        return np.stack([y, cc[0], cc[1]], -1).astype(np.uint8)
    cb, cr = cc[0] - 128, cc[1] - 128
    r = y + ((91881 * cr + 32768) >> 16)
    g = y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)
    b = y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)
