"""TEST INFRASTRUCTURE ONLY (never imported by spotter_amd): numpy restatement of the JPEG *encode* that
serve.py:139-142 runs through Pillow (`image.save(buffer, format="JPEG")`, then base64).

Pillow 12.2.0 (the reference pins 11.1.0, apps/spotter/uv.lock:582-583) writes JPEG with its bundled
libjpeg-turbo, a dependency absent from /root/reference. Pillow's JpegImagePlugin._save passes quality -1
(libjpeg's default 75), subsampling -1 (libjpeg's default 2x2 luma, i.e. 4:2:0), no optimize / progressive /
restart / dpi / EXIF / ICC, and `im.info["comment"]` if the image carries one. libjpeg-turbo's published
algorithms for that configuration, restated:
  * jcparam.c: jpeg_set_quality / jpeg_quality_scaling / jpeg_add_quant_table (Annex K tables scaled,
    force_baseline clamp to 255), the Annex K.3 Huffman tables (std_huff_tables), component ids 1/2/3,
    table selectors Y -> 0, Cb/Cr -> 1;
  * jccolor.c rgb_ycc_convert: SCALEBITS 16 fixed point, Cb/Cr rounding fudge ONE_HALF - 1;
  * jcsample.c fullsize / h2v1 / h2v2_downsample: edge expansion to the block-padded width, the 1,2,1,2 / 0,1
    rounding bias; jcprepct.c: bottom rows replicated to the row group, then to the full iMCU height;
  * jcdctmgr.c convsamp (-128) + jfdctint.c jpeg_fdct_islow (CONST_BITS 13, PASS1_BITS 2, output scaled by
    8) + quantize with compute_reciprocal's reciprocal / correction / shift (divisor = quantval << 3);
  * jccoefct.c compress_data: dummy blocks past the image edge inside the last MCU column / row (zero AC,
    DC copied from the block before them);
  * jchuff.c encode_one_block + emit_bits (0xFF byte stuffing) + flush_bits (1-bit padding);
  * jcmarker.c: SOI, JFIF APP0 (1.01, density 0 / 1:1), [COM], DQT per table, SOF0, DHT per table in scan
    order, SOS, EOI.
tests/test_jpeg_enc.py pins this restatement against Pillow's own output byte for byte; the GPU encoder
(spotter_amd/csrc/jpeg_enc.hip + jpeg_host.h) is then checked against both.
"""
from __future__ import annotations

import numpy as np

NATURAL = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                    13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                    45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])

STD_LUM_Q = [16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
             14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99]
STD_CHR_Q = [17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99, 24, 26, 56, 99, 99, 99, 99, 99,
             47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32

# Annex K.3 (jcparam.c std_huff_tables): 16 code-length counts, then the symbols
DC_LUM = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
DC_CHR = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
AC_LUM = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])
AC_CHR = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa])

# Pillow's subsampling argument -> luma (h, v) sampling (chroma at 1x1); -1 is libjpeg's default 2x2
SAMPLING = {-1: (2, 2), 0: (1, 1), 1: (2, 1), 2: (2, 2)}


def quant_tables(quality: int = -1):
    """jpeg_set_quality(quality, force_baseline=TRUE); quality -1 is jpeg_set_defaults' 75. Natural order."""
    q = 75 if quality == -1 else min(max(quality, 1), 100)
    scale = 5000 // q if q < 50 else 200 - 2 * q
    out = []
    for basic in (STD_LUM_Q, STD_CHR_Q):
        t = (np.array(basic, np.int64) * scale + 50) // 100
        out.append(np.clip(t, 1, 255))  # <= 0 -> 1; > 32767 -> 32767; force_baseline: > 255 -> 255
    return out


def _fix(x):
    return int(x * 65536 + 0.5)


def rgb_to_ycc(rgb):
    """jccolor.c rgb_ycc_convert on uint8 [H, W, 3] -> three uint8 planes."""
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    half, off = 1 << 15, 128 << 16
    y = (_fix(0.29900) * r + _fix(0.58700) * g + _fix(0.11400) * b + half) >> 16
    cb = (-_fix(0.16874) * r - _fix(0.33126) * g + _fix(0.5) * b + off + half - 1) >> 16
    cr = (_fix(0.5) * r - _fix(0.41869) * g - _fix(0.08131) * b + off + half - 1) >> 16
    return [p.astype(np.int64) for p in (y, cb, cr)]


def component_planes(rgb, hs, vs):
    """The block-padded sample planes libjpeg-turbo's prep / downsample controllers hand the FDCT, for luma
    sampling (hs, vs) with chroma at 1x1. Returns [(plane int64 [hb*8 rows, wb*8 cols], h, v)] per component."""
    H, W, _ = rgb.shape
    full = rgb_to_ycc(rgb)
    out = []
    for c, pl in enumerate(full):
        h, v = (hs, vs) if c == 0 else (1, 1)
        rh, rv = hs // h, vs // v
        wb = -(-W * h // (hs * 8))  # ceil(W * h / (max_h * 8)): jdinput/jcmaster width_in_blocks
        hb = -(-H * v // (vs * 8))
        ow = wb * 8
        # expand_right_edge: replicate the last column to ow * rh input columns
        cols = np.minimum(np.arange(ow * rh), W - 1)
        x = pl[:, cols]
        # jcprepct.c: rows padded (replicating the last) to a multiple of the row group max_v
        ng = -(-H // vs) * vs
        x = x[np.minimum(np.arange(ng), H - 1)]
        if rh == 2 and rv == 2:
            s = x[0::2, 0::2] + x[0::2, 1::2] + x[1::2, 0::2] + x[1::2, 1::2]
            bias = np.where(np.arange(ow) % 2 == 0, 1, 2)
            d = (s + bias) >> 2
        elif rh == 2 and rv == 1:
            s = x[:, 0::2] + x[:, 1::2]
            bias = np.where(np.arange(ow) % 2 == 0, 0, 1)
            d = (s + bias) >> 1
        else:
            d = x
        # then the downsampled rows padded (replicating the last) to the full iMCU height
        rows_out = -(-H // vs) * vs // rv
        d = d[:rows_out]
        imcu_rows = -(-H // (vs * 8)) * v * 8
        d = d[np.minimum(np.arange(imcu_rows), d.shape[0] - 1)]
        out.append((d, h, v, wb, hb))
    return out


def _fdct_1d(x, shift_even, pass2):
    """jfdctint.c's butterfly along axis -1 (int64 [..., 8]); pass 1: DESCALE by CONST_BITS - PASS1_BITS with the
    even DC/4 terms left-shifted by PASS1_BITS; pass 2: everything DESCALEd (CONST_BITS + PASS1_BITS / PASS1_BITS)."""
    CB, P1 = 13, 2
    d = [x[..., i] for i in range(8)]
    tmp0, tmp7 = d[0] + d[7], d[0] - d[7]
    tmp1, tmp6 = d[1] + d[6], d[1] - d[6]
    tmp2, tmp5 = d[2] + d[5], d[2] - d[5]
    tmp3, tmp4 = d[3] + d[4], d[3] - d[4]
    tmp10, tmp13 = tmp0 + tmp3, tmp0 - tmp3
    tmp11, tmp12 = tmp1 + tmp2, tmp1 - tmp2

    def ds(v, n):
        return (v + (1 << (n - 1))) >> n

    sh = CB + P1 if pass2 else CB - P1
    o = [None] * 8
    if pass2:
        o[0], o[4] = ds(tmp10 + tmp11, P1), ds(tmp10 - tmp11, P1)
    else:
        o[0], o[4] = (tmp10 + tmp11) << P1, (tmp10 - tmp11) << P1
    z1 = (tmp12 + tmp13) * 4433
    o[2] = ds(z1 + tmp13 * 6270, sh)
    o[6] = ds(z1 + tmp12 * -15137, sh)
    z1, z2, z3, z4 = tmp4 + tmp7, tmp5 + tmp6, tmp4 + tmp6, tmp5 + tmp7
    z5 = (z3 + z4) * 9633
    tmp4, tmp5, tmp6, tmp7 = tmp4 * 2446, tmp5 * 16819, tmp6 * 25172, tmp7 * 12299
    z1, z2, z3, z4 = z1 * -7373, z2 * -20995, z3 * -16069 + z5, z4 * -3196 + z5
    o[7] = ds(tmp4 + z1 + z3, sh)
    o[5] = ds(tmp5 + z2 + z4, sh)
    o[3] = ds(tmp6 + z2 + z3, sh)
    o[1] = ds(tmp7 + z1 + z4, sh)
    return np.stack(o, -1)


def fdct_islow(blocks):
    """int64 [n, 8, 8] level-shifted samples -> [n, 8, 8] DCT coefficients scaled by 8 (jpeg_fdct_islow)."""
    ws = _fdct_1d(blocks, None, False)                     # rows
    out = _fdct_1d(np.swapaxes(ws, 1, 2), None, True)      # columns
    return np.swapaxes(out, 1, 2)


def reciprocal(divisor: int):
    """jcdctmgr.c compute_reciprocal with 16-bit DCTELEM (libjpeg-turbo's SIMD build): (recip, corr, shift)."""
    if divisor == 1:
        return 1, 0, -16  # product >> (shift + 16) = product
    b = divisor.bit_length() - 1
    r = 16 + b
    fq, fr = divmod(1 << r, divisor)
    c = divisor // 2
    if fr == 0:
        fq >>= 1
        r -= 1
    elif fr <= divisor // 2:
        c += 1
    else:
        fq += 1
    return fq, c, r - 16


def quantize(coef, qtab):
    """coef int64 [n, 64] natural order, qtab [64] -> quantised int64 [n, 64] (jcdctmgr.c quantize)."""
    out = np.empty_like(coef)
    for i in range(64):
        fq, c, sh = reciprocal(int(qtab[i]) << 3)
        x = coef[:, i]
        a = (np.abs(x) + c) * fq >> (sh + 16)
        out[:, i] = np.where(x < 0, -a, a)
    return out


def coefficient_blocks(rgb, quality=-1, subsampling=-1):
    """uint8 RGB [H, W, 3] -> per component (quantised blocks int64 [hbp, wbp, 64] natural order, h, v) with
    the MCU-padded block grid (hbp = mcu_rows * v, wbp = mcu_cols * h) including jccoefct.c's dummy blocks."""
    hs, vs = SAMPLING[subsampling]
    H, W, _ = rgb.shape
    qt = quant_tables(quality)
    mcux, mcuy = -(-W // (8 * hs)), -(-H // (8 * vs))
    out = []
    for c, (pl, h, v, wb, hb) in enumerate(component_planes(rgb, hs, vs)):
        blk = pl[:hb * 8, :wb * 8].reshape(hb, 8, wb, 8).transpose(0, 2, 1, 3).reshape(-1, 8, 8) - 128
        co = quantize(fdct_islow(blk).reshape(-1, 64), qt[0 if c == 0 else 1]).reshape(hb, wb, 64)
        full = np.zeros((mcuy * v, mcux * h, 64), np.int64)
        full[:hb, :wb] = co
        # dummy blocks (jccoefct.c compress_data), walked in MCU order: a right-edge dummy copies the DC of the
        # block to its left; a dummy row below the image copies the DC of the last block of the row above
        for my in range(mcuy):
            for mx in range(mcux):
                for yy in range(v):
                    by = my * v + yy
                    for xx in range(h):
                        bx = mx * h + xx
                        if by < hb and bx < wb:
                            continue
                        if by < hb:
                            full[by, bx, 0] = full[by, bx - 1, 0]
                        else:
                            prev = (by - 1, mx * h + h - 1) if xx == 0 else (by, bx - 1)
                            full[by, bx, 0] = full[prev][0]
        out.append((full, h, v))
    return out, qt


def _derive(table):
    """jchuff.c jpeg_make_c_derived_tbl: symbol -> (code, length)."""
    bits, vals = table
    codes, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(bits[ln - 1]):
            codes[vals[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return codes


class _BitWriter:
    def __init__(self, stuff=True):
        self.out = bytearray()
        self.acc = 0
        self.n = 0
        self.stuff = stuff
        self.total = 0

    def put(self, code, size):
        self.acc = (self.acc << size) | (code & ((1 << size) - 1))
        self.n += size
        self.total += size
        while self.n >= 8:
            self.n -= 8
            byte = (self.acc >> self.n) & 0xFF
            self.out.append(byte)
            if byte == 0xFF and self.stuff:
                self.out.append(0)  # emit_byte's stuffing
        self.acc &= (1 << self.n) - 1

    def flush(self):
        self.put(0x7F, 7)  # flush_bits: pad with 1s; the partial rest is dropped
        self.acc, self.n = 0, 0


def entropy_bits(comps, stuff=True):
    """The scan's entropy-coded segment (stuffed, padded) for the interleaved baseline scan; stuff=False: the raw
    code stream (no stuffing, last partial byte zero-filled) and its bit count, the GPU encoder's output form."""
    tabs = [(_derive(DC_LUM), _derive(AC_LUM)), (_derive(DC_CHR), _derive(AC_CHR))]
    w = _BitWriter(stuff)
    last = [0] * len(comps)
    mcuy = comps[0][0].shape[0] // comps[0][2]
    mcux = comps[0][0].shape[1] // comps[0][1]
    for my in range(mcuy):
        for mx in range(mcux):
            for c, (blocks, h, v) in enumerate(comps):
                dc, ac = tabs[0 if c == 0 else 1]
                for yy in range(v):
                    for xx in range(h):
                        b = blocks[my * v + yy, mx * h + xx]
                        diff = int(b[0]) - last[c]
                        last[c] = int(b[0])
                        t, t2 = (-diff, diff - 1) if diff < 0 else (diff, diff)
                        nb = t.bit_length()
                        w.put(*dc[nb])
                        if nb:
                            w.put(t2, nb)
                        r = 0
                        for k in range(1, 64):
                            x = int(b[NATURAL[k]])
                            if x == 0:
                                r += 1
                                continue
                            while r > 15:
                                w.put(*ac[0xF0])
                                r -= 16
                            t, t2 = (-x, x - 1) if x < 0 else (x, x)
                            nb = t.bit_length()
                            w.put(*ac[(r << 4) + nb])
                            w.put(t2, nb)
                            r = 0
                        if r > 0:
                            w.put(*ac[0x00])
    if not stuff:
        n = w.total
        if w.n:
            w.out.append((w.acc << (8 - w.n)) & 0xFF)
        return bytes(w.out), n
    w.flush()
    return bytes(w.out)


def headers(W, H, comps_hv, qt, comment=None) -> bytes:
    """jcmarker.c write_file_header + [Pillow's COM] + write_frame_header + write_scan_header."""
    o = bytearray(b"\xff\xd8")
    o += b"\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00"
    if comment:
        o += b"\xff\xfe" + (len(comment) + 2).to_bytes(2, "big") + comment
    for i, t in enumerate(qt):
        o += b"\xff\xdb\x00\x43" + bytes([i]) + bytes(int(t[NATURAL[k]]) for k in range(64))
    o += b"\xff\xc0" + (8 + 3 * len(comps_hv)).to_bytes(2, "big") + b"\x08"
    o += H.to_bytes(2, "big") + W.to_bytes(2, "big") + bytes([len(comps_hv)])
    for c, (h, v) in enumerate(comps_hv):
        o += bytes([c + 1, (h << 4) | v, 0 if c == 0 else 1])
    for idx, tab in ((0x00, DC_LUM), (0x10, AC_LUM), (0x01, DC_CHR), (0x11, AC_CHR)):
        bits, vals = tab
        o += b"\xff\xc4" + (3 + 16 + len(vals)).to_bytes(2, "big") + bytes([idx]) + bytes(bits) + bytes(vals)
    o += b"\xff\xda\x00\x0c\x03\x01\x00\x02\x11\x03\x11\x00\x3f\x00"
    return bytes(o)


def encode(rgb, quality=-1, subsampling=-1, comment=None) -> bytes:
    """Pillow's Image.fromarray(rgb).save(buf, "JPEG", [quality=...], [subsampling=...]) for an RGB image whose
    info may carry a comment, restated."""
    rgb = np.asarray(rgb, np.uint8)
    H, W, _ = rgb.shape
    comps, qt = coefficient_blocks(rgb, quality, subsampling)
    hdr = headers(W, H, [(h, v) for _, h, v in comps], qt, comment)
    return hdr + entropy_bits(comps) + b"\xff\xd9"
