"""A deterministic corpus of malformed JPEGs for the host parser (spotter_amd/csrc/jpeg_host.h).

Every entry is a valid Pillow-written file (or the reference's own test_pic.jpg) with one defect: a cut at
many offsets, byte flips in the headers and in the entropy-coded data, and the structured faults a hostile
or broken encoder produces — huge / zero frame sizes, bad quantisation and Huffman table definitions (DC
symbols above 15, 16-bit precision codes above 1, counts past the segment), bad scan headers, renumbered or
displaced restart markers, bogus progressive successive-approximation sequences, stray and reserved markers,
junk between markers. Used by tests/test_jpeg_corpus.py (ASan/UBSan harness + the Pillow equivalence rule).
"""
from __future__ import annotations

import io
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg")


def _jpeg(img, mode="RGB", **kw) -> bytes:
    from PIL import Image

    b = io.BytesIO()
    Image.fromarray(img).convert(mode).save(b, "JPEG", **kw)
    return b.getvalue()


def segments(data: bytes):
    """(marker, offset of 0xFF, segment length incl. the 2 length bytes or 0) up to EOI; entropy data skipped."""
    out, p = [], 2
    while p + 1 < len(data):
        if data[p] != 0xFF:
            p += 1
            continue
        m = data[p + 1]
        if m in (0x00, 0xFF) or 0xD0 <= m <= 0xD7:
            p += 1 if m == 0xFF else 2
            continue
        if m == 0xD9:
            out.append((m, p, 0))
            break
        L = struct.unpack(">H", data[p + 2:p + 4])[0]
        out.append((m, p, L))
        p += 2 + L
        if m == 0xDA:  # skip the scan's data to its terminating marker
            while p + 1 < len(data) and not (data[p] == 0xFF and data[p + 1] not in (0x00,)
                                             and not 0xD0 <= data[p + 1] <= 0xD7):
                p += 1
    return out


def _put(data: bytes, off: int, val: bytes) -> bytes:
    return data[:off] + val + data[off + len(val):]


def _first(data, marker):
    return next(s for s in segments(data) if s[0] == marker)


def _all(data, marker):
    return [s for s in segments(data) if s[0] == marker]


def bases() -> dict:
    from spotter_amd.synthetic import synthetic_image

    img = synthetic_image(11, 48, 64)
    return {
        "test_pic": open(GOLDEN, "rb").read(),
        "base420": _jpeg(img, quality=75, subsampling=2),
        "prog420": _jpeg(img, quality=80, subsampling=2, progressive=True),
        "rst422": _jpeg(synthetic_image(12, 40, 72), quality=85, subsampling=1, restart_marker_blocks=2),
        "prog_rst": _jpeg(synthetic_image(13, 33, 47), quality=70, progressive=True, restart_marker_rows=1),
        "gray": _jpeg(synthetic_image(14, 31, 29), mode="L", quality=90),
    }


def structured(name: str, d: bytes):
    """(label, bytes) pairs: one defect each, aimed at a specific parser rule."""
    out = []
    sof = next(s for s in segments(d) if s[0] in (0xC0, 0xC1, 0xC2))
    o = sof[1] + 4  # SOF payload: P, Y, X, Nf, then 3 bytes per component
    out.append(("sof_huge", _put(d, o + 1, struct.pack(">HH", 60000, 60000))))
    out.append(("sof_zero_h", _put(d, o + 1, b"\x00\x00")))
    out.append(("sof_zero_w", _put(d, o + 3, b"\x00\x00")))
    out.append(("sof_12bit", _put(d, o, b"\x0c")))
    out.append(("sof_tq5", _put(d, o + 8, b"\x05")))
    out.append(("sof_samp0", _put(d, o + 7, b"\x00")))
    out.append(("sof_samp5", _put(d, o + 7, b"\x55")))
    out.append(("sof_len", _put(d, sof[1] + 2, struct.pack(">H", sof[2] + 3))))
    if d[o + 5] == 3:
        out.append(("sof_dup_id", _put(d, o + 9, d[o + 6:o + 7])))
        out.append(("sof_nf2", _put(d, o + 5, b"\x02")))
    dqt = _first(d, 0xDB)
    out.append(("dqt_pq2", _put(d, dqt[1] + 4, bytes([0x20 | (d[dqt[1] + 4] & 15)]))))
    out.append(("dqt_id7", _put(d, dqt[1] + 4, b"\x07")))
    out.append(("dqt_short", _put(d, dqt[1] + 2, struct.pack(">H", dqt[2] - 10))))
    for i, (m, off, L) in enumerate(_all(d, 0xC4)):
        tc = d[off + 4] >> 4
        if tc == 0:
            out.append((f"dht{i}_dc_sym200", _put(d, off + 4 + 17, b"\xc8")))
        out.append((f"dht{i}_id5", _put(d, off + 4, bytes([(tc << 4) | 5]))))
        out.append((f"dht{i}_counts", _put(d, off + 5, b"\xff" * 16)))
        out.append((f"dht{i}_overfull", _put(d, off + 5, b"\x03\x05")))  # more codes than lengths allow
        out.append((f"dht{i}_empty", _put(d, off + 5, b"\x00" * 16)))
    out.append(("dht_removed", d[:_first(d, 0xC4)[1]] + d[_first(d, 0xC4)[1] + 2 + _first(d, 0xC4)[2]:]))
    sos = _first(d, 0xDA)
    so = sos[1] + 4
    ns = d[so]
    out.append(("sos_ns4", _put(d, so, b"\x04")))
    out.append(("sos_ns0", _put(d, so, b"\x00")))
    out.append(("sos_len", _put(d, sos[1] + 2, struct.pack(">H", sos[2] + 2))))
    out.append(("sos_bad_comp", _put(d, so + 1, b"\xee")))
    out.append(("sos_sel7", _put(d, so + 2, b"\x77")))
    if ns > 1:
        out.append(("sos_dup_comp", _put(d, so + 3, d[so + 1:so + 2])))
    out.append(("sos_ss_gt_se", _put(d, so + 1 + 2 * ns, b"\x3f\x01")))
    out.append(("sos_se70", _put(d, so + 2 + 2 * ns, b"\x46")))
    out.append(("sos_ahal", _put(d, so + 3 + 2 * ns, b"\x31")))
    out.append(("sos_al15", _put(d, so + 3 + 2 * ns, b"\x0f")))
    scans = _all(d, 0xDA)
    if len(scans) > 1:  # progressive: drop the first (DC) scan, repeat a scan, break the refinement chain
        s0, s1 = scans[0], scans[1]
        out.append(("prog_no_dc", d[:s0[1]] + d[s1[1]:]))
        out.append(("prog_repeat", d[:s1[1]] + d[s0[1]:s1[1]] + d[s1[1]:]))
        for k, s in enumerate(scans[1:6]):
            p = s[1] + 4
            n = d[p]
            out.append((f"prog_scan{k}_ah", _put(d, p + 3 + 2 * n, bytes([(d[p + 3 + 2 * n] + 0x10) & 0xFF]))))
            out.append((f"prog_scan{k}_ss0", _put(d, p + 1 + 2 * n, b"\x00")))
    dri = _all(d, 0xDD)
    if dri:
        out.append(("dri_len3", _put(d, dri[0][1] + 2, b"\x00\x03")))
        out.append(("dri_zero", _put(d, dri[0][1] + 4, b"\x00\x00")))
        out.append(("dri_huge", _put(d, dri[0][1] + 4, b"\xff\xff")))
    rst = [i for i in range(len(d) - 1) if d[i] == 0xFF and 0xD0 <= d[i + 1] <= 0xD7]
    for k, i in enumerate(rst[:4]):
        out.append((f"rst{k}_renumber", _put(d, i + 1, bytes([0xD0 + ((d[i + 1] - 0xD0 + 3) & 7)]))))
        out.append((f"rst{k}_junk_before", d[:i] + b"\x12\x34" + d[i:]))
        out.append((f"rst{k}_removed", d[:i] + d[i + 2:]))
        out.append((f"rst{k}_fill", d[:i] + b"\xff\xff" + d[i:]))  # fill bytes before a marker: legal
    app = sof[1]
    out.append(("tem_marker", d[:app] + b"\xff\x01" + d[app:]))
    out.append(("reserved_marker", d[:app] + b"\xff\x02\x00\x04\x00\x00" + d[app:]))
    out.append(("second_soi", d[:app] + b"\xff\xd8" + d[app:]))
    out.append(("junk_between", d[:app] + b"\x00\x11\x22" + d[app:]))
    out.append(("fill_between", d[:app] + b"\xff\xff\xff" + d[app:]))  # legal
    out.append(("rst_outside", d[:app] + b"\xff\xd3" + d[app:]))
    out.append(("dnl", d[:app] + b"\xff\xdc\x00\x04\x00\x10" + d[app:]))
    out.append(("arith_dac", d[:app] + b"\xff\xcc\x00\x04\x00\x00" + d[app:]))
    out.append(("com_segment", d[:app] + b"\xff\xfe\x00\x07hello" + d[app:]))  # legal
    out.append(("app_huge_len", d[:app] + b"\xff\xe5\xff\xff" + d[app:]))
    out.append(("no_eoi", d[:-2]))
    out.append(("after_eoi", d + b"\x00garbage\xff\xd9"))  # legal: libjpeg stops at EOI
    out.append(("double_eoi", d + b"\xff\xd9"))
    return [(f"{name}:{lab}", x) for lab, x in out]


def mutated(name: str, d: bytes, seed: int):
    rng = np.random.default_rng(seed)
    out = []
    cuts = sorted(set(list(range(2, min(len(d), 400), 7)) + list(np.linspace(400, len(d) - 1, 25).astype(int))))
    out += [(f"{name}:cut{c}", d[:c]) for c in cuts if 2 <= c < len(d)]
    hdr_end = _first(d, 0xDA)[1] + 2 + _first(d, 0xDA)[2]
    for k in range(60):  # header flips
        i = int(rng.integers(2, hdr_end))
        out.append((f"{name}:hflip{k}", _put(d, i, bytes([d[i] ^ int(rng.integers(1, 256))]))))
    for k in range(60):  # entropy-data flips and bursts
        i = int(rng.integers(hdr_end, len(d) - 2))
        if k % 3 == 2:
            burst = bytes(rng.integers(0, 256, int(rng.integers(2, 12)), dtype=np.uint8))
            out.append((f"{name}:burst{k}", _put(d, i, burst)))
        else:
            out.append((f"{name}:dflip{k}", _put(d, i, bytes([d[i] ^ (1 << int(rng.integers(0, 8)))]))))
    return out


def corpus():
    out = []
    for i, (name, d) in enumerate(bases().items()):
        out.append((f"{name}:valid", d))
        out += structured(name, d)
        out += mutated(name, d, 1000 + i)
    return out


def pack(entries) -> bytes:
    return b"".join(struct.pack("<I", len(x)) + x for _, x in entries)
