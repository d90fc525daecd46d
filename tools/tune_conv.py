"""Per-shape GEMM tile tuning over the conv/linear shapes one bench step actually launches.

    python tools/tune_conv.py <bench --detail JSON> [--out tune.json] [--reps 10] [--min-ms 0.05]

Reads the per-shape timings `bench.py --detail` writes (shape key (M, Cout, K, k, stride, mode)),
rebuilds each GEMM (1×1 / linear: one row of M pixels; 3×3: 32 square images), times every tile
configuration its operand mode has (sp_set_conv_config) and records the fastest. The winners become
spotter_amd/csrc/tile_table.h (tools/gen_tile_table.py), the exact-shape part of the tile choice.
"""
from __future__ import annotations

import argparse
import ast
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import view

X3_CFGS = ["-", "11", "12", "13", "14", "16", "17", "33", "41", "42", "43", "44", "45", "46", "47", "49", "50", "51",
           "62", "63", "64", "65"]  # (70-75: diagnostic builds only since round 5)
F32_CFGS = ["-", "110", "111", "120", "121", "210", "211", "220", "221", "4110", "4111", "4210", "4120", "1110", "1111",
            "1120", "1121"]


def geometry(m, cout, K, k, stride):
    """(n, h, w, cin) of a GEMM with M = m rows: 1×1 convs and linears as one row of m pixels."""
    cin = K // (k * k)
    if k == 1 and stride == 1:
        return 1, 1, m, cin
    n = 32
    ho = int(round(math.sqrt(m / n)))
    if n * ho * ho != m:
        n, ho = 1, int(round(math.sqrt(m)))
    h = ho * stride
    return n, h, h, cin


_WS = {}


def workspace(dev):
    """The engine's conv workspace (Engine.SPLITK_ELEMS): split-K where the engine would split."""
    if dev not in _WS:
        _WS[dev] = torch.empty(16 << 20, device=dev)
    return _WS[dev]


def time_one(dev, m, cout, K, k, stride, mode, cfg, reps, rows=False, epi="none"):
    """rows: the bf16 variant's form of the layer (A staged from bf16 rows, bf16 rows out); epi: the launch's
    epilogue as the engine runs it ("res": BN + residual + relu, "bn": BN + relu, "none"), which decides
    between the plain and the slab / direct-store epilogue forms."""
    n, h, w, cin = geometry(m, cout, K, k, stride)
    pad = k // 2
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n * h * w * cin, device=dev, generator=g)
    wt = torch.randn(cout * K, device=dev, generator=g) * (1.0 / K ** 0.5)
    out = torch.empty(m * cout, device=dev, dtype=torch.int16 if rows else torch.float32)
    if rows:
        x = x.to(torch.bfloat16).view(torch.int16).contiguous()
    if mode == "x3":
        kw = {"wt_planes": ops.split_bf16x3(wt)}
    elif mode == "bf16":
        kw = {"wt16": torch.from_numpy(ops.bf16_bits(wt.cpu().numpy()).view("int16")).to(dev)}
    else:
        kw = {}
    ops.force_conv_config(None if cfg == "-" else cfg)

    if epi in ("res", "bn"):
        kw["scale"] = torch.rand(cout, device=dev, generator=g) + 0.5
        kw["shift"] = torch.randn(cout, device=dev, generator=g)
        kw["act"] = "relu"
    if epi == "res":
        r = torch.randn(m * cout, device=dev, generator=g)
        kw["res1"] = view(r.to(torch.bfloat16).view(torch.int16).contiguous() if rows else r, cout)

    def run():
        ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, stride, pad, view(out, cout), workspace=workspace(dev),
                   **kw)

    try:
        for _ in range(2):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps
    except RuntimeError:
        return None
    finally:
        ops.force_conv_config(None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("detail")
    ap.add_argument("--out", default="tune.json")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--min-ms", type=float, default=0.05, help="skip shapes cheaper than this per step")
    ap.add_argument("--steps", type=int, default=10, help="steps the detail file was recorded over")
    ap.add_argument("--modes", default="x3,f32,bf16", help="operand modes to tune")
    ap.add_argument("--cross", action="store_true",
                    help="also time f32-mode shapes as x3 and x3-mode shapes as f32 (both fp32-accurate): "
                         "the per-layer mode choice of Engine._pick")
    ap.add_argument("--cfgs", default=None, help="comma-separated split / bf16 configurations to time "
                                                  "(default: all of X3_CFGS)")
    a = ap.parse_args()
    x3_cfgs = a.cfgs.split(",") if a.cfgs else X3_CFGS
    dev = torch.device("cuda", 0)
    rows = json.load(open(a.detail))
    res = []
    for r in rows:
        key = ast.literal_eval(r["shape"])
        m, cout, K, k, stride, mode = key[:6]
        rows = "rows" in key[6:]
        epi = next((t[4:] for t in key[6:] if isinstance(t, str) and t.startswith("epi:")), "none")
        per_step = r["ms"] / a.steps
        if mode not in a.modes.split(",") or per_step < a.min_ms:
            continue
        launches = r["launches"] / a.steps
        times = {}
        for cfg in (F32_CFGS if mode == "f32" else x3_cfgs):
            t = time_one(dev, m, cout, K, k, stride, mode, cfg, a.reps, rows, epi)
            if t is not None:
                times[cfg] = round(t, 4)
        if a.cross and mode in ("f32", "x3"):
            other = "x3" if mode == "f32" else "f32"
            for cfg in (F32_CFGS if other == "f32" else x3_cfgs):
                t = time_one(dev, m, cout, K, k, stride, other, cfg, a.reps)
                if t is not None:
                    times[other + ":" + cfg] = round(t, 4)
        best = min(times, key=times.get)
        e = {"m": m, "cout": cout, "K": K, "k": k, "stride": stride, "mode": mode, "rows": rows, "epi": epi,
             "wino": len(key) > 6 and key[6] == "wino",
             "launches_per_step": launches,
             "default_ms": times.get("-"), "best_cfg": best, "best_ms": times[best], "times": times,
             "best_same_mode": min((c for c in times if ":" not in c), key=times.get),
             "saving_ms_per_step": round((times.get("-", times[best]) - times[best]) * launches, 4)}
        res.append(e)
        print(json.dumps(e), flush=True)
    tot = sum(e["saving_ms_per_step"] for e in res)
    json.dump({"shapes": res, "saving_ms_per_step": round(tot, 3)}, open(a.out, "w"), indent=1)
    print(json.dumps({"saving_ms_per_step": round(tot, 3)}))


if __name__ == "__main__":
    main()
