"""A/B of two LDS-DMA GEMM tile configurations (conv_glds.hip) in ONE process with interleaved rounds
(guide §5.4 rule 24): kernel variants kept side by side during development, or two tiles.

    python tools/ab_glds.py [--pairs 45:52,46:146] [--planes 3|1] [--rounds 5] [--reps 10] [--out ab.jsonl]

1. Correctness (unless --no-check): both configurations of a pair must give BIT-IDENTICAL outputs — true
   whenever they share the wave tile and MFMA shape (same products, same k16 summation order; the stage
   depth only changes when operands arrive) — on 1×1 convs with ragged M / Cout edges and residual
   epilogues, and through the batched Winograd component GEMMs.
2. Timing: per shape the two configurations alternate for --rounds rounds of --reps launches; the median
   ms of each is reported with the TFLOP/s (fp32-equivalent, 2·M·N·K).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import view

# (n, h, w, cin, cout, residual, act) 1×1 convs; (n, h, w, cin, cout, "wino") F(4x4) 3x3 convs
SHAPES = [
    (32, 40, 40, 256, 1024, True, "relu"),    # stage-3 expand (22 / step)
    (32, 40, 40, 1024, 256, False, "relu"),   # stage-3 reduce (22 / step)
    (32, 80, 80, 768, 768, False, None),      # CCFM 1x1 768 @80²
    (1, 1, 268800, 256, 1536, False, None),   # decoder value_all
    (32, 80, 80, 512, 128, False, "relu"),    # stage-1 reduce
    (32, 80, 80, 384, 384, "wino"),
    (32, 40, 40, 256, 256, "wino"),
    (32, 40, 40, 384, 384, "wino"),
    (32, 20, 20, 512, 512, "wino"),
    (32, 80, 80, 128, 512, True, "relu"),     # stage-1 expand (3 / step)
    (32, 160, 160, 64, 256, True, "relu"),    # stage-0 expand (2 / step)
    (32, 20, 20, 512, 2048, True, "relu"),    # stage-4 expand (2 / step)
]
EDGES = [(1, 1, 1000, 256, 192, True, "relu"), (3, 7, 9, 128, 320, False, None), (1, 1, 77, 512, 128, True, None)]


PLANES = 3  # 3 = the fp32-accurate split (x3), 1 = the bf16 operand mode (--planes 1)
BF16_ROWS = False  # --bf16-rows: activations / outputs / residuals as bf16 rows (with --planes 1)


def force(c):
    """Select configuration c ("46", "-": none)."""
    ops.force_conv_config(None if c == "-" else c)


def make(dev, shape, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    n, h, w, cin, cout = shape[:5]
    wino = shape[5] == "wino"
    k = 3 if wino else 1
    x = torch.randn(n * h * w * cin, device=dev, generator=g)
    if BF16_ROWS:  # the bf16 variant's maps: bf16 rows in, bf16 rows out, bf16 residual rows
        x = ((x.view(torch.int32) + 0x8000) >> 16).to(torch.int16)
    wt = torch.randn(cout * k * k * cin, device=dev, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    sc = torch.rand(cout, device=dev, generator=g) + 0.5
    sh = torch.randn(cout, device=dev, generator=g)
    out = torch.empty(n * h * w * cout, device=dev, dtype=torch.int16 if BF16_ROWS else torch.float32)
    res = (torch.randn(n * h * w * cout, device=dev, generator=g) if shape[5] is True else None)
    if BF16_ROWS and res is not None:
        res = ((res.view(torch.int32) + 0x8000) >> 16).to(torch.int16)
    kw = {}
    if wino:
        u = ops.winograd_weights_host(wt.view(cout, 3, 3, cin).cpu().numpy(), 4)
        planes = (torch.from_numpy(ops.split_bf16x3_host(u)).to(dev) if PLANES == 3 else
                  torch.from_numpy(ops.bf16_bits(u).reshape(1, -1).view("int16")).to(dev))
        t = n * ((h + 3) // 4) * ((w + 3) // 4)
        work = torch.empty(ops.wino_work_elems(4, t, cin, cout), device=dev)
        kw["wino"] = (planes, work, 4)
    elif PLANES == 3:
        kw["wt_planes"] = ops.split_bf16x3(wt)
    else:
        kw["wt16"] = torch.from_numpy(ops.bf16_bits(wt.cpu().numpy()).view("int16")).to(dev)
    act = None if wino else shape[6]

    def run():
        ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, 1, k // 2, view(out, cout), scale=sc, shift=sh,
                   act=act, res1=view(res, cout) if res is not None else None, **kw)

    flops = 2.0 * n * h * w * cout * cin * (9 if wino else 1)  # direct-equivalent for Winograd
    if wino:
        t = n * ((h + 3) // 4) * ((w + 3) // 4)
        flops = 2.0 * 36 * t * cin * cout  # the component GEMMs' own work
    return run, out, flops


def timed(run, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", default="46:146,44:144,33:133,45:145,47:147,63:163")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--planes", type=int, default=3, choices=[1, 3])
    ap.add_argument("--no-check", action="store_true", help="skip the bit-identity check (pairs of different tiles)")
    ap.add_argument("--bf16-rows", action="store_true", help="bf16 activation rows (the bf16 variant's maps)")
    a = ap.parse_args()
    global PLANES, BF16_ROWS
    PLANES = a.planes
    BF16_ROWS = a.bf16_rows
    if BF16_ROWS and PLANES != 1:
        raise SystemExit("--bf16-rows needs --planes 1")
    dev = torch.device("cuda", 0)
    pairs = [tuple(p.split(":")) for p in a.pairs.split(",")]
    lines = []

    def emit(d):
        print(json.dumps(d), flush=True)
        lines.append(d)

    # 1. bit-identical outputs
    for shape in ([] if a.no_check else EDGES + SHAPES[:1] + SHAPES[6:7]):
        run, out, _ = make(dev, shape)
        for c0, c1 in pairs:
            res = []
            for c in (c0, c1):
                force(c)
                out.fill_(-1 if BF16_ROWS else float("nan"))
                try:
                    run()
                except RuntimeError as e:
                    res.append(str(e))
                    continue
                torch.cuda.synchronize()
                res.append(out.clone())
            force("-")
            if any(isinstance(r, str) for r in res):
                emit({"check": list(shape), "pair": [c0, c1], "skipped": [r for r in res if isinstance(r, str)]})
                continue
            same = torch.equal(res[0], res[1]) and not (res[1].is_floating_point() and torch.isnan(res[1]).any().item())
            emit({"check": list(shape), "pair": [c0, c1], "planes": PLANES, "bit_identical": bool(same)})
            if not same:
                raise SystemExit(f"variant {c1} differs from {c0} on {shape}")
    # 2. interleaved timing
    which = [int(i) for i in a.shapes.split(",")] if a.shapes else range(len(SHAPES))
    for si in which:
        shape = SHAPES[si]
        run, out, flops = make(dev, shape)
        for c0, c1 in pairs:
            t = {c0: [], c1: []}
            ok = True
            for _ in range(a.rounds):
                for c in (c0, c1):
                    force(c)
                    try:
                        run()
                        torch.cuda.synchronize()
                        t[c].append(timed(run, a.reps))
                    except RuntimeError:
                        ok = False
            force("-")
            if not ok or not t[c0] or not t[c1]:
                continue
            m0, m1 = statistics.median(t[c0]), statistics.median(t[c1])
            emit({"shape": list(shape), "pair": [c0, c1], "planes": PLANES, "ms": [round(m0, 4), round(m1, 4)],
                  "tflops": [round(flops / m0 / 1e9, 1), round(flops / m1 / 1e9, 1)], "speedup": round(m0 / m1, 3)})
    if a.out:
        with open(a.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
