"""Same-process A/B of the F(4x4) Winograd transform variants (sp_set_tuning knobs) on the C2 shapes.

    python tools/ab_wino.py [--reps 20] [--out ab_wino.json]

For each 3x3 stride-1 shape of the bs32 R101vd forward that takes F(4x4), times the whole Winograd conv
(input transform + batched split GEMM + output transform) under every (layout, non-temporal accesses) variant,
interleaved over rounds so clock drift hits all variants alike, and checks that every variant's output is
bit-identical to the default's (the variants reorder memory traffic, not arithmetic). Per-kernel times come
from a rocprofv3 kernel trace of the same run.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from spotter_amd import ops
from spotter_amd.ops import view

SHAPES = [(32, 80, 80, 128, 128), (32, 40, 40, 256, 256), (32, 80, 80, 384, 384), (32, 40, 40, 384, 384),
          (32, 20, 20, 512, 512), (32, 20, 20, 384, 384)]
VARIANTS = [(0, 0), (0, 1), (0, 2), (0, 3), (1, 0), (1, 3)]  # (layout, input-transform non-temporal bits)


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def set_variant(v):
    ops.set_tuning(ops.TUNE_WINO43_LAYOUT, None if v is None else v[0])
    ops.set_tuning(ops.TUNE_WINO43_IN_NT, None if v is None else v[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="ab_wino.json")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from spotter_amd._lib import lib

    assert lib().sp_device_init(0) == 0
    res = []
    for (n, h, w, cin, cout) in SHAPES:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n * h * w * cin, device=dev, generator=g)
        wt_host = (np.random.default_rng(0).standard_normal((cout, 3, 3, cin)) / np.sqrt(9 * cin)).astype(np.float32)
        wt = torch.from_numpy(wt_host.reshape(cout, -1)).to(dev)
        planes = torch.from_numpy(ops.split_bf16x3_host(ops.winograd_weights_host(wt_host, 4))).to(dev)
        tiles = n * ((h + 3) // 4) * ((w + 3) // 4)
        work = torch.empty(36 * tiles * (cin + cout) + 64, device=dev)
        sh = torch.zeros(cout, device=dev)
        out = torch.empty(n * h * w * cout, device=dev)

        def run():
            ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, 3, 1, 1, view(out, cout), shift=sh, act="silu",
                       wino=(planes, work, 4))

        set_variant(None)
        run()
        torch.cuda.synchronize()
        ref = out.clone()
        times = {str(v): [] for v in VARIANTS}
        same = {}
        for _ in range(a.rounds):
            for v in VARIANTS:
                set_variant(v)
                out.fill_(float("nan"))
                run()
                torch.cuda.synchronize()
                same[str(v)] = bool(torch.equal(out, ref))
                times[str(v)].append(timeit(run, a.reps))
        set_variant(None)
        med = {k: round(float(np.median(t)), 4) for k, t in times.items()}
        e = {"shape": [n, h, w, cin, cout], "ms": med, "bit_identical": same,
             "map_MB": round(n * h * w * (cin + cout) * 4 / 1e6, 1)}
        res.append(e)
        print(json.dumps(e), flush=True)
    json.dump(res, open(a.out, "w"), indent=1)
    assert all(all(e["bit_identical"].values()) for e in res), "a variant changed the output"


if __name__ == "__main__":
    main()
