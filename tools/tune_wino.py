"""Tile tuning of the Winograd F(2x2,3x3) path (sp_conv3x3_winograd) against the direct implicit GEMM.

    python tools/tune_wino.py [--out tune_wino.json] [--reps 10] [--planes 3] [--shapes n,h,w,cin,cout;...]

For each 3x3 stride-1 conv shape, times the direct sp_conv2d (its production tile) and the Winograd call
with every LDS-DMA tile configuration of its batched component GEMM (sp_set_conv_config). Output: per
shape the direct time, every configuration's time and the winner (the transform kernels' own share is
read from a rocprofv3 kernel trace of the same run).
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

CFGS = ["11", "12", "13", "14", "15", "16", "17", "18", "19", "20", "33", "34", "35", "36", "37", "38", "41", "42",
        "43", "44", "45", "46", "47", "48", "49", "50", "51", "62", "63", "64", "65"]
# bs32 R101vd 640² (C2): CCFM RepVGG 3x3s at 80² / 40² / 20², backbone stride-1 3x3s of stages 1-4
SHAPES = [(32, 80, 80, 384, 384), (32, 40, 40, 384, 384), (32, 20, 20, 384, 384), (32, 40, 40, 256, 256),
          (32, 20, 20, 512, 512), (32, 80, 80, 128, 128), (32, 160, 160, 64, 64)]


def timeit(fn, reps):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="tune_wino.json")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--planes", type=int, default=3, choices=[1, 3])
    ap.add_argument("--shapes", default=None, help="n,h,w,cin,cout;... (default: the C2 shapes)")
    ap.add_argument("--cfgs", default=None)
    ap.add_argument("--m", type=int, default=2, choices=[2, 4], help="Winograd output tile F(m×m, 3×3)")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split(",")) for s in a.shapes.split(";")] if a.shapes else SHAPES
    cfgs = a.cfgs.split(",") if a.cfgs else CFGS
    dev = torch.device("cuda", 0)
    from spotter_amd._lib import lib

    assert lib().sp_device_init(0) == 0
    res = []
    for (n, h, w, cin, cout) in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(n * h * w * cin, device=dev, generator=g)
        wt_host = (np.random.default_rng(0).standard_normal((cout, 3, 3, cin)) / np.sqrt(9 * cin)).astype(np.float32)
        wt = torch.from_numpy(wt_host.reshape(cout, -1)).to(dev)
        u = ops.winograd_weights_host(wt_host, a.m)
        if a.planes == 3:
            direct_kw = {"wt_planes": ops.split_bf16x3(wt)}
            planes = torch.from_numpy(ops.split_bf16x3_host(u)).to(dev)
        else:
            direct_kw = {"wt16": torch.from_numpy(ops.bf16_bits(wt_host.reshape(cout, -1)).view(np.int16)).to(dev)}
            planes = torch.from_numpy(ops.bf16_bits(u).reshape(1, -1).view(np.int16)).to(dev)
        out = torch.empty(n * h * w * cout, device=dev)
        tiles = n * ((h + a.m - 1) // a.m) * ((w + a.m - 1) // a.m)
        work = torch.empty((a.m + 2) ** 2 * tiles * (cin + cout), device=dev)
        ws = torch.empty(16 << 20, device=dev)
        sh = torch.zeros(cout, device=dev)
        direct = timeit(lambda: ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, 3, 1, 1, view(out, cout), shift=sh,
                                           act="silu", workspace=ws, **direct_kw), a.reps)
        times = {}
        for cfg in cfgs:
            ops.force_conv_config(cfg)
            try:
                times[cfg] = round(timeit(lambda: ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, 3, 1, 1,
                                                             view(out, cout), shift=sh, act="silu",
                                                             wino=(planes, work, a.m)), a.reps), 4)
            except RuntimeError:
                pass
            finally:
                ops.force_conv_config(None)
        best = min(times, key=times.get)
        # per-stage split of the winning configuration: HIP events around each of the three launches
        stages = {}

        def hook(kind, launch, flops, nbytes, shape=None):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launch()
            e1.record()
            key = kind if kind == "conv" else f"{kind}:{shape[-1]}"
            stages.setdefault(key, []).append((e0, e1, nbytes))

        ops.force_conv_config(best)
        ops.set_launch_hook(hook)
        try:
            for _ in range(a.reps):
                ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, 3, 1, 1, view(out, cout), shift=sh, act="silu",
                           wino=(planes, work, a.m))
            torch.cuda.synchronize()
        finally:
            ops.set_launch_hook(None)
            ops.force_conv_config(None)
        split = {}
        for key, recs in stages.items():
            ms = sum(e0.elapsed_time(e1) for e0, e1, _ in recs) / len(recs)
            split[key] = {"ms": round(ms, 4), "GB/s": round(recs[0][2] / (ms * 1e-3) / 1e9, 1)}
        e = {"shape": [n, h, w, cin, cout], "m": a.m, "planes": a.planes, "direct_ms": round(direct, 4), "best_cfg": best,
             "best_ms": times[best], "speedup": round(direct / times[best], 3), "stages": split, "times": times}
        res.append(e)
        print(json.dumps(e), flush=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
