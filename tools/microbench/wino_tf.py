"""Winograd F(4×4, 3×3) transform kernels on the C2 shapes (bs32 R101vd 640²), timed per stage with HIP events
through the launch hook: algorithmic bytes / duration for the input and output transforms, next to a torch
float4 copy of the same byte count (the box's achievable streaming rate).

    python tools/microbench/wino_tf.py [--reps 20] [--out wino_tf.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from spotter_amd import ops  # noqa: E402
from spotter_amd.ops import V  # noqa: E402

# (n, h, w, cin, cout, per-step count, res1) of C2's F(4×4) convs: stage-3 3×3s, CCFM RepVGG 3×3s
SHAPES = [(32, 40, 40, 256, 256, 22, False), (32, 80, 80, 384, 384, 3, False), (32, 40, 40, 384, 384, 6, False),
          (32, 80, 80, 128, 128, 3, False), (32, 20, 20, 512, 512, 2, False), (32, 20, 20, 384, 384, 3, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    recs = []

    def hook(kind, launch, flops, nbytes, shape):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch()
        e1.record()
        recs.append((kind, shape, nbytes, e0, e1))

    res = []
    tot = {"in": 0.0, "out": 0.0}
    for (n, h, w, cin, cout, cnt, r1) in SHAPES:
        tiles = n * ((h + 3) // 4) * ((w + 3) // 4)
        x = torch.randn(n * h * w * cin, device=dev)
        out = torch.empty(n * h * w * cout, device=dev)
        wt = torch.zeros(cout * 9 * cin, device=dev)
        planes = torch.zeros(3, 36 * cout * cin, dtype=torch.int16, device=dev)
        work = torch.empty(ops.wino_work_elems(4, tiles, cin, cout), device=dev)
        sc, sh = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
        run = lambda: ops.conv2d(V(x, 0, cin), n, h, w, cin, wt, cout, 3, 1, 1, V(out, 0, cout), scale=sc,  # noqa
                                 shift=sh, act="relu", wino=(planes, work, 4))
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        recs.clear()
        ops.set_launch_hook(hook)
        try:
            for _ in range(a.reps):
                run()
        finally:
            ops.set_launch_hook(None)
        torch.cuda.synchronize()
        st = {"in": [], "out": []}
        nb = {}
        for kind, shape, nbytes, e0, e1 in recs:
            if kind == "wino_tf":
                st[shape[2]].append(e0.elapsed_time(e1))
                nb[shape[2]] = nbytes
        # the achievable streaming rate for the same bytes: a float4 copy of half of them
        src = torch.empty(nb["in"] // 8, device=dev)
        dst = torch.empty_like(src)
        for _ in range(3):
            dst.copy_(src)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            dst.copy_(src)
        e1.record()
        torch.cuda.synchronize()
        copy_ms = e0.elapsed_time(e1) / a.reps
        e = {"shape": [n, h, w, cin, cout], "per_step": cnt}
        for s in ("in", "out"):
            ms = sorted(st[s])[len(st[s]) // 2]
            e[s] = {"ms": round(ms, 4), "MB": round(nb[s] / 1e6, 1), "TBps": round(nb[s] / ms / 1e9, 2)}
            tot[s] += ms * cnt
        e["copy_same_bytes_TBps"] = round(nb["in"] / copy_ms / 1e9, 2)
        res.append(e)
        print(json.dumps(e), flush=True)
        del x, out, work, planes, src, dst
    summary = {"shapes": res, "ms_per_step": {k: round(v, 3) for k, v in tot.items()}}
    print(json.dumps(summary["ms_per_step"]))
    if a.out:
        json.dump(summary, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
