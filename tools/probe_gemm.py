"""Times 1×1 split-GEMM shapes (M rows, Cout, K) over a list of tile configurations, optionally with the
residual + ReLU epilogue of a bottleneck expand conv — the short-K study of round 2.

    python tools/probe_gemm.py --shapes 51200,1024,256;204800,256,256 --cfgs 44,45,46,73 [--res] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import view


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", required=True)
    ap.add_argument("--cfgs", default="-,44,45,46,47,63,65,70,71,72,73,74,75")
    ap.add_argument("--res", action="store_true", help="residual + relu epilogue (res1)")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from spotter_amd._lib import lib

    assert lib().sp_device_init(0) == 0
    res = []
    for sh in a.shapes.split(";"):
        m, cout, k = (int(v) for v in sh.split(","))
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(m * k, device=dev, generator=g)
        wt = torch.randn(cout * k, device=dev, generator=g) / k ** 0.5
        planes = ops.split_bf16x3(wt)
        out = torch.empty(m * cout, device=dev)
        r1 = torch.randn(m * cout, device=dev, generator=g) if a.res else None
        shift = torch.zeros(cout, device=dev)
        times = {}
        for cfg in a.cfgs.split(","):
            ops.force_conv_config(None if cfg == "-" else cfg)
            try:
                def run():
                    ops.conv2d(view(x, k), 1, 1, m, k, wt, cout, 1, 1, 0, view(out, cout), shift=shift,
                               act="relu" if a.res else None, res1=view(r1, cout) if a.res else None,
                               wt_planes=planes)
                for _ in range(2):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[cfg] = round(e0.elapsed_time(e1) / a.reps, 4)
            except RuntimeError as e:
                times[cfg] = str(e)[:60]
            finally:
                ops.force_conv_config(None)
        ok = {c: t for c, t in times.items() if isinstance(t, float)}
        best = min(ok, key=ok.get)
        tf = 2 * m * cout * k / (ok[best] * 1e-3) / 1e12
        e = {"shape": [m, cout, k], "res": a.res, "best": best, "best_ms": ok[best], "best_tflops": round(tf, 1),
             "times": times}
        res.append(e)
        print(json.dumps(e), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
