"""A/B in one process: the fp32 modes' stage-0 3×3 (Cin 64 → 64, 160² at bs32 / bs8) as the direct LDS-halo
kernel (sp_conv3x3_c64) vs the split (x3) and fp32-MFMA implicit GEMMs; then the bf16 variant's form
(sp_conv3x3_c64_bf16) vs the bf16 implicit GEMM at 160² bs256 / bs32. Interleaved rounds, median ms per
launch. python tools/ab_c64.py [--out f.jsonl]"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import V


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
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lines = []
    for n in (32, 8):
        h = w = 160
        m = n * h * w
        x = torch.randn(m * 64, device=dev)
        wf = torch.randn(64, 576, device=dev) / 24
        planes = torch.from_numpy(ops.split_bf16x3_host(wf.cpu().numpy())).to(dev)
        sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
        y = torch.empty(m * 64, device=dev)
        runs = {
            "direct": lambda: ops.conv3x3_c64(V(x, 0, 64), wf, sc, sh, V(y, 0, 64), n, h, w, act="relu"),
            "f32_gemm": lambda: ops.conv2d(V(x, 0, 64), n, h, w, 64, wf, 64, 3, 1, 1, V(y, 0, 64), scale=sc,
                                           shift=sh, act="relu"),
        }
        runs["x3_gemm"] = lambda: ops.conv2d(V(x, 0, 64), n, h, w, 64, wf, 64, 3, 1, 1, V(y, 0, 64), scale=sc,
                                                 shift=sh, act="relu", wt_planes=planes)
        t = {k: [] for k in runs}
        for _ in range(5):
            for k, r in runs.items():
                r()
                torch.cuda.synchronize()
                t[k].append(timed(r, 5))
        d = {"shape": [n, h, w, 64, 64], "ms": {k: round(statistics.median(v), 4) for k, v in t.items()}}
        d["tflops"] = {k: round(2 * m * 64 * 576 / (v * 1e-3) / 1e12, 1) for k, v in d["ms"].items()}
        print(json.dumps(d), flush=True)
        lines.append(d)
    for n in (256, 32):  # the bf16 variant: C3 (R18vd bs256) and C2-bf16 shapes, bf16 rows
        h = w = 160
        m = n * h * w
        x = torch.randint(0, 0x3f00, (m * 64,), dtype=torch.int16, device=dev)
        w16 = torch.randint(0, 0x3e00, (64 * 576,), dtype=torch.int16, device=dev)
        wf = torch.randn(64, 576, device=dev)
        sc, sh = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
        y = torch.empty(m * 64, dtype=torch.int16, device=dev)
        runs = {
            "direct_bf16": lambda: ops.conv3x3_c64_bf16(V(x, 0, 64), w16, sc, sh, V(y, 0, 64), n, h, w, act="relu"),
            "bf16_gemm": lambda: ops.conv2d(V(x, 0, 64), n, h, w, 64, wf, 64, 3, 1, 1, V(y, 0, 64), scale=sc,
                                            shift=sh, act="relu", wt16=w16),
        }
        t = {k: [] for k in runs}
        for _ in range(5):
            for k, r in runs.items():
                r()
                torch.cuda.synchronize()
                t[k].append(timed(r, 5))
        d = {"shape": [n, h, w, 64, 64], "ms": {k: round(statistics.median(v), 4) for k, v in t.items()}}
        d["tflops"] = {k: round(2 * m * 64 * 576 / (v * 1e-3) / 1e12, 1) for k, v in d["ms"].items()}
        print(json.dumps(d), flush=True)
        lines.append(d)
    if a.out:
        with open(a.out, "w") as f:
            f.write("".join(json.dumps(d) + "\n" for d in lines))


if __name__ == "__main__":
    main()
