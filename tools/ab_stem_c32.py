"""A/B in one process: the bf16 variant's Cin-32 stem 3×3s as the direct LDS-halo kernel (sp_conv3x3_c32_bf16)
vs the implicit-GEMM bf16 path on bf16 rows, at the C3 (bs256) and C2 (bs32) shapes; with --f32 the fp32-mode
kernel (sp_conv3x3_c32) vs the fp32-MFMA implicit GEMM at the C2 (bs32) and C5-sized (bs8) shapes. Interleaved
rounds, median ms per launch. python tools/ab_stem_c32.py [--f32] [--out f.jsonl]"""
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
    ap.add_argument("--f32", action="store_true", help="the fp32-mode kernel (sp_conv3x3_c32) vs the fp32-MFMA GEMM")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lines = []
    for n in ((32, 8) if a.f32 else (256, 32)):
        for cout in (32, 64):
            h = w = 320
            m = n * h * w
            sc, sh = torch.rand(cout, device=dev) + 0.5, torch.randn(cout, device=dev)
            if a.f32:
                xf, wf = torch.randn(m * 32, device=dev), torch.randn(cout, 288, device=dev)
                yf = torch.empty(m * cout, device=dev)
                runs = {
                    "direct": lambda: ops.conv3x3_c32(V(xf, 0, 32), wf, sc, sh, V(yf, 0, cout), n, h, w, cout,
                                                      act="relu"),
                    "gemm": lambda: ops.conv2d(V(xf, 0, 32), n, h, w, 32, wf, cout, 3, 1, 1, V(yf, 0, cout),
                                               scale=sc, shift=sh, act="relu"),
                }
            else:
                x = torch.randint(-16000, 16000, (m * 32,), dtype=torch.int16, device=dev)
                x &= 0x3fff  # finite bf16 patterns
                w16 = torch.randint(0, 0x3e00, (cout * 288,), dtype=torch.int16, device=dev)
                wf = torch.randn(cout * 288, device=dev)
                y = torch.empty(m * cout, dtype=torch.int16, device=dev)
                runs = {
                    "direct": lambda: ops.conv3x3_c32_bf16(V(x, 0, 32), w16, sc, sh, V(y, 0, cout), n, h, w, cout,
                                                           act="relu"),
                    "gemm": lambda: ops.conv2d(V(x, 0, 32), n, h, w, 32, wf, cout, 3, 1, 1, V(y, 0, cout),
                                               scale=sc, shift=sh, act="relu", wt16=w16),
                }
            t = {k: [] for k in runs}
            for _ in range(5):
                for k, r in runs.items():
                    r()
                    torch.cuda.synchronize()
                    t[k].append(timed(r, 5))
            d = {"shape": [n, h, w, 32, cout], "ms": {k: round(statistics.median(v), 4) for k, v in t.items()}}
            d["speedup"] = round(d["ms"]["gemm"] / d["ms"]["direct"], 3)
            d["tflops"] = {k: round(2 * m * cout * 288 / (v * 1e-3) / 1e12, 1) for k, v in d["ms"].items()}
            print(json.dumps(d), flush=True)
            lines.append(d)
    if a.out:
        with open(a.out, "w") as f:
            f.write("".join(json.dumps(d) + "\n" for d in lines))


if __name__ == "__main__":
    main()
