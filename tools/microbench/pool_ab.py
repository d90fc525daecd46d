"""sp_maxpool3x3s2 and sp_upsample2x_nearest (fp32 and bf16 rows) on the stem shapes of C2 (bs32, 320² × 64, fp32) and C3 (bs256, bf16),
timed with HIP events, plus a sha256 of each output, so two libraries (SPOTTER_HIP_LIB) can be compared for
bit-identical results and time in alternating processes on one box.

    SPOTTER_HIP_LIB=... python tools/microbench/pool_ab.py [--reps 30] [--tag old]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from spotter_amd import ops  # noqa: E402

# (n, h, w, c, bf16): C2 stem output, C3 stem output (bf16 rows), bs1
SHAPES = [(32, 320, 320, 64, False), (256, 320, 320, 64, True), (1, 320, 320, 64, False), (32, 320, 320, 64, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(3)
    res = []
    for (n, h, w, c, bf) in SHAPES:
        x = torch.randn(n * h * w * c, device=dev, generator=g)
        if bf:
            x = (x.view(torch.int32) >> 16).to(torch.int16)  # bf16 bit patterns (truncated)
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        y = torch.empty(n * ho * wo * c, dtype=x.dtype, device=dev)
        for _ in range(3):
            ops.maxpool3x3s2(x, y, n, h, w, c)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ops.maxpool3x3s2(x, y, n, h, w, c)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        nbytes = x.element_size() * n * c * (h * w + ho * wo)
        e = {"shape": [n, h, w, c, "bf16" if bf else "f32"], "us": round(ms * 1e3, 2),
             "TBps": round(nbytes / ms / 1e9, 2), "sha": hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]}
        res.append(e)
        print(json.dumps(e), flush=True)
        del x, y
    # nearest ×2 upsample into the channel slice of a concat buffer (the CCFM's top-down path): C2 fp32, C3 bf16
    for (n, h, w, c, bf) in [(32, 20, 20, 256, False), (32, 40, 40, 256, False), (256, 40, 40, 256, True),
                             (256, 20, 20, 256, True)]:
        dt = torch.int16 if bf else torch.float32
        x = torch.randn(n * h * w * c, device=dev, generator=g).to(dt)
        y = torch.zeros(n * 4 * h * w * 2 * c, dtype=dt, device=dev)
        run = lambda: ops.upsample2x(ops.V(x, 0, c), ops.V(y, 0, 2 * c), n, h, w, c)  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        nbytes = x.element_size() * n * h * w * c * 5
        e = {"shape": ["up", n, h, w, c, "bf16" if bf else "f32"], "us": round(ms * 1e3, 2),
             "TBps": round(nbytes / ms / 1e9, 2), "sha": hashlib.sha256(y.cpu().numpy().tobytes()).hexdigest()[:16]}
        res.append(e)
        print(json.dumps(e), flush=True)
        del x, y
    print(json.dumps({"tag": a.tag, "shapes": res}))


if __name__ == "__main__":
    main()
