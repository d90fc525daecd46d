"""sp_attention / sp_attention_bf16 on the model's shapes (AIFI over the 20×20 map, decoder self-attention over
300 queries; 8 heads × 32), timed with HIP events, plus a sha256 of each output so two libraries
(SPOTTER_HIP_LIB) can be compared for bit-identical results and time in alternating processes on one box.

    SPOTTER_HIP_LIB=... python tools/microbench/attn_ab.py [--reps 50] [--tag old]
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
from spotter_amd.ops import V  # noqa: E402

# (batch, n, heads, dh): AIFI at C2 / C3 batch, decoder self-attention at C2, bs1 forms
SHAPES = [(32, 400, 8, 32), (32, 300, 8, 32), (128, 400, 8, 32), (128, 300, 8, 32), (1, 400, 8, 32), (1, 300, 8, 32),
          (8, 256, 4, 64), (8, 200, 6, 48)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    out = {"tag": a.tag, "lib": os.environ.get("SPOTTER_HIP_LIB", "default"), "shapes": []}
    for (b, n, h, dh) in SHAPES:
        d = h * dh
        q, k, v = (torch.randn(b * n, d, generator=g).to(dev) for _ in range(3))
        o = torch.empty(b * n, d, device=dev)
        e = {"shape": [b, n, h, dh]}
        for bf in (False, True):
            run = lambda: ops.attention(V(q, 0, d), V(k, 0, d), V(v, 0, d), V(o, 0, d), b, n, h, dh,  # noqa
                                        dh ** -0.5, bf16=bf)
            for _ in range(5):
                run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            key = "bf16" if bf else "f32"
            e[key] = {"us": round(e0.elapsed_time(e1) / a.reps * 1e3, 2),
                      "sha": hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()[:16]}
        out["shapes"].append(e)
        print(json.dumps(e), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
