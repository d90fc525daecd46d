"""Stem conv 1 (sp_stem_conv3x3s2_nchw[_bf16]) at the C2 / C3 / bs1 batch shapes: time per launch and a digest of
the outputs, through whichever library SPOTTER_HIP_LIB names (run once per library; equal digests = bit-identical).

    SPOTTER_HIP_LIB=<lib> python tools/microbench/stem_ab.py
"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from spotter_amd import ops  # noqa: E402
from spotter_amd._lib import lib  # noqa: E402
from spotter_amd.ops import V  # noqa: E402


def main():
    assert lib().sp_device_init(0) == 0
    dev = torch.device("cuda", 0)
    res = {}
    for (n, h, w, cout, bf) in [(256, 640, 640, 32, True), (32, 640, 640, 32, False), (1, 640, 640, 32, False),
                                (3, 33, 17, 64, False), (2, 31, 45, 32, True)]:
        g = torch.Generator(device=dev).manual_seed(n + h + cout)
        x = torch.rand((n, 3, h, w), device=dev, generator=g)
        wt = torch.randn(cout * 27, device=dev, generator=g) / 27 ** 0.5
        sc = torch.rand(cout, device=dev, generator=g) + 0.5
        sh = torch.randn(cout, device=dev, generator=g) * 0.1
        ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        out = torch.empty(n * ho * wo * cout, device=dev, dtype=torch.int16 if bf else torch.float32)
        run = lambda: ops.stem_conv_nchw(x, wt, sc, sh, V(out, 0, cout), cout, act="relu")  # noqa: E731
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        key = f"{n}x{h}x{w}->{cout}{' bf16' if bf else ''}"
        res[key] = {"ms": round(e0.elapsed_time(e1) / 20, 4),
                    "digest": hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
