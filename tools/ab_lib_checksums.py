"""Checksums of split-mode (x3) conv outputs through whichever library SPOTTER_HIP_LIB names: run once per
library and compare the printed digests (bit-identity of two builds of the same kernels).

    SPOTTER_HIP_LIB=<lib> python tools/ab_lib_checksums.py
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spotter_amd import ops  # noqa: E402
from spotter_amd._lib import lib  # noqa: E402
from spotter_amd.ops import view  # noqa: E402


def main():
    assert lib().sp_device_init(0) == 0
    dev = torch.device("cuda", 0)
    h = hashlib.sha256()
    for (n, hh, w, cin, cout, k, st, cfg) in [(1, 1, 51200, 256, 1024, 1, 1, None), (1, 1, 51200, 1024, 256, 1, 1, None),
                                             (4, 40, 40, 256, 256, 3, 1, None), (2, 20, 20, 384, 384, 3, 2, None),
                                             (1, 1, 9600, 256, 512, 1, 1, None), (1, 1, 3000, 768, 768, 1, 1, "63"),
                                             (1, 1, 3000, 768, 768, 1, 1, "33"), (1, 1, 3000, 768, 768, 1, 1, "41"),
                                             (1, 1, 3000, 512, 256, 1, 1, "246"), (1, 1, 3000, 512, 256, 1, 1, "14")]:
        g = torch.Generator(device=dev).manual_seed(cin * cout + k)
        x = torch.randn(n * hh * w * cin, device=dev, generator=g)
        wt = torch.randn(cout * k * k * cin, device=dev, generator=g) / (k * k * cin) ** 0.5
        sc = torch.rand(cout, device=dev, generator=g) + 0.5
        sh = torch.randn(cout, device=dev, generator=g)
        pad = k // 2
        ho = (hh + 2 * pad - k) // st + 1
        wo = (w + 2 * pad - k) // st + 1
        out = torch.empty(n * ho * wo * cout, device=dev)
        ops.force_conv_config(cfg)
        try:
            ops.conv2d(view(x, cin), n, hh, w, cin, wt, cout, k, st, pad, view(out, cout), scale=sc, shift=sh,
                       act="relu", wt_planes=ops.split_bf16x3(wt), workspace=torch.empty(16 << 20, device=dev))
        finally:
            ops.force_conv_config(None)
        torch.cuda.synchronize()
        d = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16]
        h.update(d.encode())
        print(n, hh, w, cin, cout, k, st, cfg, d)
    print("ALL", h.hexdigest()[:16])


if __name__ == "__main__":
    main()
