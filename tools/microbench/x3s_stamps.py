"""Where the time of one conv_x3s_kernel interval goes (diagnostic build, -DSP_X3S_STAMP):
s_memtime stamps per wave of workgroup 0 around the DMA wait, the barrier, the DMA issue and the two
work regions (split / MFMA). Run with SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so.

    python tools/microbench/x3s_stamps.py [--cfg 70] [--shape 204800,768,768,1]
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from spotter_amd import _lib, ops
from spotter_amd.ops import view


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", default="70")
    ap.add_argument("--shape", default="204800,768,768,1")
    a = ap.parse_args()
    m, cout, cin, k = (int(v) for v in a.shape.split(","))
    dev = torch.device("cuda", 0)
    if k == 1:
        n, h, w = 1, 1, m
    else:
        n = 32
        h = w = int(round((m / n) ** 0.5))
    x = torch.randn(n * h * w * cin, device=dev)
    wt = torch.randn(cout * k * k * cin, device=dev) / (cin * k * k) ** 0.5
    out = torch.empty(m * cout, device=dev)
    planes = ops.split_bf16x3(wt)
    ops.force_conv_config(a.cfg)
    for _ in range(5):
        ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, 1, k // 2, view(out, cout), wt_planes=planes)
    torch.cuda.synchronize()
    buf = np.zeros(8 * 64 * 8, np.uint64)
    L = _lib.lib()
    L.sp_debug_x3s_stamps.restype = ctypes.c_int
    rc = L.sp_debug_x3s_stamps(buf.ctypes.data_as(ctypes.c_void_p))
    assert rc == 0, rc
    st = buf.reshape(8, 64, 8).astype(np.int64)
    names = ["wait_dma", "barrier", "issue_dma", "region1", "region2", "to_next"]
    res = {}
    for wv in range(8):
        d = np.diff(st[wv, :, :6], axis=1)
        nxt = st[wv, 1:, 0] - st[wv, :-1, 5]
        per = {nm: float(np.median(d[8:60, i])) for i, nm in enumerate(names[:5])}
        per["to_next"] = float(np.median(nxt[8:60]))
        per["interval"] = float(np.median(np.diff(st[wv, 8:61, 0])))
        res[f"wave{wv}"] = per
        print(json.dumps({"wave": wv, **{kk: round(v) for kk, v in per.items()}}))
    print(json.dumps({"cfg": a.cfg, "shape": a.shape, "median_cycles": res}))


if __name__ == "__main__":
    main()
