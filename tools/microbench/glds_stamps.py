"""Where a conv_glds_kernel workgroup's time goes (diagnostic build: tools/build_diag.sh stamp
-DSP_GLDS_STAMP=1): per workgroup, s_memtime at start / first stage ready / main loop end / epilogue end
and its CU. Reports the median prologue, main-loop and epilogue cycles, the cycles per k-step, and the
workgroups resident per CU over time.

    SPOTTER_HIP_LIB=spotter_amd/_diag/libspotter_stamp.so python tools/microbench/glds_stamps.py <shape> [--cfg 46]
(<shape> = index into tools/ab_glds.py SHAPES)
"""
import argparse
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import numpy as np
import torch

from ab_glds import SHAPES, make
from spotter_amd import _lib, ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", type=int)
    ap.add_argument("--cfg", default="-")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    run, out, flops = make(dev, SHAPES[a.shape])
    ops.force_conv_config(a.cfg)
    for _ in range(5):
        run()
    torch.cuda.synchronize()
    buf = np.zeros(16384 * 6, np.uint64)
    L = _lib.lib()
    L.sp_debug_glds_stamps.restype = ctypes.c_int
    assert L.sp_debug_glds_stamps(buf.ctypes.data_as(ctypes.c_void_p)) == 0
    st = buf.reshape(16384, 6).astype(np.int64)
    st = st[st[:, 0] > 0]
    pro, main_, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    hw, xcc = st[:, 4], st[:, 5]
    cu = xcc * 1000 + ((hw >> 13) & 7) * 100 + ((hw >> 12) & 1) * 20 + ((hw >> 8) & 15)
    conc = []
    for c in np.unique(cu):
        sel = cu == c
        span = st[sel, 3].max() - st[sel, 0].min()
        conc.append((st[sel, 3] - st[sel, 0]).sum() / max(span, 1))
    res = {"shape": SHAPES[a.shape], "cfg": a.cfg, "workgroups": int(len(st)), "cus": int(len(np.unique(cu))),
           "median_cycles": {"prologue": float(np.median(pro)), "main": float(np.median(main_)),
                             "epilogue": float(np.median(epi)), "total": float(np.median(st[:, 3] - st[:, 0]))},
           "p90_cycles": {"prologue": float(np.percentile(pro, 90)), "main": float(np.percentile(main_, 90)),
                          "epilogue": float(np.percentile(epi, 90))},
           "resident_wg_per_cu_mean": float(np.mean(conc))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
