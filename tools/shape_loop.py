"""Run one GEMM shape of tools/ab_glds.py in a loop with the production (or a forced) tile choice: the
target program of focused rocprofv3 --pmc passes (tools/r3_pmc_shape.sh).

    python tools/shape_loop.py <shape index in ab_glds.SHAPES> [--cfg 46] [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from ab_glds import SHAPES, make
from spotter_amd import ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("shape", type=int)
    ap.add_argument("--cfg", default="-")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    run, out, flops = make(dev, SHAPES[a.shape])
    ops.force_conv_config(a.cfg)
    for _ in range(a.iters):
        run()
    torch.cuda.synchronize()
    print("done", SHAPES[a.shape], a.cfg, flush=True)


if __name__ == "__main__":
    main()
