"""Micro-bench of sp_conv2d on the R101vd@640 bs32 shapes that dominate the step (per-shape TFLOP/s)."""
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import view

# (n, h, w, cin, cout, k, stride, act, residual)
SHAPES = [
    (32, 40, 40, 256, 256, 3, 1, "relu", False),     # stage3 3x3        14.7 ms/step
    (32, 80, 80, 384, 384, 3, 1, None, False),       # CCFM 3x3 @80²      13.4
    (32, 40, 40, 256, 1024, 1, 1, "relu", True),     # stage3 expand      12.0
    (32, 40, 40, 1024, 256, 1, 1, "relu", False),    # stage3 reduce       7.5
    (32, 160, 160, 64, 256, 1, 1, "relu", True),     # stage0 expand       5.0
    (32, 80, 80, 128, 512, 1, 1, "relu", True),      # stage1 expand       3.2
    (32, 80, 80, 384, 384, 1, 1, "silu", True),      # CCFM 1x1 @80²       3.0
    (1, 1, 268800, 256, 1536, 1, 1, None, False),    # value_all           2.7
    (32, 20, 20, 512, 2048, 1, 1, "relu", True),     # stage4 expand
    (1, 1, 9600, 256, 256, 1, 1, None, True),        # decoder linear
    (64, 40, 40, 256, 256, 3, 1, "relu", False),     # 10: stage3 3x3 at 2x batch (tail test)
    (128, 40, 40, 256, 256, 3, 1, "relu", False),    # 11: 4x batch
    (32, 320, 320, 32, 32, 3, 1, "relu", False),     # 12: stem conv2 (N=32)
    (32, 640, 640, 3, 32, 3, 2, "relu", False),      # 13: stem conv1 (Cin=3)
]


def bench_one(dev, shape, cfg):
    n, h, w, cin, cout, k, st, act, resid = shape
    if cfg:
        os.environ["SP_CONV_CFG"] = cfg
    else:
        os.environ.pop("SP_CONV_CFG", None)
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    m = n * ho * wo
    x = torch.randn(n * h * w * cin, device=dev)
    wt = torch.randn(cout * k * k * cin, device=dev) * (1.0 / (cin * k * k) ** 0.5)
    sc = torch.rand(cout, device=dev) + 0.5
    sh = torch.randn(cout, device=dev)
    out = torch.empty(m * cout, device=dev)
    r1 = torch.randn(m * cout, device=dev) if resid else None

    def run():
        ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, st, pad, view(out, cout), scale=sc, shift=sh,
                   act=act, res1=view(r1, cout) if resid else None)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * m * cout * cin * k * k
    return {"shape": [n, h, w, cin, cout, k, st], "cfg": cfg, "ms": round(ms, 4), "tflops": round(fl / ms / 1e9, 1)}


def main():
    dev = torch.device("cuda", 0)
    cfgs = sys.argv[1].split(",") if len(sys.argv) > 1 and sys.argv[1] != "-" else [None]
    which = [int(i) for i in sys.argv[2].split(",")] if len(sys.argv) > 2 else range(len(SHAPES))
    for si in which:
        shape = SHAPES[si]
        for cfg in cfgs:
            print(json.dumps(bench_one(dev, shape, cfg)), flush=True)


if __name__ == "__main__":
    main()
