"""Micro-bench of sp_conv2d on the R101vd@640 bs32 shapes that dominate the step (per-shape TFLOP/s).

    python tools/conv_bench.py [--prec fp32,f32x3,bf16] [--cfgs -,1,2] [--shapes 0,1,2] [--reps 20]

cfg "-" = the library's own tile choice; other values go to sp_set_conv_config (fp32 kernel: "<TM><TN><DB>",
bf16 / f32x3 kernels: 1..6). Prints one JSON line per (shape, precision, cfg), plus the step-weighted
total for the default choice.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from spotter_amd import ops
from spotter_amd.ops import view

# (n, h, w, cin, cout, k, stride, act, residual, launches per bs32 step)  — from bench.py --detail
SHAPES = [
    (32, 80, 80, 384, 384, 3, 1, None, False, 3),       # 0  CCFM 3x3 @80²         13.3 ms/step fp32
    (32, 40, 40, 256, 256, 3, 1, "relu", False, 22),    # 1  stage3 3x3            12.4
    (32, 40, 40, 384, 384, 3, 1, None, False, 6),       # 2  CCFM 3x3 @40²          7.2
    (32, 40, 40, 256, 1024, 1, 1, "relu", True, 23),    # 3  stage3 expand          6.8
    (32, 40, 40, 1024, 256, 1, 1, "relu", False, 22),   # 4  stage3 reduce          5.8
    (32, 80, 80, 768, 768, 1, 1, None, False, 1),       # 5  CCFM 1x1 768 @80²      2.1
    (1, 1, 268800, 256, 1536, 1, 1, None, False, 1),    # 6  decoder value_all      2.0
    (32, 160, 160, 256, 64, 1, 1, "relu", False, 4),    # 7  stage0 reduce (K=64→N)  1.8 (K=256)
    (32, 160, 160, 64, 64, 3, 1, "relu", False, 3),     # 8  stage0 3x3             1.8
    (32, 80, 80, 128, 128, 3, 1, "relu", False, 3),     # 9  stage1 3x3             1.7
    (32, 80, 80, 128, 512, 1, 1, "relu", True, 4),      # 10 stage1 expand          1.4
    (32, 20, 20, 512, 512, 3, 1, "relu", False, 2),     # 11 stage4 3x3             1.2
    (32, 320, 320, 32, 64, 3, 1, "relu", False, 1),     # 12 stem conv3             1.2
    (32, 320, 320, 32, 32, 3, 1, "relu", False, 1),     # 13 stem conv2             1.1
    (1, 1, 9600, 256, 256, 1, 1, None, True, 32),       # 14 decoder linear          0.8
    (32, 640, 640, 3, 32, 3, 2, "relu", False, 1),      # 15 stem conv1 (Cin=3)
    (32, 160, 160, 64, 256, 1, 1, "relu", True, 4),     # 16 stage0 expand
    (32, 20, 20, 384, 384, 3, 1, None, False, 3),       # 17 CCFM 3x3 @20²
    (32, 20, 20, 512, 2048, 1, 1, "relu", True, 3),     # 18 stage4 expand
    (32, 80, 80, 512, 128, 1, 1, "relu", False, 3),     # 19 stage1 reduce
    # fused bottleneck tail + projection shortcut (engine._fused_tail): K = red + cin
    (32, 160, 160, 128, 256, 1, 1, "relu", False, 1),   # 20 stage0 block0 fused tail
    (32, 80, 80, 384, 512, 1, 1, "relu", False, 1),     # 21 stage1 block0 fused tail
    (32, 40, 40, 768, 1024, 1, 1, "relu", False, 1),    # 22 stage2 block0 fused tail
    (32, 20, 20, 1536, 2048, 1, 1, "relu", False, 1),   # 23 stage3 block0 fused tail
    # bs1 /detect latency path (run with --ws: the engine hands every conv a split-K workspace)
    (1, 80, 80, 384, 384, 3, 1, None, False, 3),        # 24 CCFM 3x3 @80² bs1
    (1, 40, 40, 256, 256, 3, 1, "relu", False, 22),     # 25 stage3 3x3 bs1
    (1, 40, 40, 1024, 256, 1, 1, "relu", False, 22),    # 26 stage3 reduce bs1
    (1, 40, 40, 256, 1024, 1, 1, "relu", True, 23),     # 27 stage3 expand bs1
    # C3 (R18vd bs256) basic-block 3x3s
    (256, 80, 80, 128, 128, 3, 1, "relu", False, 3),    # 28 stage1 3x3 (C3's largest bucket)
    (256, 160, 160, 64, 64, 3, 1, "relu", False, 4),    # 29 stage0 3x3
    (256, 40, 40, 256, 256, 3, 1, "relu", False, 3),    # 30 stage2 3x3
    (1, 1, 2150400, 256, 768, 1, 1, None, False, 1),    # 31 C3 decoder value_all (3 layers x 256)
    # C3 decoder linears (bs256 x 300 queries; fp32 rows, bf16 weights) and the encoder output head
    (1, 1, 76800, 256, 256, 1, 1, None, False, 11),     # 32 dec 256->256 (v, o, bbox)
    (1, 1, 76800, 256, 512, 1, 1, None, False, 3),      # 33 dec qk (256->512)
    (1, 1, 76800, 256, 1024, 1, 1, "relu", False, 3),   # 34 dec fc1
    (1, 1, 76800, 1024, 256, 1, 1, None, True, 3),      # 35 dec fc2 (+res)
    (1, 1, 76800, 256, 288, 1, 1, None, False, 3),      # 36 dec offsets/weights
    (1, 1, 2150400, 256, 256, 1, 1, None, False, 1),    # 37 C3 enc_output
    (1, 1, 2150400, 256, 80, 1, 1, None, False, 1),     # 38 C3 enc_score
    (256, 80, 80, 128, 256, 1, 1, None, False, 2),      # 39 C3 CCFM 1x1 128->256 @80² (short K)
]


def bench_one(dev, shape, prec, cfg, reps, ws=False):
    n, h, w, cin, cout, k, st, act, resid, _ = shape
    ops.force_conv_config(cfg)
    pad = k // 2
    ho, wo = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
    m = n * ho * wo
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(n * h * w * cin, device=dev, generator=g)
    rows16 = prec == "bf16rows"  # the bf16 variant's form: bf16 activation rows in and out (A16, C_bf16)
    b16 = lambda t: t.to(torch.bfloat16).view(torch.int16).contiguous()
    wt = torch.randn(cout * k * k * cin, device=dev, generator=g) * (1.0 / (cin * k * k) ** 0.5)
    sc = torch.rand(cout, device=dev, generator=g) + 0.5
    sh = torch.randn(cout, device=dev, generator=g)
    out = torch.empty(m * cout, device=dev, dtype=torch.int16 if rows16 else torch.float32)
    r1 = torch.randn(m * cout, device=dev, generator=g) if resid else None
    if rows16:
        x = b16(x)
        r1 = b16(r1) if r1 is not None else None
    kw = {}
    if prec in ("bf16", "bf16rows"):
        kw["wt16"] = wt.to(torch.bfloat16).view(torch.int16).contiguous()
    elif prec == "f32x3":
        kw["wt_planes"] = ops.split_bf16x3(wt)

    if ws:
        kw["workspace"] = torch.empty(16 << 20, device=dev)

    def run():
        ops.conv2d(view(x, cin), n, h, w, cin, wt, cout, k, st, pad, view(out, cout), scale=sc, shift=sh,
                   act=act, res1=view(r1, cout) if resid else None, **kw)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    fl = 2.0 * m * cout * cin * k * k
    return {"shape": list(shape[:7]), "prec": prec, "cfg": cfg, "ms": round(ms, 4),
            "tflops": round(fl / ms / 1e9, 1), "ms_per_step": round(ms * shape[9], 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32")
    ap.add_argument("--cfgs", default="-")
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--ws", action="store_true", help="pass a split-K workspace (as the engine does)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    which = [int(i) for i in a.shapes.split(",")] if a.shapes else range(len(SHAPES))
    tot = {}
    for si in which:
        for prec in a.prec.split(","):
            for cfg in a.cfgs.split(","):
                try:
                    r = bench_one(dev, SHAPES[si], prec, cfg, a.reps, a.ws)
                except RuntimeError as e:  # a tile config the shape/mode cannot use (e.g. LDS overflow)
                    print(json.dumps({"shape": SHAPES[si][:7], "prec": prec, "cfg": cfg, "skipped": str(e)}), flush=True)
                    continue
                print(json.dumps(r), flush=True)
                if cfg == "-":
                    tot[prec] = tot.get(prec, 0.0) + r["ms_per_step"]
    print(json.dumps({"step_weighted_ms_default_cfg": {k: round(v, 2) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
