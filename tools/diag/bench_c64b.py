"""Time sp_conv3x3_c64_bf16 (the bf16 variant's stage-0 3x3) at C3's shape, with and without the residual.
Run from a tree's root (it imports that tree's spotter_amd): python <path>/bench_c64b.py"""
import json
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

from spotter_amd import ops
from spotter_amd.ops import V

dev = torch.device("cuda", 0)
n, h, w = 256, 160, 160
m = n * h * w
g = torch.Generator(device=dev).manual_seed(0)
b16 = lambda t: t.to(torch.bfloat16).view(torch.int16).contiguous()
x = b16(torch.randn(m * 64, device=dev, generator=g))
r = b16(torch.randn(m * 64, device=dev, generator=g))
wt = b16(torch.randn(64 * 576, device=dev, generator=g) / 24)
sc = torch.rand(64, device=dev, generator=g) + 0.5
sh = torch.randn(64, device=dev, generator=g)
y = torch.empty(m * 64, dtype=torch.int16, device=dev)
out = {}
for res in (False, True):
    def run():
        ops.conv3x3_c64_bf16(V(x, 0, 64), wt, sc, sh, V(y, 0, 64), n, h, w, act="relu",
                             res1=V(r, 0, 64) if res else None)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / 10)
    out["res" if res else "plain"] = round(sorted(ts)[1], 4)
    out["checksum_" + ("res" if res else "plain")] = int(y.view(torch.int16).to(torch.int64).sum().item())
print(json.dumps(out))

# the stem convs 2 / 3 (Cin 32 → Cout 32 / 64) at C3's 320² map
if os.environ.get("C32", "1") == "1":
    n2, h2, w2 = 256, 320, 320
    m2 = n2 * h2 * w2
    x2 = b16(torch.randn(m2 * 32, device=dev, generator=g))
    y2 = torch.empty(m2 * 64, dtype=torch.int16, device=dev)
    for cout in (32, 64):
        wt2 = b16(torch.randn(cout * 288, device=dev, generator=g) / 17)
        def run():
            ops.conv3x3_c32_bf16(V(x2, 0, 32), wt2, sc, sh, V(y2, 0, cout), n2, h2, w2, cout, act="relu")
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 10)
        out[f"c32_{cout}"] = round(sorted(ts)[1], 4)
        out[f"checksum_c32_{cout}"] = int(y2[:m2 * cout].to(torch.int64).sum().item())
    print(json.dumps(out))
