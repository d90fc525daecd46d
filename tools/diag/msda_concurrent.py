"""Is sp_msda's output independent of what runs beside it? Decoder-shaped inputs (B=16, Q=300, 640^2 maps, the
engine's ld-1536 value_all layout); the reference output comes from a quiet GPU, then the same launch repeats
on stream A while stream B runs (a) nothing, (b) large matmuls, (c) another sp_msda on its own buffers. Prints
how many repeats differ from the reference for the point-sharing kernel and for msda_vec_kernel."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from spotter_amd import ops
from spotter_amd._lib import lib
from spotter_amd.ops import V

dev = torch.device("cuda", 0)
B, Q, nH, dh, nL, nP = 16, 300, 8, 32, 3, 4
shapes, starts, S = [(80, 80), (40, 40), (20, 20)], [0, 6400, 8000], 8400
D = nH * dh
g = torch.Generator(device=dev).manual_seed(3)


def inputs():
    val = torch.randn(B * S * 6 * D, device=dev, generator=g)
    offaw = torch.cat([torch.randn(B * Q, nH * nL * nP * 2, device=dev, generator=g) * 3.0,
                       torch.randn(B * Q, nH * nL * nP, device=dev, generator=g) * 2.0], 1).contiguous()
    ref = torch.cat([torch.rand(B * Q, 2, device=dev, generator=g),
                     torch.rand(B * Q, 2, device=dev, generator=g) * 0.9 + 0.01], 1).contiguous()
    return val, offaw, ref


def launch(buf, out):
    val, offaw, ref = buf
    ops.msda(V(val, 0, 6 * D), 3 * D, V(offaw.view(-1), 0, offaw.shape[1]), ref, V(out, 0, D),
             B, S, Q, nH, dh, shapes, starts, nP, 0.5)


def run(generic, reps=60):
    lib().sp_set_tuning(4, generic)
    a, b = inputs(), inputs()
    out_ref = torch.empty(B * Q * D, device=dev)
    launch(a, out_ref)
    torch.cuda.synchronize()
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    x = torch.randn(4096, 4096, device=dev)
    res = {}
    for mode in ("alone", "matmul", "msda"):
        outs = [torch.empty(B * Q * D, device=dev) for _ in range(reps)]
        ob = torch.empty(B * Q * D, device=dev)
        for r in range(reps):
            with torch.cuda.stream(sb):
                if mode == "matmul":
                    x @ x
                elif mode == "msda":
                    launch(b, ob)
            with torch.cuda.stream(sa):
                launch(a, outs[r])
        torch.cuda.synchronize()
        diffs = [float((o - out_ref).abs().max()) for o in outs]
        nan = sum(int(torch.isnan(o).any()) for o in outs)
        res[mode] = {"n_differ": sum(d > 0 for d in diffs), "max": max(diffs), "nan": nan}
    lib().sp_set_tuning(4, 0)
    return res


for name, generic in (("h8", 0), ("vec", 1), ("h8_again", 0)):
    print(json.dumps({name: run(generic)}), flush=True)
