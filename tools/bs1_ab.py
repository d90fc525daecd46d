"""bs1 forward A/B on hipGraph replays: the split-K launches' tile, split cap and minimum k-tiles
(sp_set_splitk_config), the split-K combine ("comb": inside the GEMM launch, Engine.splitk_combine; else
the reduce launch), the fused post-LayerNorm epilogue (Engine.fuse_ln, diagnostic builds) and the decoder's
small-M linears on the split kernel ("x3dec", a second engine), same process,
variants interleaved over several rounds.

    python tools/bs1_ab.py [--preset r101vd] [--reps 100] [--rounds 3] [--variants plain:-1:16:8,ln:-1,...]

Prints one JSON line per variant: median replay ms per round, and the max |Δ| of its logits / boxes against
the first variant (bit-identical expected for the same tile; same-order sums for another tile)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from spotter_amd import ops
from spotter_amd.config import PRESETS
from spotter_amd.engine import Engine
from spotter_amd.graph import GraphRunner
from spotter_amd.weights import generate


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="plain:-1:16:8,comb:-1:16:8")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = PRESETS[a.preset]
    dev = torch.device("cuda", 0)
    eng = Engine(cfg, generate(cfg, seed=0), dev)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand((1, 3, cfg.image_size, cfg.image_size), device=dev, generator=g)
    dflt = ["plain", "-1", "16", "8"]  # plain|comb|ln|x3dec|w<n> : split-K tile : max splits : min k-tiles
    variants = [(lambda q: q + dflt[len(q):])(v.split(":")) for v in a.variants.split(",")]
    runners, ref = {}, None
    res = {}
    eng_x3 = None
    for mode, c, ms, mk in variants:
        if mode == "x3dec":  # the decoder's small-M linears on the split kernel instead of the fp32 MFMA
            if eng_x3 is None:
                import spotter_amd.engine as em

                saved = em._X3_FASTER
                em._X3_FASTER = saved | {(n, k, True) for n in range(129, 4097) for k in (256, 512, 1024)}
                try:
                    eng_x3 = Engine(cfg, generate(cfg, seed=0), dev)
                finally:
                    em._X3_FASTER = saved
            eng_run = eng_x3
        else:
            eng_run = eng
        # "w<n>": the F(4x4) Winograd size gate at pixels x Cin >= 2^n (Engine.WINO43_MIN_WORK; default 2^19)
        eng_run.WINO43_MIN_WORK = 1 << int(mode[1:]) if mode[:1] == "w" else Engine.WINO43_MIN_WORK
        eng_run.fuse_ln = mode == "ln"  # the post-LNs fused into the GEMM epilogue
        eng_run.splitk_combine = mode == "comb"  # "comb": split-K combined inside the GEMM launch
        # "nosk<rows>": linears over at most <rows> rows never split K (Engine.splitk_min_rows)
        eng_run.splitk_min_rows = int(mode[4:]) if mode.startswith("nosk") else 0
        ops.force_splitk_config(c, int(ms), int(mk))
        try:
            r = GraphRunner(eng_run, 1, cfg.image_size, cfg.image_size)
        finally:
            ops.force_splitk_config(None)
        lg, bx = r(x)
        torch.cuda.synchronize()
        out = (lg.cpu().numpy().copy(), bx.cpu().numpy().copy())
        if ref is None:
            ref = out
        key = f"{mode}:{c}:{ms}:{mk}"
        runners[key] = r
        res[key] = {"max_dlogit": float(np.abs(out[0] - ref[0]).max()), "max_dbox": float(np.abs(out[1] - ref[1]).max()),
                    "bit_identical": bool(np.array_equal(out[0], ref[0]) and np.array_equal(out[1], ref[1])), "ms": []}
    for _ in range(a.rounds):
        for key, r in runners.items():
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r.graph.replay()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            res[key]["ms"].append(round(float(np.median(ts)), 4))
    for key, r in runners.items():  # after hundreds of replays: still the same outputs
        lg, bx = r(x)
        torch.cuda.synchronize()
        res[key]["bit_identical_after_replays"] = bool(np.array_equal(lg.cpu().numpy(), ref[0])
                                                       and np.array_equal(bx.cpu().numpy(), ref[1]))
    for key, v in res.items():
        v["median_ms"] = round(float(np.median(v["ms"])), 4)
        print(json.dumps({"variant": key, **v}), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
