"""Same-process A/B of an Engine knob, alternating on one engine per config: ms per forward (HIP events over
`iters` eager forwards) and the max |Δ| of the outputs. --knob add_rows (default): the h + pos attention inputs
materialised by sp_add_rows so the q/k and offset projections take the LDS-DMA tiles, against the register-staged
A2 addend; --knob enc_head_bf16: the bf16 variant's encoder-head LayerNorm into bf16 rows, against the fp32 map.

    python tools/engine_knob_ab.py [--knob add_rows] [--configs c3,c2bf16,c2] [--iters 10] [--rounds 3] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spotter_amd import SpotterForObjectDetection  # noqa: E402
from spotter_amd.config import PRESETS  # noqa: E402

CONFIGS = {"c3": ("r18vd", "bf16", 256), "c2bf16": ("r101vd", "bf16", 32), "c2": ("r101vd", "fp32", 32)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knob", default="add_rows")
    ap.add_argument("--configs", default="c3,c2bf16,c2")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    res = []
    for name in a.configs.split(","):
        preset, prec, bs = CONFIGS[name]
        model = SpotterForObjectDetection(PRESETS[preset], use_graphs=False, precision=prec)
        eng = model.engine
        g = torch.Generator(device="cuda").manual_seed(0)
        px = torch.rand(bs, 3, 640, 640, device="cuda", generator=g)
        outs = {}
        times = {True: [], False: []}
        for r in range(a.rounds):
            for mode in ((True, False) if r % 2 == 0 else (False, True)):
                setattr(eng, a.knob, mode)
                with torch.no_grad():
                    for _ in range(2):
                        eng.forward(px)
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(a.iters):
                        lg, bx = eng.forward(px)
                    e1.record()
                    torch.cuda.synchronize()
                times[mode].append(e0.elapsed_time(e1) / a.iters)
                outs[mode] = (lg.clone(), bx.clone())
        setattr(eng, a.knob, True)
        dl = float((outs[True][0] - outs[False][0]).abs().max())
        db = float((outs[True][1] - outs[False][1]).abs().max())
        e = {"config": name, "knob": a.knob, "ms_on": sorted(times[True])[len(times[True]) // 2],
             "ms_off": sorted(times[False])[len(times[False]) // 2], "runs_on": times[True],
             "runs_off": times[False], "max_dlogit": dl, "max_dbox": db}
        e["speedup"] = round(e["ms_off"] / e["ms_on"], 4)
        res.append(e)
        print(json.dumps(e), flush=True)
        del model, eng, px, outs
        torch.cuda.empty_cache()
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump({"what": __doc__.strip().splitlines()[0], "runs": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
