"""sp_preprocess_u8 on the C5 mixed stream's batches, split by source: per-launch time of the whole bs8 batch, of
its 4K source alone and of the other seven, and the same-size C2 batch (bs32 640²): where the launch's time goes.

    python tools/microbench/pre_mix.py [--reps 50]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from bench import MIXED_SOURCES, stream_plan
from spotter_amd import ops
from spotter_amd.synthetic import synthetic_image


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    npool, plan = stream_plan(len(MIXED_SOURCES), 8)
    pool = [torch.from_numpy(synthetic_image(1234 + j, *MIXED_SOURCES[j % len(MIXED_SOURCES)])).to(dev)
            for j in range(npool)]

    def timed(imgs, out, S):
        for _ in range(3):
            ops.preprocess_u8(imgs, out, S, S)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ops.preprocess_u8(imgs, out, S, S)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    out = torch.empty(32 * 3 * 1280 * 1280, device=dev)
    res = {}
    for bi, idx in enumerate(plan[:3]):
        imgs = [pool[j] for j in idx]
        big = [im for im in imgs if im.shape[0] >= 2160]
        rest = [im for im in imgs if im.shape[0] < 2160]
        byt = sum(im.numel() for im in imgs) + len(imgs) * 3 * 1280 * 1280 * 4
        r = {"sources": [list(im.shape[:2]) for im in imgs], "ms_batch": timed(imgs, out, 1280),
             "ms_4k_only": timed(big, out, 1280) if big else None, "ms_rest": timed(rest, out, 1280),
             "ms_each": [round(timed([im], out, 1280), 4) for im in imgs]}
        r["gbps_batch"] = round(byt / r["ms_batch"] / 1e6, 1)
        res[f"batch{bi}"] = r
        print(json.dumps({f"batch{bi}": r}), flush=True)
    same = [torch.from_numpy(synthetic_image(7 + i, 640, 640)).to(dev) for i in range(32)]
    ms = timed(same, out, 640)
    res["c2_same_size_bs32"] = {"ms": round(ms, 4), "gbps": round(32 * (640 * 640 * 3 * 5) / ms / 1e6, 1)}
    print(json.dumps(res["c2_same_size_bs32"]))


if __name__ == "__main__":
    main()
