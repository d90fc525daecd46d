"""Tile re-tune with interleaved rounds: per shape, every candidate configuration is timed once per round, for
R rounds, and the median decides. tools/tune_conv.py times each configuration in one block, so box drift and
clock ramps land on whichever configuration ran at that moment; tile differences on the big C2 shapes are a
few percent, the same size as that drift.

    python tools/retune_interleaved.py <bench --detail JSON> --steps 10 [--rounds 5] [--min-ms 0.1] --out t.json

Writes tools/tune_conv.py's JSON format (times = medians, plus every round under "rounds"), so
tools/merge_tile_table.py folds the winners into spotter_amd/csrc/tile_table.h.
"""
from __future__ import annotations

import argparse
import ast
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from tune_conv import F32_CFGS, time_one  # noqa: E402

X3_CANDIDATES = ["-", "12", "14", "33", "41", "44", "47", "63", "214", "245", "246", "247", "263", "212", "241"]
# bf16 rows: the slab-epilogue tiles (cfg, launched as cfg + 100) and the transposed-roles register epilogue
# (cfg + 300, 32x32 blocks only)
BF16_CANDIDATES = ["-", "12", "13", "14", "16", "33", "41", "45", "47", "52", "53", "63", "64",
                   "312", "313", "314", "316", "333", "345", "352", "363", "364"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("detail")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--min-ms", type=float, default=0.1, help="shapes cheaper than this per step are skipped")
    ap.add_argument("--modes", default="x3,f32")
    ap.add_argument("--cands", default="", help="comma-separated candidate list (default: by mode)")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = []
    for r in sorted(json.load(open(a.detail)), key=lambda r: -r["ms"]):
        key = ast.literal_eval(r["shape"])
        m, cout, K, k, stride, mode = key[:6]
        if len(key) > 6 and key[6] == "wino":
            continue  # batched Winograd component GEMMs: wino_gemm's own rule (tools/tune_wino.py)
        if mode not in a.modes.split(",") or r["ms"] / a.steps < a.min_ms:
            continue
        rows = "rows" in key[6:]
        epi = next((t[4:] for t in key[6:] if isinstance(t, str) and t.startswith("epi:")), "none")
        cands = (a.cands.split(",") if a.cands else
                 F32_CFGS if mode == "f32" else BF16_CANDIDATES if mode == "bf16" else X3_CANDIDATES)
        rounds = {c: [] for c in cands}
        for _ in range(a.rounds):
            for c in cands:
                t = time_one(dev, m, cout, K, k, stride, mode, c, a.reps, rows, epi)
                if t is not None:
                    rounds[c].append(round(t, 5))
        times = {c: round(statistics.median(v), 4) for c, v in rounds.items() if len(v) == a.rounds}
        best = min(times, key=times.get)
        launches = r["launches"] / a.steps
        e = {"m": m, "cout": cout, "K": K, "k": k, "stride": stride, "mode": mode, "rows": rows, "epi": epi,
             "wino": False, "launches_per_step": launches, "default_ms": times.get("-"), "best_cfg": best,
             "best_ms": times[best], "times": times, "rounds": rounds, "best_same_mode": best,
             "saving_ms_per_step": round((times.get("-", times[best]) - times[best]) * launches, 4)}
        res.append(e)
        print(json.dumps({k: v for k, v in e.items() if k != "rounds"}), flush=True)
    tot = sum(e["saving_ms_per_step"] for e in res)
    json.dump({"shapes": res, "saving_ms_per_step": round(tot, 3)}, open(a.out, "w"), indent=1)
    print(json.dumps({"saving_ms_per_step": round(tot, 3)}))


if __name__ == "__main__":
    main()
