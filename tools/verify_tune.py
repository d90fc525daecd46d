"""Re-measure tools/tune_conv.py winners against the production choice in interleaved rounds (one process,
alternating configurations: guide §5.4 rule 24). tune_conv times the production choice first on freshly
allocated buffers, which biases it; only winners that hold up here should enter the tile table.

    python tools/verify_tune.py <tune.json> [--min-saving 0.02] [--rounds 5] [--reps 10] [--out verified.json]

The output has tune_conv's format ({"shapes": [...]}, times {"-": ms, cfg: ms} as interleaved medians), so
tools/gen_tile_table.py reads it directly.
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from tune_conv import time_one


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tune")
    ap.add_argument("--min-saving", type=float, default=0.02)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--out", default="verified.json")
    ap.add_argument("--skip-m", default="", help="M values to skip (e.g. the Winograd batches tune_conv read as GEMMs)")
    a = ap.parse_args()
    skip = {int(v) for v in a.skip_m.split(",") if v}
    dev = torch.device("cuda", 0)
    res = []
    for e in json.load(open(a.tune))["shapes"]:
        best = e["best_same_mode"] if "best_same_mode" in e else e["best_cfg"]
        if best == "-" or ":" in best or e["saving_ms_per_step"] < a.min_saving or e["m"] in skip:
            continue
        args = (dev, e["m"], e["cout"], e["K"], e["k"], e["stride"], e["mode"])
        t = {"-": [], best: []}
        time_one(*args, "-", 2)  # warm both
        time_one(*args, best, 2)
        for _ in range(a.rounds):
            for c in ("-", best):
                v = time_one(*args, c, a.reps)
                if v is not None:
                    t[c].append(v)
        if not t["-"] or not t[best]:
            continue
        times = {c: round(statistics.median(v), 4) for c, v in t.items()}
        out = dict(e, times=times, default_ms=times["-"], best_cfg=best if times[best] < times["-"] else "-",
                   best_ms=min(times.values()),
                   saving_ms_per_step=round((times["-"] - min(times.values())) * e["launches_per_step"], 4))
        out.pop("best_same_mode", None)
        res.append(out)
        print(json.dumps({k: out[k] for k in ("m", "cout", "K", "k", "stride", "times", "saving_ms_per_step")}),
              flush=True)
    tot = sum(x["saving_ms_per_step"] for x in res)
    json.dump({"shapes": res, "saving_ms_per_step": round(tot, 3)}, open(a.out, "w"), indent=1)
    print(json.dumps({"verified_saving_ms_per_step": round(tot, 3)}))


if __name__ == "__main__":
    main()
