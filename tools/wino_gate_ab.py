"""Same-process A/B of the Winograd size gate on the bs1 /detect latency path: two models, one with the
product gate (Engine._wino_pays), one with Winograd restricted to the old >= 8192-pixel rule, measured in
alternation (tools/latency.py's measure: p50 of the bs1 core and of the GPU-only forward).

    python tools/wino_gate_ab.py [--preset r101vd] [--iters 100] [--rounds 2] [--out f.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from spotter_amd import SpotterForObjectDetection  # noqa: E402
from spotter_amd.config import PRESETS  # noqa: E402
from tools.latency import measure  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    gate = SpotterForObjectDetection(PRESETS[a.preset], use_graphs=True)
    old = SpotterForObjectDetection(PRESETS[a.preset], use_graphs=True)
    old.engine._wino_pays = lambda pixels, cin: pixels >= old.engine.WINO_MIN_PIXELS
    res = []
    for r in range(a.rounds):
        for name, m in (("pixels_x_cin_gate", gate), ("pixels_8192_gate", old)):
            lat = measure(a.preset, a.iters, graphs=True, model=m)
            e = {"round": r, "gate": name, "p50_ms": lat["p50_ms"], "forward_p50_ms": lat["forward_p50_ms"],
                 "model_p50_ms": lat["stages_p50_ms"]["model"]}
            res.append(e)
            print(json.dumps(e), flush=True)
    if a.out:
        json.dump({"what": __doc__.strip().splitlines()[0], "preset": a.preset, "runs": res}, open(a.out, "w"),
                  indent=1)


if __name__ == "__main__":
    main()
