"""Observed parity margins of the golden tests ("measure and widen the parity margins").

Every golden parity test records, per case, the worst value it saw of each compared quantity; at the
end of the session tests/conftest.py writes them with the bars to $SPOTTER_MARGINS_OUT (default
gpurun_out/parity_margins.json), so a run shows how much of the 1e-3 score / 0.5 px bar each
configuration uses, not only that it passed.
"""
from __future__ import annotations

import json
import os

MARGINS: dict = {}
BARS = {"dsigma": 1e-3, "dbox_px": 0.5, "det_dscore": 1e-3, "det_dbox_px": 0.5, "anchors_shared_min": 298}


def record(case: str | None, **vals) -> None:
    """Fold vals into MARGINS[case]: maxima, except *_min keys (minima) and counters (*_n: sums)."""
    if not case:
        return
    d = MARGINS.setdefault(case, {})
    for k, v in vals.items():
        v = float(v)
        if k.endswith("_min"):
            d[k] = min(d.get(k, v), v)
        elif k.endswith("_n"):
            d[k] = d.get(k, 0) + v
        else:
            d[k] = max(d.get(k, v), v)


def write(path: str | None = None) -> str | None:
    if not MARGINS:
        return None
    path = path or os.environ.get("SPOTTER_MARGINS_OUT") or os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "parity_margins.json")
    out = {"bars": BARS, "cases": {}}
    for case, d in sorted(MARGINS.items()):
        row = dict(d)
        for k in ("dsigma", "dbox_px", "det_dscore", "det_dbox_px"):
            if k in row:
                row[k + "_frac_of_bar"] = row[k] / BARS[k]
        out["cases"][case] = row
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    return path
