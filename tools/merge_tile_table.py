"""Merge tools/tune_conv.py results into the existing spotter_amd/csrc/tile_table.h (entries for the shapes
and operand modes measured; every other entry and its comment kept).

    python tools/merge_tile_table.py <tune.json> [...] --tag "r4 bf16 rows" [--min-gain 0.02]

For each measured (shape, mode): when the winner beats the current choice ("-": the table entry if there
is one, else the by-shape rule) by more than --min-gain, the entry becomes the winner; otherwise the
current state stays (a measured "-" win never deletes an entry: "-" already includes it).
"""
import argparse
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_tile_table import runnable  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "spotter_amd", "csrc", "tile_table.h")
ENTRY = re.compile(r"^\s*\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (-?\d+)\},\s*(//.*)?$")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tunes", nargs="+")
    ap.add_argument("--tag", required=True)
    ap.add_argument("--min-gain", type=float, default=0.02)
    ap.add_argument("--table", default=TABLE, help="the tile_table.h to update (default: the library's)")
    ap.add_argument("--detail", action="append", default=[],
                    help="bench.py --detail file: its Winograd component GEMMs (batched, tiled by wino_gemm's own "
                         "rule, not the table) are skipped")
    a = ap.parse_args()
    import ast
    wino = set()
    for p in a.detail:
        for r in json.load(open(p)):
            k = ast.literal_eval(r["shape"])
            if len(k) > 6 and k[6] == "wino":
                wino.add(tuple(k[:3]))
    lines = open(a.table).read().split("\n")
    ent, order = {}, []
    first = last = None
    for i, l in enumerate(lines):
        m = ENTRY.match(l)
        if m and int(m.group(1)) > 0:
            key = tuple(int(m.group(k)) for k in range(1, 7))
            ent[key] = (int(m.group(7)), (m.group(8) or "").strip())
            first = i if first is None else first
            last = i
    changed = []
    for p in a.tunes:
        for e in json.load(open(p))["shapes"]:
            planes = {"x3": 3, "bf16": 1}.get(e["mode"], 0)
            key = (e["m"], e["cout"], e["K"], e["k"], e["stride"], planes)
            if (e["m"], e["cout"], e["K"]) in wino:
                continue
            times = {c: t for c, t in e["times"].items() if ":" not in c}
            if not e.get("rows", False):  # fp32-A launches: the bf16-row-only tiles are not theirs
                times = {c: t for c, t in times.items() if c == "-" or not 52 <= int(c) % 100 <= 59}
            d = times.get("-")
            best = min(times, key=times.get) if times else "-"
            if d is None or best == "-" or times[best] > d * (1 - a.min_gain):
                continue
            if planes and not runnable(int(best), e["K"] // (e["k"] * e["k"]), e["cout"]):
                continue
            ent[key] = (int(best), f"// x{d / times[best]:.3f} ({a.tag})")
            changed.append((key, best, round(d / times[best], 3)))
    body = [f"    {{{k[0]}, {k[1]}, {k[2]}, {k[3]}, {k[4]}, {k[5]}, {v[0]}}},  {v[1]}".rstrip()
            for k, v in sorted(ent.items())]
    out = lines[:first] + body + lines[last + 1:]
    open(a.table, "w").write("\n".join(out))
    for c in changed:
        print(c)
    print(f"{len(changed)} entries set; {len(ent)} in the table")


if __name__ == "__main__":
    main()
