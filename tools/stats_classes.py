"""Per-kernel-class summary of a `rocprofv3 --kernel-trace --stats` run (kernel_stats.csv, or the
rocpd SQLite database's top_kernels view), for cross-checking bench.py's HIP-event roofline (the
average conv launch duration must agree).

    python tools/stats_classes.py <kernel_stats.csv | results.db> [--csv-out kernels.csv]
"""
import csv
import json
import os
import sys

CLASSES = [("conv", ("conv_gemm", "conv_mfma16", "conv_glds", "conv_pipe", "stem_conv", "conv3x3")), ("conv_splitk_reduce", ("splitk_reduce",)), ("msda", ("msda",)),
           ("attention_bf16", ("attn_bf16",)), ("attention", ("attn_",)), ("preprocess", ("preprocess",)), ("topk", ("topk",)),
           ("layernorm", ("layernorm",)), ("postprocess_decode", ("decode_kernel",)), ("wino_tf", ("wino_",))]


def rows(path):
    """(name, calls, total_ns) per kernel symbol."""
    if path.endswith(".db"):
        import sqlite3

        con = sqlite3.connect(path)
        # top_kernels durations are in microseconds
        return [(n, int(c), float(t) * 1e3) for n, c, t, *_ in con.execute("select * from top_kernels")]
    with open(path) as f:
        return [(r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(f)]


def main(path, csv_out=None):
    out = {}
    rs = rows(path)
    if csv_out:
        with open(csv_out, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs"])
            for n, c, t in sorted(rs, key=lambda r: -r[2]):
                w.writerow([n, c, int(t), round(t / c, 1)])
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pmc_reduce import operand_planes

    for name, calls, total_ns in rs:
        short = name.replace("(anonymous namespace)", "").split("(")[0]
        if operand_planes(short) == 3:  # the dominant kernel's own class (also counted under conv)
            c = out.setdefault("conv_x3", {"calls": 0, "total_ms": 0.0})
            c["calls"] += calls
            c["total_ms"] += total_ns / 1e6
        cls = next((c for c, keys in CLASSES if any(k in short for k in keys)), "other")
        c = out.setdefault(cls, {"calls": 0, "total_ms": 0.0})
        c["calls"] += calls
        c["total_ms"] += total_ns / 1e6
    for c in out.values():
        c["avg_ms"] = round(c["total_ms"] / c["calls"], 4)
        c["total_ms"] = round(c["total_ms"], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--csv-out" else None)
