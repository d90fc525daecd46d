"""Fold the FETCH_SIZE / WRITE_SIZE passes of tools/pmc_bench.sh into HBM bytes per launch.

Per MI355X_MICROARCH.md (HBM section): rocprofv3's FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950
FETCH_SIZE counts half the bytes of wide (16 B/lane) coalesced reads, so it is doubled; WRITE_SIZE
is exact for 16 B/lane stores (the conv epilogue's float4 stores). HBM bytes = 2·FETCH + WRITE.
The conv class includes the split-K reduce kernel of the same sp_conv2d call; per-launch figures
divide by the number of conv dispatches (one per sp_conv2d call, plus the direct stem conv).

    python tools/pmc_reduce.py <outdir> [bench args]   # writes/updates profiles/pmc_traffic.json
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLASSES = [("conv", ("conv_gemm", "conv_mfma16", "conv_glds", "conv_pipe", "splitk_reduce", "stem_conv", "conv3x3")), ("msda", ("msda",)),
           ("attention_bf16", ("attn_bf16",)), ("attention", ("attn_",)),
           ("preprocess", ("preprocess",)), ("topk", ("topk",)), ("layernorm", ("layernorm",))]
LEADERS = {"conv": "conv_", "msda": "msda", "attention": "attn_mfma", "attention_bf16": "attn_bf16", "preprocess": None, "topk": "topk",
           "layernorm": "layernorm"}


def read(path, counter):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter:
                    rows.append((r["Kernel_Name"], float(r["Counter_Value"])))
    return rows


def operand_planes(short: str):
    """bf16 operand planes of a conv_mfma16.hip kernel instance from its template arguments
    (3 = the fp32-accurate split 'x3' kernels, 1 = bf16); None for other kernels."""
    import re

    m = re.search(r"(conv_glds_kernel|conv_mfma16_kernel|conv_pipe_kernel|conv_pp_kernel)<([^>]*)>", short)
    if not m:
        return None
    args = [a.strip() for a in m.group(2).split(",")]
    pos = 2 if m.group(1) == "conv_pp_kernel" else 4
    return int(args[pos]) if len(args) > pos and args[pos].isdigit() else None


def fold(rows):
    out = {}
    for name, v in rows:
        short = name.replace("(anonymous namespace)", "").split("(")[0]
        if operand_planes(short) == 3:  # the dominant kernel, broken out (it also counts under conv)
            c = out.setdefault("conv_x3", {"kib": 0.0, "n": 0})
            c["kib"] += v
            c["n"] += 1
        for cls, keys in CLASSES:
            if any(k in short for k in keys):
                c = out.setdefault(cls, {"kib": 0.0, "n": 0})
                c["kib"] += v
                lead = LEADERS[cls]
                if lead is None or lead in short:
                    c["n"] += 1
                break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--precision", default="fp32")
    ap.add_argument("--microbatches", type=int, default=None)
    ap.add_argument("--stream", default="same")
    a, _ = ap.parse_known_args()
    if a.microbatches is None:  # the engine's default split (Engine.micro_batches_for)
        a.microbatches = 1
    fe = fold(read(os.path.join(a.outdir, "fetch"), "FETCH_SIZE"))
    wr = fold(read(os.path.join(a.outdir, "write"), "WRITE_SIZE"))
    res = {}
    for cls in fe:
        if cls not in wr or not fe[cls]["n"]:
            continue
        n = fe[cls]["n"]
        fetch_b = 2 * fe[cls]["kib"] * 1024 / n
        write_b = wr[cls]["kib"] * 1024 / max(1, wr[cls]["n"])
        res[cls] = {"hbm_bytes_per_launch": int(fetch_b + write_b), "fetch_bytes_per_launch_x2": int(fetch_b),
                    "write_bytes_per_launch": int(write_b), "launches": n}
    key = f"{a.preset}_{a.size}_bs{a.batch}_{a.precision}_mb{a.microbatches}" + ("_mixed" if a.stream == "mixed" else "")
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    allr = json.load(open(path)) if os.path.exists(path) else {}
    allr[key] = {"conv_hbm_bytes_per_launch": res.get("conv", {}).get("hbm_bytes_per_launch"), "classes": res,
                 "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes, --kernel-trace); "
                           "HBM = 2*FETCH_SIZE + WRITE_SIZE (KiB->B), gfx950 correction per MI355X_MICROARCH.md"}
    with open(path, "w") as f:
        json.dump(allr, f, indent=1)
    print(json.dumps({key: allr[key]}))


if __name__ == "__main__":
    sys.exit(main())
