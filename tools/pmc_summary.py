"""Per-kernel means of every PMC counter found under <outdir> (rocprofv3 --pmc CSVs).

    python tools/pmc_summary.py <outdir> [kernel-name-filter]
"""
import csv
import glob
import json
import os
import re
import sys


def main():
    out = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = {}
    for f in glob.glob(os.path.join(out, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if filt not in name:
                    continue
                short = re.sub(r"\(anonymous namespace\)::|sp::", "", name).split("(")[0]
                short = short.replace("void ", "")
                key = (short, r["Counter_Name"])
                a = agg.setdefault(key, [0.0, 0])
                a[0] += float(r["Counter_Value"])
                a[1] += 1
    table = {}
    for (k, c), (s, n) in agg.items():
        table.setdefault(k, {})[c] = round(s / n, 1)
    for k, v in table.items():
        print(json.dumps({"kernel": k, **v}))


if __name__ == "__main__":
    main()
