"""Print a conv_bench sweep (JSONL) as shape -> [(cfg, TFLOP/s)] rows."""
import json
import sys

rows = {}
for l in open(sys.argv[1]):
    try:
        d = json.loads(l)
    except ValueError:
        continue
    if "shape" in d:
        rows.setdefault(tuple(d["shape"]), []).append((d["cfg"], d.get("tflops", d.get("skipped", "")[:40])))
for s, v in rows.items():
    print(s, v)
