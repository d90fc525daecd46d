#!/bin/bash
# quick GPU check of the current tree: the headline-config parity tests + a bench line (no CPU/latency legs)
set -euo pipefail
OUT=gpurun_out/${1:-quick}
mkdir -p "$OUT"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_model.py -x -q -k "${2:-bs32 or r101vd_matches}" --timeout 200 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -1 "$OUT/tests.log"
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --latency-iters 0 ${3:-} > "$OUT/bench.log" 2>&1
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['achieved'], r['frac'], r.get('conv_class'))"
