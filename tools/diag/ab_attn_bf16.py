"""A/B of the bf16 variant's attention core: bench.py (C3 or C2-bf16) with engine.ATTN_BF16 off / on.
    python tools/diag/ab_attn_bf16.py off|on c3|c2bf16"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import spotter_amd.engine as eng  # noqa: E402

eng.ATTN_BF16 = sys.argv[1] == "on"
args = ["--preset", "r18vd", "--precision", "bf16", "--batch", "256"] if sys.argv[2] == "c3" else ["--precision", "bf16"]
sys.argv = ["bench.py", "--no-cpu-baseline", "--latency-iters", "0"] + args
import bench  # noqa: E402

sys.exit(bench.main())
