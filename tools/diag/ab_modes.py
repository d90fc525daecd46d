"""Same-process-style A/B of the per-layer operand-mode set: runs bench.py (or tools/latency.py) with the round-4
additions to engine._X3_FASTER removed ("old") or kept ("new").  python tools/diag/ab_modes.py old|new bench|latency"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import spotter_amd.engine as eng  # noqa: E402

which, what = sys.argv[1], sys.argv[2]
if which == "old":
    eng._X3_FASTER -= {(64, 256, False), (256, 256, True)}
if what == "bench":
    sys.argv = ["bench.py", "--no-cpu-baseline", "--latency-iters", "0"]
    import bench  # noqa: E402
    sys.exit(bench.main())
sys.argv = ["latency.py", "--iters", "100"]
from tools import latency  # noqa: E402
latency.main()
