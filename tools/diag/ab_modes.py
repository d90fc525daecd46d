"""A/B of an engine-level choice: runs bench.py (or tools/latency.py) with engine.DEC_POS_IN_EPILOGUE off ("old")
or on ("new").  python tools/diag/ab_modes.py old|new bench|latency"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import spotter_amd.engine as eng  # noqa: E402

which, what = sys.argv[1], sys.argv[2]
eng.DEC_POS_IN_EPILOGUE = which == "new"
if what == "bench":
    sys.argv = ["bench.py", "--no-cpu-baseline", "--latency-iters", "0"]
    import bench  # noqa: E402
    sys.exit(bench.main())
sys.argv = ["latency.py", "--iters", "100"]
from tools import latency  # noqa: E402
latency.main()
