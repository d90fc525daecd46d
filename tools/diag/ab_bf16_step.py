"""A/B on the bf16 configs: bench.py (C3 or C2-bf16) with the decoder's pos-in-epilogue form off / on
(engine.Engine._lin_mode-gated; "off" restores the A2 loader form).  python tools/diag/ab_bf16_step.py off|on c3|c2bf16"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import spotter_amd.engine as eng  # noqa: E402

if sys.argv[1] == "off":
    src = eng.Engine.forward  # the decoder reads self._lin_mode; "off" runs it as if the linears were x3
    orig_init = eng.Engine.__init__

    def init(self, *a, **k):
        orig_init(self, *a, **k)
        self._pos_epi_off = True
    eng.Engine.__init__ = init
args = ["--preset", "r18vd", "--precision", "bf16", "--batch", "256"] if sys.argv[2] == "c3" else ["--precision", "bf16"]
sys.argv = ["bench.py", "--no-cpu-baseline", "--latency-iters", "0"] + args
import bench  # noqa: E402

sys.exit(bench.main())
