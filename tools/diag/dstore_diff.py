"""Where does the direct-store epilogue (variant 4) differ from the slab store pass? Mismatch map per case."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from spotter_amd import ops
from spotter_amd.ops import V

dev = torch.device("cuda", 0)
rng = np.random.default_rng(0)
for cfg in ("12", "46"):
    for rows, K, N, res in ((1000, 256, 192, True), (1024, 256, 256, True), (1024, 256, 256, False),
                            (1000, 256, 256, True), (1024, 256, 192, True)):
        x = torch.from_numpy(rng.standard_normal(rows * K).astype(np.float32)).to(dev)
        wt = torch.from_numpy((rng.standard_normal((N, K)) / np.sqrt(K)).astype(np.float32)).to(dev)
        kw = dict(scale=torch.ones(N, device=dev), shift=torch.zeros(N, device=dev), act=None,
                  wt_planes=ops.split_bf16x3(wt))
        if res:
            kw["res1"] = V(torch.from_numpy(rng.standard_normal(rows * N).astype(np.float32)).to(dev), 0, N)
        outs = []
        for mode in (None, 4):
            ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, mode)
            ops.force_conv_config(cfg)
            o = torch.full((rows * N,), 7.0, device=dev)
            ops.conv2d(V(x, 0, K), 1, 1, rows, K, wt, N, 1, 1, 0, V(o, 0, N), **kw)
            ops.force_conv_config(None)
            ops.set_tuning(ops.TUNE_GLDS_EPILOGUE, None)
            outs.append(o.view(rows, N).cpu().numpy())
        bad = np.argwhere(outs[0] != outs[1])
        e = {"cfg": cfg, "rows": rows, "K": K, "N": N, "res": res, "mismatches": int(len(bad))}
        if len(bad):
            e.update(rmin=int(bad[:, 0].min()), rmax=int(bad[:, 0].max()), cmin=int(bad[:, 1].min()),
                     cmax=int(bad[:, 1].max()), first=bad[:5].tolist(),
                     unwritten=int((outs[1] == 7.0).sum()), rows_bad=sorted(set((bad[:, 0] // 32).tolist()))[:20])
        print(json.dumps(e), flush=True)
