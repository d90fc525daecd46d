"""sp_msda at the bench configs' decoder shapes, both kernels for the decoder's shape alternating in one process
(sp_set_tuning(SP_TUNE_MSDA_GENERIC, v): 0 msda_h8l_kernel, the default; 1 msda_vec_kernel): per-launch time,
gathered-corner rate and bit-identity of the outputs against msda_vec_kernel. (Round 6's first measurement also
carried v = 2, the since-removed shuffle-exchange kernel: profiles/r6/msda/msda_ab.json.) Sampling offsets / logits are random (offsets × 2, like a trained decoder's spread).

    python tools/microbench/msda_ab.py [--reps 50] [--out profiles/r6/msda/msda_ab.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np
import torch

from spotter_amd import ops
from spotter_amd._lib import lib
from spotter_amd.ops import V

CASES = {  # name: (B, size, value rows bf16, decoder layers in value_all)
    "c2_fp32_bs32": (32, 640, False, 6),
    "c2_bf16_bs32": (32, 640, True, 6),
    "c3_r18_bf16_bs256": (256, 640, True, 3),
    "c5_fp32_bs8_1280": (8, 1280, False, 6),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    L = lib()
    rng = np.random.default_rng(0)
    res = {}
    for name, (B, size, bf16, layers) in CASES.items():
        Q, nH, dh, nL, nP = 300, 8, 32, 3, 4
        shapes = [(size // 8, size // 8), (size // 16, size // 16), (size // 32, size // 32)]
        starts = [0, shapes[0][0] ** 2, shapes[0][0] ** 2 + shapes[1][0] ** 2]
        S = sum(h * w for h, w in shapes)
        D = nH * dh
        ld = layers * D
        vals = torch.randn(B * S * ld, device=dev)
        value = V(vals.to(torch.bfloat16).view(torch.int16) if bf16 else vals, 0, ld)
        offaw = torch.cat([torch.randn(B * Q, nH * nL * nP * 2, device=dev) * 2.0,
                           torch.randn(B * Q, nH * nL * nP, device=dev)], 1).contiguous()
        ref = torch.cat([torch.rand(B * Q, 2, device=dev) * 0.9 + 0.05, torch.rand(B * Q, 2, device=dev) * 0.4 + 0.02],
                        1).contiguous()
        out = torch.empty(B * Q * D, device=dev)
        gathered = B * Q * nH * nL * nP * 4 * dh * (2 if bf16 else 4)

        def run():
            ops.msda(value, 2 * D, V(offaw.view(-1), 0, offaw.shape[1]), ref, V(out, 0, D), B, S, Q, nH, dh, shapes,
                     starts, nP, 0.5)

        names = {0: "h8l", 1: "vec"}
        times = {g: [] for g in names}
        outs = {}
        for rnd in range(6):
            for g in (1, 0) if rnd % 2 else (0, 1):
                L.sp_set_tuning(4, g)
                for _ in range(3):
                    run()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[g].append(e0.elapsed_time(e1) / a.reps)
                outs[g] = out.clone()
        L.sp_set_tuning(4, 0)
        ms = {g: float(np.median(times[g])) for g in names}
        r = {"B": B, "size": size, "bf16": bf16}
        for g, nm in names.items():
            r[f"ms_{nm}"] = round(ms[g], 4)
            r[f"gather_gbps_{nm}"] = round(gathered / ms[g] / 1e6, 1)
            if g != 1:
                r[f"speedup_{nm}_vs_vec"] = round(ms[1] / ms[g], 3)
                r[f"bit_identical_{nm}"] = bool(torch.equal(outs[g], outs[1]))
                r[f"max_rel_diff_{nm}"] = float((outs[g] - outs[1]).abs().max() / outs[1].abs().max())
        res[name] = r
        print(json.dumps({name: res[name]}), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
