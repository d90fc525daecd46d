"""Random row-segment gather ceiling for MSDA's access pattern on this MI355X (gather_ceiling.hip).

    python tools/microbench/gather_ceiling.py [--out profiles/r6/msda/gather_ceiling.json]

Cases: the C2 / C3-style 640^2 maps (levels 80^2, 40^2, 20^2; S = 8400) and the C5 1280^2 maps, value rows
fp32 (16-byte loads per lane, 128-byte segments per head) or bf16 (8-byte loads, 64-byte segments), in the
engine's layout (value_all: one 256-column slice of 6*256-wide rows, ld 1536) and a compact ld 256 layout;
NPT = sampling points whose corners are in flight together (1 / 4 / 12). Gathered bytes are counted as msda's
`l2_gather` counts them (4 corners x 32 channels x element size per head-sample), so bench.py's
kernel_classes.msda.l2_gather.achieved divides by `ceiling_gbps` directly.
"""
import argparse
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libgather_ceiling.so")


def build():
    src = os.path.join(HERE, "gather_ceiling.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", SO],
                       check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    build()
    L = ctypes.CDLL(SO)
    L.gather_ceiling.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L.stream_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream().cuda_stream
    Q = 300
    res = []

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.reps

    # (scale, B, bf16, ld): the bench configs' value_all layouts (C2 / C2-bf16: 6 decoder layers, ld 1536; C3 R18:
    # 3 layers, ld 768; C5: 1280², bs8) and a compact ld-256 layout beside each
    cases = [(1, 32, 0, 1536), (1, 32, 0, 256), (1, 32, 1, 1536), (1, 32, 1, 256), (1, 256, 1, 768),
             (1, 256, 1, 256), (1, 256, 0, 768), (2, 8, 0, 1536), (2, 8, 0, 256), (2, 8, 1, 1536)]
    for scale, B, bf16, ld in cases:
        S = 8400 * scale * scale
        esz = 2 if bf16 else 4
        n = B * S * ld
        val = torch.randn(n, device=dev)
        if bf16:
            val = val.to(torch.bfloat16).view(torch.int16)
        out = torch.empty(B * Q, device=dev)
        gathered = B * Q * 8 * 12 * 4 * 32 * esz
        for npt in (1, 4, 12):
            args = (bf16, npt, val.data_ptr(), ld, S, Q, B, scale, out.data_ptr(), st)
            assert L.gather_ceiling(*args) == 0
            ms = timed(lambda: L.gather_ceiling(*args))
            r = {"map": f"{80 * scale}^2+{40 * scale}^2+{20 * scale}^2", "B": B, "dtype": "bf16" if bf16 else "fp32",
                 "ld": ld, "npt": npt, "slice_MB": round(B * S * 256 * esz / 1e6, 1), "ms": round(ms, 4),
                 "gathered_MB": round(gathered / 1e6, 1), "gather_gbps": round(gathered / ms / 1e6, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
        del val
        torch.cuda.empty_cache()
    # dense streaming read of a 275 MB / 1.1 GB buffer for comparison
    dense = []
    for mb in (275, 1100):
        buf = torch.empty(mb * 1000000 // 4, device=dev)
        buf.normal_()
        out = torch.empty(1, device=dev)
        ms = timed(lambda: L.stream_read(buf.data_ptr(), buf.numel() * 4, out.data_ptr(), st))
        dense.append({"MB": mb, "ms": round(ms, 4), "gbps": round(buf.numel() * 4 / ms / 1e6, 1)})
        print(json.dumps(dense[-1]), flush=True)
        del buf
    ceil = {}
    for r in res:
        key = f"{r['dtype']} {r['map']} B{r['B']} ld{r['ld']}"
        if key not in ceil or r["gather_gbps"] > ceil[key]["gather_gbps"]:
            ceil[key] = {"gather_gbps": r["gather_gbps"], "npt": r["npt"]}
    doc = {"what": "random 128-byte (fp32) / 64-byte (bf16) row-segment gathers in msda_vec_kernel's address "
                   "pattern (one wave per query, 8 heads x 12 points x 4 corners, XCD-major grid)",
           "cases": res, "ceiling_by_case": ceil, "dense_stream": dense}
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)
    print(json.dumps({"ceiling_by_case": ceil}))


if __name__ == "__main__":
    main()
