"""Sustained MFMA rate on this MI355X (tools/microbench/mfma_peak.hip): what the matrix pipe delivers
at the clock the chip holds under a pure-MFMA load on random operands — the practical ceiling the
GEMM rooflines should be read against (MI355X_MICROARCH.md, 'DVFS give-back').

    python tools/microbench/mfma_peak.py        (builds the .so next to this file with hipcc)
"""
import ctypes
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmfma_peak.so")


def build():
    src = os.path.join(HERE, "mfma_peak.hip")
    if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", SO], check=True)


def main():
    import torch

    build()
    L = ctypes.CDLL(SO)
    dev = torch.device("cuda", 0)
    seed = torch.randn(4096 * 8, device=dev).to(torch.bfloat16).view(torch.int32)  # random normal bf16 pairs
    out = torch.empty(1 << 22, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    # flops per MFMA, MFMAs per iteration per wave
    modes = {0: ("32x32x16 bf16", 32 * 32 * 16 * 2, 8), 1: ("16x16x32 bf16", 16 * 16 * 32 * 2, 16),
             2: ("32x32x2 f32", 32 * 32 * 2 * 2, 4), 3: ("32x32x16 bf16 x3 chains", 32 * 32 * 16 * 2, 48),
             4: ("32x32x16 bf16 x3 chains + LDS B reads", 32 * 32 * 16 * 2, 48),
             5: ("16x16x32 bf16 x3 chains", 16 * 16 * 32 * 2, 48)}
    for mode, (name, fl, per) in modes.items():
        for threads in (256, 512):
            iters = {0: 4000, 1: 4000, 2: 2000}.get(mode, 700)
            blocks = 256 * (1024 // threads)
            args = (mode, blocks, threads, iters, ctypes.c_void_p(seed.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                    ctypes.c_void_p(st))
            for _ in range(3):
                L.mfma_peak(*args)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                L.mfma_peak(*args)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 10
            waves = blocks * threads // 64
            tf = waves * iters * per * fl / (ms * 1e-3) / 1e12
            res[f"{name} {threads}thr"] = {"ms": round(ms, 3), "tflops": round(tf, 1)}
            print(json.dumps({name: res[f"{name} {threads}thr"], "threads": threads}), flush=True)
    print(json.dumps({"mfma_sustained": res}))


if __name__ == "__main__":
    main()
