"""hipBLASLt yardstick (torch bf16 matmul, no epilogue) on the C3 / C2-bf16 GEMM shapes: short-K 1×1s and the
3×3s as plain GEMMs of the same M × N × K (their im2col FLOPs), next to a torch copy's streaming rate.

    python tools/microbench/hipblaslt_probe.py [--shapes M,N,K ...]
"""
import argparse
import json

import torch

SHAPES = [(2150400, 768, 256), (2150400, 256, 256), (2150400, 80, 256), (1638400, 256, 128), (51200, 1024, 256),
          (51200, 256, 1024), (1638400, 128, 1152), (409600, 256, 2304), (102400, 512, 4608), (6553600, 64, 576),
          (409600, 128, 1152)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=None)
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in s.split(",")) for s in a.shapes] if a.shapes else SHAPES
    dev = "cuda"
    res = {}
    for (M, N, K) in shapes:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = torch.randn(K, N, device=dev).to(torch.bfloat16)
        for _ in range(3):
            C = A @ W
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            C = A @ W
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        byt = (M * K + M * N + K * N) * 2
        res[f"{M}x{N}x{K}"] = {"ms": round(ms, 4), "TBps": round(byt / ms / 1e9, 2), "TF": round(2 * M * N * K / ms / 1e9, 1)}
        print(json.dumps({f"{M}x{N}x{K}": res[f"{M}x{N}x{K}"]}), flush=True)
        del A, W, C
    x = torch.empty(2150400 * 768, dtype=torch.bfloat16, device=dev)
    y = torch.empty_like(x)
    for _ in range(3):
        y.copy_(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        y.copy_(x)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(json.dumps({"copy_TBps": round(2 * x.numel() * 2 / ms / 1e9, 2)}))


if __name__ == "__main__":
    main()
