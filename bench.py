"""Throughput bench: RT-DETRv2-R101vd, 640², batch 32 per GPU, images/sec (BASELINE.json).

A step = one pass of the /detect hot path over one batch of synthetic uint8
images already resident in HBM: fused preprocess (sp_preprocess_u8) → full
RT-DETRv2 forward → post_process_object_detection (sp_postprocess). Scaling
is one process per GPU with no data-path collective (replicas, "weak"); a
gloo process group only provides the barrier and the max-over-ranks time.

    python bench.py [--gpus N --steps K --warmup W --batch 32 --preset r101vd --size 640]

Prints ONE JSON line (rank 0) with the contract fields plus `roofline` (the
dominant kernel: the fp32 MFMA implicit-GEMM conv, HIP-event timed inside the
timed region) and `cpu_baseline` (the reference HF path on the host CPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_32x32x2_f32 / 16x16x4
BF16_MFMA_PEAK_TFLOPS = 2500.0  # dense bf16 (v_mfma_f32_32x32x16_bf16), not the 2:1-sparse figure
HBM_PEAK_GBS = 8000.0
BASELINE_METRIC = "images/sec RT-DETRv2-R101 640\u00b2 bs32 at 1/2/4/8 MI355X; p50 /detect latency"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--size", type=int, default=640)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true", help="skip per-kernel HIP events")
    ap.add_argument("--latency-iters", type=int, default=100,
                    help="bs1 /detect core requests for the p50 latency half of the metric (0 = skip)")
    ap.add_argument("--detail", default=None, help="write per-conv-shape timings (JSON) here")
    ap.add_argument("--stagger", type=int, default=1, help="block offset between micro-batch streams")
    ap.add_argument("--precision", default="fp32", choices=["fp32", "fp32-mfma", "bf16", "bf16-all"],
                    help="GEMM operand precision: fp32 = fp32-accurate 3-way bf16 split GEMMs (SP_PREC_F32X3), "
                         "fp32-mfma = v_mfma_f32_32x32x2_f32 GEMMs; bf16 = the separately reported variant (C3/C4)")
    ap.add_argument("--microbatches", type=int, default=1,
                    help="concurrent per-GPU batch slices on separate streams (2 overlaps GEMM tails, "
                         "but then per-launch durations overlap)")
    return ap.parse_args()


# kernel class -> (bound, peak, unit); peaks from MI355X_MICROARCH.md (dense, no sparsity)
CLASS_BOUND = {
    "conv": ("mfma", None, "TFLOP/s"),  # fp32 or bf16 MFMA peak by --precision
    "attention": ("mfma", 157.3, "TFLOP/s"),  # flash-style attention on v_mfma_f32_16x16x4_f32 (fp32 peak)
    "msda": ("hbm", HBM_PEAK_GBS, "GB/s"),
    "preprocess": ("hbm", HBM_PEAK_GBS, "GB/s"),
    "topk": ("hbm", HBM_PEAK_GBS, "GB/s"),
    "postprocess": ("hbm", HBM_PEAK_GBS, "GB/s"),
    "layernorm": ("hbm", HBM_PEAK_GBS, "GB/s"),
    "elementwise": ("hbm", HBM_PEAK_GBS, "GB/s"),
}


def union_ms(ivs):
    union, cur_a, cur_b = 0.0, None, None
    for a, b in sorted(ivs):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                union += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        union += cur_b - cur_a
    return union


class KernelEventRecorder:
    """HIP events around every kernel launch, recorded on the launch's own stream (the
    engine makes each micro-batch stream torch's current stream before launching)."""

    def __init__(self, torch):
        self.torch = torch
        self.recs = []
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t0.record()

    def __call__(self, kind, launch, flops, nbytes, shape=None):
        t = self.torch
        e0 = t.cuda.Event(enable_timing=True)
        e1 = t.cuda.Event(enable_timing=True)
        e0.record()
        launch()
        e1.record()
        self.recs.append((kind, e0, e1, flops, nbytes, shape))

    def by_shape(self, kind="conv"):
        agg = {}
        for k, e0, e1, f, nb, shp in self.recs:
            if k != kind:
                continue
            a = agg.setdefault(str(shp), [0, 0.0, 0])
            a[0] += 1
            a[1] += e0.elapsed_time(e1)
            a[2] += f
        rows = [{"shape": k, "launches": v[0], "ms": round(v[1], 3),
                 "tflops": round(v[2] / (v[1] * 1e-3) / 1e12, 1)} for k, v in agg.items()]
        return sorted(rows, key=lambda r: -r["ms"])

    def conv_modes(self):
        """GEMM operand mode (shape[5]: f32 / bf16 / x3) -> dict(flops, ms = summed launch durations, n)."""
        out = {}
        for k, e0, e1, f, nb, shp in self.recs:
            if k != "conv" or not shp or len(shp) < 6:
                continue
            c = out.setdefault(shp[5], {"flops": 0, "ms": 0.0, "n": 0})
            c["flops"] += f
            c["ms"] += e0.elapsed_time(e1)
            c["n"] += 1
        return out

    def classes(self):
        """kind -> dict(ms = sum of launch durations, busy = union of launch intervals, flops, bytes, n)."""
        out = {}
        for k, e0, e1, f, nb, _ in self.recs:
            c = out.setdefault(k, {"ms": 0.0, "ivs": [], "flops": 0, "bytes": 0, "n": 0})
            a, b = self.t0.elapsed_time(e0), self.t0.elapsed_time(e1)
            c["ms"] += b - a
            c["ivs"].append((a, b))
            c["flops"] += f
            c["bytes"] += nb
            c["n"] += 1
        for c in out.values():
            c["busy"] = union_ms(c.pop("ivs"))
        return out


def load_traffic(args, avg_alg_bytes):
    """HBM bytes per conv launch from the committed PMC passes (tools/pmc_bench.py), if they were
    collected on this exact configuration; null otherwise."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    key = f"{args.preset}_{args.size}_bs{args.batch}_{args.precision}_mb{args.microbatches}"
    e = t.get(key)
    if not e:
        return None, None
    return e["conv_hbm_bytes_per_launch"], {"source": f"profiles/pmc_traffic.json[{key}]",
                                            "ratio_to_algorithmic": round(e["conv_hbm_bytes_per_launch"]
                                                                          / avg_alg_bytes, 3)}


def cpu_baseline(cfg, weights, seconds):
    """Reference CPU path (HF RTDetrImageProcessorPil → RTDetrV2ForObjectDetection fp32 →
    post_process_object_detection), bs=1 as /detect runs it (serve.py:96-109), on the host cores."""
    import numpy as np
    import torch
    from PIL import Image

    from oracle.hf_ref import build_hf_model, build_hf_processor
    from spotter_amd.synthetic import synthetic_image

    ncores = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    ncores = int(os.environ.get("OMP_NUM_THREADS", ncores))
    torch.set_num_threads(ncores)
    model = build_hf_model(cfg, weights)
    proc = build_hf_processor()
    imgs = [Image.fromarray(synthetic_image(500 + i, cfg.image_size, cfg.image_size)) for i in range(4)]

    def one(im):
        inp = proc(images=im, return_tensors="pt")
        with torch.no_grad():
            out = model(**inp)
        proc.post_process_object_detection(out, target_sizes=torch.tensor([[im.size[1], im.size[0]]]),
                                           threshold=0.5)

    one(imgs[0])  # warmup
    n = 0
    t0 = time.perf_counter()
    while True:
        one(imgs[n % len(imgs)])
        n += 1
        if time.perf_counter() - t0 >= seconds and n >= 3:
            break
    dt = time.perf_counter() - t0
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    return {"value": n / dt, "unit": "images/sec", "cores": torch.get_num_threads(), "kind": "reference",
            "cpu_model": cpu_model,
            "sample": f"{n} images bs=1 {cfg.image_size}x{cfg.image_size} through HF transformers "
                      f"RTDetrImageProcessorPil+RTDetrV2ForObjectDetection(fp32, synthetic {cfg.name} weights)"
                      f"+post_process_object_detection on {torch.get_num_threads()} host threads, {dt:.1f}s"}


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from spotter_amd import ops
    from spotter_amd.config import PRESETS
    from spotter_amd.engine import Engine
    from spotter_amd.synthetic import synthetic_batch
    from spotter_amd.replicas import barrier, max_over_ranks
    from spotter_amd.weights import generate

    cfg = PRESETS[args.preset].replace(image_size=args.size)
    weights = generate(cfg, seed=0)
    eng = Engine(cfg, weights, dev, precision=args.precision)
    eng.microbatches = args.microbatches
    eng.stagger = args.stagger
    B, S = args.batch, args.size
    imgs_host = synthetic_batch(B, S, S, seed0=1234 + 1000 * rank)
    imgs = [torch.from_numpy(im).to(dev) for im in imgs_host]  # resident in HBM
    px = torch.empty((B, 3, S, S), dtype=torch.float32, device=dev)
    K = cfg.num_queries
    tsz = torch.tensor([[S, S]] * B, dtype=torch.int32, device=dev)
    scores = torch.empty((B, K), device=dev)
    labels = torch.empty((B, K), dtype=torch.int64, device=dev)
    boxes = torch.empty((B, K, 4), device=dev)
    counts = torch.empty((B,), dtype=torch.int32, device=dev)
    work = torch.empty((B, K), dtype=torch.int32, device=dev)

    def step():
        ops.preprocess_u8(imgs, px, S, S)
        logits, pred = eng.forward(px)
        ops.postprocess(logits, pred, tsz, K, 0.5, scores, labels, boxes, counts, work)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    rec = None if args.no_events else KernelEventRecorder(torch)
    ops.set_launch_hook(rec)

    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    ops.set_launch_hook(None)
    elapsed = t1 - t0
    elapsed = max_over_ranks(elapsed)
    n_img = world * B * args.steps
    value = n_img / elapsed

    roof, classes = None, None
    if rec is not None and rec.recs:
        cl = rec.classes()
        bf = args.precision.startswith("bf16")
        conv_peak = BF16_MFMA_PEAK_TFLOPS if bf else FP32_MFMA_PEAK_TFLOPS
        classes = {}
        for kind, c in sorted(cl.items(), key=lambda kv: -kv[1]["ms"]):
            bound, peak, unit = CLASS_BOUND[kind]
            peak = peak or conv_peak
            # concurrent micro-batch streams overlap launches of one class: use the busy-time union
            work = c["bytes"] / 1e9 if unit == "GB/s" else c["flops"] / 1e12
            ach = work / (c["busy"] * 1e-3)
            classes[kind] = {"bound": bound, "achieved": round(ach, 2), "peak": peak, "unit": unit,
                             "frac": round(ach / peak, 4), "ms_per_step": round(c["busy"] / args.steps, 3),
                             "launches_per_step": c["n"] // args.steps}
        c = cl["conv"]
        per_launch_ms = c["ms"] / c["n"]
        ach = c["flops"] / (c["busy"] * 1e-3) / 1e12
        alg_bytes = c["bytes"] / c["n"]
        traffic, tnote = load_traffic(args, alg_bytes)
        if args.precision == "fp32-mfma":
            kname = "conv_gemm_kernel (fp32 v_mfma_f32_32x32x2f32 implicit GEMM)"
        elif bf:
            kname = ("conv_glds_kernel<PL=1> (bf16 operands, v_mfma_f32_32x32x16_bf16 implicit GEMM, LDS-DMA staged; "
                     + ("decoder linears f32x3)" if args.precision == "bf16" else "decoder linears bf16)"))
        else:
            kname = ("conv_glds_kernel<PL=3> (fp32 operands split hi/mid/lo bf16, 6 v_mfma_f32_32x32x16_bf16 "
                     "per 32x32x16 block, implicit GEMM, LDS-DMA staged) + conv_gemm_kernel (fp32 "
                     "v_mfma_f32_32x32x2f32) on thin layers and decoder linears; split in 'modes'")
        roof = {"bound": "mfma", "kernel": kname,
                "achieved": round(ach, 2), "peak": conv_peak, "unit": "TFLOP/s",
                "frac": round(ach / conv_peak, 4), "traffic": traffic,
                "launches_per_step": c["n"] // args.steps, "avg_launch_ms": round(per_launch_ms, 4),
                "gflop_per_launch": round(c["flops"] / c["n"] / 1e9, 3),
                "algorithmic_bytes_per_launch": int(alg_bytes),
                "gflop_per_step": round(c["flops"] / args.steps / 1e9, 2),
                "conv_busy_ms_per_step": round(c["busy"] / args.steps, 3),
                "note": "achieved = algorithmic conv/linear FLOPs / wall time with >=1 conv_gemm launch in flight "
                        "(HIP events on the launch streams); traffic = HBM bytes per conv launch from PMC "
                        "FETCH_SIZE x2 + WRITE_SIZE (MI355X_MICROARCH.md gfx950 correction)"}
        if tnote:
            roof["traffic_source"] = tnote
        # per operand mode: share of the class's FLOPs and time, and the matrix pipe's own instruction rate
        # (the fp32-accurate split issues 6 bf16 MFMAs per fp32 32x32x16 product block)
        modes = {}
        per_mfma = {"x3": (6, "v_mfma_f32_32x32x16_bf16", BF16_MFMA_PEAK_TFLOPS),
                    "bf16": (1, "v_mfma_f32_32x32x16_bf16", BF16_MFMA_PEAK_TFLOPS),
                    "f32": (1, "v_mfma_f32_32x32x2_f32", FP32_MFMA_PEAK_TFLOPS),
                    "direct": (1, "v_fma_f32 (VALU stem conv, no MFMA)", FP32_MFMA_PEAK_TFLOPS)}
        for md, c in rec.conv_modes().items():
            a = c["flops"] / (c["ms"] * 1e-3) / 1e12
            mult, instr, pk = per_mfma[md]
            modes[md] = {"flop_share": round(c["flops"] / max(1, cl["conv"]["flops"]), 4),
                         "ms_per_step": round(c["ms"] / args.steps, 3), "launches_per_step": c["n"] // args.steps,
                         "achieved": round(a, 2), "unit": "TFLOP/s",
                         "mfma_issue": {"instr": instr, "mfma_per_fp32_block": mult,
                                        "achieved": round(mult * a, 1), "peak": pk, "frac": round(mult * a / pk, 4)}}
        roof["modes"] = modes

    if rec is not None and args.detail and rank == 0:
        with open(args.detail, "w") as f:
            json.dump(rec.by_shape(), f, indent=1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(cfg, weights, args.cpu_baseline_seconds)
        except Exception as e:  # keep the GPU line even if the host path is unavailable
            cpu = {"value": None, "unit": "images/sec", "cores": None, "kind": "reference",
                   "sample": f"unavailable: {type(e).__name__}: {e}"}

    lat = None
    if rank == 0 and world == 1 and args.latency_iters > 0:
        try:
            from tools.latency import measure

            lat = measure(args.preset, args.latency_iters, graphs=True)
        except Exception as e:
            lat = {"error": f"{type(e).__name__}: {e}"}

    if rank == 0:
        line = {
            "metric": (BASELINE_METRIC if (args.preset, S, B, args.precision) == ("r101vd", 640, 32, "fp32")
                       else f"images/sec RT-DETRv2-{args.preset} {S}² bs{B} {args.precision}"),
            "value": round(value, 2), "unit": "images/sec", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.precision,
            "data": "synthetic uint8 RGB images (seeded), synthetic deterministic weights",
            "config": {"workload": f"RT-DETRv2-{args.preset} {S}x{S} batch={B}/GPU preprocess+forward+postprocess",
                       "model": f"rtdetr_v2_{args.preset}", "global_batch": B * world, "image_size": S,
                       "parallelism": f"replicas x{world}"},
            "roofline": roof, "kernel_classes": classes, "cpu_baseline": cpu, "latency": lat,
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
