"""p50/p95 latency of the /detect core at batch 1 (serve.py:96-117 minus HTTP/draw/JPEG):
JPEG decode (GPU by default, as the drop-in's open_image; --decode host: Pillow) → processor → model →
post_process → labels/boxes on the host.

    python tools/latency.py [--iters 200] [--no-graph]
"""
import argparse
import io
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from PIL import Image

from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
from spotter_amd.config import PRESETS


def measure(preset="r101vd", iters=200, graphs=True, model=None, decode="gpu"):
    """p50/p95 of the bs1 /detect core on the test fixture JPEG, plus the GPU-only forward p50. decode: "gpu"
    opens the image with the drop-in's open_image (serve.py:96 as INTEGRATION.md §2 changes it: JPEG decoded
    on the GPU, host pixels fetched lazily), "host" with the reference's Image.open (Pillow on the CPU)."""
    if decode == "gpu":
        from spotter_amd.jpeg import open_image

        def open_fn(b):
            return open_image(b)
    else:
        def open_fn(b):
            return Image.open(io.BytesIO(b))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "tests", "golden", "test_pic.jpg"), "rb") as f:
        jpeg = f.read()
    model = model or SpotterForObjectDetection(PRESETS[preset], use_graphs=graphs)
    proc = SpotterImageProcessor()

    def detect():
        with open_fn(jpeg) as raw:
            image = raw.convert("RGB")
            inputs = proc(images=image, return_tensors="pt").to("cpu")
            with torch.no_grad():
                out = model(**inputs)
            det = proc.post_process_object_detection(out, target_sizes=torch.tensor([[image.size[1], image.size[0]]]),
                                                     threshold=0.5)[0]
            labels = [model.config.id2label[int(l.item())] for l in det["labels"]]
            boxes = det["boxes"].tolist()
        return labels, boxes

    for _ in range(5):
        detect()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        detect()
        ts.append(time.perf_counter() - t0)
    with open_fn(jpeg) as raw:
        x = proc(images=raw.convert("RGB"))["pixel_values"]
    fw = []
    for _ in range(50):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model(pixel_values=x)
        torch.cuda.synchronize()
        fw.append(time.perf_counter() - t0)
    # per-stage p50 (each stage synchronised): where the non-forward part of the p50 goes
    stages = {"decode": [], "processor": [], "model": [], "post_process": []}
    for _ in range(min(iters, 50)):
        t0 = time.perf_counter()
        with open_fn(jpeg) as raw:
            image = raw.convert("RGB")
        t1 = time.perf_counter()
        inputs = proc(images=image, return_tensors="pt").to("cpu")
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        with torch.no_grad():
            out = model(**inputs)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        det = proc.post_process_object_detection(out, target_sizes=torch.tensor([[image.size[1], image.size[0]]]),
                                                 threshold=0.5)[0]
        _ = ([model.config.id2label[int(l.item())] for l in det["labels"]], det["boxes"].tolist())
        t4 = time.perf_counter()
        for k, a, b in (("decode", t0, t1), ("processor", t1, t2), ("model", t2, t3), ("post_process", t3, t4)):
            stages[k].append((b - a) * 1e3)
    ts, fw = np.array(ts) * 1e3, np.array(fw) * 1e3
    return {"metric": "p50 /detect core latency (bs1, 1200x717 JPEG: decode, preprocess, forward, "
                      "post_process, labels/boxes to host)", "graphs": graphs,
            "decode": decode, "p50_ms": round(float(np.percentile(ts, 50)), 3), "p95_ms": round(float(np.percentile(ts, 95)), 3),
            "forward_p50_ms": round(float(np.percentile(fw, 50)), 3), "iters": iters, "preset": preset,
            "stages_p50_ms": {k: round(float(np.percentile(v, 50)), 3) for k, v in stages.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--decode", default="gpu", choices=["gpu", "host"])
    a = ap.parse_args()
    print(json.dumps(measure(a.preset, a.iters, not a.no_graph, decode=a.decode)))


if __name__ == "__main__":
    main()
