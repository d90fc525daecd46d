"""p50 / p95 of the WHOLE /detect request on one replica, end to end:

    request JSON → URL validation → HTTP fetch (local server) → JPEG decode (GPU, the drop-in's open_image;
    --decode host: Pillow as the reference) → processor → model
    → post_process → id2label + amenity filter → draw boxes/labels → JPEG re-encode → base64
    → response JSON

This restates, for timing, the per-request flow of the reference deployment
(apps/spotter/src/spotter/serve.py:74-77 fetch, :96-117 decode → processor → model →
post-process → labels, :119-142 draw + JPEG + base64, :179-196 request parse and response),
driving the drop-in processor / model. The reference class itself cannot be imported on the
GPU box (ray, tenacity and /root/reference are absent there); tests/test_dropin_reference.py
runs the real class in the build container. The fetch goes over real HTTP (httpx, as
serve.py:74-77) to a local threaded server holding the test fixture JPEG
(tests/golden/test_pic.jpg, 1200×717), so only the network distance is missing.

    python tools/detect_path.py [--iters 200] [--preset r101vd]
"""
from __future__ import annotations

import argparse
import asyncio
import base64
import http.server
import io
import json
import os
import socketserver
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# COCO label → amenity (data of reference serve.py:31-59; the keys are HF COCO names)
AMENITIES = {
    "refrigerator": "refrigerator", "oven": "oven", "microwave": "microwave", "sink": "sink",
    "dining table": "dining area", "toaster": "toaster", "wine glass": "kitchen", "cup": "kitchen",
    "fork": "kitchen", "knife": "kitchen", "spoon": "kitchen", "bowl": "kitchen", "tv": "TV",
    "couch": "sofa", "chair": "chair", "bed": "bed", "toilet": "bathroom", "hair drier": "hair dryer",
    "laptop": "workspace", "mouse": "workspace", "keyboard": "workspace", "car": "parking",
}


class _Quiet(http.server.SimpleHTTPRequestHandler):
    payload = b""

    def do_GET(self):  # noqa: N802
        self.send_response(200)
        self.send_header("Content-Type", "image/jpeg")
        self.send_header("Content-Length", str(len(self.payload)))
        self.end_headers()
        self.wfile.write(self.payload)

    def log_message(self, *a):
        pass


def serve_bytes(payload: bytes):
    handler = type("H", (_Quiet,), {"payload": payload})
    srv = socketserver.ThreadingTCPServer(("127.0.0.1", 0), handler)
    srv.daemon_threads = True
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    return srv, f"http://127.0.0.1:{srv.server_address[1]}/test_pic.jpg"


def opener(decode: str):
    """(serve.py:96's `Image.open(BytesIO(image_bytes))`, serve.py:119's `ImageDraw`): the drop-in's module-scope
    `Image` (spotter_amd.jpeg.image_module(): GPU JPEG decode, and GPU JPEG encode in the later save) and
    `ImageDraw` (spotter_amd.draw.draw_module()); or, with decode="host", the reference's own
    PIL modules (host decode, Pillow draw and encode)."""
    if decode == "gpu":
        from spotter_amd.draw import draw_module
        from spotter_amd.jpeg import image_module

        Image, ImageDraw = image_module(), draw_module()
    else:
        from PIL import Image, ImageDraw
    return (lambda data: Image.open(io.BytesIO(data))), ImageDraw


async def process_image(client, url, proc, model, stamps, open_fn=None, jitter=None):
    """One image of a /detect request (serve.py:79-148 order), with per-stage time stamps. jitter (a numpy
    Generator): shift every box by one random sub-pixel offset per image before drawing, so a benchmark that
    repeats one image draws at varied fractional positions like varied traffic does."""
    import torch

    open_fn, ImageDraw = open_fn or opener("gpu")
    t0 = time.perf_counter()
    r = await client.get(url)
    r.raise_for_status()
    t1 = time.perf_counter()
    with open_fn(r.content) as raw:
        image = raw.convert("RGB")
        t2 = time.perf_counter()
        inputs = proc(images=image, return_tensors="pt").to("cpu")
        with torch.no_grad():
            outputs = model(**inputs)
        det = proc.post_process_object_detection(outputs, target_sizes=torch.tensor([[image.size[1], image.size[0]]]),
                                                 threshold=0.5)[0]
        labels = [model.config.id2label[int(l.item())] for l in det["labels"]]
        boxes = det["boxes"].tolist()
        if jitter is not None:
            dx, dy = (float(v) for v in jitter.random(2))
            boxes = [[b[0] + dx, b[1] + dy, b[2] + dx, b[3] + dy] for b in boxes]
        t3 = time.perf_counter()
        draw = ImageDraw.Draw(image)
        found = []
        for label, box in zip(labels, boxes):
            if label not in AMENITIES:
                continue
            draw.rectangle(box, outline="red", width=3)
            draw.text(xy=(box[0] + 5, box[1] + 5), text=AMENITIES[label], fill="white", stroke_width=1,
                      stroke_fill="black")
            found.append({"label": AMENITIES[label], "box": box})
        t3b = time.perf_counter()
        buf = io.BytesIO()
        image.save(buf, format="JPEG")
        b64 = base64.b64encode(buf.getvalue()).decode("utf-8")
        t4 = time.perf_counter()
    for k, a, b in (("fetch", t0, t1), ("decode", t1, t2), ("detect", t2, t3), ("draw_jpeg_b64", t3, t4),
                    ("draw", t3, t3b), ("jpeg_b64", t3b, t4)):
        stamps.setdefault(k, []).append((b - a) * 1e3)
    stamps.setdefault("n_drawn", []).append(len(found))
    return {"url": url, "detections": found, "labeled_image_base64": b64}


async def handle(body: bytes, client, proc, model, stamps, open_fn=None, jitter=None):
    """serve.py:179-196: parse the request, process its images, build the response JSON."""
    from pydantic import BaseModel, HttpUrl

    class DetectionRequest(BaseModel):  # the request contract of reference schemas.py:6-7
        image_urls: list[HttpUrl]

    req = DetectionRequest.model_validate(json.loads(body))
    results = await asyncio.gather(*[process_image(client, str(u), proc, model, stamps, open_fn, jitter)
                                     for u in req.image_urls])
    found = sorted({d["label"] for r in results for d in r["detections"]})
    desc = f"The property contains: {', '.join(found)}." if found else "No relevant amenities detected."
    return json.dumps({"amenities_description": desc, "images": results})


def measure(preset="r101vd", iters=200, model=None, decode="gpu", jitter=False):
    import httpx
    import numpy as np
    import torch

    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.config import PRESETS

    with open(os.path.join(ROOT, "tests", "golden", "test_pic.jpg"), "rb") as f:
        jpeg = f.read()
    srv, url = serve_bytes(jpeg)
    model = model or SpotterForObjectDetection(PRESETS[preset], use_graphs=True)
    proc = SpotterImageProcessor()
    body = json.dumps({"image_urls": [url]}).encode()
    open_fn = opener(decode)
    rng = np.random.default_rng(0) if jitter else None

    async def run():
        stamps, total = {}, []
        async with httpx.AsyncClient() as client:
            for i in range(iters + 5):
                t0 = time.perf_counter()
                await handle(body, client, proc, model, stamps if i >= 5 else {}, open_fn, rng)
                if i >= 5:
                    total.append((time.perf_counter() - t0) * 1e3)
        return stamps, total

    try:
        stamps, total = asyncio.run(run())
    finally:
        srv.shutdown()
    torch.cuda.synchronize()
    total = np.array(total)
    return {"metric": "p50 /detect latency, whole request (HTTP fetch from a local server, JPEG decode, "
                      "preprocess, forward, post-process, labels, draw, JPEG re-encode, base64, response JSON), "
                      "bs1, 1200x717 JPEG",
            "p50_ms": round(float(np.percentile(total, 50)), 3), "p95_ms": round(float(np.percentile(total, 95)), 3),
            "iters": iters, "preset": preset, "decode": decode, "box_jitter": bool(jitter),
            "stages_p50_ms": {k: round(float(np.percentile(v, 50)), 3) for k, v in stamps.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--decode", default="gpu", choices=["gpu", "host"])
    ap.add_argument("--jitter", action="store_true", help="draw each request's boxes at a random sub-pixel offset")
    a = ap.parse_args()
    print(json.dumps(measure(a.preset, a.iters, decode=a.decode, jitter=a.jitter)))


if __name__ == "__main__":
    main()
