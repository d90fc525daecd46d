"""What one deployed MI355X serves: k Serve-replica processes sharing one GPU, each running the whole /detect
request loop of tools/detect_path.py (HTTP fetch from a local server → GPU JPEG decode → processor → model →
post-process → labels → draw → GPU JPEG encode → base64 → response JSON), back to back, for a fixed window.

The unchanged deployment class runs one image at a time on its event loop (reference serve.py:99-100,
179-181), so a replica serves at most one request per whole-request latency; more throughput per GPU needs
more replicas per GPU (Ray Serve `num_replicas` with fractional `ray_actor_options.num_gpus`). This measures
that trade: aggregate images/s and p50 / p95 whole-request latency for k = 1, 2, 4 ... processes on one GPU,
per precision (fp32 = the parity path, bf16 = C4).

    python tools/served_sweep.py --k 1 2 4 --precision fp32 bf16 --seconds 10 --out profiles/r6/served

Each worker process is started before any GPU call of the parent (the parent never touches the GPU), builds
its model, warms up (graph capture, decoder buffers), reports ready on stdout and waits for a common start
time on stdin; all workers then run requests until the common end time. Aggregate img/s = all requests
completed inside the window / the window.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def stub_worker(ms: float):
    """CPU test stand-in for worker(): the same READY / start / RESULT protocol, a request is a sleep of `ms`."""
    print("READY", flush=True)
    t_start, t_end = (float(v) for v in sys.stdin.readline().split())
    while time.time() < t_start:
        time.sleep(0.0005)
    lat = []
    while time.time() < t_end:
        t0 = time.time()
        time.sleep(ms / 1e3)
        if time.time() <= t_end:
            lat.append((time.time() - t0) * 1e3)
    print("RESULT " + json.dumps({"pid": os.getpid(), "requests": len(lat), "lat_ms": [round(x, 3) for x in lat]}),
          flush=True)


def worker(preset: str, precision: str, warmup: int):
    import asyncio

    import httpx
    import numpy as np
    import torch

    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.config import PRESETS
    from tools.detect_path import handle, opener, serve_bytes

    with open(os.path.join(ROOT, "tests", "golden", "test_pic.jpg"), "rb") as f:
        jpeg = f.read()
    srv, url = serve_bytes(jpeg)
    model = SpotterForObjectDetection(PRESETS[preset], use_graphs=True, precision=precision)
    proc = SpotterImageProcessor()
    body = json.dumps({"image_urls": [url]}).encode()
    open_fn = opener("gpu")
    rng = np.random.default_rng(os.getpid())

    async def run():
        lat = []
        async with httpx.AsyncClient() as client:
            for _ in range(warmup):
                await handle(body, client, proc, model, {}, open_fn, rng)
            torch.cuda.synchronize()
            print("READY", flush=True)
            t_start, t_end = (float(v) for v in sys.stdin.readline().split())
            while time.time() < t_start:
                await asyncio.sleep(0.0005)
            while True:
                t0 = time.time()
                if t0 >= t_end:
                    break
                await handle(body, client, proc, model, {}, open_fn, rng)
                t1 = time.time()
                if t1 <= t_end:  # only requests completed inside the window count
                    lat.append((t1 - t0) * 1e3)
        return lat

    try:
        lat = asyncio.run(run())
    finally:
        srv.shutdown()
    print("RESULT " + json.dumps({"pid": os.getpid(), "requests": len(lat), "lat_ms": [round(x, 3) for x in lat]}),
          flush=True)


def sweep_point(k: int, precision: str, preset: str, seconds: float, warmup: int, timeout: float,
                stub_ms: float | None = None):
    import numpy as np

    env = dict(os.environ)
    extra = ["--stub-ms", str(stub_ms)] if stub_ms is not None else []
    procs = [subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), "--worker", "--preset", preset,
                               "--precision", precision,
                               "--warmup", str(warmup), *extra],
                              stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True, env=env, cwd=ROOT)
             for _ in range(k)]
    try:
        deadline = time.time() + timeout
        for p in procs:  # every worker built its model and warmed up
            while True:
                line = p.stdout.readline()
                if not line:
                    raise RuntimeError(f"worker {p.pid} exited before READY (rc {p.wait()})")
                if line.startswith("READY"):
                    break
                if time.time() > deadline:
                    raise RuntimeError("workers not ready in time")
        t_start = time.time() + 0.5
        t_end = t_start + seconds
        for p in procs:
            p.stdin.write(f"{t_start} {t_end}\n")
            p.stdin.flush()
        res = []
        for p in procs:
            out, _ = p.communicate(timeout=seconds + timeout)
            line = next((l for l in out.splitlines() if l.startswith("RESULT ")), None)
            if p.returncode != 0 or line is None:
                raise RuntimeError(f"worker {p.pid} failed (rc {p.returncode})")
            res.append(json.loads(line[len("RESULT "):]))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    lat = np.array([x for r in res for x in r["lat_ms"]])
    n = int(lat.size)
    return {"k_processes": k, "precision": precision, "preset": preset, "window_s": seconds,
            "requests": n, "img_per_s": round(n / seconds, 1),
            "per_process_img_per_s": [round(r["requests"] / seconds, 1) for r in res],
            "p50_ms": round(float(np.percentile(lat, 50)), 3) if n else None,
            "p95_ms": round(float(np.percentile(lat, 95)), 3) if n else None,
            "p99_ms": round(float(np.percentile(lat, 99)), 3) if n else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--k", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--precision", nargs="+", default=["fp32", "bf16"])
    ap.add_argument("--preset", default="r101vd")
    ap.add_argument("--seconds", type=float, default=10.0)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--timeout", type=float, default=240.0, help="per sweep point: workers ready / finished")
    ap.add_argument("--out", default=None, help="directory for one JSON per precision")
    ap.add_argument("--stub-ms", type=float, default=None, help=argparse.SUPPRESS)  # CPU test: no GPU worker
    a = ap.parse_args()
    if a.worker:
        if a.stub_ms is not None:
            return stub_worker(a.stub_ms)
        return worker(a.preset, a.precision[0], a.warmup)
    if max(a.k) > 12:
        raise SystemExit("at most 12 processes per GPU (the box allows 16 GPU processes in all)")
    for prec in a.precision:
        pts = []
        for k in a.k:
            r = sweep_point(k, prec, a.preset, a.seconds, a.warmup, a.timeout)
            print(json.dumps(r), flush=True)
            pts.append(r)
        best = max(pts, key=lambda r: r["img_per_s"])
        doc = {"what": "whole /detect request loop (tools/detect_path.py) in k processes sharing one MI355X, "
                       "1200x717 JPEG fixture, bs1 per request as the unchanged serve.py runs it",
               "precision": prec, "preset": a.preset, "points": pts,
               "best_k": best["k_processes"], "best_img_per_s": best["img_per_s"]}
        if a.out:
            os.makedirs(a.out, exist_ok=True)
            with open(os.path.join(a.out, f"served_{a.preset}_{prec}.json"), "w") as f:
                json.dump(doc, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
