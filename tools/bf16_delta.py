"""bf16 variant vs the fp32 reference outputs (tests/golden): the accuracy delta we can state offline.

COCO-val mAP needs the real checkpoint and COCO images (both unreachable offline: "parity unpinned"),
so the bf16 delta is reported against the HF fp32 goldens on the synthetic-weight model, two ways:

* detection agreement at the serving threshold 0.5: matched detections (same label, IoU >= 0.5),
  recall of the fp32 detections, |Δscore| of matched pairs, extra detections;
* COCO-style AP (tools/coco_ap.py, IoU 0.50:0.95, 101-point) of the bf16 path's ranked candidates
  (post-process threshold 0, the model's own 300 per image, maxDets 300) with the fp32 detections
  above 0.5 taken as ground truth: AP 1.0 means bf16 reproduces fp32's detections exactly.

    python tools/bf16_delta.py [bf16|bf16-all] [--reps 8] [--out profiles/r3/bf16_delta.json]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def iou(a, b):
    x0, y0 = max(a[0], b[0]), max(a[1], b[1])
    x1, y1 = min(a[2], b[2]), min(a[3], b[3])
    inter = max(0.0, x1 - x0) * max(0.0, y1 - y0)
    ua = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / ua if ua > 0 else 0.0


def match_stats(dets, g):
    """Detection agreement of per-image `dets` (post_process dicts, image i ↔ golden image i % n) with
    the fp32 goldens: same label and IoU >= 0.5, |Δscore| of the matched pairs."""
    n_gold = len(g["det_counts"])
    starts = np.concatenate([[0], np.cumsum(g["det_counts"])]).astype(int)
    tot = dict(expected=0, matched=0, extra=0, max_dscore=0.0, max_dbox_px=0.0)
    ds = []
    for i, det in enumerate(dets):
        gi = i % n_gold
        a, b_ = starts[gi], starts[gi + 1]
        es, el, eb = g["det_scores"][a:b_], g["det_labels"][a:b_], g["det_boxes"][a:b_]
        used = set()
        for s, l, b in zip(es, el, eb):
            best, bi = 0.0, -1
            for j in range(len(det["scores"])):
                if j in used or int(det["labels"][j]) != int(l):
                    continue
                v = iou(b, det["boxes"][j].tolist())
                if v > best:
                    best, bi = v, j
            if bi >= 0 and best >= 0.5:
                used.add(bi)
                tot["matched"] += 1
                ds.append(abs(float(det["scores"][bi]) - float(s)))
                tot["max_dscore"] = max(tot["max_dscore"], ds[-1])
                tot["max_dbox_px"] = max(tot["max_dbox_px"], float(np.abs(det["boxes"][bi].numpy() - b).max()))
        tot["expected"] += len(es)
        tot["extra"] += len(det["scores"]) - len(used)
    tot["recall_vs_fp32"] = tot["matched"] / max(1, tot["expected"])
    tot["p50_dscore"] = float(np.percentile(ds, 50)) if ds else 0.0
    tot["p95_dscore"] = float(np.percentile(ds, 95)) if ds else 0.0
    return tot


def golden_gt(g, n):
    """The fp32 golden detections (score > 0.5) of images 0..n-1 (image i ↔ golden i % count) as AP ground truth."""
    starts = np.concatenate([[0], np.cumsum(g["det_counts"])]).astype(int)
    out = []
    for i in range(n):
        gi = i % len(g["det_counts"])
        a, b = starts[gi], starts[gi + 1]
        out.append({"boxes": g["det_boxes"][a:b], "labels": g["det_labels"][a:b]})
    return out


def ap_vs_fp32(out, g, proc):
    """COCO-style AP of a model output's ranked candidates (threshold 0: the 300 per image the
    post-process keeps) against the fp32 golden detections; maxDets 300 (the model's own cap)."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from coco_ap import average_precision

    n = out.logits.shape[0]
    tsz = torch.tensor(np.tile(g["target_sizes"], (n // len(g["det_counts"]) + 1, 1))[:n])
    cand = proc.post_process_object_detection(out, target_sizes=tsz, threshold=0.0)
    dets = [{k: v.numpy() for k, v in c.items()} for c in cand]
    r = average_precision(dets, golden_gt(g, n), max_dets=300)
    return {"map": r["map"], "ap50": r["ap50"], "ap75": r["ap75"]}


def delta(preset, tag=None, precision="bf16", reps=1, **ekw):
    """The golden images (tiled `reps` times into one batch) through Engine(precision) → agreement
    with the fp32 goldens at threshold 0.5 and the AP of the ranked candidates."""
    from tests.test_gpu_model import load_images
    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.config import PRESETS
    from spotter_amd.engine import Engine

    g = np.load(os.path.join(GOLD, f"{tag or preset + '_640'}.npz"))
    size = int(g["size"])
    model = SpotterForObjectDetection(PRESETS[preset], use_graphs=False)
    model._engine = Engine(model.cfg, model._host_weights(), torch.device("cuda", 0), precision=precision, **ekw)
    proc = SpotterImageProcessor(size={"height": size, "width": size})
    imgs = load_images(g) * reps
    with torch.no_grad():
        out = model(**proc(images=imgs))
    tsz = torch.tensor(np.tile(g["target_sizes"], (reps, 1)))
    dets = proc.post_process_object_detection(out, target_sizes=tsz, threshold=0.5)
    st = match_stats(dets, g)
    st["ap_vs_fp32"] = ap_vs_fp32(out, g, proc)
    st["images"] = len(imgs)
    return st


if __name__ == "__main__":
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("precision", nargs="?", default="bf16")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--out", default=None)
    ap.add_argument("--fp32-maps", action="store_true", help="bf16 modes: fp32 backbone maps (Engine bf16_store=False)")
    a = ap.parse_args()
    ekw = {"bf16_store": False} if a.fp32_maps else {}
    res = {p: delta(p, precision=a.precision, reps=a.reps, **ekw) for p in ("r18vd", "r101vd")}
    res["precision"] = a.precision
    res["backbone_maps"] = "fp32" if a.fp32_maps else ("bf16" if a.precision.startswith("bf16") else "fp32")
    line = json.dumps({"metric": "bf16 variant delta vs HF fp32 goldens (synthetic weights; COCO-val unpinned)",
                       **res})
    print(line)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        open(a.out, "w").write(line + "\n")
