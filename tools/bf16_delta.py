"""bf16 variant vs the fp32 reference outputs (tests/golden): the accuracy delta we can state offline.

COCO-val mAP needs the real checkpoint and COCO images (both unreachable offline), so the bf16 delta is
reported as detection agreement with the HF fp32 goldens on the synthetic-weight model: matched
detections (same label, IoU >= 0.5), max |Δscore| of matched pairs, and missed / extra detections.
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


def delta(preset, tag=None, precision="bf16"):
    from tests.test_gpu_model import load_images
    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.config import PRESETS
    from spotter_amd.engine import Engine

    g = np.load(os.path.join(GOLD, f"{tag or preset + '_640'}.npz"))
    size = int(g["size"])
    model = SpotterForObjectDetection(PRESETS[preset], use_graphs=False)
    model._engine = Engine(model.cfg, model._host_weights(), torch.device("cuda", 0), precision=precision)
    proc = SpotterImageProcessor(size={"height": size, "width": size})
    dets = []
    for i, img in enumerate(load_images(g)):
        out = model(**proc(images=img))
        th, tw = g["target_sizes"][i]
        dets.append(proc.post_process_object_detection(out, target_sizes=torch.tensor([[th, tw]]), threshold=0.5)[0])
    return match_stats(dets, g)


if __name__ == "__main__":
    prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    res = {p: delta(p, precision=prec) for p in ("r18vd", "r101vd")}
    res["precision"] = prec
    print(json.dumps({"metric": "bf16 variant detection delta vs HF fp32 goldens (synthetic weights)", **res}))
