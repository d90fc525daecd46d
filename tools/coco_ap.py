"""COCO-style average precision in numpy (the accuracy statement of the bf16 variant).

Follows pycocotools' COCOeval for bbox (evaluateImg / accumulate), restricted to what the offline
comparison needs: area range "all", maxDets 100, no crowd regions.

* per image and class, detections sorted by score (stable) and cut at maxDets; each detection in
  turn takes the unmatched ground truth of highest IoU >= t (ties: the first such in GT order);
* per class, all images' detections merged by score (stable mergesort), cumulative TP / FP,
  precision made monotone from the right, then read at the 101 recall points 0, 0.01, ..., 1
  (searchsorted 'left'; 0 beyond the last reached recall);
* AP = mean over those points, mAP = mean over IoU thresholds 0.50:0.05:0.95 and over the classes
  that have ground truth (pycocotools' -1 entries are excluded).

Real COCO-val AP needs the real checkpoint and the COCO images, neither reachable offline ("parity
unpinned"); this routine is used to state the bf16 variant's AP against the fp32 path's own
detections taken as ground truth (tools/bf16_delta.py), and is unit-tested on hand-built cases
(tests/test_host.py).
"""
from __future__ import annotations

import numpy as np

IOU_THRS = np.linspace(0.5, 0.95, 10)
REC_THRS = np.linspace(0.0, 1.0, 101)


def box_iou(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """IoU matrix of xyxy boxes a [n,4] × b [m,4] (float64)."""
    a = np.asarray(a, np.float64).reshape(-1, 4)
    b = np.asarray(b, np.float64).reshape(-1, 4)
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    area_a = (a[:, 2] - a[:, 0]) * (a[:, 3] - a[:, 1])
    area_b = (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1])
    union = area_a[:, None] + area_b[None, :] - inter
    return np.where(union > 0, inter / np.where(union > 0, union, 1), 0.0)


def _match(det_boxes, gt_boxes, t):
    """Greedy COCO matching of score-sorted detections: bool TP flags at IoU threshold t."""
    tp = np.zeros(len(det_boxes), bool)
    if len(det_boxes) == 0 or len(gt_boxes) == 0:
        return tp
    ious = box_iou(det_boxes, gt_boxes)
    taken = np.zeros(len(gt_boxes), bool)
    for d in range(len(det_boxes)):
        best, m = min(t, 1 - 1e-10), -1
        for g in range(len(gt_boxes)):
            if taken[g] or ious[d, g] < best:
                continue
            best, m = ious[d, g], g
        if m >= 0:
            taken[m] = True
            tp[d] = True
    return tp


def average_precision(dets, gts, max_dets: int = 100, iou_thrs=IOU_THRS):
    """dets / gts: per image, dicts with "boxes" [n,4] xyxy, "labels" [n] (+ "scores" [n] for dets).
    Returns {"map": mAP over IoU thresholds and classes with GT, "ap50": AP at IoU 0.5, "ap75",
    "per_class": {label: AP}} (nan where no class has ground truth)."""
    assert len(dets) == len(gts)
    classes = sorted({int(l) for g in gts for l in np.asarray(g["labels"]).reshape(-1)})
    ap = np.full((len(iou_thrs), len(classes)), np.nan)
    for ci, c in enumerate(classes):
        npig = 0
        per_t_scores, per_t_tp = [[] for _ in iou_thrs], [[] for _ in iou_thrs]
        for d, g in zip(dets, gts):
            gl = np.asarray(g["labels"]).reshape(-1)
            gb = np.asarray(g["boxes"], np.float64).reshape(-1, 4)[gl == c]
            npig += len(gb)
            dl = np.asarray(d["labels"]).reshape(-1)
            ds = np.asarray(d["scores"], np.float64).reshape(-1)[dl == c]
            db = np.asarray(d["boxes"], np.float64).reshape(-1, 4)[dl == c]
            order = np.argsort(-ds, kind="mergesort")[:max_dets]
            ds, db = ds[order], db[order]
            for ti, t in enumerate(iou_thrs):
                per_t_scores[ti].append(ds)
                per_t_tp[ti].append(_match(db, gb, t))
        if npig == 0:
            continue
        for ti in range(len(iou_thrs)):
            s = np.concatenate(per_t_scores[ti])
            tpf = np.concatenate(per_t_tp[ti])
            order = np.argsort(-s, kind="mergesort")
            tpf = tpf[order]
            tps = np.cumsum(tpf).astype(np.float64)
            fps = np.cumsum(~tpf).astype(np.float64)
            rc = tps / npig
            pr = tps / np.maximum(tps + fps, np.finfo(np.float64).eps)
            for i in range(len(pr) - 1, 0, -1):
                pr[i - 1] = max(pr[i - 1], pr[i])
            q = np.zeros(len(REC_THRS))
            inds = np.searchsorted(rc, REC_THRS, side="left")
            ok = inds < len(pr)
            q[ok] = pr[inds[ok]]
            ap[ti, ci] = q.mean()
    res = {"map": float(np.nanmean(ap)) if classes else float("nan"),
           "per_class": {c: float(np.nanmean(ap[:, i])) for i, c in enumerate(classes)}}
    for name, t in (("ap50", 0.5), ("ap75", 0.75)):
        hit = np.where(np.isclose(np.asarray(iou_thrs), t))[0]
        res[name] = float(np.nanmean(ap[hit[0]])) if len(hit) and classes else float("nan")
    return res
