"""Diagnostic: the bf16 variant's backbone with bf16 maps vs fp32 maps, stage by stage (relative error of
each stage output and of the logits). python tools/diag_bf16store.py [preset] [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from spotter_amd.config import PRESETS
from spotter_amd.engine import Engine
from spotter_amd.weights import generate
from spotter_amd import ops
from spotter_amd.synthetic import synthetic_batch


def main():
    preset = sys.argv[1] if len(sys.argv) > 1 else "r18vd"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cfg = PRESETS[preset]
    w = generate(cfg, seed=0)
    dev = torch.device("cuda", 0)
    px = torch.rand(B, 3, 640, 640, device=dev)
    res = {}
    for store in (False, True):
        eng = Engine(cfg, w, dev, precision="bf16", bf16_store=store)
        feats = []
        g = eng.backbone(px, B, 640, 640)
        try:
            while True:
                next(g)
        except StopIteration as e:
            feats = e.value
        outs = []
        for (t, h, ww, c) in feats:
            a = t[: B * h * ww * c]
            if a.dtype == torch.int16:
                a = torch.from_numpy(ops._bf16_float(a.cpu().numpy().view(np.uint16))).float()
            outs.append(a.cpu().float().numpy().reshape(-1))
        lg, bx = eng.forward(px)
        torch.cuda.synchronize()
        res[store] = (outs, lg.cpu().numpy(), bx.cpu().numpy())
    for i, (a, b) in enumerate(zip(res[False][0], res[True][0])):
        print(f"stage feat {i}: max|a| {np.abs(a).max():.4g} max|a-b| {np.abs(a - b).max():.4g} "
              f"rel {np.abs(a - b).max() / max(np.abs(a).max(), 1e-9):.3g}")
    for nm, k in (("logits", 1), ("boxes", 2)):
        a, b = res[False][k], res[True][k]
        print(f"{nm}: max|a-b| {np.abs(a - b).max():.4g}")


if __name__ == "__main__" and not (os.environ.get("DIAG_INPROJ") or os.environ.get("DIAG_WS") or os.environ.get("DIAG_LOCK")):
    main()


def in_proj_check(preset="r18vd", B=2):
    """in_proj on the bf16 maps vs the same values as fp32 rows: must be bit-identical."""
    from spotter_amd.ops import view
    cfg = PRESETS[preset]
    w = generate(cfg, seed=0)
    dev = torch.device("cuda", 0)
    px = torch.rand(B, 3, 640, 640, device=dev)
    eng = Engine(cfg, w, dev, precision="bf16", bf16_store=True)
    g = eng.backbone(px, B, 640, 640)
    try:
        while True:
            next(g)
    except StopIteration as e:
        feats = e.value
    for l, (t, h, ww, c) in enumerate(feats):
        a16 = t[: B * h * ww * c].contiguous()
        a32 = torch.from_numpy(ops._bf16_float(a16.cpu().numpy().view(np.uint16))).to(dev)
        cw = eng.in_proj[l]
        o1 = torch.empty(B * h * ww * cw.cout, device=dev)
        o2 = torch.empty(B * h * ww * cw.cout, device=dev)
        eng._cv(view(a32, c), B, h, ww, cw, 1, view(o1, cw.cout))
        eng._cv(view(a16, c), B, h, ww, cw, 1, view(o2, cw.cout))
        torch.cuda.synchronize()
        d = (o1 - o2).abs().max().item()
        print(f"in_proj {l}: M={B*h*ww} K={c} N={cw.cout} max|fp32-rows - bf16-rows| = {d}  max|o| {o1.abs().max().item():.4g}")


if __name__ == "__main__" and os.environ.get("DIAG_INPROJ"):
    in_proj_check(*(sys.argv[1:2] or ["r18vd"]))


def ws_compare(preset="r18vd", B=8):
    """Run the whole eager forward with bf16 maps and with fp32 maps; relative difference of every fp32
    workspace buffer both engines hold (in allocation order)."""
    cfg = PRESETS[preset]
    w = generate(cfg, seed=0)
    dev = torch.device("cuda", 0)
    px = torch.rand(B, 3, 640, 640, device=dev)
    engs = {}
    for store in (False, True):
        eng = Engine(cfg, w, dev, precision="bf16", bf16_store=store)
        lg = torch.empty(B * 300 * cfg.num_labels, device=dev)
        bx = torch.empty(B * 300 * 4, device=dev)
        for _ in eng._run(px, lg.view(B, 300, -1), bx.view(B, 300, 4)):
            pass
        torch.cuda.synchronize()
        engs[store] = (eng, lg, bx)
    wa, wb = engs[False][0]._ws, engs[True][0]._ws
    for k, ta in wa.items():
        tb = wb.get(k)
        if tb is None or ta.dtype != torch.float32 or tb.dtype != torch.float32 or ta.numel() != tb.numel():
            continue
        a, b = ta.float(), tb.float()
        s = a.abs().max().item()
        d = (a - b).abs().max().item()
        print(f"{k:24s} n={ta.numel():>10d} max|a| {s:9.4g} max|a-b| {d:9.4g} rel {d / max(s, 1e-12):.3g}")
    print("logits", (engs[False][1] - engs[True][1]).abs().max().item())


if __name__ == "__main__" and os.environ.get("DIAG_WS"):
    ws_compare(*(sys.argv[1:2] or ["r18vd"]))


def lockstep(preset="r18vd", B=256):
    """Backbone block by block, both storage modes in lockstep: first buffer whose values diverge."""
    cfg = PRESETS[preset]
    w = generate(cfg, seed=0)
    dev = torch.device("cuda", 0)
    px = torch.rand(B, 3, 640, 640, device=dev)
    ea = Engine(cfg, w, dev, precision="bf16", bf16_store=False)
    eb = Engine(cfg, w, dev, precision="bf16", bf16_store=True)
    ga, gb = ea.backbone(px, B, 640, 640), eb.backbone(px, B, 640, 640)

    def f32(t):
        if t.dtype == torch.int16:
            return (t.to(torch.int32) << 16).view(torch.float32)
        return t

    step = 0
    while True:
        try:
            next(ga)
            next(gb)
        except StopIteration:
            break
        torch.cuda.synchronize()
        for k in eb._ws:
            if k not in ea._ws or k == "splitk":
                continue
            a, b = ea._ws[k], f32(eb._ws[k])
            n = min(a.numel(), b.numel())
            s = a[:n].abs().max().item()
            d = (a[:n] - b[:n]).abs().max().item()
            flag = "  <<<" if d > 0.05 * max(s, 1e-9) else ""
            print(f"block {step:2d} {k:12s} n={n:>11d} max|a| {s:8.4g} max|a-b| {d:8.4g}{flag}")
        step += 1


if __name__ == "__main__" and os.environ.get("DIAG_LOCK"):
    lockstep(sys.argv[1] if len(sys.argv) > 1 else "r18vd", int(sys.argv[2]) if len(sys.argv) > 2 else 256)
