"""CPU: the oracle is pinned against the reference's HF path (tests/golden) and Pillow."""
import hashlib
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_pil_resize_restatement_bit_exact_vs_pillow():
    from PIL import Image

    from oracle.pil_resize import resize_bilinear_u8
    from spotter_amd.synthetic import synthetic_image

    for (h, w, oh, ow) in [(480, 800, 640, 640), (333, 517, 640, 640), (300, 200, 640, 640), (717, 1200, 640, 640),
                           (1080, 1920, 1280, 1280), (640, 640, 640, 640), (2, 3000, 640, 640), (1, 1, 64, 64)]:
        img = synthetic_image(h + w, h, w)
        ref = np.asarray(Image.fromarray(img).resize((ow, oh), Image.BILINEAR))
        np.testing.assert_array_equal(resize_bilinear_u8(img, oh, ow), ref, err_msg=str((h, w)))


def test_preprocess_oracle_matches_golden_digests():
    from PIL import Image

    from oracle.pil_resize import preprocess
    from spotter_amd.synthetic import synthetic_image

    g = np.load(os.path.join(GOLD, "preprocess.npz"))
    with Image.open(os.path.join(GOLD, "test_pic.jpg")) as im:
        pic = np.asarray(im.convert("RGB"))
    checked = 0
    for (h, w, o), seed, dig in zip(g["sizes"], g["seeds"], g["digests"]):
        if h * w > 2e6:
            continue  # keep the CPU suite fast; the GPU test covers every size
        img = pic if seed < 0 else synthetic_image(int(seed), int(h), int(w))
        assert sha(preprocess(img, (int(o), int(o)))) == str(dig), (h, w, o)
        checked += 1
    assert checked >= 15


def _detections_match(r, scores, labels, boxes, score_tol=1e-3, box_tol=0.5):
    assert len(r["scores"]) == len(scores)
    used = set()
    for s, l, b in zip(scores, labels, boxes):
        c = [i for i in range(len(r["scores"])) if i not in used and r["labels"][i] == l and
             abs(r["scores"][i] - s) <= score_tol and np.abs(r["boxes"][i] - b).max() <= box_tol]
        assert c, (s, l, b)
        used.add(c[0])


@pytest.mark.parametrize("preset", ["r18vd", "r101vd"])
def test_numpy_oracle_matches_hf_goldens(preset):
    """oracle/rtdetr_np.forward + post_process vs tests/golden (made by HF transformers)."""
    from PIL import Image

    from oracle import rtdetr_np
    from oracle.pil_resize import preprocess
    from spotter_amd.config import PRESETS
    from spotter_amd.synthetic import golden_source
    from spotter_amd.weights import generate

    g = np.load(os.path.join(GOLD, f"{preset}_640.npz"))
    cfg = PRESETS[preset]
    w = generate(cfg, seed=0)
    off = 0
    n_img = 2 if preset == "r101vd" else len(g["seeds"])
    for i in range(n_img):
        img = golden_source(int(g["seeds"][i]), 640, 640, os.path.join(GOLD, "test_pic.jpg"))
        st = rtdetr_np.forward(preprocess(img)[None], w, cfg)
        common = set(st["enc_topk_ind"][0].tolist()) & set(g["enc_topk_ind"][i].tolist())
        assert len(common) >= 298
        th, tw = g["target_sizes"][i]
        r = rtdetr_np.post_process(st["logits"], st["pred_boxes"], [(th, tw)], 0.5)[0]
        n = int(g["det_counts"][i])
        _detections_match(r, g["det_scores"][off:off + n], g["det_labels"][off:off + n], g["det_boxes"][off:off + n])
        off += n


def test_post_process_restatement_matches_hf():
    import torch

    from oracle.hf_ref import build_hf_processor
    from oracle.rtdetr_np import post_process

    rng = np.random.default_rng(0)
    logits = (rng.standard_normal((2, 300, 80)) - 3).astype(np.float32)
    boxes = rng.uniform(0.02, 0.98, (2, 300, 4)).astype(np.float32)

    class O:
        pass

    o = O()
    o.logits, o.pred_boxes = torch.from_numpy(logits), torch.from_numpy(boxes)
    ts = [(717, 1200), (640, 480)]
    ref = build_hf_processor().post_process_object_detection(o, threshold=0.5, target_sizes=torch.tensor(ts))
    mine = post_process(logits, boxes, ts, 0.5)
    for a, b in zip(mine, ref):
        np.testing.assert_array_equal(a["labels"], b["labels"].numpy())
        np.testing.assert_allclose(a["scores"], b["scores"].numpy(), rtol=0, atol=2e-7)  # 1-ulp exp differences
        np.testing.assert_allclose(a["boxes"], b["boxes"].numpy(), rtol=1e-6, atol=1e-4)
