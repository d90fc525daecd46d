"""Two-stream micro-batch determinism with one suspect at a time switched: repeat forward(microbatches=2) and count
repeats whose logits differ from the first (a race shows as n_differ > 0)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor, ops
from spotter_amd._lib import lib
from spotter_amd.config import PRESETS
from tests.test_gpu_model import load_images

g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests", "golden",
                         "r18vd_640.npz"))
imgs = (load_images(g) * 64)[:16]
px = SpotterImageProcessor()(images=imgs, return_tensors="pt")["pixel_values"].to("cuda")


def trial(name, setup=None, teardown=None, reps=20):
    model = SpotterForObjectDetection(PRESETS["r18vd"], use_graphs=False)
    eng = model.engine
    if setup:
        setup(eng)
    outs = []
    try:
        for _ in range(reps):
            with torch.no_grad():
                lg, _ = eng.forward(px, microbatches=2)
            outs.append(lg.clone())
        torch.cuda.synchronize()
    finally:
        if teardown:
            teardown(eng)
    h = px.shape[0] // 2
    d0 = [float((o[:h] - outs[0][:h]).abs().max()) for o in outs[1:]]
    d1 = [float((o[h:] - outs[0][h:]).abs().max()) for o in outs[1:]]
    print(json.dumps({name: {"n_differ_first_half": sum(x > 0 for x in d0), "n_differ_second_half": sum(x > 0 for x in d1),
                             "max": max(d0 + d1)}}), flush=True)


trial("baseline")
trial("msda_vec", lambda e: lib().sp_set_tuning(4, 1), lambda e: lib().sp_set_tuning(4, 0))
trial("no_splitk", lambda e: setattr(e, "_splitk", lambda: {}))
