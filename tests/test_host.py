"""CPU: host logic — weight inventory vs HF, C-ABI exports, drop-in interface, replicas."""
import os
import pickle
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("preset,params", [("r18vd", 20_174_608), ("r101vd", 76_556_268)])
def test_param_inventory_matches_hf(preset, params):
    from oracle.hf_ref import build_hf_model
    from spotter_amd.config import PRESETS
    from spotter_amd.weights import generate, param_specs

    cfg = PRESETS[preset]
    w = generate(cfg)
    m = build_hf_model(cfg, w)  # strict load: every key and shape must match
    assert sum(p.numel() for p in m.parameters()) == params
    assert len({k for k, _, _ in param_specs(cfg)}) == len(w)


def test_weights_are_deterministic():
    from spotter_amd.config import PRESETS
    from spotter_amd.weights import generate

    a = generate(PRESETS["r18vd"], seed=0)
    b = generate(PRESETS["r18vd"], seed=0)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    k = "model.decoder.layers.0.mlp.fc1.weight"
    assert abs(float(a[k][0, 0]) - float(generate(PRESETS["r18vd"], seed=0)[k][0, 0])) == 0


def _header_functions():
    src = open(os.path.join(ROOT, "include", "spotter_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sp_\w+)\s*\(", src, re.M)))


def test_library_exports_every_header_symbol():
    from spotter_amd import _lib
    from spotter_amd.build_ext import LIB, build

    if not os.path.exists(LIB):
        build(verbose=False)
    names = _header_functions()
    assert set(names) == set(_lib.EXPORTS), set(names) ^ set(_lib.EXPORTS)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (sp_\w+)", out))
    assert set(names) <= exported, set(names) - exported
    L = _lib.load()  # dlopen + bind, no device call
    assert L.sp_abi_version() == _lib.ABI_VERSION


def test_arg_errors_are_reported_without_a_gpu():
    """Argument validation runs on the host and returns <0 with a message (no device touched)."""
    import ctypes as C

    from spotter_amd import _lib

    L = _lib.load()
    assert L.sp_layernorm(None, 0, None, None, None, 0, 0, 0, 1e-5, None) < 0
    assert b"sp_layernorm" in L.sp_last_error()
    d = _lib.SpConvDesc()
    assert L.sp_conv2d(C.byref(d), None) < 0
    assert b"sp_conv2d" in L.sp_last_error()
    assert L.sp_topk_rows(C.c_void_p(16), 0, 1, 100000, 1, 0, 10, None, C.c_void_p(16), None) < 0
    assert b"n=100000" in L.sp_last_error()


def test_dropin_interface_and_pickling():
    """The attributes AmenitiesDetector reads (serve.py:67-68, 98-117) and Ray-style pickling."""
    import torch

    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.processor import SpotterBatchFeature

    proc = SpotterImageProcessor.from_pretrained("PekingU/rtdetr_v2_r101vd")
    model = SpotterForObjectDetection.from_pretrained("PekingU/rtdetr_v2_r101vd").to(torch.device("cpu"))
    assert hasattr(proc, "post_process_object_detection")
    assert model.config.id2label[62] == "tv" and model.config.id2label[57] == "couch"
    assert model.config.id2label[60] == "dining table" and model.config.id2label[78] == "hair drier"
    m2 = pickle.loads(pickle.dumps(model))
    p2 = pickle.loads(pickle.dumps(proc))
    assert m2.cfg.name == "r101vd" and p2.size == {"height": 640, "width": 640}
    bf = SpotterBatchFeature(pixel_values=torch.zeros(1))
    assert bf.to(torch.device("cpu")) is bf and bf.pixel_values is bf["pixel_values"]


def test_replica_shard_and_gloo_max():
    import torch.multiprocessing as mp

    from spotter_amd.replicas import shard

    for n, world in [(32, 1), (32, 8), (33, 4), (3, 8)]:
        parts = [list(shard(n, r, world)) for r in range(world)]
        assert sum(parts, []) == list(range(n))
        assert max(map(len, parts)) - min(map(len, parts)) <= 1
    mp.spawn(_gloo_worker, args=(2,), nprocs=2, join=True)


def _gloo_worker(rank, world):
    import torch.distributed as dist

    from spotter_amd.replicas import barrier, max_over_ranks

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    barrier()
    assert max_over_ranks(1.0 + rank) == float(world)
    dist.destroy_process_group()


def test_checkpoint_key_renames():
    from spotter_amd.checkpoint import rename_key

    assert rename_key("model.decoder.layers.0.self_attn.out_proj.weight") == "model.decoder.layers.0.self_attn.o_proj.weight"
    assert rename_key("model.decoder.layers.3.fc1.bias") == "model.decoder.layers.3.mlp.fc1.bias"
    assert rename_key("model.encoder.encoder.0.layers.0.fc2.weight") == "model.encoder.aifi.0.layers.0.mlp.fc2.weight"
