"""CPU: host logic — weight inventory vs HF, C-ABI exports, drop-in interface, replicas."""
import os
import pickle
import re
import subprocess
import sys

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
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(sp_\w+)\s*\(", src, re.M)))


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


def test_ctypes_descriptors_match_the_header_layout(tmp_path):
    """The ctypes mirrors of the C-ABI descriptor structs (spotter_amd/_lib.py) have the header's size and
    field offsets, checked against a C program compiled from include/spotter_hip.h."""
    import ctypes

    from spotter_amd import _lib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    structs = {"sp_conv_desc": _lib.SpConvDesc, "sp_msda_desc": _lib.SpMsdaDesc}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "spotter_hip.h"', "int main(void) {"]
    for cname, py in structs.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        cname, f, v = ln.split()
        got[(cname, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == ctypes.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)


def test_product_library_reads_no_environment():
    """Tile / transform choices come from the ABI (sp_set_conv_config) and the compiled tables only: the
    environment overrides of the tuning tools exist only in an SP_TUNING_BUILD=1 library."""
    from spotter_amd.build_ext import LIB, build

    if not os.path.exists(LIB):
        build(verbose=False)
    out = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True).stdout
    assert not re.search(r"\b(secure_)?getenv\b", out), "libspotter_hip.so imports getenv"


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
    d = _lib.SpConvDesc(A=16, C=16, KH=3, KW=3, stride=2, pad=1)
    assert L.sp_conv3x3_winograd(C.byref(d), C.c_void_p(16), 0, C.c_void_p(16), 0, None) < 0
    assert b"stride-1" in L.sp_last_error()


def test_dropin_interface_and_pickling():
    """The attributes AmenitiesDetector reads (serve.py:67-68, 98-117) and Ray-style pickling."""
    import torch

    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.processor import SpotterBatchFeature

    proc = SpotterImageProcessor.from_pretrained("synthetic:r101vd")
    model = SpotterForObjectDetection.from_pretrained("synthetic:r101vd").to(torch.device("cpu"))
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


def test_bench_launcher_spawns_one_replica_per_gpu():
    """bench.py --gpus 2 (no torch.distributed launcher) spawns two replica processes, each pinned to
    its own device by HIP_VISIBLE_DEVICES, that meet only in the gloo barrier / max.
    The GPU step is stubbed (a sleep), so this runs on the CPU."""
    import json
    import sys

    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        env.pop(v, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--stub-step-ms", "20"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 64
    assert [p["rank"] for p in line["per_rank"]] == [0, 1]
    assert [p["device"] for p in line["per_rank"]] == ["0", "1"]
    # whole-job value = both replicas' images over the max elapsed (each ~32 img / 20 ms)
    assert 2 * 32 / 0.040 < line["value"] <= 2 * 32 / 0.020 * 1.01


@pytest.mark.parametrize("fail_rank", [1, 0])
def test_bench_launcher_fails_fast_when_a_replica_dies(fail_rank):
    """One replica exits 3 before the rendezvous: the launcher reports that code within seconds and
    kills the other rank, which would otherwise wait in the gloo rendezvous until its timeout."""
    import sys
    import time

    env = dict(os.environ)
    for v in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        env.pop(v, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--stub-step-ms", "20", "--stub-fail-rank", str(fail_rank)],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert f"replica rank {fail_rank} exited with 3" in r.stderr
    assert time.time() - t0 < 60
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.parametrize("preset", ["r18vd", "r101vd"])
def test_config_from_hf_reads_hf_config_json(preset, tmp_path):
    """config.json as HF itself writes it (RTDetrV2Config.save_pretrained) → the same SpotterConfig as the
    preset; our own writer (checkpoint.hf_config_dict) is read back identically; no field is unknown."""
    import dataclasses
    import json

    from transformers import RTDetrResNetConfig, RTDetrV2Config

    from spotter_amd.checkpoint import config_from_hf, hf_config_dict, unknown_fields
    from spotter_amd.config import PRESETS

    cfg = PRESETS[preset]
    kw = cfg.to_hf_kwargs()
    RTDetrV2Config(backbone_config=RTDetrResNetConfig(**kw["backbone"]), **kw["model"]).save_pretrained(tmp_path)
    js = json.loads((tmp_path / "config.json").read_text())
    assert unknown_fields(js) == []
    got = dataclasses.asdict(config_from_hf(js))
    want = dataclasses.asdict(cfg)
    assert {k: (got[k], want[k]) for k in got if k != "name" and got[k] != want[k]} == {}
    assert dataclasses.asdict(config_from_hf(hf_config_dict(cfg))) == got


@pytest.mark.parametrize("field,value", [("decoder_method", "discrete"), ("normalize_before", True),
                                         ("encoder_activation_function", "tanh"), ("learn_initial_query", True),
                                         ("decoder_n_points", [4, 4, 4]), ("num_feature_levels", 4),
                                         ("use_focal_loss", False)])
def test_config_from_hf_refuses_unimplemented_values(field, value):
    from spotter_amd.checkpoint import UnsupportedConfig, config_from_hf, hf_config_dict
    from spotter_amd.config import PRESETS

    js = hf_config_dict(PRESETS["r18vd"])
    js[field] = value
    with pytest.raises(UnsupportedConfig):
        config_from_hf(js)
    js = hf_config_dict(PRESETS["r18vd"])
    js["backbone_config"]["hidden_act"] = "tanh"
    with pytest.raises(UnsupportedConfig):
        config_from_hf(js)


def test_config_from_hf_reads_nondefault_supported_values():
    """Supported non-default values are carried, not dropped (activations, eps, eval / anchor sizes)."""
    from spotter_amd.checkpoint import config_from_hf, hf_config_dict
    from spotter_amd.config import PRESETS

    js = hf_config_dict(PRESETS["r18vd"])
    js.update(encoder_activation_function="relu", activation_function="gelu", decoder_activation_function="silu",
              layer_norm_eps=1e-6, batch_norm_eps=1e-3, eval_size=[640, 640], anchor_image_size=[640, 640],
              positional_encoding_temperature=20)
    c = config_from_hf(js)
    assert (c.encoder_activation_function, c.activation_function, c.decoder_activation_function) == ("relu", "gelu", "silu")
    assert (c.layer_norm_eps, c.batch_norm_eps, c.eval_size, c.anchor_image_size) == (1e-6, 1e-3, (640, 640), (640, 640))
    assert c.positional_encoding_temperature == 20


def test_local_checkpoint_round_trip(tmp_path):
    """save_local writes config.json + model.safetensors with 4.x key names (the inverse of
    conversion_mapping.py:1042-1047); load_local maps them back to exactly the generated tensors."""
    from safetensors.numpy import load_file

    from spotter_amd.checkpoint import load_local, save_local
    from spotter_amd.config import PRESETS
    from spotter_amd.weights import generate

    cfg = PRESETS["r18vd"]
    w = generate(cfg, seed=3)
    save_local(str(tmp_path), cfg, w)
    raw = load_file(str(tmp_path / "model.safetensors"))
    assert any(".out_proj." in k for k in raw) and not any(".o_proj." in k for k in raw)
    assert any(".layers.0.fc1." in k for k in raw) and not any(".mlp.fc" in k for k in raw)
    assert any(k.startswith("model.encoder.encoder.0.layers.0.") for k in raw)
    cfg2, w2 = load_local(str(tmp_path))
    assert cfg2.depths == cfg.depths and cfg2.encoder_hidden_dim == cfg.encoder_hidden_dim
    assert set(w2) == set(w)
    assert all(np.array_equal(w2[k], w[k]) for k in w)


def _fake_hub_cache(root, repo, cfg, weights, commit="0123abcd"):
    """A HF hub cache entry laid out as huggingface_hub writes it: refs/main → snapshots/<commit>/."""
    import json

    from spotter_amd.checkpoint import save_local

    base = root / ("models--" + repo.replace("/", "--"))
    snap = base / "snapshots" / commit
    save_local(str(snap), cfg, weights)
    (snap / "preprocessor_config.json").write_text(json.dumps(
        {"image_processor_type": "RTDetrImageProcessor", "do_resize": True, "size": {"height": 640, "width": 640},
         "resample": 2, "do_rescale": True, "rescale_factor": 1 / 255, "do_normalize": False, "do_pad": False,
         "format": "coco_detection", "do_convert_annotations": True}))
    (base / "refs").mkdir(parents=True)
    (base / "refs" / "main").write_text(commit)
    return snap


def test_hub_name_resolves_to_the_cached_snapshot(tmp_path, monkeypatch):
    """from_pretrained(<hub name>) loads the snapshot HF's cache holds under that name (the reference
    image pre-fetches MODEL_NAME there: apps/spotter/Dockerfile:17 → download.py:23-27, then
    serve.py:203-204 loads it by name): same config and tensors, and the processor reads the
    snapshot's preprocessor_config.json. A name not in the cache raises; synthetic is opt-in only."""
    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor
    from spotter_amd.checkpoint import resolve_pretrained
    from spotter_amd.config import PRESETS
    from spotter_amd.weights import generate

    cfg = PRESETS["r18vd"]
    w = generate(cfg, seed=5)
    snap = _fake_hub_cache(tmp_path / "hub", "PekingU/rtdetr_v2_r101vd", cfg, w)
    for var in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE", "TRANSFORMERS_CACHE"):
        monkeypatch.delenv(var, raising=False)
    monkeypatch.setenv("HF_HOME", str(tmp_path))
    assert resolve_pretrained("PekingU/rtdetr_v2_r101vd") == str(snap)
    m = SpotterForObjectDetection.from_pretrained("PekingU/rtdetr_v2_r101vd")
    assert m.cfg.depths == cfg.depths and set(m._weights) == set(w)
    assert all(np.array_equal(m._weights[k], w[k]) for k in w)
    p = SpotterImageProcessor.from_pretrained("PekingU/rtdetr_v2_r101vd")
    assert p.size == {"height": 640, "width": 640} and p.resample == 2
    with pytest.raises(OSError, match="no local directory and no cached snapshot"):
        SpotterForObjectDetection.from_pretrained("PekingU/rtdetr_v2_r50vd")
    with pytest.raises(OSError):
        SpotterImageProcessor.from_pretrained("PekingU/rtdetr_v2_r50vd")
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))  # the explicit cache variable
    monkeypatch.setenv("HF_HOME", str(tmp_path / "elsewhere"))
    assert resolve_pretrained("PekingU/rtdetr_v2_r101vd") == str(snap)
    assert SpotterForObjectDetection.from_pretrained("synthetic:r101vd")._weights is None
    assert SpotterForObjectDetection.from_pretrained("x", synthetic=True).cfg.name == "r101vd"


def test_processor_refuses_arithmetic_it_does_not_implement(tmp_path):
    """preprocessor_config.json fields that change the arithmetic are honoured or refused, never ignored."""
    import json

    from spotter_amd import SpotterImageProcessor

    for bad in ({"resample": 3}, {"resample": 0}, {"do_normalize": True}, {"do_pad": True},
                {"rescale_factor": 1 / 127.5}, {"size": {"shortest_edge": 640}}):
        d = tmp_path / ("c%d" % len(list(tmp_path.iterdir())))
        d.mkdir()
        (d / "preprocessor_config.json").write_text(json.dumps(dict({"resample": 2}, **bad)))
        with pytest.raises(NotImplementedError):
            SpotterImageProcessor.from_pretrained(str(d))
    ok = tmp_path / "ok"
    ok.mkdir()
    (ok / "preprocessor_config.json").write_text(json.dumps({"resample": 2, "size": {"height": 800, "width": 800}}))
    assert SpotterImageProcessor.from_pretrained(str(ok)).size == {"height": 800, "width": 800}


def test_loader_skips_bookkeeping_keys_and_warns_on_unknown(tmp_path):
    """Keys some transformers versions add on save (underscore bookkeeping, generic PretrainedConfig
    attributes) do not stop a real checkpoint from loading; an unknown key is reported, not fatal."""
    import json

    from spotter_amd.checkpoint import hf_config_dict, load_local, unknown_fields
    from spotter_amd.config import PRESETS

    js = hf_config_dict(PRESETS["r18vd"])
    js.update(_attn_implementation_autoset=True, _commit_hash="abc", use_cache=True, pad_token_id=None,
              output_scores=False)
    assert unknown_fields(js) == []
    js["some_future_field"] = 1
    assert unknown_fields(js) == ["some_future_field"]
    (tmp_path / "config.json").write_text(json.dumps(js))
    with pytest.warns(UserWarning, match="some_future_field"):
        cfg, w = load_local(str(tmp_path))
    assert cfg.depths == PRESETS["r18vd"].depths and w == {}
    from spotter_amd.checkpoint import UnsupportedConfig

    with pytest.raises(UnsupportedConfig, match="some_future_field"):
        load_local(str(tmp_path), strict=True)  # what the image build check uses
    js["decoder_future_gate"] = True  # named like a model field: refused even when not strict
    (tmp_path / "config.json").write_text(json.dumps(js))
    with pytest.raises(UnsupportedConfig, match="decoder_future_gate"):
        load_local(str(tmp_path))


@pytest.mark.parametrize("wm", [2, 4])
def test_winograd_weight_transform_reproduces_the_direct_conv(wm):
    """ops.winograd_weights_host (U = G g Gᵀ, fp64 on the host) composed with the F(m×m,3x3) input /
    output transforms the kernels apply (Bᵀ d B, Aᵀ M A with ops.WINO_BT / WINO_AT, the constants of
    winograd.hip) is the 3x3 stride-1 pad-1 cross-correlation: checked in fp64 on a ragged map (H, W not
    multiples of the tile) against a direct conv."""
    from spotter_amd import ops

    rng = np.random.default_rng(3)
    n, h, w, ci, co = 2, 5, 7, 6, 4
    a = wm + 2
    x = rng.standard_normal((n, h, w, ci))
    g = rng.standard_normal((co, 3, 3, ci)).astype(np.float32)
    u = ops.winograd_weights_host(g, wm).astype(np.float64).reshape(a, a, co, ci)
    bt, at = ops.WINO_BT[wm], ops.WINO_AT[wm]
    th, tw = (h + wm - 1) // wm, (w + wm - 1) // wm
    xp = np.zeros((n, wm * th + 2, wm * tw + 2, ci))
    xp[:, 1:h + 1, 1:w + 1] = x
    y = np.zeros((n, wm * th, wm * tw, co))
    for ty in range(th):
        for tx in range(tw):
            d = xp[:, wm * ty:wm * ty + a, wm * tx:wm * tx + a]            # [n, a, a, ci]
            v = np.einsum("ai,nijc,bj->nabc", bt, d, bt)
            m = np.einsum("nabc,aboc->nabo", v, u)
            y[:, wm * ty:wm * ty + wm, wm * tx:wm * tx + wm] = np.einsum("pa,nabo,qb->npqo", at, m, at)
    ref = np.zeros((n, h, w, co))
    xq = np.pad(x, ((0, 0), (1, 1), (1, 1), (0, 0)))
    for i in range(3):
        for j in range(3):
            ref += np.einsum("nhwc,oc->nhwo", xq[:, i:i + h, j:j + w], g[:, i, j, :].astype(np.float64))
    np.testing.assert_allclose(y[:, :h, :w], ref, rtol=1e-6, atol=1e-5)


def test_winograd_kernel_constants_match_host_matrices():
    """The Bᵀ / Aᵀ constants compiled into winograd.hip (kBT43, kAT43) are the matrices the host-side
    weight transform and the CPU reproduction test use (ops.WINO_BT / WINO_AT), entry for entry."""
    from spotter_amd import ops

    src = open(os.path.join(os.path.dirname(__file__), "..", "spotter_amd", "csrc", "winograd.hip")).read()
    for name, ref in (("kBT43", ops.WINO_BT[4]), ("kAT43", ops.WINO_AT[4])):
        body = src[src.index(f"constexpr float {name}"):]
        body = body[body.index("{"):body.index("};")]
        vals = [float(v.rstrip("f")) for v in re.findall(r"-?\d+\.\d*f?", body)]
        assert np.array_equal(np.array(vals).reshape(ref.shape), ref), name


def test_weight_split_on_host_matches_torch_rne():
    """ops.split_bf16x3_host / bf16_bits (numpy, pack time) against torch's own RNE bf16 cast on the CPU:
    hi / mid / lo bit-identical to the chained casts, and hi + mid + lo == w exactly."""
    import torch

    from spotter_amd import ops

    rng = np.random.default_rng(0)
    w = np.concatenate([rng.standard_normal(4096).astype(np.float32) * 10.0 ** rng.integers(-8, 8, 4096),
                        np.array([0.0, -0.0, 1.0, 1 + 2 ** -8, 1 + 2 ** -9, 3e-39, 65504.0])]).astype(np.float32)
    planes = ops.split_bf16x3_host(w).view(np.uint16)
    t = torch.from_numpy(w)
    hi = t.to(torch.bfloat16)
    r1 = t - hi.float()
    mid = r1.to(torch.bfloat16)
    lo = (r1 - mid.float()).to(torch.bfloat16)
    for got, ref in zip(planes, (hi, mid, lo)):
        assert np.array_equal(got, ref.view(torch.int16).numpy().view(np.uint16))
    f = [(p.astype(np.uint32) << 16).view(np.float32).astype(np.float64) for p in planes]
    normal = (np.abs(w) >= 1e-30) | (w == 0)  # far enough from the subnormal range for lo to stay exact
    assert np.array_equal((f[0] + f[1] + f[2])[normal], w.astype(np.float64)[normal])


def test_rayservice_template_renders():
    """deploy/rayservice-template.yaml rendered as spotter-manager renders the reference template
    (Go text/template, the single action {{.DockerImage}}, handlers.go:98-118) and decoded as YAML
    (handlers.go:124-150): GVR ray.io/v1alpha1 (handlers.go:152-156), one Serve replica per MI355X."""
    import yaml

    src = open(os.path.join(ROOT, "deploy", "rayservice-template.yaml")).read()
    body = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    assert re.findall(r"{{[^}]*}}", body) and set(re.findall(r"{{[^}]*}}", body)) == {"{{.DockerImage}}"}
    image = "registry.local/spotter-mi355x:test"
    doc = yaml.safe_load(body.replace("{{.DockerImage}}", image))
    assert doc["apiVersion"] == "ray.io/v1alpha1" and doc["kind"] == "RayService"
    assert doc["metadata"]["name"] == "spotter-ray-service"
    serve = yaml.safe_load(doc["spec"]["serveConfigV2"])
    app = serve["applications"][0]
    assert (app["name"], app["import_path"], app["route_prefix"]) == ("spotter-serve", "spotter.serve:deployment", "/detect")
    dep = app["deployments"][0]
    assert dep["name"] == "AmenitiesDetector"
    per_gpu = round(1 / dep["ray_actor_options"]["num_gpus"])
    assert per_gpu * dep["ray_actor_options"]["num_gpus"] == 1
    rc = doc["spec"]["rayClusterConfig"]
    head = rc["headGroupSpec"]["template"]["spec"]["containers"][0]
    assert head["image"] == image and rc["headGroupSpec"]["rayStartParams"]["num-gpus"] == "0"
    (wg,) = rc["workerGroupSpecs"]
    worker = wg["template"]["spec"]["containers"][0]
    assert worker["image"] == image
    gpus = worker["resources"]["limits"]["amd.com/gpu"]
    assert worker["resources"]["requests"]["amd.com/gpu"] == gpus
    assert int(wg["rayStartParams"]["num-gpus"]) == gpus == 8 and dep["num_replicas"] == gpus * per_gpu
    # replicas per GPU = the measured k-sweep's (profiles/r6/served, C4's bf16 and the fp32 parity path): the most
    # whole-request throughput whose p95 stays within 1.5x the single replica's
    import json

    for prec in ("bf16", "fp32"):
        with open(os.path.join(ROOT, "profiles", "r6", "served", f"served_r101vd_{prec}.json")) as f:
            pts = json.load(f)["points"]
        one = next(p for p in pts if p["k_processes"] == 1)
        ok = [p for p in pts if p["p95_ms"] <= 1.5 * one["p95_ms"]]
        assert max(ok, key=lambda p: p["img_per_s"])["k_processes"] == per_gpu, prec
    env = {e["name"]: e["value"] for e in worker["env"]}
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    # as the reference template (configs/rayservice-template.yaml:41-59): no pod overrides MODEL_NAME,
    # the image's ENV decides for head and workers alike
    assert "MODEL_NAME" not in env and "MODEL_NAME" not in {e["name"] for e in head.get("env", [])}
    # C4 (BASELINE configs[3]): bf16 replicas, set where serve.py is imported (head: app build) and run (workers)
    head_env = {e["name"]: e["value"] for e in head.get("env", [])}
    assert env["SPOTTER_PRECISION"] == head_env["SPOTTER_PRECISION"] == "bf16"


def _dockerfile_recipe():
    """(ARG MODEL_NAME default, the directory the checkpoint context is copied to) from deploy/Dockerfile.rocm."""
    text = open(os.path.join(ROOT, "deploy", "Dockerfile.rocm")).read()
    default = re.search(r'^ARG MODEL_NAME="([^"]*)"', text, re.M).group(1)
    ckpt_dir = re.search(r"^COPY --from=checkpoint / (\S+)", text, re.M).group(1).rstrip("/")
    assert "python -m spotter_amd.checkpoint --check \"$MODEL_NAME\"" in text
    return default, ckpt_dir


def _pod_model_names(image_env):
    """MODEL_NAME each container of the rendered template sees: its own env entry, else the image ENV."""
    import yaml

    src = open(os.path.join(ROOT, "deploy", "rayservice-template.yaml")).read()
    body = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    rc = yaml.safe_load(body.replace("{{.DockerImage}}", "img"))["spec"]["rayClusterConfig"]
    conts = list(rc["headGroupSpec"]["template"]["spec"]["containers"])
    for wg in rc["workerGroupSpecs"]:
        conts += wg["template"]["spec"]["containers"]
    return {c["name"]: {e["name"]: e["value"] for e in c.get("env", [])}.get("MODEL_NAME", image_env) for c in conts}


def test_every_pod_model_name_resolves_for_each_build_recipe(tmp_path, monkeypatch):
    """The two documented image recipes of deploy/Dockerfile.rocm, replayed on a scratch filesystem:
    (1) the default hub name, pre-fetched into the HF cache by spotter_download (the checkpoint
    directory stays empty), (2) --build-context checkpoint=<dir> --build-arg MODEL_NAME=<that dir>.
    For each, the MODEL_NAME every pod of the rendered template sees resolves to a directory holding
    config.json, and the image's build check accepts it. The broken mix (MODEL_NAME = the checkpoint
    directory without the checkpoint context) is refused by the build check instead of by every replica."""
    from spotter_amd import checkpoint
    from spotter_amd.config import PRESETS
    from spotter_amd.weights import generate

    default, ckpt_dir = _dockerfile_recipe()
    cfg = PRESETS["r18vd"]
    w = generate(cfg, seed=1)
    for var in ("HF_HUB_CACHE", "HUGGINGFACE_HUB_CACHE", "TRANSFORMERS_CACHE"):
        monkeypatch.delenv(var, raising=False)
    root = tmp_path / "img"
    baked = root / ckpt_dir.lstrip("/")

    def check(image_env):
        names = _pod_model_names(image_env)
        assert len(names) >= 2 and set(names.values()) == {image_env}, names
        for n in names.values():
            local = str(root / n.lstrip("/")) if n.startswith("/") else n
            d = checkpoint.resolve_pretrained(local)
            assert os.path.isfile(os.path.join(d, "config.json"))
            assert checkpoint.check_image_model(local) == d

    # recipe 1: hub name, snapshot in the image's HF cache, /models/... empty
    monkeypatch.setenv("HF_HOME", str(root / "hf"))
    _fake_hub_cache(root / "hf" / "hub", default, cfg, w)
    baked.mkdir(parents=True)
    check(default)
    # the broken mix: MODEL_NAME = the (empty) checkpoint directory → refused at build time
    with pytest.raises(OSError, match="without config.json"):
        checkpoint.check_image_model(str(baked))
    # recipe 2: the checkpoint context baked into ckpt_dir, MODEL_NAME = that directory
    monkeypatch.setenv("HF_HOME", str(tmp_path / "empty_hf"))
    checkpoint.save_local(str(baked), cfg, w)
    check(ckpt_dir)


def test_dockerfile_copies_exist_in_their_contexts():
    """deploy/Dockerfile.rocm builds from the spotter repo root (as the reference apps/spotter/Dockerfile)
    plus this repo as the named context `spotter_amd`: every COPY source exists in its context."""
    ref = "/root/reference"
    lines = open(os.path.join(ROOT, "deploy", "Dockerfile.rocm")).read().splitlines()
    copies = [l.split()[1:] for l in lines if l.startswith("COPY ")]
    assert copies
    for args in copies:
        frm = next((a.split("=", 1)[1] for a in args if a.startswith("--from=")), None)
        srcs = [a for a in args if not a.startswith("--")][:-1]
        for s in srcs:
            if frm == "spotter_amd":
                assert os.path.exists(os.path.join(ROOT, s)), s
            elif frm == "checkpoint":
                assert s == "/"
            elif os.path.isdir(ref):  # the spotter repo root, when present in this container
                assert os.path.exists(os.path.join(ref, s)), s
    stages = [l.split()[-1] for l in lines if l.startswith("FROM ")]
    assert {"checkpoint", "spotter_amd"} <= set(stages)
    text = "\n".join(lines)
    # the image applies and verifies the drop-in itself (no hand edit of serve.py before docker build)
    assert "python -m spotter_amd.dropin src/spotter/serve.py" in text and "d.check(" in text
    assert text.index("spotter_amd.dropin src/spotter/serve.py") > text.index("COPY apps/spotter/src ./src")


def test_dropin_script_patches_serve_py(tmp_path):
    """spotter_amd.dropin (run by the Dockerfile) on a copy of the reference serve.py: the module-scope lines
    of serve.py:203-204 are replaced (plus the module-scope `Image` rebinding), a second run is a no-op, and
    a serve.py whose lines moved is refused."""
    import sys

    from spotter_amd import dropin

    ref = "/root/reference/apps/spotter/src/spotter/serve.py"
    if os.path.exists(ref):
        src = open(ref).read()
    else:  # the GPU box has no reference: the three lines as the reference writes them
        src = (f"import os\nmodel_name = os.environ.get('MODEL_NAME')\n"
               f"{dropin.OLD_MODEL}\n{dropin.OLD_PROC}\n")
    p = tmp_path / "serve.py"
    p.write_text(src)
    for _ in range(2):
        r = subprocess.run([sys.executable, "-m", "spotter_amd.dropin", str(p)], cwd=ROOT, capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr
    out = p.read_text()
    dropin.check(out)
    assert out.count("SpotterForObjectDetection.from_pretrained(") == 1 and out.count(dropin.PRECISION_ARG) == 1
    assert out.count("Image = image_module()") == 1
    assert out.count("with Image.open(BytesIO(image_bytes)) as img_raw:") == src.count("with Image.open(")
    back = out
    for old, new in dropin.REPLACEMENTS:
        back = back.replace(new, old)
    assert back == src
    bad = tmp_path / "bad.py"
    bad.write_text(src.replace(dropin.OLD_PROC, "processor = AutoImageProcessor.from_pretrained(other)"))
    r = subprocess.run([sys.executable, "-m", "spotter_amd.dropin", str(bad)], cwd=ROOT, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "expected exactly one" in r.stderr


def test_detect_path_harness_with_fake_model():
    """tools/detect_path.py (the whole-/detect latency harness) on the CPU with a fake processor/model:
    real HTTP fetch, decode, label filter, draw, JPEG + base64, response JSON."""
    import asyncio
    import base64
    import io
    import json
    import sys

    import httpx
    import torch
    from PIL import Image

    sys.path.insert(0, ROOT)
    from tools import detect_path

    class Proc:
        def __call__(self, images, return_tensors="pt"):
            class B(dict):
                def to(self, d):
                    return self
            return B(pixel_values=torch.zeros(1, 3, 8, 8))

        def post_process_object_detection(self, outputs, target_sizes, threshold):
            return [{"scores": torch.tensor([0.9, 0.8]), "labels": torch.tensor([62, 65]),
                     "boxes": torch.tensor([[10.0, 20.0, 110.0, 220.0], [1.0, 2.0, 3.0, 4.0]])}]

    class Cfg:
        id2label = {62: "tv", 65: "remote"}

    class Model:
        config = Cfg()

        def __call__(self, **kw):
            return None

    jpeg = open(os.path.join(ROOT, "tests", "golden", "test_pic.jpg"), "rb").read()
    srv, url = detect_path.serve_bytes(jpeg)

    async def run():
        async with httpx.AsyncClient() as client:
            # no GPU here: the reference's host decode (the GPU path is test_gpu_jpeg.py's)
            return await detect_path.handle(json.dumps({"image_urls": [url]}).encode(), client, Proc(), Model(), {},
                                            detect_path.opener("host"))

    try:
        out = json.loads(asyncio.run(run()))
    finally:
        srv.shutdown()
    assert out["amenities_description"] == "The property contains: TV."
    (img,) = out["images"]
    assert img["detections"] == [{"label": "TV", "box": [10.0, 20.0, 110.0, 220.0]}]
    with Image.open(io.BytesIO(base64.b64decode(img["labeled_image_base64"]))) as im:
        assert im.size == (1200, 717)


def test_microbatcher_coalesces_concurrent_calls():
    """spotter_amd.batching on the CPU with a fake engine: 16 concurrent threads' bs1 calls run as a
    few batched forwards, every caller gets its own rows, mixed image sizes never share a batch,
    and a failing forward reaches every caller of that batch."""
    import threading

    import torch

    from spotter_amd.batching import MicroBatcher

    seen = []

    def run(x):
        seen.append(tuple(x.shape))
        time.sleep(0.01)
        return x[:, 0, 0, :1].repeat(1, 3).unsqueeze(-1), x[:, 0, :4, 0].unsqueeze(1)

    import time
    mb = MicroBatcher(run, "cpu", max_batch=8, max_wait_ms=20)
    res = {}

    def caller(i):
        s = 8 if i % 4 else 16
        x = torch.full((1, 3, s, s), float(i))
        res[i] = mb(x)

    th = [threading.Thread(target=caller, args=(i,)) for i in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert all(float(res[i][0].flatten()[0]) == i and res[i][0].shape == (1, 3, 1) for i in range(16))
    assert mb.images == 16 and mb.batches < 16
    assert all(b <= 8 for b, *_ in seen) and len({s[2] for s in seen if s[0] > 1}) <= 2
    assert all(len({sh[2]}) == 1 for sh in seen)

    def boom(x):
        raise RuntimeError("kernel failed")

    mb2 = MicroBatcher(boom, "cpu", max_batch=4, max_wait_ms=5)
    with pytest.raises(RuntimeError, match="kernel failed"):
        mb2(torch.zeros(1, 3, 8, 8))
    mb.close()
    mb2.close()


def test_microbatcher_cancelled_caller_does_not_fail_the_others():
    """A caller that cancels its Future while its batch runs: the other callers of that batch still get
    their rows, the pending count returns to zero (so coalescing stays on), the collector survives."""
    import threading
    import time

    import torch

    from spotter_amd.batching import MicroBatcher

    gate = threading.Event()

    def run(x):
        gate.wait(5)
        return x[:, 0, 0, :1].unsqueeze(-1), x[:, 0, :1, :4]

    mb = MicroBatcher(run, "cpu", max_batch=8, max_wait_ms=100)
    futs = [mb.submit(torch.full((1, 3, 4, 4), float(i))) for i in range(3)]
    time.sleep(0.2)  # all three taken into one batch, blocked in run
    assert futs[1].cancel()
    gate.set()
    assert float(futs[0].result(5)[0].flatten()[0]) == 0.0 and float(futs[2].result(5)[0].flatten()[0]) == 2.0
    assert futs[1].cancelled()
    time.sleep(0.05)
    assert mb._pending == 0
    assert float(mb(torch.full((1, 3, 4, 4), 7.0))[0].flatten()[0]) == 7.0  # the collector is alive
    mb.close()


def test_microbatcher_lone_serial_caller_is_not_delayed():
    """The unchanged serve.py calls the model once per image, serially: with nobody else pending the
    batcher dispatches at once instead of waiting max_wait_ms for company."""
    import time

    import torch

    from spotter_amd.batching import MicroBatcher

    mb = MicroBatcher(lambda x: (x[:, :1, 0, :3], x[:, 0, :1, :4]), "cpu", max_batch=32, max_wait_ms=200)
    x = torch.zeros(1, 3, 8, 8)
    mb(x)  # thread warm-up
    t0 = time.perf_counter()
    for _ in range(20):
        mb(x)
    per_call = (time.perf_counter() - t0) / 20
    mb.close()
    assert per_call < 0.05, per_call  # far below the 200 ms wait window
    assert mb.batches == 21 and mb._pending == 0


def test_tile_table_entries_can_run_their_configuration():
    """Every exact-shape entry of csrc/tile_table.h names a configuration its shape can launch (the LDS-DMA
    tiles need Cin % BK == 0): an entry the generic kernel would shadow is dead weight."""
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_tile_table import runnable

    src = open(os.path.join(ROOT, "spotter_amd", "csrc", "tile_table.h")).read()
    rows = [tuple(map(int, m)) for m in re.findall(r"\{(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (-?\d+)\},", src)]
    assert len(rows) > 50
    bad = [r for r in rows if r[0] and r[5] and not runnable(r[6], r[2] // (r[3] * r[3]), r[1])]
    assert bad == []


def _ap():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import coco_ap

    return coco_ap


def test_coco_ap_hand_built_cases():
    """tools/coco_ap.py (COCOeval bbox restated: greedy best-IoU matching, 101-point interpolated precision,
    IoU 0.50:0.95) on cases whose AP is known by hand."""
    ap = _ap().average_precision
    g = {"boxes": np.array([[0, 0, 10, 10], [20, 20, 30, 30]], float), "labels": np.array([1, 1])}
    perfect = dict(g, scores=np.array([0.9, 0.8]))
    assert ap([perfect], [g])["map"] == 1.0
    # hit (0.9), false positive (0.8), hit (0.7): precision 1 up to recall 0.5, then 2/3 (envelope)
    d = {"boxes": np.array([[0, 0, 10, 10], [50, 50, 60, 60], [20, 20, 30, 30]], float),
         "labels": np.array([1, 1, 1]), "scores": np.array([0.9, 0.8, 0.7])}
    assert abs(ap([d], [g])["map"] - (51 * 1.0 + 50 * (2 / 3)) / 101) < 1e-12
    # one detection with IoU 0.6 against its only GT: a hit at IoU 0.50, 0.55, 0.60 only → AP 0.3
    one = {"boxes": np.array([[0, 0, 10, 10]], float), "labels": np.array([3])}
    shifted = {"boxes": np.array([[0, 0, 10, 6]], float), "labels": np.array([3]), "scores": np.array([0.5])}
    assert abs(_ap().box_iou(shifted["boxes"], one["boxes"])[0, 0] - 0.6) < 1e-12
    r = ap([shifted], [one])
    assert abs(r["map"] - 0.3) < 1e-12 and r["ap50"] == 1.0 and r["ap75"] == 0.0
    # a duplicate of a matched detection is a false positive; a wrong label is not a hit at all
    dup = {"boxes": np.array([[0, 0, 10, 10]] * 2, float), "labels": np.array([3, 3]), "scores": np.array([0.9, 0.8])}
    assert ap([dup], [one])["map"] == 1.0  # the FP comes after recall 1 was reached
    dup2 = dict(dup, scores=np.array([0.8, 0.9]))
    assert ap([dup2], [one])["map"] == 1.0
    wrong = dict(dup, labels=np.array([4, 4]))
    assert ap([wrong], [one])["map"] == 0.0
    # two images, classes averaged: class 1 perfect, class 2 missed entirely → mAP 0.5
    g2 = {"boxes": np.array([[0, 0, 5, 5]], float), "labels": np.array([2])}
    none = {"boxes": np.zeros((0, 4)), "labels": np.zeros(0, int), "scores": np.zeros(0)}
    r = ap([perfect, none], [g, g2])
    assert r["per_class"] == {1: 1.0, 2: 0.0} and r["map"] == 0.5
    # maxDets: only the top 100 detections per image count
    many = {"boxes": np.array([[100, 100, 110, 110]] * 100 + [[0, 0, 10, 10]], float),
            "labels": np.ones(101, int), "scores": np.concatenate([np.full(100, 0.9), [0.1]])}
    assert ap([many], [{"boxes": one["boxes"], "labels": np.array([1])}])["map"] == 0.0


def test_engine_refuses_fused_layernorm_on_bf16_linears():
    """fuse_ln runs the linears on fp32 weights: with bf16 linears ("bf16", and its round-2 alias
    "bf16-all") that would change the operand precision silently, so the Engine refuses at construction
    (before any device call), not at the first forward."""
    from spotter_amd.config import PRESETS
    from spotter_amd.engine import Engine

    for prec in ("bf16", "bf16-all"):
        with pytest.raises(ValueError, match="fuse_ln"):
            Engine(PRESETS["r18vd"], {}, "cpu", precision=prec, fuse_ln=True)


def test_served_sweep_coordinates_its_workers():
    """tools/served_sweep.py's coordination on CPU (stub workers: a request is a 5 ms sleep): k processes report
    ready, start on a common clock, count only requests finished inside the window, and the aggregate is the sum."""
    sys.path.insert(0, ROOT)
    from tools.served_sweep import sweep_point

    r = sweep_point(3, "fp32", "r101vd", 1.0, 0, 60.0, stub_ms=5.0)
    assert r["k_processes"] == 3 and len(r["per_process_img_per_s"]) == 3
    assert 3 * 120 <= r["requests"] <= 3 * 200, r
    assert abs(sum(r["per_process_img_per_s"]) - r["img_per_s"]) < 1.0
    assert 5.0 <= r["p50_ms"] < 20.0


def test_product_library_build_flags():
    """The product library has neither the fused-LayerNorm tiles nor bounds checks (sp_build_flags, no device
    call): Engine(fuse_ln=True) is refused at construction, and sp_bounds_report says it is not a
    bounds-check build."""
    import ctypes

    from spotter_amd._lib import LIB_PATH, load
    from spotter_amd.build_ext import LIB
    from spotter_amd.config import PRESETS
    from spotter_amd.engine import Engine

    if LIB_PATH != LIB:
        pytest.skip("SPOTTER_HIP_LIB selects another library")
    L = load()
    assert L.sp_build_flags() == 0
    buf = ctypes.create_string_buffer(256)
    assert L.sp_bounds_report(buf, 256) == -1 and b"not a bounds-check build" in L.sp_last_error()
    with pytest.raises(ValueError, match="diagnostic library"):
        Engine(PRESETS["r18vd"], {}, "cpu", precision="fp32", fuse_ln=True)


def test_merge_tile_table_keeps_entries_and_skips_winograd(tmp_path):
    """tools/merge_tile_table.py (round 4): a measured winner beyond --min-gain replaces or adds its (shape,
    mode) entry, a "-" win or a small gain leaves the table as it was, the Winograd component GEMMs of a
    --detail file are skipped (wino_gemm tiles them by rule), a tile the shape cannot run (Cin % BK) is not
    written, and every other entry keeps its comment."""
    import json
    import subprocess
    import sys

    table = tmp_path / "tile_table.h"
    table.write_text("#pragma once\nconstexpr TileEntry kTileTable[] = {\n"
                     "    {100, 256, 512, 1, 1, 3, 46},  // x1.1 keep me\n"
                     "    {200, 128, 256, 1, 1, 3, 45},  // x1.05 replaced\n"
                     "    {0, 0, 0, 0, 0, 0, -1},\n};\n")
    shapes = [
        {"m": 200, "cout": 128, "K": 256, "k": 1, "stride": 1, "mode": "x3", "times": {"-": 1.0, "46": 0.95, "247": 0.9},
         "best_same_mode": "247"},
        {"m": 300, "cout": 256, "K": 256, "k": 1, "stride": 1, "mode": "x3", "times": {"-": 1.0, "245": 0.99},
         "best_same_mode": "245"},
        {"m": 400, "cout": 256, "K": 256, "k": 1, "stride": 1, "mode": "x3", "times": {"-": 1.0, "245": 0.5},
         "best_same_mode": "245"},
        {"m": 500, "cout": 64, "K": 48, "k": 1, "stride": 1, "mode": "x3", "times": {"-": 1.0, "45": 0.5},
         "best_same_mode": "45"},
        {"m": 600, "cout": 256, "K": 256, "k": 1, "stride": 1, "mode": "x3", "times": {"-": 1.0, "246": 0.7},
         "best_same_mode": "246"},
    ]
    tune = tmp_path / "tune.json"
    tune.write_text(json.dumps({"shapes": shapes}))
    detail = tmp_path / "detail.json"
    detail.write_text(json.dumps([{"shape": "(400, 256, 256, 1, 1, 'x3', 'wino', 100)", "ms": 1.0, "launches": 1}]))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "merge_tile_table.py"), str(tune), "--tag", "t",
                        "--table", str(table), "--detail", str(detail)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    src = table.read_text()
    assert "{100, 256, 512, 1, 1, 3, 46},  // x1.1 keep me" in src
    assert "{200, 128, 256, 1, 1, 3, 247}," in src and "replaced" not in src
    assert "{300," not in src  # 1 % gain: below --min-gain
    assert "{400," not in src  # a Winograd component GEMM of the detail file
    assert "{500," not in src  # Cin 48: the LDS-DMA tile cannot run it
    assert "{600, 256, 256, 1, 1, 3, 246}," in src
    assert src.rstrip().endswith("};") and "{0, 0, 0, 0, 0, 0, -1}," in src
