"""CPU: the reference's own deployment module runs unchanged on top of spotter_amd.

Loads apps/spotter/src/spotter/serve.py and schemas.py from /root/reference (this container only;
skipped where the reference is absent, e.g. on the GPU box), applies exactly the module-scope change
documented in INTEGRATION.md §2 in memory (spotter_amd.dropin; the AmenitiesDetector class text is compared
with the reference's), stubs the packages this image lacks (ray.serve,
tenacity), and checks the AmenitiesDetector contract: construction (serve.py:66-72), the module-
level `deployment = AmenitiesDetector.bind(model, processor)` (serve.py:199-205) with a picklable
model, and the mocked `_process_single_image` flow of the reference's own unit tests
(apps/spotter/tests/spotter/test_serve.py:80-148) driven through our processor/model types.
"""
import asyncio
import importlib.util
import linecache
import os
import pickle
import sys
import types
from io import BytesIO
from unittest.mock import AsyncMock, MagicMock, patch

import pytest

REF = "/root/reference/apps/spotter/src/spotter"
pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")


def _stub_modules():
    ray = types.ModuleType("ray")
    serve = types.ModuleType("ray.serve")

    class _Deployment:
        def __init__(self, cls):
            self.func_or_class = cls

        def bind(self, *args, **kwargs):
            return ("bound", self.func_or_class, pickle.dumps((args, kwargs)))

    serve.deployment = lambda cls: _Deployment(cls)
    ray.serve = serve
    ten = types.ModuleType("tenacity")

    class AsyncRetrying:
        def __init__(self, **kw):
            pass

        def __aiter__(self):
            self._done = False
            return self

        async def __anext__(self):
            if self._done:
                raise StopAsyncIteration
            self._done = True

            class _A:
                def __enter__(s):
                    return s

                def __exit__(s, *a):
                    return False
            return _A()

    ten.AsyncRetrying = AsyncRetrying
    ten.stop_after_attempt = lambda n: n
    ten.wait_exponential = lambda **kw: kw
    return {"ray": ray, "ray.serve": serve, "tenacity": ten}


def _load_patched_serve(monkeypatch, tmp_path):
    """The reference serve.py with the drop-in applied by the same code the image runs
    (spotter_amd.dropin, deploy/Dockerfile.rocm), MODEL_NAME = the reference's hub name, resolved
    from a local HF cache snapshot (an R18 checkpoint stored under that name keeps the test small)."""
    from spotter_amd.checkpoint import save_local
    from spotter_amd.config import PRESETS
    from spotter_amd.dropin import patch_source
    from spotter_amd.weights import generate

    src = patch_source(open(os.path.join(REF, "serve.py")).read())
    base = tmp_path / "hub" / "models--PekingU--rtdetr_v2_r101vd"
    save_local(str(base / "snapshots" / "c0ffee"), PRESETS["r18vd"], generate(PRESETS["r18vd"], seed=0))
    (base / "snapshots" / "c0ffee" / "preprocessor_config.json").write_text(
        '{"do_resize": true, "size": {"height": 640, "width": 640}, "resample": 2, "do_rescale": true}')
    (base / "refs").mkdir(parents=True)
    (base / "refs" / "main").write_text("c0ffee")
    monkeypatch.setenv("HF_HUB_CACHE", str(tmp_path / "hub"))
    for name, mod in _stub_modules().items():
        monkeypatch.setitem(sys.modules, name, mod)
    pkg = types.ModuleType("spotter")
    pkg.__path__ = [REF]
    monkeypatch.setitem(sys.modules, "spotter", pkg)
    spec = importlib.util.spec_from_file_location("spotter.schemas", os.path.join(REF, "schemas.py"))
    schemas = importlib.util.module_from_spec(spec)
    monkeypatch.setitem(sys.modules, "spotter.schemas", schemas)
    spec.loader.exec_module(schemas)
    monkeypatch.setenv("MODEL_NAME", "PekingU/rtdetr_v2_r101vd")
    mod = types.ModuleType("spotter.serve")
    # the patched text under a name of its own, so inspect reads the code that actually ran
    mod.__file__ = "<spotter_amd drop-in serve.py>"
    linecache.cache[mod.__file__] = (len(src), None, src.splitlines(True), mod.__file__)
    monkeypatch.setitem(sys.modules, "spotter.serve", mod)
    exec(compile(src, mod.__file__, "exec"), mod.__dict__)
    return mod, schemas


def test_deployment_class_is_byte_identical_to_the_reference(monkeypatch, tmp_path):
    """north_star: the Ray Serve deployment class stays unchanged. The drop-in edits module-scope lines only
    (serve.py:203-204 and the `Image` rebinding), so AmenitiesDetector's source, decorator included, is the
    reference's text (serve.py:64-196), and its `Image.open` resolves to the GPU-decoding module."""
    import ast
    import inspect

    serve, _ = _load_patched_serve(monkeypatch, tmp_path)
    ref = open(os.path.join(REF, "serve.py")).read()
    node = next(n for n in ast.parse(ref).body if isinstance(n, ast.ClassDef) and n.name == "AmenitiesDetector")
    first = min([node.lineno] + [d.lineno for d in node.decorator_list])
    ref_text = "".join(ref.splitlines(True)[first - 1:node.end_lineno])
    cls = serve.deployment[1]
    assert inspect.getsourcefile(cls) == "<spotter_amd drop-in serve.py>"
    assert inspect.getsource(cls) == ref_text
    from spotter_amd.jpeg import _ImageModule

    from spotter_amd.draw import _DrawModule

    assert isinstance(serve.Image, _ImageModule) and isinstance(serve.ImageDraw, _DrawModule)


def test_reference_deployment_module_binds_our_objects(monkeypatch, tmp_path):
    from spotter_amd import SpotterForObjectDetection, SpotterImageProcessor

    serve, _ = _load_patched_serve(monkeypatch, tmp_path)
    assert isinstance(serve.model, SpotterForObjectDetection)
    assert isinstance(serve.processor, SpotterImageProcessor)
    kind, cls, blob = serve.deployment
    assert kind == "bound" and cls.__name__ == "AmenitiesDetector"
    (m, p), _ = pickle.loads(blob)  # what Ray ships to each replica: no device state inside
    assert m._engine is None and m.config.id2label[62] == "tv"
    assert m.cfg.depths == [2, 2, 2, 2] and m._weights is not None  # the cached snapshot, not a preset
    det = cls(model=m, processor=p)  # serve.py:66-72 constructor check passes
    assert det.processor is p


def test_reference_process_single_image_flow_with_our_types(monkeypatch, tmp_path):
    """serve.py:79-148 with our model/processor; kernels replaced by canned outputs (CPU only)."""
    import torch

    from spotter_amd import SpotterImageProcessor
    from spotter_amd.model import SpotterDetectionOutput

    serve, schemas = _load_patched_serve(monkeypatch, tmp_path)
    cls = serve.deployment[1]
    det = cls(model=serve.model, processor=serve.processor)
    det.client = AsyncMock()
    img_bytes = open(os.path.join(os.path.dirname(__file__), "golden", "test_pic.jpg"), "rb").read()
    det._fetch_image_bytes = AsyncMock(return_value=img_bytes)
    logits = torch.full((1, 300, 80), -9.0)
    logits[0, 0, 62] = 3.0   # tv
    logits[0, 1, 57] = 2.0   # couch
    logits[0, 2, 65] = 1.0   # remote (not an amenity)
    boxes = torch.tensor([[[0.5, 0.5, 0.2, 0.2]] * 300])

    def fake_pp(outputs, threshold=0.5, target_sizes=None, use_focal_loss=True):
        # the CPU oracle stands in for sp_postprocess (no GPU in this test)
        from oracle.rtdetr_np import post_process
        r = post_process(outputs.logits.numpy(), outputs.pred_boxes.numpy(), target_sizes.tolist(), threshold)[0]
        return [{k: torch.from_numpy(v) for k, v in r.items()}]

    from spotter_amd.processor import SpotterBatchFeature

    def fake_proc(self, images=None, return_tensors="pt"):
        assert images.mode == "RGB" and images.size == (1200, 717)
        return SpotterBatchFeature(pixel_values=torch.zeros(1, 3, 640, 640))

    # no GPU here: the GPU JPEG decoder declines, so open_image takes the reference's own Image.open
    from spotter_amd import jpeg

    def no_gpu(device=None):
        class _D:
            def decode(self, data):
                raise jpeg.UnsupportedJpeg("CPU test")
        return _D()

    monkeypatch.setattr(jpeg, "decoder", no_gpu)
    with patch.object(SpotterImageProcessor, "__call__", fake_proc), \
         patch.object(type(serve.model), "__call__", lambda self, **kw: SpotterDetectionOutput(logits, boxes)), \
         patch.object(SpotterImageProcessor, "post_process_object_detection", lambda self, *a, **k: fake_pp(*a, **k)):
        res = asyncio.run(det._process_single_image("local_test_image.jpg"))
    assert isinstance(res, schemas.DetectionSuccessResult), getattr(res, "error", "")
    assert [d.label for d in res.detections] == ["TV", "sofa"]
    assert res.detections[0].box == pytest.approx([480.0, 286.8, 720.0, 430.2], abs=1e-3)
    assert len(res.labeled_image_base64) > 500


def _template_env(container: str) -> dict:
    """The env of one container of deploy/rayservice-template.yaml, rendered as spotter-manager renders it."""
    import yaml

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, "deploy", "rayservice-template.yaml")).read()
    body = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    rc = yaml.safe_load(body.replace("{{.DockerImage}}", "img"))["spec"]["rayClusterConfig"]
    conts = list(rc["headGroupSpec"]["template"]["spec"]["containers"])
    for wg in rc["workerGroupSpecs"]:
        conts += wg["template"]["spec"]["containers"]
    (c,) = [c for c in conts if c["name"] == container]
    return {e["name"]: e["value"] for e in c.get("env", [])}


@pytest.mark.parametrize("pod", ["ray-head", "ray-worker"])
def test_rendered_template_configures_a_bf16_engine(monkeypatch, tmp_path, pod):
    """C4 as deployed: the env of each pod of the rendered template, the reference serve.py with the drop-in
    applied, imported as Serve imports it; the bound model (pickled, as Ray ships it to a replica) carries
    precision "bf16", which the engine maps to bf16 conv and linear operands (config.PRECISIONS)."""
    from spotter_amd.config import PRECISIONS

    env = _template_env(pod)
    assert env["SPOTTER_PRECISION"] == "bf16"
    monkeypatch.setenv("SPOTTER_PRECISION", env["SPOTTER_PRECISION"])
    serve, _ = _load_patched_serve(monkeypatch, tmp_path)
    assert serve.model.precision == "bf16"
    (m, _p), _ = pickle.loads(serve.deployment[2])
    assert m.precision == "bf16" and PRECISIONS[m.precision] == ("bf16", "bf16") and m._engine is None


def test_default_and_unknown_precision(monkeypatch, tmp_path):
    """Without SPOTTER_PRECISION the drop-in keeps the fp32 parity path; an unknown value fails serve.py's
    import (the deployment does not come up) instead of the first request."""
    monkeypatch.delenv("SPOTTER_PRECISION", raising=False)
    serve, _ = _load_patched_serve(monkeypatch, tmp_path)
    assert serve.model.precision == "fp32"
    monkeypatch.setenv("SPOTTER_PRECISION", "fp16")
    with pytest.raises(ValueError, match="SPOTTER_PRECISION"):
        _load_patched_serve(monkeypatch, tmp_path / "again")
