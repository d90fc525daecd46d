import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libspotter_hip.so")
    config.addinivalue_line("markers", "slow: long-running")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


_BOUNDS_LOG = []


@pytest.fixture(autouse=True)
def _bounds_check(request):
    """Bounds-check library (SPOTTER_HIP_LIB=spotter_amd/_bounds/libspotter_bounds.so, SP_BUILD_BOUNDS): after
    every GPU test, collect the kernels' index violations (sp_bounds_report); any hit fails that test. With the
    product library this does nothing."""
    yield
    if "gpu" not in request.node.keywords or not os.environ.get("SPOTTER_HIP_LIB"):
        return
    import ctypes

    from spotter_amd._lib import SP_BUILD_BOUNDS, lib

    L = lib()
    if not L.sp_build_flags() & SP_BUILD_BOUNDS:
        return
    buf = ctypes.create_string_buffer(8192)
    hits = L.sp_bounds_report(buf, len(buf))
    _BOUNDS_LOG.append({"test": request.node.nodeid, "hits": int(hits),
                        "report": buf.value.decode(errors="replace")})
    assert hits == 0, f"bounds-check build: {hits} index violations\n{buf.value.decode(errors='replace')}"


def pytest_sessionfinish(session, exitstatus):
    if _BOUNDS_LOG:
        import json

        out = os.path.join(ROOT, "gpurun_out", "bounds_report.json")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        with open(out, "w") as f:
            json.dump({"tests": len(_BOUNDS_LOG), "tests_with_hits": sum(1 for r in _BOUNDS_LOG if r["hits"]),
                       "total_hits": sum(max(0, r["hits"]) for r in _BOUNDS_LOG),
                       "hits": [r for r in _BOUNDS_LOG if r["hits"]]}, f, indent=1)
        print(f"\nbounds report -> {out}")
    _write_margins()


def _write_margins():
    """Write the observed parity margins of the golden tests (tests/margins.py), if any ran."""
    here = os.path.dirname(os.path.abspath(__file__))
    if here not in sys.path:
        sys.path.insert(0, here)
    import margins

    path = margins.write()
    if path:
        print(f"\nparity margins -> {path}")
