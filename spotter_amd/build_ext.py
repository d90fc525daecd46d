"""Builds libspotter_hip.so in-tree with hipcc for gfx950 (MI355X).

    python -m spotter_amd.build_ext [--force] [--bounds]

Objects go to spotter_amd/_build/, the library to spotter_amd/libspotter_hip.so
(git-ignored; it travels to the GPU box with the gpurun snapshot). Sources are
compiled in parallel and only when newer than their object.

--bounds: the bounds-check diagnostic library instead (every unit with -DSP_BOUNDS=1; objects in
spotter_amd/_build_bounds/, library spotter_amd/_bounds/libspotter_bounds.so; select it with
SPOTTER_HIP_LIB). Its kernels count index violations (SP_BCHECK, csrc/common.h) for sp_bounds_report.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libspotter_hip.so")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-ffp-contract=fast",
         "-Xarch_host", "-ffp-contract=off", "-munsafe-fp-atomics", f"-I{INCLUDE}"]
# SP_TUNING_BUILD=1 compiles the tuning-only environment overrides in (e.g. SP_WINO43_VW in winograd.hip);
# the product library reads no environment. Rebuild with --force when toggling it.
if os.environ.get("SP_TUNING_BUILD") == "1":
    FLAGS.append("-DSP_TUNING_BUILD")


def sources():
    # the heavy template units first, so the parallel build ends with the short ones
    heavy = ("conv_glds_p", "conv_mfma16", "conv_gemm")
    srcs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    return sorted(srcs, key=lambda p: not os.path.basename(p).startswith(heavy))


def _includes(path: str, seen: set) -> set:
    """The quoted #include files a source pulls in, transitively (what its object depends on)."""
    import re

    with open(path) as f:
        names = re.findall(r'^\s*#\s*include\s+"([^"]+)"', f.read(), re.M)
    for n in names:
        q = os.path.normpath(os.path.join(os.path.dirname(path), n))
        if q not in seen and os.path.exists(q):
            seen.add(q)
            _includes(q, seen)
    return seen


def _deps_mtime(src: str):
    return max([os.path.getmtime(src)] + [os.path.getmtime(h) for h in _includes(src, set())])


BOUNDS_BUILD = os.path.join(HERE, "_build_bounds")
BOUNDS_LIB = os.path.join(HERE, "_bounds", "libspotter_bounds.so")


def _compile(src: str, force: bool, build_dir: str = BUILD, extra=()) -> str:
    obj = os.path.join(build_dir, os.path.basename(src).replace(".hip", ".o"))
    if not force and os.path.exists(obj):
        if os.path.getmtime(obj) >= _deps_mtime(src):
            return obj
    cmd = [HIPCC, *FLAGS, *extra, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True, bounds: bool = False) -> str:
    build_dir, lib, extra = (BOUNDS_BUILD, BOUNDS_LIB, ("-DSP_BOUNDS=1",)) if bounds else (BUILD, LIB, ())
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    srcs = sources()
    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(lambda s: _compile(s, force, build_dir, extra), srcs))
    if force or not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", lib]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        if verbose:
            print(f"built {lib}")
    return lib


if __name__ == "__main__":
    build(force="--force" in sys.argv, bounds="--bounds" in sys.argv)
