#!/usr/bin/env python3
"""Build libmilnce_hip.so (all HIP kernels + the C ABI) for gfx950, in-tree.

    python csrc/build.py [--jobs N] [--debug | --check]

``--debug`` (-O1 -g) and ``--check`` (-O3 with the KASSERT kernel invariant checks, common.h)
build separate objects into ``libmilnce_hip_debug.so`` / ``libmilnce_hip_check.so``; select one
at run time with ``MILNCE_LIB_PATH``.

Each ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950 -O3`` into an object
(parallel, incremental on mtime) and linked into ``mil_nce_howto100m_amd/_native/libmilnce_hip.so``,
which Python loads through ctypes (``ops/_lib.py``). No torch headers are involved, so a full
rebuild takes seconds and the library travels to the GPU box with the source snapshot.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT_DIR = os.path.join(ROOT, "mil_nce_howto100m_amd", "_native")
LIB = os.path.join(OUT_DIR, "libmilnce_hip.so")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("MILNCE_ARCH", "gfx950")


def flags(mode: str):
    f = ["--offload-arch=" + ARCH, "-std=c++17", "-fPIC", "-I" + HERE, "-Wno-unused-result"]
    f += {"debug": ["-O1", "-g"], "check": ["-O3", "-DMILNCE_KCHECK"],
          "trace": ["-O3", "-DBOX_TRACE=1"]}.get(mode, ["-O3"])
    if mode.startswith("def_"):  # A/B libraries: def_NAME=VALUE[,NAME=VALUE] (python csrc/build.py --define ...)
        f += ["-D" + d for d in mode[4:].split(",")]
    return f


def _paths(mode: str):
    if mode == "release":
        return OBJ_DIR, LIB
    return OBJ_DIR + "_" + mode, os.path.join(OUT_DIR, f"libmilnce_hip_{mode}.so")


def compile_one(src: str, mode: str) -> str:
    obj = os.path.join(_paths(mode)[0], os.path.basename(src)[:-4] + ".o")
    deps = [src] + glob.glob(os.path.join(HERE, "*.h"))
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(d) for d in deps):
        return obj
    cmd = [HIPCC] + flags(mode) + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, debug: bool = False, verbose: bool = True, mode: str = "") -> str:
    mode = mode or ("debug" if debug else "release")
    obj_dir, lib = _paths(mode)
    os.makedirs(OUT_DIR, exist_ok=True)
    os.makedirs(obj_dir, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(HERE, "*.hip")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: compile_one(s, mode), srcs))
    newest = max(os.path.getmtime(o) for o in objs)
    if not os.path.exists(lib) or os.path.getmtime(lib) < newest:
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", lib] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    # every kernel's host launch stub must be in the library: clang can silently drop one (e.g.
    # for kernels in an anonymous namespace, or with template-sized local arrays), which only
    # shows as an undefined symbol when the library is loaded
    r = subprocess.run(["nm", "-C", "--undefined-only", lib], capture_output=True, text=True)
    missing = [ln.split(None, 1)[1] for ln in r.stdout.splitlines() if "_kernel" in ln and ln.split()[0] == "U"]
    if missing:
        raise RuntimeError(f"{lib}: undefined kernel symbols (dropped launch stubs): {missing[:4]}")
    if verbose:
        print(f"built {lib} from {len(srcs)} sources")
    return lib


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("--check", action="store_true", help="build with the KASSERT kernel checks")
    ap.add_argument("--trace", action="store_true", help="box conv phase timestamps (tools/box_trace.py)")
    ap.add_argument("--define", default="", help="NAME=VALUE[,...]: an A/B library libmilnce_hip_def_....so")
    a = ap.parse_args()
    try:
        if a.define:
            build(a.jobs, mode="def_" + a.define)
        else:
            build(a.jobs, mode="check" if a.check else ("trace" if a.trace else ("debug" if a.debug else "release")))
    except RuntimeError as e:
        print(e, file=sys.stderr)
        sys.exit(1)
