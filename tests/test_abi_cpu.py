"""The ctypes signatures in ops/_lib.py match the C ABI declared in csrc/*.hip (argument count
and pointer-vs-scalar kinds), so a mismatch fails here instead of on the GPU box."""
import glob
import os
import re

import pytest

from mil_nce_howto100m_amd.ops import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _c_decls():
    out = {}
    for path in glob.glob(os.path.join(ROOT, "csrc", "*.hip")):
        src = open(path).read()
        for m in re.finditer(r"MILNCE_API\s+(?:\w+\s+)+?(\w+)\s*\(([^)]*)\)", src):
            params = [p.strip() for p in m.group(2).replace("\n", " ").split(",") if p.strip()]
            out[m.group(1)] = params
    return out


def _kind(param: str) -> str:
    if "*" in param or "hipStream_t" in param:
        return "P"
    if re.match(r"(long long|int64_t)\b", param):
        return "L"
    if param.startswith("double"):
        return "D"
    if param.startswith("float"):
        return "F"
    return "I"


def test_signatures_match_c_declarations():
    decls = _c_decls()
    names = {_lib.P: "P", _lib.I: "I", _lib.F: "F", _lib.D: "D", _lib.L: "L"}
    bad = []
    for name, sig in _lib.SIGNATURES.items():
        assert name in decls, f"{name} not declared in csrc"
        want = [_kind(p) for p in decls[name]]
        have = [names[t] for t in sig]
        if want != have:
            bad.append((name, "".join(have), "".join(want)))
    assert not bad, bad


def test_library_has_no_undefined_kernel_stubs():
    """Every kernel's host launch stub is defined in libmilnce_hip.so: clang's host pass can drop a
    template kernel's stub without an error (seen with a lambda-captured array sized by a
    template-dependent constant), which only fails at dlopen time on the GPU box."""
    import shutil
    import subprocess
    from mil_nce_howto100m_amd.ops._lib import LIB_PATH
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not os.path.exists(LIB_PATH):
        pytest.skip("library not built")
    out = subprocess.run([nm, "-D", "--undefined-only", LIB_PATH], capture_output=True, text=True).stdout
    bad = [ln.split()[-1] for ln in out.splitlines() if ln.split() and ln.split()[-1].startswith("_Z")]
    assert not bad, bad[:10]
