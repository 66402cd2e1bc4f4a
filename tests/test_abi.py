"""The C ABI library loads and exports every symbol include/*.h declares (CPU only)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

import repkiller_amd as rk


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for name in os.listdir(inc):
        if name.endswith(".h"):
            with open(os.path.join(inc, name)) as f:
                text = f.read()
            syms |= set(re.findall(r"^\s*(?:int|void|const char \*)\s*\*?\s*(rk_\w+)\s*\(", text,
                                   re.M))
    return syms


def test_header_declares_python_exports():
    assert declared_symbols() == set(rk.EXPORTS)


@pytest.mark.parametrize("sym", sorted(declared_symbols()))
def test_library_exports(sym):
    lib = rk.load_library()
    assert hasattr(lib, sym)
    assert ctypes.cast(getattr(lib, sym), ctypes.c_void_p).value


def test_device_code_is_gfx950():
    out = os.popen(f"/opt/rocm/lib/llvm/bin/clang-offload-bundler --list --type=o "
                   f"--input={rk.LIB_PATH} 2>/dev/null").read()
    # the bundle may be embedded differently; fall back to scanning for the target id
    with open(rk.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob or "gfx950" in out


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(rk.RkError) as e:
        rk.Context(0)
    assert e.value.code == -8  # RK_E_NODEVICE
