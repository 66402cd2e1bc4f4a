"""ctypes binding of the CPU restatement (oracle/rk_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline.  The product
(repkiller_amd) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
LIB = os.path.join(_HERE, "_build", "librk_oracle.so")
CLI = os.path.join(_HERE, "_build", "rk_oracle")
REF_DRIVER = os.path.join(_HERE, "_ref", "ref_driver")      # the reference itself (oracle/ref.mk)
REF_MAIN = os.path.join(_HERE, "_ref", "repkiller_fix")
REF_SRC = "/root/reference/src"

_lib = None


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-f", "oracle/oracle.mk"], cwd=_ROOT, check=True)


def build_reference() -> bool:
    """Compile the reference from its sources (only where /root/reference exists)."""
    if not os.path.isdir(REF_SRC):
        return False
    subprocess.run(["make", "-s", "-f", "oracle/ref.mk"], cwd=_ROOT, check=True)
    return True


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build_oracle()
        l = ctypes.CDLL(LIB)
        vp = ctypes.c_void_p
        l.rko_classify.restype = ctypes.c_int
        l.rko_classify.argtypes = [ctypes.c_uint64, vp, vp, vp, vp, ctypes.c_uint64,
                                   ctypes.c_uint64, ctypes.c_double, ctypes.c_double, vp, vp, vp,
                                   ctypes.POINTER(ctypes.c_uint64),
                                   ctypes.POINTER(ctypes.c_uint64)]
        l.rko_std_sort.restype = None
        l.rko_std_sort.argtypes = [vp, ctypes.c_size_t]
        _lib = l
    return _lib


def _p(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def classify(x_start, y_start, length, strand, len_x_hdr: int, len_y_hdr: int,
             len_ratio: float = 0.3, pos_ratio: float = 0.3):
    """Returns (rc, gid, repval, out_order, n_groups) -- same contract as rk_classify
    (all three arrays in output order, length n_out)."""
    x = np.ascontiguousarray(x_start, np.uint64)
    y = np.ascontiguousarray(y_start, np.uint64)
    ln = np.ascontiguousarray(length, np.uint64)
    s = np.ascontiguousarray(strand, np.uint8)
    n = x.shape[0]
    gid = np.empty(n, np.uint32)
    rep = np.empty(n, np.uint8)
    order = np.empty(n, np.uint32)
    n_out, n_groups = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = lib().rko_classify(n, _p(x), _p(y), _p(ln), _p(s), len_x_hdr, len_y_hdr, len_ratio,
                            pos_ratio, _p(gid), _p(rep), _p(order), ctypes.byref(n_out),
                            ctypes.byref(n_groups))
    k = n_out.value
    return rc, gid[:k].copy(), rep[:k].copy(), order[:k].copy(), int(n_groups.value)


REC = np.dtype([("key", np.uint64), ("tag", np.uint32), ("pad", np.uint32)])


def std_sort(keys: np.ndarray) -> np.ndarray:
    """libstdc++ std::sort permutation of `keys` (restated): returns the tags in sorted order."""
    r = np.zeros(keys.shape[0], REC)
    r["key"] = keys
    r["tag"] = np.arange(keys.shape[0], dtype=np.uint32)
    lib().rko_std_sort(_p(r), r.shape[0])
    return r["tag"].copy()


def run_cli(binary: str, inp: str, out: str, lr: float = 0.3, pr: float = 0.3,
            timeout: float = 600.0):
    """Run rk_oracle / ref_driver / repkiller_fix; returns (returncode, stderr)."""
    p = subprocess.run([binary, inp, out, repr(lr), repr(pr)], capture_output=True, text=True,
                       timeout=timeout)
    return p.returncode, p.stderr
