"""repkiller_amd -- MI355X-native repeat-fragment classifier (estebanpw/repkiller hot path).

Python binding over the C ABI in ``include/repkiller_amd.h`` (``librepkiller_amd.so``,
built in-tree by ``make -C repkiller_amd/csrc``).  The classification runs only
on a gfx950 GPU through hand-written HIP kernels; there is no CPU fallback --
:class:`Context` raises if the library or the device is missing.

Mapping to the reference (``/root/reference/src``):

=====================================  ============================================
reference                              here
=====================================  ============================================
``FragmentsDatabase(ifstream&, ...)``  :class:`FragmentsDatabase` (``rk_db_load_csv``)
``generate_fragment_groups`` +         :meth:`Context.classify` /
``generate_diagonal_func`` +           :meth:`Context.classify_device`
``sort_groups`` + repeat flag          (``rk_classify`` / ``rk_classify_device``)
``save_all_frag_pairs``                :meth:`FragmentsDatabase.save_all_frag_pairs`
``SaverQueue``                         :class:`SaverQueue` (``rk_saver_*``)
=====================================  ============================================
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RK_LIB=<path>: load another build of the library (A/B measurements)
LIB_PATH = os.environ.get("RK_LIB") or os.path.join(_HERE, "librepkiller_amd.so")
CLI_PATH = os.path.join(_HERE, "bin", "rk_repkiller")

RK_OK = 0
N_PHASES = 10  # RK_N_PHASES
STATUS = {
    0: "RK_OK", -1: "RK_E_ARG", -2: "RK_E_IO", -3: "RK_E_COUNT", -4: "RK_E_UB_BUCKET",
    -5: "RK_E_UB_CENTER", -6: "RK_E_NOMEM", -7: "RK_E_HIP", -8: "RK_E_NODEVICE",
    -9: "RK_E_TOO_MANY", -10: "RK_E_INTERNAL", -11: "RK_E_PEER",
}

# every symbol include/repkiller_amd.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "rk_create", "rk_destroy", "rk_last_error", "rk_classify", "rk_classify_device",
    "rk_classify_pairs", "rk_classify_device_pairs",
    "rk_get_stats", "rk_std_sort_segments", "rk_set_profiling", "rk_get_phase_ms", "rk_reset_phases", "rk_phase_name",
    "rk_get_kernel_timing", "rk_kernel_count", "rk_kernel_name",
    "rk_db_load_csv", "rk_db_free", "rk_db_view", "rk_db_write_csv",
    "rk_db_save_soa", "rk_db_load_soa", "rk_saver_start", "rk_saver_add", "rk_saver_stop", "rk_synth_generate",
    "rk_synth_write_csv", "rk_comm_create_host", "rk_comm_rccl_id", "rk_comm_create_rccl",
    "rk_comm_destroy", "rk_comm_last_error", "rk_classify_sharded", "rk_get_shard_stats",
    "rk_shard_copy_result", "rk_comm_create_local", "rk_classify_sharded_host",
    "rk_comm_abandon", "rk_set_pipeline",
)


class RkError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{STATUS.get(code, code)}{': ' + msg if msg else ''}")


_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


class FragsSoA(ctypes.Structure):
    _fields_ = [("x_start", ctypes.c_void_p), ("y_start", ctypes.c_void_p),
                ("length", ctypes.c_void_p), ("strand", ctypes.c_void_p), ("n", ctypes.c_uint64)]


class Params(ctypes.Structure):
    _fields_ = [("len_x_hdr", ctypes.c_uint64), ("len_y_hdr", ctypes.c_uint64),
                ("len_ratio", ctypes.c_double), ("pos_ratio", ctypes.c_double)]


class Result(ctypes.Structure):
    _fields_ = [("out_order", ctypes.c_void_p), ("gid", ctypes.c_void_p),
                ("repval", ctypes.c_void_p), ("n_out", ctypes.c_uint64),
                ("n_groups", ctypes.c_uint64)]


class Stats(ctypes.Structure):
    _fields_ = [("n_in", ctypes.c_uint64), ("n_proc", ctypes.c_uint64),
                ("n_groups", ctypes.c_uint64), ("x_sweeps", ctypes.c_uint32),
                ("y_sweeps", ctypes.c_uint32), ("jump_rounds", ctypes.c_uint32),
                ("x_hits", ctypes.c_uint64), ("y_hits", ctypes.c_uint64),
                ("device_ms", ctypes.c_double), ("pipeline", ctypes.c_uint32),
                ("record_fallback", ctypes.c_uint32), ("h2d_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double), ("wire", ctypes.c_uint32),
                ("sweep_repeats", ctypes.c_uint32), ("numa_input", ctypes.c_int32),
                ("numa_threads", ctypes.c_int32), ("numa_staging", ctypes.c_int32),
                ("numa_gpu", ctypes.c_int32)]


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_uint64)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64), ctypes.c_void_p,
                                ctypes.POINTER(ctypes.c_uint64))


class CommHostOps(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("allgather", ALLGATHER_FN),
                ("alltoallv", ALLTOALLV_FN)]


class ShardResult(ctypes.Structure):
    _fields_ = [("out_order", ctypes.c_void_p), ("gid", ctypes.c_void_p),
                ("repval", ctypes.c_void_p), ("n_out", ctypes.c_uint64),
                ("out_offset", ctypes.c_uint64), ("n_out_total", ctypes.c_uint64),
                ("n_groups", ctypes.c_uint64)]


class ShardStats(ctypes.Structure):
    _fields_ = [("n_in", ctypes.c_uint64), ("n_total", ctypes.c_uint64),
                ("n_slice", ctypes.c_uint64), ("x_ghosts", ctypes.c_uint64),
                ("y_entries", ctypes.c_uint64), ("x_rounds", ctypes.c_uint32),
                ("y_rounds", ctypes.c_uint32), ("x_reruns", ctypes.c_uint32),
                ("y_reruns", ctypes.c_uint32), ("root_rounds", ctypes.c_uint32),
                ("bytes_sent", ctypes.c_uint64), ("ms_total", ctypes.c_double),
                ("ms_ingress", ctypes.c_double), ("ms_x", ctypes.c_double),
                ("ms_y", ctypes.c_double), ("ms_roots", ctypes.c_double),
                ("ms_members", ctypes.c_double), ("generic_driver", ctypes.c_uint32),
                ("order_split", ctypes.c_uint32), ("gathers", ctypes.c_uint32),
                ("exchanges", ctypes.c_uint32), ("host_syncs", ctypes.c_uint32),
                ("agree_skipped", ctypes.c_uint32), ("fast_path", ctypes.c_uint32),
                ("fast_retry", ctypes.c_uint32), ("fast_stages", ctypes.c_uint32)]


class SynthParams(ctypes.Structure):
    _fields_ = [("n", ctypes.c_uint64), ("genome_len", ctypes.c_uint64),
                ("seed", ctypes.c_uint64), ("family_frac", ctypes.c_double),
                ("copies_lo", ctypes.c_uint32), ("copies_hi", ctypes.c_uint32)]


_lib = None


def load_library() -> ctypes.CDLL:
    """Load librepkiller_amd.so; raise loudly when it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64.so.7; when it is imported AFTER this library
    # the process ends up with two HIP runtimes and torch.cuda cannot initialise.
    # Importing it first makes both share one runtime (SONAME match).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} missing: run `make -C repkiller_amd/csrc` "
                           "(or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    sig = {
        "rk_create": (ctypes.c_int, [ctypes.POINTER(vp), ctypes.c_int]),
        "rk_destroy": (None, [vp]),
        "rk_last_error": (ctypes.c_char_p, [vp]),
        "rk_classify": (ctypes.c_int, [vp, ctypes.POINTER(FragsSoA), ctypes.POINTER(Params),
                                       ctypes.POINTER(Result)]),
        "rk_classify_device": (ctypes.c_int, [vp, ctypes.POINTER(FragsSoA),
                                              ctypes.POINTER(Params), ctypes.POINTER(Result)]),
        "rk_classify_pairs": (ctypes.c_int, [vp, ctypes.POINTER(FragsSoA),
                                             ctypes.POINTER(Params), ctypes.c_uint32,
                                             ctypes.POINTER(Result)]),
        "rk_classify_device_pairs": (ctypes.c_int, [vp, ctypes.POINTER(FragsSoA),
                                                    ctypes.POINTER(Params), ctypes.c_uint32,
                                                    ctypes.POINTER(Result)]),
        "rk_get_stats": (ctypes.c_int, [vp, ctypes.POINTER(Stats)]),
        "rk_set_profiling": (ctypes.c_int, [vp, ctypes.c_int]),
        "rk_std_sort_segments": (ctypes.c_int, [vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32,
                                                vp]),
        "rk_get_phase_ms": (ctypes.c_int, [vp, ctypes.POINTER(ctypes.c_double), _u32p]),
        "rk_reset_phases": (ctypes.c_int, [vp]),
        "rk_get_kernel_timing": (ctypes.c_int, [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                ctypes.POINTER(ctypes.c_double), _u64p]),
        "rk_kernel_count": (ctypes.c_int, []),
        "rk_kernel_name": (ctypes.c_char_p, [ctypes.c_int]),
        "rk_phase_name": (ctypes.c_char_p, [ctypes.c_int]),
        "rk_db_load_csv": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(vp)]),
        "rk_db_free": (None, [vp]),
        "rk_db_save_soa": (ctypes.c_int, [vp, ctypes.c_char_p]),
        "rk_db_load_soa": (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(vp)]),
        "rk_db_view": (ctypes.c_int, [vp, ctypes.POINTER(FragsSoA), _u64p, _u64p, _u64p]),
        "rk_db_write_csv": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(Result)]),
        "rk_saver_start": (ctypes.c_int, [vp, ctypes.POINTER(vp)]),
        "rk_saver_add": (ctypes.c_int, [vp, ctypes.c_char_p, ctypes.POINTER(Result),
                                        ctypes.c_uint64]),
        "rk_saver_stop": (ctypes.c_int, [vp]),
        "rk_synth_generate": (ctypes.c_int, [ctypes.POINTER(SynthParams), vp, vp, vp, vp, vp]),
        "rk_synth_write_csv": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint64, vp, vp, vp, vp,
                                              vp, ctypes.c_uint64, ctypes.c_uint64]),
        "rk_comm_create_host": (ctypes.c_int, [ctypes.c_int, ctypes.c_int,
                                               ctypes.POINTER(CommHostOps), ctypes.POINTER(vp)]),
        "rk_comm_rccl_id": (ctypes.c_int, [vp]),
        "rk_comm_create_rccl": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, vp,
                                               ctypes.POINTER(vp)]),
        "rk_comm_destroy": (None, [vp]),
        "rk_comm_last_error": (ctypes.c_char_p, [vp]),
        "rk_comm_abandon": (ctypes.c_int, [vp, ctypes.c_int]),
        "rk_set_pipeline": (ctypes.c_int, [vp, ctypes.c_int]),
        "rk_classify_sharded": (ctypes.c_int, [vp, vp, ctypes.POINTER(FragsSoA),
                                               ctypes.POINTER(Params), ctypes.c_int32,
                                               ctypes.POINTER(ShardResult)]),
        "rk_get_shard_stats": (ctypes.c_int, [vp, ctypes.POINTER(ShardStats)]),
        "rk_comm_create_local": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(vp)]),
        "rk_classify_sharded_host": (ctypes.c_int, [vp, vp, ctypes.POINTER(FragsSoA),
                                                    ctypes.POINTER(Params), ctypes.c_int32,
                                                    ctypes.POINTER(ShardResult)]),
        "rk_shard_copy_result": (ctypes.c_int, [vp, ctypes.POINTER(ShardResult), vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _check(rc: int, msg: str = ""):
    if rc != RK_OK:
        raise RkError(rc, msg)


# --------------------------------------------------------------- synthetic --

@dataclass
class Frags:
    """Fragments in FILE order (what FragmentsDatabase reads, SoA)."""
    x_start: np.ndarray
    y_start: np.ndarray
    length: np.ndarray
    strand: np.ndarray
    ident: np.ndarray | None = None

    @property
    def n(self) -> int:
        return int(self.x_start.shape[0])


def synth(n: int, genome_len: int, seed: int, family_frac: float = 0.8,
          copies: tuple[int, int] = (2, 30), with_ident: bool = True) -> Frags:
    """Deterministic synthetic fragment set (SURVEY.md §8d generator).
    with_ident=False skips the identity column (only the CSV writer reads it)."""
    lib = load_library()
    f = Frags(np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.uint64),
              np.empty(n, np.uint8), np.empty(n, np.uint64) if with_ident else None)
    p = SynthParams(n, genome_len, seed, family_frac, copies[0], copies[1])
    _check(lib.rk_synth_generate(ctypes.byref(p), _ptr(f.x_start), _ptr(f.y_start),
                                 _ptr(f.length), _ptr(f.strand),
                                 _ptr(f.ident) if f.ident is not None else 0))
    return f


def write_input_csv(path: str, f: Frags, len_x_hdr: int, len_y_hdr: int) -> None:
    lib = load_library()
    ident = f.ident if f.ident is not None else f.length
    _check(lib.rk_synth_write_csv(path.encode(), f.n, _ptr(f.x_start), _ptr(f.y_start),
                                  _ptr(f.length), _ptr(f.strand), _ptr(ident),
                                  len_x_hdr, len_y_hdr))


# ------------------------------------------------------------------ ingress --

@dataclass
class ClassifyResult:
    """All arrays in OUTPUT order (length n_out): row k of the reference's CSV is
    input row out_order[k], with group id gid[k] and repeat flag repval[k]."""
    gid: np.ndarray        # uint32 group id (block column, creation order)
    repval: np.ndarray     # uint8 0 singleton / 1 representative / 2 repeated
    out_order: np.ndarray  # uint32 input row
    n_groups: int

    def as_struct(self) -> Result:
        return Result(_ptr(self.out_order), _ptr(self.gid), _ptr(self.repval),
                      int(self.out_order.shape[0]), self.n_groups)


class FragmentsDatabase:
    """Parsed fragment CSV (FragmentsDatabase.cpp:17-101 acceptance rules)."""

    def __init__(self, path: str, soa: bool = False):
        """path: the fragment CSV, or with soa=True a binary SoA cache written by
        save_soa (the parsed columns: no parse at all)."""
        lib = load_library()
        h = ctypes.c_void_p()
        rc = (lib.rk_db_load_soa if soa else lib.rk_db_load_csv)(path.encode(), ctypes.byref(h))
        if rc == -2:
            raise RkError(rc, f"Could not open input file {path}.")
        if rc == -3:
            raise RkError(rc, "Unexpected number of fragments")
        if rc == -1 and soa:
            raise RkError(rc, f"{path} is not a complete SoA cache file")
        _check(rc)
        self._h = h
        soa = FragsSoA()
        lx, ly, tot = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _check(lib.rk_db_view(h, ctypes.byref(soa), ctypes.byref(lx), ctypes.byref(ly),
                              ctypes.byref(tot)))
        self.len_x_hdr, self.len_y_hdr, self.total_hdr = lx.value, ly.value, tot.value
        n = soa.n

        def view(ptr, dtype, count):
            if count == 0:
                return np.empty(0, dtype)
            buf = (ctypes.c_uint8 * (count * np.dtype(dtype).itemsize)).from_address(ptr)
            return np.frombuffer(buf, dtype=dtype).copy()

        self.frags = Frags(view(soa.x_start, np.uint64, n), view(soa.y_start, np.uint64, n),
                           view(soa.length, np.uint64, n), view(soa.strand, np.uint8, n))

    @classmethod
    def load_soa(cls, path: str) -> "FragmentsDatabase":
        """A database from a binary SoA cache (rk_db_load_soa)."""
        return cls(path, soa=True)

    def save_soa(self, path: str) -> None:
        """The parsed columns as a binary SoA cache (rk_db_save_soa)."""
        rc = load_library().rk_db_save_soa(self._h, path.encode())
        if rc == -2:
            raise RkError(rc, f"Could not write {path}")
        _check(rc)

    def getTotalFrags(self) -> int:  # FragmentsDatabase.h:32
        return self.frags.n

    def getA(self) -> int:  # FragmentsDatabase.h:23 (vsize)
        return 1 + (self.len_x_hdr + 1) // 10

    def save_all_frag_pairs(self, path: str, res: ClassifyResult) -> None:
        """commonFunctions.cpp:131-146 (header echo + one line per member)."""
        r = res.as_struct()
        rc = load_library().rk_db_write_csv(self._h, path.encode(), ctypes.byref(r))
        if rc == -2:
            raise RkError(rc, "Could not open output directory " + path)
        _check(rc)

    def close(self):
        if getattr(self, "_h", None):
            load_library().rk_db_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SaverQueue:
    """SaverQueue.h:37-41 -- background CSV writer (start / addRequest / stop)."""

    def __init__(self, db: FragmentsDatabase):
        self._db = db
        self._h = ctypes.c_void_p()
        _check(load_library().rk_saver_start(db._h, ctypes.byref(self._h)))

    def addRequest(self, path: str, res: ClassifyResult) -> None:
        r = res.as_struct()
        _check(load_library().rk_saver_add(self._h, path.encode(), ctypes.byref(r),
                                           int(res.gid.shape[0])))

    def stop(self) -> None:
        if self._h:
            rc = load_library().rk_saver_stop(self._h)
            self._h = None
            _check(rc)


# ----------------------------------------------------------- classification --

class Context:
    """One device + stream + workspace (rk_ctx).  GPU only."""

    def __init__(self, device: int = 0):
        lib = load_library()
        self._h = ctypes.c_void_p()
        rc = lib.rk_create(ctypes.byref(self._h), device)
        if rc != RK_OK:
            raise RkError(rc, f"rk_create(device={device}) failed: a gfx950 GPU is required "
                              "(no CPU fallback)")
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            load_library().rk_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        return load_library().rk_last_error(self._h).decode()

    def stats(self) -> dict:
        s = Stats()
        _check(load_library().rk_get_stats(self._h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in Stats._fields_}

    def set_pipeline(self, pipeline: str) -> None:
        """'auto' (the record pipeline where rows pack into 16-B records) or
        'generic' (rk_set_pipeline)."""
        _check(load_library().rk_set_pipeline(self._h, {"auto": 0, "generic": 1}[pipeline]))

    def set_profiling(self, on: bool = True, only: str | None = None) -> None:
        """Phase events and launch timing on/off; `only` = a kernel name
        (rk_kernel_name) restricts the launch timing to that kernel."""
        lib = load_library()
        mode = int(bool(on))
        if on and only:
            names = [lib.rk_kernel_name(k).decode() for k in range(lib.rk_kernel_count())]
            mode = 2 + names.index(only)
        _check(lib.rk_set_profiling(self._h, mode))

    def reset_phases(self) -> None:
        _check(load_library().rk_reset_phases(self._h))

    def phases(self) -> dict:
        """{phase name: (accumulated device ms, calls)} since the last reset."""
        lib = load_library()
        ms = (ctypes.c_double * N_PHASES)()
        calls = (ctypes.c_uint32 * N_PHASES)()
        _check(lib.rk_get_phase_ms(self._h, ms, calls))
        return {lib.rk_phase_name(i).decode(): (ms[i], calls[i]) for i in range(N_PHASES)}

    def std_sort_segments(self, keys: np.ndarray, seg_off: np.ndarray) -> np.ndarray:
        """libstdc++ std::sort permutation of every segment of `keys`, on the GPU."""
        k = np.ascontiguousarray(keys, np.uint64)
        off = np.ascontiguousarray(seg_off, np.uint32)
        perm = np.empty(k.shape[0], np.uint32)
        rc = load_library().rk_std_sort_segments(self._h, _ptr(k), k.shape[0], _ptr(off),
                                                 off.shape[0] - 1, _ptr(perm))
        if rc != RK_OK:
            raise RkError(rc, self.last_error())
        return perm

    def kernel_timing(self) -> dict:
        """Per-kernel HIP-event timing while profiling:
        {name: {"total_ms", "algo_bytes", "launches"}} for kernels that ran."""
        lib = load_library()
        out = {}
        for k in range(lib.rk_kernel_count()):
            ms, by, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_uint64()
            _check(lib.rk_get_kernel_timing(self._h, k, ctypes.byref(ms), ctypes.byref(by),
                                            ctypes.byref(n)))
            if n.value:
                out[lib.rk_kernel_name(k).decode()] = {"total_ms": ms.value, "algo_bytes": by.value,
                                                       "launches": n.value}
        return out

    def classify(self, f: Frags, len_x_hdr: int, len_y_hdr: int, len_ratio: float = 0.3,
                 pos_ratio: float = 0.3) -> ClassifyResult:
        """Host arrays in, host arrays out (rk_classify)."""
        n = f.n
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((f.x_start, np.uint64), (f.y_start, np.uint64), (f.length, np.uint64),
                 (f.strand, np.uint8))]
        soa = FragsSoA(_ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), _ptr(arrs[3]), n)
        gid = np.empty(n, np.uint32)
        rep = np.empty(n, np.uint8)
        order = np.empty(n, np.uint32)
        res = Result(_ptr(order), _ptr(gid), _ptr(rep), 0, 0)
        prm = Params(len_x_hdr, len_y_hdr, len_ratio, pos_ratio)
        rc = load_library().rk_classify(self._h, ctypes.byref(soa), ctypes.byref(prm),
                                        ctypes.byref(res))
        if rc != RK_OK:
            raise RkError(rc, self.last_error())
        k = res.n_out
        return ClassifyResult(gid[:k].copy(), rep[:k].copy(), order[:k].copy(), int(res.n_groups))

    def classify_into(self, f: Frags, len_x_hdr: int, len_y_hdr: int, len_ratio: float,
                      pos_ratio: float, gid: np.ndarray, rep: np.ndarray,
                      order: np.ndarray) -> tuple:
        """rk_classify into caller-owned host arrays (no copies; the arrays may
        be page-locked, e.g. views of pinned torch tensors).  Returns
        (n_out, n_groups)."""
        n = f.n
        for a, t in ((f.x_start, np.uint64), (f.y_start, np.uint64), (f.length, np.uint64),
                     (f.strand, np.uint8), (gid, np.uint32), (rep, np.uint8), (order, np.uint32)):
            if a.dtype != t or not a.flags.c_contiguous or a.shape[0] < n:
                raise ValueError("classify_into: contiguous arrays of the ABI dtypes required")
        soa = FragsSoA(_ptr(f.x_start), _ptr(f.y_start), _ptr(f.length), _ptr(f.strand), n)
        res = Result(_ptr(order), _ptr(gid), _ptr(rep), 0, 0)
        prm = Params(len_x_hdr, len_y_hdr, len_ratio, pos_ratio)
        rc = load_library().rk_classify(self._h, ctypes.byref(soa), ctypes.byref(prm),
                                        ctypes.byref(res))
        if rc != RK_OK:
            raise RkError(rc, self.last_error())
        return int(res.n_out), int(res.n_groups)

    def classify_pairs(self, f: Frags, len_x_hdr: int, len_y_hdr: int,
                       pairs) -> list:
        """Several (len_ratio, pos_ratio) pairs over one fragment set
        (rk_classify_pairs; the pair loop of repkiller.cpp:60-72)."""
        pairs = list(pairs)
        n, q = f.n, len(pairs)
        arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
                ((f.x_start, np.uint64), (f.y_start, np.uint64), (f.length, np.uint64),
                 (f.strand, np.uint8))]
        soa = FragsSoA(_ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2]), _ptr(arrs[3]), n)
        gid = np.empty((q, n), np.uint32)
        rep = np.empty((q, n), np.uint8)
        order = np.empty((q, n), np.uint32)
        res = (Result * max(q, 1))()
        prm = (Params * max(q, 1))()
        for i, (lr, pr) in enumerate(pairs):
            res[i] = Result(_ptr(order[i]), _ptr(gid[i]), _ptr(rep[i]), 0, 0)
            prm[i] = Params(len_x_hdr, len_y_hdr, lr, pr)
        rc = load_library().rk_classify_pairs(self._h, ctypes.byref(soa), prm, q, res)
        if rc != RK_OK:
            raise RkError(rc, self.last_error())
        out = []
        for i in range(q):
            k = res[i].n_out
            out.append(ClassifyResult(gid[i, :k].copy(), rep[i, :k].copy(), order[i, :k].copy(),
                                      int(res[i].n_groups)))
        return out

    def classify_device(self, x, y, length, strand, gid, repval, out_order, len_x_hdr: int,
                        len_y_hdr: int, len_ratio: float = 0.3, pos_ratio: float = 0.3):
        """Device tensors (torch, on this context's GPU) in and out (rk_classify_device).

        Returns (n_out, n_groups).  Inputs: uint64/int64 x, y, length and uint8 strand;
        outputs: int32/uint32 gid and out_order, uint8 repval, all of length n, the
        first n_out entries filled in output order.
        """
        n = int(x.shape[0])
        soa = FragsSoA(x.data_ptr(), y.data_ptr(), length.data_ptr(), strand.data_ptr(), n)
        res = Result(out_order.data_ptr(), gid.data_ptr(), repval.data_ptr(), 0, 0)
        prm = Params(len_x_hdr, len_y_hdr, len_ratio, pos_ratio)
        rc = load_library().rk_classify_device(self._h, ctypes.byref(soa), ctypes.byref(prm),
                                               ctypes.byref(res))
        if rc != RK_OK:
            raise RkError(rc, self.last_error())
        return int(res.n_out), int(res.n_groups)


# ---------------------------------------------------- one set over many GPUs --

class Comm:
    """rk_comm: the collectives rk_classify_sharded runs on.

    ``Comm.rccl(rank, size, device)`` -- RCCL over xGMI (production); the unique
    id is broadcast with the default torch.distributed process group.
    ``Comm.torch_host(rank, size)`` -- host callbacks over the default
    torch.distributed group (gloo): device blocks are staged through host memory.
    """

    def __init__(self, handle, rank: int, size: int, keep=None):
        self._h = handle
        self.rank, self.size = rank, size
        self._keep = keep  # ctypes callbacks must outlive the comm

    @classmethod
    def rccl(cls, rank: int, size: int, device: int) -> "Comm":
        import torch
        import torch.distributed as dist
        lib = load_library()
        ident = (ctypes.c_uint8 * 128)()
        if rank == 0:
            _check(lib.rk_comm_rccl_id(ident), "rk_comm_rccl_id")
        t = torch.tensor(list(bytes(ident)), dtype=torch.uint8)
        if size > 1:
            dist.broadcast(t, src=0)
        ident = (ctypes.c_uint8 * 128)(*t.tolist())
        h = ctypes.c_void_p()
        # RCCL prints an init banner on stdout: keep stdout for the caller's output
        import sys
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            rc = lib.rk_comm_create_rccl(rank, size, device, ident, ctypes.byref(h))
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        _check(rc, "rk_comm_create_rccl")
        return cls(h, rank, size)

    @classmethod
    def torch_host(cls, rank: int, size: int, group=None) -> "Comm":
        import torch
        import torch.distributed as dist

        def allgather(_user, send, recv, nbytes):
            try:
                src = torch.empty(nbytes, dtype=torch.uint8)
                if nbytes:
                    ctypes.memmove(src.data_ptr(), send, nbytes)
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(size)]
                dist.all_gather(outs, src, group=group)
                for q, o in enumerate(outs):
                    if nbytes:
                        ctypes.memmove(recv + q * nbytes, o.data_ptr(), nbytes)
                return 0
            except Exception as e:  # noqa: BLE001 -- reported as a status code
                print(f"rk host allgather failed: {e!r}")
                return 1

        def alltoallv(_user, send, sb, recv, rb):
            try:
                sbl = [int(sb[q]) for q in range(size)]
                rbl = [int(rb[q]) for q in range(size)]
                src = torch.empty(sum(sbl), dtype=torch.uint8)
                if sum(sbl):
                    ctypes.memmove(src.data_ptr(), send, sum(sbl))
                dst = torch.empty(sum(rbl), dtype=torch.uint8)
                dist.all_to_all_single(dst, src, rbl, sbl, group=group)
                if sum(rbl):
                    ctypes.memmove(recv, dst.data_ptr(), sum(rbl))
                return 0
            except Exception as e:  # noqa: BLE001
                print(f"rk host alltoallv failed: {e!r}")
                return 1

        ag, a2a = ALLGATHER_FN(allgather), ALLTOALLV_FN(alltoallv)
        ops = CommHostOps(None, ag, a2a)
        h = ctypes.c_void_p()
        _check(load_library().rk_comm_create_host(rank, size, ctypes.byref(ops),
                                                  ctypes.byref(h)))
        return cls(h, rank, size, keep=(ag, a2a, ops))

    @classmethod
    def local(cls, size: int) -> list["Comm"]:
        """``size`` ranks inside this process (one thread per rank,
        rk_comm_create_local): device blocks move by device copies."""
        hs = (ctypes.c_void_p * size)()
        _check(load_library().rk_comm_create_local(size, hs), "rk_comm_create_local")
        return [cls(ctypes.c_void_p(hs[r]), r, size) for r in range(size)]

    def last_error(self) -> str:
        return load_library().rk_comm_last_error(self._h).decode()

    def close(self):
        if getattr(self, "_h", None):
            load_library().rk_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class ShardOutput:
    """This rank's share of the global output: rows [out_offset, out_offset + n_out)."""
    result: ClassifyResult | None  # host copies (None when not copied)
    out_offset: int
    n_out: int
    n_out_total: int
    n_groups: int
    raw: ShardResult


def classify_sharded(ctx: "Context", comm: Comm, x, y, length, strand, len_x_hdr: int,
                     len_y_hdr: int, len_ratio: float = 0.3, pos_ratio: float = 0.3,
                     lead_in: int = -1, copy: bool = True) -> ShardOutput:
    """rk_classify_sharded on device tensors holding this rank's block of input rows."""
    lib = load_library()
    n = int(x.shape[0])
    soa = FragsSoA(x.data_ptr(), y.data_ptr(), length.data_ptr(), strand.data_ptr(), n)
    prm = Params(len_x_hdr, len_y_hdr, len_ratio, pos_ratio)
    res = ShardResult()
    rc = lib.rk_classify_sharded(ctx._h, comm._h, ctypes.byref(soa), ctypes.byref(prm),
                                 lead_in, ctypes.byref(res))
    if rc != RK_OK:
        raise RkError(rc, ctx.last_error())
    out = ShardOutput(None, int(res.out_offset), int(res.n_out), int(res.n_out_total),
                      int(res.n_groups), res)
    if copy:
        out.result = shard_copy(ctx, out)
    return out


def shard_copy(ctx: "Context", out: ShardOutput) -> ClassifyResult:
    """Host copies of this rank's output share (rk_shard_copy_result) of the last
    rk_classify_sharded call on ``ctx``; global file rows and group ids."""
    k = out.n_out
    order, gid, rep = np.empty(k, np.uint32), np.empty(k, np.uint32), np.empty(k, np.uint8)
    _check(load_library().rk_shard_copy_result(ctx._h, ctypes.byref(out.raw), _ptr(order),
                                               _ptr(gid), _ptr(rep)), ctx.last_error())
    return ClassifyResult(gid, rep, order, out.n_groups)


def classify_sharded_threads(f: Frags, ranks: int, len_x_hdr: int, len_y_hdr: int,
                             len_ratio: float = 0.3, pos_ratio: float = 0.3,
                             devices: list[int] | None = None) -> ClassifyResult:
    """ONE host fragment set over ``ranks`` ranks of this process (the CLI's
    ``--gpus P`` path, rk_cli.cpp): rank r holds the file-order rows
    [n r / P, n (r + 1) / P), runs rk_classify_sharded_host on its own context
    (device ``devices[r]``, default 0 for every rank) and copies its output
    share into the whole result at its offset."""
    import threading
    lib = load_library()
    n = f.n
    devices = devices or [0] * ranks
    comms = Comm.local(ranks)
    order, gid, rep = np.empty(n, np.uint32), np.empty(n, np.uint32), np.empty(n, np.uint8)
    status, errs, totals = [0] * ranks, [""] * ranks, [None] * ranks
    prm = Params(len_x_hdr, len_y_hdr, len_ratio, pos_ratio)

    def rank_body(r):
        h = ctypes.c_void_p()
        status[r] = lib.rk_create(ctypes.byref(h), devices[r])
        if status[r]:
            errs[r] = f"rk_create(device {devices[r]})"
            lib.rk_comm_abandon(comms[r]._h, status[r])
            return
        try:
            a, b = n * r // ranks, n * (r + 1) // ranks
            soa = FragsSoA(*[int(c.ctypes.data) + a * c.itemsize
                             for c in (f.x_start, f.y_start, f.length, f.strand)], b - a)
            res = ShardResult()
            status[r] = lib.rk_classify_sharded_host(h, comms[r]._h, ctypes.byref(soa),
                                                     ctypes.byref(prm), -1, ctypes.byref(res))
            if not status[r]:
                o = int(res.out_offset)
                status[r] = lib.rk_shard_copy_result(
                    h, ctypes.byref(res), order.ctypes.data + 4 * o, gid.ctypes.data + 4 * o,
                    rep.ctypes.data + o)
                totals[r] = (int(res.n_out_total), int(res.n_groups))
            if status[r]:
                errs[r] = lib.rk_last_error(h).decode()
        finally:
            lib.rk_destroy(h)

    threads = [threading.Thread(target=rank_body, args=(r,)) for r in range(ranks)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for c in comms:
        c.close()
    for r in range(ranks):
        if status[r]:
            raise RkError(status[r], f"rank {r}: {errs[r]}")
    n_out, ng = totals[0]
    assert all(t == totals[0] for t in totals), totals
    return ClassifyResult(gid[:n_out], rep[:n_out], order[:n_out], ng)


def shard_stats(ctx: "Context") -> dict:
    s = ShardStats()
    _check(load_library().rk_get_shard_stats(ctx._h, ctypes.byref(s)))
    return {k: getattr(s, k) for k, _ in ShardStats._fields_}


def build(jobs: int = 8) -> None:
    """Compile librepkiller_amd.so + the CLI for gfx950 (hipcc cross-compiles without a GPU)."""
    import subprocess
    subprocess.run(["make", "-C", os.path.join(_HERE, "csrc"), f"-j{jobs}"], check=True)
