"""rk_classify's host boundary (rk_io.hip): host SoA in, host results out.

The reference classifies fragments held in host memory (FragmentsDatabase,
FragmentsDatabase.cpp:84-97) and saves host-side results (save_frag_pair,
commonFunctions.cpp:119-129).  rk_classify uploads through a copy stream --
page-locked buffers by DMA, pageable ones through a ring of 32-MB pinned
staging slots filled by host threads -- and downloads the same way.  These
tests check that every route gives the bytes the device entry point gives,
including inputs that span several staging slots and row counts that end
mid-slot, and that the transfer times are reported.
"""
import numpy as np
import pytest
import torch

import repkiller_amd as rk
from oracle import rk_oracle as ro

pytestmark = pytest.mark.gpu


def device_result(ctx, f, L, lr=0.3, pr=0.3):
    dev = torch.device("cuda", 0)
    cols = [torch.from_numpy(np.ascontiguousarray(a).view(np.int64) if a.dtype == np.uint64
                             else np.ascontiguousarray(a)).to(dev)
            for a in (f.x_start, f.y_start, f.length, f.strand)]
    n = f.n
    gid = torch.empty(n, dtype=torch.int32, device=dev)
    rep = torch.empty(n, dtype=torch.uint8, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    n_out, ng = ctx.classify_device(*cols, gid, rep, order, L, L, lr, pr)
    return (gid[:n_out].cpu().numpy().view(np.uint32), rep[:n_out].cpu().numpy(),
            order[:n_out].cpu().numpy().view(np.uint32), ng)


_PINNED = []  # the pinned tensors behind the numpy views


def pinned_copy(a: np.ndarray) -> np.ndarray:
    t = torch.empty(a.shape[0], dtype={np.uint64: torch.int64, np.uint8: torch.uint8,
                                        np.uint32: torch.int32}[a.dtype.type], pin_memory=True)
    _PINNED.append(t)
    h = t.numpy().view(a.dtype)
    h[:] = a
    return h


@pytest.mark.parametrize("n", [5_000_003, 300_000])
def test_pageable_and_pinned_match_device(gpu_ctx, n):
    """5M rows = 40 MB per u64 column: every column spans two staging slots and
    ends mid-slot; 300k rows fit one slot."""
    L = 300_000_000 if n > 1_000_000 else 20_000_000
    f = rk.synth(n, L, seed=71)
    want = device_result(gpu_ctx, f, L)
    got = gpu_ctx.classify(f, L, L, 0.3, 0.3)  # numpy buffers: pageable
    st = gpu_ctx.stats()
    assert got.n_groups == want[3]
    assert np.array_equal(got.gid, want[0])
    assert np.array_equal(got.repval, want[1])
    assert np.array_equal(got.out_order, want[2])
    assert st["h2d_ms"] > 0 and st["d2h_ms"] > 0
    # page-locked inputs and outputs (DMA straight from / into them)
    fp = rk.Frags(*[pinned_copy(a) for a in (f.x_start, f.y_start, f.length, f.strand)])
    gid = pinned_copy(np.zeros(n, np.uint32))
    rep = pinned_copy(np.zeros(n, np.uint8))
    order = pinned_copy(np.zeros(n, np.uint32))
    n_out, ng = gpu_ctx.classify_into(fp, L, L, 0.3, 0.3, gid, rep, order)
    assert ng == want[3] and n_out == want[0].shape[0]
    assert np.array_equal(gid[:n_out], want[0])
    assert np.array_equal(rep[:n_out], want[1])
    assert np.array_equal(order[:n_out], want[2])


def test_mixed_pinned_and_pageable(gpu_ctx):
    """Some columns page-locked, some not, in one call."""
    n, L = 1_200_000, 100_000_000
    f = rk.synth(n, L, seed=72)
    want = device_result(gpu_ctx, f, L)
    fm = rk.Frags(pinned_copy(f.x_start), f.y_start.copy(), pinned_copy(f.length),
                  f.strand.copy())
    gid = np.zeros(n, np.uint32)
    rep = pinned_copy(np.zeros(n, np.uint8))
    order = np.zeros(n, np.uint32)
    n_out, ng = gpu_ctx.classify_into(fm, L, L, 0.3, 0.3, gid, rep, order)
    assert ng == want[3]
    assert np.array_equal(gid[:n_out], want[0])
    assert np.array_equal(rep[:n_out], want[1])
    assert np.array_equal(order[:n_out], want[2])


@pytest.mark.parametrize("n", [0, 1, 17, 4097])
def test_tiny_host_inputs_vs_oracle(gpu_ctx, n):
    L = 1_000_000
    f = rk.synth(max(n, 1), L, seed=73)
    if n == 0:
        f = rk.Frags(*[a[:0].copy() for a in (f.x_start, f.y_start, f.length, f.strand)])
    got = gpu_ctx.classify(f, L, L, 0.3, 0.3)
    rc, gid, rep, order, ng = ro.classify(f.x_start, f.y_start, f.length, f.strand, L, L, 0.3, 0.3)
    assert rc == 0 and got.n_groups == ng
    assert np.array_equal(got.out_order, order)
    assert np.array_equal(got.gid, gid)
    assert np.array_equal(got.repval, rep)
