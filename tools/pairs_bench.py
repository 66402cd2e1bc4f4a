#!/usr/bin/env python3
"""Several (len_ratio, pos_ratio) pairs over one fragment set: one
rk_classify_device_pairs call against the same pairs as separate
rk_classify_device calls (the reference re-runs the whole
path per pair, repkiller.cpp:60-72).  Device-resident inputs; prints one JSON
line with device milliseconds per variant and checks the results agree.

  python tools/pairs_bench.py [--n 50000000] [--genome 3000000000] [--pairs 4]
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import repkiller_amd as rk  # noqa: E402

RATIOS = [(0.3, 0.3), (0.05, 0.05), (1.5, 0.7), (0.3, 2.0), (0.1, 0.5), (0.7, 0.1),
          (2.0, 2.0), (0.2, 0.2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000_000)
    ap.add_argument("--genome", type=int, default=3_000_000_000)
    ap.add_argument("--pairs", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    pairs = RATIOS[:a.pairs]
    q, L = len(pairs), a.genome
    f = rk.synth(a.n, L, seed=3)
    dev = torch.device("cuda", 0)
    t = lambda v: torch.from_numpy(v.view(np.int64) if v.dtype == np.uint64 else v).to(dev)
    x, y, ln, s = t(f.x_start), t(f.y_start), t(f.length), t(f.strand)
    n = f.n
    del f
    gid = torch.empty((q, n), dtype=torch.int32, device=dev)
    rep = torch.empty((q, n), dtype=torch.uint8, device=dev)
    order = torch.empty((q, n), dtype=torch.int32, device=dev)
    ctx = rk.Context(0)
    lib = rk.load_library()
    soa = rk.FragsSoA(x.data_ptr(), y.data_ptr(), ln.data_ptr(), s.data_ptr(), n)
    prm = (rk.Params * q)(*[rk.Params(L, L, lr, pr) for lr, pr in pairs])
    res = (rk.Result * q)(*[rk.Result(order[i].data_ptr(), gid[i].data_ptr(), rep[i].data_ptr(),
                                      0, 0) for i in range(q)])
    st = rk.Stats()

    def batched():
        rk._check(lib.rk_classify_device_pairs(ctx._h, ctypes.byref(soa), prm, q, res),
                  ctx.last_error())
        lib.rk_get_stats(ctx._h, ctypes.byref(st))
        return st.device_ms

    def single():
        tot = 0.0
        for i in range(q):
            rk._check(lib.rk_classify_device(ctx._h, ctypes.byref(soa), ctypes.byref(prm[i]),
                                             ctypes.byref(res[i])), ctx.last_error())
            lib.rk_get_stats(ctx._h, ctypes.byref(st))
            tot += st.device_ms
        return tot

    single()  # warm-up (workspace allocation)
    ref = [(int(res[i].n_groups), torch.clone(order[i]), torch.clone(gid[i])) for i in range(q)]
    t_single = min(single() for _ in range(a.reps))
    t_batched = min(batched() for _ in range(a.reps))
    same = all(int(res[i].n_groups) == ref[i][0] and torch.equal(order[i], ref[i][1])
               and torch.equal(gid[i], ref[i][2]) for i in range(q))
    print(json.dumps({"fragments": n, "genome_bp": L, "pairs": pairs,
                      "separate_ms": round(t_single, 3), "batched_ms": round(t_batched, 3),
                      "speedup": round(t_single / t_batched, 3),
                      "pairs_per_s_batched": round(q / (t_batched / 1e3), 2),
                      "frag_pairs_per_s_batched": round(n * q / (t_batched / 1e3), 0),
                      "identical": same}), flush=True)


if __name__ == "__main__":
    main()
