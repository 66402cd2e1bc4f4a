#!/usr/bin/env python3
"""Time the libstdc++ depth-limit heapsort fallback on McIlroy median-of-3
killers (tests/sort_cases.py) through rk_std_sort_segments, and check the
permutation against the oracle's restated std::sort (test infrastructure).
usage: heap_killer_check.py [--tied] [n ...]   (keys from tools/mb/killer_<n>.npy
when present, else generated; the killer's heap segment is all-equal keys.
--tied also times each killer with its never-compared members re-keyed over 3
values, `killer_with_keys(n, 3, 1)`, whose heap segment is heavily tied)"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import repkiller_amd as rk  # noqa: E402
from oracle import rk_oracle as ro  # noqa: E402
from sort_cases import mcilroy_killer  # noqa: E402

out = []
ctx = rk.Context(0)
args = sys.argv[1:]
tied = "--tied" in args
cases = []
for n in [int(a) for a in args if a != "--tied"] or [100000]:
    path = os.path.join(ROOT, "tools", "mb", f"killer_{n}.npy")
    keys = np.load(path) if os.path.exists(path) else mcilroy_killer(n)
    cases.append((n, "all-equal heap segment", keys))
    if tied:
        gas = keys == keys.max()
        k = keys.copy()
        k[gas] = np.uint64(n + 1) + np.random.default_rng(1).integers(0, 3, int(gas.sum())).astype(np.uint64)
        cases.append((n, "tied heap segment (3 keys)", k))
for n, kind, keys in cases:
    off = np.array([0, n], np.uint32)
    runs = []
    for _ in range(2):  # the first call also pays the context's lazy set-up
        t = time.time()
        perm = ctx.std_sort_segments(keys, off)
        runs.append(time.time() - t)
    gpu_s = min(runs)
    t = time.time()
    ref = ro.std_sort(keys)
    cpu_s = time.time() - t
    ok = bool(np.array_equal(perm, ref))
    rec = {"n": n, "kind": kind, "gpu_s": round(gpu_s, 4), "gpu_first_s": round(runs[0], 4), "oracle_s": round(cpu_s, 4), "bit_exact": ok,
           "equal_keys": int((keys == keys.max()).sum())}
    print(json.dumps(rec), flush=True)
    out.append(rec)
ctx.close()
