#!/usr/bin/env python3
"""Time the libstdc++ depth-limit heapsort fallback on McIlroy median-of-3
killers (tests/sort_cases.py) through rk_std_sort_segments, and check the
permutation against the oracle's restated std::sort (test infrastructure).
usage: heap_killer_check.py [n ...]   (keys from tools/mb/killer_<n>.npy when
present, else generated)"""
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
for n in [int(a) for a in sys.argv[1:]] or [100000]:
    path = os.path.join(ROOT, "tools", "mb", f"killer_{n}.npy")
    keys = np.load(path) if os.path.exists(path) else mcilroy_killer(n)
    off = np.array([0, n], np.uint32)
    t = time.time()
    perm = ctx.std_sort_segments(keys, off)
    gpu_s = time.time() - t
    t = time.time()
    ref = ro.std_sort(keys)
    cpu_s = time.time() - t
    ok = bool(np.array_equal(perm, ref))
    rec = {"n": n, "gpu_s": round(gpu_s, 4), "oracle_s": round(cpu_s, 4), "bit_exact": ok,
           "equal_keys": int((keys == keys.max()).sum())}
    print(json.dumps(rec), flush=True)
    out.append(rec)
ctx.close()
