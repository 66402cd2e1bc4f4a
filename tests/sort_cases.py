"""Key sequences for the std::sort parity tests (CPU and GPU).

`mcilroy_killer(n)` builds, with McIlroy's "antiqsort" adversary run against
the libstdc++ introsort control flow, an input on which the depth limit is
hit and the heapsort fallback runs (checked by `heap_fallbacks`).
"""
import math

import numpy as np


def _introsort_trace(n, less):
    """libstdc++ __introsort_loop over items 0..n-1 with comparator `less`;
    returns the number of depth-limit (heapsort) fallbacks."""
    a = list(range(n))
    hits = [0]

    def loop(f, l, d):
        while l - f > 16:
            if d == 0:
                hits[0] += 1
                return
            d -= 1
            A, B, C = f + 1, f + (l - f) // 2, l - 1
            if less(a[A], a[B]):
                m = B if less(a[B], a[C]) else (C if less(a[A], a[C]) else A)
            else:
                m = A if less(a[A], a[C]) else (C if less(a[B], a[C]) else B)
            a[f], a[m] = a[m], a[f]
            i, j = f + 1, l
            while True:
                while less(a[i], a[f]):
                    i += 1
                j -= 1
                while less(a[f], a[j]):
                    j -= 1
                if not i < j:
                    break
                a[i], a[j] = a[j], a[i]
                i += 1
            loop(i, l, d)
            l = i

    loop(0, n, 2 * int(math.log2(n)))
    return hits[0]


def mcilroy_killer(n: int) -> np.ndarray:
    gas = n
    val = [gas] * n
    st = {"solid": 0, "cand": 0}

    def less(x, y):
        if val[x] == gas and val[y] == gas:
            z = x if x == st["cand"] else y
            val[z] = st["solid"]
            st["solid"] += 1
        if val[x] == gas:
            st["cand"] = x
        elif val[y] == gas:
            st["cand"] = y
        return val[x] < val[y]

    _introsort_trace(n, less)
    return np.array(val, np.uint64)


def killer_with_keys(n: int, span: int, seed: int, base: int = 0) -> np.ndarray:
    """A median-of-3 killer whose never-compared ("gas") items get keys of
    their own: uniform in [gas + 1, gas + span], all above the solid ones, so
    every comparison the introsort made before its depth limit keeps its
    outcome (same partitions, same heapsort segment) while the heapsort then
    orders varied keys (span 1: all equal; 3: heavy ties; 2^40: distinct).
    `base` is added to every key (base >= 2^32: 64-bit keys)."""
    k = mcilroy_killer(n).astype(np.uint64)
    gas = k == n
    rng = np.random.default_rng(seed)
    k[gas] = np.uint64(n + 1) + rng.integers(0, span, int(gas.sum())).astype(np.uint64)
    return k + np.uint64(base)


def heap_fallbacks(keys: np.ndarray) -> int:
    k = [int(v) for v in keys]
    return _introsort_trace(len(k), lambda x, y: k[x] < k[y])


def sort_cases():
    rng = np.random.default_rng(7)
    cases = [np.array([], np.uint64), np.array([5], np.uint64)]
    for n in (2, 3, 16, 17, 18, 31, 64, 65, 100, 257, 1000, 5000):
        cases.append(rng.integers(0, 4, n).astype(np.uint64))        # heavy ties
        cases.append(rng.integers(0, 1 << 40, n).astype(np.uint64))  # distinct
    cases.append(np.zeros(300, np.uint64))
    cases.append(np.arange(400, dtype=np.uint64)[::-1].copy())
    for n in (40, 64, 100, 512, 1000, 3000):  # depth-limit heapsort fallback
        cases.append(mcilroy_killer(n))
    return cases
