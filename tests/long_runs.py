"""A fragment set of long, dense bucket runs (shared by the single-device and
sharded parity tests)."""
import numpy as np

import repkiller_amd as rk


def long_run_set(runs_len: int, seed: int) -> rk.Frags:
    """Consecutive 100-bp buckets, each holding `runs_len` entries on both axes:
    centres anywhere in the bucket (4 % of them at the edges, which probe the
    neighbour bucket), lengths on a x1.5 ladder (8 .. 2.3e6) so few entries
    match each other -- with tight ratios a run keeps more than 128 ACTIVE
    entries and its neighbour more than 64 (the LDS lists of k_sweep_long32
    overflow), with wide ratios the lists hold -- and repeated (centre,
    length) pairs, which hit."""
    rng = np.random.default_rng(seed)
    nb = 24
    b0 = 20_000  # centres >= 2 Mbp: every ladder length fits before its centre
    n = nb * runs_len
    bucket = np.repeat(np.arange(nb), runs_len) + b0
    off = rng.integers(0, 100, n)
    L = np.round(8 * 1.5 ** rng.integers(0, 32, n)).astype(np.int64)
    dup = rng.random(n) < 0.3  # copy an earlier entry of the same bucket
    src = np.maximum(np.arange(n) - rng.integers(1, runs_len, n), 0)
    same = (bucket[src] == bucket) & dup
    off[same], L[same] = off[src[same]], L[src[same]]
    c = bucket * 100 + off
    x = c - L // 2
    y = x + rng.choice([0, 3_000_000], n)
    strand = np.where(rng.random(n) < 0.5, ord("f"), ord("r")).astype(np.uint8)
    perm = rng.permutation(n)  # file order is not processing order
    return rk.Frags(x[perm].astype(np.uint64), y[perm].astype(np.uint64),
                    L[perm].astype(np.uint64), strand[perm])
