"""Debug: the call sequence that fails in the suite, on one context."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import repkiller_amd as rk
sys.path.insert(0, os.path.join(ROOT, "tools", "dbg"))
from wide_runs import case

ctx = rk.Context(0)
steps = sys.argv[1].split(",")
for s in steps:
    if s == "big":
        f = rk.synth(200_000, 10_000_000, seed=21); L = 10_000_000
    elif s == "ws":
        f = rk.synth(20_000, 1_000_000, seed=41)
        rng = np.random.default_rng(41); k = 40
        wide = rk.Frags(rng.integers(1, 1_000_000, k).astype(np.uint64), rng.integers(1, 1_000_000, k).astype(np.uint64),
                        (np.uint64(2**31) + rng.integers(0, 3, k).astype(np.uint64) * np.uint64(7)), np.full(k, ord('f'), np.uint8))
        f = rk.Frags(np.concatenate([f.x_start, wide.x_start]), np.concatenate([f.y_start, wide.y_start]),
                     np.concatenate([f.length, wide.length]), np.concatenate([f.strand, wide.strand]))
        L = 5_000_000_000
    else:
        f = case(); L = 5_000_000_000
    try:
        r = ctx.classify(f, L, L, 0.05, 0.05)
        print(s, "ok", r.n_groups, ctx.stats()["pipeline"], flush=True)
    except rk.RkError as e:
        print(s, "ERROR", e, flush=True)
