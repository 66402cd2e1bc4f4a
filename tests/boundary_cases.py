"""Inputs whose length / centre differences land exactly on L*ratio.

deviation (SequenceOcupationList.cpp:20-31) returns 0 when sim_len or sim_pos
is negative and 0.4*sl + 0.6*sp otherwise; the device decides "deviation > 0"
by comparisons instead of divisions (rk_occupancy.hip, matches()).  These
inputs -- short fragments packed ~10 per 100-bp bucket -- hit sl == 0 and
sp == 0 often, and the ratio list covers NaN / inf / extreme magnitudes, which
the reference accepts (commonFunctions.cpp:26-27 only rejects <= 0).
Outputs are pinned by the reference itself (tests/golden/boundary_hashes.json,
written by tests/golden/make_golden.py --boundary).
"""
from __future__ import annotations

import numpy as np

N, GENOME, SEED = 20_000, 200_000, 5
RATIOS = [("0.5", "0.5"), ("1.0", "1.0"), ("0.25", "2.0"), ("0.1", "0.3"), ("2.0", "0.125"),
          ("nan", "0.5"), ("0.5", "nan"), ("inf", "0.5"), ("1e-300", "1e300"),
          ("1e300", "1e-300")]


def short_dense(rk, n: int = N, genome: int = GENOME, seed: int = SEED):
    rng = np.random.default_rng(seed)
    ln = rng.integers(6, 15, n).astype(np.uint64)
    x = rng.integers(1, genome - 20, n).astype(np.uint64)
    y = rng.integers(1, genome - 20, n).astype(np.uint64)
    st = np.where(rng.random(n) < 0.5, ord("f"), ord("r")).astype(np.uint8)
    return rk.Frags(x, y, ln, st)
