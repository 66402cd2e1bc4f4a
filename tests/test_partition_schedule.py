"""Phase A's block-wide Hoare scan (rk_groupsort.hip: block_partition_q) as a
schedule model, against libstdc++'s __unguarded_partition_pivot run
sequentially (commonFunctions.cpp:148-159 -> std::sort).  CPU only.

The kernel runs the two cursors a chunk at a time into stopper queues and
swaps each round's pairs up to the first crossing; its scans may read a slot
swapped earlier in the same partition either before or after the swap lands.
The model replays that schedule -- the same chunking, queue refill rule, pair
rounds, crossing test and cut -- with every scanned slot read at a random one
of the two moments, and must leave the same keys, tags and cut as the
sequential partition on every input (ties, runs, few and many keys).
"""
import random

import pytest


def _median_to_first(K, T, f, l):
    a, b, c = f + 1, f + (l - f) // 2, l - 1
    ka, kb, kc = K[a], K[b], K[c]
    if ka < kb:
        m = b if kb < kc else (c if ka < kc else a)
    else:
        m = a if ka < kc else (c if kb < kc else b)
    K[f], K[m] = K[m], K[f]
    T[f], T[m] = T[m], T[f]


def _sequential(K, T, f, l):
    _median_to_first(K, T, f, l)
    p, first, last = K[f], f + 1, l
    while True:
        while K[first] < p:
            first += 1
        last -= 1
        while p < K[last]:
            last -= 1
        if not first < last:
            return first
        K[first], K[last] = K[last], K[first]
        T[first], T[last] = T[last], T[first]
        first += 1


def _queued(K, T, f, l, C, rng):
    _median_to_first(K, T, f, l)
    p, lpos, rpos = K[f], f + 1, l
    QL, QR, popped, lastR = [], [], 0, None

    def scan(xs):  # each slot as read at issue, or re-read now (both are legal)
        return [(x, K[x], T[x]) if rng.random() < 0.5 else (x, k, t) for x, k, t in xs]

    pl = [(x, K[x], T[x]) for x in range(lpos, min(lpos + C, l))]
    pr = [(x, K[x], T[x]) for x in range(rpos - 1, max(rpos - 1 - C, f - 1), -1)]
    while True:
        addl = len(QL) < C and lpos < l
        addr = len(QR) < C and rpos > f
        if not addl and not QL:
            return lastR if popped else (QR[0][0] if QR else f + 1)
        if not addr and not QR:
            return QL[0][0]
        if addl:
            QL += [e for e in scan(pl) if not e[1] < p]
            lpos += C
            if lpos < l:
                pl = [(x, K[x], T[x]) for x in range(lpos, min(lpos + C, l))]
        if addr:
            QR += [e for e in scan(pr) if not p < e[1]]
            rpos = rpos - C if rpos - f > C else f
            if rpos > f:
                pr = [(x, K[x], T[x]) for x in range(rpos - 1, max(rpos - 1 - C, f - 1), -1)]
        m = min(len(QL), len(QR), C)
        cross = next((i for i in range(m) if QL[i][0] >= QR[i][0]), None)
        kc = m if cross is None else cross
        for i in range(kc):
            (xl, kl, tl), (xr, kr, tr) = QL[i], QR[i]
            K[xl], K[xr], T[xl], T[xr] = kr, kl, tr, tl
        if kc:
            lastR = QR[kc - 1][0]
        if cross is not None:
            cl = QL[kc][0]
            return min(cl, lastR) if popped + kc else cl
        QL, QR, popped = QL[kc:], QR[kc:], popped + kc


@pytest.mark.parametrize("seed", range(4))
def test_queued_partition_matches_sequential(seed):
    rng = random.Random(seed)
    for _ in range(2500):
        n = rng.randint(4, 260)
        nk = rng.choice([1, 2, 3, 5, 20, 1000])
        K = [rng.randrange(nk) for _ in range(n)]
        if rng.random() < 0.2:
            K.sort()
        if rng.random() < 0.1:
            K.sort(reverse=True)
        T = list(range(n))
        f, l = rng.randint(0, 2), n - rng.randint(0, 2)
        if l - f < 4:  # (phase A partitions only segments above 512)
            continue
        K2, T2 = K[:], T[:]
        cut = _sequential(K, T, f, l)
        assert _queued(K2, T2, f, l, rng.choice([1, 2, 3, 4, 8, 16, 64]), rng) == cut
        assert K2 == K and T2 == T
