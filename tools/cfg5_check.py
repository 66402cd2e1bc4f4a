"""BASELINE cfg5 on ONE MI355X: 1B fragments, 15 Gbp repeat-rich self-comparison.

Classifies the full set three times from HBM-resident inputs and prints one JSON
line: per-run wall time, workspace footprint, group counts and a verdict on the
size-independent properties the full-size parity tests check at 50-60M
(tests/test_large_configs.py::device_properties), restated in O(n) host memory:
run 1 == run 3 (determinism), output order a permutation of the kept rows, gids
dense in output order, repeat flags by group position, and every group sorted
by |yStart - diag_func[xStart/10]| (commonFunctions.cpp:148-177).

usage: python tools/cfg5_check.py [--n N] [--genome-bp L] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import repkiller_amd as rk  # noqa: E402

T0 = time.perf_counter()


def log(msg):
    print(f"[{time.perf_counter() - T0:7.1f}s] {msg}", flush=True)


def check(f, L, n_out, ng, gid, rep, order):
    """gid/rep/order: host uint32/uint8/uint32 arrays of length n_out."""
    n = f.n
    vsize = 1 + (L + 1) // 10
    b = (f.x_start // np.uint64(10)).astype(np.int64)
    keep = b != vsize - 1
    assert n_out == int(keep.sum()), ("n_out", n_out)
    seen = np.zeros(n, np.bool_)
    seen[order] = True
    assert np.array_equal(seen, keep), "order is not a permutation of the kept rows"
    del seen, keep
    log("permutation ok")
    step = np.diff(gid)  # uint32: a decrease wraps to a huge value
    assert gid[0] == 0 and gid[-1] == ng - 1 and bool(np.all(step <= 1)), "gids"
    same = step == 0
    del step
    starts = np.flatnonzero(np.r_[True, ~same])
    sizes = np.diff(np.r_[starts, n_out])
    want = np.full(n_out, 2, np.uint8)
    want[starts] = 1
    want[starts[sizes == 1]] = 0
    assert np.array_equal(rep, want), "repeat flags"
    del want, starts, sizes
    log("gids and repeat flags ok")
    # diag_func[b] = yStart of the LAST fragment (file order) of xStart/10 bucket b
    last = np.full(vsize, -1, np.int64)
    np.maximum.at(last, b, np.arange(n, dtype=np.int64))
    bo = b[order]
    del b
    ha = np.abs(f.y_start[order].astype(np.int64) - f.y_start[last[bo]].astype(np.int64))
    del last, bo
    assert bool(np.all(ha[1:][same] >= ha[:-1][same])), "in-group order"
    log("in-group sort keys ok")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000_000)
    ap.add_argument("--genome-bp", type=int, default=15_000_000_000)
    ap.add_argument("--runs", type=int, default=3)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    n, L = a.n, a.genome_bp
    import threading  # a progress line every minute through the long host phases

    def beat():
        while True:
            time.sleep(60)
            log("...")
    threading.Thread(target=beat, daemon=True).start()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = rk.Context(0)
    log(f"synth {n} fragments over {L} bp (repeat-rich)")
    f = rk.synth(n, L, seed=3, family_frac=0.95, copies=(100, 600))
    log("upload")
    x = torch.from_numpy(f.x_start.view(np.int64)).to(dev)
    y = torch.from_numpy(f.y_start.view(np.int64)).to(dev)
    ln = torch.from_numpy(f.length.view(np.int64)).to(dev)
    s = torch.from_numpy(f.strand).to(dev)
    gid = torch.empty(n, dtype=torch.int32, device=dev)
    rep = torch.empty(n, dtype=torch.uint8, device=dev)
    order = torch.empty(n, dtype=torch.int32, device=dev)
    times, first = [], None
    res = None
    for r in range(a.runs):
        torch.cuda.synchronize()
        t = time.perf_counter()
        res = ctx.classify_device(x, y, ln, s, gid, rep, order, L, L)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
        log(f"run {r}: {times[-1] * 1e3:.1f} ms, n_out {res[0]}, groups {res[1]}, "
            f"HBM in use {torch.cuda.memory_allocated() / 2**30:.1f} GiB (torch) / "
            f"{(torch.cuda.mem_get_info()[1] - torch.cuda.mem_get_info()[0]) / 2**30:.1f} "
            f"GiB (device)")
        if r == 0:
            m = res[0]
            first = (res, gid[:m].cpu().numpy().view(np.uint32).copy(),
                     rep[:m].cpu().numpy().copy(), order[:m].cpu().numpy().view(np.uint32).copy())
    n_out, ng = res
    det = (first[0] == res
           and np.array_equal(first[1], gid[:n_out].cpu().numpy().view(np.uint32))
           and np.array_equal(first[2], rep[:n_out].cpu().numpy())
           and np.array_equal(first[3], order[:n_out].cpu().numpy().view(np.uint32)))
    log(f"deterministic: {det}")
    free, total = torch.cuda.mem_get_info()
    del x, y, ln, s, gid, rep, order
    verdict = "skipped"
    if not a.no_check:
        check(f, L, n_out, ng, first[1], first[2], first[3])
        verdict = "ok"
    best = min(times[1:]) if len(times) > 1 else times[0]
    line = {"workload": "cfg5: 1B fragments, 15 Gbp repeat-rich self-comparison, one MI355X"
            if n == 1_000_000_000 else f"{n} fragments, {L} bp repeat-rich",
            "fragments": n, "genome_bp": L, "n_out": int(n_out), "groups": int(ng),
            "ms_per_run": [round(t * 1e3, 1) for t in times],
            "fragments_per_s_best": round(n / best, 1),
            "device_used_GiB_at_end": round((total - free) / 2**30, 1),
            "deterministic": bool(det), "properties": verdict}
    print(json.dumps(line), flush=True)
    if a.out:
        with open(a.out, "w") as fo:
            json.dump(line, fo, indent=1)
    if not det:
        sys.exit(1)


if __name__ == "__main__":
    main()
