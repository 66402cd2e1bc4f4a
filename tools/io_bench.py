#!/usr/bin/env python3
"""End-to-end file path: CSV ingress -> GPU classification -> CSV egress.

SURVEY.md §8(f) rows 1-2: the reference spends most of its wall time parsing
the fragment CSV (FragmentsDatabase.cpp:17-100) and formatting the output
(commonFunctions.cpp:101-146).  This times the repo's host ingress
(rk_db_load_csv: mmap + parallel parse with the reference's acceptance rules)
and egress (rk_db_write_csv: parallel formatting) around the device path on
one synthetic file, next to the reference itself (oracle/_ref/ref_driver,
1 core) on the same file, and checks that both outputs are byte-identical.

  python tools/io_bench.py [--n 50000000] [--genome 3000000000] [--tmp DIR]

(default: cfg3, the headline config: 50M fragments over 3 Gbp)

Prints one JSON line.  Test/benchmark infrastructure: the reference binary is
only timed and compared against, never used to produce results.
"""
from __future__ import annotations

import argparse
import filecmp
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401  (one shared HIP runtime)

import repkiller_amd as rk  # noqa: E402


def heartbeat(stop, t0):
    """A progress line every 30 s on stderr (the reference's run is minutes of silence)."""
    while not stop.wait(30):
        print(f"[io_bench] {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)


def main():
    import threading
    stop = threading.Event()
    threading.Thread(target=heartbeat, args=(stop, time.perf_counter()), daemon=True).start()
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50_000_000)
    ap.add_argument("--genome", type=int, default=3_000_000_000)  # cfg3
    ap.add_argument("--no-ref", action="store_true")
    ap.add_argument("--tmp", default=os.environ.get("TMPDIR", "/tmp"))
    args = ap.parse_args()
    n, L = args.n, args.genome
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    cpu = "unknown"
    with open("/proc/cpuinfo") as fh:
        for line in fh:
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    out = {"fragments": n, "genome_bp": L, "seed": 3,
           "host": {"nproc": os.cpu_count(), "affinity_cpus": aff, "cpu_model": cpu},
           "note": "ours: rk_db_load_csv (mmap + parallel parse) -> rk_classify (host buffers, "
                   "PCIe included) -> rk_db_write_csv (parallel formatting); reference: "
                   "oracle/_ref/ref_driver (the reference's own code, one core) on the same file"}
    with tempfile.TemporaryDirectory(dir=args.tmp) as d:
        inp = os.path.join(d, "in.csv")
        f = rk.synth(n, L, seed=3)
        rk.write_input_csv(inp, f, L, L)
        del f
        out["csv_bytes"] = os.path.getsize(inp)
        ctx = rk.Context(0)
        t0 = time.perf_counter()
        db = rk.FragmentsDatabase(inp)
        t1 = time.perf_counter()
        res = ctx.classify(db.frags, db.len_x_hdr, db.len_y_hdr, 0.3, 0.3)
        t2 = time.perf_counter()
        ours = os.path.join(d, "ours.csv")
        db.save_all_frag_pairs(ours, res)
        t3 = time.perf_counter()
        out.update(load_s=round(t1 - t0, 3), classify_s=round(t2 - t1, 3),
                   save_s=round(t3 - t2, 3), total_s=round(t3 - t0, 3),
                   host_threads=os.cpu_count())
        # the binary SoA cache: written once, then a load
        # with no parse; the classification from it must write the same bytes
        cache = os.path.join(d, "db.soa")
        t4 = time.perf_counter()
        db.save_soa(cache)
        t5 = time.perf_counter()
        db2 = rk.FragmentsDatabase.load_soa(cache)
        t6 = time.perf_counter()
        res2 = ctx.classify(db2.frags, db2.len_x_hdr, db2.len_y_hdr, 0.3, 0.3)
        t7 = time.perf_counter()
        ours2 = os.path.join(d, "ours_soa.csv")
        db2.save_all_frag_pairs(ours2, res2)
        t8 = time.perf_counter()
        out["soa_cache"] = {"bytes": os.path.getsize(cache), "save_s": round(t5 - t4, 3),
                            "load_s": round(t6 - t5, 3), "classify_s": round(t7 - t6, 3),
                            "save_csv_s": round(t8 - t7, 3), "total_s": round(t8 - t5, 3),
                            "same_csv_as_csv_route": filecmp.cmp(ours, ours2, shallow=False)}
        os.remove(ours2)
        os.remove(cache)
        del db2, res2
        ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
        if not args.no_ref and os.path.exists(ref):
            theirs = os.path.join(d, "ref.csv")
            t0 = time.perf_counter()
            p = subprocess.run([ref, inp, theirs, "0.3", "0.3"], capture_output=True, text=True)
            out["reference_wall_s"] = round(time.perf_counter() - t0, 3)
            t = json.loads(p.stderr.strip().splitlines()[-1])
            out["reference"] = {k: round(t[k], 3) for k in ("load_s", "group_s", "diag_sort_s",
                                                             "save_s")}
            out["reference"]["total_s"] = round(sum(out["reference"].values()), 3)
            out["byte_identical"] = filecmp.cmp(ours, theirs, shallow=False)
            out["output_bytes"] = os.path.getsize(ours)
            out["speedup_total"] = round(out["reference"]["total_s"] / out["total_s"], 1)
    stop.set()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
