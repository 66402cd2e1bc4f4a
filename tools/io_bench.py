#!/usr/bin/env python3
"""End-to-end file path: CSV ingress -> GPU classification -> CSV egress.

SURVEY.md §8(f) rows 1-2: the reference spends most of its wall time parsing
the fragment CSV (FragmentsDatabase.cpp:17-100) and formatting the output
(commonFunctions.cpp:101-146).  This times the repo's host ingress
(rk_db_load_csv: mmap + parallel parse with the reference's acceptance rules)
and egress (rk_db_write_csv: parallel formatting) around the device path on
one synthetic file, next to the reference itself (oracle/_ref/ref_driver,
1 core) on the same file, and checks that both outputs are byte-identical.

  python tools/io_bench.py [--n 10000000] [--genome 600000000]

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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--genome", type=int, default=600_000_000)  # cfg3 density
    ap.add_argument("--no-ref", action="store_true")
    args = ap.parse_args()
    n, L = args.n, args.genome
    out = {"fragments": n, "genome_bp": L}
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as d:
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
        ref = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
        if not args.no_ref and os.path.exists(ref):
            theirs = os.path.join(d, "ref.csv")
            p = subprocess.run([ref, inp, theirs, "0.3", "0.3"], capture_output=True, text=True)
            t = json.loads(p.stderr.strip().splitlines()[-1])
            out["reference"] = {k: round(t[k], 3) for k in ("load_s", "group_s", "diag_sort_s",
                                                             "save_s")}
            out["reference"]["total_s"] = round(sum(out["reference"].values()), 3)
            out["byte_identical"] = filecmp.cmp(ours, theirs, shallow=False)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
