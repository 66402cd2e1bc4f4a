#!/usr/bin/env python3
"""Reference-pinned digests of the BASELINE configs too large for the
fixtures of make_golden.py (cfg3: 50M fragments, cfg4: 200M fragments).

TEST INFRASTRUCTURE ONLY.  Writes tests/golden/large_hashes.json (DATA: input
and output digests, no reference source).

  cfg3 (50M, 3 Gbp, seed 3) -- pinned by the REFERENCE ITSELF: the synthetic
       set is written as CSV, oracle/_ref/ref_driver (the reference compiled
       from /root/reference/src by oracle/ref.mk) classifies it (~24 GB RSS,
       ~4 min) and the SHA-256 of its output CSV is recorded.  The C
       restatement (oracle/_build/rk_oracle) must reproduce the same bytes;
       its result arrays then give the array digest the GPU test checks.
  cfg4 (200M, 3 Gbp, seed 4) -- the reference would need ~97 GB of RAM here
       (24.2 GB per 50M), more than this container has, so the
       restatement (pinned at cfg3 above and on every fixture) supplies the
       array digest.
  cfg5q (250M, 3.75 Gbp, seed 5, repeat-rich) -- cfg5's shape (long bucket
       runs, groups of 10^4-10^5 members) at a quarter of its size; the
       restatement supplies the array digest, as for cfg4.

Digests
  input_arrays_sha256   sha256(x_start | y_start | length | strand), the
                        generator's arrays as little-endian bytes
  input_csv_sha256      sha256 of write_input_csv's file (cfg3 only)
  output_csv_sha256     sha256 of the reference's output CSV (cfg3 only)
  result_sha256         sha256(out_order u32 | gid u32 | repval u8), output
                        order, little-endian

  python tests/golden/make_golden_large.py [cfg3] [cfg4] [cfg5q]   (repo root)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import repkiller_amd as rk  # noqa: E402
from oracle import rk_oracle as ro  # noqa: E402

OUT = os.path.join(HERE, "large_hashes.json")
CONFIGS = {
    "cfg3": dict(n=50_000_000, genome_len=3_000_000_000, seed=3),
    "cfg4": dict(n=200_000_000, genome_len=3_000_000_000, seed=4),
    # cfg5's repeat-rich shape (95 % family fragments, 100..600 copies per
    # family, cfg5's 0.067 fragments per bp) at a quarter of its size: the
    # largest set the restatement classifies in this container's 64 GB
    "cfg5q": dict(n=250_000_000, genome_len=3_750_000_000, seed=5, family_frac=0.95,
                  copies=(100, 600)),
}


def arrays_sha256(*arrs) -> str:
    h = hashlib.sha256()
    for a in arrs:
        h.update(np.ascontiguousarray(a).view(np.uint8).data)
    return h.hexdigest()


def file_sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def main(which):
    ro.build_oracle()
    have_ref = ro.build_reference()
    table = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            table = json.load(f)
    tmp = tempfile.mkdtemp(dir="/tmp")
    for name in which:
        kw = CONFIGS[name]
        L = kw["genome_len"]
        lr = pr = 0.3
        t0 = time.time()
        f = rk.synth(**kw)
        e = {"synth": kw, "len_ratio": lr, "pos_ratio": pr,
             "input_arrays_sha256": arrays_sha256(f.x_start, f.y_start, f.length, f.strand)}
        print(name, "synth", round(time.time() - t0, 1), "s", flush=True)
        if name == "cfg3":
            assert have_ref, "cfg3 is pinned by the reference: /root/reference is needed"
            inp = os.path.join(tmp, "in.csv")
            out_ref = os.path.join(tmp, "ref.out.csv")
            out_ora = os.path.join(tmp, "oracle.out.csv")
            rk.write_input_csv(inp, f, L, L)
            e["input_csv_sha256"] = file_sha256(inp)
            rc, err = ro.run_cli(ro.REF_DRIVER, inp, out_ref, lr, pr, timeout=3600)
            assert rc == 0, err
            e["ref_timing"] = json.loads(err.strip().splitlines()[-1])
            e["output_csv_sha256"] = file_sha256(out_ref)
            os.remove(out_ref)
            print(name, "reference", e["ref_timing"], flush=True)
            rc, err = ro.run_cli(ro.CLI, inp, out_ora, lr, pr, timeout=3600)
            assert rc == 0, err
            assert file_sha256(out_ora) == e["output_csv_sha256"], \
                "the restatement disagrees with the reference at cfg3"
            os.remove(out_ora)
            os.remove(inp)
            e["oracle_csv_matches_reference"] = True
        t0 = time.time()
        rc, gid, rep, order, ng = ro.classify(f.x_start, f.y_start, f.length, f.strand, L, L,
                                              lr, pr)
        assert rc == 0
        e["oracle_classify_s"] = round(time.time() - t0, 2)
        e["n_out"] = int(order.size)
        e["n_groups"] = ng
        e["result_sha256"] = arrays_sha256(order.astype("<u4"), gid.astype("<u4"), rep)
        print(name, e, flush=True)
        table[name] = e
        with open(OUT, "w") as fo:
            json.dump(table, fo, indent=1, sort_keys=True)
        del f, gid, rep, order
    os.rmdir(tmp)


if __name__ == "__main__":
    main([a for a in sys.argv[1:] if a in CONFIGS] or list(CONFIGS))
