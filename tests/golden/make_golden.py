#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the REFERENCE ITSELF.

Needs /root/reference (read-only) to build oracle/_ref/ref_driver with
oracle/ref.mk, and the product library for the synthetic generator
(repkiller_amd.synth / write_input_csv -- input making only).  Everything
written here is DATA (inputs + the reference's outputs); no reference source.

  python tests/golden/make_golden.py          # from the repo root

Outputs
  edge/<name>.in.csv, edge/<name>.out.csv     hand-written edge inputs (SURVEY.md §4
                                              E1-E14) and the reference's output
  edge/manifest.json                          ratios + expected outcome per case
  corpus10k.in.csv.gz / corpus10k.out.csv.gz  cfg1 synthetic set and reference output
  hashes.json                                 SHA-256 of generator input and reference
                                              output for 1M-fragment sets (cfg2, repeat-rich)
  boundary_hashes.json                        same for tests/boundary_cases.py (deviation
                                              boundaries, NaN/inf/extreme ratios); only
                                              this file with --boundary
"""
from __future__ import annotations

import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import repkiller_amd as rk  # noqa: E402
from oracle import rk_oracle as ro  # noqa: E402

EDGE = os.path.join(HERE, "edge")


def header(lx: int, ly: int, total: int, tag: str = "edge") -> str:
    return (f"All by-Identity Ungapped Fragments (Hits based approach)\n"
            f"[golden fixture {tag}]\n"
            "SeqX filename\t: X.fasta\nSeqY filename\t: Y.fasta\n"
            "SeqX name\t: X\nSeqY name\t: Y\n"
            f"SeqX length\t: {lx}\nSeqY length\t: {ly}\n"
            "Min.fragment.length\t: 0\nMin.Identity\t: 0\nTotal hits\t: 0\n"
            "Total hits (used)\t: 0\n"
            f"Total fragments\t: {total}\n"
            "========================================================\n"
            "Type,xStart,yStart,xEnd,yEnd,Strand(f/r),block,length,score,ident,similarity,"
            "%ident,SeqX,SeqY\n"
            "========================================================\n")


def frag(x, y, L, strand="f", sim="90.00", score=None, ident=None) -> str:
    ident = ident if ident is not None else int(L * 0.9)
    score = score if score is not None else 4 * ident
    return f"Frag,{x},{y},{x + L - 1},{y + L - 1},{strand},0,{L},{score},{ident},{sim},{sim},0,0\n"


def cases():
    """(name, text, len_ratio, pos_ratio, kind) -- kind: 'ref' = the reference's
    output is the expectation; 'error:<CODE>' = the reference aborts or is
    undefined there and the build must return that error."""
    c = []
    # E1 last-bucket drop: lenX = 1000+1, vsize = 101, xStart 1000..1009 never grouped
    body = frag(100, 200, 50) + frag(1000, 300, 50) + frag(1005, 305, 50) + frag(500, 600, 80)
    c.append(("e01_last_bucket", header(1000, 1000, 4) + body, 0.3, 0.3, "ref"))
    # E2 neighbour asymmetry (c+1/c+2 probes only while c < max_index = len/100)
    a, b = frag(151, 500, 100), frag(150, 800, 98)
    c.append(("e02a_upward_probe_off", header(1000, 1000, 2) + a + b, 0.3, 0.3, "ref"))
    c.append(("e02b_upward_probe_on", header(100000, 100000, 2) + a + b, 0.3, 0.3, "ref"))
    a2, b2 = frag(150, 500, 98), frag(151, 800, 100)
    c.append(("e02c_downward_probe", header(1000, 1000, 2) + a2 + b2, 0.3, 0.3, "ref"))
    # E3 strand classes: 'f' vs everything else ('r' and 'x' share the reverse lists)
    body = frag(300, 300, 100, "f") + frag(300, 300, 100, "x") + frag(301, 301, 100, "r") + \
        frag(302, 302, 100, "f")
    c.append(("e03_strands", header(10000, 10000, 4) + body, 0.3, 0.3, "ref"))
    # E4 ident comes from the similarity column (stof(v[10])), truncated
    body = "Frag,100,200,199,299,f,0,100,300,77,90.5,88.0,0,0\n" + \
        "Frag,400,900,449,949,r,0,50,100,11,33.99,1.0,0,0\n"
    c.append(("e04_ident_from_similarity", header(10000, 10000, 2) + body, 0.3, 0.3, "ref"))
    # E5 in-group order: |yStart - yStart(last of xStart/10 bucket)|, stable below 17
    body = frag(100, 5000, 100) + frag(101, 3000, 100) + frag(102, 9000, 100) + \
        frag(103, 4000, 100)
    c.append(("e05a_in_group_order", header(20000, 20000, 4) + body, 0.3, 0.3, "ref"))
    # E5b: 40 members, many equal keys -> introsort permutation (not stable)
    rows = []
    for k in range(40):
        rows.append(frag(1000 + (k % 9), 7000 + 37 * ((k * 7) % 11), 120 + (k % 3)))
    c.append(("e05b_big_group_ties", header(30000, 30000, 40) + "".join(rows), 0.3, 0.3, "ref"))
    # E6 parse rules
    body = "".join([
        "Frag,200,300,299,399,f,0,100,400,90,1e50,90,0,0\n",        # ERANGE: skipped
        "Frag,210,310,309,409,f,0,100,400,90,nan,90,0,0\n",         # ident 2^63, prints nan
        "Frag,220,320,319,419,f,0,100,400,90,-nan,90,0,0\n",
        "Frag,230,330,329,429,r,0,100,400,90,inf,90,0,0\n",         # ident 0
        "Frag,240,340,339,439,r,0,100,400,90,-5.5,90,0,0\n",        # ident 2^64-5
        "Frag,250,350,349,449,f,0,100,400,90,1e19,90,0,0\n",        # >= 2^63 path
        "Frag,260,360,359,459,f,0,100,400,90,3e19,90,0,0\n",        # >= 2^64 -> 0
        "Frag,270,370,369,469,f,0,100,400,90,1e-50,90,0,0\n",       # underflow: skipped
        "Frag,280,380,379,479,f,0,100,400,90,1e-40,90,0,0\n",       # subnormal
        "Frag,290,390,389,489,f,0,100,400,90,88.25,90,0,0\r\n",     # CRLF
        "Frag,300,400,399,499,f,0,100,400,90,88.25,90,0,\n",        # empty 14th: skipped
        "CSB,310,410,409,509,f,0,100,400,90,88.25,90,0,0\n",        # not Frag: skipped
        "Frag, 1005 ,500,1104,599,f,0,100,400,90,70,90,0,0\n",      # spaces: atoll
        "Frag,320,420,419,519,f,0,100,400,90,88.25,90,0\n",         # 13 fields: last repeated
        "Frag,1,2\n",                                               # 3 fields: '2' x 12
        "Frag,330,430,429,529,r,0,100,400,90,77,90,0,0,9,9,9,9\n",  # extra fields
        "Frag\n",                                                   # stof('Frag') throws
        "Frag,abc,440,439,539,f,0,100,400,90,60,90,0,0\n",          # atoll -> 0
        "Frag,+340,440,439,539,f,0,+100,400,90,60,90,0,0\n",        # explicit sign
        "Frag,0x10,450,449,549,f,0,100,400,90,0x1p3,90,0,0\n",      # atoll 0; strtof hex 8
        "Frag,350,460,459,559,f,0,100,400,90, 42.5abc,90,0,0\n",    # leading space, trailing junk
        "\n",
        "Frag,,470,469,569,f,0,100,400,90,60,90,0,0\n",             # empty field: skipped
    ])
    c.append(("e06_parse_rules", header(20000, 20000, 40) + body, 0.3, 0.3, "ref"))
    # E7 zero length: deviation is NaN / -inf; identity prints -nan or inf
    body = frag(500, 500, 0, ident=0) + frag(500, 500, 0, ident=5) + frag(500, 500, 100) + \
        frag(501, 501, 0, ident=0)
    c.append(("e07_zero_length", header(20000, 20000, 4) + body, 0.3, 0.3, "ref"))
    # E8 more Frag lines than the header total: reference throws (rc 134)
    body = frag(100, 100, 50) + frag(200, 200, 50) + frag(300, 300, 50)
    c.append(("e08_count_overflow", header(1000, 1000, 2) + body, 0.3, 0.3, "error:RK_E_COUNT"))
    # E12 truncated header: getline at EOF keeps the previous line (10 lines only)
    txt = "".join(header(5000, 5000, 0).splitlines(True)[:10])
    c.append(("e12_short_header", txt, 0.3, 0.3, "ref"))
    # E13 header only, no trailing newline on the last line
    c.append(("e13_no_fragments", header(5000, 5000, 0).rstrip("\n"), 0.3, 0.3, "ref"))
    # E14 exact deviation tie between two ACTIVE entries: the newest wins
    body = frag(1000, 100, 60) + frag(1000, 9000, 140) + frag(1000, 4000, 100)
    c.append(("e14_tie_newest_wins", header(20000, 20000, 3) + body, 0.5, 0.3, "ref"))
    # E15 file order inside an xStart/10 bucket vs across buckets
    body = frag(119, 700, 80) + frag(111, 705, 80) + frag(95, 702, 80) + frag(110, 2000, 80)
    c.append(("e15_processing_order", header(20000, 20000, 4) + body, 0.3, 0.3, "ref"))
    # E16 last line without newline is still read
    body = frag(100, 100, 50) + frag(100, 100, 50).rstrip("\n")
    c.append(("e16_no_final_newline", header(1000, 1000, 2) + body, 0.3, 0.3, "ref"))
    # E11 undefined behaviour in the reference -> the build returns an error
    c.append(("e11a_ub_xstart_bucket", header(1000, 1000, 1) + frag(1020, 10, 10), 0.3, 0.3,
              "error:RK_E_UB_BUCKET"))
    c.append(("e11b_ub_x_center", header(1000, 1000, 1) + frag(990, 10, 400), 0.3, 0.3,
              "error:RK_E_UB_CENTER"))
    c.append(("e11c_ub_y_center", header(1000, 1000, 1) + frag(10, 995, 300), 0.3, 0.3,
              "error:RK_E_UB_CENTER"))
    c.append(("e11d_ub_tiny_sequence", header(50, 50, 1) + frag(40, 10, 116), 0.3, 0.3,
              "error:RK_E_UB_CENTER"))
    return c


def sha256_file(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def main():
    if not ro.build_reference():
        sys.exit("the reference (/root/reference) is needed to regenerate fixtures")
    ro.build_oracle()
    os.makedirs(EDGE, exist_ok=True)
    manifest = {}
    for name, text, lr, pr, kind in cases():
        inp = os.path.join(EDGE, name + ".in.csv")
        out = os.path.join(EDGE, name + ".out.csv")
        with open(inp, "w", newline="") as f:
            f.write(text)
        entry = {"len_ratio": lr, "pos_ratio": pr, "expect": kind}
        if kind == "ref" or kind == "error:RK_E_COUNT":
            rc, err = ro.run_cli(ro.REF_DRIVER, inp, out, lr, pr)
            entry["ref_rc"] = rc
            if kind == "ref":
                assert rc == 0, (name, rc, err)
            else:
                assert rc != 0, (name, "reference was expected to abort")
                if os.path.exists(out):
                    os.remove(out)
        manifest[name] = entry
    with open(os.path.join(EDGE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)

    tmp = tempfile.mkdtemp()
    try:
        # cfg1 corpus: 10k fragments over 1 Mbp (seed = config number)
        fr = rk.synth(10000, 1_000_000, seed=1)
        inp, out = os.path.join(tmp, "c1.csv"), os.path.join(tmp, "c1.out.csv")
        rk.write_input_csv(inp, fr, 1_000_000, 1_000_000)
        rc, err = ro.run_cli(ro.REF_DRIVER, inp, out, 0.3, 0.3)
        assert rc == 0, err
        for src, dst in ((inp, "corpus10k.in.csv.gz"), (out, "corpus10k.out.csv.gz")):
            with open(src, "rb") as fi, gzip.GzipFile(os.path.join(HERE, dst), "wb",
                                                      mtime=0) as fo:
                shutil.copyfileobj(fi, fo)
        # 1M sets: pinned by hash (input regenerated deterministically by rk.synth)
        hashes = {}
        sets = {
            "cfg2_1M_100Mbp": dict(n=1_000_000, genome_len=100_000_000, seed=2),
            "repeat_rich_1M_100Mbp": dict(n=1_000_000, genome_len=100_000_000, seed=5,
                                          family_frac=0.95, copies=(100, 600)),
        }
        for name, kw in sets.items():
            for lr, pr in ((0.3, 0.3), (0.05, 0.05)):
                fr = rk.synth(**kw)
                L = kw["genome_len"]
                inp, out = os.path.join(tmp, "in.csv"), os.path.join(tmp, "out.csv")
                rk.write_input_csv(inp, fr, L, L)
                rc, err = ro.run_cli(ro.REF_DRIVER, inp, out, lr, pr)
                assert rc == 0, err
                key = f"{name}@{lr},{pr}"
                hashes[key] = {"synth": {k: (list(v) if isinstance(v, tuple) else v)
                                         for k, v in kw.items()},
                               "len_ratio": lr, "pos_ratio": pr,
                               "input_sha256": sha256_file(inp),
                               "output_sha256": sha256_file(out),
                               "ref_timing": json.loads(err.strip().splitlines()[-1])}
                print(key, hashes[key]["output_sha256"])
        with open(os.path.join(HERE, "hashes.json"), "w") as f:
            json.dump(hashes, f, indent=1, sort_keys=True)
    finally:
        shutil.rmtree(tmp)


def boundary():
    sys.path.insert(0, os.path.dirname(HERE))
    import boundary_cases as bc
    tmp = tempfile.mkdtemp()
    try:
        fr = bc.short_dense(rk)
        inp = os.path.join(tmp, "in.csv")
        rk.write_input_csv(inp, fr, bc.GENOME, bc.GENOME)
        out = {"input_sha256": sha256_file(inp), "outputs": {}}
        for lr, pr in bc.RATIOS:
            o = os.path.join(tmp, "out.csv")
            p = subprocess.run([ro.REF_DRIVER, inp, o, lr, pr], capture_output=True, text=True)
            assert p.returncode == 0, p.stderr
            out["outputs"][f"{lr},{pr}"] = sha256_file(o)
            print(lr, pr, out["outputs"][f"{lr},{pr}"])
        with open(os.path.join(HERE, "boundary_hashes.json"), "w") as f:
            json.dump(out, f, indent=1, sort_keys=True)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    if "--boundary" in sys.argv:
        boundary()
    else:
        main()
