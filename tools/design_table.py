#!/usr/bin/env python3
"""Regenerate DESIGN.md's kernel table from profiles/r1_bench.json (HIP-event
timing inside bench.py's timed steps, cfg3), profiles/traffic.json (PMC HBM
bytes) and profiles/r1_bench_cfg5.json (the same timing at cfg5, one GPU)."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEGIN, END = "<!-- kernel-table:begin -->", "<!-- kernel-table:end -->"
JOBS = [
    ("k_prep_keys", "processing key, 32-B row record, UB checks, 32-bit-length flag", "61"),
    ("k_digit_hist", "tile digit histograms, rows written tile-major", "4"),
    ("k_digit_scatter", "stable LSD radix pass: rank by ballots, LDS staging, XCD-contiguous tiles", "16 (12 without values)"),
    ("k_gather_proc", "processing-order SoA (one random 32-B gather per row)", "84"),
    ("k_sort_keys", "in-group key from the last yStart of each xStart/10 run", "32"),
    ("k_csr_fill_x", "X axis in bucket order: packed 8-B record + neighbour code", "30"),
    ("k_sweep_fast", "occupancy decisions, first sweep: a wavefront per 64-position window, ballot rounds, 32-bit candidate tests; X decisions write X results and X-hit parents", "26"),
    ("k_sweep_fast_more", "later sweeps: one wavefront per 64 windows handles the still-pending ones", "-"),
    ("k_sweep_long32", "runs of more than 64 entries, 64 entries at a time against LDS lists of the run's and the neighbour run's live entries", "-"),
    ("k_csr_fill_y", "Y axis in bucket order (one random 16-B gather)", "30"),
    ("k_jump", "chase parent chains to the root (bounded, concurrent compression)", "16"),
    ("k_assign_gid", "gid from the root's rank", "12"),
    ("k_group_offsets", "group bounds", "4"),
    ("k_build_records", "(key, tag, row) per member in gid order (one 16-B gather)", "36"),
    ("k_sort_small", "exact libstdc++ introsort, <= 16 members: stable rank", "16 per member"),
    ("k_sort_groups_reg", "17..64 members sorted in registers by one wavefront", "16 per member"),
    ("k_sort_groups_lds", "65..2048 members in LDS (compact tiers), register-finished segments", "16 per member"),
    ("k_sort_groups_split", "groups above 2048: block-wide partitions down to 512-member segments", "16 per member"),
    ("k_sort_segments", "those segments, one LDS wavefront each, own depth budget", "16 per member"),
    ("k_emit", "gid, flag, output order", "29"),
]


def main():
    d = json.load(open(os.path.join(ROOT, "profiles", "r1_bench.json")))
    t = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["kernels"]
    k = d["kernels"]
    c5p = os.path.join(ROOT, "profiles", "r1_bench_cfg5.json")
    k5 = json.load(open(c5p))["kernels"] if os.path.exists(c5p) else {}
    rows = ["| kernel | job | algorithmic B / element | ms / step | algorithmic GB/s | "
            "PMC HBM MB / launch | cfg5 ms / step |",
            "|---|---|---|---|---|---|---|"]
    for name, job, algo in JOBS:
        kk, tr = k.get(name, {}), t.get(name, {})
        ln = kk.get("launches_per_step", 0)
        hb = tr.get("hbm_bytes_per_launch")
        c5 = k5.get(name, {}).get("ms_per_step")
        rows.append(f"| `{name}`{' (x%g)' % ln if ln and ln != 1 else ''} | {job} | {algo} | "
                    f"{kk.get('ms_per_step', 0):.2f} | {kk.get('algo_GBps') or '-'} | "
                    f"{round(hb / 1e6) if hb else '-'} | {f'{c5:.1f}' if c5 else '-'} |")
    r = d["roofline"]
    rows.append("")
    rows.append(f"Step: {d['ms_per_step']:.2f} ms ({d['value'] / 1e9:.2f} G fragments/s); "
                f"roofline kernel `{r['kernel']}`: {r['launches_per_step']:g} launches, "
                f"{r['launch_ms']:.3f} ms each on average, {r['achieved']:.0f} GB/s, frac "
                f"{r['frac']:.3f}; PMC traffic {r['traffic'] / 1e6 if r['traffic'] else 0:.0f} MB per "
                f"launch against {r['algorithmic_bytes_per_launch'] / 1e6:.0f} MB algorithmic.")
    path = os.path.join(ROOT, "DESIGN.md")
    s = open(path).read()
    a, b = s.index(BEGIN) + len(BEGIN), s.index(END)
    open(path, "w").write(s[:a] + "\n" + "\n".join(rows) + "\n" + s[b:])


if __name__ == "__main__":
    main()
