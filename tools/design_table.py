#!/usr/bin/env python3
"""Regenerate DESIGN.md's kernel table from profiles/r6_bench.json (HIP-event
timing inside bench.py's timed steps, cfg3), profiles/traffic.json
(PMC HBM bytes, cfg3) and profiles/r6_bench_cfg5.json (the same timing at cfg5,
one GPU) when present."""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BEGIN, END = "<!-- kernel-table:begin -->", "<!-- kernel-table:end -->"
BENCH, CFG5 = "r6_bench.json", "r6_bench_cfg5.json"
# bench kernel name -> the PMC summary's name (tools/pmc_summary.py uses the bench's names)
PMC_NAME = {"k_nw_assign": "k_nw_assign_jump"}
JOBS = [
    ("k_nw_order_hist", "one read of the file-order SoA: digit histograms of the processing key and the Y key, kept / forward counts, longest length, bounds and pack checks", "25"),
    ("k_onesweep", "one LSD pass: 16-B records 6144 per tile (2 coarse processing-order passes: the key's top 15 bits as 8 + 7 at cfg3, the second also counting each coarse key), 12-B records 7168 per tile (2 coarse Y passes after X, 8 + 7 bits, the first carrying the X-hit bits, the second counting each coarse key; 3 member passes by gid, 8 + 8 + 8 at cfg3's 24-bit gids): ballot ranks, LDS placement in rounds, decoupled look-back, digit-segment write-out", "32 / 24 (pass 1: 41; first Y pass: 24.1)"),
    ("k_seg_fine (order)", "one block per coarse-key segment (<= 4096 records in LDS): the 14 fine bits by ballot-ranked LSD rounds, then the final records, the Y records and the X-chunk counts (an LDS window of chunk counters)", "44"),
    ("k_seg_fine (Y)", "one block per coarse Y-key segment (<= 4096 records in LDS): the 11 fine bits by ballot-ranked LSD rounds, then the Y axis' CSR arrays (key, entry, packed record, neighbour code, state from the carried X-hit bit) written as whole lines", "30"),
    ("k_seg_big", "segments above 4096 records: the same passes through global memory, one block each", "-"),
    ("k_nw_xcount", "(RK_NW_SPLIT=0 only) entries per (strand, X chunk) and owned rows per chunk, over the processing order", "16"),
    ("k_nw_xchunk", "X axis: a wavefront per chunk places its entries (bin counts, scan, ballot ranks) and writes the owned rows' member records (in-group sort keys)", "50"),
    ("k_sweep_fast", "occupancy decisions, first sweep: a wavefront per 64-position window, ballot rounds, 32-bit candidate tests", "26"),
    ("k_sweep_fast_more", "later sweeps: one wavefront per 64 windows handles the still-pending ones", "-"),
    ("k_sweep_long32", "runs of more than 64 entries: a pre-scan for the run's open entries (none: the run is done), then 64 entries at a time against LDS lists (redundant ACTIVE records dropped when a list would overflow)", "-"),
    ("k_nw_x_bits", "X hits as a bitmask by processing index (ballots over the X states at each fragment's X position), read in order by the first Y pass", "5"),
    ("k_nw_fill_y", "Y states from the bitmask for later ratio pairs (X hits sit in the Y lists)", "5"),
    ("k_jump", "(RK_ROOTS_FUSED=0 only) chase parent chains to the root, round by round", "16"),
    ("k_nw_assign", "`k_nw_assign_jump`: after the scan of the parents' root flags, each member chases its chain (up to 32 links; longer ones listed for `k_nw_assign_rest`), writes the root back as its parent and takes gid = the root's rank, with the member-sort histograms", "20"),
    ("k_group_offsets", "group bounds", "4"),
    ("k_sort_small", "groups of 2..16 members (insertion sort == stable rank): 16 lanes per group from the tier list, width-16 shuffles; singletons are not touched (second stream)", "12 per member"),
    ("k_sort_groups_reg", "17..64 members in registers (17..32: two groups per wavefront, second stream; 33..64: main stream, after its LDS tiers)", "12 per member"),
    ("k_sort_groups_lds", "65..2048 members in LDS: partitions down to the leaves (a segment of <= 64 partitioned in registers: read once, stoppers by ballots, partners by lane permutes, written once), then the final insertion pass with ballot-found leaf bounds (257..2048: second stream, first)", "12 per member"),
    ("k_sort_groups_split", "groups above 2048: partitions down to 512-member segments, each a block-wide Hoare scan (both cursors a chunk at a time into LDS stopper queues, pairs swapped from the queues), groups claimed largest first", "12 per member"),
    ("k_sort_segments", "those segments, one LDS wavefront each", "12 per member"),
    ("k_heap_segments", "depth-exhausted segments of >= 2048 members (median-of-3 killers only): make_heap level-parallel; sort_heap by one wavefront: all-equal keys (the killer) as a spine FIFO, else top 13 heap levels in LDS", "-"),
    ("k_emit", "gid, flag, output order", "29"),
]


def main():
    d = json.load(open(os.path.join(ROOT, "profiles", BENCH)))
    t = json.load(open(os.path.join(ROOT, "profiles", "traffic.json")))["kernels"]
    k = d["kernels"]
    c5p = os.path.join(ROOT, "profiles", CFG5)
    k5 = json.load(open(c5p))["kernels"] if os.path.exists(c5p) else {}
    rows = ["| kernel | job | algorithmic B / element | ms / step | algorithmic GB/s | "
            "PMC HBM MB / launch | cfg5 ms / step |",
            "|---|---|---|---|---|---|---|"]
    for name, job, algo in JOBS:
        kk, tr = k.get(name, {}), t.get(PMC_NAME.get(name, name), {})
        ln = kk.get("launches_per_step", 0)
        hb = tr.get("hbm_bytes_per_launch")
        c5 = k5.get(name, {}).get("ms_per_step")
        rows.append(f"| `{name}`{' (x%g)' % ln if ln and ln != 1 else ''} | {job} | {algo} | "
                    f"{kk.get('ms_per_step', 0):.2f} | {kk.get('algo_GBps') or '-'} | "
                    f"{round(hb / 1e6) if hb else '-'} | {f'{c5:.1f}' if c5 else '-'} |")
    r = d["roofline"]
    step_bytes = sum(v.get("launches_per_step", 0) *
                     t.get(PMC_NAME.get(n, n), {}).get("hbm_bytes_per_launch", 0)
                     for n, v in k.items())
    rows.append("")
    rows.append(f"Step: {d['ms_per_step']:.2f} ms ({d['value'] / 1e9:.2f} G fragments/s); "
                f"roofline kernel `{r['kernel']}`: {r['launches_per_step']:g} launches, "
                f"{r['launch_ms']:.3f} ms each on average, {r['achieved']:.0f} GB/s, frac "
                f"{r['frac']:.3f}; PMC traffic "
                f"{t.get(r['kernel'], {}).get('hbm_bytes_per_launch', 0) / 1e6:.0f} MB per launch "
                f"against {r['algorithmic_bytes_per_launch'] / 1e6:.0f} MB algorithmic; "
                f"PMC traffic of the listed kernels {step_bytes / 1e9:.1f} GB per step.")
    path = os.path.join(ROOT, "DESIGN.md")
    s = open(path).read()
    a, b = s.index(BEGIN) + len(BEGIN), s.index(END)
    open(path, "w").write(s[:a] + "\n" + "\n".join(rows) + "\n" + s[b:])


if __name__ == "__main__":
    main()
