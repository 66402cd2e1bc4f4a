#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (tools/pmc_run.sh) per kernel.

HBM bytes per launch = FETCH_SIZE*k + WRITE_SIZE (KB units, x1024), where k=2
corrects gfx950's FETCH_SIZE under-count of wide coalesced reads
(MI355X_MICROARCH.md "HBM": FETCH_SIZE reads exactly half the bytes of a
16-B/lane streaming read).  Both raw and corrected values are printed; the
correction is calibrated per access pattern, so the raw numbers are kept too.
Writes profiles/traffic.json (cfg3) or profiles/traffic_<config>.json when
--write is given (--config names the bench config the passes ran).
"""
import collections
import csv
import glob
import json
import os
import re
import sys

# the segment kernel's instantiations by their emit type (bench.py's names)
SEG_EMIT = {"OrderEmit": "k_seg_fine (order)", "CsrEmit": "k_seg_fine (Y)",
            "MemberEmit": "k_seg_fine (members)"}


def kernel_key(name: str) -> str:
    m = re.search(r"(k_\w+)", name)
    nm = m.group(1) if m else name
    if nm == "k_seg_fine":
        for emit, key in SEG_EMIT.items():
            if emit in name:
                return key
    return nm


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(path)):
            nm = kernel_key(r["Kernel_Name"])
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            agg[nm][r["Counter_Name"]].append((float(r["Counter_Value"]), dur))
    return agg

def main():
    config = "cfg3"  # the bench config the PMC passes ran (bench.py --config)
    argv = sys.argv[1:]
    if "--config" in argv:
        i = argv.index("--config")
        config = argv[i + 1]
        del argv[i:i + 2]
    args = [a for a in argv if a != "--write"]
    d = args[0] if args else "gpurun_out/pmc"
    agg = load(d)
    out = {}
    for nm in sorted(agg, key=lambda k: -sum(v[1] for v in agg[k].get("FETCH_SIZE", [(0, 0)]))):
        c = agg[nm]
        avg = {k: sum(x[0] for x in v) / len(v) for k, v in c.items()}
        if "FETCH_SIZE" not in avg:
            continue
        fetch = avg["FETCH_SIZE"] * 1024
        write = avg.get("WRITE_SIZE", 0.0) * 1024
        ms = sum(x[1] for x in c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        row = {"launches": len(c["FETCH_SIZE"]), "avg_ms": round(ms, 4),
               "fetch_bytes_raw": round(fetch), "write_bytes": round(write),
               "hbm_bytes_per_launch": round(2 * fetch + write),
               "hbm_GBps_corrected": round((2 * fetch + write) / (ms * 1e-3) / 1e9, 1) if ms else None}
        for k in ("SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                  "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "TCC_HIT_sum",
                  "TCC_MISS_sum"):
            if k in avg:
                row[k] = round(avg[k])
        out[nm] = row
        print(nm, row)
    if "--write" in sys.argv:
        os.makedirs("profiles", exist_ok=True)
        meta = {"method": "rocprofv3 --pmc, one pass per counter group (tools/pmc_run.sh); "
                          "hbm_bytes_per_launch = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 "
                          "(MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts half of a 16-B/lane "
                          "streaming read)",
                "command": " ".join(args[1:]) or "python3 bench.py --no-cpu --steps 3 --warmup 1"}
        name = "traffic.json" if config == "cfg3" else f"traffic_{config}.json"
        with open(os.path.join("profiles", name), "w") as f:
            json.dump({"meta": meta, "config": config, "kernels": out}, f, indent=1,
                      sort_keys=True)

if __name__ == "__main__":
    main()
