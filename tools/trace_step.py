#!/usr/bin/env python3
"""Timeline of the last classification step in a rocprofv3 kernel_trace.csv:
queue, start/end (us from the step's first kernel), duration, kernel name.
usage: trace_step.py KERNEL_TRACE_CSV [first-kernel-name] [from-name]"""
import csv
import re
import sys

path = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_nw_order_hist"
frm = sys.argv[3] if len(sys.argv) > 3 else None
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
s, e = idx[-2], idx[-1]
t0 = int(rows[s]["Start_Timestamp"])
on = frm is None
for r in rows[s:e]:
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    nm = m.group(1) if m else r["Kernel_Name"][:30]
    on = on or (frm in nm)
    if not on:
        continue
    a = (int(r["Start_Timestamp"]) - t0) / 1e3
    b = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{r.get('Queue_Id', '?'):>3} {a:9.1f} {b:9.1f} {b - a:8.1f} {nm}")
