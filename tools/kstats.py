#!/usr/bin/env python3
"""Per-step kernel table from a rocprofv3 --stats kernel_stats.csv (calls / classify calls)."""
import csv
import re
import sys

path, ncalls = sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in list(csv.DictReader(open(path)))[:40]:
    m = re.search(r"(k_\w+)", r["Name"])
    nm = m.group(1) if m else r["Name"][:30]
    print(f"{nm:30s} calls/step={int(r['Calls']) / ncalls:7.1f} ms/step={float(r['TotalDurationNs']) / ncalls / 1e6:8.3f} "
          f"avg_us={float(r['AverageNs']) / 1e3:9.1f} max_us={float(r['MaxNs']) / 1e3:9.1f}")
