"""Summarise bench JSON lines: step time, phases, top kernels.  usage: bsum.py FILE..."""
import json
import sys

for fn in sys.argv[1:]:
    try:
        d = json.loads(open(fn).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(fn, "unreadable", e)
        continue
    print(f"== {fn}: {d['ms_per_step']} ms/step  value {d['value']/1e9:.3f} G/s  "
          f"roofline {d.get('roofline', {}) and d['roofline'].get('kernel')} "
          f"{d.get('roofline', {}) and d['roofline'].get('frac')}")
    print("   phases", d.get("phases_ms"))
    ks = sorted(d.get("kernels", {}).items(), key=lambda kv: -kv[1]["ms_per_step"])[:12]
    print("   " + "  ".join(f"{k}={v['ms_per_step']}" for k, v in ks))
