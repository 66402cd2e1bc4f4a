"""Summarise an RK_NW_TRACE file: per record pass, the per-tile phase times
(prologue: block start -> loads issued; load+rank; scan+look-back;
scatter+write) in microseconds (100 MHz clock)."""
import sys

import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
npass = int(raw[0])
hdr = raw[1:1 + 2 * npass].reshape(npass, 2)
body = raw[1 + 2 * npass:]
for p, (off, tiles) in enumerate(hdr):
    t = body[off:off + tiles * 8].reshape(tiles, 8).astype(np.int64)
    t0, t1, t2, t3, te = t[:, 0], t[:, 1], t[:, 2], t[:, 3], t[:, 6]
    span = (t3.max() - te.min()) / 100.0
    ph = [(t0 - te) / 100.0, (t1 - t0) / 100.0, (t2 - t1) / 100.0, (t3 - t2) / 100.0, (t3 - te) / 100.0]
    # concurrency: average number of tiles in flight
    conc = (t3 - te).sum() / max(1, (t3.max() - te.min()))
    print(f"pass {p}: tiles {tiles} span {span:.1f} us  in-flight {conc:.0f}  "
          + "  ".join(f"{nm} mean {x.mean():.2f} p50 {np.median(x):.2f} p99 {np.percentile(x, 99):.2f}"
                      for nm, x in zip(("prologue", "rank", "lookback", "write", "block"), ph)))
