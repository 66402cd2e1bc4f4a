#!/usr/bin/env python3
"""Host read rate of page-locked (torch pin_memory) against pageable (numpy)
buffers: one thread copying 400 MB out of each into a prefaulted pageable
buffer, best of 5.  The wire upload packs the caller's columns on host threads
(rk_io.hip io_h2d_rows), so its rate follows how fast the host reads them."""
import json
import time

import numpy as np
import torch


def rate(src: np.ndarray, dst: np.ndarray) -> float:
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        np.copyto(dst, src)
        best = min(best, time.perf_counter() - t)
    return src.nbytes / best / 1e9


def main():
    n = 50_000_000
    dst = np.empty(n, np.uint64)
    dst[:] = 0
    page = np.arange(n, dtype=np.uint64)
    pin_t = torch.empty(n, dtype=torch.int64, pin_memory=True)
    pin_t.copy_(torch.from_numpy(page.view(np.int64)))
    pin = pin_t.numpy().view(np.uint64)
    print(json.dumps({"bytes": int(page.nbytes),
                      "pageable_read_GBps": round(rate(page, dst), 2),
                      "pinned_read_GBps": round(rate(pin, dst), 2)}))


if __name__ == "__main__":
    main()
