#!/usr/bin/env python3
"""Host read rate of page-locked (torch pin_memory) against pageable (numpy)
buffers: one thread copying 400 MB out of each into a prefaulted pageable
buffer, best of 5, and how each buffer is mapped (/proc/self/smaps: the
mapping's AnonHugePages, i.e. whether it is backed by 2-MB transparent huge
pages).  The wire upload packs the caller's columns on host threads
(rk_io.hip io_h2d_rows), so its rate follows how fast the host reads them;
the hardware prefetchers stop at every page boundary of a 4-KB-page buffer."""
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


def mapping(addr: int) -> dict:
    """The smaps entry of the mapping holding addr: its size and huge-page share."""
    cur = None
    with open("/proc/self/smaps") as fh:
        for line in fh:
            head = line.split()[0]
            if "-" in head and not head.endswith(":"):
                lo, hi = (int(x, 16) for x in head.split("-"))
                cur = {"kB": (hi - lo) // 1024} if lo <= addr < hi else None
            elif cur is not None and head in ("AnonHugePages:", "KernelPageSize:", "Locked:"):
                cur[head[:-1]] = line.split()[1] + " kB"
                if head == "Locked:":
                    return cur
    return cur or {}


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
                      "pinned_read_GBps": round(rate(pin, dst), 2),
                      "pageable_mapping": mapping(page.ctypes.data),
                      "pinned_mapping": mapping(pin.ctypes.data)}))


if __name__ == "__main__":
    main()
