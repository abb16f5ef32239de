"""Host-side ceilings of the PCIe-inclusive paths on the GPU box (not a test): memcpy between
pinned (hipHostMalloc through torch) and pageable memory, and positioned reads of a page-cached
file, each split over T threads (ctypes releases the GIL).  One JSON line per (what, T).

    python tools/host_copy_probe.py [--mib 1024]
"""
import argparse
import ctypes as C
import json
import os
import threading
import time

import numpy as np
import torch

libc = C.CDLL(None)
libc.memcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
libc.pread.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_long]
libc.pread.restype = C.c_ssize_t


def par(T, n, fn):
    th = [threading.Thread(target=fn, args=(n * t // T, n * (t + 1) // T)) for t in range(T)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    a = ap.parse_args()
    n = a.mib << 20
    pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    pin.fill_(1)
    page = np.ones(n, np.uint8)
    pp, gp = pin.data_ptr(), page.ctypes.data
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "probe.bin")
    page.tofile(path)
    fd = os.open(path, os.O_RDONLY)
    for T in (1, 2, 4, 8, 12, 16):
        for what, fn in (("pinned_to_pageable", lambda lo, hi: libc.memcpy(gp + lo, pp + lo, hi - lo)),
                         ("pageable_to_pinned", lambda lo, hi: libc.memcpy(pp + lo, gp + lo, hi - lo)),
                         ("pread_to_pinned", lambda lo, hi: libc.pread(fd, pp + lo, hi - lo, lo)),
                         ("pread_to_pageable", lambda lo, hi: libc.pread(fd, gp + lo, hi - lo, lo))):
            best = min(par(T, n, fn) for _ in range(3))
            print(json.dumps({"what": what, "threads": T, "GB_per_s": round(n / best / 1e9, 2)}), flush=True)
    os.close(fd)
    os.remove(path)
    print(json.dumps({"cpus": os.cpu_count(), "affinity": len(os.sched_getaffinity(0))}))


if __name__ == "__main__":
    main()
