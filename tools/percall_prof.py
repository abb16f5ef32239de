"""Per-call drop-in path timing (diagnostics): blosc1_compress / blosc1_decompress on host buffers,
C1's 4 MB chunk, one call at a time (bench/b2bench.c:199, 227).  Run under
rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace to see where a call's time goes.
    python tools/percall_prof.py [exact|fast] [ncalls]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "c-blosc2_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import torch  # noqa: F401  (one HIP runtime)
import blosc2_amd as B
from datagen import b2bench_values


def main(mode="exact", n=20):
    L = B.lib()
    L.b2h_set_blosclz_mode({"exact": 0, "fast": 1}[mode])
    L.blosc1_set_compressor(b"blosclz")
    size = 4_000_000
    src = b2bench_values(1_000_000, 19)
    cap = size + 32
    dst = np.zeros(cap, np.uint8)
    back = np.zeros(size, np.uint8)
    p = lambda a: a.ctypes.data
    c = L.blosc1_compress(5, 1, 4, size, p(src), p(dst), cap)
    L.blosc1_decompress(p(dst), p(back), size)
    tc, td = [], []
    for _ in range(int(n)):
        t0 = time.perf_counter()
        c = L.blosc1_compress(5, 1, 4, size, p(src), p(dst), cap)
        t1 = time.perf_counter()
        L.blosc1_decompress(p(dst), p(back), size)
        t2 = time.perf_counter()
        tc.append(t1 - t0)
        td.append(t2 - t1)
    assert np.array_equal(back, src.view(np.uint8))
    print(f"{mode}: csize {c}, compress {np.median(tc) * 1e3:.3f} ms/call "
          f"({size / np.median(tc) / 1e9:.2f} GB/s), decompress {np.median(td) * 1e3:.3f} ms/call "
          f"({size / np.median(td) / 1e9:.2f} GB/s)")


if __name__ == "__main__":
    main(*sys.argv[1:3])
