"""Encoder micro-benchmark fixtures (diagnostics only): the four 64 KiB byte planes of the first
256 KiB block of the T workload (gen_f32, shuffle ts=4) and the oracle's BloscLZ clevel-5 stream of
each (empty file when the oracle stores the plane raw).   python tools/make_enc_fixtures.py"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from datagen import gen_f32  # noqa: E402
from oracle_lib import oracle, p  # noqa: E402

blk = gen_f32(0, 65536).view(np.uint8)
planes = blk.reshape(-1, 4).T.copy()
L = oracle()
for k in range(4):
    x = np.ascontiguousarray(planes[k])
    out = np.zeros(x.nbytes + 64, np.uint8)
    n = L.or_blosclz_compress(5, p(x), x.nbytes, p(out), x.nbytes)
    x.tofile(os.path.join(HERE, "fixtures", f"f32_p{k}.bin"))
    out[:max(n, 0)].tofile(os.path.join(HERE, "fixtures", f"f32_p{k}.out"))
    print(f"plane {k}: {x.nbytes} -> {n}")
