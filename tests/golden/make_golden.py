"""Generate tests/golden/chunks.{json,npz}: small chunks compressed by the REFERENCE library
(oracle/_ref/libblosc2_ref.so, built from /root/reference sources by oracle/Makefile) with
nthreads=1.  Inputs are deterministic (tests/datagen.py).  Each case stays a few KiB to a few
hundred KiB so the fixture is small; together they cover every stream kind: zero run, byte run,
raw (incompressible), LZ, leftover block, memcpyed (clevel 0 / tiny / incompressible chunk),
SPECIAL_ZERO, and the filters shuffle / bitshuffle / delta / trunc-prec.

Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from datagen import gen_f32, int64_ramp, mixed_bytes  # noqa: E402
from oracle_lib import ref, ref_compress  # noqa: E402

SH, BSH, DEL, TRN = 1, 2, 3, 4


def cases():
    rng = np.random.default_rng(2024)
    f32 = gen_f32(0, 16384)
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH])
    yield dict(src=f32, clevel=9, typesize=4, filters=[0, 0, 0, 0, 0, SH])
    yield dict(src=f32, clevel=1, typesize=4, filters=[0, 0, 0, 0, 0, SH])
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, BSH])
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, 0])
    yield dict(src=f32[:10000], clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH], blocksize=12000)
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, TRN, DEL, SH], filters_meta=[0, 0, 0, -6, 0, 0],
               lossless=False)  # leftover
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, 0, TRN, SH], filters_meta=[0, 0, 0, 0, 12, 0],
               lossless=False)
    yield dict(src=f32, clevel=5, typesize=4, filters=[0, 0, 0, 0, DEL, SH])
    yield dict(src=gen_f32(100, 8), clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH])  # tiny -> memcpyed
    yield dict(src=f32[:4096], clevel=0, typesize=4, filters=[0, 0, 0, 0, 0, SH])       # clevel 0
    r64 = int64_ramp(0, 16384)
    yield dict(src=r64, clevel=5, typesize=8, filters=[0, 0, 0, 0, DEL, SH])
    yield dict(src=r64, clevel=5, typesize=8, filters=[0, 0, 0, 0, DEL, BSH])
    yield dict(src=r64, clevel=9, typesize=8, filters=[0, 0, 0, 0, 0, SH])
    yield dict(src=np.zeros(32768, np.uint8), clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH])  # SPECIAL_ZERO
    yield dict(src=np.full(32768, 7, np.uint8), clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH])  # byte runs
    yield dict(src=rng.integers(0, 256, 16384, dtype=np.uint8), clevel=5, typesize=4,
               filters=[0, 0, 0, 0, 0, SH])                                                   # incompressible
    for seed in range(8):
        n = int(rng.integers(2000, 40000))
        yield dict(src=mixed_bytes(seed, n), clevel=int(rng.integers(1, 10)), typesize=1,
                   filters=[0, 0, 0, 0, 0, 0], splitmode=2)
    for seed in range(8):
        ts = int(rng.choice([2, 4, 8, 16]))
        n = int(rng.integers(2000, 40000)) // ts * ts
        yield dict(src=mixed_bytes(50 + seed, n), clevel=int(rng.integers(1, 10)), typesize=ts,
                   filters=[0, 0, 0, 0, 0, int(rng.choice([SH, BSH]))],
                   blocksize=int(rng.choice([0, 8192, 32768])))
    for cl in range(1, 10):
        yield dict(src=gen_f32(cl * 1000, 8192), clevel=cl, typesize=4, filters=[0, 0, 0, 0, 0, SH])
    # odd typesizes and the filters_meta "byte group" shuffle
    yield dict(src=mixed_bytes(77, 30000), clevel=5, typesize=3, filters=[0, 0, 0, 0, 0, SH])
    yield dict(src=mixed_bytes(78, 30000), clevel=5, typesize=12, filters=[0, 0, 0, 0, DEL, SH])
    yield dict(src=gen_f32(5, 16384), clevel=5, typesize=4, filters=[0, 0, 0, 0, 0, SH],
               filters_meta=[0, 0, 0, 0, 0, 2])


def main():
    assert ref() is not None, "build the reference first: make -C oracle ref"
    man, arrays = [], {}
    for i, c in enumerate(cases()):
        src = np.ascontiguousarray(c.pop("src"))
        kw = dict(clevel=5, typesize=4, filters=[0] * 6, filters_meta=[0] * 6, blocksize=0, splitmode=4)
        kw.update(c)
        lossless = kw.pop("lossless", True)
        # the reference rewrites its input in place when >= 3 filters are active
        # (blosc/blosc2.c:1048, 1173-1176), so it gets a private copy
        out = ref_compress(src.copy(), **kw)
        assert isinstance(out, np.ndarray), (i, out)
        arrays[f"in_{i}"] = src.view(np.uint8).reshape(-1).copy()
        arrays[f"out_{i}"] = out
        man.append(dict(kw, nbytes=int(src.nbytes), cbytes=int(out.nbytes), lossless=lossless))
    np.savez_compressed(os.path.join(HERE, "chunks.npz"), **arrays)
    json.dump(man, open(os.path.join(HERE, "chunks.json"), "w"), indent=1)
    print(len(man), "cases")


if __name__ == "__main__":
    main()
