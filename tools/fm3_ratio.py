"""Segmented fast-mode parse (tools/fm_model.c fm3_*): stream-size ratios against exact mode
(the oracle's blosclz_compress) and today's fast mode, for segment sizes S, on the streams of T,
C1, C3 and C4 (CPU only).  Also checks that every segmented stream
decodes with the oracle's blosclz_decompress restatement.
  python tools/fm3_ratio.py [S ...]"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from datagen import b2bench_values, gen_f32, int64_ramp  # noqa: E402
from oracle_lib import oracle, p  # noqa: E402

FM = C.CDLL(os.path.join(HERE, "..", "oracle", "libfm_model.so"))
for f in ("fm_blosclz_compress", "fm3_blosclz_compress"):
    getattr(FM, f).argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
FM.fm_set_segment.argtypes = [C.c_int]
O = oracle()


def planes(raw, ts, bs, bit=False, delta=False):
    out = []
    for b in range(raw.nbytes // bs):
        blk = np.ascontiguousarray(raw[b * bs:(b + 1) * bs])
        if delta:
            x = blk.view(np.uint64)
            ref0 = raw[:bs].view(np.uint64)   # block 0 of the chunk (chunk = the whole array here)
            d = x.copy()
            if b == 0:
                d[1:] = x[1:] ^ x[:-1]
            else:
                d = x ^ ref0
            blk = d.view(np.uint8)
        sh = np.empty_like(blk)
        if bit:
            O.or_bitshuffle(ts, bs, p(blk), p(sh))
            out.append(sh)
        else:
            O.or_shuffle(ts, bs, p(blk), p(sh))
            out += [np.ascontiguousarray(sh[j * (bs // ts):(j + 1) * (bs // ts)]) for j in range(ts)]
    return out


def sizes(streams, fn, clevel=5):
    tot, bad = 0, 0
    for s in streams:
        out = np.zeros(s.nbytes + s.nbytes // 8 + 64, np.uint8)
        n = fn(clevel, p(s), s.nbytes, p(out), s.nbytes, 13)
        if n > 0 and fn is FM.fm3_blosclz_compress:
            back = np.zeros(s.nbytes, np.uint8)
            if O.or_blosclz_decompress(p(out), n, p(back), s.nbytes) != s.nbytes or not np.array_equal(back, s):
                bad += 1
        tot += (n if n > 0 else s.nbytes) + 4
    return tot, bad


def exact(streams, clevel=5):
    tot = 0
    for s in streams:
        out = np.zeros(s.nbytes + 64, np.uint8)
        n = O.or_blosclz_compress(clevel, p(s), s.nbytes, p(out), s.nbytes)
        tot += (n if n > 0 else s.nbytes) + 4
    return tot


def main():
    segs = [int(a) for a in sys.argv[1:]] or [1024, 2048, 4096, 8192]
    cfgs = {
        "T": planes(gen_f32(0, 4 << 20).view(np.uint8), 4, 262144),
        "C1": planes(b2bench_values(1 << 20, 19).view(np.uint8), 4, 262144),
        "C3": planes(gen_f32(77, 1 << 20).view(np.uint8), 4, 262144, bit=True),
        "C4": planes(int64_ramp(0, 1 << 17).view(np.uint8), 8, 262144, delta=True),
    }
    for name, st in cfgs.items():
        ex = exact(st)
        fa, _ = sizes(st, FM.fm_blosclz_compress)
        row = [f"{name}: {len(st)} streams, exact {ex}, fast {fa / ex:.4f}"]
        for S in segs:
            FM.fm_set_segment(S)
            s3, bad = sizes(st, FM.fm3_blosclz_compress)
            row.append(f"S={S} {s3 / ex:.4f}" + (f" ({bad} undecodable)" if bad else ""))
        print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
