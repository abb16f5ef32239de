"""Generate the contiguous-frame fixtures (tests/golden/frame_*.b2frame + frames.json) with the
reference library compiled from /root/reference sources (oracle/_ref/libblosc2_ref.so): super-chunks
built with blosc2_schunk_new / blosc2_schunk_append_buffer / blosc2_schunk_fill_special
(blosc/schunk.c) and serialised with blosc2_schunk_to_buffer (blosc/frame.c).  Test-fixture
generator only; run in the container where the reference exists:

    python tests/golden/make_frames.py
"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from b2ctypes import cparams, dparams, CParams, DParams  # noqa: E402
from datagen import gen_f32, int64_ramp  # noqa: E402
from oracle_lib import ref  # noqa: E402


class Storage(C.Structure):
    """blosc2_storage (reference include/blosc2.h:1758-1771)."""
    _fields_ = [("contiguous", C.c_bool), ("urlpath", C.c_char_p), ("cparams", C.POINTER(CParams)),
                ("dparams", C.POINTER(DParams)), ("io", C.c_void_p)]


# name, cparams, list of ("data", array) / ("zeros", nitems) appends
def cases():
    f32 = gen_f32(0, 4 * 65536 + 25_000)            # 4 full 256 KiB chunks + a 100 KB tail
    ramp = int64_ramp(0, 8 * 16384)                 # 8 x 128 KiB
    yield ("frame_f32_shuffle", dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)), 262144,
           [("data", f32[i * 65536:(i + 1) * 65536]) for i in range(4)] + [("data", f32[4 * 65536:])])
    yield ("frame_i64_delta", dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1)), 131072,
           [("data", ramp[i * 16384:(i + 1) * 16384]) for i in range(8)])
    yield ("frame_f32_bytedelta", dict(clevel=9, typesize=4, filters=(0, 0, 0, 0, 1, 35),
                                       filters_meta=(0, 0, 0, 0, 0, 4)), 131072,
           [("data", f32[i * 32768:(i + 1) * 32768]) for i in range(3)])
    yield ("frame_special_zeros", dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)), 65536,
           [("zeros", 3 * 16384 + 1000)])


def main():
    R = ref()
    assert R is not None, "build oracle/_ref first (make -C oracle ref)"
    R.blosc2_schunk_new.argtypes, R.blosc2_schunk_new.restype = [C.POINTER(Storage)], C.c_void_p
    R.blosc2_schunk_append_buffer.argtypes, R.blosc2_schunk_append_buffer.restype = [C.c_void_p, C.c_void_p, C.c_int32], C.c_int64
    R.blosc2_schunk_fill_special.argtypes, R.blosc2_schunk_fill_special.restype = [C.c_void_p, C.c_int64, C.c_int, C.c_int32], C.c_int64
    R.blosc2_schunk_to_buffer.argtypes, R.blosc2_schunk_to_buffer.restype = [C.c_void_p, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_bool)], C.c_int64
    R.blosc2_schunk_free.argtypes, R.blosc2_schunk_free.restype = [C.c_void_p], C.c_int
    manifest = []
    for name, kw, chunk, appends in cases():
        cp = cparams(nthreads=1, **kw)
        dp = dparams(nthreads=1)
        st = Storage(True, None, C.pointer(cp), C.pointer(dp), None)
        sc = R.blosc2_schunk_new(C.byref(st))
        assert sc
        raw = []
        for kind, a in appends:
            if kind == "data":
                assert R.blosc2_schunk_append_buffer(sc, a.ctypes.data, a.nbytes) > 0
                raw.append(a.view(np.uint8).reshape(-1))
            else:
                assert R.blosc2_schunk_fill_special(sc, a, 1, chunk) >= 0   # BLOSC2_SPECIAL_ZERO
                raw.append(np.zeros(a * kw["typesize"], np.uint8))
        buf = C.POINTER(C.c_uint8)()
        nf = C.c_bool()
        n = R.blosc2_schunk_to_buffer(sc, C.byref(buf), C.byref(nf))
        assert n > 0
        frame = np.ctypeslib.as_array(buf, shape=(n,)).copy()
        R.blosc2_schunk_free(sc)
        data = np.concatenate(raw)
        frame.tofile(os.path.join(HERE, name + ".b2frame"))
        import hashlib
        manifest.append(dict(name=name, cparams=kw, chunksize=chunk, nbytes=int(data.nbytes),
                             sha256=hashlib.sha256(data.tobytes()).hexdigest(),
                             generator="tests/golden/make_frames.py:cases " + name))
        print(name, n, "bytes frame for", data.nbytes)
    json.dump(manifest, open(os.path.join(HERE, "frames.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
