"""Contiguous-frame read path: frames written by the reference library
(tests/golden/make_frames.py -> tests/golden/frame_*.b2frame) read back through b2h_frame_* and
decoded on the device, checked against the data the frames were built from and against a CPU
reading of the same frames (header fields of blosc/frame.h:29-49, offsets index = a Blosc chunk
decoded by the oracle restatement)."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

from b2ctypes import REPO
from datagen import gen_f32, int64_ramp
from oracle_lib import oracle_decompress

GOLD = os.path.join(REPO, "tests", "golden")
MANIFEST = json.load(open(os.path.join(GOLD, "frames.json")))


def frame_bytes(name):
    return np.fromfile(os.path.join(GOLD, name + ".b2frame"), np.uint8)


def source_data(case):
    """The bytes each frame was built from (tests/golden/make_frames.py:cases)."""
    name = case["name"]
    if name == "frame_f32_shuffle":
        return gen_f32(0, 4 * 65536 + 25_000).view(np.uint8)
    if name == "frame_i64_delta":
        return int64_ramp(0, 8 * 16384).view(np.uint8)
    if name == "frame_f32_bytedelta":
        return gen_f32(0, 3 * 32768).view(np.uint8)
    return np.zeros(case["nbytes"], np.uint8)


def be(b, off, n):
    return int.from_bytes(bytes(b[off:off + n]), "big", signed=(n == 4))


def cpu_read_frame(f):
    """CPU reading of a contiguous frame with the oracle: header fields (blosc/frame.h:29-49),
    offsets index at header_len + cbytes (blosc/frame.c:2102-2155), chunks decoded one by one."""
    header_len, nbytes, cbytes = be(f, 11, 4), be(f, 30, 8), be(f, 39, 8)
    typesize, chunksize = be(f, 48, 4), be(f, 58, 4)
    nchunks = nbytes // chunksize + (1 if nbytes % chunksize else 0)
    off_pos = header_len + cbytes
    off_cbytes = int(np.frombuffer(f[off_pos + 12:off_pos + 16].tobytes(), np.int32)[0])
    offsets = oracle_decompress(f[off_pos:off_pos + off_cbytes].copy(), nchunks * 8).view(np.int64)
    out = []
    for i in range(nchunks):
        n = chunksize if i < nchunks - 1 or nbytes % chunksize == 0 else nbytes % chunksize
        o = int(offsets[i])
        if o < 0:
            assert (o >> 56) & 7 == 1   # BLOSC2_SPECIAL_ZERO
            out.append(np.zeros(n, np.uint8))
            continue
        p = header_len + o
        cb = int(np.frombuffer(f[p + 12:p + 16].tobytes(), np.int32)[0])
        out.append(oracle_decompress(f[p:p + cb].copy(), n))
    return dict(nbytes=nbytes, typesize=typesize, chunksize=chunksize, nchunks=nchunks), np.concatenate(out)


@pytest.mark.parametrize("case", MANIFEST, ids=[c["name"] for c in MANIFEST])
def test_frame_fixture_cpu_reading(case):
    """The committed frames decode (on the CPU oracle) to the data they were built from."""
    info, data = cpu_read_frame(frame_bytes(case["name"]))
    assert info["nbytes"] == case["nbytes"] and info["chunksize"] == case["chunksize"]
    assert hashlib.sha256(data.tobytes()).hexdigest() == case["sha256"]
    assert np.array_equal(data, source_data(case))


class FrameInfo(C.Structure):
    _fields_ = [("nbytes", C.c_int64), ("cbytes", C.c_int64), ("nchunks", C.c_int64),
                ("typesize", C.c_int32), ("blocksize", C.c_int32), ("chunksize", C.c_int32),
                ("compcode", C.c_uint8), ("clevel", C.c_uint8),
                ("filters", C.c_uint8 * 6), ("filters_meta", C.c_uint8 * 6)]


@pytest.fixture(scope="module")
def L():
    import torch  # noqa: F401
    import sys
    sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
    import blosc2_amd
    L = blosc2_amd.lib()
    vp = C.c_void_p
    L.b2h_frame_open.argtypes, L.b2h_frame_open.restype = [C.c_char_p, C.POINTER(C.c_int)], vp
    L.b2h_frame_from_buffer.argtypes, L.b2h_frame_from_buffer.restype = [vp, C.c_int64, C.POINTER(C.c_int)], vp
    L.b2h_frame_free.argtypes, L.b2h_frame_free.restype = [vp], None
    L.b2h_frame_get_info.argtypes, L.b2h_frame_get_info.restype = [vp, C.POINTER(FrameInfo)], C.c_int
    L.b2h_frame_decompress.argtypes, L.b2h_frame_decompress.restype = [vp, vp, C.c_int64], C.c_int64
    L.b2h_frame_decompress_chunk.argtypes, L.b2h_frame_decompress_chunk.restype = [vp, C.c_int64, vp, C.c_int32], C.c_int
    L.b2h_frame_get_slice.argtypes, L.b2h_frame_get_slice.restype = [vp, C.c_int64, C.c_int64, vp], C.c_int
    return L


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST, ids=[c["name"] for c in MANIFEST])
def test_frame_device_read(L, case):
    import torch
    want = source_data(case)
    path = os.path.join(GOLD, case["name"] + ".b2frame").encode()
    err = C.c_int(0)
    fr = L.b2h_frame_open(path, C.byref(err))
    assert fr, err.value
    info = FrameInfo()
    assert L.b2h_frame_get_info(fr, C.byref(info)) == 0
    assert info.nbytes == case["nbytes"] and info.chunksize == case["chunksize"]
    assert info.typesize == case["cparams"]["typesize"]
    assert list(info.filters) == list(case["cparams"]["filters"])
    d = torch.full((info.nbytes + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # the frame runs on its own non-blocking stream
    assert L.b2h_frame_decompress(fr, d.data_ptr(), d.numel()) == info.nbytes
    got = d[:info.nbytes].cpu().numpy()
    assert np.array_equal(got, want)
    # per-chunk reads (blosc2_schunk_decompress_chunk semantics)
    for i in range(info.nchunks):
        n = min(info.chunksize, info.nbytes - i * info.chunksize)
        buf = np.zeros(info.chunksize, np.uint8)
        assert L.b2h_frame_decompress_chunk(fr, i, buf.ctypes.data, buf.nbytes) == n
        assert np.array_equal(buf[:n], want[i * info.chunksize:i * info.chunksize + n])
    small = np.zeros(8, np.uint8)
    assert L.b2h_frame_decompress_chunk(fr, 0, small.ctypes.data, 8) == -6       # WRITE_BUFFER
    assert L.b2h_frame_decompress_chunk(fr, info.nchunks, small.ctypes.data, 8) == -12   # INVALID_PARAM
    L.b2h_frame_free(fr)


@pytest.mark.gpu
def test_frame_from_buffer_and_damage(L):
    f = frame_bytes("frame_i64_delta")
    err = C.c_int(0)
    fr = L.b2h_frame_from_buffer(f.ctypes.data, f.nbytes, C.byref(err))
    assert fr and err.value == 0
    L.b2h_frame_free(fr)
    bad = f.copy()
    bad[3] ^= 0xFF                                      # magic
    assert not L.b2h_frame_from_buffer(bad.ctypes.data, bad.nbytes, C.byref(err)) and err.value == -11
    bad = f.copy()
    bad[26] = 1                                         # sparse frame type
    assert not L.b2h_frame_from_buffer(bad.ctypes.data, bad.nbytes, C.byref(err)) and err.value == -24
    assert not L.b2h_frame_from_buffer(f.ctypes.data, 60, C.byref(err)) and err.value == -5
    assert not L.b2h_frame_open(b"/nonexistent/frame.b2frame", C.byref(err)) and err.value == -15


@pytest.mark.gpu
@pytest.mark.parametrize("case", MANIFEST, ids=[c["name"] for c in MANIFEST])
def test_frame_get_slice(L, case):
    """b2h_frame_get_slice == blosc2_schunk_get_slice_buffer (blosc/schunk.c:1662-1760): item
    ranges inside one block, across block and chunk boundaries, whole chunks, the ragged tail."""
    import torch
    want = source_data(case)
    ts = case["cparams"]["typesize"]
    nitems = case["nbytes"] // ts
    cs = case["chunksize"] // ts
    err = C.c_int(0)
    fr = L.b2h_frame_open(os.path.join(GOLD, case["name"] + ".b2frame").encode(), C.byref(err))
    assert fr, err.value
    ranges = [(0, 1), (5, 17), (cs - 3, cs + 9), (cs, 2 * cs), (cs // 2, 3 * cs + 11),
              (nitems - 7, nitems), (0, nitems), (nitems // 3, nitems // 3)]
    for a, b in ranges:
        a, b = max(0, min(a, nitems)), max(0, min(b, nitems))
        d = torch.full(((b - a) * ts + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()   # the frame runs on its own non-blocking stream
        assert L.b2h_frame_get_slice(fr, a, b, d.data_ptr()) == 0, (a, b)
        got = d.cpu().numpy()
        assert np.array_equal(got[:(b - a) * ts], want[a * ts:b * ts]), (a, b)
        assert (got[(b - a) * ts:] == 0xEE).all(), (a, b)      # nothing written past the slice
    d = torch.zeros(64, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()   # the frame runs on its own non-blocking stream
    assert L.b2h_frame_get_slice(fr, 0, nitems + 1, d.data_ptr()) == -12
    assert L.b2h_frame_get_slice(fr, 5, 4, d.data_ptr()) == -12
    L.b2h_frame_free(fr)
