"""GPU tier: the multi-device fan-out reachable from C (include/b2h.h b2h_schunk_append_buffers /
b2h_schunk_decompress_buffers; c-blosc2_amd/csrc/b2h_schunk.cpp).

The reference's C caller loops blosc2_schunk_append_buffer / blosc2_schunk_decompress_chunk over its
chunks (blosc/schunk.c:1459-1530); here many chunks from host memory go out to `ndevices` workers
(one host thread each, worker k on device k % count).  The box has one GPU, so 2-5 workers share it:
that still runs the partition, the per-worker contexts, the sticky-blocksize hand-over at each
worker's first chunk and the in-order append.  Checked: every chunk equals the serial
blosc2_schunk_append_buffer's (and, in exact mode, the oracle's), the super-chunk's context ends in
the serial state (the next serial append agrees), the decompressed host buffers equal the source,
status codes and argument errors match blosc2_schunk_decompress_chunk's.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _chunks(nchunks, chunk, seed):
    from datagen import gen_f32
    raw = gen_f32(seed, nchunks * chunk // 4).view(np.uint8)
    sizes = np.full(nchunks, chunk, np.int32)
    sizes[-1] = chunk - 4 * 1234          # a shorter last chunk: a different plan, the blocksize walk moves
    sizes[nchunks // 2] = chunk // 2      # and one in the middle (a worker may start right after it)
    return raw, sizes


@pytest.mark.parametrize("lz_mode", [0, 1], ids=["exact", "fast"])
@pytest.mark.parametrize("workers", [1, 2, 5])
def test_gpu_append_buffers_equals_serial_appends(lz_mode, workers):
    import blosc2_amd as B
    from oracle_lib import oracle_compress
    L = B.lib()
    chunk, n = 1 << 20, 11
    raw, sizes = _chunks(n, chunk, 40 + workers)
    kw = dict(clevel=5, typesize=4)
    fan = B.SChunk(B.cparams(**kw, lz_mode=lz_mode), B.dparams())
    ser = B.SChunk(B.cparams(**kw, lz_mode=lz_mode), B.dparams())
    r = L.b2h_schunk_append_buffers(fan.p, _p(raw), _p(sizes), n, chunk, workers)
    assert r == n, r
    for i in range(n):
        assert ser.append_buffer(raw[i * chunk:i * chunk + int(sizes[i])]) == i + 1
    for i in range(n):
        a, b = fan.chunk(i), ser.chunk(i)
        assert isinstance(a, np.ndarray) and np.array_equal(a, b), i
        if lz_mode == 0 and i in (0, n // 2, n - 1):
            assert np.array_equal(a, oracle_compress(raw[i * chunk:i * chunk + int(sizes[i])], **kw)), i
    # the context carries on from the serial state: one more chunk of each agrees
    extra = raw[:chunk]
    assert fan.append_buffer(extra) == ser.append_buffer(extra) == n + 1
    assert np.array_equal(fan.chunk(n), ser.chunk(n))
    assert fan.counters() == ser.counters()

    # decompress through the fan-out into host memory
    dst_stride = chunk + 64
    out = np.zeros((n + 1) * dst_stride, np.uint8)
    st = np.zeros(n + 1, np.int32)
    rc = L.b2h_schunk_decompress_buffers(fan.p, 0, n + 1, _p(out), dst_stride, chunk, _p(st), workers)
    assert rc == 0, rc
    want = list(sizes) + [chunk]
    assert list(st) == want
    for i in range(n):
        assert np.array_equal(out[i * dst_stride:i * dst_stride + int(sizes[i])], raw[i * chunk:i * chunk + int(sizes[i])]), i
    assert np.array_equal(out[n * dst_stride:n * dst_stride + chunk], extra)
    fan.free()
    ser.free()


@pytest.mark.parametrize("workers", [1, 2])
def test_gpu_fanout_streams_groups(workers):
    """Ranges larger than one staging group (128 MiB) stream through the pinned ring: 80 chunks of
    4 MiB (3 groups for one worker), chunk for chunk the serial appends' bytes, and back."""
    import blosc2_amd as B
    L = B.lib()
    chunk, n = 4 << 20, 80
    raw, sizes = _chunks(n, chunk, 90 + workers)
    fan = B.SChunk(B.cparams(clevel=5, typesize=4, lz_mode=1), B.dparams())
    ser = B.SChunk(B.cparams(clevel=5, typesize=4, lz_mode=1), B.dparams())
    assert L.b2h_schunk_append_buffers(fan.p, _p(raw), _p(sizes), n, chunk, workers) == n
    for i in range(n):
        assert ser.append_buffer(raw[i * chunk:i * chunk + int(sizes[i])]) == i + 1
    for i in range(n):
        assert np.array_equal(fan.chunk(i), ser.chunk(i)), i
    assert fan.counters() == ser.counters()
    out = np.zeros(n * chunk, np.uint8)
    st = np.zeros(n, np.int32)
    assert L.b2h_schunk_decompress_buffers(fan.p, 0, n, _p(out), chunk, chunk, _p(st), workers) == 0
    assert list(st) == list(sizes)
    for i in range(n):
        assert np.array_equal(out[i * chunk:i * chunk + int(sizes[i])], raw[i * chunk:i * chunk + int(sizes[i])]), i
    fan.free()
    ser.free()


def test_gpu_fanout_argument_errors():
    import blosc2_amd as B
    L = B.lib()
    chunk = 1 << 16
    raw, sizes = _chunks(4, chunk, 7)
    sc = B.SChunk(B.cparams(clevel=5, typesize=4), B.dparams())
    assert L.b2h_schunk_append_buffers(sc.p, _p(raw), _p(sizes), 4, chunk, 0) == 4
    out = np.zeros(4 * chunk, np.uint8)
    st = np.zeros(4, np.int32)
    INVALID = -12   # BLOSC2_ERROR_INVALID_PARAM
    assert L.b2h_schunk_decompress_buffers(sc.p, 2, 3, _p(out), chunk, chunk, _p(st), 2) == INVALID   # past the end
    assert L.b2h_schunk_decompress_buffers(sc.p, 0, 2, _p(out), chunk // 2, chunk, _p(st), 2) == INVALID   # stride < capacity
    bad = sizes.copy()
    bad[1] = chunk + 1   # longer than the source stride
    assert L.b2h_schunk_append_buffers(sc.p, _p(raw), _p(bad), 4, chunk, 2) == INVALID
    assert sc.s.nchunks == 4   # nothing appended on error
    # too small a destination: the chunk's own status, as blosc2_schunk_decompress_chunk reports it
    rc = L.b2h_schunk_decompress_buffers(sc.p, 0, 4, _p(out), chunk, 1000, _p(st), 2)
    r0, _ = sc.decompress_chunk(0, 1000)
    assert st[0] == r0 < 0
    sc.free()


@pytest.mark.parametrize("workers", [1, 2])
def test_gpu_fanout_postfilter_over_groups(workers):
    """A decompression context with a postfilter: every chunk of a range spanning
    several 128 MiB staging groups must go through the postfilter (out = in * 2, the callback of
    tests/plugins/b2h_prepost.c), none through the device-only staged path.  The staged decode
    classifies group g + 1 on a helper thread while group g runs the postfilter path; the
    postfilter field of the shared context is never rewritten during a call."""
    import blosc2_amd as B
    from b2ctypes import REPO
    L = B.lib()
    PP = C.CDLL(os.path.join(REPO, "tests", "plugins", "libb2h_prepost.so"))

    class PPUser(C.Structure):
        _fields_ = [("mode", C.c_int32), ("fail_block", C.c_int32), ("inputs", C.c_void_p * 2),
                    ("nrec", C.c_int32), ("cap", C.c_int32), ("rec", C.c_void_p)]

    class PostParams(C.Structure):
        _fields_ = [("user_data", C.c_void_p), ("input", C.c_void_p), ("output", C.c_void_p),
                    ("size", C.c_int32), ("typesize", C.c_int32), ("offset", C.c_int32),
                    ("nchunk", C.c_int64), ("nblock", C.c_int32), ("tid", C.c_int32), ("ttmp", C.c_void_p),
                    ("ttmp_nbytes", C.c_size_t), ("ctx", C.c_void_p)]
    user = PPUser(0, -1, (C.c_void_p * 2)(None, None), 0, 0, None)   # no call record (threads)
    post = PostParams()
    post.user_data = C.cast(C.pointer(user), C.c_void_p)
    dp = B.dparams()
    dp.postfilter, dp.postparams = C.cast(PP.b2h_postfilter, C.c_void_p), C.cast(C.pointer(post), C.c_void_p)
    chunk, n = 4 << 20, 72                     # 288 MiB: 3 groups for one worker
    raw = (np.arange(n * chunk // 4, dtype=np.int32) % 100_003).view(np.uint8)
    sizes = np.full(n, chunk, np.int32)
    sc = B.SChunk(B.cparams(clevel=5, typesize=4, lz_mode=1), dp)
    assert L.b2h_schunk_append_buffers(sc.p, _p(raw), _p(sizes), n, chunk, workers) == n
    out = np.zeros(n * chunk, np.uint8)
    st = np.zeros(n, np.int32)
    assert L.b2h_schunk_decompress_buffers(sc.p, 0, n, _p(out), chunk, chunk, _p(st), workers) == 0
    assert (st == chunk).all()
    want = (raw.view(np.int32) * 2).view(np.uint8)
    bad = [i for i in range(n) if not np.array_equal(out[i * chunk:(i + 1) * chunk], want[i * chunk:(i + 1) * chunk])]
    assert not bad, bad[:8]
    sc.free()
