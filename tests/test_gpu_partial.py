"""GPU tier, partial decode, each against the reference
library built here (oracle/_ref) on the same inputs:

  * blosc2_decompress_block_ctx (ref blosc/blosc2.c:4580-4687): every block of chunks covering
    split / unsplit / leftover blocks, bitshuffle, DELTA (block decoded as the reference's serial
    blosc_d does with dest_offset 0), LZ4, memcpyed and special chunks; error codes;
  * b2h_frame_get_slice (ref blosc2_schunk_get_slice_buffer, schunk.c:1662-1760) on frames with
    many blocks per chunk, where edge chunks now decode only their touched blocks;
  * b2h_frame_get_sparse_buffer (ref blosc2_schunk_get_sparse_buffer, schunk.c:1921-2110):
    random and clustered coordinates, duplicates, DELTA, special chunks, error codes.

The frames are built at run time by the reference (blosc2_schunk_new / append_buffer /
fill_special / to_buffer) from the seeded generators in tests/datagen.py.
"""
import ctypes as C

import numpy as np
import pytest

from b2ctypes import CParams, DParams, cparams as ref_cparams, dparams as ref_dparams
from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import p, ref

pytestmark = pytest.mark.gpu


class Storage(C.Structure):
    """blosc2_storage (reference include/blosc2.h:1758-1771)."""
    _fields_ = [("contiguous", C.c_bool), ("urlpath", C.c_char_p), ("cparams", C.POINTER(CParams)),
                ("dparams", C.POINTER(DParams)), ("io", C.c_void_p)]


@pytest.fixture(scope="module")
def libs():
    import torch  # noqa: F401  (torch's HIP runtime first, then the engine)
    import blosc2_amd as B
    L = B.lib()
    assert L.b2h_device_count() > 0
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref absent")
    vp, i64 = C.c_void_p, C.c_int64
    for lib in (L, R):
        lib.blosc2_decompress_block_ctx.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, C.c_int32]
        lib.blosc2_decompress_block_ctx.restype = C.c_int
    L.b2h_frame_from_buffer.argtypes, L.b2h_frame_from_buffer.restype = [vp, i64, C.POINTER(C.c_int)], vp
    L.b2h_frame_free.argtypes, L.b2h_frame_free.restype = [vp], None
    L.b2h_frame_get_slice.argtypes, L.b2h_frame_get_slice.restype = [vp, i64, i64, vp], C.c_int
    L.b2h_frame_get_sparse_buffer.argtypes = [vp, i64, vp, vp]
    L.b2h_frame_get_sparse_buffer.restype = C.c_int
    R.blosc2_schunk_new.argtypes, R.blosc2_schunk_new.restype = [C.POINTER(Storage)], vp
    R.blosc2_schunk_append_buffer.argtypes, R.blosc2_schunk_append_buffer.restype = [vp, vp, C.c_int32], i64
    R.blosc2_schunk_fill_special.argtypes, R.blosc2_schunk_fill_special.restype = [vp, i64, C.c_int, C.c_int32], i64
    R.blosc2_schunk_to_buffer.argtypes = [vp, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_bool)]
    R.blosc2_schunk_to_buffer.restype = i64
    R.blosc2_schunk_from_buffer.argtypes, R.blosc2_schunk_from_buffer.restype = [vp, i64, C.c_bool], vp
    R.blosc2_schunk_free.argtypes, R.blosc2_schunk_free.restype = [vp], C.c_int
    R.blosc2_schunk_get_slice_buffer.argtypes, R.blosc2_schunk_get_slice_buffer.restype = [vp, i64, i64, vp], C.c_int
    R.blosc2_schunk_get_sparse_buffer.argtypes, R.blosc2_schunk_get_sparse_buffer.restype = [vp, i64, vp, vp], C.c_int
    R.blosc2_set_nthreads(1)
    return B, L, R


# ------------------------------------------------------------------ decompress_block_ctx ----
def _ref_chunk(R, raw, **kw):
    cp = ref_cparams(nthreads=1, **kw)
    ctx = R.blosc2_create_cctx(cp)
    src = raw.copy()
    out = np.zeros(raw.nbytes + 64, np.uint8)
    n = R.blosc2_compress_ctx(ctx, p(src), raw.nbytes, p(out), out.nbytes)
    R.blosc2_free_ctx(ctx)
    assert n > 0
    return out[:n].copy()


def _blocks(lib, dparams_fn, chunk, nblocks, bs):
    ctx = lib.blosc2_create_dctx(dparams_fn())
    outs = []
    for b in range(-1, nblocks + 1):
        buf = np.full(bs + 16, 0xEE, np.uint8)
        rc = lib.blosc2_decompress_block_ctx(ctx, p(chunk), chunk.nbytes, b, p(buf), bs + 16)
        outs.append((rc, buf.copy()))
    small = np.zeros(8, np.uint8)
    outs.append((lib.blosc2_decompress_block_ctx(ctx, p(chunk), chunk.nbytes, 0, p(small), 8), None))
    lib.blosc2_free_ctx(ctx)
    return outs


BLOCK_CASES = [
    # name, raw, cparams
    ("shuffle_split_leftover", gen_f32(1, 70_001).view(np.uint8), dict(typesize=4, blocksize=16384, filters=(0, 0, 0, 0, 0, 1))),
    ("bitshuffle", int64_ramp(5, 40_000).view(np.uint8), dict(typesize=8, blocksize=32768, filters=(0, 0, 0, 0, 0, 2))),
    ("delta_shuffle", int64_ramp(9, 30_000).view(np.uint8), dict(typesize=8, blocksize=16384, filters=(0, 0, 0, 0, 2, 1))),
    ("lz4_noshuffle_nosplit", mixed_bytes(3, 100_000), dict(typesize=1, blocksize=8192, filters=(0,) * 6, compcode=1, splitmode=2)),
    ("memcpyed", mixed_bytes(4, 50_000), dict(typesize=1, blocksize=8192, clevel=0, filters=(0,) * 6)),
    ("zeros_special", np.zeros(90_000, np.uint8), dict(typesize=4, blocksize=16384, filters=(0, 0, 0, 0, 0, 1))),
]


@pytest.mark.parametrize("case", BLOCK_CASES, ids=[c[0] for c in BLOCK_CASES])
def test_decompress_block_ctx_matches_reference(libs, case):
    B, L, R = libs
    name, raw, kw = case
    chunk = _ref_chunk(R, raw, **kw)
    bs = int(np.frombuffer(chunk[8:12].tobytes(), np.int32)[0])
    nbytes = raw.nbytes
    nblocks = -(-nbytes // bs)
    ours = _blocks(L, B.dparams, chunk, nblocks, bs)
    want = _blocks(R, ref_dparams, chunk, nblocks, bs)
    for b, ((rc, got), (rrc, exp)) in enumerate(zip(ours, want)):
        assert rc == rrc, (name, b - 1, rc, rrc)
        if rc > 0:
            assert np.array_equal(got[:rc], exp[:rc]), (name, b - 1)
    # without DELTA the block is the chunk's own slice of the input
    if 2 not in kw["filters"]:
        for b in range(nblocks):
            rc, got = ours[b + 1]
            assert np.array_equal(got[:rc], raw[b * bs:b * bs + rc]), (name, b)


# ------------------------------------------------------------------------------- frames ----
FRAME_CASES = [
    # name, source bytes, cparams, chunksize (bytes), specials: list of appended zero-chunk positions
    ("f32_shuffle_16k_blocks", gen_f32(2, 5 * 65536 + 12_345).view(np.uint8),
     dict(typesize=4, blocksize=16384, filters=(0, 0, 0, 0, 0, 1)), 262144, [2]),
    ("i64_delta_shuffle_8k_blocks", int64_ramp(7, 6 * 16384 + 999).view(np.uint8),
     dict(typesize=8, blocksize=8192, filters=(0, 0, 0, 0, 2, 1)), 131072, []),
    ("u8_lz4_bitshuffle", mixed_bytes(8, 3 * 65536 + 4320),
     dict(typesize=2, blocksize=4096, filters=(0, 0, 0, 0, 0, 2), compcode=1), 65536, [1]),
]


def _build_frame(R, raw, kw, chunksize, specials):
    cp = ref_cparams(nthreads=1, **kw)
    dp = ref_dparams(nthreads=1)
    st = Storage(True, None, C.pointer(cp), C.pointer(dp), None)
    sc = R.blosc2_schunk_new(C.byref(st))
    assert sc
    parts, pos, k = [], 0, 0
    while pos < raw.nbytes:
        n = min(chunksize, raw.nbytes - pos)
        # a zero chunk: the reference stores it as a special (zero-run) chunk
        a = np.zeros(n, np.uint8) if k in specials else raw[pos:pos + n].copy()
        assert R.blosc2_schunk_append_buffer(sc, p(a), n) > 0
        parts.append(a)
        pos += n
        k += 1
    buf = C.POINTER(C.c_uint8)()
    nf = C.c_bool()
    n = R.blosc2_schunk_to_buffer(sc, C.byref(buf), C.byref(nf))
    assert n > 0
    frame = np.ctypeslib.as_array(buf, shape=(n,)).copy()
    R.blosc2_schunk_free(sc)
    return frame, np.concatenate(parts)


@pytest.fixture(scope="module", params=FRAME_CASES, ids=[c[0] for c in FRAME_CASES])
def frame(libs, request):
    B, L, R = libs
    name, raw, kw, chunksize, specials = request.param
    fbytes, data = _build_frame(R, raw, kw, chunksize, specials)
    err = C.c_int(0)
    fr = L.b2h_frame_from_buffer(p(fbytes), fbytes.nbytes, C.byref(err))
    assert fr, err.value
    # frame-backed (copy=False), as b2h_frame is: blocksize from the frame header (frame.c:2957)
    sc = R.blosc2_schunk_from_buffer(p(fbytes), fbytes.nbytes, False)
    assert sc
    yield dict(name=name, fr=fr, sc=sc, data=data, ts=kw["typesize"], chunksize=chunksize, fbytes=fbytes)
    L.b2h_frame_free(fr)
    R.blosc2_schunk_free(sc)


def test_frame_slice_block_masked_edges(libs, frame):
    import torch
    B, L, R = libs
    ts, data = frame["ts"], frame["data"]
    nitems, cs = data.nbytes // ts, frame["chunksize"] // ts
    rng = np.random.default_rng(17)
    ranges = [(1, 2), (cs - 5, cs + 5), (cs + 100, 2 * cs - 100), (3, nitems - 3), (nitems - 1, nitems)]
    ranges += [tuple(sorted(rng.integers(0, nitems + 1, 2))) for _ in range(12)]
    for a, b in ranges:
        a, b = int(a), int(b)
        d = torch.full(((b - a) * ts + 64,), 0xEE, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        assert L.b2h_frame_get_slice(frame["fr"], a, b, d.data_ptr()) == 0, (a, b)
        got = d.cpu().numpy()
        exp = np.zeros(max((b - a) * ts, 1), np.uint8)
        if b > a:
            assert R.blosc2_schunk_get_slice_buffer(frame["sc"], a, b, p(exp)) == 0
        assert np.array_equal(got[:(b - a) * ts], exp[:(b - a) * ts]), (a, b)
        assert np.array_equal(got[:(b - a) * ts], data[a * ts:b * ts]), (a, b)
        assert (got[(b - a) * ts:] == 0xEE).all(), (a, b)


def _sparse(lib, fn, handle, coords, ts):
    c = np.ascontiguousarray(coords, np.int64)
    out = np.full(max(len(c), 1) * ts, 0xEE, np.uint8)
    rc = getattr(lib, fn)(handle, len(c), p(c) if len(c) else None, p(out))
    return rc, out[:len(c) * ts]


def test_frame_sparse_matches_reference(libs, frame):
    B, L, R = libs
    ts, data = frame["ts"], frame["data"]
    nitems, cs = data.nbytes // ts, frame["chunksize"] // ts
    rng = np.random.default_rng(23)
    sets = [
        rng.integers(0, nitems, 1),
        rng.integers(0, nitems, 1000),                             # random, duplicates likely
        np.concatenate([np.arange(cs - 40, cs + 40), [0, nitems - 1, 5, 5]]),   # clustered + repeats
        np.arange(nitems - 1, -1, -max(1, nitems // 777)),         # strided, descending
    ]
    for coords in sets:
        rc, got = _sparse(L, "b2h_frame_get_sparse_buffer", frame["fr"], coords, ts)
        rrc, exp = _sparse(R, "blosc2_schunk_get_sparse_buffer", frame["sc"], coords, ts)
        assert rc == rrc == 0, (rc, rrc)
        assert np.array_equal(got, exp)
        items = data.reshape(-1, ts)[np.asarray(coords, np.int64)].reshape(-1)
        assert np.array_equal(got, items)
    # error codes as the reference's
    for coords in ([nitems], [-1], [0, nitems + 5]):
        rc, _ = _sparse(L, "b2h_frame_get_sparse_buffer", frame["fr"], coords, ts)
        rrc, _ = _sparse(R, "blosc2_schunk_get_sparse_buffer", frame["sc"], coords, ts)
        assert rc == rrc == -12, (coords, rc, rrc)
    out = np.zeros(8, np.uint8)
    assert L.b2h_frame_get_sparse_buffer(frame["fr"], -1, None, p(out)) == \
        R.blosc2_schunk_get_sparse_buffer(frame["sc"], -1, None, p(out)) == -12
    assert L.b2h_frame_get_sparse_buffer(frame["fr"], 0, None, None) == 0
    assert L.b2h_frame_get_sparse_buffer(frame["fr"], 3, None, p(out)) == -12


def test_schunk_sparse_buffer_matches_reference(libs, frame):
    """blosc2_schunk_get_sparse_buffer on the reference's handle type (include/blosc2.h:2290,
    blosc/schunk.c:1922-2110): this library's frame-attached handle (from_buffer copy=False) and
    its in-memory copy (copy=True) against the reference's handle of the same flavour on the same
    frame -- the items, and the error codes of schunk.c:1923-1953 (a copy whose chunks have
    different blocksizes has blocksize 0: INVALID_PARAM in both)."""
    B, L, R = libs
    vp, i64 = C.c_void_p, C.c_int64
    L.blosc2_schunk_from_buffer.argtypes, L.blosc2_schunk_from_buffer.restype = [vp, i64, C.c_bool], vp
    L.blosc2_schunk_free.argtypes, L.blosc2_schunk_free.restype = [vp], C.c_int
    L.blosc2_schunk_get_sparse_buffer.argtypes = [vp, i64, vp, vp]
    L.blosc2_schunk_get_sparse_buffer.restype = C.c_int
    ts, data, fb = frame["ts"], frame["data"], frame["fbytes"]
    nitems, cs = data.nbytes // ts, frame["chunksize"] // ts
    rng = np.random.default_rng(31)
    sets = [
        rng.integers(0, nitems, 1),                                               # one: the getitem path
        rng.integers(0, nitems, 1500),                                            # random, duplicates
        np.concatenate([np.arange(cs - 40, cs + 40), [0, nitems - 1, 5, 5]]),     # clustered + repeats
        np.arange(nitems - 1, -1, -max(1, nitems // 501)),                        # strided, descending
        np.arange(0, nitems, 3),                                                  # every block of every chunk
    ]
    for copy in (False, True):
        sc = L.blosc2_schunk_from_buffer(p(fb), fb.nbytes, copy)
        rsc = R.blosc2_schunk_from_buffer(p(fb), fb.nbytes, copy)
        assert sc and rsc
        for coords in sets:
            rc, got = _sparse(L, "blosc2_schunk_get_sparse_buffer", sc, coords, ts)
            rrc, exp = _sparse(R, "blosc2_schunk_get_sparse_buffer", rsc, coords, ts)
            assert rc == rrc, (copy, rc, rrc)
            if rc < 0:
                continue
            assert np.array_equal(got, exp), copy
            assert np.array_equal(got, data.reshape(-1, ts)[np.asarray(coords, np.int64)].reshape(-1)), copy
        if not copy:   # the attached handle always has the frame's blocksize: every set decodes
            assert _sparse(L, "blosc2_schunk_get_sparse_buffer", sc, sets[1], ts)[0] == 0
        for coords in ([nitems], [-1], [0, nitems + 5], [3, 4, -2]):
            rc, _ = _sparse(L, "blosc2_schunk_get_sparse_buffer", sc, coords, ts)
            rrc, _ = _sparse(R, "blosc2_schunk_get_sparse_buffer", rsc, coords, ts)
            assert rc == rrc == -12, (coords, rc, rrc)
        out = np.zeros(64, np.uint8)
        c3 = np.arange(3, dtype=np.int64)
        for args in ((-1, None, p(out)), (0, None, None), (3, None, p(out)), (3, p(c3), None)):
            assert L.blosc2_schunk_get_sparse_buffer(sc, *args) == R.blosc2_schunk_get_sparse_buffer(rsc, *args), args
        assert L.blosc2_schunk_free(sc) == 0
        R.blosc2_schunk_free(rsc)
    assert L.blosc2_schunk_get_sparse_buffer(None, 3, p(np.arange(3, dtype=np.int64)), p(np.zeros(64, np.uint8))) == \
        R.blosc2_schunk_get_sparse_buffer(None, 3, p(np.arange(3, dtype=np.int64)), p(np.zeros(64, np.uint8))) == -12


@pytest.mark.parametrize("filters", [(0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 2, 1), (0, 0, 0, 0, 0, 2)],
                         ids=["shuffle", "delta_shuffle", "bitshuffle"])
def test_inmemory_schunk_sparse_buffer_matches_reference(libs, filters):
    """The in-memory super-chunk (blosc2_schunk_new, sparse storage, append_buffer) of both
    libraries, same cparams: sparse reads equal, including a zero-special chunk and a short last
    chunk; DELTA takes the per-item getitem path (schunk.c:1944-1948)."""
    B, L, R = libs
    vp, i64 = C.c_void_p, C.c_int64
    L.blosc2_schunk_get_sparse_buffer.argtypes = [vp, i64, vp, vp]
    L.blosc2_schunk_get_sparse_buffer.restype = C.c_int
    ts, chunk = 8, 1 << 17
    raw = int64_ramp(41, 5 * chunk // 8 + 777).view(np.uint8).copy()
    raw[2 * chunk:3 * chunk] = 0
    kw = dict(typesize=ts, blocksize=16384, filters=filters, clevel=5)
    ours = B.SChunk(B.cparams(**kw), B.dparams())
    rst = Storage(False, None, C.pointer(ref_cparams(nthreads=1, **kw)), C.pointer(ref_dparams(nthreads=1)), None)
    theirs = R.blosc2_schunk_new(C.byref(rst))
    for pos in range(0, raw.nbytes, chunk):
        a = raw[pos:pos + chunk].copy()
        assert ours.append_buffer(a) > 0
        assert R.blosc2_schunk_append_buffer(theirs, p(a), a.nbytes) > 0
    nitems = raw.nbytes // ts
    rng = np.random.default_rng(5)
    for coords in (rng.integers(0, nitems, 2000), np.arange(nitems - 1, 0, -97), [7]):
        rc, got = _sparse(L, "blosc2_schunk_get_sparse_buffer", ours.p, coords, ts)
        rrc, exp = _sparse(R, "blosc2_schunk_get_sparse_buffer", theirs, coords, ts)
        assert rc == rrc == 0, (rc, rrc)
        assert np.array_equal(got, exp)
        if 2 not in filters:
            assert np.array_equal(got, raw.reshape(-1, ts)[np.asarray(coords, np.int64)].reshape(-1))
    ours.free()
    R.blosc2_schunk_free(theirs)
