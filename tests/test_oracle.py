"""CPU tier: pin the oracle restatement (oracle/blosc2_oracle.c) against the reference's own
known-answer vectors (compat/*.cdata, copied into tests/golden/) and, where it was built from the
reference sources (oracle/_ref), against the reference library itself."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

from datagen import gen_f32, int64_ramp, mixed_bytes
from b2ctypes import dparams
from oracle_lib import oracle, oracle_compress, oracle_decompress, p, ref, ref_compress

GOLD = os.path.join(os.path.dirname(__file__), "golden")
RAMP = np.arange(1_000_000, dtype=np.int32)   # compat/filegen.c:23, 178-180

# sha256 of compat/shuffle-2.20.0.cdata and compat/bitshuffle-2.20.0.cdata (4 MB each, not copied)
SHUFFLE_KAT = "40e1351bba9155c3d765d66b5b4d25cb104aa2ad4b844b0a5d20af40cab2b920"
BITSHUFFLE_KAT = "a1bba6ced356ddca157010f340b8b5a39a5cd43a77b7c99cd1cb8896e853169d"


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_shuffle_kat():
    out = np.zeros(RAMP.nbytes, np.uint8)
    assert oracle().or_shuffle(4, RAMP.nbytes, p(RAMP), p(out)) == RAMP.nbytes
    assert sha(out) == SHUFFLE_KAT
    back = np.zeros_like(out)
    oracle().or_unshuffle(4, RAMP.nbytes, p(out), p(back))
    assert np.array_equal(back.view(np.int32), RAMP)


def test_bitshuffle_kat():
    out = np.zeros(RAMP.nbytes, np.uint8)
    oracle().or_bitshuffle(4, RAMP.nbytes, p(RAMP), p(out))
    assert sha(out) == BITSHUFFLE_KAT
    back = np.zeros_like(out)
    oracle().or_bitunshuffle(4, RAMP.nbytes, p(out), p(back), 5)
    assert np.array_equal(back.view(np.int32), RAMP)


def test_blosclz_chunk_kat():
    """compat/blosc-blosclz-3.0.0.cdata == blosc1_compress(9, SHUFFLE, 4, ramp) with 1 thread."""
    gold = np.fromfile(os.path.join(GOLD, "blosc-blosclz-3.0.0.cdata"), np.uint8)
    got = oracle_compress(RAMP, clevel=9, typesize=4)
    assert isinstance(got, np.ndarray) and got.nbytes == gold.nbytes == 16910
    assert np.array_equal(got, gold)
    dec = oracle_decompress(gold, RAMP.nbytes)
    assert np.array_equal(dec.view(np.int32), RAMP)


@pytest.mark.parametrize("name", ["blosc-1.3.0-blosclz.cdata", "blosc-1.7.0-blosclz.cdata",
                                  "blosc-1.11.1-blosclz.cdata", "blosc-1.14.0-blosclz.cdata"])
def test_blosc1_decode_kat(name):
    """Blosc1 16-byte-header chunks decode to the ramp (compat/CMakeLists.txt:11-33)."""
    gold = np.fromfile(os.path.join(GOLD, name), np.uint8)
    dec = oracle_decompress(gold, RAMP.nbytes)
    assert isinstance(dec, np.ndarray), dec
    assert np.array_equal(dec.view(np.int32), RAMP)


def test_golden_chunks():
    """Small chunks produced by the reference (tests/golden/make_golden.py) re-encode byte-exactly."""
    man = json.load(open(os.path.join(GOLD, "chunks.json")))
    data = np.load(os.path.join(GOLD, "chunks.npz"))
    assert len(man) >= 40
    for i, case in enumerate(man):
        src = data[f"in_{i}"]
        want = data[f"out_{i}"]
        kw = {k: case[k] for k in ("clevel", "typesize", "filters", "filters_meta", "blocksize", "splitmode")}
        got = oracle_compress(src, **kw)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), (i, case)
        dec = oracle_decompress(want, src.nbytes)
        if case.get("lossless", True):
            assert np.array_equal(dec, src.view(np.uint8)), (i, case)


# ---------------------------------------------------------------- oracle vs reference ----
needs_ref = pytest.mark.skipif(ref() is None, reason="reference not built (oracle/_ref)")


def _bytes_equal(a, b):
    return isinstance(a, np.ndarray) and isinstance(b, np.ndarray) and np.array_equal(a, b)


@needs_ref
@pytest.mark.parametrize("ts", [1, 2, 3, 4, 7, 8, 16, 17, 80])
@pytest.mark.parametrize("nelem", [7, 192, 500, 1792, 8000])
def test_filters_vs_ref(ts, nelem):
    """test_shuffle_roundtrip_*.csv / test_bitshuffle_roundtrip.csv style grid, byte-exact."""
    R, O = ref(), oracle()
    rng = np.random.default_rng(ts * 1000 + nelem)
    src = rng.integers(0, 256, ts * nelem + 3, dtype=np.uint8)
    n = src.nbytes
    a, b = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    for fo, fr in (("or_shuffle", "blosc2_shuffle"), ("or_unshuffle", "blosc2_unshuffle"),
                   ("or_bitshuffle", "blosc2_bitshuffle")):
        getattr(O, fo)(ts, n, p(src), p(a))
        getattr(R, fr)(ts, n, p(src), p(b))
        assert np.array_equal(a, b), fo
    O.or_bitunshuffle(ts, n, p(src), p(a), 6)
    R.blosc2_bitunshuffle(ts, n, p(src), p(b))
    assert np.array_equal(a, b)


def _inputs():
    yield "f32", gen_f32(0, 1 << 18), 4
    yield "ramp64", int64_ramp(5, 1 << 17), 8
    yield "mixed", mixed_bytes(3, 700_001), 1
    yield "mixed4", mixed_bytes(4, 400_000).view(np.int32), 4
    yield "zeros", np.zeros(300_000, np.uint8), 4
    yield "const", np.full(100_000, 0x41, np.uint8), 2
    yield "rand", np.random.default_rng(9).integers(0, 256, 250_000, dtype=np.uint8), 4


@needs_ref
@pytest.mark.parametrize("clevel", [1, 2, 3, 5, 9])
@pytest.mark.parametrize("filters", [(0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 2), (0, 0, 0, 0, 3, 1),
                                     (0, 0, 0, 0, 0, 0)])
def test_chunks_vs_ref(clevel, filters):
    for name, src, ts in _inputs():
        want = ref_compress(src, clevel=clevel, typesize=ts, filters=filters)
        got = oracle_compress(src, clevel=clevel, typesize=ts, filters=filters)
        assert _bytes_equal(got, want), (name, clevel, filters)


@needs_ref
def test_trunc_delta_vs_ref():
    src = gen_f32(7, 1 << 16)
    for filters, meta in (((0, 0, 0, 0, 4, 1), (0, 0, 0, 0, 10, 0)), ((0, 0, 0, 4, 3, 1), (0, 0, 0, -6, 0, 0)),
                          ((0, 0, 0, 0, 1, 3), (0,) * 6)):
        want = ref_compress(src, clevel=5, typesize=4, filters=filters, filters_meta=meta)
        got = oracle_compress(src, clevel=5, typesize=4, filters=filters, filters_meta=meta)
        assert _bytes_equal(got, want), filters


@needs_ref
@pytest.mark.parametrize("seed", range(12))
def test_blosclz_streams_vs_ref(seed):
    """Raw codec: random lengths/clevels, oracle BloscLZ vs reference chunks with NEVER_SPLIT
    and no filters (so each block is one BloscLZ stream)."""
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 300_000))
    src = mixed_bytes(seed + 100, n)
    cl = int(rng.integers(1, 10))
    bs = int(rng.choice([0, 4096, 65536, 100_000]))
    want = ref_compress(src, clevel=cl, typesize=1, filters=(0,) * 6, blocksize=bs, splitmode=2)
    got = oracle_compress(src, clevel=cl, typesize=1, filters=(0,) * 6, blocksize=bs, splitmode=2)
    assert _bytes_equal(got, want), (n, cl, bs)
    dec = oracle_decompress(want, n)
    assert np.array_equal(dec, src)


# ---- registered plugin filters the device also runs: bytedelta (35), int_trunc (36) ----
PLUGIN_PIPES = [
    dict(typesize=4, filters=(0, 0, 0, 0, 1, 35), filters_meta=(0, 0, 0, 0, 0, 4)),
    dict(typesize=8, filters=(0, 0, 0, 0, 1, 35), filters_meta=(0, 0, 0, 0, 0, 8)),
    dict(typesize=4, filters=(0, 0, 0, 0, 35, 1), filters_meta=(0, 0, 0, 0, 4, 0)),
    dict(typesize=2, filters=(0, 0, 0, 36, 1, 35), filters_meta=(0, 0, 0, 9, 0, 2)),
    dict(typesize=8, filters=(0, 0, 0, 0, 36, 1), filters_meta=(0, 0, 0, 0, (-20) & 0xFF, 0)),
    dict(typesize=4, filters=(0, 0, 0, 36, 3, 35), filters_meta=(0, 0, 0, 20, 0, 3)),
    dict(typesize=1, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, 5)),
]


def plugin_input(kw, n, seed):
    from datagen import gen_f32, int64_ramp
    ts = kw["typesize"]
    if ts == 4:
        return gen_f32(seed, n // 4).view(np.uint8)
    if ts == 8:
        return int64_ramp(seed * 1000, n // 8).view(np.uint8)
    rng = np.random.default_rng(seed)
    return (np.cumsum(rng.integers(-3, 4, n // ts), dtype=np.int64) & (256 ** ts - 1)).astype(
        {1: np.uint8, 2: np.uint16}[ts]).view(np.uint8)


@pytest.mark.parametrize("case", range(len(PLUGIN_PIPES)))
@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_plugin_filters_oracle_vs_reference(case, clevel):
    """bytedelta / int_trunc pipelines (plugins/filters/*/test_*.c shapes: SHUFFLE then BYTEDELTA):
    the oracle restatement produces the reference library's chunk bytes and decodes them back."""
    R = ref()
    if R is None:
        pytest.skip("reference library not built")
    kw = dict(PLUGIN_PIPES[case], clevel=clevel)
    for n, bs in ((200_000, 0), (3 * 65536 + 4096, 65536)):
        src = plugin_input(kw, n, case * 7 + clevel)
        want = ref_compress(src, blocksize=bs, **kw)
        got = oracle_compress(src, blocksize=bs, **kw)
        assert isinstance(want, np.ndarray) and isinstance(got, np.ndarray)
        assert np.array_equal(got, want), (kw, n)
        dec = oracle_decompress(want, src.nbytes)
        rdec = np.zeros(src.nbytes, np.uint8)
        dctx = R.blosc2_create_dctx(dparams())
        assert R.blosc2_decompress_ctx(dctx, p(want), want.nbytes, p(rdec), rdec.nbytes) == src.nbytes
        R.blosc2_free_ctx(dctx)
        assert np.array_equal(dec, rdec)
        if 36 not in kw["filters"]:
            assert np.array_equal(dec, src)


def test_plugin_filter_errors_match_reference():
    """int_trunc with an impossible precision and bytedelta with meta 0 outside a super-chunk fail
    the pipeline (BLOSC2_ERROR_FILTER_PIPELINE) in both."""
    R = ref()
    if R is None:
        pytest.skip("reference library not built")
    src = gen_f32(0, 50_000).view(np.uint8)
    for kw in (dict(typesize=4, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, 40)),
               dict(typesize=4, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, (-32) & 0xFF)),
               dict(typesize=3, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, 4))):
        assert ref_compress(src[:49_998] if kw["typesize"] == 3 else src, **kw) == -18, kw
        assert oracle_compress(src[:49_998] if kw["typesize"] == 3 else src, **kw) == -18, kw


# ---------------------------------------------------------------------------------- LZ4 ----
# LZ4 (compformat 1) is a third-party dependency absent from /root/reference; the image ships
# lz4 1.9.3 (/opt/conda/lib/liblz4.so.1, the library oracle/_ref links).  The restatement is
# pinned byte-for-byte against that library directly, and at chunk level against oracle/_ref.
LZ4_SO = "/opt/conda/lib/liblz4.so.1"
needs_lz4 = pytest.mark.skipif(not os.path.exists(LZ4_SO), reason="liblz4 not in this image")


def _lz4_inputs():
    f = gen_f32(0, 1 << 16).view(np.uint8)
    sh = np.ascontiguousarray(f[:262144].reshape(-1, 4).T).reshape(-1)
    rng = np.random.default_rng(11)
    yield from (f[:65536], f[:65536 + 11], f[:200_000], sh[:65536], sh[196608:], sh)
    yield int64_ramp(0, 16384).view(np.uint8)
    for n in (0, 1, 12, 13, 14, 100, 4096, 70_000):
        yield rng.integers(0, 4, n, dtype=np.uint8)
        yield rng.integers(0, 256, n, dtype=np.uint8)
    yield np.zeros(65536, np.uint8)
    yield np.tile(np.arange(7, dtype=np.uint8), 20_000)


@needs_lz4
def test_lz4_codec_vs_liblz4():
    """or_lz4_compress == LZ4_compress_fast for every acceleration blosc uses (10 - clevel) and
    output limits below and above LZ4_compressBound; or_lz4_decompress inverts it."""
    L, O = C.CDLL(LZ4_SO), oracle()
    for a in _lz4_inputs():
        a = np.ascontiguousarray(a)
        for accel in (1, 2, 5, 9):
            for maxout in (a.nbytes, a.nbytes // 2, max(a.nbytes // 8, 1), a.nbytes + a.nbytes // 255 + 16):
                o1, o2 = np.zeros(maxout + 64, np.uint8), np.zeros(maxout + 64, np.uint8)
                r1 = L.LZ4_compress_fast(p(a), p(o1), a.nbytes, maxout, accel)
                r2 = O.or_lz4_compress(accel, p(a), a.nbytes, p(o2), maxout)
                assert r1 == r2 and np.array_equal(o1[:r1], o2[:r2]), (a.nbytes, accel, maxout)
                if r1 > 0 and a.nbytes:
                    d = np.zeros(a.nbytes + 8, np.uint8)
                    assert O.or_lz4_decompress(p(o1), r1, p(d), a.nbytes) == a.nbytes
                    assert np.array_equal(d[:a.nbytes], a)


@needs_lz4
def test_lz4_decoder_rejections_vs_liblz4():
    """Corrupted / truncated streams: the restatement accepts exactly what LZ4_decompress_safe
    accepts, with the same output."""
    L, O = C.CDLL(LZ4_SO), oracle()
    rng = np.random.default_rng(5)
    for a in (gen_f32(3, 1 << 14).view(np.uint8), int64_ramp(0, 8192).view(np.uint8)):
        o = np.zeros(a.nbytes * 2 + 64, np.uint8)
        r = L.LZ4_compress_fast(p(a), p(o), a.nbytes, o.nbytes, 1)
        for t in range(400):
            c = o[:r].copy()
            if t % 3 == 0:
                c[rng.integers(0, r)] = rng.integers(0, 256)
            elif t % 3 == 1:
                c = c[:rng.integers(1, r)].copy()
            else:
                for _ in range(3):
                    c[rng.integers(0, r)] ^= 1 << rng.integers(0, 8)
            for cap in (a.nbytes, a.nbytes + 7):
                d1, d2 = np.zeros(cap + 64, np.uint8), np.zeros(cap + 64, np.uint8)
                r1 = L.LZ4_decompress_safe(p(c), p(d1), c.nbytes, cap)
                r2 = O.or_lz4_decompress(p(c), c.nbytes, p(d2), cap)
                assert (r1 >= 0) == (r2 >= 0), (t, cap, r1, r2)
                if r1 >= 0:
                    assert r1 == r2 and np.array_equal(d1[:r1], d2[:r2])


@needs_ref
@pytest.mark.parametrize("clevel", [1, 5, 9])
@pytest.mark.parametrize("filters", [(0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 2), (0, 0, 0, 0, 3, 1),
                                     (0, 0, 0, 0, 0, 0)])
def test_lz4_chunks_vs_ref(clevel, filters):
    """Whole chunks with compcode BLOSC_LZ4: the oracle's bytes are the reference library's."""
    for name, src, ts in _inputs():
        want = ref_compress(src, clevel=clevel, typesize=ts, filters=filters, compcode=1)
        got = oracle_compress(src, clevel=clevel, typesize=ts, filters=filters, compcode=1)
        assert _bytes_equal(got, want), (name, clevel, filters)
        back = oracle_decompress(got, src.nbytes)
        assert np.array_equal(back, src.view(np.uint8).reshape(-1)), name


@needs_ref
@pytest.mark.parametrize("clevel", [1, 5, 9])
@pytest.mark.parametrize("filters", [(0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 3, 1)])
def test_lz4_dict_chunks_match_reference(clevel, filters):
    """LZ4 with use_dict (blosc/blosc2.c:3151-3235 -> LZ4_loadDict + LZ4_compress_fast_continue,
    lz4 1.9.3 external-dictionary mode): the oracle's chunks are the reference library's byte for
    byte -- the dictionary taken from the training pass's filtered blocks with the size word
    stored over four of them -- and decode (oracle and reference) back to the input."""
    R = ref()
    for name, src, ts in _inputs():
        kw = dict(clevel=clevel, typesize=ts, filters=filters, compcode=1, use_dict=1)
        want = ref_compress(src, **kw)
        got = oracle_compress(src, **kw)
        assert _bytes_equal(got, want), (name, clevel, filters)
        raw = src.view(np.uint8).reshape(-1)
        back = oracle_decompress(got, raw.nbytes)
        out = np.zeros(raw.nbytes + 64, np.uint8)
        ctx = R.blosc2_create_dctx(dparams(nthreads=1))
        rc = R.blosc2_decompress_ctx(ctx, p(got), got.nbytes, p(out), out.nbytes)
        R.blosc2_free_ctx(ctx)
        if got[2] & 0x02:
            # the memcpyed fallback keeps the dictionary flag, and the reference then reads the
            # dictionary size from the data (blosc/blosc2.c:2790-2803): its own chunk fails
            assert rc < 0 and isinstance(back, int) and back == rc, (name, rc, back)
            continue
        assert rc == raw.nbytes and np.array_equal(out[:raw.nbytes], raw), name
        assert np.array_equal(back, raw), name


def _ref_chunk(src, destsize, **kw):
    from b2ctypes import cparams
    R = ref()
    ctx = R.blosc2_create_cctx(cparams(**kw))
    raw = src.view(np.uint8).reshape(-1).copy()
    out = np.zeros(raw.nbytes + (1 << 18), np.uint8)   # the training pass may store past destsize
    n = R.blosc2_compress_ctx(ctx, p(raw), raw.nbytes, p(out), destsize)
    R.blosc2_free_ctx(ctx)
    return out[:n] if n > 0 else n


def _oracle_chunk(src, destsize, **kw):
    from oracle_lib import or_cparams
    raw = src.view(np.uint8).reshape(-1)
    out = np.zeros(max(destsize, raw.nbytes + 32) + 64, np.uint8)
    n = oracle().or_compress_chunk(C.byref(or_cparams(**kw)), p(raw), raw.nbytes, p(out), destsize)
    return out[:n] if n > 0 else n


@needs_ref
def test_lz4_dict_destsize_sweep():
    """use_dict under tight destsizes: the training pass needs only the header to fit, gives the
    chunk up (0) when a block finds no room at all, and reports BLOSC2_ERROR_WRITE_BUFFER when a
    block finds some (blosc/blosc2.c:1343-1356, 1417-1420, 2940-2965, 3036-3052)."""
    for src, ts in ((mixed_bytes(11, 40_000), 1), (gen_f32(3, 10_000), 4)):
        for bs in (0, 64, 256, 4096):
            for ds in list(range(28, 80, 3)) + [100, 300, 1000, 4128, 4129, 8000, 39999, 40031, 40032, 40033]:
                kw = dict(clevel=5, typesize=ts, compcode=1, use_dict=1, blocksize=bs)
                a, b = _oracle_chunk(src, ds, **kw), _ref_chunk(src, ds, **kw)
                assert (a == b) if isinstance(b, int) else _bytes_equal(a, b), (ts, bs, ds, b)


@needs_ref
@pytest.mark.parametrize("filters,meta", [((0, 0, 0, 3, 1, 2), (0,) * 6), ((0, 0, 0, 4, 3, 1), (0, 0, 0, 16, 0, 0))])
def test_lz4_dict_three_filters_vs_ref(filters, meta):
    """Three filters rewrite the input during the training pass; the real pass filters it again."""
    src = gen_f32(7, 300_000)
    for clevel in (1, 5, 9):
        kw = dict(clevel=clevel, typesize=4, filters=filters, filters_meta=meta, compcode=1, use_dict=1)
        assert _bytes_equal(oracle_compress(src, **kw), ref_compress(src, **kw)), kw


LZ4_KATS = ["blosc-lz4-3.0.0.cdata", "blosc-1.11.1-lz4.cdata", "blosc-1.14.0-lz4.cdata",
            "blosc-1.17.1-lz4-bitshuffle4-memcpy.cdata", "blosc-1.17.1-lz4-bitshuffle8-nomemcpy.cdata",
            "blosc-1.18.0-lz4-bitshuffle4-memcpy.cdata", "blosc-1.18.0-lz4-bitshuffle8-nomemcpy.cdata"]


@pytest.mark.parametrize("name", LZ4_KATS)
def test_lz4_decode_kats(name):
    """compat/*lz4*.cdata (the int32 ramp of compat/filegen.c:178-180, written by Blosc 1.11 .. 3.0
    with LZ4) decode to the ramp (compat/CMakeLists.txt:15-33 `filegen decompress`)."""
    gold = np.fromfile(os.path.join(GOLD, name), np.uint8)
    nbytes, ts = int(gold[4:8].view(np.int32)[0]), int(gold[3])
    out = oracle_decompress(gold, nbytes)
    assert isinstance(out, np.ndarray)
    # The 1.17/1.18 bitshuffle files hold the first 641 09x bytes of the ramp.  Their last block is
    # a format-version-2 bitshuffle whose trailing nbytes % ts bytes the reference never writes
    # (blosc/shuffle.c:489-500 un-bitshuffles n elements and copies no tail; the caller's buffer
    # keeps its old bytes there): only whole elements are compared.
    whole = nbytes - nbytes % ts if gold[0] == 2 and gold[2] & 4 else nbytes
    assert np.array_equal(out[:whole], RAMP.view(np.uint8)[:whole])


def test_lz4_chunk_kat():
    """compat/blosc-lz4-3.0.0.cdata == blosc1_compress(9, SHUFFLE, 4, ramp) with LZ4, 1 thread
    (compat/filegen.c:91): the oracle re-encodes it byte-identically."""
    gold = np.fromfile(os.path.join(GOLD, "blosc-lz4-3.0.0.cdata"), np.uint8)
    got = oracle_compress(RAMP, clevel=9, typesize=4, compcode=1, splitmode=4)
    assert isinstance(got, np.ndarray) and np.array_equal(got, gold)
