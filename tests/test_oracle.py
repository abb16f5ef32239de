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
