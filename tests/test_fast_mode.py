"""BloscLZ fast mode (c-blosc2_amd/csrc/b2h_lzfast.h; model tools/fm_model.c).

North star contract for the codec: output round-trip-identical through the reference's decoder
(blosclz_decompress, blosc/blosclz.c:685-795) with the ratio matching.  Fast mode keeps the
reference's grammar, greedy rule, limits, entropy-probe decision and emission and changes only
which earlier position the hash table offers as a candidate (tile-ordered inserts, independent of
the parse).  Checked here:
  CPU:  the model's streams decode with the oracle's blosclz_decompress restatement (and the
        reference build when present) for every clevel on mixed data; on T-shaped data (shuffled
        gen_f32 planes) its raw/compress decisions equal the exact probe's and its ratio is within
        0.1 % of exact mode's (2^13 table) -- tolerance stated in the test;
  GPU:  every LZ stream the kernel emits is byte-identical to the model's for the same filtered
        stream (the kernel's LDS exchange applies lanes in order, as the model assumes); whole
        chunks round-trip through the oracle decoder, the reference build and the device decoder;
        T's chunk ratio in fast mode is >= exact mode's x 0.999.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

from b2ctypes import REPO
from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import oracle, oracle_compress, oracle_decompress, p, ref

sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
FM_SO = os.path.join(REPO, "oracle", "libfm_model.so")
TABLOG = 13   # the kernel's default (B2H_FAST_TABLOG)


def fm():
    if not os.path.exists(FM_SO):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"])
    L = C.CDLL(FM_SO)
    L.fm_blosclz_compress.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_int, C.c_int]
    L.fm_probe_ratio.argtypes = [C.c_int, C.c_void_p, C.c_int, C.c_int]
    L.fm_probe_ratio.restype = C.c_double
    L.fm_set_depth.argtypes = [C.c_int]
    L.fm_set_noskip.argtypes = [C.c_int]
    return L


def fm_compress(stream, clevel, maxout=None, tablog=TABLOG, depth=1, noskip=False):
    """The model's stream; depth 8 = the engine's BloscLZ mode 2 (deep candidates); noskip = mode 3
    (every position inserted in order: the serial parse the segmented walk reproduces)."""
    n = stream.nbytes
    out = np.zeros(n + 64, np.uint8)
    L = fm()
    L.fm_set_depth(depth)
    L.fm_set_noskip(1 if noskip else 0)
    try:
        m = L.fm_blosclz_compress(clevel, p(stream), n, p(out), n if maxout is None else maxout, tablog)
    finally:
        L.fm_set_depth(1)
        L.fm_set_noskip(0)
    return out[:m] if m > 0 else None


def shuffled_planes(raw, ts=4, bs=262144):
    """The 64 KiB streams of T's chunks: each 256 KiB block byte-shuffled, split in ts planes."""
    O = oracle()
    out = []
    for b in range(raw.nbytes // bs):
        blk = np.ascontiguousarray(raw[b * bs:(b + 1) * bs])
        sh = np.empty_like(blk)
        O.or_shuffle(ts, bs, p(blk), p(sh))
        out += [np.ascontiguousarray(sh[j * (bs // ts):(j + 1) * (bs // ts)]) for j in range(ts)]
    return out


# ----------------------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("clevel", range(1, 10))
def test_model_streams_decode_with_reference_decoder(clevel):
    O = oracle()
    rng = np.random.default_rng(clevel)
    for k in range(6):
        n = int(rng.integers(100, 300_000))
        src = mixed_bytes(int(rng.integers(0, 1 << 30)), n)
        for tl in (12, 13, 14):
            z = fm_compress(src, clevel, tablog=tl)
            if z is None:
                continue
            dec = np.zeros(n, np.uint8)
            assert O.or_blosclz_decompress(p(z), z.nbytes, p(dec), n) == n, (clevel, k, tl)
            assert np.array_equal(dec, src), (clevel, k, tl)
            assert z[0] >> 5 == 1                      # the blosclz marker bit (blosclz.c:613)


def test_model_matches_exact_decisions_and_ratio_on_T():
    """Shuffled gen_f32 planes (4 chunks of 4 MiB = 256 streams): same raw/compress decisions as
    the exact probe; total ratio within 0.1 % of exact mode (tolerance of the 2^13 table)."""
    O = oracle()
    raw = gen_f32(0, 4 << 20).view(np.uint8)
    ex = fa = 0
    for s in shuffled_planes(raw):
        out = np.zeros(s.nbytes + 64, np.uint8)
        n = O.or_blosclz_compress(5, p(s), s.nbytes, p(out), s.nbytes)
        z = fm_compress(s, 5)
        assert (n > 0) == (z is not None)
        ex += (n if n > 0 else s.nbytes) + 4
        fa += (z.nbytes if z is not None else s.nbytes) + 4
    assert fa <= ex * 1.001, (ex, fa)


def test_model_ratio_on_C1_known_gap():
    """C1 (b2bench int32 get_value(i, 19)): fast mode's most-recent-position candidates find
    shorter matches than the reference's table on these long-period patterns (ratio 12.2 vs 20.6,
    DESIGN.md §5) -- a documented gap of the opt-in mode, pinned here so that it cannot widen
    unnoticed; every stream still decodes with the reference decoder."""
    from datagen import b2bench_values
    O = oracle()
    raw = b2bench_values(1 << 18, 19).view(np.uint8)   # 1 MiB of C1's data
    ex = fa = 0
    for s in shuffled_planes(raw):
        out = np.zeros(s.nbytes + 64, np.uint8)
        n = O.or_blosclz_compress(5, p(s), s.nbytes, p(out), s.nbytes)
        z = fm_compress(s, 5)
        ex += (n if n > 0 else s.nbytes) + 4
        fa += (z.nbytes if z is not None else s.nbytes) + 4
        if z is not None:
            back = np.zeros(s.nbytes, np.uint8)
            assert O.or_blosclz_decompress(p(z), z.nbytes, p(back), s.nbytes) == s.nbytes
            assert np.array_equal(back, s)
    assert fa <= ex * 1.75, (raw.nbytes / ex, raw.nbytes / fa)


def _exact_size(s, clevel=5):
    out = np.zeros(s.nbytes + 64, np.uint8)
    n = oracle().or_blosclz_compress(clevel, p(s), s.nbytes, p(out), s.nbytes)
    return (n if n > 0 else s.nbytes) + 4


def _bitshuffled_blocks(raw, ts=4, bs=262144):
    O = oracle()
    out = []
    for b in range(raw.nbytes // bs):
        blk = np.ascontiguousarray(raw[b * bs:(b + 1) * bs])
        sh = np.empty_like(blk)
        O.or_bitshuffle(ts, bs, p(blk), p(sh))
        out.append(sh)
    return out


@pytest.mark.parametrize("data", ["C1", "T", "C3", "mixed"])
def test_model_deep_candidates_ratio(data):
    """BloscLZ mode 2 (deep candidates, depth 8): the ratio gap of plain fast mode closes -- on C1's
    data (b2bench get_value(i, 19), where depth 1 loses 40 %), T's shuffled planes, C3's bitshuffled
    256 KiB streams and mixed bytes the model's total size is <= exact mode's / 0.99 (measured:
    C1 -1.4 %, T -2.0 %, C3 -3.4 %, mixed -13 %, i.e. smaller than the reference's); every stream
    decodes with the reference decoder's restatement."""
    from datagen import b2bench_values
    O = oracle()
    if data == "C1":
        streams = shuffled_planes(b2bench_values(1 << 19, 19).view(np.uint8))
    elif data == "T":
        streams = shuffled_planes(gen_f32(0, 2 << 20).view(np.uint8))
    elif data == "C3":
        streams = _bitshuffled_blocks(gen_f32(0, 1 << 20).view(np.uint8))
    else:
        streams = [mixed_bytes(s, 65536) for s in range(8)]
    ex = fa = 0
    for s in streams:
        z = fm_compress(s, 5, depth=8)
        ex += _exact_size(s)
        fa += (z.nbytes if z is not None else s.nbytes) + 4
        if z is not None:
            back = np.zeros(s.nbytes, np.uint8)
            assert O.or_blosclz_decompress(p(z), z.nbytes, p(back), s.nbytes) == s.nbytes
            assert np.array_equal(back, s)
    assert fa * 0.99 <= ex, (data, ex, fa)


@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_model_deep_streams_decode(clevel):
    O = oracle()
    rng = np.random.default_rng(50 + clevel)
    for k in range(4):
        n = int(rng.integers(100, 200_000))
        src = mixed_bytes(int(rng.integers(0, 1 << 30)), n)
        z = fm_compress(src, clevel, depth=8)
        if z is None:
            continue
        dec = np.zeros(n, np.uint8)
        assert O.or_blosclz_decompress(p(z), z.nbytes, p(dec), n) == n
        assert np.array_equal(dec, src)


def test_model_reference_build_decodes():
    R = ref()
    if R is None:
        pytest.skip("reference build absent")
    # a whole chunk assembled from model streams is checked on the GPU tier; here one stream
    # through the reference's own blosclz_decompress symbol
    if not hasattr(R, "blosclz_decompress"):
        pytest.skip("blosclz_decompress not exported by the reference build")
    R.blosclz_decompress.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int]
    src = mixed_bytes(77, 200_000)
    z = fm_compress(src, 9)
    dec = np.zeros(src.nbytes, np.uint8)
    assert R.blosclz_decompress(p(z), z.nbytes, p(dec), src.nbytes) == src.nbytes
    assert np.array_equal(dec, src)


# ----------------------------------------------------------------------------- GPU ----
def _streams_of_chunk(chunk):
    """(neblock, csize, payload) of every stream of an extended-header chunk (chunk format:
    README_CHUNK_FORMAT.rst -- header, bstarts, per stream an int32 csize + payload)."""
    h = chunk[:32]
    ts = int(h[3])
    nbytes, bs = (int(x) for x in np.frombuffer(h[4:12].tobytes(), np.int32))
    dont_split = (h[2] >> 4) & 1
    nblocks = -(-nbytes // bs)
    bstarts = np.frombuffer(chunk[32:32 + 4 * nblocks].tobytes(), np.int32)
    out = []
    for b in range(nblocks):
        bsize = min(bs, nbytes - b * bs)
        ns = ts if (not dont_split and bsize == bs) else 1
        pos = int(bstarts[b])
        for _ in range(ns):
            cs = int(np.frombuffer(chunk[pos:pos + 4].tobytes(), np.int32)[0])
            pos += 4
            pl = chunk[pos:pos + cs] if cs > 0 else chunk[pos:pos + (1 if cs < 0 else 0)]
            out.append((bsize // ns, cs, pl))
            pos += cs if cs > 0 else (1 if cs < 0 else 0)
    return out


def _filtered_streams(src, ts, bs, filt, split):
    O = oracle()
    raw = src.view(np.uint8).reshape(-1)
    out = []
    for b in range(-(-raw.nbytes // bs)):
        blk = np.ascontiguousarray(raw[b * bs:(b + 1) * bs])
        f = np.empty_like(blk)
        if filt == 1:
            O.or_shuffle(ts, blk.nbytes, p(blk), p(f))
        elif filt == 2:
            O.or_bitshuffle(ts, blk.nbytes, p(blk), p(f))
        else:
            f[:] = blk
        ns = ts if (split and blk.nbytes == bs) else 1
        nb = blk.nbytes // ns
        out += [np.ascontiguousarray(f[j * nb:(j + 1) * nb]) for j in range(ns)]
    return out


@pytest.fixture(scope="module")
def fast():
    """The engine; every fast-mode call below selects the encoder per context through
    cparams.codec_params (include/b2h.h b2h_codec_params), never through the process default."""
    import torch  # noqa: F401
    import blosc2_amd as B
    L = B.lib()
    default = L.b2h_set_blosclz_mode(-1)   # query only
    yield B
    assert L.b2h_set_blosclz_mode(-1) == default   # no test changed the process default


CASES = [
    ("gen_f32 T chunk", lambda: gen_f32(0, 1 << 20), dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1))),
    ("gen_f32 clevel 9", lambda: gen_f32(5, 1 << 18), dict(clevel=9, typesize=4, filters=(0, 0, 0, 0, 0, 1))),
    ("gen_f32 clevel 1", lambda: gen_f32(9, 1 << 18), dict(clevel=1, typesize=4, filters=(0, 0, 0, 0, 0, 1))),
    ("C3 bitshuffle 256K stream", lambda: gen_f32(1 << 16, 1 << 16),
     dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 2), blocksize=262144)),
    ("mixed bytes noshuffle", lambda: mixed_bytes(4, 700_000), dict(clevel=7, typesize=1, filters=(0,) * 6)),
    ("int64 ramp shuffle", lambda: int64_ramp(3, 1 << 17), dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 0, 1))),
]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [1, 2, 3], ids=["fast", "deep", "seg"])
@pytest.mark.parametrize("name,mk,kw", CASES, ids=[c[0] for c in CASES])
def test_gpu_fast_streams_match_model(fast, name, mk, kw, mode):
    """Every LZ stream the kernel writes equals the model's (mode 2: the model at depth 8; mode 3:
    the model with every position inserted in order, fm_set_noskip)."""
    B = fast
    src = mk()
    raw = src.view(np.uint8).reshape(-1)
    cp = B.cparams(**kw, lz_mode=mode)
    L = B.lib()
    ctx = L.blosc2_create_cctx(cp)
    got = B.compress_ctx(ctx, src, destsize=2 * raw.nbytes + 64)   # ample: maxout = neblock everywhere
    L.blosc2_free_ctx(ctx)
    assert isinstance(got, np.ndarray), got
    bs = int(np.frombuffer(got[8:12].tobytes(), np.int32)[0])
    split = not ((got[2] >> 4) & 1)
    streams = _streams_of_chunk(got)
    filt = _filtered_streams(src, kw["typesize"], bs, kw["filters"][5], split)
    assert len(streams) == len(filt)
    n_lz = 0
    for k, ((nb, cs, pl), s) in enumerate(zip(streams, filt)):
        assert nb == s.nbytes
        model = fm_compress(s, kw["clevel"], depth=8 if mode == 2 else 1, noskip=mode == 3)
        if 0 < cs < nb:
            n_lz += 1
            assert model is not None and np.array_equal(pl, model), (name, k, cs)
        elif cs == nb:
            assert model is None or model.nbytes >= nb, (name, k)
    assert n_lz > 0 or name.startswith("int64")
    # the chunk decodes with the oracle, the reference build and the device
    assert np.array_equal(oracle_decompress(got, raw.nbytes), raw)
    R = ref()
    if R is not None:
        from b2ctypes import dparams as rdp
        dctx = R.blosc2_create_dctx(rdp())
        dec = np.zeros(raw.nbytes, np.uint8)
        assert R.blosc2_decompress_ctx(dctx, p(got), got.nbytes, p(dec), raw.nbytes) == raw.nbytes
        R.blosc2_free_ctx(dctx)
        assert np.array_equal(dec, raw)
    assert np.array_equal(B.decompress(got, raw.nbytes), raw)


@pytest.mark.gpu
@pytest.mark.parametrize("lzmode", [1, 3], ids=["fast", "seg"])
@pytest.mark.parametrize("seed", range(4))
def test_gpu_fast_random_chunks_roundtrip(fast, seed, lzmode):
    """Random pipelines / sizes / clevels (the exact-mode grid of test_gpu_parity) in fast mode:
    round trip through the oracle decoder and the device; tight destsize keeps the serial
    maxout rule working (0 / memcpy fallbacks, never an overrun)."""
    from test_gpu_parity import _cases
    B = fast
    for src, kw in _cases(100 + seed, 10):
        raw = src.view(np.uint8).reshape(-1)
        got = B.compress(src, **kw, lz_mode=lzmode)
        assert isinstance(got, np.ndarray), kw
        lossless = kw["filters"][4] != 4
        dec = oracle_decompress(got, raw.nbytes)
        assert isinstance(dec, np.ndarray), kw
        if lossless:
            assert np.array_equal(dec, raw), kw
        assert np.array_equal(B.decompress(got, raw.nbytes), dec), kw
        # ratio is judged on the configurations (T / C3 below and in bench.py); on arbitrary data
        # the smaller table may find fewer far matches -- bounded here only as a sanity check
        ex = oracle_compress(src, **kw)
        assert got.nbytes <= ex.nbytes * 1.10 + 64, (kw, got.nbytes, ex.nbytes)


@pytest.mark.gpu
def test_gpu_fast_ratio_T(fast):
    """T's shape (float32 ts=4 SHUFFLE clevel 5, 4 MiB chunks), 16 chunks on the device batch path:
    fast-mode cratio >= exact-mode cratio x 0.999 and an exact round trip."""
    import torch
    B = fast
    L = B.lib()
    dev = torch.device("cuda")
    chunk, n = 4 << 20, 16
    src = torch.from_numpy(gen_f32(0, n * chunk // 4).view(np.uint8)).to(dev)
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    sizes = {}
    for mode in (0, 1, 3):
        cp = B.cparams(clevel=5, typesize=4, lz_mode=mode)
        comp = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        cb = torch.zeros(n, dtype=torch.int32, device=dev)
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
        out = torch.zeros_like(src)
        st = torch.zeros(n, dtype=torch.int32, device=dev)
        B.decompress_batch(comp.data_ptr(), stride, cb.data_ptr(), n, out.data_ptr(), chunk, chunk, st.data_ptr(), 0)
        torch.cuda.synchronize()
        assert torch.equal(out, src) and bool((st == chunk).all())
        sizes[mode] = int(cb.to(torch.int64).sum())
    assert sizes[1] <= sizes[0] * 1.001, sizes
    assert sizes[3] <= sizes[0] * 1.001, sizes


@pytest.mark.gpu
@pytest.mark.parametrize("data", ["C1", "T", "C3"])
def test_gpu_deep_mode_ratio(fast, data):
    """BloscLZ mode 2 on the device: chunk ratio >= exact mode's x 0.99 on C1's data (b2bench
    get_value(i, 19), 4 MiB, ts 4 SHUFFLE), T's (gen_f32 4 MiB) and C3's (BITSHUFFLE, 256 KiB
    blocks); every chunk decodes with the oracle and the device."""
    from datagen import b2bench_values
    B = fast
    if data == "C1":
        src, kw = b2bench_values(1 << 20, 19), dict(clevel=5, typesize=4)
    elif data == "T":
        src, kw = gen_f32(0, 1 << 20), dict(clevel=5, typesize=4)
    else:
        src, kw = gen_f32(1 << 16, 1 << 20), dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 2), blocksize=262144)
    raw = src.view(np.uint8).reshape(-1)
    deep = B.compress(src, **kw, lz_mode=B.DEEP)
    ex = oracle_compress(src, **kw)
    assert isinstance(deep, np.ndarray) and isinstance(ex, np.ndarray)
    assert deep.nbytes * 0.99 <= ex.nbytes, (data, raw.nbytes / ex.nbytes, raw.nbytes / deep.nbytes)
    assert np.array_equal(oracle_decompress(deep, raw.nbytes), raw)
    assert np.array_equal(np.asarray(B.decompress(deep, raw.nbytes)).view(np.uint8).reshape(-1), raw)


@pytest.mark.gpu
@pytest.mark.parametrize("lzmode", [1, 2, 0, 3], ids=["fast", "deep", "exact", "seg"])
@pytest.mark.parametrize("shape", ["T", "ts4_runplanes", "leftover", "clevel9_ts8", "ds8", "ds8_ramp", "ds2_leftover",
                                   "ds4_odd_leftover"])
def test_gpu_fused_launch_matches_separate_launches(fast, shape, lzmode, monkeypatch):
    """The one-launch fast-mode encode (byte shuffle, finalize and payload scatter inside the
    encoder launch, k_encode_fast_fused) writes the same chunks as the separate launches
    (B2H_FUSE=0; 83 is the default, 3 also claims scatter items between streams), in both BloscLZ
    modes (exact: k_encode_fused, per-wave hand-offs; its chunks also equal the oracle's; mode 3:
    k_encode_seg_fused, the same per-wave protocol), on T's shape (4 MiB chunks: fused shuffle) and on shapes where only the
    finalize/scatter is fused (a leftover block not of whole 64-byte groups, typesize 8)."""
    import torch
    B = fast
    dev = torch.device("cuda")
    if shape == "T":
        chunk, n, kw = 4 << 20, 24, dict(clevel=5, typesize=4)
    elif shape == "ts4_runplanes":   # the SHUFFLE job's run verdict (b2h_engine.hip shuffle4_block_runs)
        chunk, n, kw = 1 << 20, 12, dict(clevel=5, typesize=4)
    elif shape == "leftover":
        chunk, n, kw = (1 << 20) + 4 * 37, 12, dict(clevel=5, typesize=4, blocksize=1 << 18)
    elif shape == "clevel9_ts8":
        chunk, n, kw = 1 << 20, 12, dict(clevel=9, typesize=8)
    elif shape == "ds8":   # C4's pipeline: (DELTA, SHUFFLE) filtered inside the encoder launch
        chunk, n, kw = 1 << 20, 12, dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))
    elif shape == "ds8_ramp":   # C4 exactly: the blocks after the first are runs in every plane
        chunk, n, kw = 1 << 20, 12, dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))
    elif shape == "ds2_leftover":   # a leftover block of whole 64-byte groups: still fused
        chunk, n, kw = (1 << 20) + 64 * 3, 12, dict(clevel=5, typesize=2, filters=(0, 0, 0, 0, 3, 1), blocksize=1 << 18)
    else:   # leftover not of whole 64-byte groups: the separate k_ffilter_ds launch
        chunk, n, kw = (1 << 20) + 4 * 37, 12, dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 3, 1), blocksize=1 << 18)
    if shape == "ts4_runplanes":
        # planes 2 and 3 runs of 0x0B / 0x0A, planes 0 and 1 noise; in every third 256 KiB block
        # one byte of plane 2 differs (one block near its end, the others anywhere)
        rng = np.random.default_rng(13)
        v = rng.integers(0, 1 << 16, n * chunk // 4, dtype=np.uint32) | np.uint32(0x0A0B0000)
        per = (1 << 18) // 4
        for b in range(0, n * chunk // (1 << 18), 3):
            e = b * per + (per - 1 if b % 2 else int(rng.integers(0, per)))
            v[e] ^= np.uint32(0x00010000)
        src = torch.from_numpy(v.view(np.uint8).copy()).to(dev)
    elif shape == "ds8_ramp":
        src = torch.from_numpy(int64_ramp(7, n * chunk // 8).view(np.uint8).copy()).to(dev)
    elif shape.startswith("ds"):
        rng = np.random.default_rng(11)   # a ramp with jitter: run, raw and LZ streams after the filters
        ramp = int64_ramp(7, n * chunk // 8 + 1) * 3 + rng.integers(0, 8, n * chunk // 8 + 1)
        src = torch.from_numpy(ramp.view(np.uint8)[:n * chunk].copy()).to(dev)
    else:
        src = torch.from_numpy(gen_f32(3, n * chunk // 4).view(np.uint8)).to(dev)
    cap = chunk + 64
    stride = (cap + 255) // 256 * 256
    cp = B.cparams(**kw, lz_mode=lzmode)
    got = {}
    for fuse in ("83", "3", "0"):
        # exact mode fuses only with bit 4 (k_encode_fused), mode 3 only with bit 8 (k_encode_seg_fused)
        monkeypatch.setenv("B2H_FUSE", fuse if lzmode in (1, 2) or fuse == "0" else str(int(fuse) | (4 if lzmode == 0 else 8)))
        comp = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        cb = torch.zeros(n, dtype=torch.int32, device=dev)
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        cbh = cb.cpu().numpy()
        assert (cbh > 0).all(), cbh
        compb = comp.cpu().numpy().reshape(n, stride)
        got[fuse] = [compb[i, :cbh[i]].copy() for i in range(n)]
    if shape.startswith("ds") and lzmode in (1, 2):
        # the (DELTA, SHUFFLE) jobs run by their own launch ahead of the encoder (B2H_DS_PREPASS)
        monkeypatch.setenv("B2H_FUSE", "83")
        monkeypatch.setenv("B2H_DS_PREPASS", "1")
        comp = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
        cb = torch.zeros(n, dtype=torch.int32, device=dev)
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        monkeypatch.delenv("B2H_DS_PREPASS")
        cbh = cb.cpu().numpy()
        compb = comp.cpu().numpy().reshape(n, stride)
        got["pre"] = [compb[i, :cbh[i]].copy() for i in range(n)]
    for fz in [k for k in got if k != "0"]:
        for a, b in zip(got[fz], got["0"]):
            assert np.array_equal(a, b), fz
    raw = src.cpu().numpy()
    for i in range(0, n, 5):
        assert np.array_equal(oracle_decompress(got["83"][i], chunk), raw[i * chunk:(i + 1) * chunk])
        if lzmode == 0:   # exact mode: the reference's own chunk
            ex = oracle_compress(raw[i * chunk:(i + 1) * chunk], **kw)
            assert np.array_equal(got["83"][i], ex)


@pytest.mark.gpu
def test_gpu_blosclz_mode_per_context_on_threads(fast):
    """VERDICT r2 boundary item: the BloscLZ encoder is a property of the context
    (cparams.codec_params -> b2h_codec_params), not a process switch.  Two host threads compress
    the same T-shaped chunks concurrently, one through a fast-mode context and one through an
    exact-mode context: each gets its own mode's bytes every time (exact = the reference's chunk,
    fast = the fast encoder's chunk of a lone call), and the process default never changes."""
    import threading
    B = fast
    L = B.lib()
    src = gen_f32(17, 1 << 20)
    want = {B.EXACT: oracle_compress(src, clevel=5, typesize=4)}
    want[B.FAST] = B.compress(src, clevel=5, typesize=4, lz_mode=B.FAST)
    assert not np.array_equal(want[B.FAST], want[B.EXACT])   # T data: the two encoders differ
    default = L.b2h_set_blosclz_mode(-1)
    errs = []

    def run(mode):
        try:
            ctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=4, lz_mode=mode))
            for _ in range(6):
                got = B.compress_ctx(ctx, src)
                if not np.array_equal(got, want[mode]):
                    errs.append(mode)
            L.blosc2_free_ctx(ctx)
        except Exception as e:  # pragma: no cover - reported below
            errs.append(repr(e))

    th = [threading.Thread(target=run, args=(m,)) for m in (B.FAST, B.EXACT, B.FAST, B.EXACT)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs
    assert L.b2h_set_blosclz_mode(-1) == default
    # a context without codec_params follows the process default
    plain = B.compress(src, clevel=5, typesize=4)
    assert np.array_equal(plain, want[B.FAST] if default == 1 else want[B.EXACT])


@pytest.mark.gpu
@pytest.mark.parametrize("lzmode", [1, 0], ids=["fast", "exact"])
def test_gpu_fused_small_grid_has_no_timeouts(fast, lzmode, monkeypatch):
    """VERDICT r2 hardening: the fused launch with its persistent grid capped at 1, 2 and 5
    workgroups (B2H_FUSE_GRID) -- a lone workgroup then runs every shuffle job, stream, chunk
    finalisation and scatter item, so every hand-off wait has to be met by itself or a peer --
    writes the separate launches' chunks.  A timed-out wait (sync[4]) would turn every chunk of the
    batch into E_FAILURE, which the cbytes check catches."""
    import torch
    B = fast
    chunk, n = 4 << 20, 6
    src = torch.from_numpy(gen_f32(21, n * chunk // 4).view(np.uint8)).cuda()
    cap = chunk + 64
    stride = (cap + 255) // 256 * 256
    cp = B.cparams(clevel=5, typesize=4, lz_mode=lzmode)

    def run():
        comp = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        cb = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        cbh = cb.cpu().numpy()
        assert (cbh > 0).all(), cbh
        compb = comp.cpu().numpy().reshape(n, stride)
        return [compb[i, :cbh[i]].copy() for i in range(n)]
    monkeypatch.setenv("B2H_FUSE", "0")
    want = run()
    monkeypatch.setenv("B2H_FUSE", "83" if lzmode == 1 else "87")
    for grid in ("1", "2", "5"):
        monkeypatch.setenv("B2H_FUSE_GRID", grid)
        got = run()
        assert all(np.array_equal(a, b) for a, b in zip(got, want)), grid


@pytest.mark.gpu
def test_gpu_fused_launches_on_two_streams_at_once(fast):
    """Two super-chunks on two host threads append device batches at the same time: two fused
    launches, each sized for the whole chip, on two contexts' own streams and workspaces, compete
    for the CUs (part of one launch's grid may wait for the other to leave).  Every chunk equals a
    lone call's chunk, and no batch reports a failed hand-off wait."""
    import threading
    import torch
    B = fast
    chunk, n = 4 << 20, 16
    L = B.lib()
    host = [gen_f32(s, n * chunk // 4).view(np.uint8) for s in (31, 32)]
    dev = [torch.from_numpy(h).cuda() for h in host]
    want = [[B.compress(h[i * chunk:(i + 1) * chunk], clevel=5, typesize=4, lz_mode=B.FAST) for i in range(n)]
            for h in host]
    errs = []

    def run(k):
        try:
            for _ in range(3):
                sc = B.SChunk(B.cparams(clevel=5, typesize=4, lz_mode=B.FAST), B.dparams())
                sizes = (C.c_int32 * n)(*([chunk] * n))
                r = L.b2h_schunk_append_device(sc.p, C.c_void_p(dev[k].data_ptr()), sizes, n, chunk)
                if r != n:
                    errs.append((k, "append", r))
                for i in range(n):
                    if not np.array_equal(sc.chunk(i), want[k][i]):
                        errs.append((k, i))
                sc.free()
        except Exception as e:   # noqa: BLE001 -- reported to the main thread
            errs.append((k, repr(e)))
    th = [threading.Thread(target=run, args=(k,)) for k in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not any(t.is_alive() for t in th)
    assert not errs, errs


@pytest.mark.gpu
@pytest.mark.parametrize("lzmode", [1, 0], ids=["fast", "exact"])
def test_gpu_fused_timeout_falls_back_to_separate_launches(fast, lzmode, monkeypatch):
    """ADVICE r2 / VERDICT r4 item 8: a fused launch whose hand-off wait times out (simulated:
    B2H_FUSE_SIMULATE_TIMEOUT starts it with the timeout flag set) no longer fails its batch: the
    separate launches queued behind it, gated on its timeout word, redo the batch on the stream
    (the asynchronous batch API), and blosc2_compress_ctx returns the normal chunk too."""
    import torch
    B = fast
    L = B.lib()
    src = gen_f32(23, 1 << 20)
    monkeypatch.setenv("B2H_FUSE", "83" if lzmode == 1 else "87")
    want = B.compress(src, clevel=5, typesize=4, lz_mode=lzmode)
    monkeypatch.setenv("B2H_FUSE_SIMULATE_TIMEOUT", "1")
    ctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=4, lz_mode=lzmode))
    try:
        got = B.compress_ctx(ctx, src)
    finally:
        L.blosc2_free_ctx(ctx)
    assert np.array_equal(got, want)
    assert np.array_equal(oracle_decompress(got, src.nbytes), src.view(np.uint8))
    chunk, n = 4 << 20, 3
    dsrc = torch.from_numpy(gen_f32(29, n * chunk // 4).view(np.uint8)).cuda()
    stride = chunk + 256
    out = {}
    for sim in ("1", None):
        if sim:
            monkeypatch.setenv("B2H_FUSE_SIMULATE_TIMEOUT", sim)
        else:
            monkeypatch.delenv("B2H_FUSE_SIMULATE_TIMEOUT")
        comp = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        cb = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.compress_batch(B.cparams(clevel=5, typesize=4, lz_mode=lzmode), dsrc.data_ptr(), chunk, n, chunk,
                         comp.data_ptr(), stride, chunk + 64, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        assert L.b2h_debug_fuse_timed_out() == (1 if sim else 0)
        cbh = cb.cpu().numpy()
        assert (cbh > 0).all(), cbh   # the rescue launches redid the batch
        cm = comp.cpu().numpy().reshape(n, stride)
        out[sim] = [cm[i, :cbh[i]].copy() for i in range(n)]
    for a, b in zip(out["1"], out[None]):
        assert np.array_equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [1, 2, 5])
@pytest.mark.parametrize("kind", ["runs", "raw", "zeros"])
@pytest.mark.parametrize("lzmode", [1, 2], ids=["fast", "deep"])
def test_gpu_fused_uniform_stream_batches(fast, lzmode, kind, grid, monkeypatch):
    """the shape that exposed round 4's non-uniform barrier loops (DESIGN §3,
    "Barrier loops must be structurized as uniform") -- batches whose streams are ALL runs, all raw
    (incompressible) or all zero runs, through k_encode_fast_fused with a persistent grid of 1, 2
    or 5 workgroups (B2H_FUSE_GRID: a few workgroups do every shuffle job, stream, finalisation and
    scatter item).  The launch must not time out, and its chunks equal the separate launches'."""
    import torch
    B = fast
    L = B.lib()
    chunk, n = 1 << 20, 6
    if kind == "runs":
        host = np.repeat(np.arange(1, n * chunk // 262144 + 1, dtype=np.uint8), 262144)   # every plane a run
    elif kind == "raw":
        host = np.random.default_rng(5).integers(0, 256, n * chunk, dtype=np.uint8)
    else:
        host = np.zeros(n * chunk, np.uint8)
    src = torch.from_numpy(host).cuda()
    stride = chunk + 256
    cp = B.cparams(clevel=5, typesize=4, lz_mode=lzmode)
    out = {}
    for fuse in ("83", "0"):
        monkeypatch.setenv("B2H_FUSE", fuse)
        monkeypatch.setenv("B2H_FUSE_GRID", str(grid))
        comp = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        cb = torch.zeros(n, dtype=torch.int32, device="cuda")
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, chunk + 64, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        if fuse == "83":
            assert L.b2h_debug_fuse_timed_out() == 0, "fused launch timed out"
        cbh = cb.cpu().numpy()
        assert (cbh > 0).all(), cbh
        cm = comp.cpu().numpy().reshape(n, stride)
        out[fuse] = [cm[i, :cbh[i]].copy() for i in range(n)]
    for i, (a, b) in enumerate(zip(out["83"], out["0"])):
        assert np.array_equal(a, b), i
    assert np.array_equal(B.decompress(np.concatenate([out["83"][0]]), chunk), host[:chunk])


@pytest.mark.parametrize("data", ["T", "C3", "C1", "C4"])
def test_model_noskip_ratio_and_decode(data):
    """BloscLZ mode 3's semantics (every position inserted in order, fm_set_noskip) against exact
    mode's stream bytes: T <= 1.001 x exact (measured 1.0004), C3 <= 1.0025 x (1.0019), C1 / C4 as
    the ratio-pinning tests above allow; every stream decodes with the reference decoder's
    restatement."""
    from datagen import b2bench_values
    O = oracle()
    if data == "T":
        streams, cap = shuffled_planes(gen_f32(0, 2 << 20).view(np.uint8)), 1.001
    elif data == "C3":
        streams, cap = _bitshuffled_blocks(gen_f32(77, 1 << 20).view(np.uint8)), 1.0025
    elif data == "C1":
        streams, cap = shuffled_planes(b2bench_values(1 << 19, 19).view(np.uint8)), 1.75
    else:
        raw = int64_ramp(0, 1 << 17).view(np.uint8)
        streams, cap = shuffled_planes(raw, ts=8), 1.01
    ex = fa = 0
    for s in streams:
        z = fm_compress(s, 5, noskip=True)
        ex += _exact_size(s)
        fa += (z.nbytes if z is not None else s.nbytes) + 4
        if z is not None:
            back = np.zeros(s.nbytes, np.uint8)
            assert O.or_blosclz_decompress(p(z), z.nbytes, p(back), s.nbytes) == s.nbytes
            assert np.array_equal(back, s)
    assert fa <= ex * cap, (data, ex, fa, fa / ex)
