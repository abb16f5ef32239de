"""GPU tier: the HIP path (through the drop-in C ABI and the device batch ABI) against the oracle
restatement, the reference library built from its sources (oracle/_ref, when present) and the
reference's own golden vectors.  Bar: byte-identical chunks, exact round trips."""
import ctypes as C
import hashlib
import json
import os
import sys

import numpy as np
import pytest

from b2ctypes import REPO
from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import oracle, oracle_compress, oracle_decompress, p, ref, ref_compress

sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))

pytestmark = pytest.mark.gpu
GOLD = os.path.join(REPO, "tests", "golden")
RAMP = np.arange(1_000_000, dtype=np.int32)


@pytest.fixture(scope="module")
def B():
    import torch  # noqa: F401  (same HIP runtime as bench.py: torch first, then the engine)
    import blosc2_amd
    L = blosc2_amd.lib()
    assert L.b2h_device_count() > 0
    return blosc2_amd


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_shuffle_kats(B):
    L = B.lib()
    out = np.zeros(RAMP.nbytes, np.uint8)
    assert L.blosc2_shuffle(4, RAMP.nbytes, B._p(RAMP), B._p(out)) == RAMP.nbytes
    assert sha(out) == "40e1351bba9155c3d765d66b5b4d25cb104aa2ad4b844b0a5d20af40cab2b920"
    back = np.zeros_like(out)
    L.blosc2_unshuffle(4, RAMP.nbytes, B._p(out), B._p(back))
    assert np.array_equal(back.view(np.int32), RAMP)
    L.blosc2_bitshuffle(4, RAMP.nbytes, B._p(RAMP), B._p(out))
    assert sha(out) == "a1bba6ced356ddca157010f340b8b5a39a5cd43a77b7c99cd1cb8896e853169d"
    L.blosc2_bitunshuffle(4, RAMP.nbytes, B._p(out), B._p(back))
    assert np.array_equal(back.view(np.int32), RAMP)


@pytest.mark.parametrize("ts", [1, 2, 3, 4, 7, 8, 16, 17, 80])
@pytest.mark.parametrize("nelem", [7, 192, 500, 1792, 8000, 100000])
def test_shuffle_grid_vs_oracle(B, ts, nelem):
    """test_shuffle_roundtrip_*.csv grid: GPU vs oracle, byte-exact, both directions."""
    L, O = B.lib(), oracle()
    src = np.random.default_rng(ts * 7 + nelem).integers(0, 256, ts * nelem + 3, dtype=np.uint8)
    n = src.nbytes
    g, o = np.zeros(n, np.uint8), np.zeros(n, np.uint8)
    for fg, fo in (("blosc2_shuffle", "or_shuffle"), ("blosc2_unshuffle", "or_unshuffle"),
                   ("blosc2_bitshuffle", "or_bitshuffle")):
        getattr(L, fg)(ts, n, B._p(src), B._p(g))
        getattr(O, fo)(ts, n, p(src), p(o))
        assert np.array_equal(g, o), fg
    L.blosc2_bitunshuffle(ts, n, B._p(src), B._p(g))
    O.or_bitunshuffle(ts, n, p(src), p(o), 6)
    assert np.array_equal(g, o)


def test_blosclz_chunk_kat(B):
    """compat/blosc-blosclz-3.0.0.cdata == blosc1_compress(9, SHUFFLE, 4, ramp)."""
    L = B.lib()
    gold = np.fromfile(os.path.join(GOLD, "blosc-blosclz-3.0.0.cdata"), np.uint8)
    L.blosc1_set_compressor(b"blosclz")
    out = np.zeros(RAMP.nbytes, np.uint8)
    n = L.blosc1_compress(9, 1, 4, RAMP.nbytes, B._p(RAMP), B._p(out), RAMP.nbytes)
    assert n == gold.nbytes
    assert np.array_equal(out[:n], gold)
    dec = np.zeros(RAMP.nbytes, np.uint8)
    assert L.blosc1_decompress(B._p(gold), B._p(dec), RAMP.nbytes) == RAMP.nbytes
    assert np.array_equal(dec.view(np.int32), RAMP)


@pytest.mark.parametrize("name", ["blosc-1.3.0-blosclz.cdata", "blosc-1.7.0-blosclz.cdata",
                                  "blosc-1.11.1-blosclz.cdata", "blosc-1.14.0-blosclz.cdata"])
def test_blosc1_decode_kats(B, name):
    gold = np.fromfile(os.path.join(GOLD, name), np.uint8)
    dec = B.decompress(gold, RAMP.nbytes)
    assert isinstance(dec, np.ndarray), dec
    assert np.array_equal(dec.view(np.int32), RAMP)


def test_golden_chunks(B):
    """Reference-produced chunks (tests/golden/make_golden.py): GPU compress is byte-identical,
    GPU decompress restores the input."""
    man = json.load(open(os.path.join(GOLD, "chunks.json")))
    data = np.load(os.path.join(GOLD, "chunks.npz"))
    for i, case in enumerate(man):
        src, want = data[f"in_{i}"], data[f"out_{i}"]
        kw = {k: case[k] for k in ("clevel", "typesize", "filters", "filters_meta", "blocksize", "splitmode")}
        got = B.compress(src, **kw)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), (i, case)
        dec = B.decompress(want, src.nbytes)
        assert isinstance(dec, np.ndarray), (i, dec)
        assert np.array_equal(dec, oracle_decompress(want, src.nbytes)), (i, case)
        if case.get("lossless", True):
            assert np.array_equal(dec, src), (i, case)


def _cases(seed, count):
    rng = np.random.default_rng(seed)
    for _ in range(count):
        ts = int(rng.choice([1, 2, 4, 8, 16]))
        kind = int(rng.integers(0, 4))
        n = int(rng.integers(1, 600_000)) // ts * ts or ts
        if kind == 0:
            src = gen_f32(int(rng.integers(0, 1 << 30)), max(1, n // 4))
            ts = 4
        elif kind == 1:
            src = int64_ramp(int(rng.integers(0, 1 << 40)), max(1, n // 8))
            ts = 8
        else:
            src = mixed_bytes(int(rng.integers(0, 1 << 30)), n)
        f5 = int(rng.choice([0, 1, 2]))
        f4 = int(rng.choice([0, 3])) if kind != 2 or ts in (1, 2, 4, 8) else 0
        yield src, dict(clevel=int(rng.integers(1, 10)), typesize=ts, filters=(0, 0, 0, 0, f4, f5),
                        blocksize=int(rng.choice([0, 0, 16384, 131072])),
                        splitmode=int(rng.choice([1, 2, 4])))


@pytest.mark.parametrize("seed", range(6))
def test_random_chunks_vs_oracle(B, seed):
    for src, kw in _cases(seed, 10):
        want = oracle_compress(src, **kw)
        got = B.compress(src, **kw)
        assert isinstance(want, np.ndarray)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), kw
        if ref() is not None:
            assert np.array_equal(ref_compress(src, **kw), want), kw
        dec = B.decompress(got, src.nbytes)
        assert np.array_equal(dec, src.view(np.uint8).reshape(-1)), kw


@pytest.mark.parametrize("slack", [-200_000, -70_000, -5000, -300, -40, 0, 32])
def test_tight_destsize_serial_semantics(B, slack):
    """destsize below nbytes+32 exercises the serial maxout reduction (blosc/blosc2.c:1343-1350),
    the memcpy fallback and the 'does not fit' (0) return."""
    L = B.lib()
    for src, ts in ((mixed_bytes(11, 400_000), 1), (gen_f32(3, 100_000), 4)):
        destsize = src.nbytes + 32 + slack
        cp = B.cparams(clevel=5, typesize=ts)
        ctx = L.blosc2_create_cctx(cp)
        got = B.compress_ctx(ctx, src, destsize=destsize)
        L.blosc2_free_ctx(ctx)
        oc = oracle()
        from oracle_lib import or_cparams
        ocp = or_cparams(clevel=5, typesize=ts)
        raw = src.view(np.uint8).reshape(-1)
        out = np.zeros(raw.nbytes + 64, np.uint8)
        n = oc.or_compress_chunk(C.byref(ocp), p(raw), raw.nbytes, p(out), destsize)
        if n > 0:
            assert isinstance(got, np.ndarray) and np.array_equal(got, out[:n]), (slack, ts)
        else:
            assert got == n, (slack, ts, got, n)


def test_context_blocksize_is_sticky(B):
    """A compression context keeps the blocksize of its previous call (blosc/blosc2.c:2414)."""
    L = B.lib()
    ctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=4))
    small, big = np.arange(1000, dtype=np.int32), np.arange(1 << 20, dtype=np.int32)
    outs = [B.compress_ctx(ctx, x) for x in (small, big)]
    L.blosc2_free_ctx(ctx)
    assert outs[1][8:12].view(np.int32)[0] == 4000
    if ref() is not None:
        R = ref()
        from b2ctypes import cparams as rcp
        rctx = R.blosc2_create_cctx(rcp(clevel=5, typesize=4))
        for x, g in zip((small, big), outs):
            o = np.zeros(x.nbytes + 64, np.uint8)
            n = R.blosc2_compress_ctx(rctx, p(x), x.nbytes, p(o), x.nbytes + 32)
            assert np.array_equal(o[:n], g)
        R.blosc2_free_ctx(rctx)


def test_maskout_and_getitem(B):
    L = B.lib()
    src = gen_f32(0, 1 << 18)
    chunk = B.compress(src, clevel=5, typesize=4, blocksize=65536)
    nblocks = src.nbytes // 65536
    mask = (C.c_bool * nblocks)(*[i % 3 == 1 for i in range(nblocks)])
    ctx = L.blosc2_create_dctx(B.dparams())
    L.blosc2_set_maskout(ctx, mask, nblocks)
    out = np.full(src.nbytes, 0xEE, np.uint8)
    assert L.blosc2_decompress_ctx(ctx, B._p(chunk), chunk.nbytes, B._p(out), out.nbytes) == src.nbytes
    raw = src.view(np.uint8)
    for b in range(nblocks):
        blk = slice(b * 65536, (b + 1) * 65536)
        if b % 3 == 1:
            assert np.all(out[blk] == 0xEE)
        else:
            assert np.array_equal(out[blk], raw[blk])
    # getitem: items [70000, 70000+5000)
    item = np.zeros(5000 * 4, np.uint8)
    assert L.blosc2_getitem_ctx(ctx, B._p(chunk), chunk.nbytes, 70000, 5000, B._p(item), item.nbytes) == item.nbytes
    assert np.array_equal(item.view(np.float32), src[70000:75000])
    L.blosc2_free_ctx(ctx)


def test_device_batch_matches_per_chunk(B):
    """b2h_compress_batch over many chunks == per-chunk oracle bytes; batch decompress restores."""
    import torch
    nchunks, chunk = 48, 1 << 20
    host = gen_f32(0, nchunks * chunk // 4)
    cases = [dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)),
             dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 2), blocksize=262144),
             dict(clevel=9, typesize=4, filters=(0, 0, 0, 0, 3, 1)),
             dict(clevel=1, typesize=4, filters=(0, 0, 0, 4, 3, 1), filters_meta=(0, 0, 0, 20, 0, 0))]
    dsrc = torch.from_numpy(host.view(np.uint8)).cuda()
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    ddst = torch.zeros(nchunks * stride, dtype=torch.uint8, device="cuda")
    dcb = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    for kw in cases:
        cp = B.cparams(**kw)
        B.compress_batch(cp, dsrc.data_ptr(), chunk, nchunks, chunk, ddst.data_ptr(), stride, cap, dcb.data_ptr())
        torch.cuda.synchronize()
        cbytes = dcb.cpu().numpy()
        out = ddst.cpu().numpy()
        for i in range(nchunks):
            want = oracle_compress(host[i * chunk // 4:(i + 1) * chunk // 4], **kw)
            assert cbytes[i] == want.nbytes and np.array_equal(out[i * stride:i * stride + cbytes[i]], want), (kw, i)
        dout = torch.zeros(nchunks * chunk, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
        B.decompress_batch(ddst.data_ptr(), stride, dcb.data_ptr(), nchunks, dout.data_ptr(), chunk, chunk,
                           dst.data_ptr())
        torch.cuda.synchronize()
        assert (dst.cpu().numpy() == chunk).all()
        if kw["filters"][3] != 4:   # trunc-prec is lossy
            assert torch.equal(dout, dsrc)


def test_fused_unshuffle_layouts(B):
    """SHUFFLE ts=4 chunks are unshuffled inside the decode launch by the wave completing each
    block (b2h_engine.hip finish_block): whole 1 KiB rows, remainder quads, blocks whose item count
    is not a multiple of 4, a bsize % 4 tail, never-split blocks, and destinations at odd offsets
    (the byte path) -- every chunk equal to its source after a strided batch decompress."""
    import torch
    cases = [dict(typesize=4, blocksize=4 * 3085, filters=(0, 0, 0, 0, 0, 1)),            # n % 4 == 1
             dict(typesize=4, blocksize=4 * 1024 * 5 + 16, filters=(0, 0, 0, 0, 0, 1)),   # rows + quads
             dict(typesize=4, blocksize=65536, filters=(0, 0, 0, 0, 0, 1), splitmode=2),  # never split
             dict(typesize=4, blocksize=0, filters=(0, 0, 0, 0, 0, 1), clevel=9)]
    nbytes = [300_001, 262_144 + 4 * 777, 1 << 20, 4 * 100_003 + 2]
    for kw in cases:
        for odd in (0, 3):
            kwc = dict(kw)
            clevel = kwc.pop("clevel", 5)
            raws = [gen_f32(11 + i, (n + 3) // 4).view(np.uint8)[:n].copy() for i, n in enumerate(nbytes)]
            chunks = [oracle_compress(r, clevel=clevel, **kwc) for r in raws]
            stride = max(c.nbytes for c in chunks) + 64
            cap = max(nbytes)
            dstride = cap + odd
            host = np.zeros(len(chunks) * stride, np.uint8)
            for i, c in enumerate(chunks):
                host[i * stride:i * stride + c.nbytes] = c
            dsrc = torch.from_numpy(host).cuda()
            dcb = torch.tensor([c.nbytes for c in chunks], dtype=torch.int32, device="cuda")
            dout = torch.full((len(chunks) * dstride + 64,), 0xEE, dtype=torch.uint8, device="cuda")
            dst = torch.zeros(len(chunks), dtype=torch.int32, device="cuda")
            B.decompress_batch(dsrc.data_ptr(), stride, dcb.data_ptr(), len(chunks), dout.data_ptr(), dstride, cap,
                               dst.data_ptr())
            torch.cuda.synchronize()
            assert list(dst.cpu().numpy()) == nbytes, (kw, odd)
            out = dout.cpu().numpy()
            for i, r in enumerate(raws):
                assert np.array_equal(out[i * dstride:i * dstride + r.nbytes], r), (kw, odd, i)


def test_ragged_batch_matches_oracle_without_host_wait(B):
    """b2h_compress_batch_sizes: a super-chunk's chunks with a short last one (ref
    blosc2_schunk_append_buffer, blosc/schunk.c:1459-1477: destsize nbytes + 32 per chunk) ride in
    one call, byte-identical per chunk to the oracle, queued without a host wait; the strided batch
    decompression restores every chunk, the short one included."""
    import time
    import torch
    chunk, nfull, tail = 1 << 20, 6, 123_457 * 4
    sizes = [chunk] * nfull + [tail]
    host = gen_f32(3, (nfull * chunk + tail) // 4)
    raw = host.view(np.uint8)
    stride = chunk + 256
    dsrc = torch.zeros(len(sizes) * stride, dtype=torch.uint8, device="cuda")
    for i, n in enumerate(sizes):
        dsrc[i * stride:i * stride + n] = torch.from_numpy(raw[i * chunk:i * chunk + n].copy()).cuda()
    ddst = torch.zeros(len(sizes) * stride, dtype=torch.uint8, device="cuda")
    dcb = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    for kw in (dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)),
               dict(clevel=9, typesize=4, filters=(0, 0, 0, 0, 3, 1), blocksize=65536)):
        cp = B.cparams(**kw)
        s = torch.cuda.Stream()
        torch.cuda.synchronize()
        with torch.cuda.stream(s):
            torch.cuda._sleep(200_000_000)   # keep the stream busy: a host wait inside would block here
            t0 = time.perf_counter()
            B.compress_batch_sizes(cp, dsrc.data_ptr(), sizes, stride, ddst.data_ptr(), stride, 0, dcb.data_ptr(),
                                   s.cuda_stream)
            queued = time.perf_counter() - t0
        s.synchronize()
        assert queued < 0.05, queued
        cbytes = dcb.cpu().numpy()
        out = ddst.cpu().numpy()
        for i, n in enumerate(sizes):
            want = oracle_compress(raw[i * chunk:i * chunk + n].copy().view(np.float32), **kw)
            assert cbytes[i] == want.nbytes and np.array_equal(out[i * stride:i * stride + cbytes[i]], want), (kw, i)
        dout = torch.zeros(len(sizes) * chunk, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
        B.decompress_batch(ddst.data_ptr(), stride, dcb.data_ptr(), len(sizes), dout.data_ptr(), chunk, chunk,
                           dst.data_ptr())
        torch.cuda.synchronize()
        assert list(dst.cpu().numpy()) == sizes
        back = dout.cpu().numpy()
        for i, n in enumerate(sizes):
            assert np.array_equal(back[i * chunk:i * chunk + n], raw[i * chunk:i * chunk + n]), i


@pytest.mark.slow
def test_c2_shuffle_256mib_roundtrip(B):
    """C2 at full size: 256 MiB float32 shuffle ts=4 on device vs a numpy transpose (bit-exact)."""
    import torch
    n = 256 << 20
    host = gen_f32(0, n // 4)
    d = torch.from_numpy(host.view(np.uint8)).cuda()
    o = torch.empty_like(d)
    L = B.lib()
    assert L.b2h_shuffle(4, n, C.c_void_p(d.data_ptr()), C.c_void_p(o.data_ptr()), 0, None) == n
    torch.cuda.synchronize()
    want = host.view(np.uint8).reshape(-1, 4).T.reshape(-1)
    assert np.array_equal(o.cpu().numpy(), want)
    back = torch.empty_like(d)
    L.b2h_shuffle(4, n, C.c_void_p(o.data_ptr()), C.c_void_p(back.data_ptr()), 1, None)
    torch.cuda.synchronize()
    assert torch.equal(back, d)


def _far_match_data(n, seed):
    """Streams whose matches reach further back than the decoder's LDS ring (32 KiB): a 20 KB
    random segment repeated every 36 KB (zeros and a short period in between)."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, 20_000, dtype=np.uint8)
    parts = []
    while sum(p.nbytes for p in parts) < n:
        parts += [a, np.zeros(14_000, np.uint8), np.tile(rng.integers(0, 256, 5, dtype=np.uint8), 400)]
    return np.concatenate(parts)[:n]


@pytest.mark.parametrize("bs", [65536, 262144])
@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_far_matches_long_streams(B, bs, clevel):
    """Single-stream blocks (typesize 1) of 64 / 256 KiB: LZ distances up to the far limit, match
    sources older than the decoder's LDS ring; compress == oracle, decompress round-trips."""
    src = _far_match_data(3 * bs + 1000, clevel * 31 + bs)
    kw = dict(clevel=clevel, typesize=1, filters=(0, 0, 0, 0, 0, 0), blocksize=bs)
    want = oracle_compress(src, **kw)
    got = B.compress(src, **kw)
    assert isinstance(got, np.ndarray) and np.array_equal(got, want)
    assert want.nbytes < 0.8 * src.nbytes        # the far matches were actually taken
    dec = B.decompress(got, src.nbytes)
    assert isinstance(dec, np.ndarray) and np.array_equal(dec, src)


@pytest.mark.parametrize("seed", range(4))
def test_corrupted_streams_match_oracle(B, seed):
    """Damaged LZ payloads: the device decoder accepts / rejects exactly like the oracle
    (blosclz_decompress bound checks, blosc_d's size check), and agrees on the bytes it accepts."""
    rng = np.random.default_rng(seed)
    src = gen_f32(seed << 20, 1 << 16)
    good = oracle_compress(src, clevel=5, typesize=4)
    hdr = 32 + 4 * ((src.nbytes + 262143) // 262144)
    for _ in range(25):
        bad = good.copy()
        k = int(rng.integers(1, 4))
        for pos in rng.integers(hdr + 4, bad.nbytes, k):
            bad[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        o = oracle_decompress(bad, src.nbytes)
        g = B.decompress(bad, src.nbytes)
        if isinstance(o, np.ndarray):
            assert isinstance(g, np.ndarray) and np.array_equal(g, o)
        else:
            assert not isinstance(g, np.ndarray) and g < 0


def _long_match_data(n, seed):
    """A random 4 KiB segment repeated with one byte changed every ~190 bytes: streams of
    (literal, ~190-byte match) token pairs, so one 64-token decode batch outputs several KiB --
    more than half of the decoder's 8 KiB LDS ring."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, 4096, dtype=np.uint8)
    parts = [base]
    while sum(p.nbytes for p in parts) < n:
        seg = base.copy()
        for pos in range(int(rng.integers(0, 60)), seg.nbytes, 190):
            seg[pos] ^= np.uint8(1 + int(rng.integers(0, 255)))
        parts.append(seg)
    return np.concatenate(parts)[:n]


@pytest.mark.parametrize("bs", [65536, 262144])
def test_long_match_batches(B, bs):
    """Decode batches whose output approaches the ring capacity (flush frontier bookkeeping):
    compress == oracle, decompress round-trips and equals the oracle's decode."""
    src = _long_match_data(2 * bs + 777, bs)
    kw = dict(clevel=5, typesize=1, filters=(0, 0, 0, 0, 0, 0), blocksize=bs)
    want = oracle_compress(src, **kw)
    got = B.compress(src, **kw)
    assert isinstance(got, np.ndarray) and np.array_equal(got, want)
    assert want.nbytes < 0.2 * src.nbytes        # long matches were taken
    dec = B.decompress(got, src.nbytes)
    assert isinstance(dec, np.ndarray) and np.array_equal(dec, src)


@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_plugin_filters_vs_oracle(B, clevel):
    """bytedelta (35) / int_trunc (36) pipelines on the device: chunks byte-identical to the oracle
    (itself pinned to the reference library in test_oracle.py), decode == the oracle's decode."""
    from test_oracle import PLUGIN_PIPES, plugin_input
    for case, pipe in enumerate(PLUGIN_PIPES):
        kw = dict(pipe, clevel=clevel)
        for n, bs in ((200_000, 0), (3 * 65536 + 4096, 65536), (1 << 20, 262144)):
            src = plugin_input(kw, n, case * 7 + clevel)
            want = oracle_compress(src, blocksize=bs, **kw)
            got = B.compress(src, blocksize=bs, **kw)
            assert isinstance(got, np.ndarray) and np.array_equal(got, want), (kw, n, bs)
            dec = B.decompress(want, src.nbytes)
            assert isinstance(dec, np.ndarray) and np.array_equal(dec, oracle_decompress(want, src.nbytes)), (kw, n)
            if 36 not in kw["filters"]:
                assert np.array_equal(dec, src)


def test_plugin_filter_errors(B):
    """Failing plugin filters end the pipeline with BLOSC2_ERROR_FILTER_PIPELINE, as in the reference."""
    src = gen_f32(0, 50_000).view(np.uint8)
    for kw in (dict(typesize=4, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, 40)),
               dict(typesize=4, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, (-32) & 0xFF)),
               dict(typesize=3, filters=(0, 0, 0, 0, 0, 36), filters_meta=(0, 0, 0, 0, 0, 4)),
               dict(typesize=4, filters=(0, 0, 0, 0, 1, 35), filters_meta=(0,) * 6)):   # meta 0, no schunk
        s = src[:49_998] if kw["typesize"] == 3 else src
        assert B.compress(s, clevel=5, **kw) == -18, kw


def _tunable(seed, n, q):
    """Random bytes where a fraction q of 16-byte groups repeat the group 64 bytes earlier: the
    entropy probe's ratio sweeps across the clevel thresholds (blosc/blosclz.c:463-468) as q varies."""
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, n, dtype=np.uint8)
    for g in np.nonzero(rng.random(n // 16) < q)[0]:
        if g >= 4:
            a[16 * g:16 * g + 16] = a[16 * (g - 4):16 * (g - 4) + 16]
    return a


@pytest.mark.parametrize("clevel", [1, 2, 3, 5, 7, 8, 9])
def test_probe_threshold_sweep(B, clevel):
    """Streams whose probe ratio lands on either side of the threshold: the device's exact early
    decisions of the probe (early reject / early accept) give the oracle's chunks."""
    for i, q in enumerate(np.linspace(0.0, 0.9, 19)):
        src = _tunable(clevel * 100 + i, 4 * 65536 + 999, float(q))
        kw = dict(clevel=clevel, typesize=1, filters=(0, 0, 0, 0, 0, 0), blocksize=65536, splitmode=2)
        want = oracle_compress(src, **kw)
        got = B.compress(src, **kw)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), (clevel, q)


@pytest.mark.gpu
@pytest.mark.parametrize("ts", [2, 4, 8])
def test_fused_delta_shuffle_vs_oracle(B, ts):
    """(DELTA, SHUFFLE) pipelines run as one fused pass per block in both directions (k_ffilter_ds,
    unshuffle_scan/xor_fast); blocks that are not whole quads fall back to the two stages.  Sizes
    cover whole-quad leftovers, ragged leftovers, one-block chunks and several blocks; the chunks
    must be byte-identical to the oracle and round-trip."""
    rng = np.random.default_rng(ts)
    sizes = [4 * ts, 4 * ts * 1000, 65536, 65536 + 4 * ts * 7, 65536 + ts * 3, 300_000 // ts * ts,
             (1 << 20) + 4 * ts, (1 << 20) - ts]
    for n in sizes:
        for kind in range(3):
            if kind == 0:
                src = int64_ramp(int(rng.integers(0, 1 << 40)), -(-n // 8)).view(np.uint8)[:n].copy()
            elif kind == 1:
                src = gen_f32(int(rng.integers(0, 1 << 30)), -(-n // 4)).view(np.uint8)[:n].copy()
            else:
                src = mixed_bytes(int(rng.integers(0, 1 << 30)), n)
            for meta in (0, ts):
                kw = dict(clevel=int(rng.integers(1, 10)), typesize=ts, filters=(0, 0, 0, 0, 3, 1),
                          filters_meta=(0, 0, 0, 0, 0, meta), blocksize=int(rng.choice([0, 16384, 65536])))
                want = oracle_compress(src, **kw)
                got = B.compress(src, **kw)
                assert isinstance(got, np.ndarray) and np.array_equal(got, want), (n, kind, kw)
                dec = B.decompress(got, src.nbytes)
                assert np.array_equal(dec, src), (n, kind, kw)


@pytest.mark.gpu
def test_learned_pull_order_keeps_chunks(B):
    """The encoder pulls streams plane by plane in the cost order learned from the previous batch
    of the same split (k_plane_cost -> pull_to_stream).  Scheduling only: a repeated compression
    (second call runs on the learned order), other splits in between, and ragged leftover blocks
    must all give the oracle's chunk."""
    for n, ts in ((4 << 20, 4), (3_000_000, 4), (1 << 20, 8), (777_777 // 2 * 2, 2), (1 << 20, 16),
                  (4 << 20, 4)):
        src = gen_f32(n, n // 4).view(np.uint8)[: n // ts * ts].copy() if ts == 4 else mixed_bytes(n, n // ts * ts)
        kw = dict(clevel=5, typesize=ts, filters=(0, 0, 0, 0, 0, 1), blocksize=65536)
        want = oracle_compress(src, **kw)
        for _ in range(2):
            got = B.compress(src, **kw)
            assert isinstance(got, np.ndarray) and np.array_equal(got, want), (n, ts)


@pytest.mark.parametrize("shape", [(-1, -1), (1, 0), (1, 3), (1, 1), (0, 1)])
def test_exact_encoder_shapes_same_bytes(B, shape):
    """Every exact-encoder workgroup shape (b2h_set_encode_shape: auto, LDS tables only, 1 LDS + 3 /
    1 global-table waves, global tables only) gives the oracle's bytes: u16 positions (64 KiB
    streams) and u32 (256 KiB BITSHUFFLE blocks, unsplit), a batch small enough for the LDS-only
    shape (auto picks it) and one of 600 chunks that is not (auto: 1 + 3), plus the per-call path."""
    import torch
    L = B.lib()
    L.b2h_set_blosclz_mode(0)
    assert L.b2h_set_encode_shape(*shape) >= -1
    assert L.b2h_set_encode_shape(-2, 0) == (-1 if shape == (-1, -1) else 16 * shape[0] + shape[1])
    try:
        chunk = 1 << 18
        cases = [(dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)), 600),
                 (dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 2), blocksize=262144), 6)]
        for kw, nchunks in cases:
            host = gen_f32(7, nchunks * chunk // 4)
            dsrc = torch.from_numpy(host.view(np.uint8)).cuda()
            cap = chunk + 32
            stride = (cap + 255) // 256 * 256
            ddst = torch.zeros(nchunks * stride, dtype=torch.uint8, device="cuda")
            dcb = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
            B.compress_batch(B.cparams(**kw), dsrc.data_ptr(), chunk, nchunks, chunk, ddst.data_ptr(), stride, cap,
                             dcb.data_ptr())
            torch.cuda.synchronize()
            cbytes = dcb.cpu().numpy()
            out = ddst.cpu().numpy()
            for i in sorted({0, nchunks // 2, nchunks - 1}):
                want = oracle_compress(host[i * chunk // 4:(i + 1) * chunk // 4], **kw)
                assert cbytes[i] == want.nbytes and np.array_equal(out[i * stride:i * stride + cbytes[i]], want), (kw, i)
        # the per-call drop-in path (one chunk per call)
        src = RAMP.copy()
        dst = np.zeros(src.nbytes + 32, np.uint8)
        L.blosc1_set_compressor(b"blosclz")
        n = L.blosc1_compress(5, 1, 4, src.nbytes, B._p(src), B._p(dst), dst.nbytes)
        want = oracle_compress(src, clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1))
        assert n == want.nbytes and np.array_equal(dst[:n], want)
    finally:
        L.b2h_set_encode_shape(-1, -1)


@pytest.mark.parametrize("rlog", [None, "12", "13", "14", "15"])
def test_decoder_ring_sizes_same_output(B, rlog, monkeypatch):
    """The decoder's LDS ring (B2H_DEC_RING; unset: 32 KiB for batches whose streams all fit its
    resident waves, else 8 KiB) never changes the output: exact-mode chunks of T's shape and of
    C1's b2bench data (long far matches), decoded at every ring size, equal the input."""
    import torch
    from datagen import b2bench_values
    if rlog is None:
        monkeypatch.delenv("B2H_DEC_RING", raising=False)
    else:
        monkeypatch.setenv("B2H_DEC_RING", rlog)
    L = B.lib()
    L.b2h_set_blosclz_mode(0)
    for name, host, kw in [("f32", gen_f32(5, 3 * (1 << 20) // 4), dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1))),
                           ("b2bench", b2bench_values(1_000_000, 19), dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1)))]:
        raw = host.view(np.uint8).reshape(-1)
        chunk = oracle_compress(host, **kw)
        assert isinstance(chunk, np.ndarray)
        out = np.zeros(raw.nbytes, np.uint8)
        dctx = L.blosc2_create_dctx(B.dparams())
        n = L.blosc2_decompress_ctx(dctx, B._p(chunk), chunk.nbytes, B._p(out), out.nbytes)
        L.blosc2_free_ctx(dctx)
        assert n == raw.nbytes and np.array_equal(out, raw), (name, rlog)
