"""GPU tier: LZ4 chunks with a dictionary (cparams.use_dict; blosc2_compress_ctx's training pass and
LZ4_loadDict + LZ4_compress_fast_continue, blosc/blosc2.c:3146-3235 and 455-465).  The device
chunks are compared byte for byte with the oracle (oracle/blosc2_oracle.c or_compress_chunk with
use_dict, itself pinned to the reference build in tests/test_oracle.py) and with the reference
library when oracle/_ref is present; they decode on the device back to the input."""
import ctypes as C

import numpy as np
import pytest

from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import oracle, oracle_decompress, or_cparams, p, ref, ref_compress

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B():
    import torch  # noqa: F401
    import blosc2_amd
    assert blosc2_amd.lib().b2h_device_count() > 0
    return blosc2_amd


def _oracle_chunk(src, destsize=None, **kw):
    raw = src.view(np.uint8).reshape(-1)
    destsize = raw.nbytes + 32 if destsize is None else destsize
    out = np.zeros(max(destsize, raw.nbytes + 32) + 64, np.uint8)
    n = oracle().or_compress_chunk(C.byref(or_cparams(**kw)), p(raw), raw.nbytes, p(out), destsize)
    return out[:n] if n > 0 else n


def _long_matches(n, seed):
    """Repeated 3-40 KiB phrases: matches that reach back into the dictionary and run on."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, 40_000, dtype=np.uint8)
    out, k = [], 0
    while k < n:
        a = int(rng.integers(0, 30_000))
        m = int(rng.integers(3_000, 10_000))
        out.append(base[a:a + m])
        out.append(rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8))
        k += m
    return np.concatenate(out)[:n]


def _inputs():
    yield "f32", gen_f32(0, 1 << 18), 4
    yield "ramp64", int64_ramp(5, 1 << 17), 8
    yield "mixed", mixed_bytes(3, 700_001), 1
    yield "mixed4", mixed_bytes(4, 400_000).view(np.int32), 4
    yield "zeros", np.zeros(300_000, np.uint8), 4
    yield "rand", np.random.default_rng(9).integers(0, 256, 250_000, dtype=np.uint8), 4
    yield "long", _long_matches(1 << 20, 2), 1
    yield "small", mixed_bytes(6, 6_000), 1


FILTERS = [(0, 0, 0, 0, 0, 1), (0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 3, 1), (0, 0, 0, 0, 0, 2)]


@pytest.mark.parametrize("clevel", [1, 5, 9])
@pytest.mark.parametrize("filters", FILTERS)
def test_lz4_dict_chunks_vs_oracle(B, clevel, filters):
    for name, src, ts in _inputs():
        for bs in (0, 65536, 262144):
            kw = dict(clevel=clevel, typesize=ts, filters=filters, compcode=1, use_dict=1, blocksize=bs)
            want = _oracle_chunk(src, **kw)
            got = B.compress(src, **kw)
            assert isinstance(want, np.ndarray)
            assert isinstance(got, np.ndarray) and np.array_equal(got, want), (name, kw)
            if ref() is not None:
                assert np.array_equal(ref_compress(src, **kw), want), (name, kw)
            raw = src.view(np.uint8).reshape(-1)
            dec = B.decompress(got, raw.nbytes)
            if got[2] & 0x02:   # memcpyed with the dictionary flag: undecodable, as the reference's
                assert isinstance(dec, int) and dec == oracle_decompress(got, raw.nbytes), (name, kw)
            else:
                assert isinstance(dec, np.ndarray) and np.array_equal(dec, raw), (name, kw)


@pytest.mark.parametrize("filters,meta", [((0, 0, 0, 3, 1, 2), (0,) * 6),
                                          ((0, 0, 0, 4, 3, 1), (0, 0, 0, 16, 0, 0))])
def test_lz4_dict_three_filters(B, filters, meta):
    """Three active filters rewrite the input during the training pass (pipeline_forward's buffer
    cycle), and the real pass filters the rewritten input: the device runs the chain twice."""
    src = gen_f32(7, 300_000)
    for clevel in (1, 5, 9):
        kw = dict(clevel=clevel, typesize=4, filters=filters, filters_meta=meta, compcode=1, use_dict=1)
        want = _oracle_chunk(src, **kw)
        got = B.compress(src, **kw)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), kw
        if ref() is not None:
            assert np.array_equal(ref_compress(src, **kw), want), kw


def _tight(B, src, ts, destsize, bs=0):
    L = B.lib()
    ctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=ts, compcode=1, use_dict=1, blocksize=bs))
    got = B.compress_ctx(ctx, src, destsize=destsize)
    L.blosc2_free_ctx(ctx)
    want = _oracle_chunk(src, destsize=destsize, clevel=5, typesize=ts, compcode=1, use_dict=1, blocksize=bs)
    if isinstance(want, np.ndarray):
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), (destsize, ts, bs)
    else:
        assert got == want, (destsize, ts, bs, got, want)


@pytest.mark.parametrize("slack", [-200_000, -5000, -40, -1, 0, 32])
def test_lz4_dict_tight_destsize(B, slack):
    """destsize below nbytes+32: the training pass gives the chunk up (0) or overruns
    (BLOSC2_ERROR_WRITE_BUFFER); at or above it, the dictionary pass or its memcpy fallback."""
    for src, ts in ((mixed_bytes(11, 400_000), 1), (gen_f32(3, 100_000), 4),
                    (np.random.default_rng(1).integers(0, 256, 200_000, dtype=np.uint8), 1)):
        _tight(B, src, ts, src.nbytes + 32 + slack)


def test_lz4_dict_destsize_sweep(B):
    """The sweep of tests/test_oracle.py::test_lz4_dict_destsize_sweep (pinned to the reference)."""
    for src, ts in ((mixed_bytes(11, 40_000), 1), (gen_f32(3, 10_000), 4)):
        for bs in (0, 64, 256, 4096):
            for ds in list(range(28, 80, 3)) + [100, 300, 1000, 4128, 4129, 8000, 39999, 40031, 40032, 40033]:
                _tight(B, src, ts, ds, bs)


def test_use_dict_other_codecs_refused(B):
    """BloscLZ with use_dict: BLOSC2_ERROR_CODEC_PARAM (blosc/blosc2.c:2514-2521)."""
    src = gen_f32(1, 100_000)
    got = B.compress(src, clevel=5, typesize=4, compcode=0, use_dict=1)
    assert got == -8
    want = _oracle_chunk(src, clevel=5, typesize=4, compcode=0, use_dict=1)
    assert want == -8
    if ref() is not None:
        assert ref_compress(src, clevel=5, typesize=4, compcode=0, use_dict=1) == -8


def test_lz4_dict_device_batch(B):
    """b2h_compress_batch with use_dict == per-chunk oracle bytes; b2h_decompress_batch restores."""
    import torch
    nchunks, chunk = 24, 1 << 20
    host = gen_f32(4, nchunks * chunk // 4)
    dsrc = torch.from_numpy(host.view(np.uint8)).cuda()
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    for kw in (dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1), compcode=1, use_dict=1),
               dict(clevel=9, typesize=4, filters=(0, 0, 0, 0, 3, 1), compcode=1, use_dict=1, blocksize=65536)):
        ddst = torch.zeros(nchunks * stride, dtype=torch.uint8, device="cuda")
        dcb = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
        B.compress_batch(B.cparams(**kw), dsrc.data_ptr(), chunk, nchunks, chunk, ddst.data_ptr(), stride,
                         cap, dcb.data_ptr())
        torch.cuda.synchronize()
        cbytes, out = dcb.cpu().numpy(), ddst.cpu().numpy()
        for i in range(nchunks):
            want = _oracle_chunk(host[i * chunk // 4:(i + 1) * chunk // 4], **kw)
            assert cbytes[i] == want.nbytes and np.array_equal(out[i * stride:i * stride + cbytes[i]], want), (kw, i)
            assert out[i * stride + 31] & 0x01, "dictionary flag"
        dout = torch.zeros(nchunks * chunk, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
        B.decompress_batch(ddst.data_ptr(), stride, dcb.data_ptr(), nchunks, dout.data_ptr(), chunk, chunk,
                           dst.data_ptr())
        torch.cuda.synchronize()
        assert (dst.cpu().numpy() == chunk).all()
        assert torch.equal(dout, dsrc)
