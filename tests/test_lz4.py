"""LZ4 codec (compformat 1) on the device: chunks compressed with
compcode=BLOSC_LZ4 through the drop-in ABI are byte-identical to the oracle restatement (itself
pinned to liblz4 1.9.3 and to oracle/_ref, tests/test_oracle.py::test_lz4_*), the compat LZ4 KATs
decode and re-encode on the device, and device decode agrees with the oracle on damaged streams."""
import os
import sys

import numpy as np
import pytest

from b2ctypes import REPO
from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import oracle_compress, oracle_decompress, ref, ref_compress

sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))

pytestmark = pytest.mark.gpu
GOLD = os.path.join(REPO, "tests", "golden")
RAMP = np.arange(1_000_000, dtype=np.int32)
LZ4 = 1


@pytest.fixture(scope="module")
def B():
    import torch  # noqa: F401
    import blosc2_amd
    assert blosc2_amd.lib().b2h_device_count() > 0
    return blosc2_amd


def test_lz4_chunk_kat(B):
    """compat/blosc-lz4-3.0.0.cdata: device compress reproduces it, device decompress inverts it."""
    gold = np.fromfile(os.path.join(GOLD, "blosc-lz4-3.0.0.cdata"), np.uint8)
    got = B.compress(RAMP, clevel=9, typesize=4, compcode=LZ4, splitmode=4)
    assert isinstance(got, np.ndarray) and np.array_equal(got, gold)
    assert np.array_equal(B.decompress(gold, RAMP.nbytes).view(np.int32), RAMP)


@pytest.mark.parametrize("name", ["blosc-1.11.1-lz4.cdata", "blosc-1.14.0-lz4.cdata",
                                  "blosc-1.17.1-lz4-bitshuffle4-memcpy.cdata",
                                  "blosc-1.17.1-lz4-bitshuffle8-nomemcpy.cdata",
                                  "blosc-1.18.0-lz4-bitshuffle4-memcpy.cdata",
                                  "blosc-1.18.0-lz4-bitshuffle8-nomemcpy.cdata"])
def test_lz4_legacy_kats(B, name):
    gold = np.fromfile(os.path.join(GOLD, name), np.uint8)
    nbytes = int(gold[4:8].view(np.int32)[0])
    want = oracle_decompress(gold, nbytes)
    got = B.decompress(gold, nbytes)
    # format-version-2 bitshuffle leaves the trailing nbytes % ts bytes of its last block unwritten
    # in the reference (blosc/shuffle.c:489-500; see tests/test_oracle.py::test_lz4_decode_kats)
    ts = int(gold[3])
    whole = nbytes - nbytes % ts if gold[0] == 2 and gold[2] & 4 else nbytes
    assert isinstance(got, np.ndarray) and np.array_equal(got[:whole], want[:whole])


def _cases(seed, n):
    rng = np.random.default_rng(seed)
    for _ in range(n):
        kind = int(rng.integers(0, 3))
        size = int(rng.integers(1, 600_000))
        if kind == 0:
            src, ts = gen_f32(int(rng.integers(0, 1 << 30)), max(1, size // 4)), 4
        elif kind == 1:
            src, ts = int64_ramp(int(rng.integers(0, 1 << 30)), max(1, size // 8)), 8
        else:
            ts = int(rng.choice([1, 2, 4]))   # delta leaves nbytes % ts bytes unwritten: keep whole elements
            src = mixed_bytes(int(rng.integers(0, 1 << 30)), size // ts * ts or ts)
        yield src, dict(clevel=int(rng.integers(1, 10)), typesize=ts,
                        filters=(0, 0, 0, 0, int(rng.choice([0, 3])) if ts in (1, 2, 4, 8) else 0,
                                 int(rng.choice([0, 1, 2]))),
                        blocksize=int(rng.choice([0, 0, 16384, 131072, 262144])),
                        splitmode=int(rng.choice([1, 2, 4])), compcode=LZ4)


@pytest.mark.parametrize("seed", range(5))
def test_lz4_random_chunks_vs_oracle(B, seed):
    for src, kw in _cases(100 + seed, 10):
        want = oracle_compress(src, **kw)
        got = B.compress(src, **kw)
        assert isinstance(want, np.ndarray)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), kw
        if ref() is not None:
            assert np.array_equal(ref_compress(src, **kw), want), kw
        dec = B.decompress(got, src.nbytes)
        assert np.array_equal(dec, src.view(np.uint8).reshape(-1)), kw


@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_lz4_north_star_shapes(B, clevel):
    """T's shape with LZ4: float32 ts=4 SHUFFLE, 4 MiB chunk (256 KiB blocks x 4 streams of 64 KiB,
    the byU16 table) and NEVER_SPLIT 256 KiB streams (the byU32 table with the 5-byte hash)."""
    src = gen_f32(clevel << 22, 1 << 20)
    for split in (4, 2):
        kw = dict(clevel=clevel, typesize=4, filters=(0, 0, 0, 0, 0, 1), compcode=LZ4, splitmode=split)
        want = oracle_compress(src, **kw)
        got = B.compress(src, **kw)
        assert isinstance(got, np.ndarray) and np.array_equal(got, want), kw
        assert np.array_equal(B.decompress(got, src.nbytes).view(np.float32), src)


@pytest.mark.parametrize("slack", [-300_000, -5000, -40, 0])
def test_lz4_tight_destsize(B, slack):
    """Reduced maxout per stream (blosc/blosc2.c:1343-1350) with LZ4's limited-output checks."""
    import ctypes as C
    from oracle_lib import oracle, or_cparams, p
    L = B.lib()
    src = gen_f32(5, 200_000)
    destsize = src.nbytes + 32 + slack
    ctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=4, compcode=LZ4))
    got = B.compress_ctx(ctx, src, destsize=destsize)
    L.blosc2_free_ctx(ctx)
    ocp = or_cparams(clevel=5, typesize=4, compcode=LZ4)
    raw = src.view(np.uint8).reshape(-1)
    out = np.zeros(raw.nbytes + 64, np.uint8)
    n = oracle().or_compress_chunk(C.byref(ocp), p(raw), raw.nbytes, p(out), destsize)
    if n > 0:
        assert isinstance(got, np.ndarray) and np.array_equal(got, out[:n])
    else:
        assert got == n


@pytest.mark.parametrize("seed", range(3))
def test_lz4_corrupted_streams_match_oracle(B, seed):
    rng = np.random.default_rng(seed)
    src = gen_f32(seed << 20, 1 << 16)
    good = oracle_compress(src, clevel=5, typesize=4, compcode=LZ4)
    hdr = 32 + 4 * ((src.nbytes + 262143) // 262144)
    for _ in range(25):
        bad = good.copy()
        for pos in rng.integers(hdr + 4, bad.nbytes, int(rng.integers(1, 4))):
            bad[pos] ^= np.uint8(1 << int(rng.integers(0, 8)))
        o = oracle_decompress(bad, src.nbytes)
        g = B.decompress(bad, src.nbytes)
        if isinstance(o, np.ndarray):
            assert isinstance(g, np.ndarray) and np.array_equal(g, o)
        else:
            assert not isinstance(g, np.ndarray) and g < 0


def test_lz4_device_batch(B):
    """b2h_compress_batch / b2h_decompress_batch with compcode LZ4 over 32 x 4 MiB chunks."""
    import torch
    nchunks, chunk = 32, 1 << 22
    host = gen_f32(0, nchunks * chunk // 4)
    kw = dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1), compcode=LZ4)
    dsrc = torch.from_numpy(host.view(np.uint8)).cuda()
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    ddst = torch.zeros(nchunks * stride, dtype=torch.uint8, device="cuda")
    dcb = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    B.compress_batch(B.cparams(**kw), dsrc.data_ptr(), chunk, nchunks, chunk, ddst.data_ptr(), stride, cap,
                     dcb.data_ptr())
    torch.cuda.synchronize()
    cbytes, out = dcb.cpu().numpy(), ddst.cpu().numpy()
    for i in (0, 7, nchunks - 1):
        want = oracle_compress(host[i * chunk // 4:(i + 1) * chunk // 4], **kw)
        assert cbytes[i] == want.nbytes and np.array_equal(out[i * stride:i * stride + cbytes[i]], want), i
    dout = torch.zeros(nchunks * chunk, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    B.decompress_batch(ddst.data_ptr(), stride, dcb.data_ptr(), nchunks, dout.data_ptr(), chunk, chunk,
                       dst.data_ptr())
    torch.cuda.synchronize()
    assert (dst.cpu().numpy() == chunk).all()
    assert torch.equal(dout, dsrc)
