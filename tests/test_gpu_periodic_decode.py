"""GPU tier: long overlapping BloscLZ matches, the decoder's periodic copy (b2h_lz.h copy_general:
after the first D bytes -- the smallest multiple of lcm(distance, 16) that is >= 1 KiB -- a match
copies 16 bytes per lane from D back) and its ring-resident slab copies, against the oracle
(blosc/blosclz.c:685-795 restated in oracle/blosc2_oracle.c).

Periodic data of many periods (1 .. 8000 bytes) behind prefixes of 0 .. 13 bytes, so the long
match starts at every alignment of the output; typesize 1, no filter, one 256 KiB block (one
stream), clevel 9.  Each chunk goes through the single-chunk host path (blosc2_decompress_ctx)
and all of them through one device batch.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu

PERIODS = [1, 2, 3, 7, 16, 24, 33, 64, 100, 256, 257, 1000, 1024, 1500, 3000, 5000, 8000]


def _periodic(period, prefix, nbytes, seed):
    rng = np.random.default_rng(seed)
    pat = rng.integers(0, 256, period, dtype=np.uint8)
    body = np.resize(pat, nbytes - prefix)
    return np.concatenate([rng.integers(0, 256, prefix, dtype=np.uint8), body])


def test_gpu_periodic_long_matches():
    import torch
    import blosc2_amd as B
    from oracle_lib import oracle_compress, oracle_decompress
    nbytes = 256 * 1024 - 37   # a ragged tail as well
    kw = dict(clevel=9, typesize=1, filters=(0, 0, 0, 0, 0, 0), blocksize=256 * 1024)
    raws, chunks = [], []
    for i, period in enumerate(PERIODS):
        for prefix in (0, 5, 13):
            raw = _periodic(period, prefix, nbytes, 1000 * i + prefix)
            c = oracle_compress(raw, **kw)
            assert isinstance(c, np.ndarray), (period, prefix)
            assert np.array_equal(oracle_decompress(c, nbytes), raw), (period, prefix)
            got = np.asarray(B.decompress(c, nbytes)).view(np.uint8).reshape(-1)[:nbytes]
            assert np.array_equal(got, raw), (period, prefix)
            raws.append(raw)
            chunks.append(c)
    n = len(chunks)
    sstride = max(c.nbytes for c in chunks) + 256
    host = np.zeros(n * sstride, np.uint8)
    cbytes = np.zeros(n, np.int32)
    for i, c in enumerate(chunks):
        host[i * sstride:i * sstride + c.nbytes] = c
        cbytes[i] = c.nbytes
    dsrc = torch.from_numpy(host).cuda()
    dcb = torch.from_numpy(cbytes).cuda()
    dstride = (nbytes + 255) // 256 * 256
    dout = torch.zeros(n * dstride, dtype=torch.uint8, device="cuda")
    st = torch.zeros(n, dtype=torch.int32, device="cuda")
    B.decompress_batch(dsrc.data_ptr(), sstride, dcb.data_ptr(), n, dout.data_ptr(), dstride, nbytes, st.data_ptr())
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == nbytes).all(), st.cpu().numpy()
    back = dout.cpu().numpy()
    for i, r in enumerate(raws):
        assert np.array_equal(back[i * dstride:i * dstride + nbytes], r), i


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_gpu_periodic_long_match_encode(mode):
    """The encoders' match extension over the same data (b2h_lz.h wave_match_end: 4 KiB steps in
    one round trip, lanes past the bound reading the step's first bytes): exact-mode chunks are
    the oracle's byte for byte; fast-mode chunks decode with the oracle to the input."""
    import blosc2_amd as B
    from oracle_lib import oracle_compress, oracle_decompress
    nbytes = 256 * 1024 - 37
    kw = dict(clevel=9, typesize=1, filters=(0, 0, 0, 0, 0, 0), blocksize=256 * 1024)
    for i, period in enumerate(PERIODS):
        for prefix in (0, 13):
            raw = _periodic(period, prefix, nbytes, 7 * i + prefix)
            c = B.compress(raw, lz_mode=B.EXACT if mode == "exact" else B.FAST, **kw)
            assert isinstance(c, np.ndarray), (period, prefix)
            if mode == "exact":
                want = oracle_compress(raw, **kw)
                assert np.array_equal(c, want), (period, prefix)
            assert np.array_equal(oracle_decompress(c, nbytes), raw), (period, prefix)
