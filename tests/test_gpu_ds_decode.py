"""GPU tier: (DELTA, SHUFFLE) chunk decode, both by the separate k_dfilter pass (the default) and
undone inside the decode launch (k_decode finish_block, DChunk::fuse_ds; the C4 pipeline, measured
slower than the separate pass -- DESIGN.md §3; compiled in only with -DB2H_DEC_FUSE_DS_BUILD=1 and
then chosen by B2H_DEC_FUSE_DS=1 -- in a default build the "in-launch" cases check that the variable
is ignored): block 0's completing wave un-shuffles and XOR-scans it, every other block is
un-shuffled and XORed with the final block 0 once that is published (a block that finishes first
parks and is taken exactly once).  Checked against the oracle's chunks decoded on
the CPU (blosc/delta.c:18-161 + blosc/shuffle-generic.h:34-83 restated in oracle/blosc2_oracle.c):
typesizes 2 / 4 / 8, several blocksizes, leftover blocks that do and do not fuse (a leftover that
is not whole quads keeps the chunk on the k_dfilter path), destinations at 16-byte-aligned and at
odd strides (the element loop), and many chunks per batch so blocks race block 0.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu


def _data(ts, nbytes, seed, kind="noisy"):
    """Smooth integer series with noise (LZ, raw and run streams all occur after DELTA+SHUFFLE);
    kind "ramp": C4's int ramp, whose blocks after the first are runs in every plane."""
    rng = np.random.default_rng(seed)
    if kind == "ramp":
        dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[ts]
        return (np.arange(nbytes // ts, dtype=np.uint64) + seed * 1000003).astype(dt).view(np.uint8)[:nbytes]
    n = nbytes // ts
    dt = {2: np.uint16, 4: np.uint32, 8: np.uint64}[ts]
    base = np.cumsum(rng.integers(0, 3, n)).astype(dt)
    noise = rng.integers(0, 4, n).astype(dt) * (rng.random(n) < 0.2)
    return (base + noise).view(np.uint8)[:nbytes]


@pytest.mark.parametrize("ts,blocksize,nbytes", [
    (8, 65536, 6 * 65536 + 32 * 100),     # leftover of whole quads: fused
    (4, 16384, 9 * 16384),                # no leftover
    (2, 32768, 3 * 32768 + 8 * 77),       # leftover of whole quads (8-byte quads at ts 2)
    (8, 65536, 2 * 65536 + 8 * 5),        # leftover NOT whole quads: the k_dfilter path
])
@pytest.mark.parametrize("align", [0, 3])
@pytest.mark.parametrize("fused", ["1", "0"], ids=["in-launch", "k_dfilter"])
@pytest.mark.parametrize("kind", ["noisy", "ramp"])
def test_gpu_fused_delta_shuffle_decode(ts, blocksize, nbytes, align, fused, kind, monkeypatch):
    import torch
    monkeypatch.setenv("B2H_DEC_FUSE_DS", fused)
    import blosc2_amd as B
    from oracle_lib import oracle_compress, oracle_decompress
    kw = dict(clevel=5, typesize=ts, filters=(0, 0, 0, 0, 3, 1), blocksize=blocksize)
    nch = 48
    raws = [_data(ts, nbytes, 100 * ts + i, kind) for i in range(nch)]
    chunks = [oracle_compress(r, **kw) for r in raws]
    for c, r in zip(chunks, raws):
        assert isinstance(c, np.ndarray) and np.array_equal(oracle_decompress(c, nbytes), r)
    sstride = max(c.nbytes for c in chunks) + 256
    host = np.zeros(nch * sstride, np.uint8)
    cbytes = np.zeros(nch, np.int32)
    for i, c in enumerate(chunks):
        host[i * sstride:i * sstride + c.nbytes] = c
        cbytes[i] = c.nbytes
    dsrc = torch.from_numpy(host).cuda()
    dcb = torch.from_numpy(cbytes).cuda()
    dstride = (nbytes + 255) // 256 * 256 + align   # align 3: every chunk but the first at an odd address
    dout = torch.zeros(nch * dstride + 64, dtype=torch.uint8, device="cuda")
    st = torch.zeros(nch, dtype=torch.int32, device="cuda")
    B.decompress_batch(dsrc.data_ptr(), sstride, dcb.data_ptr(), nch, dout.data_ptr(), dstride, nbytes, st.data_ptr())
    torch.cuda.synchronize()
    assert (st.cpu().numpy() == nbytes).all(), st.cpu().numpy()
    back = dout.cpu().numpy()
    for i, r in enumerate(raws):
        assert np.array_equal(back[i * dstride:i * dstride + nbytes], r), i
    # the single-chunk host path (blosc2_decompress_ctx) decodes the same bytes
    got = B.decompress(chunks[0], nbytes)
    assert np.array_equal(np.asarray(got).view(np.uint8).reshape(-1)[:nbytes], raws[0])


@pytest.mark.parametrize("splitmode", [1, 2], ids=["always", "never"])
@pytest.mark.parametrize("kind", ["noisy", "ramp"])
def test_gpu_ds_run_planes_masks_and_items(splitmode, kind):
    """k_decode leaves the run streams of (DELTA, SHUFFLE) chunks unstaged and k_dfilter reads their
    planes as the csize word's byte (DChunk::ds_runs): whole chunks, masked
    blocks (the caller's bytes stay), getitem and decompress_block (each block un-deltaed against
    itself) and an unsplit chunk (one stream per block) agree with the oracle / the reference."""
    import ctypes as C
    import blosc2_amd as B
    from oracle_lib import oracle_compress, oracle_decompress, ref
    ts, bs, nbytes = 8, 65536, 5 * 65536 + 8 * 100
    raw = _data(ts, nbytes, 7, kind)
    kw = dict(clevel=5, typesize=ts, filters=(0, 0, 0, 0, 3, 1), blocksize=bs, splitmode=splitmode)
    chunk = oracle_compress(raw, **kw)
    assert np.array_equal(oracle_decompress(chunk, nbytes), raw)
    assert np.array_equal(np.asarray(B.decompress(chunk, nbytes)).view(np.uint8).reshape(-1)[:nbytes], raw)
    L = B.lib()
    nblocks = -(-nbytes // bs)
    mask = np.array([b % 2 == 1 for b in range(nblocks)], np.bool_)
    ctx = L.blosc2_create_dctx(B.dparams())
    L.blosc2_set_maskout.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    assert L.blosc2_set_maskout(ctx, mask.ctypes.data, nblocks) == 0
    out = np.full(nbytes, 0x5A, np.uint8)
    assert L.blosc2_decompress_ctx(ctx, chunk.ctypes.data, chunk.nbytes, out.ctypes.data, nbytes) == nbytes
    for b in range(nblocks):
        lo, hi = b * bs, min(nbytes, (b + 1) * bs)
        want = np.full(hi - lo, 0x5A, np.uint8) if mask[b] else raw[lo:hi]
        assert np.array_equal(out[lo:hi], want), b
    R = ref()
    if R is not None:
        vp = C.c_void_p
        for lib in (L, R):
            lib.blosc2_decompress_block_ctx.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, C.c_int32]
        rctx = R.blosc2_create_dctx(__import__("b2ctypes").dparams())
        for b in range(nblocks):
            g, r = np.zeros(bs, np.uint8), np.zeros(bs, np.uint8)
            ng = L.blosc2_decompress_block_ctx(ctx, chunk.ctypes.data, chunk.nbytes, b, g.ctypes.data, bs)
            nr = R.blosc2_decompress_block_ctx(rctx, chunk.ctypes.data, chunk.nbytes, b, r.ctypes.data, bs)
            assert ng == nr and np.array_equal(g, r), b
        for start, nitems in ((5, 9000), (8191, 2), (0, nbytes // ts)):
            g, r = np.zeros(nitems * ts, np.uint8), np.zeros(nitems * ts, np.uint8)
            ng = L.blosc2_getitem_ctx(ctx, chunk.ctypes.data, chunk.nbytes, start, nitems, g.ctypes.data, g.nbytes)
            nr = R.blosc2_getitem_ctx(rctx, chunk.ctypes.data, chunk.nbytes, start, nitems, r.ctypes.data, r.nbytes)
            assert ng == nr and np.array_equal(g, r), (start, nitems)
        R.blosc2_free_ctx(rctx)
    L.blosc2_free_ctx(ctx)
