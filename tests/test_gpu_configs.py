"""GPU tier: every configuration of BASELINE.json by name, each through the
C-ABI of the MI355X engine and checked against the reference library built from its own sources
(oracle/_ref; the oracle restatement when _ref is absent).

  C1  bench/b2bench.c blosclz shuffle, typesize 4, 1e6 int32 get_value(i, 19) (b2bench.c:73-81)
  C2  shuffle filter only, typesize 4, 256 MiB float32 gen_f32, bit-exact vs shuffle-generic.c
  C3  bitshuffle + blosclz clevel 5, 256 KiB blocks = 256 KiB chunks (one block, one stream)
  C4  DELTA + SHUFFLE + blosclz clevel 5, typesize 8, int64 ramp, 1 MiB chunks, a super-chunk
      appended in one device batch with a ragged last chunk (blosc/schunk.c:1459-1477)
  C5  C4 sharded over ranks by the multi-GPU chunk scheduler (c-blosc2_amd/schunk_dist.py)

Bars: exact mode byte-identical per chunk to the reference (nthreads = 1); fast mode decoded by
the reference's own decoder back to the input, with the ratio tolerances stated below.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from datagen import b2bench_values, gen_f32, int64_ramp
from oracle_lib import oracle, oracle_compress, oracle_decompress, p, ref, ref_compress

pytestmark = pytest.mark.gpu

# Fast mode's ratio tolerances vs exact mode (= the reference's ratio), per configuration.
# T is gated in tests/test_fast_mode.py::test_gpu_fast_ratio_T and in bench.py.
C3_FAST_RATIO_TOL = 0.0025   # fast >= exact * (1 - 0.25 %)   (256 KiB streams, 2^13-entry table)


@pytest.fixture(scope="module")
def B():
    import torch  # noqa: F401  (torch's HIP runtime first, then the engine)
    import blosc2_amd
    assert blosc2_amd.lib().b2h_device_count() > 0
    return blosc2_amd


def _want(src, **kw):
    """The reference's chunk (its library built here), else the oracle's."""
    return ref_compress(src, **kw) if ref() is not None else oracle_compress(src, **kw)


def _decode_ref(chunk, nbytes):
    R = ref()
    if R is None:
        return oracle_decompress(chunk, nbytes)
    out = np.zeros(max(nbytes, 1), np.uint8)
    n = R.blosc2_decompress(p(chunk), chunk.nbytes, p(out), nbytes)
    return out[:nbytes] if n == nbytes else n


def _batch(B, kw, raw, sizes, mode=None):
    """Compress chunks of `sizes` (host) from `raw` through b2h_compress_batch_sizes, decompress
    them with b2h_decompress_batch; returns (chunks, restored host bytes)."""
    import torch
    stride = max(sizes) + 256
    off = np.concatenate([[0], np.cumsum(sizes)])
    host = np.zeros(len(sizes) * stride, np.uint8)
    for i, n in enumerate(sizes):
        host[i * stride:i * stride + n] = raw[off[i]:off[i + 1]]
    dsrc = torch.from_numpy(host).cuda()
    ddst = torch.zeros_like(dsrc)
    dcb = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    B.compress_batch_sizes(B.cparams(**kw, lz_mode=mode), dsrc.data_ptr(), list(sizes), stride, ddst.data_ptr(),
                           stride, 0, dcb.data_ptr())
    torch.cuda.synchronize()
    cb = dcb.cpu().numpy()
    assert (cb > 0).all(), cb.min()
    out = ddst.cpu().numpy()
    chunks = [out[i * stride:i * stride + cb[i]].copy() for i in range(len(sizes))]
    dout = torch.zeros(len(sizes) * stride, dtype=torch.uint8, device="cuda")
    dst = torch.zeros(len(sizes), dtype=torch.int32, device="cuda")
    B.decompress_batch(ddst.data_ptr(), stride, dcb.data_ptr(), len(sizes), dout.data_ptr(), stride, max(sizes),
                       dst.data_ptr())
    torch.cuda.synchronize()
    assert list(dst.cpu().numpy()) == list(sizes)
    back = dout.cpu().numpy()
    restored = np.concatenate([back[i * stride:i * stride + n] for i, n in enumerate(sizes)])
    return chunks, restored


# ------------------------------------------------------------------------------- C1 ----
def test_C1_b2bench_blosclz_shuffle_clevel5(B):
    """C1 as b2bench runs it (bench/b2bench.c:199, 227): blosc1_compress(5, SHUFFLE, 4, ...) of the
    1e6 int32 get_value(i, 19) buffer -- byte-identical to the reference, ratio 20.59, and the same
    bytes through the device batch path (4 MB chunks of the b2bench working set)."""
    L = B.lib()
    src = b2bench_values(1_000_000, 19)
    L.blosc1_set_compressor(b"blosclz")
    out = np.zeros(src.nbytes + 32, np.uint8)
    n = L.blosc1_compress(5, 1, 4, src.nbytes, B._p(src), B._p(out), src.nbytes + 32)
    want = _want(src, clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1))
    assert n == want.nbytes and np.array_equal(out[:n], want)
    assert abs(src.nbytes / n - 20.59) < 0.01
    raw = np.tile(src.view(np.uint8), 4)
    chunks, back = _batch(B, dict(clevel=5, typesize=4), raw, [src.nbytes] * 4, mode=0)
    for c in chunks:
        assert np.array_equal(c, want)
    assert np.array_equal(back, raw)


# ------------------------------------------------------------------------------- C2 ----
def test_C2_shuffle_256mib_bit_exact(B):
    """C2: blosc2_shuffle(4, 256 MiB) of gen_f32 through the drop-in, bit-exact vs the oracle's
    shuffle_generic restatement (blosc/shuffle-generic.h:34-55); unshuffle restores the input."""
    L, O = B.lib(), oracle()
    n = 256 << 20
    src = gen_f32(0, n // 4)
    got = np.empty(n, np.uint8)
    assert L.blosc2_shuffle(4, n, B._p(src), B._p(got)) == n
    want = np.empty(n, np.uint8)
    assert O.or_shuffle(4, n, p(src), p(want)) == n
    assert np.array_equal(got, want)
    back = np.empty(n, np.uint8)
    assert L.blosc2_unshuffle(4, n, B._p(got), B._p(back)) == n
    assert np.array_equal(back, src.view(np.uint8))


# ------------------------------------------------------------------------------- C3 ----
C3_KW = dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 2), blocksize=262144)
C3_CHUNKS = 256


def _c3_raw():
    return gen_f32(0, C3_CHUNKS * 65536).view(np.uint8)   # continuing global index


def test_C3_bitshuffle_blosclz_batch_exact_vs_reference(B):
    """C3 shape: 256 chunks x 256 KiB (one block, one stream each: bitshuffle never splits,
    blosc/stune.c:212) in one device batch, exact mode: every chunk byte-identical to the
    reference's, the reference's ratio (1.775 on this data), exact round trip."""
    raw = _c3_raw()
    chunks, back = _batch(B, C3_KW, raw, [262144] * C3_CHUNKS, mode=0)
    assert np.array_equal(back, raw)
    for i in range(C3_CHUNKS):
        want = _want(raw[i * 262144:(i + 1) * 262144].view(np.float32), **C3_KW)
        assert np.array_equal(chunks[i], want), i
    ratio = raw.nbytes / sum(c.nbytes for c in chunks)
    assert abs(ratio - 1.775) < 0.005, ratio


def test_C3_bitshuffle_blosclz_fast_mode_ratio_gate(B):
    """C3 in fast mode: every chunk decoded by the reference's decoder back to the input, and the
    ratio within C3_FAST_RATIO_TOL of exact mode's."""
    raw = _c3_raw()
    fast, back = _batch(B, C3_KW, raw, [262144] * C3_CHUNKS, mode=1)
    assert np.array_equal(back, raw)
    for i in range(0, C3_CHUNKS, 7):
        assert np.array_equal(_decode_ref(fast[i], 262144), raw[i * 262144:(i + 1) * 262144]), i
    exact, _ = _batch(B, C3_KW, raw, [262144] * C3_CHUNKS, mode=0)
    rf = raw.nbytes / sum(c.nbytes for c in fast)
    re = raw.nbytes / sum(c.nbytes for c in exact)
    assert rf >= re * (1 - C3_FAST_RATIO_TOL), (rf, re)


# ------------------------------------------------------------------------------- C4 ----
C4_KW = dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))
C4_CHUNK = 1 << 20


def test_C4_delta_shuffle_schunk_ragged_batch_vs_reference(B):
    """C4 shape: a super-chunk of 512 full 1 MiB chunks + a ragged last chunk of the int64 ramp,
    DELTA + SHUFFLE ts 8 clevel 5, appended in ONE b2h_compress_batch_sizes call (destsize
    nbytes + 32 each, as blosc2_schunk_append_buffer, blosc/schunk.c:1459-1477): every chunk
    byte-identical to the reference's, exact round trip through b2h_decompress_batch."""
    sizes = [C4_CHUNK] * 512 + [8 * 12_345]
    raw = int64_ramp(0, sum(sizes) // 8).view(np.uint8)
    chunks, back = _batch(B, C4_KW, raw, sizes, mode=0)
    assert np.array_equal(back, raw)
    off = 0
    for i, n in enumerate(sizes):
        want = _want(raw[off:off + n].view(np.int64), **C4_KW)
        assert np.array_equal(chunks[i], want), i
        off += n
    ratio = raw.nbytes / sum(c.nbytes for c in chunks)
    assert ratio > 700, ratio


# ------------------------------------------------------------------------------- C5 ----
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _c5_worker(rank, world, port, backend, nchunks, q):
    import torch
    import torch.distributed as dist
    import schunk_dist as SD
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.from_numpy(int64_ramp(0, nchunks * C4_CHUNK // 8).view(np.uint8)).to(dev) if rank == 0 else None
        comp, decomp = SD.device_engine(C4_KW)
        res = SD.compress_schunk(full, C4_CHUNK, nchunks, C4_KW, dev, comp)
        frame, offsets = res if rank == 0 else (None, None)
        back = SD.decompress_schunk(frame, offsets, C4_CHUNK, nchunks, dev, decomp)
        torch.cuda.synchronize()
        if rank == 0:
            q.put(("ok", frame.cpu().numpy(), offsets.cpu().numpy(), bool(torch.equal(back, full))))
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("backend,world,nchunks", [("gloo", 2, 33), ("nccl", 1, 16)])
def test_C5_sharded_schunk_hip_engine(B, backend, world, nchunks):
    """C5's path: the C4 super-chunk sharded in contiguous chunk ranges over `world` ranks (gloo:
    two ranks sharing the box's one GPU; nccl = RCCL), one engine batch per rank, gathered in
    chunk order on rank 0 -- the frame equals the reference's chunks appended one at a time, and
    the distributed decompression restores the super-chunk."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_worker, args=(r, world, port, backend, nchunks, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    status, frame, offsets, ok = q.get(timeout=100)
    for pr in procs:
        pr.join(timeout=60)
    assert status == "ok", frame
    assert all(pr.exitcode == 0 for pr in procs)
    raw = int64_ramp(0, nchunks * C4_CHUNK // 8)
    expect = [_want(raw[i * C4_CHUNK // 8:(i + 1) * C4_CHUNK // 8], **C4_KW) for i in range(nchunks)]
    assert offsets.tolist() == [0] + list(np.cumsum([e.nbytes for e in expect]))
    assert np.array_equal(frame, np.concatenate(expect))
    assert ok
