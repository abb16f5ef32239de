"""Multi-rank super-chunk scheduler (c-blosc2_amd/schunk_dist.py) on CPU with gloo, world_size 2
and 3 (uneven shards).  The per-rank chunk engine is stood in by the oracle (CPU restatement), so
these tests cover the distribution logic only: shard ranges, padded scatter, variable-size
gather, chunk order and the offsets index.  Expected: the gathered frame equals the chunks the
oracle produces serially, one chunk at a time, exactly as blosc/schunk.c:1459-1477 appends them.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

import schunk_dist as SD  # noqa: E402

CHUNK = 64 * 1024
KW = dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))   # DELTA + SHUFFLE (config C4 shape)


def _data(nchunks):
    from datagen import int64_ramp, gen_f32
    a = int64_ramp(0, nchunks * CHUNK // 8).view(np.uint8).copy()
    # make a few chunks incompressible-ish so chunk sizes differ widely
    b = gen_f32(0, CHUNK // 4).view(np.uint8)
    for i in range(1, nchunks, 3):
        a[i * CHUNK:(i + 1) * CHUNK] = b
    return a


def _oracle_compress_batch(cparams, src, chunk_nbytes, n, comp, stride, cap, cbytes):
    import oracle_lib
    s = src.numpy()
    for i in range(n):
        out = oracle_lib.oracle_compress(s[i * chunk_nbytes:(i + 1) * chunk_nbytes].copy(), **cparams)
        assert not isinstance(out, int) and out.nbytes <= cap
        comp[i * stride:i * stride + out.nbytes] = torch.from_numpy(out.copy())
        cbytes[i] = out.nbytes


def _oracle_decompress_batch(comp, stride, cbytes, n, out, chunk_nbytes):
    import oracle_lib
    c = comp.numpy()
    for i in range(n):
        k = int(cbytes[i])
        dec = oracle_lib.oracle_decompress(c[i * stride:i * stride + k].copy(), chunk_nbytes)
        out[i * chunk_nbytes:(i + 1) * chunk_nbytes] = torch.from_numpy(dec.copy())


def _worker(rank, world, port, nchunks, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        full = torch.from_numpy(_data(nchunks)) if rank == 0 else None
        dev = torch.device("cpu")
        res = SD.compress_schunk(full, CHUNK, nchunks, KW, dev, _oracle_compress_batch)
        if rank == 0:
            frame, offsets = res
        else:
            assert res is None
            frame, offsets = None, None
        back = SD.decompress_schunk(frame, offsets, CHUNK, nchunks, dev, _oracle_decompress_batch)
        if rank == 0:
            q.put(("ok", frame.numpy().copy(), offsets.numpy().copy(), back.numpy().copy()))
        else:
            assert back is None
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,nchunks", [(2, 6), (3, 7), (2, 1)])
def test_schunk_distributed_roundtrip(world, nchunks):
    import oracle_lib
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nchunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, frame, offsets, back = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", frame
    assert all(p.exitcode == 0 for p in procs)
    data = _data(nchunks)
    # serial reference order: one chunk at a time
    expect = [oracle_lib.oracle_compress(data[i * CHUNK:(i + 1) * CHUNK].copy(), **KW) for i in range(nchunks)]
    sizes = [e.nbytes for e in expect]
    assert offsets.tolist() == [0] + list(np.cumsum(sizes))
    assert np.array_equal(frame, np.concatenate(expect))
    assert np.array_equal(back, data)


def test_shard_ranges_cover():
    for n in range(0, 40):
        for w in range(1, 9):
            spans = [SD.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def _failing_worker(rank, world, port, q):
    """Rank 1's chunk engine reports a chunk that did not fit (cbytes 0)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def comp(cparams, src, chunk_nbytes, n, out, stride, cap, cbytes):
        _oracle_compress_batch(cparams, src, chunk_nbytes, n, out, stride, cap, cbytes)
        if rank == 1:
            cbytes[0] = 0
        if rank == 2:
            raise RuntimeError("b2h_compress_batch: -12")

    try:
        full = torch.from_numpy(_data(4)) if rank == 0 else None
        SD.compress_schunk(full, CHUNK, 4, KW, torch.device("cpu"), comp)
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_schunk_failure_on_one_rank_raises_everywhere():
    """a rank whose chunk fails must not leave the others blocked in the gather: the
    failure travels in the gather's size exchange and every rank raises together, well before any
    timeout (rank 1: a chunk of size 0; rank 2: its launch raises)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_failing_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
    for r in range(3):
        assert "compression failed on rank(s) [1, 2]" in got[r], got
