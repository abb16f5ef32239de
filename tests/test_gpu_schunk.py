"""GPU tier: the multi-GPU super-chunk scheduler (c-blosc2_amd/schunk_dist.py) driving the real HIP
engine (reference fan-out blosc/schunk.c:1459-1530).

The box has one GPU, so the N > 1 path runs with two ranks sharing cuda:0 over gloo (device tensors
staged through host memory), and the RCCL path with one rank; the gloo CPU tests
(tests/test_schunk_dist.py) cover world sizes 2 and 3 of the same code.  Expected: the gathered
frame equals the chunks the oracle produces one at a time, exactly as blosc2_schunk_append_buffer
appends them, and the distributed decompression restores the input.
"""
import os
import socket
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

pytestmark = pytest.mark.gpu

CHUNK = 256 * 1024
KW = dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))   # C4's pipeline (DELTA + SHUFFLE, ts 8)


def _data(nchunks):
    from datagen import int64_ramp, gen_f32
    a = int64_ramp(0, nchunks * CHUNK // 8).view(np.uint8).copy()
    b = gen_f32(0, CHUNK // 4).view(np.uint8)
    for i in range(1, nchunks, 3):       # chunk sizes differ widely
        a[i * CHUNK:(i + 1) * CHUNK] = b
    return a


def _worker(rank, world, port, backend, nchunks, q):
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
        full = torch.from_numpy(_data(nchunks)).to(dev) if rank == 0 else None
        comp, decomp = SD.device_engine(KW)
        res = SD.compress_schunk(full, CHUNK, nchunks, KW, dev, comp)
        frame, offsets = res if rank == 0 else (None, None)
        back = SD.decompress_schunk(frame, offsets, CHUNK, nchunks, dev, decomp)
        torch.cuda.synchronize()
        if rank == 0:
            q.put(("ok", frame.cpu().numpy(), offsets.cpu().numpy(), back.cpu().numpy()))
    except Exception as e:  # report to the parent instead of hanging it
        q.put(("err", repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("backend,world,nchunks", [("nccl", 1, 9), ("gloo", 2, 9), ("gloo", 2, 1)])
def test_schunk_scheduler_with_hip_engine(backend, world, nchunks):
    import torch.multiprocessing as mp
    from oracle_lib import oracle_compress
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, backend, nchunks, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    status, frame, offsets, back = q.get(timeout=100)
    for pr in procs:
        pr.join(timeout=60)
    assert status == "ok", frame
    assert all(pr.exitcode == 0 for pr in procs)
    data = _data(nchunks)
    expect = [oracle_compress(data[i * CHUNK:(i + 1) * CHUNK].copy(), **KW) for i in range(nchunks)]
    assert offsets.tolist() == [0] + list(np.cumsum([e.nbytes for e in expect]))
    assert np.array_equal(frame, np.concatenate(expect))
    assert np.array_equal(back, data)
