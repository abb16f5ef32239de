"""The north_star's end-to-end read path on one MI355X, from a frame FILE: the T workload (1024 x
4 MiB float32 chunks, SHUFFLE + BloscLZ clevel 5) written as a contiguous frame with
blosc2_schunk_to_file, then read back through the reference's entry points --

  open+host    blosc2_schunk_open (filesystem backend, lazy) + b2h_schunk_decompress_buffers of
               every chunk into a pageable host buffer (the C caller's drop-in for the loop of
               blosc2_schunk_decompress_chunk, blosc/schunk.c:1481-1530);
  open+hbm     blosc2_schunk_open + b2h_schunk_decompress_device of every chunk (64-chunk groups)
               into HBM;
  frame+hbm    b2h_frame_open (whole file into pinned memory, one H2D) + b2h_frame_decompress;
  mmap+host    blosc2_schunk_open_udio with the memory-mapped backend + decompress_buffers;

each timed warm (file in the page cache) and cold (pages dropped with posix_fadvise DONTNEED
after an fsync: the disk's own rate).  Also the host-to-host fan-out on the in-memory super-chunk
(b2h_schunk_append_buffers / _decompress_buffers, pageable buffers).  Every read is checked
against the source.  One JSON line per measurement.

    python tools/frame_e2e.py [--chunks 1024] [--dir /tmp] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
sys.path.insert(0, REPO)
import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

GiB = float(1 << 30)
CHUNK = 4 << 20


def drop_cache(path):
    fd = os.open(path, os.O_RDONLY)
    try:
        os.fsync(fd)
        os.posix_fadvise(fd, 0, 0, os.POSIX_FADV_DONTNEED)
    finally:
        os.close(fd)


def emit(name, nbytes, secs, **kw):
    print(json.dumps({"measure": name, "GiB_per_s": round(nbytes / GiB / secs, 2), "seconds": round(secs, 4),
                      "bytes": nbytes, **kw}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    n = a.chunks
    N = n * CHUNK
    L = B.bind_schunk(B.lib())
    dev = torch.device("cuda")
    src = gen_f32_device(0, N // 4, dev).view(torch.uint8).cpu().numpy()   # pageable host input
    out = np.empty(N, np.uint8)
    out.fill(0)   # pre-faulted
    st = np.zeros(n, np.int32)
    sizes = np.full(n, CHUNK, np.int32)
    cp = B.cparams(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, B.SHUFFLE))

    # host-to-host fan-out on an in-memory super-chunk (1 GPU)
    best_c = best_d = 1e9
    sc = None
    for r in range(a.reps):
        if sc is not None:
            sc.free()
        sc = B.SChunk(cp, L=L)
        t0 = time.perf_counter()
        got = L.b2h_schunk_append_buffers(sc.p, src.ctypes.data, sizes.ctypes.data, n, CHUNK, 0)
        best_c = min(best_c, time.perf_counter() - t0)
        assert got == n, got
        t0 = time.perf_counter()
        rc = L.b2h_schunk_decompress_buffers(sc.p, 0, n, out.ctypes.data, CHUNK, CHUNK, st.ctypes.data, 0)
        best_d = min(best_d, time.perf_counter() - t0)
        assert rc == 0 and (st == CHUNK).all() and np.array_equal(out, src)
        out[:CHUNK] = 0
    cbytes = sc.s.cbytes
    emit("fanout_compress_host_to_host", N, best_c, ratio=round(N / cbytes, 3))
    emit("fanout_decompress_host_to_host", N, best_d)

    # the frame file
    path = os.path.join(a.dir, "t_e2e.b2frame")
    t0 = time.perf_counter()
    flen = L.blosc2_schunk_to_file(sc.p, path.encode())
    tw = time.perf_counter() - t0
    assert flen == os.path.getsize(path)
    emit("schunk_to_file", flen, tw, frame_bytes=flen)
    sc.free()

    def check():
        assert (st == CHUNK).all(), st[:8]
        assert np.array_equal(out, src)
        out[:CHUNK] = 0

    def open_host(io=None):
        p = L.blosc2_schunk_open_udio(path.encode(), C.byref(io)) if io else L.blosc2_schunk_open(path.encode())
        assert p
        s = B.SChunk.wrap(p, L)
        rc = L.b2h_schunk_decompress_buffers(s.p, 0, n, out.ctypes.data, CHUNK, CHUNK, st.ctypes.data, 0)
        s.free()
        assert rc == 0, rc

    d_out = torch.empty(N, dtype=torch.uint8, device=dev)

    def open_hbm():
        p = L.blosc2_schunk_open(path.encode())
        assert p
        s = B.SChunk.wrap(p, L)
        for g in range(0, n, 64):
            m = min(64, n - g)
            rc = L.b2h_schunk_decompress_device(s.p, g, m, d_out.data_ptr() + g * CHUNK, CHUNK, CHUNK,
                                                st[g:].ctypes.data)
            assert rc == 0, rc
        torch.cuda.synchronize()
        s.free()

    L.b2h_frame_open.argtypes, L.b2h_frame_open.restype = [C.c_char_p, C.POINTER(C.c_int)], C.c_void_p
    L.b2h_frame_decompress.argtypes, L.b2h_frame_decompress.restype = [C.c_void_p, C.c_void_p, C.c_int64], C.c_int64
    L.b2h_frame_free.argtypes = [C.c_void_p]

    def frame_hbm():
        err = C.c_int(0)
        f = L.b2h_frame_open(path.encode(), C.byref(err))
        assert f, err.value
        got = L.b2h_frame_decompress(f, d_out.data_ptr(), N)
        L.b2h_frame_free(f)
        assert got == N, got

    def hbm_check():
        assert torch.equal(d_out[:1 << 20].cpu(), torch.from_numpy(src[:1 << 20]))
        assert torch.equal(d_out[-(1 << 20):].cpu(), torch.from_numpy(src[-(1 << 20):]))
        d_out[:CHUNK].zero_()

    mm = []

    def mmap_host():
        m = B.StdioMmap.defaults(b"r")
        mm.append(m)
        io = B.IO(1, b"filesystem_mmap", C.cast(C.pointer(m), C.c_void_p))
        open_host(io)

    for name, fn, chk in (("open+host", open_host, check), ("open+hbm", open_hbm, hbm_check),
                          ("frame+hbm", frame_hbm, hbm_check), ("mmap+host", mmap_host, check)):
        for cold in (True, False):
            best = 1e9
            for r in range(a.reps if not cold else 1):
                if cold:
                    drop_cache(path)
                t0 = time.perf_counter()
                fn()
                best = min(best, time.perf_counter() - t0)
                chk()
            emit("frame_file_" + name, N, best, cache="cold" if cold else "warm", frame_bytes=flen,
                 disk_GiB_per_s=round(flen / GiB / best, 2))
    os.remove(path)


if __name__ == "__main__":
    main()
