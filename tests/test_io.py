"""CPU tier: the IO backend registry and the built-in backends (host code only, b2h_io.cpp).

The registry follows blosc/blosc2.c:6784-6847 (user ids >= BLOSC2_IO_REGISTERED, a known id with
the same name is a no-op, another name an error; ids 0 and 1 are the filesystem and memory-mapped
backends); the filesystem backend follows blosc/blosc2-stdio.c:120-300 (positioned reads and
writes, item counts returned) and is checked against the reference build's own blosc2_stdio_*;
the memory-mapped backend serves the read modes (pointers into the mapping)."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, HERE)

import blosc2_amd as B  # noqa: E402

PLUGIN_IO = -30


def _lib():
    L = B.bind_schunk(B.lib())
    vp, i64 = C.c_void_p, C.c_int64
    for pre in ("blosc2_stdio", "blosc2_stdio_mmap"):
        getattr(L, pre + "_open").argtypes, getattr(L, pre + "_open").restype = [C.c_char_p, C.c_char_p, vp], vp
        getattr(L, pre + "_close").argtypes = [vp]
        getattr(L, pre + "_size").argtypes, getattr(L, pre + "_size").restype = [vp], i64
        getattr(L, pre + "_write").argtypes, getattr(L, pre + "_write").restype = [vp, i64, i64, i64, vp], i64
        getattr(L, pre + "_read").argtypes, getattr(L, pre + "_read").restype = [C.POINTER(vp), i64, i64, i64, vp], i64
        getattr(L, pre + "_truncate").argtypes = [vp, i64]
        getattr(L, pre + "_destroy").argtypes = [vp]
    return L


def _cb(p):
    return C.cast(p, C.POINTER(B.IOCb)).contents


def test_registry_rules():
    L = _lib()
    fs, mm = L.blosc2_get_io_cb(0), L.blosc2_get_io_cb(1)
    assert fs and mm and not L.blosc2_get_io_cb(77)
    assert _cb(fs).name == b"filesystem" and _cb(fs).is_allocation_necessary
    assert _cb(mm).name == b"filesystem_mmap" and not _cb(mm).is_allocation_necessary
    assert L.blosc2_get_io_cb(0) == fs            # registered once

    def mk(i, name):
        c = _cb(fs)
        return B.IOCb(i, name, True, c.open, c.close, c.size, c.write, c.read, c.truncate, c.destroy)
    low = mk(100, b"low")
    assert L.blosc2_register_io_cb(C.byref(low)) == PLUGIN_IO      # ids < 160 are Blosc's
    mine = mk(231, b"mine")
    assert L.blosc2_register_io_cb(C.byref(mine)) == 0
    assert L.blosc2_register_io_cb(C.byref(mine)) == 0             # same id, same name: no-op
    other = mk(231, b"other")
    assert L.blosc2_register_io_cb(C.byref(other)) == PLUGIN_IO    # same id, another name
    got = L.blosc2_get_io_cb(231)
    assert got and _cb(got).name == b"mine"


def test_stdio_backend_matches_reference(tmp_path):
    from oracle_lib import ref
    L = _lib()
    R = ref()
    libs = [("ours", L)]
    if R is not None:
        for fn in ("open", "close", "size", "write", "read", "truncate"):
            f, g = getattr(R, "blosc2_stdio_" + fn), getattr(L, "blosc2_stdio_" + fn)
            f.argtypes, f.restype = g.argtypes, g.restype
        libs.append(("ref", R))
    payload = np.arange(100_000, dtype=np.uint8)
    results = []
    for tag, X in libs:
        path = str(tmp_path / (tag + ".bin")).encode()
        fp = X.blosc2_stdio_open(path, b"wb+", None)
        assert fp
        r = [X.blosc2_stdio_write(payload.ctypes.data, 1, payload.size, 0, fp),
             X.blosc2_stdio_write(payload.ctypes.data, 1000, 10, 200_000, fp),      # past the end: a hole
             X.blosc2_stdio_size(fp)]
        buf = np.zeros(300_000, np.uint8)
        p = C.c_void_p(buf.ctypes.data)
        r.append(X.blosc2_stdio_read(C.byref(p), 1, 50, 209_990, fp))             # short: 10 of 50 items
        r.append(X.blosc2_stdio_read(C.byref(p), 4, 1000, 4, fp))
        r.append(bytes(buf[:4000]))
        r.append(X.blosc2_stdio_truncate(fp, 150_000))
        r.append(X.blosc2_stdio_size(fp))
        r.append(X.blosc2_stdio_read(C.byref(p), 1, 10, 149_995, fp))             # 5 bytes left
        assert X.blosc2_stdio_close(fp) == 0
        results.append(r)
    assert results[0][:3] == [100_000, 10, 210_000]
    assert results[0][3] == 10 and results[0][4] == 1000
    assert results[0][5] == payload[4:4004].tobytes()
    assert results[0][6:] == [0, 150_000, 5]
    if len(results) == 2:
        assert results[0] == results[1]


def test_mmap_backend_reads_in_place(tmp_path):
    L = _lib()
    path = tmp_path / "m.bin"
    data = np.random.default_rng(1).integers(0, 256, 50_000, dtype=np.uint8)
    data.tofile(path)
    m = B.StdioMmap.defaults(b"r")
    fp = L.blosc2_stdio_mmap_open(str(path).encode(), b"r", C.addressof(m))
    assert fp == C.addressof(m) and m.addr and m.file_size == data.size
    assert L.blosc2_stdio_mmap_size(fp) == data.size
    p = C.c_void_p()
    assert L.blosc2_stdio_mmap_read(C.byref(p), 1, 1000, 777, fp) == 1000
    assert p.value == m.addr + 777
    assert np.array_equal(np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), (1000,)), data[777:1777])
    assert L.blosc2_stdio_mmap_read(C.byref(p), 1, 1000, data.size - 10, fp) == 10    # clipped at the end
    assert L.blosc2_stdio_mmap_write(data.ctypes.data, 1, 10, 0, fp) == 0            # read-only
    assert L.blosc2_stdio_mmap_close(fp) == 0 and m.addr                             # mapping stays
    assert L.blosc2_stdio_mmap_destroy(C.addressof(m)) == 0 and not m.addr
    w = B.StdioMmap.defaults(b"w+")
    assert not L.blosc2_stdio_mmap_open(str(path).encode(), b"w+", C.addressof(w))   # writable modes refused
