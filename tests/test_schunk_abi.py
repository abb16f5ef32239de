"""CPU tier: the super-chunk layer of the drop-in (include/blosc2.h blosc2_schunk_*,
c-blosc2_amd/csrc/b2h_schunk.cpp) against the reference build (oracle/_ref, blosc/schunk.c).

Everything here is host bookkeeping -- no chunk is compressed or decompressed: the chunks are
header-only special chunks (blosc2_chunk_zeros / repeatval, written on the host) and the
reference's own golden chunks (tests/golden/*.cdata).  Checked: the structs are ABI-identical to the
reference header (offsets compiled by gcc from both headers), and one script of index operations
(append / insert / update / delete, copy and ownership hand-over, the chunksize and VL-block rules,
the error codes) leaves both libraries' super-chunks with the same counters and the same chunks.
The compute side (append_buffer, decompress, slices, device batches) is tests/test_gpu_schunk_api.py.
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np
import pytest

from b2ctypes import REPO

sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
import blosc2_amd as B  # noqa: E402

REF_INC = "/root/reference/include"
GOLD = os.path.join(REPO, "tests", "golden")

LAYOUT_C = r"""
#include <stdio.h>
#include <stddef.h>
#include "blosc2.h"
#define F(T, f) printf(#T "." #f " %zu\n", offsetof(T, f))
#define S(T) printf(#T " %zu\n", sizeof(T))
int main(void) {
  S(blosc2_schunk); F(blosc2_schunk, typesize); F(blosc2_schunk, chunksize); F(blosc2_schunk, flags2);
  F(blosc2_schunk, filters); F(blosc2_schunk, nchunks); F(blosc2_schunk, cbytes); F(blosc2_schunk, data);
  F(blosc2_schunk, data_len); F(blosc2_schunk, storage); F(blosc2_schunk, cctx); F(blosc2_schunk, dctx);
  F(blosc2_schunk, metalayers); F(blosc2_schunk, nmetalayers); F(blosc2_schunk, vlmetalayers);
  F(blosc2_schunk, nvlmetalayers); F(blosc2_schunk, tuner_id); F(blosc2_schunk, ndim);
  F(blosc2_schunk, blockshape); F(blosc2_schunk, view); F(blosc2_schunk, change_tick);
  S(blosc2_storage); F(blosc2_storage, urlpath); F(blosc2_storage, cparams); F(blosc2_storage, io);
  S(blosc2_io); F(blosc2_io, name); F(blosc2_io, params);
  S(blosc2_metalayer); F(blosc2_metalayer, content_len);
  S(blosc2_cparams); F(blosc2_cparams, schunk); F(blosc2_cparams, filters); F(blosc2_cparams, prefilter);
  F(blosc2_cparams, tuner_id); F(blosc2_cparams, codec_params); F(blosc2_cparams, filter_params);
  S(blosc2_dparams); F(blosc2_dparams, postfilter); F(blosc2_dparams, typesize);
  return 0;
}
"""


def _layout(tmp_path, inc, tag):
    src = tmp_path / f"layout_{tag}.c"
    exe = tmp_path / f"layout_{tag}"
    src.write_text(LAYOUT_C)
    # (the reference header defines helpers that call into its library: left unresolved, never run)
    subprocess.check_call(["gcc", "-std=gnu99", "-w", "-O1", f"-I{inc}", str(src), "-o", str(exe),
                           "-Wl,--unresolved-symbols=ignore-all"])
    return dict(line.rsplit(" ", 1) for line in subprocess.check_output([str(exe)], text=True).splitlines())


def test_schunk_structs_abi_identical(tmp_path):
    ours = _layout(tmp_path, os.path.join(REPO, "include"), "ours")
    # the ctypes mirror agrees with the C header
    assert int(ours["blosc2_schunk"]) == C.sizeof(B.Schunk)
    for f in ("nchunks", "cbytes", "data", "storage", "cctx", "nmetalayers", "vlmetalayers", "tuner_id",
              "blockshape", "view", "change_tick"):
        assert int(ours[f"blosc2_schunk.{f}"]) == getattr(B.Schunk, f).offset, f
    assert int(ours["blosc2_storage"]) == C.sizeof(B.Storage)
    if not os.path.isdir(REF_INC):
        pytest.skip("reference headers absent")
    assert ours == _layout(tmp_path, REF_INC, "ref")


def _ref_lib():
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build absent")
    return B.bind_schunk(R)


def _special(L, kind, nbytes, typesize=4, value=7):
    """A header-only chunk written by library L (no device work)."""
    from b2ctypes import CParams as RefCParams, cparams as rcp
    is_ref = not hasattr(L, "b2h_device_count")
    cp = rcp(typesize=typesize) if is_ref else B.cparams(typesize=typesize)
    ctype = RefCParams if is_ref else B.CParams
    out = np.zeros(64, np.uint8)
    if kind == "zeros":
        L.blosc2_chunk_zeros.argtypes = [ctype, C.c_int32, C.c_void_p, C.c_int32]
        n = L.blosc2_chunk_zeros(cp, nbytes, B._p(out), 64)
    else:
        L.blosc2_chunk_repeatval.argtypes = [ctype, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
        v = np.full(typesize, value, np.uint8)
        n = L.blosc2_chunk_repeatval(cp, nbytes, B._p(out), 64, B._p(v))
    assert n > 0
    return out[:n].copy()


def _gold(name):
    return np.fromfile(os.path.join(GOLD, name), np.uint8)


def _new(L, typesize=4):
    from b2ctypes import cparams as rcp, dparams as rdp
    is_ref = not hasattr(L, "b2h_device_count")
    cp = rcp(typesize=typesize) if is_ref else B.cparams(typesize=typesize)
    dp = rdp() if is_ref else B.dparams()
    return B.SChunk(cp, dp, L=L)


def _chunks(sc):
    return [sc.chunk(i) for i in range(sc.s.nchunks)]


def _same(a, b, what):
    ca, cb = a.counters(), b.counters()
    assert ca == cb, (what, ca, cb)
    xa, xb = _chunks(a), _chunks(b)
    assert len(xa) == len(xb)
    for i, (u, v) in enumerate(zip(xa, xb)):
        assert np.array_equal(u, v), (what, i)


def _script(L, ops):
    """Run `ops` on a fresh super-chunk of library L; returns (schunk, [return codes])."""
    sc = _new(L)
    libc = C.CDLL(None)
    libc.malloc.restype, libc.malloc.argtypes = C.c_void_p, [C.c_size_t]
    rcs = []
    for op, *args in ops:
        if op == "append":
            rcs.append(sc.append_chunk(_special(L, *args)))
        elif op == "append_gold":
            rcs.append(sc.append_chunk(_gold(args[0])))
        elif op == "append_owned":   # copy = false: the super-chunk takes (and shrinks) a malloc'd buffer
            c = _special(L, *args)
            buf = libc.malloc(1 << 16)
            C.memmove(buf, c.ctypes.data, c.nbytes)
            rcs.append(L.blosc2_schunk_append_chunk(sc.p, C.c_void_p(buf), False))
        elif op == "insert":
            rcs.append(sc.insert_chunk(args[0], _special(L, *args[1:])))
        elif op == "update":
            rcs.append(sc.update_chunk(args[0], _special(L, *args[1:])))
        elif op == "update_gold":
            rcs.append(sc.update_chunk(args[0], _gold(args[1])))
        elif op == "delete":
            rcs.append(sc.delete_chunk(args[0]))
        elif op == "append_raw":
            rcs.append(sc.append_chunk(args[0]))
        rcs.append(sc.counters())
    return sc, rcs


SCRIPTS = {
    "fixed_then_short_then_variable": [
        ("append", "zeros", 4000), ("append", "repeat", 4000), ("append", "zeros", 1000),
        ("append", "zeros", 4000), ("insert", 1, "repeat", 4000), ("delete", 0), ("delete", 3),
        ("update", 0, "zeros", 4000)],
    "bigger_chunk_goes_variable": [
        ("append", "zeros", 4096), ("append", "zeros", 4096), ("append", "repeat", 8192),
        ("append", "zeros", 100)],
    "insert_irregular_in_the_middle": [
        ("append", "zeros", 4096), ("append", "zeros", 4096), ("insert", 1, "zeros", 2048)],
    "update_irregular": [
        ("append", "zeros", 4096), ("append", "zeros", 4096), ("append", "zeros", 4096),
        ("update", 1, "repeat", 1024), ("update", 2, "zeros", 4096)],
    "update_last_smaller_keeps_fixed": [
        ("append", "zeros", 4096), ("append", "zeros", 4096), ("update", 1, "zeros", 1000),
        ("append", "zeros", 4096)],
    "emptied_then_bigger_is_refused": [
        ("append", "zeros", 4096), ("delete", 0), ("append", "zeros", 8192), ("append", "zeros", 4096)],
    "golden_chunks": [
        ("append_gold", "blosc-blosclz-3.0.0.cdata"), ("append_gold", "blosc-lz4-3.0.0.cdata"),
        ("update_gold", 0, "blosc-1.14.0-blosclz.cdata"), ("append", "zeros", 124), ("delete", 1)],
    "owned_buffers": [
        ("append_owned", "zeros", 4096), ("append_owned", "repeat", 4096), ("append", "zeros", 4096)],
    "out_of_range": [
        ("append", "zeros", 64), ("insert", 3, "zeros", 64), ("insert", -1, "zeros", 64),
        ("update", 1, "zeros", 64), ("delete", 5), ("delete", -2), ("insert", 1, "zeros", 64)],
}


@pytest.mark.parametrize("name", sorted(SCRIPTS))
def test_schunk_index_ops_match_reference(name):
    R = _ref_lib()
    L = B.lib()
    a, ra = _script(L, SCRIPTS[name])
    b, rb = _script(R, SCRIPTS[name])
    try:
        assert ra == rb
        _same(a, b, name)
    finally:
        a.free()
        b.free()


def test_schunk_vl_block_chunks_do_not_mix():
    """A chunk whose flags2 carries BLOSC2_VL_BLOCKS is refused next to regular chunks
    (schunk.c:985-997): same codes, same state."""
    R = _ref_lib()
    L = B.lib()
    out = []
    for lib in (L, R):
        gold = _gold("blosc-blosclz-3.0.0.cdata")
        vl = _special(lib, "repeat", 4096)
        vl[2] |= 0x5                 # extended header announced (both shuffle bits) ...
        vl[0x1e] |= 0x1              # ... carrying the VL-block flag
        vl[0x1f] &= 0x0F             # and no special kind (VL + special is an invalid header)
        sc = _new(lib)
        codes = [sc.append_chunk(gold), sc.append_chunk(vl), sc.insert_chunk(0, vl), sc.counters()]
        out.append((codes, _chunks(sc)))
        sc.free()
    assert out[0][0] == out[1][0]
    assert all(np.array_equal(u, v) for u, v in zip(out[0][1], out[1][1]))


def test_schunk_params_getters_match_reference():
    R = _ref_lib()
    L = B.lib()
    got = []
    for lib in (L, R):
        sc = _new(lib, typesize=8)
        cpp, dpp = C.c_void_p(), C.c_void_p()
        assert lib.blosc2_schunk_get_cparams(sc.p, C.byref(cpp)) == 0
        assert lib.blosc2_schunk_get_dparams(sc.p, C.byref(dpp)) == 0
        cp = C.cast(cpp, C.POINTER(B.CParams)).contents
        dp = C.cast(dpp, C.POINTER(B.DParams)).contents
        got.append((cp.clevel, cp.typesize, cp.compcode, cp.blocksize, cp.splitmode, list(cp.filters),
                    cp.nthreads, cp.schunk == C.cast(sc.p, C.c_void_p).value, dp.nthreads,
                    dp.schunk == C.cast(sc.p, C.c_void_p).value))
        libc = C.CDLL(None)
        libc.free.argtypes = [C.c_void_p]
        libc.free(cpp)
        libc.free(dpp)
        sc.free()
    assert got[0] == got[1]


def test_schunk_new_refuses_frame_storage():
    """Frame-backed storage is outside the device engine: NULL, not a silent in-memory schunk."""
    L = B.lib()
    st = B.Storage(True, None, None, None, None)
    assert not L.blosc2_schunk_new(C.byref(st))
    st = B.Storage(False, b"/tmp/b2h_never_created.b2frame", None, None, None)
    assert not L.blosc2_schunk_new(C.byref(st))
    # defaults: NULL storage members take the library defaults (frame.c:2847-2874)
    sc = L.blosc2_schunk_new(C.byref(B.Storage(False, None, None, None, None)))
    assert sc and sc.contents.typesize == 8 and sc.contents.clevel == 5 and sc.contents.chunksize == -1
    L.blosc2_schunk_free(sc)
