"""CPU tier: the C-ABI library loads and exports every entry point include/*.h declares, and the
host-only logic (header inspection, registry rules) behaves like the reference.  No compute calls:
there is no GPU here, and the compute entry points must fail loudly without one."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from b2ctypes import REPO

import sys
sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
import blosc2_amd as B  # noqa: E402

GOLD = os.path.join(REPO, "tests", "golden")


def declared_symbols():
    names = []
    for h in ("blosc2.h", "b2h.h"):
        txt = open(os.path.join(REPO, "include", h)).read()
        names += re.findall(r"^BLOSC_EXPORT[^;(]*?\b(\w+)\s*\(", txt, flags=re.M)
    return sorted(set(names))


def test_all_declared_symbols_exported():
    lib = C.CDLL(B.LIB_PATH)
    names = declared_symbols()
    assert len(names) >= 50
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_header_inspection_matches_reference_fields():
    L = B.lib()
    gold = np.fromfile(os.path.join(GOLD, "blosc-blosclz-3.0.0.cdata"), np.uint8)
    nb, cb, bs = C.c_int32(), C.c_int32(), C.c_int32()
    assert L.blosc2_cbuffer_sizes(B._p(gold), C.byref(nb), C.byref(cb), C.byref(bs)) == 0
    assert (nb.value, cb.value, bs.value) == (4_000_000, 16910, 2 * 1024 * 1024)
    v, vlz = C.c_int(), C.c_int()
    L.blosc2_cbuffer_versions(B._p(gold), C.byref(v), C.byref(vlz))
    assert (v.value, vlz.value) == (5, 1)
    L.blosc2_cbuffer_complib.restype = C.c_char_p
    assert L.blosc2_cbuffer_complib(B._p(gold)) == b"BloscLZ"
    ts, fl = C.c_size_t(), C.c_int()
    L.blosc1_cbuffer_metainfo(B._p(gold), C.byref(ts), C.byref(fl))
    assert (ts.value, fl.value) == (4, 5)
    n = C.c_size_t()
    assert L.blosc1_cbuffer_validate(B._p(gold), C.c_size_t(16910), C.byref(n)) == 0 and n.value == 4_000_000
    assert L.blosc2_get_version_string() == b"3.3.3.dev"


def test_registry_id_rules():
    """blosc2_register_codec/filter only accept user ids >= 160 (blosc/blosc2.c:6680-6737)."""
    L = B.lib()

    class Codec(C.Structure):
        _fields_ = [("compcode", C.c_uint8), ("compname", C.c_char_p), ("complib", C.c_uint8),
                    ("version", C.c_uint8), ("encoder", C.c_void_p), ("decoder", C.c_void_p)]

    class Filter(C.Structure):
        _fields_ = [("id", C.c_uint8), ("name", C.c_char_p), ("version", C.c_uint8),
                    ("forward", C.c_void_p), ("backward", C.c_void_p)]
    assert L.blosc2_register_codec(C.byref(Codec(100, b"low", 0, 1, None, None))) < 0
    assert L.blosc2_register_codec(C.byref(Codec(200, b"mine", 0, 1, None, None))) == 0
    assert L.blosc2_register_filter(C.byref(Filter(40, b"low", 1, None, None))) < 0
    assert L.blosc2_register_filter(C.byref(Filter(201, b"mine", 1, None, None))) == 0
    L.blosc2_compname_to_compcode.argtypes = [C.c_char_p]
    assert L.blosc2_compname_to_compcode(b"mine") == 200
    assert L.blosc2_compname_to_compcode(b"blosclz") == 0


def test_context_params_roundtrip():
    L = B.lib()
    L.blosc2_ctx_get_cparams.argtypes = [C.c_void_p, C.POINTER(B.CParams)]
    cp = B.cparams(clevel=7, typesize=4, filters=(0, 0, 0, 0, 3, 2), blocksize=65536)
    ctx = L.blosc2_create_cctx(cp)
    out = B.CParams()
    assert L.blosc2_ctx_get_cparams(ctx, C.byref(out)) == 0
    assert (out.clevel, out.typesize, out.blocksize, list(out.filters)) == (7, 4, 65536, [0, 0, 0, 0, 3, 2])
    L.blosc2_free_ctx(ctx)
    # an undefined built-in filter id is rejected at context creation (blosc/blosc2.c:6052-6066)
    assert L.blosc2_create_cctx(B.cparams(filters=(0, 0, 0, 0, 0, 7))) is None


@pytest.mark.skipif(B.lib().b2h_device_count() > 0, reason="a GPU is present")
def test_no_gpu_fails_loudly():
    """Without a GPU the compute entry points return an error: there is no CPU fallback."""
    L = B.lib()
    src = np.arange(1000, dtype=np.int32)
    ctx = L.blosc2_create_cctx(B.cparams(typesize=4))
    out = np.zeros(src.nbytes + 64, np.uint8)
    assert L.blosc2_compress_ctx(ctx, B._p(src), src.nbytes, B._p(out), out.nbytes) < 0
    L.blosc2_free_ctx(ctx)


@pytest.mark.parametrize("ts,nbytes,blocksize", [(4, 4 << 20, 0), (8, 1 << 20, 0), (4, 40, 0), (8, 0, 0),
                                                 (2, 1000, 256), (16, 1 << 16, 0)])
def test_special_chunk_creators_match_reference(ts, nbytes, blocksize):
    """blosc2_chunk_zeros/nans/uninit/repeatval are header-only (blosc/blosc2.c:6452-6637): the
    drop-in writes the same bytes as the reference build (host logic, no GPU involved)."""
    from oracle_lib import ref
    from b2ctypes import CParams as RefCParams, cparams as rcp
    R = ref()
    if R is None:
        pytest.skip("reference build absent")
    L = B.lib()
    val = np.arange(3, ts + 3, dtype=np.uint8)
    for lib, ctype, mk in ((L, B.CParams, lambda: B.cparams(typesize=ts, blocksize=blocksize)),
                           (R, RefCParams, lambda: rcp(typesize=ts, blocksize=blocksize))):
        for fn in ("blosc2_chunk_zeros", "blosc2_chunk_nans", "blosc2_chunk_uninit"):
            getattr(lib, fn).argtypes = [ctype, C.c_int32, C.c_void_p, C.c_int32]
        lib.blosc2_chunk_repeatval.argtypes = [ctype, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    for fn in ("blosc2_chunk_zeros", "blosc2_chunk_nans", "blosc2_chunk_uninit", "blosc2_chunk_repeatval"):
        extra = (C.c_void_p(val.ctypes.data),) if fn.endswith("repeatval") else ()
        a, b = np.zeros(64, np.uint8), np.zeros(64, np.uint8)
        na = getattr(L, fn)(B.cparams(typesize=ts, blocksize=blocksize), nbytes, C.c_void_p(a.ctypes.data), 64, *extra)
        nb = getattr(R, fn)(rcp(typesize=ts, blocksize=blocksize), nbytes, C.c_void_p(b.ctypes.data), 64, *extra)
        assert na == nb, (fn, na, nb)
        assert np.array_equal(a, b), fn
    # too-small destination and ragged nbytes are refused the same way
    for fn in ("blosc2_chunk_nans", "blosc2_chunk_uninit"):
        a = np.zeros(64, np.uint8)
        assert getattr(L, fn)(B.cparams(typesize=ts), nbytes + (1 if ts > 1 else 0), C.c_void_p(a.ctypes.data), 64) == \
            (getattr(R, fn)(rcp(typesize=ts), nbytes + (1 if ts > 1 else 0), C.c_void_p(a.ctypes.data), 64))
        assert getattr(L, fn)(B.cparams(typesize=ts), nbytes, C.c_void_p(a.ctypes.data), 31) == \
            getattr(R, fn)(rcp(typesize=ts), nbytes, C.c_void_p(a.ctypes.data), 31)


def test_error_strings_match_reference():
    """blosc2_error_string (reference blosc/blosc2.c:6916-6995) for every BLOSC2_ERROR_* code and
    a few codes outside the table; print_error is the header-inline alias (include/blosc2.h)."""
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build absent")
    L = B.lib()
    for lib in (L, R):
        lib.blosc2_error_string.argtypes, lib.blosc2_error_string.restype = [C.c_int], C.c_char_p
    for code in range(-45, 3):
        assert L.blosc2_error_string(code) == R.blosc2_error_string(code), code
    assert L.blosc2_error_string(-37) == b"Frame lock failure"
    assert L.blosc2_error_string(0) == b"Unknown error"


def test_timestamp_helpers_match_reference():
    """blosc_set_timestamp / blosc_elapsed_nsecs / blosc_elapsed_secs (reference
    include/blosc2.h:2600-2636, blosc/timestamp.c) on a struct timespec."""
    from oracle_lib import ref
    R = ref()
    if R is None:
        pytest.skip("reference build absent")

    class TS(C.Structure):
        _fields_ = [("tv_sec", C.c_long), ("tv_nsec", C.c_long)]
    L = B.lib()
    for lib in (L, R):
        lib.blosc_set_timestamp.argtypes, lib.blosc_set_timestamp.restype = [C.POINTER(TS)], None
        for fn in ("blosc_elapsed_nsecs", "blosc_elapsed_secs"):
            getattr(lib, fn).argtypes, getattr(lib, fn).restype = [TS, TS], C.c_double
    a, b = TS(5, 999_999_000), TS(7, 1_500)
    for fn in ("blosc_elapsed_nsecs", "blosc_elapsed_secs"):
        assert getattr(L, fn)(a, b) == getattr(R, fn)(a, b), fn
        assert getattr(L, fn)(b, a) == getattr(R, fn)(b, a), fn
    assert L.blosc_elapsed_nsecs(a, b) == 1_000_002_500.0
    t0, t1 = TS(), TS()
    L.blosc_set_timestamp(C.byref(t0))
    L.blosc_set_timestamp(C.byref(t1))
    assert 0.0 <= L.blosc_elapsed_secs(t0, t1) < 1.0


# The reference's own C callers on the hot path: each must compile against
# include/blosc2.h and link against libblosc2.so with no undefined symbol.  b2bench.c is C1's
# harness (bench/b2bench.c:171-231 times blosc1_compress / blosc1_decompress with
# blosc_set_timestamp / blosc_elapsed_*).  Build container only: nothing of the reference travels.
REF_CALLERS = ["bench/b2bench.c", "bench/delta_schunk.c", "bench/trunc_prec_schunk.c", "bench/sum_openmp.c",
               "examples/simple.c", "examples/contexts.c", "examples/multithread.c", "examples/noinit.c",
               "examples/schunk_simple.c", "examples/schunk_postfilter.c", "examples/delta_schunk_ex.c",
               "examples/get_set_slice.c", "examples/urfilters.c", "examples/urcodecs.c",
               "examples/get_blocksize.c", "examples/find_roots.c", "examples/frame_roundtrip.c",
               "examples/frame_offset.c", "examples/frame_backed_schunk.c", "examples/compress_file.c",
               "examples/decompress_file.c"]


@pytest.mark.skipif(not os.path.isdir("/root/reference/bench"), reason="reference sources absent")
@pytest.mark.parametrize("src", REF_CALLERS)
def test_reference_callers_compile_and_link(src, tmp_path):
    import subprocess
    out = tmp_path / "a.out"
    cmd = ["gcc", "-O1", "-Wall", "-Werror=implicit-function-declaration", "-I", os.path.join(REPO, "include"),
           os.path.join("/root/reference", src), "-o", str(out), "-L", os.path.dirname(B.LIB_PATH), "-lblosc2",
           "-lm", "-lpthread", "-fopenmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    assert out.exists()
