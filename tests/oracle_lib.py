"""Loader for the oracle restatement (oracle/liboracle.so) and, when built, the reference
library compiled from /root/reference sources (oracle/_ref/libblosc2_ref.so).  Test-only."""
import ctypes as C
import os
import subprocess

import numpy as np

from b2ctypes import ORACLE_SO, REF_SO, REPO, bind, cparams

_oracle = None
_ref = None


class OrCParams(C.Structure):
    _fields_ = [("compcode", C.c_int), ("clevel", C.c_int), ("typesize", C.c_int),
                ("blocksize", C.c_int), ("splitmode", C.c_int),
                ("filters", C.c_uint8 * 6), ("filters_meta", C.c_uint8 * 6), ("use_dict", C.c_int)]


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"])
        L = C.CDLL(ORACLE_SO)
        vp, i32 = C.c_void_p, C.c_int32
        for n in ("or_shuffle", "or_unshuffle", "or_bitshuffle"):
            getattr(L, n).argtypes, getattr(L, n).restype = [i32, i32, vp, vp], i32
        L.or_bitunshuffle.argtypes, L.or_bitunshuffle.restype = [i32, i32, vp, vp, C.c_uint8], i32
        L.or_delta_encode.argtypes, L.or_delta_encode.restype = [vp, i32, i32, i32, vp, vp], None
        L.or_delta_decode.argtypes, L.or_delta_decode.restype = [vp, i32, i32, i32, vp], None
        L.or_trunc_prec.argtypes, L.or_trunc_prec.restype = [C.c_int8, i32, i32, vp, vp], C.c_int
        L.or_int_trunc.argtypes, L.or_int_trunc.restype = [C.c_int8, i32, i32, vp, vp], C.c_int
        L.or_bytedelta_encode.argtypes, L.or_bytedelta_encode.restype = [i32, i32, vp, vp], None
        L.or_bytedelta_decode.argtypes, L.or_bytedelta_decode.restype = [i32, i32, vp, vp], None
        L.or_blosclz_compress.argtypes = [C.c_int, vp, C.c_int, vp, C.c_int]
        L.or_blosclz_decompress.argtypes = [vp, C.c_int, vp, C.c_int]
        L.or_compute_blocksize.argtypes, L.or_compute_blocksize.restype = [C.POINTER(OrCParams), i32], i32
        L.or_compress_chunk.argtypes = [C.POINTER(OrCParams), vp, i32, vp, i32]
        L.or_decompress_chunk.argtypes = [vp, i32, vp, i32]
        _oracle = L
    return _oracle


class Filter(C.Structure):
    """blosc2_filter (reference include/blosc2.h:2742-2753)."""
    _fields_ = [("id", C.c_uint8), ("name", C.c_char_p), ("version", C.c_uint8),
                ("forward", C.c_void_p), ("backward", C.c_void_p)]


_keep = []


def ref():
    """The reference library, or None when it was not built (e.g. /root/reference absent).  The
    bytedelta (35) and int_trunc (36) plugin filters compiled into it are registered the way
    plugins/filters/filters-registry.c:43-57 does at blosc2_init (HAVE_PLUGINS is off there)."""
    global _ref
    if _ref is None and os.path.exists(REF_SO):
        R = bind(C.CDLL(REF_SO))
        R.blosc2_init()
        R.register_filter_private.argtypes, R.register_filter_private.restype = [C.POINTER(Filter)], C.c_int
        for fid, name, fw, bw in ((35, b"bytedelta", "bytedelta_forward", "bytedelta_backward"),
                                  (36, b"int_trunc", "int_trunc_forward", "int_trunc_backward")):
            f = Filter(fid, name, 1, C.cast(getattr(R, fw), C.c_void_p), C.cast(getattr(R, bw), C.c_void_p))
            _keep.append(f)
            assert R.register_filter_private(C.byref(f)) == 0
        _ref = R
    return _ref


def or_cparams(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1), filters_meta=(0,) * 6,
               blocksize=0, splitmode=4, compcode=0, use_dict=0):
    p = OrCParams()
    p.compcode, p.clevel, p.typesize, p.blocksize, p.splitmode = compcode, clevel, typesize, blocksize, splitmode
    p.use_dict = use_dict
    for i in range(6):
        p.filters[i], p.filters_meta[i] = filters[i], filters_meta[i] & 0xFF
    return p


def p(a):
    return C.c_void_p(a.ctypes.data)


def oracle_compress(src: np.ndarray, **kw):
    cp = or_cparams(**kw)
    raw = src.view(np.uint8).reshape(-1)
    out = np.zeros(raw.nbytes + 64, np.uint8)
    n = oracle().or_compress_chunk(C.byref(cp), p(raw), raw.nbytes, p(out), raw.nbytes + 32)
    return out[:n] if n > 0 else n


def oracle_decompress(chunk: np.ndarray, nbytes: int):
    out = np.zeros(max(nbytes, 1), np.uint8)
    n = oracle().or_decompress_chunk(p(chunk), chunk.nbytes, p(out), nbytes)
    return out[:nbytes] if n >= 0 else n


def ref_compress(src: np.ndarray, **kw):
    """blosc2_compress_ctx on the reference (nthreads=1) with a fresh context."""
    R = ref()
    cp = cparams(clevel=kw.get("clevel", 5), typesize=kw.get("typesize", 4),
                 filters=kw.get("filters", (0, 0, 0, 0, 0, 1)),
                 filters_meta=kw.get("filters_meta", (0,) * 6),
                 blocksize=kw.get("blocksize", 0), splitmode=kw.get("splitmode", 4),
                 compcode=kw.get("compcode", 0), use_dict=kw.get("use_dict", 0))
    ctx = R.blosc2_create_cctx(cp)
    raw = src.view(np.uint8).reshape(-1).copy()   # the reference may rewrite its input
    out = np.zeros(raw.nbytes + 64, np.uint8)
    n = R.blosc2_compress_ctx(ctx, p(raw), raw.nbytes, p(out), raw.nbytes + 32)
    R.blosc2_free_ctx(ctx)
    return out[:n] if n > 0 else n
