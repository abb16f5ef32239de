"""Python host-side mirror of the drop-in library (c-blosc2_amd/lib/libblosc2.so).

This mirrors the reference's C entry points one-to-one over ctypes (same names, same argument
meaning, same integer return codes) so tests and bench read like the reference's own C tests.
It never falls back to anything: if the HIP library is missing, importing this module raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# B2H_LIB: an alternative build of the same library (diagnostic A/B runs of build variants)
LIB_PATH = os.environ.get("B2H_LIB") or os.path.join(HERE, "lib", "libblosc2.so")

MAX_FILTERS = 6
NOFILTER, SHUFFLE, BITSHUFFLE, DELTA, TRUNC_PREC = 0, 1, 2, 3, 4
ALWAYS_SPLIT, NEVER_SPLIT, AUTO_SPLIT, FORWARD_COMPAT_SPLIT = 1, 2, 3, 4
BLOSC2_MAX_OVERHEAD = 32


class CParams(C.Structure):
    """blosc2_cparams (include/blosc2.h; reference include/blosc2.h:1173-1211)."""
    _fields_ = [
        ("compcode", C.c_uint8), ("compcode_meta", C.c_uint8), ("clevel", C.c_uint8),
        ("use_dict", C.c_int), ("typesize", C.c_int32), ("nthreads", C.c_int16),
        ("blocksize", C.c_int32), ("splitmode", C.c_int32), ("schunk", C.c_void_p),
        ("filters", C.c_uint8 * MAX_FILTERS), ("filters_meta", C.c_uint8 * MAX_FILTERS),
        ("prefilter", C.c_void_p), ("preparams", C.c_void_p), ("tuner_params", C.c_void_p),
        ("tuner_id", C.c_int), ("instr_codec", C.c_bool), ("codec_params", C.c_void_p),
        ("filter_params", C.c_void_p * MAX_FILTERS),
    ]


class DParams(C.Structure):
    """blosc2_dparams (reference include/blosc2.h:1232-1243)."""
    _fields_ = [("nthreads", C.c_int16), ("schunk", C.c_void_p), ("postfilter", C.c_void_p),
                ("postparams", C.c_void_p), ("typesize", C.c_int32)]


B2H_CODEC_PARAMS_MAGIC = 0x68623262
EXACT, FAST, DEEP, SEG = 0, 1, 2, 3   # BloscLZ encoder modes (include/b2h.h b2h_codec_params)


class CodecParams(C.Structure):
    """b2h_codec_params (include/b2h.h): a context's BloscLZ encoder, carried by cparams.codec_params."""
    _fields_ = [("magic", C.c_uint32), ("blosclz_mode", C.c_int32)]


def cparams(clevel=5, typesize=8, filters=(0, 0, 0, 0, 0, SHUFFLE), filters_meta=(0,) * 6,
            blocksize=0, splitmode=FORWARD_COMPAT_SPLIT, compcode=0, nthreads=1, use_dict=0, lz_mode=None):
    """blosc2_cparams; lz_mode (EXACT / FAST) selects the BloscLZ encoder of this context only
    (None: the process default, b2h_set_blosclz_mode)."""
    p = CParams()
    p.compcode, p.clevel, p.typesize, p.nthreads = compcode, clevel, typesize, nthreads
    p.use_dict = use_dict
    p.blocksize, p.splitmode = blocksize, splitmode
    for i in range(MAX_FILTERS):
        p.filters[i] = filters[i]
        p.filters_meta[i] = filters_meta[i] & 0xFF
    if lz_mode is not None:
        cpp = CodecParams(B2H_CODEC_PARAMS_MAGIC, lz_mode)
        p._codec_params_keep = cpp   # kept alive with the struct that points at it
        p.codec_params = C.cast(C.pointer(cpp), C.c_void_p)
    return p


def dparams(nthreads=1):
    d = DParams()
    d.nthreads, d.typesize = nthreads, 8
    return d


class Storage(C.Structure):
    """blosc2_storage (reference include/blosc2.h:1758-1776); params as plain pointers."""
    _fields_ = [("contiguous", C.c_bool), ("urlpath", C.c_char_p), ("cparams", C.c_void_p),
                ("dparams", C.c_void_p), ("io", C.c_void_p)]


class IO(C.Structure):
    """blosc2_io (reference include/blosc2.h:1047-1059)."""
    _fields_ = [("id", C.c_uint8), ("name", C.c_char_p), ("params", C.c_void_p)]


OPEN_CB = C.CFUNCTYPE(C.c_void_p, C.c_char_p, C.c_char_p, C.c_void_p)
CLOSE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p)
SIZE_CB = C.CFUNCTYPE(C.c_int64, C.c_void_p)
WRITE_CB = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
READ_CB = C.CFUNCTYPE(C.c_int64, C.POINTER(C.c_void_p), C.c_int64, C.c_int64, C.c_int64, C.c_void_p)
TRUNCATE_CB = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int64)
DESTROY_CB = C.CFUNCTYPE(C.c_int, C.c_void_p)


class IOCb(C.Structure):
    """blosc2_io_cb (reference include/blosc2.h:1018-1041)."""
    _fields_ = [("id", C.c_uint8), ("name", C.c_char_p), ("is_allocation_necessary", C.c_bool),
                ("open", OPEN_CB), ("close", CLOSE_CB), ("size", SIZE_CB), ("write", WRITE_CB),
                ("read", READ_CB), ("truncate", TRUNCATE_CB), ("destroy", DESTROY_CB)]


class StdioMmap(C.Structure):
    """blosc2_stdio_mmap (reference include/blosc2/blosc2-stdio.h:76-116, POSIX layout)."""
    _fields_ = [("mode", C.c_char_p), ("initial_mapping_size", C.c_size_t), ("needs_free", C.c_bool),
                ("addr", C.c_void_p), ("urlpath", C.c_char_p), ("file_size", C.c_size_t),
                ("mapping_size", C.c_size_t), ("is_memory_only", C.c_bool), ("file", C.c_void_p),
                ("fd", C.c_int), ("access_flags", C.c_int64), ("map_flags", C.c_int64)]

    @classmethod
    def defaults(cls, mode=b"r"):
        return cls(mode, 1 << 30, False, None, None, 0, 0, False, None, -1, -1, -1)


class Schunk(C.Structure):
    """blosc2_schunk (reference include/blosc2.h:1823-1892), ABI-identical."""
    _fields_ = [
        ("version", C.c_uint8), ("compcode", C.c_uint8), ("compcode_meta", C.c_uint8), ("clevel", C.c_uint8),
        ("splitmode", C.c_uint8), ("typesize", C.c_int32), ("blocksize", C.c_int32), ("chunksize", C.c_int32),
        ("flags2", C.c_uint8), ("use_dict", C.c_uint8), ("filters", C.c_uint8 * MAX_FILTERS),
        ("filters_meta", C.c_uint8 * MAX_FILTERS), ("nchunks", C.c_int64), ("current_nchunk", C.c_int64),
        ("nbytes", C.c_int64), ("cbytes", C.c_int64), ("data", C.POINTER(C.c_void_p)), ("data_len", C.c_size_t),
        ("storage", C.POINTER(Storage)), ("frame", C.c_void_p), ("cctx", C.c_void_p), ("dctx", C.c_void_p),
        ("metalayers", C.c_void_p * 16), ("nmetalayers", C.c_uint16), ("vlmetalayers", C.c_void_p * 8192),
        ("nvlmetalayers", C.c_int16), ("tuner_params", C.c_void_p), ("tuner_id", C.c_int), ("ndim", C.c_int8),
        ("blockshape", C.c_void_p), ("view", C.c_bool), ("change_tick", C.c_int64),
    ]


SCHUNK_COUNTERS = ("nchunks", "current_nchunk", "nbytes", "cbytes", "chunksize", "flags2", "typesize",
                   "blocksize", "clevel", "compcode", "splitmode", "use_dict", "data_len")


_LIBC = None


def _libc():
    global _LIBC
    if _LIBC is None:
        _LIBC = C.CDLL(None)
        _LIBC.free.argtypes = [C.c_void_p]
    return _LIBC


def bind_schunk(lib):
    """argtypes of the super-chunk entry points (include/blosc2.h:1905-2328): shared by the product
    and the oracle/_ref build, whose structs are the same ABI."""
    vp, i32, i64, sp = C.c_void_p, C.c_int32, C.c_int64, C.POINTER(Schunk)
    sig = {
        "blosc2_schunk_new": ([C.POINTER(Storage)], sp), "blosc2_schunk_free": ([sp], C.c_int),
        "blosc2_schunk_append_chunk": ([sp, vp, C.c_bool], i64),
        "blosc2_schunk_insert_chunk": ([sp, i64, vp, C.c_bool], i64),
        "blosc2_schunk_update_chunk": ([sp, i64, vp, C.c_bool], i64),
        "blosc2_schunk_delete_chunk": ([sp, i64], i64),
        "blosc2_schunk_append_buffer": ([sp, vp, i32], i64),
        "blosc2_schunk_decompress_chunk": ([sp, i64, vp, i32], C.c_int),
        "blosc2_schunk_get_chunk": ([sp, i64, C.POINTER(vp), C.POINTER(C.c_bool)], C.c_int),
        "blosc2_schunk_get_lazychunk": ([sp, i64, C.POINTER(vp), C.POINTER(C.c_bool)], C.c_int),
        "blosc2_schunk_get_slice_buffer": ([sp, i64, i64, vp], C.c_int),
        "blosc2_schunk_set_slice_buffer": ([sp, i64, i64, vp], C.c_int),
        "b2h_schunk_set_slice_device": ([sp, i64, i64, vp], C.c_int),
        "blosc2_schunk_get_cparams": ([sp, C.POINTER(vp)], C.c_int),
        "blosc2_schunk_get_dparams": ([sp, C.POINTER(vp)], C.c_int),
        "blosc2_getitem_bytes_ctx": ([vp, vp, i32, i32, i32, vp, i32], C.c_int),
        "b2h_schunk_append_device": ([sp, vp, vp, i32, i64], i64),
        "b2h_schunk_decompress_device": ([sp, i64, i32, vp, i64, i32, vp], C.c_int),
        "b2h_schunk_append_buffers": ([sp, vp, vp, i32, i64, i32], i64),
        "b2h_schunk_decompress_buffers": ([sp, i64, i32, vp, i64, i32, vp, i32], C.c_int),
        "b2h_schunk_get_slice_device": ([sp, i64, i64, vp], C.c_int),
        "blosc2_schunk_from_buffer": ([vp, i64, C.c_bool], sp),
        "blosc2_schunk_open": ([C.c_char_p], sp),
        "blosc2_schunk_open_offset": ([C.c_char_p, i64], sp),
        "blosc2_schunk_open_udio": ([C.c_char_p, vp], sp),
        "blosc2_schunk_open_offset_udio": ([C.c_char_p, i64, vp], sp),
        "blosc2_schunk_to_buffer": ([sp, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_bool)], i64),
        "blosc2_schunk_to_file": ([sp, C.c_char_p], i64),
        "blosc2_schunk_append_file": ([sp, C.c_char_p], i64),
        "blosc2_register_io_cb": ([vp], C.c_int),
        "blosc2_get_io_cb": ([C.c_uint8], vp),
        "blosc2_meta_add": ([sp, C.c_char_p, vp, i32], C.c_int),
        "blosc2_vlmeta_add": ([sp, C.c_char_p, vp, i32, vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.argtypes, f.restype = args, res
    return lib


def _bind(lib):
    vp, i32, i16, i64 = C.c_void_p, C.c_int32, C.c_int16, C.c_int64
    sig = {
        "blosc2_init": ([], None), "blosc2_destroy": ([], None),
        "blosc2_create_cctx": ([CParams], vp), "blosc2_create_dctx": ([DParams], vp),
        "blosc2_free_ctx": ([vp], None),
        "blosc2_compress_ctx": ([vp, vp, i32, vp, i32], C.c_int),
        "blosc2_decompress_ctx": ([vp, vp, i32, vp, i32], C.c_int),
        "blosc2_getitem_ctx": ([vp, vp, i32, C.c_int, C.c_int, vp, i32], C.c_int),
        "blosc2_set_maskout": ([vp, vp, C.c_int], C.c_int),
        "blosc2_shuffle": ([i32, i32, vp, vp], i32), "blosc2_unshuffle": ([i32, i32, vp, vp], i32),
        "blosc2_bitshuffle": ([i32, i32, vp, vp], i32), "blosc2_bitunshuffle": ([i32, i32, vp, vp], i32),
        "blosc2_set_nthreads": ([i16], i16),
        "blosc1_set_compressor": ([C.c_char_p], C.c_int),
        "blosc1_compress": ([C.c_int, C.c_int, C.c_size_t, C.c_size_t, vp, vp, C.c_size_t], C.c_int),
        "blosc1_decompress": ([vp, vp, C.c_size_t], C.c_int),
        "blosc2_compress": ([C.c_int, C.c_int, i32, vp, i32, vp, i32], C.c_int),
        "blosc2_decompress": ([vp, i32, vp, i32], C.c_int),
        "blosc2_cbuffer_sizes": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)], C.c_int),
        "blosc2_get_version_string": ([], C.c_char_p),
        "b2h_compress_batch": ([C.POINTER(CParams), vp, i32, i32, i64, vp, i64, i32, vp, vp], C.c_int),
        "b2h_compress_batch_sizes": ([C.POINTER(CParams), vp, vp, i32, i64, vp, i64, i32, vp, vp], C.c_int),
        "b2h_decompress_batch": ([vp, i64, vp, i32, vp, i64, i32, vp, vp], C.c_int),
        "b2h_pack_chunks": ([vp, i64, vp, i32, vp, vp, vp], C.c_int),
        "b2h_unpack_chunks": ([vp, vp, i32, vp, i64, vp, vp], C.c_int),
        "b2h_device_copy": ([vp, vp, i64, vp], C.c_int),
        "b2h_shuffle": ([i32, i32, vp, vp, C.c_int, vp], i32),
        "b2h_bitshuffle": ([i32, i32, vp, vp, C.c_int, vp], i32),
        "b2h_enable_timing": ([C.c_int], None),
        "b2h_set_blosclz_mode": ([C.c_int], C.c_int),
        "b2h_last_times": ([C.POINTER(C.c_float)], None),
        "b2h_mean_times": ([C.POINTER(C.c_float)], None),
        "b2h_last_error": ([], C.c_char_p),
        "b2h_device_count": ([], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes, f.restype = args, res
    return bind_schunk(lib)


_lib = None


def lib():
    """Load the HIP library (raises if it was not built: there is no fallback)."""
    global _lib
    if _lib is None:
        # One HIP runtime per process: torch bundles its own libamdhip64 (SONAME libamdhip64.so.7).
        # Loading torch first lets our library bind to that same copy; loading ours first would
        # pull /opt/rocm's copy and torch would then add a second runtime.
        if os.environ.get("B2H_NO_TORCH") is None:
            try:
                import torch  # noqa: F401
            except ImportError:
                pass
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make -C c-blosc2_amd` "
                               "(the MI355X engine has no CPU fallback)")
        _lib = _bind(C.CDLL(LIB_PATH))
        _lib.blosc2_init()
    return _lib


def _p(a):
    return C.c_void_p(a.ctypes.data)


# ------------------------------------------------------------ host-buffer convenience ----
def compress_ctx(ctx, src: np.ndarray, destsize=None):
    raw = np.ascontiguousarray(src).view(np.uint8).reshape(-1)
    if destsize is None:
        destsize = raw.nbytes + BLOSC2_MAX_OVERHEAD
    out = np.zeros(destsize + 16, np.uint8)
    n = lib().blosc2_compress_ctx(ctx, _p(raw), raw.nbytes, _p(out), destsize)
    return out[:n] if n > 0 else n


def decompress_ctx(ctx, chunk: np.ndarray, nbytes: int):
    out = np.zeros(max(nbytes, 1), np.uint8)
    n = lib().blosc2_decompress_ctx(ctx, _p(chunk), chunk.nbytes, _p(out), nbytes)
    return out[:nbytes] if n >= 0 else n


def compress(src: np.ndarray, **kw):
    """One chunk through a fresh compression context (blosc2_create_cctx + compress_ctx)."""
    L = lib()
    ctx = L.blosc2_create_cctx(cparams(**kw))
    try:
        return compress_ctx(ctx, src)
    finally:
        L.blosc2_free_ctx(ctx)


def decompress(chunk: np.ndarray, nbytes: int):
    L = lib()
    ctx = L.blosc2_create_dctx(dparams())
    try:
        return decompress_ctx(ctx, chunk, nbytes)
    finally:
        L.blosc2_free_ctx(ctx)


# ------------------------------------------------------------- device batch interface ----
def compress_batch(cp: CParams, d_src: int, chunk_nbytes: int, nchunks: int, src_stride: int,
                   d_dst: int, dst_stride: int, dst_capacity: int, d_cbytes: int, stream: int = 0):
    rc = lib().b2h_compress_batch(C.byref(cp), C.c_void_p(d_src), chunk_nbytes, nchunks, src_stride,
                                  C.c_void_p(d_dst), dst_stride, dst_capacity, C.c_void_p(d_cbytes),
                                  C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_compress_batch: {rc} {lib().b2h_last_error()}")


def compress_batch_sizes(cp: CParams, d_src: int, nbytes, src_stride: int, d_dst: int, dst_stride: int,
                         dst_capacity: int, d_cbytes: int, stream: int = 0):
    """Chunks of per-chunk sizes (host sequence `nbytes`), e.g. a super-chunk's ragged tail."""
    sizes = (C.c_int32 * len(nbytes))(*nbytes)
    rc = lib().b2h_compress_batch_sizes(C.byref(cp), C.c_void_p(d_src), sizes, len(nbytes), src_stride,
                                        C.c_void_p(d_dst), dst_stride, dst_capacity, C.c_void_p(d_cbytes),
                                        C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_compress_batch_sizes: {rc} {lib().b2h_last_error()}")


def decompress_batch(d_src: int, src_stride: int, d_cbytes: int, nchunks: int, d_dst: int,
                     dst_stride: int, dst_capacity: int, d_status: int, stream: int = 0):
    rc = lib().b2h_decompress_batch(C.c_void_p(d_src), src_stride, C.c_void_p(d_cbytes), nchunks,
                                    C.c_void_p(d_dst), dst_stride, dst_capacity, C.c_void_p(d_status),
                                    C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_decompress_batch: {rc} {lib().b2h_last_error()}")


def pack_chunks(d_src: int, src_stride: int, d_sizes: int, n: int, d_dst: int, d_offsets: int, stream: int = 0):
    """b2h_pack_chunks: chunk i (d_src + i*src_stride, d_sizes[i] bytes) -> d_dst, offsets[n+1]."""
    rc = lib().b2h_pack_chunks(C.c_void_p(d_src), src_stride, C.c_void_p(d_sizes), n, C.c_void_p(d_dst),
                               C.c_void_p(d_offsets), C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_pack_chunks: {rc} {lib().b2h_last_error()}")


def unpack_chunks(d_src: int, d_offsets: int, n: int, d_dst: int, dst_stride: int, d_sizes: int, stream: int = 0):
    """b2h_unpack_chunks: d_src[offsets[i], offsets[i+1]) -> d_dst + i*dst_stride (+ sizes)."""
    rc = lib().b2h_unpack_chunks(C.c_void_p(d_src), C.c_void_p(d_offsets), n, C.c_void_p(d_dst), dst_stride,
                                 C.c_void_p(d_sizes), C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_unpack_chunks: {rc} {lib().b2h_last_error()}")


def device_copy(d_dst: int, d_src: int, nbytes: int, stream: int = 0):
    rc = lib().b2h_device_copy(C.c_void_p(d_dst), C.c_void_p(d_src), nbytes, C.c_void_p(stream))
    if rc < 0:
        raise RuntimeError(f"b2h_device_copy: {rc} {lib().b2h_last_error()}")


def last_times():
    """Per-phase kernel times (ms) of the latest batch (waits for its events)."""
    buf = (C.c_float * 5)()
    lib().b2h_last_times(buf)
    return dict(zip(("filter_ms", "encode_ms", "finalize_ms", "decode_ms", "unfilter_ms"), list(buf)))


def mean_times():
    """Per-phase kernel times (ms), mean over every batch since b2h_enable_timing(1)."""
    buf = (C.c_float * 5)()
    lib().b2h_mean_times(buf)
    return dict(zip(("filter_ms", "encode_ms", "finalize_ms", "decode_ms", "unfilter_ms"), list(buf)))


# ------------------------------------------------------------------------- super-chunks ----
class SChunk:
    """An in-memory super-chunk (blosc2_schunk_new with sparse storage) of a library `L` (the
    product by default; tests drive the oracle/_ref build through the same class).  `cparams` /
    `dparams` are that library's own structs."""

    def __init__(self, cparams_, dparams_=None, L=None):
        self.L = L if L is not None else lib()
        self._keep = (cparams_, dparams_)
        st = Storage(False, None, C.cast(C.pointer(cparams_), C.c_void_p),
                     C.cast(C.pointer(dparams_), C.c_void_p) if dparams_ is not None else None, None)
        self.p = self.L.blosc2_schunk_new(C.byref(st))
        if not self.p:
            raise RuntimeError("blosc2_schunk_new failed")

    @classmethod
    def wrap(cls, p, L):
        """Take ownership of a super-chunk pointer `p` of library `L` (blosc2_schunk_open & co.)."""
        self = cls.__new__(cls)
        self.L, self._keep, self.p = L, None, p
        return self

    @property
    def s(self):
        return self.p.contents

    def counters(self):
        return {k: getattr(self.s, k) for k in SCHUNK_COUNTERS}

    def append_buffer(self, a: np.ndarray):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        return self.L.blosc2_schunk_append_buffer(self.p, _p(raw), raw.nbytes)

    def append_chunk(self, chunk: np.ndarray, copy=True):
        return self.L.blosc2_schunk_append_chunk(self.p, _p(chunk), copy)

    def insert_chunk(self, n, chunk: np.ndarray, copy=True):
        return self.L.blosc2_schunk_insert_chunk(self.p, n, _p(chunk), copy)

    def update_chunk(self, n, chunk: np.ndarray, copy=True):
        return self.L.blosc2_schunk_update_chunk(self.p, n, _p(chunk), copy)

    def delete_chunk(self, n):
        return self.L.blosc2_schunk_delete_chunk(self.p, n)

    def chunk(self, n):
        """The n-th compressed chunk (a copy), or the error code."""
        cp, nf = C.c_void_p(), C.c_bool()
        cb = self.L.blosc2_schunk_get_chunk(self.p, n, C.byref(cp), C.byref(nf))
        if cb <= 0:
            return cb
        out = np.ctypeslib.as_array(C.cast(cp, C.POINTER(C.c_uint8)), (cb,)).copy()
        if nf.value:   # read off a frame file (frame_get_chunk): the caller's to free
            _libc().free(cp)
        return out

    def decompress_chunk(self, n, nbytes):
        out = np.zeros(max(nbytes, 1), np.uint8)
        rc = self.L.blosc2_schunk_decompress_chunk(self.p, n, _p(out), nbytes)
        return (rc, out[:max(rc, 0)])

    def get_slice(self, start, stop, itemsize=None):
        ts = itemsize or self.s.typesize
        out = np.zeros(max((stop - start) * ts, 1), np.uint8)
        rc = self.L.blosc2_schunk_get_slice_buffer(self.p, start, stop, _p(out))
        return (rc, out[:max((stop - start) * ts, 0)])

    def set_slice(self, start, stop, a: np.ndarray):
        raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
        return self.L.blosc2_schunk_set_slice_buffer(self.p, start, stop, _p(raw))

    def free(self):
        if self.p:
            self.L.blosc2_schunk_free(self.p)
            self.p = None
