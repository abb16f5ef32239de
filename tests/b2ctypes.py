"""ctypes mirror of the blosc2 C ABI (include/blosc2.h), shared by the oracle/_ref and the
product library so one test can drive both.  Test helper only."""
import ctypes as C
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(REPO, "oracle", "_ref", "libblosc2_ref.so")
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle.so")
PRODUCT_SO = os.path.join(REPO, "c-blosc2_amd", "lib", "libblosc2.so")

MAX_FILTERS = 6


class CParams(C.Structure):
    """blosc2_cparams (reference include/blosc2.h:1173-1211)."""
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


def cparams(clevel=5, typesize=8, filters=(0, 0, 0, 0, 0, 1), filters_meta=(0,) * 6,
            blocksize=0, splitmode=4, compcode=0, nthreads=1, use_dict=0):
    p = CParams()
    p.compcode, p.clevel, p.typesize, p.nthreads = compcode, clevel, typesize, nthreads
    p.use_dict = use_dict
    p.blocksize, p.splitmode = blocksize, splitmode
    for i in range(MAX_FILTERS):
        p.filters[i] = filters[i]
        p.filters_meta[i] = filters_meta[i] & 0xFF
    return p


def dparams(nthreads=1):
    d = DParams()
    d.nthreads, d.typesize = nthreads, 8
    return d


def bind(lib):
    """Declare the argtypes/restypes of the blosc2 entry points on a CDLL."""
    vp, i32, i16 = C.c_void_p, C.c_int32, C.c_int16
    sig = {
        "blosc2_init": ([], None), "blosc2_destroy": ([], None),
        "blosc2_create_cctx": ([CParams], vp), "blosc2_create_dctx": ([DParams], vp),
        "blosc2_free_ctx": ([vp], None),
        "blosc2_compress_ctx": ([vp, vp, i32, vp, i32], C.c_int),
        "blosc2_decompress_ctx": ([vp, vp, i32, vp, i32], C.c_int),
        "blosc2_getitem_ctx": ([vp, vp, i32, C.c_int, C.c_int, vp, i32], C.c_int),
        "blosc2_shuffle": ([i32, i32, vp, vp], i32), "blosc2_unshuffle": ([i32, i32, vp, vp], i32),
        "blosc2_bitshuffle": ([i32, i32, vp, vp], i32), "blosc2_bitunshuffle": ([i32, i32, vp, vp], i32),
        "blosc2_set_nthreads": ([i16], C.c_int16),
        "blosc1_set_compressor": ([C.c_char_p], C.c_int),
        "blosc1_compress": ([C.c_int, C.c_int, C.c_size_t, C.c_size_t, vp, vp, C.c_size_t], C.c_int),
        "blosc1_decompress": ([vp, vp, C.c_size_t], C.c_int),
        "blosc2_compress": ([C.c_int, C.c_int, i32, vp, i32, vp, i32], C.c_int),
        "blosc2_decompress": ([vp, i32, vp, i32], C.c_int),
        "blosc2_cbuffer_sizes": ([vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name, None)
        if f is not None:
            f.argtypes, f.restype = args, res
    return lib


def ptr(a):
    return C.c_void_p(a.ctypes.data)
