"""GPU tier: user-registered filters and codecs.

A chunk whose pipeline holds a registered user filter or codec runs the reference's semantics with
the user's callbacks per block / per stream between the device stages (blosc2_api.cpp
compress_hybrid / decompress_hybrid; reference blosc/blosc2.c:1055-1180 pipeline_forward,
1210-1469 blosc_c, 1473-1609 pipeline_backward, 1987-2136 blosc_d, 913-971 fill_filter /
fill_codec).  The plugins are tests/plugins/b2h_testplug.c (built by oracle/Makefile), registered
with the SAME function pointers in the engine and in the reference library built here
(oracle/_ref), and also by name only, where both libraries load libblosc2_<name>.so lazily.

Every case checks: the engine's chunk is byte-identical to the reference's (nthreads=1 on the
reference: its threaded path appends blocks in completion order), both libraries decode both
chunks back to the input, and block masks keep the caller's bytes.
"""
import ctypes as C
import os

import numpy as np
import pytest

from b2ctypes import REPO, cparams as ref_cparams
from datagen import gen_f32, int64_ramp, mixed_bytes
from oracle_lib import p, ref

pytestmark = pytest.mark.gpu

PLUG = os.path.join(REPO, "tests", "plugins")
FILT_ID, CODEC_ID = 220, 221          # explicit callbacks
LAZY_FILT_ID, LAZY_CODEC_ID = 230, 231  # registered by name, loaded on first use


class Codec(C.Structure):
    """blosc2_codec (reference include/blosc2.h:2714-2730)."""
    _fields_ = [("compcode", C.c_uint8), ("compname", C.c_char_p), ("complib", C.c_uint8),
                ("version", C.c_uint8), ("encoder", C.c_void_p), ("decoder", C.c_void_p)]


class Filter(C.Structure):
    """blosc2_filter (reference include/blosc2.h:2742-2753)."""
    _fields_ = [("id", C.c_uint8), ("name", C.c_char_p), ("version", C.c_uint8),
                ("forward", C.c_void_p), ("backward", C.c_void_p)]


_keep = []


def _register(lib):
    fl = C.CDLL(os.path.join(PLUG, "libblosc2_b2hfilt.so"))
    co = C.CDLL(os.path.join(PLUG, "libblosc2_b2hcodec.so"))
    _keep.extend([fl, co])
    lib.blosc2_register_filter.argtypes = [C.POINTER(Filter)]
    lib.blosc2_register_codec.argtypes = [C.POINTER(Codec)]
    regs = [
        lib.blosc2_register_filter(C.byref(Filter(FILT_ID, b"b2hfilt_explicit", 1,
                                                  C.cast(fl.b2h_filt_forward, C.c_void_p),
                                                  C.cast(fl.b2h_filt_backward, C.c_void_p)))),
        lib.blosc2_register_codec(C.byref(Codec(CODEC_ID, b"b2hcodec_explicit", CODEC_ID, 3,
                                                C.cast(co.b2h_codec_encoder, C.c_void_p),
                                                C.cast(co.b2h_codec_decoder, C.c_void_p)))),
        # by name only: fill_filter / fill_codec dlopen("libblosc2_<name>.so"); the copies loaded
        # above by path carry that soname, so the loader finds them without a search path
        lib.blosc2_register_filter(C.byref(Filter(LAZY_FILT_ID, b"b2hfilt", 1, None, None))),
        lib.blosc2_register_codec(C.byref(Codec(LAZY_CODEC_ID, b"b2hcodec", LAZY_CODEC_ID, 2, None, None))),
    ]
    assert regs == [0, 0, 0, 0], regs


@pytest.fixture(scope="module")
def libs():
    import torch  # noqa: F401  (torch's HIP runtime first, then the engine)
    import blosc2_amd as B
    assert B.lib().b2h_device_count() > 0
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref absent")
    _register(B.lib())
    _register(R)
    return B, R


def _compress(lib, cp_fn, raw, *, compcode, meta, filters, fmeta, ts, clevel, blocksize, splitmode, nthreads):
    cp = cp_fn(clevel=clevel, typesize=ts, filters=filters, filters_meta=fmeta, blocksize=blocksize,
               splitmode=splitmode, compcode=compcode, nthreads=nthreads)
    cp.compcode_meta = meta
    ctx = lib.blosc2_create_cctx(cp)
    src = raw.copy()   # the >= 3-filter pipelines rewrite their input, as the reference does
    cap = raw.nbytes + 64
    out = np.zeros(cap, np.uint8)
    n = lib.blosc2_compress_ctx(ctx, p(src), raw.nbytes, p(out), cap)
    lib.blosc2_free_ctx(ctx)
    return out[:n].copy() if n > 0 else n


def _decompress(lib, dp_fn, chunk, nbytes, mask=None, fill=0):
    ctx = lib.blosc2_create_dctx(dp_fn())
    out = np.full(max(nbytes, 1), fill, np.uint8)
    if mask is not None:
        m = np.asarray(mask, np.bool_)
        lib.blosc2_set_maskout.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        assert lib.blosc2_set_maskout(ctx, p(m), len(m)) == 0
    n = lib.blosc2_decompress_ctx(ctx, p(chunk), chunk.nbytes, p(out), nbytes)
    lib.blosc2_free_ctx(ctx)
    return out[:nbytes] if n >= 0 else n


def _data(kind, nbytes):
    if kind == "f32":
        return gen_f32(7, nbytes // 4).view(np.uint8)
    if kind == "ramp":
        return int64_ramp(3, nbytes // 8).view(np.uint8)
    if kind == "zeros":
        return np.zeros(nbytes, np.uint8)
    if kind == "steps":   # long byte runs: the run-length codec compresses, runs of streams appear
        return np.repeat(np.arange(nbytes // 512 + 1, dtype=np.uint8), 512)[:nbytes]
    return mixed_bytes(11, nbytes)


CASES = [
    # name, data, nbytes, filters, filters_meta, compcode, compcode_meta, typesize, clevel, blocksize, splitmode
    ("user_filter_then_shuffle_blosclz", "f32", 1 << 18, (0, 0, 0, 0, FILT_ID, 1), (0, 0, 0, 0, 3, 0), 0, 0, 4, 5, 0, 4),
    ("shuffle_then_user_filter_user_codec", "f32", 1 << 18, (0, 0, 0, 0, 1, FILT_ID), (0,) * 6, CODEC_ID, 0x5A, 4, 5, 0, 4),
    ("user_delta_shuffle_lz4_three_filters", "ramp", 1 << 18, (FILT_ID, 2, 1, 0, 0, 0), (1, 0, 0, 0, 0, 0), 1, 0, 8, 5, 0, 4),
    ("user_codec_steps_always_split_ragged", "steps", 100_000, (0, 0, 0, 0, 0, 1), (0,) * 6, CODEC_ID, 7, 4, 9, 16384, 1),
    ("user_codec_bitshuffle_never_split", "ramp", 1 << 17, (0, 0, 0, 0, 0, 2), (0,) * 6, CODEC_ID, 0, 8, 5, 0, 2),
    ("user_codec_special_zero", "zeros", 1 << 17, (0, 0, 0, 0, 0, 1), (0,) * 6, CODEC_ID, 0, 4, 5, 0, 4),
    ("user_codec_memcpy_fallback", "mixed", 1 << 16, (0,) * 6, (0,) * 6, CODEC_ID, 0, 1, 5, 0, 4),
    ("user_codec_small_memcpyed", "f32", 64, (0, 0, 0, 0, 0, 1), (0,) * 6, CODEC_ID, 0, 4, 5, 0, 4),
    ("user_filter_delta_bytedelta_blosclz", "f32", 300_000, (0, 0, 0, 2, FILT_ID, 35), (0, 0, 0, 0, 9, 4), 0, 0, 4, 5, 0, 4),
    ("lazy_filter_lazy_codec", "steps", 1 << 18, (0, 0, 0, 0, 0, LAZY_FILT_ID), (0, 0, 0, 0, 0, 2), LAZY_CODEC_ID, 1, 2, 5, 0, 4),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_user_plugins_match_reference(libs, case):
    B, R = libs
    name, kind, nbytes, filters, fmeta, compcode, meta, ts, clevel, bsz, split = case
    raw = _data(kind, nbytes)
    kw = dict(compcode=compcode, meta=meta, filters=filters, fmeta=fmeta, ts=ts, clevel=clevel,
              blocksize=bsz, splitmode=split)
    ours = _compress(B.lib(), B.cparams, raw, nthreads=1, **kw)
    want = _compress(R, ref_cparams, raw, nthreads=1, **kw)
    assert isinstance(want, np.ndarray), (name, want)
    assert isinstance(ours, np.ndarray), (name, ours)
    assert ours.nbytes == want.nbytes and np.array_equal(ours, want), (name, ours.nbytes, want.nbytes)
    # nthreads > 1 on the engine runs the same per-block callbacks: same bytes
    assert np.array_equal(_compress(B.lib(), B.cparams, raw, nthreads=4, **kw), want), name
    for lib, dpf in ((B.lib(), B.dparams), (R, lambda: __import__("b2ctypes").dparams())):
        assert np.array_equal(_decompress(lib, dpf, ours, nbytes), raw), name
    # block mask: masked blocks keep the caller's bytes, the rest decode (blosc/blosc2.c:1734-1737)
    bs = int(np.frombuffer(ours[8:12].tobytes(), np.int32)[0])
    nblocks = -(-nbytes // bs) if nbytes else 0
    if nblocks >= 2 and not (ours[2] & 0x2) and ((ours[31] >> 4) & 7) == 0:
        mask = [(b % 2) == 1 for b in range(nblocks)]
        got = _decompress(B.lib(), B.dparams, ours, nbytes, mask=mask, fill=0xEE)
        exp = raw.copy()
        for b in range(nblocks):
            if mask[b]:
                exp[b * bs:(b + 1) * bs] = 0xEE
        assert np.array_equal(got, exp), name


def test_unknown_user_codec_fails_loudly(libs):
    """A chunk naming an unregistered user codec fails with BLOSC2_ERROR_CODEC_SUPPORT (-7) in both
    libraries (blosc/blosc2.c:2118-2119)."""
    B, R = libs
    raw = _data("steps", 1 << 16)
    chunk = _compress(B.lib(), B.cparams, raw, compcode=CODEC_ID, meta=0, filters=(0,) * 6, fmeta=(0,) * 6, ts=1,
                      clevel=5, blocksize=0, splitmode=4, nthreads=1)
    bad = chunk.copy()
    bad[22] = 250   # UDCOMPCODE of a codec nobody registered
    assert _decompress(B.lib(), B.dparams, bad, raw.nbytes) == -7
    assert _decompress(R, lambda: __import__("b2ctypes").dparams(), bad, raw.nbytes) == -7


def test_threads_callback_runs_user_callbacks(libs):
    """With blosc2_set_threads_callback and nthreads > 1, the per-block filter callbacks and the
    per-stream decoder callbacks go through the caller's backend (ref blosc/blosc2.c:181-185,
    include/blosc2.h:744); the chunk stays byte-identical to the reference's."""
    B, R = libs
    L = B.lib()
    JOB = C.CFUNCTYPE(None, C.c_void_p)
    CB = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int, C.c_size_t, C.c_void_p)
    calls = []

    def run(data, dojob, numjobs, elsize, jobdata):
        calls.append(numjobs)
        job = JOB(dojob)
        for i in range(numjobs):
            job(jobdata + i * elsize)

    cb = CB(run)
    L.blosc2_set_threads_callback.argtypes = [CB, C.c_void_p]
    L.blosc2_set_threads_callback(cb, None)
    try:
        raw = _data("steps", 1 << 18)
        kw = dict(compcode=CODEC_ID, meta=3, filters=(0, 0, 0, 0, 0, FILT_ID), fmeta=(0,) * 6, ts=4, clevel=5,
                  blocksize=16384, splitmode=4)
        ours = _compress(L, B.cparams, raw, nthreads=4, **kw)
        want = _compress(R, ref_cparams, raw, nthreads=1, **kw)
        assert np.array_equal(ours, want)
        ctx = L.blosc2_create_dctx(B.dparams(nthreads=4))
        out = np.zeros(raw.nbytes, np.uint8)
        assert L.blosc2_decompress_ctx(ctx, p(ours), ours.nbytes, p(out), raw.nbytes) == raw.nbytes
        L.blosc2_free_ctx(ctx)
        assert np.array_equal(out, raw)
        assert calls and all(n > 1 for n in calls), calls
    finally:
        L.blosc2_set_threads_callback(CB(), None)
