"""GPU tier: cparams.prefilter / dparams.postfilter.

The reference calls a prefilter per block at the head of pipeline_forward and a postfilter per
block at the tail of pipeline_backward, memcpyed and special chunks included
(/root/reference/blosc/blosc2.c:1069-1110, 1239-1250, 1586-1606, 1880-1931; the params copied
into the context at 6215-6219, 6279-6283).  Here the callbacks run on the host between the device
stages (blosc2_api.cpp call_prefilter / call_postfilter).  Modelled on the reference's own tests
(tests/test_prefilter.c, tests/test_postfilter.c:87-200): the same callbacks
(tests/plugins/b2h_prepost.c) are given to this engine and to the reference build, and every case
compares, against the reference at nthreads 1:
  * the chunk bytes (prefilter) or the decompressed bytes (postfilter), byte for byte;
  * the return codes, including a callback failing at one block (FILTER_PIPELINE / POSTFILTER);
  * the sequence of calls with their params (nblock, size, typesize, offset, nchunk, ttmp_nbytes).
Not compared: a postfilter over DELTA chunks -- the reference un-deltas into a scratch buffer the
data never reached (pipeline_backward 1489-1491 keeps _dest off `dest` when a postfilter is set,
and delta_decoder works in place), so its output depends on stale memory; and bytes a callback
leaves unwritten.
"""
import ctypes as C
import os

import numpy as np
import pytest

from b2ctypes import REPO, cparams as ref_cparams, dparams as ref_dparams
from datagen import gen_f32, mixed_bytes
from oracle_lib import p, ref

pytestmark = pytest.mark.gpu

PLUG = os.path.join(REPO, "tests", "plugins", "libb2h_prepost.so")
FILTER_PIPELINE, POSTFILTER = -18, -27  # BLOSC2_ERROR_FILTER_PIPELINE / _POSTFILTER (include/blosc2.h)
SIZE = 500 * 1000                       # test_postfilter.c:12


class PPUser(C.Structure):
    """b2h_pp_user (tests/plugins/b2h_prepost.c)."""
    _fields_ = [("mode", C.c_int32), ("fail_block", C.c_int32), ("inputs", C.c_void_p * 2),
                ("nrec", C.c_int32), ("cap", C.c_int32), ("rec", C.c_void_p)]


class PreParams(C.Structure):
    """blosc2_prefilter_params (reference include/blosc2.h:1118-1132)."""
    _fields_ = [("user_data", C.c_void_p), ("input", C.c_void_p), ("output", C.c_void_p),
                ("output_size", C.c_int32), ("output_typesize", C.c_int32), ("output_offset", C.c_int32),
                ("nchunk", C.c_int64), ("nblock", C.c_int32), ("tid", C.c_int32), ("ttmp", C.c_void_p),
                ("ttmp_nbytes", C.c_size_t), ("ctx", C.c_void_p), ("output_is_disposable", C.c_bool)]


class PostParams(C.Structure):
    """blosc2_postfilter_params (reference include/blosc2.h:1138-1151)."""
    _fields_ = [("user_data", C.c_void_p), ("input", C.c_void_p), ("output", C.c_void_p),
                ("size", C.c_int32), ("typesize", C.c_int32), ("offset", C.c_int32),
                ("nchunk", C.c_int64), ("nblock", C.c_int32), ("tid", C.c_int32), ("ttmp", C.c_void_p),
                ("ttmp_nbytes", C.c_size_t), ("ctx", C.c_void_p)]


@pytest.fixture(scope="module")
def libs():
    import torch  # noqa: F401  (torch's HIP runtime first, then the engine)
    import blosc2_amd as B
    L = B.lib()
    assert L.b2h_device_count() > 0
    R = ref()
    if R is None:
        pytest.skip("reference build oracle/_ref absent")
    PP = C.CDLL(PLUG)
    vp = C.c_void_p
    for lib in (L, R):
        lib.blosc2_decompress_block_ctx.argtypes = [vp, vp, C.c_int32, C.c_int32, vp, C.c_int32]
        lib.blosc2_decompress_block_ctx.restype = C.c_int
        lib.blosc2_chunk_repeatval.restype = C.c_int
    R.blosc2_set_nthreads(1)
    return B, L, R, PP


class Calls:
    """User data + the call record of one library's callbacks."""

    def __init__(self, mode, fail_block=-1, inputs=(None, None), cap=4096):
        self.rec = np.zeros((cap, 8), np.int64)
        self.inputs = inputs
        self.u = PPUser(mode, fail_block, (C.c_void_p * 2)(*(a.ctypes.data if a is not None else None for a in inputs)),
                        0, cap, self.rec.ctypes.data)

    def calls(self):
        return self.rec[: self.u.nrec].copy()


def _pre(PP, calls, disposable=False, output_typesize=0):
    pr = PreParams()
    pr.user_data = C.cast(C.pointer(calls.u), C.c_void_p)
    pr.output_is_disposable = disposable
    pr.output_typesize = output_typesize
    return pr, C.cast(PP.b2h_prefilter, C.c_void_p)


def _compress(lib, cp_fn, PP, raw, calls, disposable=False, **kw):
    cp = cp_fn(**kw)
    pr, fn = _pre(PP, calls, disposable)
    cp.prefilter, cp.preparams = fn, C.cast(C.pointer(pr), C.c_void_p)
    ctx = lib.blosc2_create_cctx(cp)
    assert ctx
    src = raw.copy()   # a prefilter + >= 2 filters rewrite the input, as in the reference
    cap = raw.nbytes + 64
    out = np.zeros(cap, np.uint8)
    n = lib.blosc2_compress_ctx(ctx, p(src), raw.nbytes, p(out), cap)
    lib.blosc2_free_ctx(ctx)
    return (out[:n].copy() if n > 0 else n), calls.calls()


def _dctx(lib, dp_fn, PP, calls):
    dp = dp_fn()
    po = PostParams()
    po.user_data = C.cast(C.pointer(calls.u), C.c_void_p)
    dp.postfilter, dp.postparams = C.cast(PP.b2h_postfilter, C.c_void_p), C.cast(C.pointer(po), C.c_void_p)
    ctx = lib.blosc2_create_dctx(dp)
    assert ctx
    return ctx


def _ref_chunk(R, raw, **kw):
    ctx = R.blosc2_create_cctx(ref_cparams(**kw))
    out = np.zeros(raw.nbytes + 64, np.uint8)
    n = R.blosc2_compress_ctx(ctx, p(raw), raw.nbytes, p(out), out.nbytes)
    R.blosc2_free_ctx(ctx)
    assert n > 0
    return out[:n].copy()


def _ramp(cnt=False):
    data = np.zeros(SIZE, np.int32) if cnt else np.arange(SIZE, dtype=np.int32)
    data2 = np.full(SIZE, 2, np.int32) if cnt else (np.arange(SIZE, dtype=np.int32) * 2)
    return data, data2


# ------------------------------------------------------------------------------- postfilter ----
# name, data, compression kwargs, postfilter mode, fail_block
POST_CASES = [
    ("cl0_memcpyed_x2", "ramp", dict(clevel=0, typesize=4, blocksize=2048), 0, -1),     # test_postfilter.c:237-241
    ("cl1_x2", "ramp", dict(clevel=1, typesize=4, blocksize=2048), 0, -1),
    ("cl7_x2", "ramp", dict(clevel=7, typesize=4, blocksize=2048), 0, -1),
    ("cl9_inputs1_x3", "ramp", dict(clevel=9, typesize=4, blocksize=2048), 1, -1),
    ("cl0_inputs2_sum", "ramp", dict(clevel=0, typesize=4, blocksize=2048), 2, -1),
    ("special_zero_x2", "zeros", dict(clevel=5, typesize=4, blocksize=2048), 0, -1),   # :270-277
    ("special_zero_sum", "zeros", dict(clevel=9, typesize=4, blocksize=2048), 2, -1),
    ("noshuffle_cl9_x2", "zeros", dict(clevel=9, typesize=4, blocksize=2048, filters=(0,) * 6), 0, -1),  # :279-284
    ("f32_split_bytes", "f32", dict(clevel=5, typesize=4, blocksize=65536), 3, -1),
    ("bitshuffle_lz4_leftover", "mixed", dict(clevel=5, typesize=4, blocksize=16384, compcode=1,
                                              filters=(0, 0, 0, 0, 0, 2)), 3, -1),
    ("fails_at_block_3", "ramp", dict(clevel=5, typesize=4, blocksize=65536), 0, 3),
    ("memcpyed_fails_at_block_0", "ramp", dict(clevel=0, typesize=4, blocksize=65536), 3, 0),
]


def _post_data(kind):
    if kind == "ramp":
        return _ramp()[0].view(np.uint8)
    if kind == "zeros":
        return _ramp(cnt=True)[0].view(np.uint8)
    if kind == "f32":
        return gen_f32(5, SIZE).view(np.uint8)
    return mixed_bytes(13, 4 * SIZE - 12)   # a leftover block


def _decompress(lib, dp_fn, PP, chunk, nbytes, calls, mask=None):
    ctx = _dctx(lib, dp_fn, PP, calls)
    if mask is not None:
        m = np.asarray(mask, np.bool_)
        lib.blosc2_set_maskout.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        assert lib.blosc2_set_maskout(ctx, p(m), len(m)) == 0
    out = np.full(nbytes, 0x5A, np.uint8)
    n = lib.blosc2_decompress_ctx(ctx, p(chunk), chunk.nbytes, p(out), nbytes)
    lib.blosc2_free_ctx(ctx)
    return n, out


@pytest.mark.parametrize("case", POST_CASES, ids=[c[0] for c in POST_CASES])
def test_postfilter_decompress_matches_reference(libs, case):
    B, L, R, PP = libs
    _, kind, kw, mode, fail = case
    raw = _post_data(kind)
    chunk = _ref_chunk(R, raw, **kw)
    d1, d2 = _ramp(cnt=(kind == "zeros"))
    res = {}
    for name, lib, dpf in (("gpu", L, B.dparams), ("ref", R, ref_dparams)):
        calls = Calls(mode, fail, inputs=(d1.view(np.uint8), d2.view(np.uint8)))
        n, out = _decompress(lib, dpf, PP, chunk, raw.nbytes, calls)
        res[name] = (n, out, calls.calls())
    (ng, og, cg), (nr, orf, cr) = res["gpu"], res["ref"]
    assert ng == nr, (ng, nr)
    assert len(cg) > 0 and np.array_equal(cg, cr), (cg[:4], cr[:4])
    if nr >= 0:
        assert nr == raw.nbytes
    # blocks written before a failing callback agree too (the reference stops at the failing block)
    assert np.array_equal(og, orf)
    if fail < 0 and mode == 0:
        assert np.array_equal(og.view(np.int32), raw.view(np.int32) * 2)


def test_postfilter_maskout_getitem_block_match_reference(libs):
    """Masked blocks are skipped (no call, dest kept); getitem and decompress_block run the
    callback over each touched block, memcpyed chunks included (no short-circuit, blosc2.c:4336)."""
    B, L, R, PP = libs
    raw = _ramp()[0].view(np.uint8)
    for kw in (dict(clevel=5, typesize=4, blocksize=65536), dict(clevel=0, typesize=4, blocksize=65536)):
        chunk = _ref_chunk(R, raw, **kw)
        nblocks = -(-raw.nbytes // 65536)
        mask = [(b % 3 == 1) for b in range(nblocks)]
        got = {}
        for name, lib, dpf in (("gpu", L, B.dparams), ("ref", R, ref_dparams)):
            calls = Calls(3)
            n, out = _decompress(lib, dpf, PP, chunk, raw.nbytes, calls, mask=mask)
            items = []
            for start, nitems in ((3, 10), (3, SIZE - 3), (16383, 2), (0, SIZE)):
                c2 = Calls(3)
                ctx = _dctx(lib, dpf, PP, c2)
                buf = np.zeros(nitems * 4, np.uint8)
                r = lib.blosc2_getitem_ctx(ctx, p(chunk), chunk.nbytes, start, nitems, p(buf), buf.nbytes)
                lib.blosc2_free_ctx(ctx)
                items.append((r, buf, c2.calls()))
            blocks = []
            for b in (0, 3, nblocks - 1):
                c3 = Calls(0)
                ctx = _dctx(lib, dpf, PP, c3)
                buf = np.zeros(65536, np.uint8)
                r = lib.blosc2_decompress_block_ctx(ctx, p(chunk), chunk.nbytes, b, p(buf), buf.nbytes)
                lib.blosc2_free_ctx(ctx)
                blocks.append((r, buf, c3.calls()))
            got[name] = (n, out, calls.calls(), items, blocks)
        g, r = got["gpu"], got["ref"]
        assert g[0] == r[0] == raw.nbytes
        assert np.array_equal(g[1], r[1]) and np.array_equal(g[2], r[2])
        for (ga, gb, gc), (ra, rb, rc) in zip(g[3] + g[4], r[3] + r[4]):
            assert ga == ra and np.array_equal(gb, rb) and np.array_equal(gc, rc), (ga, ra, gc[:3], rc[:3])


def test_postfilter_repeatval_typesize(libs):
    """A special-value chunk passes its value's width as the typesize (blosc_d 1743-1746)."""
    B, L, R, PP = libs
    nbytes = 8 * 40000
    val = np.array([0x0102030405060708], np.int64)
    out_sizes = {}
    for name, lib, dpf, cpf in (("gpu", L, B.dparams, B.cparams), ("ref", R, ref_dparams, ref_cparams)):
        cp = cpf(clevel=5, typesize=8, blocksize=32768)
        chunk = np.zeros(64, np.uint8)
        lib.blosc2_chunk_repeatval.argtypes = [type(cp), C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
        n = lib.blosc2_chunk_repeatval(cp, nbytes, p(chunk), 64, p(val))
        assert n == 40
        calls = Calls(3)
        r, out = _decompress(lib, dpf, PP, chunk[:n].copy(), nbytes, calls)
        out_sizes[name] = (r, out, calls.calls())
    assert out_sizes["gpu"][0] == out_sizes["ref"][0] == nbytes
    assert np.array_equal(out_sizes["gpu"][1], out_sizes["ref"][1])
    assert np.array_equal(out_sizes["gpu"][2], out_sizes["ref"][2])


# -------------------------------------------------------------------------------- prefilter ----
PRE_CASES = [
    # name, data, compression kwargs, prefilter mode, fail_block, disposable
    ("cl0_memcpyed_x2", "ramp", dict(clevel=0, typesize=4), 0, -1, False),   # test_prefilter.c:178-200
    ("cl1_x2", "ramp", dict(clevel=1, typesize=4), 0, -1, False),
    ("cl7_x2", "ramp", dict(clevel=7, typesize=4), 0, -1, False),
    ("cl9_x2", "ramp", dict(clevel=9, typesize=4), 0, -1, False),
    ("cl0_inputs1_x3", "ramp", dict(clevel=0, typesize=4), 1, -1, False),
    ("cl1_inputs1_x3", "ramp", dict(clevel=1, typesize=4), 1, -1, False),
    ("cl5_inputs2_sum", "ramp", dict(clevel=5, typesize=4), 2, -1, False),
    ("cl9_inputs2_sum", "ramp", dict(clevel=9, typesize=4), 2, -1, False),
    ("bytes_small_blocks", "f32", dict(clevel=5, typesize=4, blocksize=8192), 3, -1, False),
    ("delta_shuffle_two_pass", "ramp", dict(clevel=5, typesize=8, blocksize=65536, filters=(0, 0, 0, 0, 3, 1)), 3, -1, False),
    ("two_filters_rewrite_input", "f32", dict(clevel=5, typesize=4, blocksize=32768, filters=(0, 0, 0, 0, 2, 1)), 3, -1, False),
    ("lz4_bitshuffle", "f32", dict(clevel=5, typesize=4, blocksize=65536, compcode=1, filters=(0, 0, 0, 0, 0, 2)), 3, -1, False),
    ("memcpy_fallback_calls_twice", "mixed", dict(clevel=5, typesize=1, blocksize=65536, filters=(0,) * 6), 3, -1, False),
    ("fails_at_block_2", "ramp", dict(clevel=5, typesize=4, blocksize=65536), 0, 2, False),
    ("memcpyed_fails_at_block_1", "ramp", dict(clevel=0, typesize=4, blocksize=65536), 0, 1, False),
    ("disposable_failure_at_block_1", "ramp", dict(clevel=5, typesize=4, blocksize=65536), 3, 1, True),
]


@pytest.mark.parametrize("case", PRE_CASES, ids=[c[0] for c in PRE_CASES])
def test_prefilter_compress_matches_reference(libs, case):
    B, L, R, PP = libs
    _, kind, kw, mode, fail, disposable = case
    d1, d2 = _ramp()
    raw = {"ramp": d1.view(np.uint8), "f32": gen_f32(9, SIZE).view(np.uint8),
           "mixed": np.random.default_rng(3).integers(0, 256, 4 * SIZE, dtype=np.uint8)}[kind]
    res = {}
    for name, lib, cpf in (("gpu", L, B.cparams), ("ref", R, ref_cparams)):
        calls = Calls(mode, fail, inputs=(d1.view(np.uint8), d2.view(np.uint8)))
        res[name] = _compress(lib, cpf, PP, raw, calls, disposable=disposable, **kw)
    (cg, callg), (cr, callr) = res["gpu"], res["ref"]
    assert len(callg) > 0 and np.array_equal(callg, callr), (callg[:4], callr[:4], len(callg), len(callr))
    if isinstance(cr, int):
        assert cg == cr
        return
    assert not isinstance(cg, int), cg
    assert cg.nbytes == cr.nbytes and np.array_equal(cg, cr)
    if fail < 0 and mode == 0:
        # the reference's decoder gives the prefilter's output back (test_prefilter.c:117-119)
        ctx = R.blosc2_create_dctx(ref_dparams())
        back = np.zeros(raw.nbytes, np.uint8)
        assert R.blosc2_decompress_ctx(ctx, p(cg), cg.nbytes, p(back), back.nbytes) == raw.nbytes
        R.blosc2_free_ctx(ctx)
        assert np.array_equal(back.view(np.int32), d1 * 2)


def test_prefilter_refused_by_device_batch(libs):
    """The device batch API has no host stage: a prefilter is refused loudly, never skipped."""
    B, L, R, PP = libs
    import torch
    cp = B.cparams(clevel=5, typesize=4)
    calls = Calls(0)
    pr, fn = _pre(PP, calls)
    cp.prefilter, cp.preparams = fn, C.cast(C.pointer(pr), C.c_void_p)
    src = torch.zeros(1 << 20, dtype=torch.uint8, device="cuda")
    dst = torch.zeros((1 << 20) + 64, dtype=torch.uint8, device="cuda")
    cb = torch.zeros(1, dtype=torch.int32, device="cuda")
    rc = L.b2h_compress_batch(C.byref(cp), C.c_void_p(src.data_ptr()), 1 << 20, 1, 1 << 20, C.c_void_p(dst.data_ptr()),
                              (1 << 20) + 64, (1 << 20) + 32, C.c_void_p(cb.data_ptr()), None)
    assert rc == FILTER_PIPELINE
    assert calls.u.nrec == 0
