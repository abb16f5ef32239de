"""GPU tier, drop-in boundary and configurations that round 1 left untested:

  * C1, the reference's own headline CPU benchmark (bench/b2bench.c:105-274): 1e6 int32 values of
    get_value(i, 19) (b2bench.c:73-81) through blosc1_compress(clevel, SHUFFLE, 4, ...) for clevel
    0..9 (b2bench.c:199) -- byte-identical to the oracle and to the reference library built here;
  * special chunks (blosc2_chunk_zeros/nans/repeatval/uninit, blosc/blosc2.c:6452-6637) decoded on
    the device, and the header checks of read_chunk_header (blosc2.c:796-825) / set_nans;
  * concurrency: distinct contexts on distinct host threads (include/blosc2.h:1462-1466), and the
    batch API on two streams sharing one device workspace;
  * the strided batch decompression is stream-ordered (no host wait inside the call).
"""
import ctypes as C
import threading

import numpy as np
import pytest

from b2ctypes import cparams as ref_cparams
from datagen import b2bench_values, gen_f32, int64_ramp, mixed_bytes
from oracle_lib import oracle_compress, oracle_decompress, p, ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def B():
    import torch  # noqa: F401  (torch's HIP runtime first, then the engine)
    import blosc2_amd
    assert blosc2_amd.lib().b2h_device_count() > 0
    return blosc2_amd


# ------------------------------------------------------------------------------- C1 ----
def test_c1_b2bench_clevels(B):
    """b2bench `blosclz shuffle single 1 4000000 4 19`: every clevel byte-identical to the oracle
    and the reference build, and decoded back exactly through blosc1_decompress."""
    L = B.lib()
    src = b2bench_values(1_000_000, 19)
    assert src.dtype == np.int32 and int(src[1]) == (((1 << 26) ^ (1 << 18) ^ (1 << 11) ^ (1 << 3) ^ 1) & ((1 << 19) - 1))
    L.blosc1_set_compressor(b"blosclz")
    R = ref()
    if R is not None:
        R.blosc1_set_compressor(b"blosclz")
        R.blosc2_set_nthreads(1)
    size = src.nbytes
    for clevel in range(10):
        out = np.zeros(size + 32, np.uint8)
        n = L.blosc1_compress(clevel, 1, 4, size, B._p(src), B._p(out), size + 32)
        assert n > 0, (clevel, n)
        want = oracle_compress(src, clevel=clevel, typesize=4, filters=(0, 0, 0, 0, 0, 1))
        assert np.array_equal(out[:n], want), clevel
        if R is not None:
            rout = np.zeros(size + 32, np.uint8)
            rsrc = src.copy()   # the reference may rewrite its input; keep the copy alive
            rn = R.blosc1_compress(clevel, 1, 4, size, p(rsrc), p(rout), size + 32)
            assert rn == n and np.array_equal(rout[:rn], out[:n]), clevel
        dec = np.zeros(size, np.uint8)
        assert L.blosc1_decompress(B._p(out), B._p(dec), size) == size
        assert np.array_equal(dec.view(np.int32), src), clevel
    # the ratio b2bench prints at clevel 5 for this input (reference run here: 20.59)
    out = np.zeros(size + 32, np.uint8)
    n = L.blosc1_compress(5, 1, 4, size, B._p(src), B._p(out), size + 32)
    assert abs(size / n - 20.59) < 0.01


# --------------------------------------------------------------------- special chunks ----
def _chunk(B, fn, nbytes, ts, *extra):
    _bind_specials(B.lib(), B.CParams)
    out = np.zeros(64, np.uint8)
    n = getattr(B.lib(), fn)(B.cparams(typesize=ts), nbytes, B._p(out), 64, *extra)
    return out[:n] if n > 0 else n


def _bind_specials(L, cp_type):
    for fn in ("blosc2_chunk_zeros", "blosc2_chunk_nans", "blosc2_chunk_uninit"):
        getattr(L, fn).argtypes = [cp_type, C.c_int32, C.c_void_p, C.c_int32]
        getattr(L, fn).restype = C.c_int
    L.blosc2_chunk_repeatval.argtypes = [cp_type, C.c_int32, C.c_void_p, C.c_int32, C.c_void_p]
    L.blosc2_chunk_repeatval.restype = C.c_int


@pytest.mark.parametrize("ts,nbytes", [(4, 4 << 20), (8, 1 << 20), (4, 40), (8, 0)])
def test_special_chunks_vs_reference(B, ts, nbytes):
    from b2ctypes import CParams as RefCParams
    L = B.lib()
    _bind_specials(L, B.CParams)
    R = ref()
    if R is not None:
        _bind_specials(R, RefCParams)
    val = np.arange(1, ts + 1, dtype=np.uint8)
    kinds = [("blosc2_chunk_zeros", ()), ("blosc2_chunk_nans", ()), ("blosc2_chunk_uninit", ()),
             ("blosc2_chunk_repeatval", (B._p(val),))]
    for fn, extra in kinds:
        ch = _chunk(B, fn, nbytes, ts, *extra)
        assert isinstance(ch, np.ndarray), (fn, ch)
        if R is not None:
            rout = np.zeros(64, np.uint8)
            rn = getattr(R, fn)(ref_cparams(typesize=ts), nbytes, p(rout), 64, *((p(val),) if extra else ()))
            assert rn == ch.nbytes and np.array_equal(rout[:rn], ch), fn
        dec = B.decompress(ch, nbytes)
        if fn == "blosc2_chunk_repeatval" and nbytes == 0:
            # read_chunk_header refuses a VALUE chunk whose typesize exceeds nbytes (blosc2.c:808-811)
            assert dec == -11, dec
            if R is not None:
                from b2ctypes import dparams as rdp
                dctx = R.blosc2_create_dctx(rdp())
                tmp = np.zeros(8, np.uint8)
                assert R.blosc2_decompress_ctx(dctx, p(ch), ch.nbytes, p(tmp), 0) == -11
                R.blosc2_free_ctx(dctx)
            continue
        assert isinstance(dec, np.ndarray), (fn, dec)
        if fn == "blosc2_chunk_zeros":
            assert not dec.any()
        elif fn == "blosc2_chunk_nans" and nbytes:
            f = dec.view(np.float32 if ts == 4 else np.float64)
            assert np.isnan(f).all()
        elif fn == "blosc2_chunk_repeatval":
            assert np.array_equal(dec, np.tile(val, nbytes // ts))
        if fn != "blosc2_chunk_uninit":
            want = oracle_decompress(ch, nbytes)
            assert isinstance(want, np.ndarray) and np.array_equal(dec, want), fn


def test_special_chunk_header_checks(B):
    """read_chunk_header rejects a VALUE chunk without its value (cbytes 32 -> typesize 0) and with
    nbytes % typesize != 0; set_nans rejects typesize other than 4 / 8."""
    val = np.arange(4, dtype=np.uint8)
    ch = _chunk(B, "blosc2_chunk_repeatval", 4096, 4, B._p(val))
    bad = ch.copy()
    bad[12:16] = np.frombuffer(np.int32(32).tobytes(), np.uint8)   # cbytes = 32: no value bytes
    assert B.decompress(bad[:32].copy(), 4096) < 0
    bad = ch.copy()
    bad[4:8] = np.frombuffer(np.int32(4094).tobytes(), np.uint8)   # nbytes not a multiple of 4
    assert B.decompress(bad, 4096) < 0
    nan2 = _chunk(B, "blosc2_chunk_nans", 4096, 2)
    assert isinstance(nan2, np.ndarray)
    assert B.decompress(nan2, 4096) == -3   # BLOSC2_ERROR_DATA (set_nans: unsupported typesize)


# ---------------------------------------------------------------------- concurrency ----
def test_distinct_contexts_on_threads(B):
    """Two host threads, each with its own compression and decompression context, hammering the
    device at the same time: every chunk stays byte-identical to the oracle."""
    L = B.lib()
    inputs = [(gen_f32(7 + 1000 * k, 1 << 18), 4) for k in range(3)] + \
             [(int64_ramp(5 + k, 1 << 17), 8) for k in range(3)] + [(mixed_bytes(3 + k, 700_000), 1) for k in range(2)]
    want = [oracle_compress(a, clevel=5, typesize=ts) for a, ts in inputs]
    errors = []

    def worker(tid):
        try:
            for it in range(6):
                k = (tid + it) % len(inputs)
                a, ts = inputs[k]
                cctx = L.blosc2_create_cctx(B.cparams(clevel=5, typesize=ts))
                dctx = L.blosc2_create_dctx(B.dparams())
                got = B.compress_ctx(cctx, a)
                if not (isinstance(got, np.ndarray) and np.array_equal(got, want[k])):
                    errors.append(("compress", tid, it))
                back = B.decompress_ctx(dctx, got, a.nbytes) if isinstance(got, np.ndarray) else None
                if back is None or not np.array_equal(back, a.view(np.uint8).reshape(-1)):
                    errors.append(("decompress", tid, it))
                L.blosc2_free_ctx(cctx)
                L.blosc2_free_ctx(dctx)
        except Exception as e:  # pragma: no cover
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_batches_on_two_streams_share_workspace(B):
    """compress on stream A, then immediately a decompression of other chunks on stream B through
    the same default workspace: the second call waits for the first's kernels on the device."""
    import torch
    dev = torch.device("cuda")
    chunk, n = 1 << 20, 64
    a = torch.from_numpy(gen_f32(0, n * chunk // 4).view(np.uint8)).to(dev)
    b = torch.from_numpy(int64_ramp(3, n * chunk // 8).view(np.uint8)).to(dev)
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    ca = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    cb = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    sa = torch.zeros(n, dtype=torch.int32, device=dev)
    sb = torch.zeros(n, dtype=torch.int32, device=dev)
    cpa, cpb = B.cparams(clevel=5, typesize=4), B.cparams(clevel=5, typesize=8, filters=(0, 0, 0, 0, 3, 1))
    B.compress_batch(cpb, b.data_ptr(), chunk, n, chunk, cb.data_ptr(), stride, cap, sb.data_ptr(), 0)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outb = torch.zeros_like(b)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    for _ in range(3):
        B.compress_batch(cpa, a.data_ptr(), chunk, n, chunk, ca.data_ptr(), stride, cap, sa.data_ptr(), s1.cuda_stream)
        B.decompress_batch(cb.data_ptr(), stride, sb.data_ptr(), n, outb.data_ptr(), chunk, chunk, st.data_ptr(),
                           s2.cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(outb, b) and bool((st == chunk).all())
    host = ca.cpu().numpy()
    sizes = sa.cpu().numpy()
    for i in (0, 17, n - 1):
        want = oracle_compress(a[i * chunk:(i + 1) * chunk].cpu().numpy(), clevel=5, typesize=4)
        assert np.array_equal(host[i * stride:i * stride + sizes[i]], want), i


def test_strided_decompress_is_stream_ordered(B):
    """b2h_decompress_batch returns while earlier work on its stream is still running (no host
    synchronisation inside the call), and the result is right once the stream drains."""
    import torch
    dev = torch.device("cuda")
    chunk, n = 1 << 20, 32
    a = torch.from_numpy(gen_f32(11, n * chunk // 4).view(np.uint8)).to(dev)
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    comp = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    cbytes = torch.zeros(n, dtype=torch.int32, device=dev)
    out = torch.zeros_like(a)
    status = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    B.compress_batch(B.cparams(clevel=5, typesize=4), a.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap,
                     cbytes.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000_000)          # ~0.1 s of device time queued ahead of the call
    B.decompress_batch(comp.data_ptr(), stride, cbytes.data_ptr(), n, out.data_ptr(), chunk, chunk,
                       status.data_ptr(), s.cuda_stream)
    assert not s.query(), "the call waited for the stream"
    torch.cuda.synchronize()
    assert torch.equal(out, a) and bool((status == chunk).all())


def test_pack_unpack_chunks(B):
    """b2h_pack_chunks / b2h_unpack_chunks against a plain index gather (ragged sizes, empties)."""
    import torch
    dev = torch.device("cuda")
    rng = np.random.default_rng(5)
    n, stride = 300, 4096 + 256
    sizes = rng.integers(0, stride + 1, n).astype(np.int32)
    sizes[::17] = 0
    buf = torch.from_numpy(rng.integers(0, 256, n * stride, dtype=np.uint8)).to(dev)
    d_sizes = torch.from_numpy(sizes).to(dev)
    total = int(sizes.sum())
    packed = torch.empty(total + 1, dtype=torch.uint8, device=dev)
    offs = torch.empty(n + 1, dtype=torch.int64, device=dev)
    B.pack_chunks(buf.data_ptr(), stride, d_sizes.data_ptr(), n, packed.data_ptr(), offs.data_ptr(), 0)
    torch.cuda.synchronize()
    want_off = np.concatenate([[0], np.cumsum(sizes.astype(np.int64))])
    assert np.array_equal(offs.cpu().numpy(), want_off)
    h = buf.cpu().numpy()
    want = np.concatenate([h[i * stride:i * stride + sizes[i]] for i in range(n)])
    assert np.array_equal(packed[:total].cpu().numpy(), want)
    back = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    got_sizes = torch.zeros(n, dtype=torch.int32, device=dev)
    B.unpack_chunks(packed.data_ptr(), offs.data_ptr(), n, back.data_ptr(), stride, got_sizes.data_ptr(), 0)
    torch.cuda.synchronize()
    assert np.array_equal(got_sizes.cpu().numpy(), sizes)
    bh = back.cpu().numpy()
    for i in range(n):
        assert np.array_equal(bh[i * stride:i * stride + sizes[i]], h[i * stride:i * stride + sizes[i]]), i


# ------------------------------------------------------------------ resource lifetime ----
def test_free_resources_then_reuse(B):
    """blosc2_free_resources (ref include/blosc2.h:872, blosc/blosc2.c:6001-6006) releases the
    engine's device scratch; the next call re-creates it.  Before blosc2_init it fails."""
    L = B.lib()
    L.blosc2_free_resources.restype = C.c_int
    src = gen_f32(3, 1 << 18)
    want = oracle_compress(src, clevel=5, typesize=4)
    L.blosc2_init()
    L.blosc1_set_compressor(b"blosclz")   # the global API's settings (other tests change them)
    L.blosc1_set_blocksize(C.c_size_t(0))
    L.blosc1_set_splitmode(4)
    L.blosc2_set_delta(0)
    for _ in range(2):
        out = np.zeros(src.nbytes + 32, np.uint8)
        n = L.blosc2_compress(5, 1, 4, B._p(src), src.nbytes, B._p(out), out.nbytes)
        assert n == want.nbytes and np.array_equal(out[:n], want)
        assert L.blosc2_free_resources() == 0
    L.blosc2_destroy()
    assert L.blosc2_free_resources() == -1   # BLOSC2_ERROR_FAILURE: not initialised
    L.blosc2_init()
