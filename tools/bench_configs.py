"""The other BASELINE.json configurations on one MI355X (bench.py measures the headline one, T).
Each prints one JSON line; every run checks its own results.

  C1  b2bench's own config (1e6 int32 get_value(i, 19), 67 x 4 MB, clevel 5 shuffle BloscLZ), GPU
      batch vs the reference library built here at nthreads 1.
  C2  shuffle filter only, ts=4, 256 MiB gen_f32: one blosc2_shuffle over the whole buffer and the
      unshuffle back, bit-exact against the oracle restatement (blosc/shuffle-generic.c).
  C3  bitshuffle + BloscLZ clevel 5, ts=4, 256 KiB blocks x 4096 chunks (1 GiB gen_f32, continuing
      global index): exact round trip; the first chunks byte-identical to the oracle.
  C4  schunk of 10 000 x 1 MiB chunks, DELTA + SHUFFLE + BloscLZ clevel 5, int64 ramp (ts=8, auto
      512 KiB blocks): exact round trip, sample chunks byte-identical to the oracle.
  E2E the T workload from and back to pinned host memory over 3 streams in 64-chunk groups:
      H2D + compress + pack + D2H of the packed compressed bytes, and H2D of those bytes + unpack
      + decompress + D2H (PCIe-inclusive; never `value`); exact host round trip.

    python tools/bench_configs.py [--only C1,C2,C3,C4,E2E,LZ4] [--steps K] [--lz-mode exact|fast|deep]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)
import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

GiB = float(1 << 30)
HBM_PEAK_GBS = 8000.0


def _timed(fn, steps, stream):
    """Average ms of `fn` over `steps` runs after one warmup, HIP events on `stream`."""
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s = torch.cuda.ExternalStream(stream) if stream else torch.cuda.current_stream()
    a.record(s)
    for _ in range(steps):
        fn()
    b.record(s)
    torch.cuda.synchronize()
    return a.elapsed_time(b) / steps


def c2(steps):
    from oracle_lib import oracle, p
    n = 256 << 20
    src = gen_f32_device(0, n // 4, torch.device("cuda")).view(torch.uint8)
    dst = torch.empty_like(src)
    back = torch.empty_like(src)
    L = B.lib()
    st = torch.cuda.current_stream().cuda_stream
    t_s = _timed(lambda: L.b2h_shuffle(4, n, src.data_ptr(), dst.data_ptr(), 0, st), steps, st)
    t_u = _timed(lambda: L.b2h_shuffle(4, n, dst.data_ptr(), back.data_ptr(), 1, st), steps, st)
    host = src.cpu().numpy()
    want = np.empty_like(host)
    oracle().or_shuffle(4, n, p(host), p(want))
    exact = bool(np.array_equal(dst.cpu().numpy(), want)) and bool(torch.equal(back, src))
    return {"config": "C2: shuffle only ts=4, 256 MiB gen_f32, one blosc2_shuffle call", "bit_exact_vs_oracle": exact,
            "shuffle_ms": round(t_s, 4), "unshuffle_ms": round(t_u, 4),
            "shuffle_GiBps": round(n / GiB / (t_s * 1e-3), 2), "unshuffle_GiBps": round(n / GiB / (t_u * 1e-3), 2),
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "achieved_shuffle": round(2 * n / (t_s * 1e-3) / 1e9, 1),
                         "frac_shuffle": round(2 * n / (t_s * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "achieved_unshuffle": round(2 * n / (t_u * 1e-3) / 1e9, 1),
                         "frac_unshuffle": round(2 * n / (t_u * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}


def _batch_roundtrip(name, src_u8, chunk, nch, cp, steps, check):
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    comp = torch.empty(nch * stride, dtype=torch.uint8, device="cuda")
    cb = torch.zeros(nch, dtype=torch.int32, device="cuda")
    out = torch.empty(nch * chunk, dtype=torch.uint8, device="cuda")
    status = torch.zeros(nch, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    enc = lambda: B.compress_batch(cp, src_u8.data_ptr(), chunk, nch, chunk, comp.data_ptr(), stride, cap,  # noqa: E731
                                   cb.data_ptr(), st)
    dec = lambda: B.decompress_batch(comp.data_ptr(), stride, cb.data_ptr(), nch, out.data_ptr(), chunk,  # noqa: E731
                                     chunk, status.data_ptr(), st)
    t_c = _timed(enc, steps, st)
    t_d = _timed(dec, steps, st)
    exact = bool(torch.equal(out, src_u8[:nch * chunk])) and bool((status == chunk).all())
    C = int(cb.sum().item())
    N = nch * chunk
    # fast mode is round-trip identical, not byte-identical: the oracle comparison is exact mode's
    sample_ok = check(comp, cb, stride) if B.lib().b2h_set_blosclz_mode(-1) == 0 else "n/a (fast mode)"
    return {"config": name, "round_trip_exact": exact, "sample_chunks_match_oracle": sample_ok,
            "cratio": round(N / C, 4), "compress_ms": round(t_c, 3), "decompress_ms": round(t_d, 3),
            "GiBps_c_plus_d": round(N / GiB / ((t_c + t_d) * 1e-3), 3),
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "achieved": round(2 * (N + C) / ((t_c + t_d) * 1e-3) / 1e9, 1),
                         "frac": round(2 * (N + C) / ((t_c + t_d) * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)}}


def _oracle_check(src_u8, chunk, idxs, kw):
    from oracle_lib import oracle_compress

    def check(comp, cb, stride):
        cbh = cb.cpu().numpy()
        for i in idxs:
            raw = src_u8[i * chunk:(i + 1) * chunk].cpu().numpy()
            want = oracle_compress(raw, **kw)
            got = comp[i * stride:i * stride + int(cbh[i])].cpu().numpy()
            if not np.array_equal(got, want):
                return False
        return True
    return check


def c3(steps):
    chunk, nch = 256 << 10, 4096
    src = gen_f32_device(0, nch * chunk // 4, torch.device("cuda")).view(torch.uint8)
    kw = dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, B.BITSHUFFLE), blocksize=262144)
    cp = B.cparams(**kw)
    return _batch_roundtrip("C3: BITSHUFFLE+BloscLZ clevel 5 ts=4, 256 KiB blocks x 4096 chunks (gen_f32)",
                            src, chunk, nch, cp, steps, _oracle_check(src, chunk, (0, 1, 2047, 4095), kw))


def c4(steps):
    chunk, nch = 1 << 20, 10000
    src = torch.arange(0, nch * chunk // 8, dtype=torch.int64, device="cuda").view(torch.uint8)
    kw = dict(clevel=5, typesize=8, filters=(0, 0, 0, 0, B.DELTA, B.SHUFFLE))
    cp = B.cparams(**kw)
    return _batch_roundtrip("C4: schunk 10000 x 1 MiB, DELTA+SHUFFLE+BloscLZ clevel 5, int64 ramp",
                            src, chunk, nch, cp, steps, _oracle_check(src, chunk, (0, 1, 5000, 9999), kw))


def e2e(steps, group_chunks=64, nstreams=3):
    """T from pinned host memory and back, PCIe-inclusive, pipelined over `nstreams` streams in
    groups of `group_chunks` chunks.
      compress:   H2D raw group -> b2h_compress_batch -> b2h_pack_chunks (sizes scan + copy) ->
                  D2H of exactly the packed compressed bytes (+ the group's offsets);
      decompress: H2D of the packed bytes from host -> b2h_unpack_chunks -> b2h_decompress_batch
                  -> D2H of the raw group.
    The decompress direction starts from the host copy only (its device buffers are separate and
    zeroed), so the check host-out == host-in proves the compressed bytes crossed PCIe intact.
    Group g's D2H is queued once its offsets are on the host (event wait on the host thread), two
    groups behind the compute, so copies overlap the next groups' kernels."""
    chunk, nch = 4 << 20, 1024
    N = chunk * nch
    G, GN = nch // group_chunks, group_chunks * chunk
    dev = torch.device("cuda")
    h_src = torch.empty(N, dtype=torch.uint8, pin_memory=True)
    h_src.copy_(gen_f32_device(0, N // 4, dev).view(torch.uint8).cpu())
    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    cp = B.cparams(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, B.SHUFFLE))
    streams = [torch.cuda.Stream() for _ in range(nstreams)]

    def bufs():
        return dict(raw=torch.empty(GN, dtype=torch.uint8, device=dev),
                    comp=torch.zeros(group_chunks * stride, dtype=torch.uint8, device=dev),
                    packed=torch.zeros(group_chunks * stride, dtype=torch.uint8, device=dev),
                    cb=torch.zeros(group_chunks, dtype=torch.int32, device=dev),
                    off=torch.zeros(group_chunks + 1, dtype=torch.int64, device=dev),
                    status=torch.zeros(group_chunks, dtype=torch.int32, device=dev))
    cbuf = [bufs() for _ in range(nstreams)]
    dbuf = [bufs() for _ in range(nstreams)]
    h_off = [torch.zeros(group_chunks + 1, dtype=torch.int64, pin_memory=True) for _ in range(G)]
    h_packed = torch.empty(nch * stride, dtype=torch.uint8, pin_memory=True)
    h_out = torch.empty(N, dtype=torch.uint8, pin_memory=True)
    base = [0] * (G + 1)
    statuses = torch.zeros(nch, dtype=torch.int32, device=dev)

    def compress_all():
        evs = [None] * G

        def drain(g):   # the group's compressed bytes to the host, packed
            evs[g].synchronize()
            n = int(h_off[g][group_chunks])
            base[g + 1] = base[g] + n
            k = g % nstreams
            with torch.cuda.stream(streams[k]):
                h_packed[base[g]:base[g] + n].copy_(cbuf[k]["packed"][:n], non_blocking=True)
        for g in range(G):
            k = g % nstreams
            s, b = streams[k], cbuf[k]
            with torch.cuda.stream(s):
                b["raw"].copy_(h_src[g * GN:(g + 1) * GN], non_blocking=True)
                B.compress_batch(cp, b["raw"].data_ptr(), chunk, group_chunks, chunk, b["comp"].data_ptr(), stride, cap,
                                 b["cb"].data_ptr(), s.cuda_stream)
                B.pack_chunks(b["comp"].data_ptr(), stride, b["cb"].data_ptr(), group_chunks, b["packed"].data_ptr(),
                              b["off"].data_ptr(), s.cuda_stream)
                h_off[g].copy_(b["off"], non_blocking=True)
                evs[g] = torch.cuda.Event()
                evs[g].record(s)
            if g >= nstreams - 1:
                drain(g - (nstreams - 1))
        for g in range(max(0, G - (nstreams - 1)), G):
            drain(g)
        torch.cuda.synchronize()

    def decompress_group(g, strs, h_from):
        k = g % nstreams
        s, b = strs[k], dbuf[k]
        n = base[g + 1] - base[g]
        with torch.cuda.stream(s):
            b["packed"][:n].copy_(h_from[base[g]:base[g + 1]], non_blocking=True)
            b["off"].copy_(h_off[g], non_blocking=True)
            B.unpack_chunks(b["packed"].data_ptr(), b["off"].data_ptr(), group_chunks, b["comp"].data_ptr(), stride,
                            b["cb"].data_ptr(), s.cuda_stream)
            B.decompress_batch(b["comp"].data_ptr(), stride, b["cb"].data_ptr(), group_chunks, b["raw"].data_ptr(),
                               chunk, chunk, b["status"].data_ptr(), s.cuda_stream)
            statuses[g * group_chunks:(g + 1) * group_chunks].copy_(b["status"], non_blocking=True)
            h_out[g * GN:(g + 1) * GN].copy_(b["raw"], non_blocking=True)

    dstreams = [torch.cuda.Stream() for _ in range(nstreams)]

    def duplex_all(h_from):
        """Both directions at once: group g compresses (H2D raw, D2H packed) on `streams` while group g
        of the previous pass's packed bytes decompresses (H2D packed, D2H raw) on `dstreams`, so both
        PCIe directions carry traffic together (the sequential passes leave one direction idle)."""
        evs = [None] * G
        done = [0] * (G + 1)

        def drain(g):
            evs[g].synchronize()
            n = int(h_off[g][group_chunks])
            done[g + 1] = done[g] + n
            k = g % nstreams
            with torch.cuda.stream(streams[k]):
                h_packed[done[g]:done[g] + n].copy_(cbuf[k]["packed"][:n], non_blocking=True)
        for g in range(G):
            k = g % nstreams
            s, b = streams[k], cbuf[k]
            with torch.cuda.stream(s):
                b["raw"].copy_(h_src[g * GN:(g + 1) * GN], non_blocking=True)
                B.compress_batch(cp, b["raw"].data_ptr(), chunk, group_chunks, chunk, b["comp"].data_ptr(), stride, cap,
                                 b["cb"].data_ptr(), s.cuda_stream)
                B.pack_chunks(b["comp"].data_ptr(), stride, b["cb"].data_ptr(), group_chunks, b["packed"].data_ptr(),
                              b["off"].data_ptr(), s.cuda_stream)
                h_off2[g].copy_(b["off"], non_blocking=True)
                evs[g] = torch.cuda.Event()
                evs[g].record(s)
            decompress_group(g, dstreams, h_from)
            if g >= nstreams - 1:
                drain(g - (nstreams - 1))
        for g in range(max(0, G - (nstreams - 1)), G):
            drain(g)
        torch.cuda.synchronize()
        return done[G]

    def decompress_all():
        for g in range(G):
            k = g % nstreams
            s, b = streams[k], dbuf[k]
            n = base[g + 1] - base[g]
            with torch.cuda.stream(s):
                b["packed"][:n].copy_(h_packed[base[g]:base[g + 1]], non_blocking=True)
                b["off"].copy_(h_off[g], non_blocking=True)
                B.unpack_chunks(b["packed"].data_ptr(), b["off"].data_ptr(), group_chunks, b["comp"].data_ptr(), stride,
                                b["cb"].data_ptr(), s.cuda_stream)
                B.decompress_batch(b["comp"].data_ptr(), stride, b["cb"].data_ptr(), group_chunks, b["raw"].data_ptr(),
                                   chunk, chunk, b["status"].data_ptr(), s.cuda_stream)
                statuses[g * group_chunks:(g + 1) * group_chunks].copy_(b["status"], non_blocking=True)
                h_out[g * GN:(g + 1) * GN].copy_(b["raw"], non_blocking=True)
        torch.cuda.synchronize()

    compress_all()   # warmup (and the sizes)
    decompress_all()
    tc, td = [], []
    for _ in range(steps):
        h_out.zero_()
        for b in dbuf:
            b["comp"].zero_()
            b["packed"].zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        compress_all()
        t1 = time.perf_counter()
        decompress_all()
        t2 = time.perf_counter()
        tc.append(t1 - t0)
        td.append(t2 - t1)
    C = base[G]
    exact = bool(torch.equal(h_out, h_src)) and bool((statuses == chunk).all())
    tcm, tdm = float(np.median(tc)), float(np.median(td))
    # duplex: compress and decompress of the whole workload together (the decompress side reads a
    # copy of the packed bytes, the compress side rewrites h_packed; the duplex's compressed bytes
    # and offsets are compared with the sequential pass's afterwards)
    h_from = h_packed[:C].clone().pin_memory()
    h_off2 = [torch.zeros(group_chunks + 1, dtype=torch.int64, pin_memory=True) for _ in range(G)]
    tdup = []
    dup_exact = True
    for _ in range(steps):
        h_out.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        C2 = duplex_all(h_from)
        tdup.append(time.perf_counter() - t0)
        dup_exact = dup_exact and C2 == C and bool(torch.equal(h_out, h_src)) and bool((statuses == chunk).all()) \
            and bool(torch.equal(h_packed[:C], h_from)) and all(torch.equal(a, b) for a, b in zip(h_off, h_off2))
    tdupm = float(np.median(tdup))
    mode = {0: "exact", 1: "fast", 2: "deep", 3: "seg"}[B.lib().b2h_set_blosclz_mode(-1)]
    return {"config": f"E2E: T from/to pinned host memory, {nstreams} streams x groups of {group_chunks} chunks "
                      "(H2D + compress + pack + D2H of the packed bytes; H2D of the packed bytes + unpack + "
                      "decompress + D2H)", "blosclz_mode": mode,
            "round_trip_exact": exact, "compressed_bytes_over_pcie": C, "cratio": round(N / C, 4),
            "compress_GiBps": round(N / GiB / tcm, 3), "decompress_GiBps": round(N / GiB / tdm, 3),
            "GiBps_c_plus_d": round(N / GiB / (tcm + tdm), 3),
            "pcie_bytes_per_s": {"compress": round((N + C) / tcm / 1e9, 2), "decompress": round((N + C) / tdm / 1e9, 2),
                                 "unit": "GB/s (H2D + D2H bytes / wall)"},
            "duplex": {"what": "compress and decompress of the workload overlapped (both PCIe directions busy)",
                       "round_trip_exact": dup_exact, "ms": round(tdupm * 1e3, 2),
                       "GiBps_c_plus_d": round(N / GiB / tdupm, 3),
                       "pcie_GBps_both_directions": round(2 * (N + C) / tdupm / 1e9, 2)}}


def c1(steps, nchunks=67, clevel=5):
    """C1, the reference's own headline CPU benchmark (`b2bench blosclz shuffle single 1 4000000 4
    19`, bench/b2bench.c:105-274): 1e6 int32 get_value(i, 19) (b2bench.c:73-81), the same 4 MB
    buffer compressed into 67 chunks (the 256 MiB working set), clevel 5, SHUFFLE, ts 4, BloscLZ.
    GPU: one batch over the 67 chunks (src_stride 0: every chunk reads the same buffer); CPU: the
    reference library built here (oracle/_ref), nthreads 1, as b2bench runs it.  MB/s = 1e6 B/s."""
    from datagen import b2bench_values
    from oracle_lib import oracle_compress, p, ref
    size = 4_000_000
    src = b2bench_values(1_000_000, 19)
    cap = size + 32
    stride = (cap + 255) // 256 * 256
    d_src = torch.from_numpy(src.view(np.uint8).copy()).cuda()
    comp = torch.empty(nchunks * stride, dtype=torch.uint8, device="cuda")
    cb = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    out = torch.empty(nchunks * size, dtype=torch.uint8, device="cuda")
    status = torch.zeros(nchunks, dtype=torch.int32, device="cuda")
    cp = B.cparams(clevel=clevel, typesize=4, filters=(0, 0, 0, 0, 0, B.SHUFFLE))
    st = torch.cuda.current_stream().cuda_stream
    t_c = _timed(lambda: B.compress_batch(cp, d_src.data_ptr(), size, nchunks, 0, comp.data_ptr(), stride, cap,
                                          cb.data_ptr(), st), steps, st)
    t_d = _timed(lambda: B.decompress_batch(comp.data_ptr(), stride, cb.data_ptr(), nchunks, out.data_ptr(), size,
                                            size, status.data_ptr(), st), steps, st)
    cbh = cb.cpu().numpy()
    want = oracle_compress(src, clevel=clevel, typesize=4, filters=(0, 0, 0, 0, 0, 1))
    chunk0 = comp[:int(cbh[0])].cpu().numpy()
    exact = bool((status == size).all()) and bool(torch.equal(out.view(nchunks, size)[nchunks - 1], d_src))
    res = {"config": "C1: b2bench blosclz shuffle single 1 4000000 4 19 (67 x 4 MB, clevel 5)",
           "chunk_matches_oracle": bool(np.array_equal(chunk0, want)), "round_trip_exact": exact,
           "cratio": round(size / float(cbh[0]), 2),
           "gpu_compress_MBps": round(nchunks * size / (t_c * 1e-3) / 1e6, 1),
           "gpu_decompress_MBps": round(nchunks * size / (t_d * 1e-3) / 1e6, 1)}
    # the drop-in per-call path, as b2bench calls it (bench/b2bench.c:199, 227): blosc1_compress /
    # blosc1_decompress on HOST buffers, one 4 MB chunk per call (each call: H2D, one launch chain,
    # D2H, synchronise) -- SURVEY §7 hard part 5, the single-chunk latency
    L = B.lib()
    L.blosc1_set_compressor(b"blosclz")
    hsrc = src.copy()
    hdst = np.zeros((nchunks, cap), np.uint8)
    hback = np.zeros(size, np.uint8)
    n0 = L.blosc1_compress(clevel, 1, 4, size, p(hsrc), p(hdst[0]), cap)   # warm-up (context, buffers)
    L.blosc1_decompress(p(hdst[0]), p(hback), size)
    pc, pd = [], []
    for _ in range(3):
        t0 = time.perf_counter()
        for i in range(nchunks):
            L.blosc1_compress(clevel, 1, 4, size, p(hsrc), p(hdst[i]), cap)
        t1 = time.perf_counter()
        for i in range(nchunks):
            L.blosc1_decompress(p(hdst[i]), p(hback), size)
        t2 = time.perf_counter()
        pc.append(t1 - t0)
        pd.append(t2 - t1)
    res["gpu_per_call_host_buffers"] = {
        "compress_MBps": round(nchunks * size / float(np.median(pc)) / 1e6, 1),
        "decompress_MBps": round(nchunks * size / float(np.median(pd)) / 1e6, 1),
        "compress_ms_per_call": round(float(np.median(pc)) / nchunks * 1e3, 3),
        "decompress_ms_per_call": round(float(np.median(pd)) / nchunks * 1e3, 3),
        "chunk_bytes_equal_batch": bool(n0 == int(cbh[0]) and np.array_equal(hdst[0][:n0], chunk0)),
        "round_trip_exact": bool(np.array_equal(hback, src.view(np.uint8))),
        "note": "product blosc1_compress / blosc1_decompress per 4 MB host chunk (PCIe both ways inside "
                "every call), median of 3 passes over the 67 chunks"}
    R = ref()
    if R is not None:
        R.blosc1_set_compressor(b"blosclz")
        R.blosc2_set_nthreads(1)
        rsrc = src.copy()
        dst = np.zeros((nchunks, cap), np.uint8)
        back = np.zeros(size, np.uint8)
        tc, td = [], []
        for _ in range(3):
            t0 = time.perf_counter()
            for i in range(nchunks):
                n = R.blosc1_compress(clevel, 1, 4, size, p(rsrc), p(dst[i]), cap)
            t1 = time.perf_counter()
            for i in range(nchunks):
                R.blosc1_decompress(p(dst[i]), p(back), size)
            t2 = time.perf_counter()
            tc.append(t1 - t0)
            td.append(t2 - t1)
        res["cpu_reference_nthreads1"] = {
            "compress_MBps": round(nchunks * size / float(np.median(tc)) / 1e6, 1),
            "decompress_MBps": round(nchunks * size / float(np.median(td)) / 1e6, 1),
            "chunk_bytes_equal_gpu": bool(n == int(cbh[0]) and np.array_equal(dst[0][:n], chunk0)),
            "note": "oracle/_ref, blosc1_compress / blosc1_decompress per chunk, median of 3"}
    return res


def lz4t(steps):
    """T's workload with the LZ4 codec: float32 ts=4 SHUFFLE+LZ4 clevel 5,
    256 KiB blocks (4 x 64 KiB streams), 4 MiB chunks x 1024."""
    chunk, nch = 4 << 20, 1024
    src = gen_f32_device(0, nch * chunk // 4, torch.device("cuda")).view(torch.uint8)
    kw = dict(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, B.SHUFFLE), compcode=1)
    cp = B.cparams(**kw)
    return _batch_roundtrip("T-LZ4: float32 ts=4 SHUFFLE+LZ4 clevel 5, 256 KiB blocks, 4 MiB x 1024 (gen_f32)",
                            src, chunk, nch, cp, steps, _oracle_check(src, chunk, (0, 1, 511, 1023), kw))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C1,C2,C3,C4,E2E,LZ4")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--lz-mode", default="exact", choices=["exact", "fast", "deep", "seg"])
    args = ap.parse_args()
    torch.cuda.set_device(0)
    B.lib().b2h_set_blosclz_mode({"exact": 0, "fast": 1, "deep": 2, "seg": 3}[args.lz_mode])
    for name in args.only.split(","):
        r = {"C1": c1, "C2": c2, "C3": c3, "C4": c4, "E2E": e2e, "LZ4": lz4t}[name](args.steps)
        print(json.dumps(r), flush=True)
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
