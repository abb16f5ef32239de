"""Headline benchmark: device-resident GiB/s compress+decompress, float32 shuffle+BloscLZ.

Workload (BASELINE.json / SURVEY.md §8d config "T"): float32, typesize 4, filters = SHUFFLE,
BloscLZ clevel 5, stune blocksize (256 KiB), 4 MiB chunks x 1024 = 4 GiB per GPU, gen_f32 data.
One step = compress every chunk of the rank's shard with b2h_compress_batch and decompress them
all again with b2h_decompress_batch; inputs and outputs stay in HBM.  Weak scaling: every rank
owns 4 GiB (global element offset rank*N); for N > 1 rank 0 builds the whole super-chunk input
and RCCL-scatters the shards over xGMI (timed separately, excluded from `value`).

    python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import ctypes as C
import json
import re
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import blosc2_amd as B  # noqa: E402

MASK64 = (1 << 64) - 1
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def _lsr(x, k):
    """logical right shift of int64 tensors holding uint64 bit patterns"""
    return (x >> k) & ((1 << (64 - k)) - 1)


def gen_f32_device(start, count, device):
    """gen_f32 on the GPU: same formula as tests/datagen.py:gen_f32 (device sinf may
    differ from numpy in the last ulp; the data is synthetic either way)."""
    out = torch.empty(count, dtype=torch.float32, device=device)
    step = 1 << 26
    c1 = np.int64(np.uint64(0x9E3779B97F4A7C15).view(np.int64))
    c2 = np.int64(np.uint64(0xBF58476D1CE4E5B9).view(np.int64))
    c3 = np.int64(np.uint64(0x94D049BB133111EB).view(np.int64))
    for s in range(0, count, step):
        n = min(step, count - s)
        g = torch.arange(start + s, start + s + n, dtype=torch.int64, device=device)
        x = (g ^ 1234) + int(c1)
        z = (x ^ _lsr(x, 30)) * int(c2)
        z = (z ^ _lsr(z, 27)) * int(c3)
        z = z ^ _lsr(z, 31)
        noise = _lsr(z, 40).to(torch.float32) * np.float32(2.0 ** -24) * np.float32(0.01)
        ph = (g % 4096).to(torch.float32) * np.float32(2 * np.pi / 4096)
        out[s:s + n] = (np.float32(20) + np.float32(5) * torch.sin(ph) + noise)
    return out


def _cpu_roundtrip(R, raw, nchunks, chunk_nbytes, threads, reps):
    """Median-of-`reps` compress and decompress seconds of the reference library over `nchunks`
    chunks of `raw` with blosc2_compress_ctx / blosc2_decompress_ctx (nthreads = threads)."""
    import oracle_lib
    out = np.zeros(chunk_nbytes + 64, np.uint8)
    tc, td = [], []
    for _ in range(reps):
        outs = []
        if R is not None:
            from b2ctypes import cparams as rcp, dparams as rdp
            cctx = R.blosc2_create_cctx(rcp(clevel=5, typesize=4, nthreads=threads))
            dctx = R.blosc2_create_dctx(rdp(nthreads=threads))
            t0 = time.perf_counter()
            for i in range(nchunks):
                n = R.blosc2_compress_ctx(cctx, C.c_void_p(raw.ctypes.data + i * chunk_nbytes), chunk_nbytes,
                                          C.c_void_p(out.ctypes.data), chunk_nbytes + 32)
                outs.append(out[:n].copy())
            t1 = time.perf_counter()
            dec = np.empty(chunk_nbytes, np.uint8)
            for ch in outs:
                R.blosc2_decompress_ctx(dctx, C.c_void_p(ch.ctypes.data), ch.nbytes,
                                        C.c_void_p(dec.ctypes.data), chunk_nbytes)
            t2 = time.perf_counter()
            R.blosc2_free_ctx(cctx)
            R.blosc2_free_ctx(dctx)
        else:
            src = raw.view(np.float32)
            t0 = time.perf_counter()
            for i in range(nchunks):
                outs.append(oracle_lib.oracle_compress(src[i * chunk_nbytes // 4:(i + 1) * chunk_nbytes // 4],
                                                       clevel=5, typesize=4))
            t1 = time.perf_counter()
            for ch in outs:
                oracle_lib.oracle_decompress(ch, chunk_nbytes)
            t2 = time.perf_counter()
        tc.append(t1 - t0)
        td.append(t2 - t1)
    return float(np.median(tc)), float(np.median(td))


def cpu_baseline(nchunks_sample, chunk_nbytes, threads, reps=5):
    """The reference library (oracle/_ref, built from /root/reference sources) timed on the host
    cores on a bounded sample of the same workload (median of `reps`), at nthreads = threads
    (the headline `value`) and at nthreads = 1 on a smaller sample.  Falls back to the oracle
    port (single thread) if the reference build is absent.  Returns dict for the JSON line."""
    from datagen import gen_f32
    import oracle_lib
    R = oracle_lib.ref()
    if R is None:
        threads = 1
    raw = gen_f32(0, nchunks_sample * chunk_nbytes // 4).view(np.uint8)
    nbytes = nchunks_sample * chunk_nbytes
    tc, td = _cpu_roundtrip(R, raw, nchunks_sample, chunk_nbytes, threads, reps)
    n1 = max(1, nchunks_sample // 16)
    tc1, td1 = _cpu_roundtrip(R, raw, n1, chunk_nbytes, 1, max(1, reps // 2))
    b1 = n1 * chunk_nbytes
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(nbytes / (tc + td) / 2 ** 30, 4), "unit": "GiB/s",
            "cores": threads, "kind": "reference" if R is not None else "port",
            "sample": f"{nchunks_sample} x {chunk_nbytes >> 20} MiB gen_f32 chunks (same cparams), median of "
                      f"{reps}: compress {nbytes / tc / 2**30:.3f} GiB/s + decompress {nbytes / td / 2**30:.3f} GiB/s "
                      f"at nthreads={threads}; nthreads=1 on {n1} chunks: "
                      f"{b1 / (tc1 + td1) / 2**30:.3f} GiB/s (c {b1 / tc1 / 2**30:.3f}, d {b1 / td1 / 2**30:.3f}); "
                      f"host CPU: {cpu}"}


def pmc_traffic(kernel, workload):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary of this workload
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from the FETCH_SIZE/WRITE_SIZE
    rocprofv3 passes over this same bench command); (None, None) when there is none."""
    import glob
    best = None
    def version(f):   # r1_v8_pmc_traffic.json -> (1, 8): newest round/version wins (mtimes do not survive a checkout)
        return tuple(int(x) for x in re.findall(r"\d+", os.path.basename(f).split("_pmc")[0]))
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), key=version):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        for k, v in d.get("kernels", {}).items():
            if k.split("<")[0].endswith(kernel) and "hbm_bytes_per_launch" in v:
                best = (v["hbm_bytes_per_launch"], os.path.basename(f))
    return best if best else (None, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=1024)
    ap.add_argument("--chunk-mib", type=int, default=4)
    ap.add_argument("--clevel", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-chunks", type=int, default=256)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    L = B.lib()
    chunk = args.chunk_mib << 20
    nch = args.chunks
    shard = nch * chunk
    stream = torch.cuda.current_stream().cuda_stream

    # ---- input: rank-local shard of the super-chunk (RCCL scatter from rank 0 when N > 1)
    scatter_s = None
    if world > 1:
        recv = torch.empty(shard // 4, dtype=torch.float32, device=dev)
        parts = None
        if rank == 0:
            parts = [gen_f32_device(r * (shard // 4), shard // 4, dev) for r in range(world)]
        dist.barrier()
        torch.cuda.synchronize()
        t = time.perf_counter()
        dist.scatter(recv, parts, src=0)
        torch.cuda.synchronize()
        scatter_s = time.perf_counter() - t
        del parts
        src = recv
    else:
        src = gen_f32_device(0, shard // 4, dev)
    src_u8 = src.view(torch.uint8)

    cap = chunk + 32
    stride = (cap + 255) // 256 * 256
    comp = torch.empty(nch * stride, dtype=torch.uint8, device=dev)
    cbytes = torch.zeros(nch, dtype=torch.int32, device=dev)
    out = torch.empty(shard, dtype=torch.uint8, device=dev)
    status = torch.zeros(nch, dtype=torch.int32, device=dev)
    cp = B.cparams(clevel=args.clevel, typesize=4, filters=(0, 0, 0, 0, 0, B.SHUFFLE))

    def step():
        B.compress_batch(cp, src_u8.data_ptr(), chunk, nch, chunk, comp.data_ptr(), stride, cap,
                         cbytes.data_ptr(), stream)
        B.decompress_batch(comp.data_ptr(), stride, cbytes.data_ptr(), nch, out.data_ptr(), chunk, chunk,
                           status.data_ptr(), stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness of the measured configuration (outside the timed region)
    assert torch.equal(out, src_u8), "round trip mismatch"
    assert bool((status == chunk).all()), "decompress status"
    total_c = int(cbytes.sum().item())

    L.b2h_enable_timing(1)
    enc_ms, dec_ms = [], []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        t = B.last_times()          # waits on this step's events only
        enc_ms.append(t["encode_ms"])
        dec_ms.append(t["decode_ms"])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    L.b2h_enable_timing(0)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())

    if rank == 0:
        n_all = shard * world * args.steps
        value = n_all / elapsed / 2 ** 30
        enc = float(np.mean(enc_ms))
        # dominant kernel: k_encode; algorithmic bytes per launch = N (read) + C (written)
        alg = shard + total_c
        achieved = alg / (enc * 1e-3) / 1e9
        workload = ("T: float32 ts=4 SHUFFLE+BloscLZ clevel 5, 256 KiB blocks, "
                    f"{args.chunk_mib} MiB chunks x {nch} per GPU")
        traffic, traffic_src = pmc_traffic("k_encode", workload)
        res = {
            "metric": "device-resident GiB/s compress+decompress, f32 shuffle+blosclz, 1/2/4/8 GPU",
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic gen_f32 (SURVEY §8d), generated on device",
            "config": {"workload": workload,
                       "chunks_per_gpu": nch, "chunk_bytes": chunk, "clevel": args.clevel,
                       "parallelism": f"chunk-sharded x{world}",
                       "cratio": round(shard / total_c, 4)},
            "roofline": {"bound": "hbm", "kernel": "k_encode", "achieved": round(achieved, 2),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": round(traffic) if traffic else None,
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": alg,
                         "encode_ms": round(enc, 3), "decode_ms": round(float(np.mean(dec_ms)), 3)},
        }
        if scatter_s is not None:
            res["config"]["rccl_scatter_s"] = round(scatter_s, 4)
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample_chunks, chunk, min(16, os.cpu_count() or 1))
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
