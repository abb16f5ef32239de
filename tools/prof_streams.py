"""Per-stream encoder diagnostics (not a test): kind, size, cycles and start time of every stream of
one fast-mode batch, grouped by (block, plane).  Workloads: T (gen_f32, ts 4 SHUFFLE) or C4
(int64 ramp, ts 8 DELTA + SHUFFLE, 1 MiB chunks).
    python tools/prof_streams.py {T|C4} [nchunks] [lz_mode]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "c-blosc2_amd"))
sys.path.insert(0, REPO)
import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
nch = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dev = torch.device("cuda", 0)
if wl == "T":
    chunk, ts, filters = 4 << 20, 4, (0, 0, 0, 0, 0, 1)
    src = gen_f32_device(0, nch * chunk // 4, dev).view(torch.uint8)
else:
    chunk, ts, filters = 1 << 20, 8, (0, 0, 0, 0, 3, 1)
    src = torch.arange(nch * chunk // 8, dtype=torch.int64, device=dev).view(torch.uint8)
stride = chunk + 256
dst = torch.empty(nch * stride, dtype=torch.uint8, device=dev)
cb = torch.zeros(nch, dtype=torch.int32, device=dev)
cp = B.cparams(clevel=5, typesize=ts, filters=filters, lz_mode=mode)
L = B.lib()
L.b2h_enable_timing(1)
for _ in range(3):
    B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
torch.cuda.synchronize()
print("times:", B.last_times())
bs = 256 << 10 if wl == "T" else 512 << 10
nblk = chunk // bs
ns = nch * nblk * ts
rec = np.zeros(ns, dtype=[("kind", "i4"), ("size", "i4"), ("peak", "i4"), ("windows", "i4"), ("cycles", "i8"),
                          ("t0", "i8")])
L.b2h_debug_stream_results.argtypes = [C.c_void_p, C.c_int32]
assert L.b2h_debug_stream_results(rec.ctypes.data, ns) == ns
rec["windows"] &= (1 << 30) - 1
idx = np.arange(ns) % (nblk * ts)
blk, plane = idx // ts, idx % ts
start = (rec["t0"] >> 24).astype(np.int64)
start -= start.min()
dur = rec["t0"] & 0xffffff
kinds = ["zero", "byte", "raw", "lz"]
print(f"{wl}: {nch} chunks, {ns} streams; span {start.max() / 100:.0f} us (100 MHz realtime)")
for b in range(nblk):
    for p in range(ts):
        r = rec[(blk == b) & (plane == p)]
        d = dur[(blk == b) & (plane == p)]
        kc = np.bincount(r["kind"], minlength=4)
        print(f"  block {b} plane {p}: kinds {dict(zip(kinds, kc.tolist()))} size {r['size'].mean():8.0f} "
              f"windows {r['windows'].mean():6.1f} cycles {r['cycles'].mean():9.0f} dur {d.mean() / 100:7.1f} us")
tot = dur.sum() / 100
print(f"stream-us total {tot:.0f}; by kind:", {kinds[k]: round(float(dur[rec['kind'] == k].sum() / 100 / max(tot, 1)), 3)
                                              for k in range(4)})
# concurrency over the launch: streams in flight per 0.5 ms bin (100 MHz realtime), and when the
# last stream of each kind started / ended
end = start + dur
span = int(end.max())
pts = np.arange(25000, span, 50000)
act = [int(((start <= t) & (end > t)).sum()) for t in pts]
print("in flight at 0.25, 0.75, ... ms:", act)
lz = rec["kind"] == 3
print("LZ in flight:", [int(((start <= t) & (end > t) & lz).sum()) for t in pts])
for q in (0.5, 0.9, 0.99):
    print(f"  LZ stream duration p{int(q * 100)}: {np.quantile(dur[lz], q) / 100:.0f} us")
for k in range(4):
    m = rec["kind"] == k
    if m.any():
        print(f"  {kinds[k]}: last start {start[m].max() / 100:.0f} us, last end {end[m].max() / 100:.0f} us")
