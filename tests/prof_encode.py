"""Encoder diagnostics (not a test): per-stream windows and cycles on the T workload."""
import ctypes as C, os, sys, time
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE); sys.path.insert(0, os.path.join(os.path.dirname(HERE), "c-blosc2_amd"))
import torch
import blosc2_amd as B
sys.path.insert(0, os.path.dirname(HERE))
from bench import gen_f32_device

nch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
chunk = 4 << 20
src = gen_f32_device(0, nch * chunk // 4, torch.device("cuda", 0)).view(torch.uint8)
stride = chunk + 256
dst = torch.empty(nch * stride, dtype=torch.uint8, device="cuda")
cb = torch.zeros(nch, dtype=torch.int32, device="cuda")
cp = B.cparams(clevel=5, typesize=4, lz_mode=int(sys.argv[2]) if len(sys.argv) > 2 else None)
L = B.lib()
L.b2h_enable_timing(1)
for _ in range(2):
    B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
torch.cuda.synchronize()
print("times", B.last_times())
ns = nch * 16 * 4
rec = np.zeros(ns, dtype=[("kind", "i4"), ("size", "i4"), ("peak", "i4"), ("windows", "i4"), ("cycles", "i8"), ("t0", "i8")])
L.b2h_debug_stream_results.argtypes = [C.c_void_p, C.c_int32]
assert L.b2h_debug_stream_results(rec.ctypes.data, ns) == ns
plane = np.arange(ns) % 4
glb = (rec["windows"] >> 30) & 1
rec["windows"] &= (1 << 30) - 1
for p in range(4):
    for t, name in ((0, "lds"), (1, "glb")):
        r = rec[(plane == p) & (glb == t)]
        if r.size:
            print(f"  plane {p} {name}: streams {r.size} cycles mean {r['cycles'].mean():.0f} "
                  f"cyc/window {r['cycles'].sum() / max(1, r['windows'].sum()):.0f}")
for p in range(4):
    r = rec[plane == p]
    print(f"plane {p}: kinds {np.bincount(r['kind'], minlength=4).tolist()} size mean {r['size'].mean():.0f} "
          f"windows mean {r['windows'].mean():.0f} max {r['windows'].max()} cycles mean {r['cycles'].mean():.0f} "
          f"max {r['cycles'].max()} cyc/window {r['cycles'].sum() / max(1, r['windows'].sum()):.0f}")

# occupancy reconstruction from start/end stamps (s_memtime is chip-global on gfx950)
rec2 = np.zeros(ns, dtype=[("kind", "i4"), ("size", "i4"), ("peak", "i4"), ("windows", "i4"), ("cycles", "i8"), ("t0", "i8")])
assert L.b2h_debug_stream_results(rec2.ctypes.data, ns) == ns

# occupancy from 100 MHz realtime stamps: t_start = (rt0 << 24) | duration
raw = rec2["t0"].astype(np.uint64)
rt0 = (raw >> np.uint64(24)).astype(np.int64)
dur = (raw & np.uint64(0xffffff)).astype(np.int64)
s0 = rt0 - rt0.min(); s1 = s0 + dur
ev = np.concatenate([np.stack([s0, np.ones(ns)], 1), np.stack([s1, -np.ones(ns)], 1)])
ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
act = np.cumsum(ev[:, 1])
print(f"realtime span {s1.max()/100:.0f} us, max concurrent {act.max():.0f}, avg concurrent {dur.sum()/s1.max():.1f}")
for p in range(4):
    print(f"plane {p} mean duration {dur[plane == p].mean()/100:.1f} us")
bins = 20
edges = np.linspace(0, s1.max(), bins + 1)
conc = [int(((s0 < edges[i + 1]) & (s1 > edges[i])).sum()) for i in range(bins)]
started = [int(((s0 >= edges[i]) & (s0 < edges[i + 1])).sum()) for i in range(bins)]
print("overlapping per bin:", conc)
print("started per bin:", started)
order = np.argsort(s0)
print("first 8 starts (us):", (s0[order[:8]] / 100).tolist(), "stream ids", order[:8].tolist())
print("start of stream id quantiles:", [int(s0[min(ns - 1, q)] / 100) for q in (0, 1024, 2048, 4096, 8192, 12288, ns - 1)])
