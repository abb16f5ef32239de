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
cp = B.cparams(clevel=5, typesize=4)
L = B.lib()
L.b2h_enable_timing(1)
for _ in range(2):
    B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
torch.cuda.synchronize()
print("times", B.last_times())
ns = nch * 16 * 4
rec = np.zeros(ns, dtype=[("kind", "i4"), ("size", "i4"), ("peak", "i4"), ("windows", "i4"), ("cycles", "i8")])
L.b2h_debug_stream_results.argtypes = [C.c_void_p, C.c_int32]
assert L.b2h_debug_stream_results(rec.ctypes.data, ns) == ns
plane = np.arange(ns) % 4
for p in range(4):
    r = rec[plane == p]
    print(f"plane {p}: kinds {np.bincount(r['kind'], minlength=4).tolist()} size mean {r['size'].mean():.0f} "
          f"windows mean {r['windows'].mean():.0f} max {r['windows'].max()} cycles mean {r['cycles'].mean():.0f} "
          f"max {r['cycles'].max()} cyc/window {r['cycles'].sum() / max(1, r['windows'].sum()):.0f}")
