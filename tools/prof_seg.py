"""BloscLZ mode 3 phase profile (not a test; needs a -DB2H_SEG_PROF build in B2H_LIB): per-phase
cycle sums per stream over one T batch.
    B2H_LIB=variants/libblosc2_segprof.so python tools/prof_seg.py [nchunks]"""
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

nch = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
chunk = 4 << 20
src = gen_f32_device(0, nch * chunk // 4, dev).view(torch.uint8)
stride = chunk + 256
dst = torch.empty(nch * stride, dtype=torch.uint8, device=dev)
cb = torch.zeros(nch, dtype=torch.int32, device=dev)
cp = B.cparams(clevel=5, typesize=4, filters=(0, 0, 0, 0, 0, 1), lz_mode=3)
L = B.lib()
L.b2h_debug_seg_prof.argtypes = [C.c_void_p]
buf = np.zeros(32, np.uint64)
B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
torch.cuda.synchronize()
L.b2h_debug_seg_prof(buf.ctypes.data)
L.b2h_enable_timing(1)
B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
torch.cuda.synchronize()
L.b2h_debug_seg_prof(buf.ctypes.data)
print("times:", B.last_times())
ns = int(buf[17])
for name, b in (("probe", 0), ("emit", 8)):
    npass = max(int(buf[b + 4]), 1)
    print(f"{name}: passes {npass}, per pass: candidates {buf[b] / npass:9.0f} cyc, counting walks {buf[b + 1] / npass:9.0f}, "
          f"emitting walk {buf[b + 2] / npass:9.0f}, rounds {buf[b + 3] / npass:.2f}, max steps/lane {buf[b + 5] / npass:.1f}")
print(f"run tests: {ns} streams, {buf[16] / max(ns, 1):.0f} cyc each")
for name, b in (("counting walks", 20), ("emitting walk", 24)):
    print(f"{name} (all passes, wave-cycles): record+literal skip {buf[b]:.3e}, lane match end {buf[b + 1]:.3e}, "
          f"wave extensions {buf[b + 2]:.3e} ({buf[b + 3]} of them)")
