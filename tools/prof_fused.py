"""Per-phase clock of the fused fast encoder launch (diagnostics; a -DB2H_SEG_PROF build of the
library, e.g. B2H_LIB=c-blosc2_amd/lib_prof/libblosc2_fprof.so): where the wave pairs' time goes --
filter jobs (and the DS job's two passes), ready-word waits, stream encodes.
    B2H_LIB=... python tools/prof_fused.py {T|C4} [nchunks]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

wl = sys.argv[1] if len(sys.argv) > 1 else "C4"
nch = int(sys.argv[2]) if len(sys.argv) > 2 else (10000 if wl == "C4" else 1024)
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
cp = B.cparams(clevel=5, typesize=ts, filters=filters, lz_mode=1)
L = B.lib()
prof = np.zeros(32, np.uint64)
for it in range(3):
    L.b2h_debug_seg_prof(C.c_void_p(prof.ctypes.data))   # reset
    B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
    torch.cuda.synchronize()
    L.b2h_debug_seg_prof(C.c_void_p(prof.ctypes.data))
p = prof.astype(np.float64)
jobs, streams = max(p[20], 1), max(p[21], 1)
print(f"{wl}: {int(p[20])} filter jobs, {int(p[21])} streams encoded (per launch)")
print(f"  job cycles total {p[16] / 1e9:.3f} G (mean {p[16] / jobs:.0f}; store drain {p[19] / jobs:.0f}; "
      f"DS verdict pass {p[22] / jobs:.0f}, store pass {p[23] / jobs:.0f})")
print(f"  ready-word waits {p[17] / 1e9:.3f} G cycles; stream encodes {p[18] / 1e9:.3f} G (mean {p[18] / streams:.0f})")
