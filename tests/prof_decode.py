"""Decoder diagnostics (not a test): per-stream decode cycles by stream kind on the T workload.
Run with B2H_DECODE_DEBUG=1 on a GPU box:  B2H_DECODE_DEBUG=1 python tests/prof_decode.py 256"""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "c-blosc2_amd"))
sys.path.insert(0, os.path.dirname(HERE))
import torch  # noqa: E402
import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

nch = int(sys.argv[1]) if len(sys.argv) > 1 else 64
chunk = 4 << 20
src = gen_f32_device(0, nch * chunk // 4, torch.device("cuda", 0)).view(torch.uint8)
stride = chunk + 256
dst = torch.empty(nch * stride, dtype=torch.uint8, device="cuda")
cb = torch.zeros(nch, dtype=torch.int32, device="cuda")
out = torch.empty(nch * chunk, dtype=torch.uint8, device="cuda")
status = torch.zeros(nch, dtype=torch.int32, device="cuda")
cp = B.cparams(clevel=5, typesize=4, lz_mode=int(sys.argv[2]) if len(sys.argv) > 2 else None)
L = B.lib()
L.b2h_enable_timing(1)
B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
for _ in range(2):
    B.decompress_batch(dst.data_ptr(), stride, cb.data_ptr(), nch, out.data_ptr(), chunk, chunk, status.data_ptr())
torch.cuda.synchronize()
assert torch.equal(out, src)
print("times", B.last_times())
if not os.environ.get("B2H_DECODE_DEBUG"):
    sys.exit(0)
ns = nch * 16 * 4
rec = np.zeros((ns, 2), np.int64)
L.b2h_debug_decode_cycles.argtypes = [C.c_void_p, C.c_int32]
assert L.b2h_debug_decode_cycles(rec.ctypes.data, ns) == ns
names = ["zero", "run", "raw", "lz"]
for k in range(4):
    m = rec[:, 1] == k
    if m.any():
        cyc = rec[m, 0]
        print(f"{names[k]:4s}: {m.sum():6d} streams, cycles mean {cyc.mean():10.0f} max {cyc.max():10d} "
              f"(share of wave time {cyc.sum() / rec[:, 0].sum():.3f})")
