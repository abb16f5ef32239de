"""Fused-encode diagnostics (not a test): T batch (1024 x 4 MiB) compressed under B2H_FUSE modes
given on the command line; prints the stage times and the per-stream encode cycles / durations."""
import ctypes as C
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
sys.path.insert(0, os.path.join(HERE, "..", "c-blosc2_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
import torch  # noqa: E402

import blosc2_amd as B  # noqa: E402
from bench import gen_f32_device  # noqa: E402

lzm = int(os.environ.get("LZMODE", "1"))   # 1 fast, 0 exact
modes = sys.argv[1:] or ["0", "19"]
nch, chunk = 1024, 4 << 20
src = gen_f32_device(0, nch * chunk // 4, torch.device("cuda", 0)).view(torch.uint8)
stride = chunk + 256
dst = torch.empty(nch * stride, dtype=torch.uint8, device="cuda")
cb = torch.zeros(nch, dtype=torch.int32, device="cuda")
cp = B.cparams(clevel=5, typesize=4)
L = B.lib()
L.b2h_set_blosclz_mode(lzm)
L.b2h_enable_timing(1)
L.b2h_debug_stream_results.argtypes = [C.c_void_p, C.c_int32]
ns = nch * 64
for m in modes:
    os.environ["B2H_FUSE"] = m
    ts = []
    for _ in range(4):
        B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, dst.data_ptr(), stride, chunk + 32, cb.data_ptr())
        torch.cuda.synchronize()
        ts.append(B.last_times())
    rec = np.zeros(ns, dtype=[("kind", "i4"), ("size", "i4"), ("peak", "i4"), ("windows", "i4"),
                              ("cycles", "i8"), ("t0", "i8")])
    assert L.b2h_debug_stream_results(rec.ctypes.data, ns) == ns
    dur = (rec["t0"] & 0xffffff) / 100.0          # us (100 MHz)
    start = (rec["t0"] >> 24) / 100.0
    start -= start.min()
    end = start + dur
    print(f"B2H_FUSE={m}: times {ts[-1]}", flush=True)
    print(f"   stream cycles sum {rec['cycles'].sum() / 1e9:.3f} G, mean dur {dur.mean():.1f} us, "
          f"span {end.max():.0f} us, p50/p99 end {np.percentile(end, 50):.0f}/{np.percentile(end, 99):.0f} us, "
          f"per-plane mean dur {[round(float(dur[np.arange(ns) % 4 == k].mean()), 1) for k in range(4)]}", flush=True)
