"""C4 decode, per-stream cycles by kind (diagnostics; B2H_DECODE_DEBUG=1): which streams of the
(DELTA, SHUFFLE) int64-ramp batch hold k_decode's time.   B2H_DECODE_DEBUG=1 python tools/prof_c4_decode.py"""
import collections
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "c-blosc2_amd"))
import blosc2_amd as B


def main(nch=2000):
    chunk = 1 << 20
    src = torch.arange(0, nch * chunk // 8, dtype=torch.int64, device="cuda").view(torch.uint8)
    cp = B.cparams(clevel=5, typesize=8, filters=(0, 0, 0, 0, B.DELTA, B.SHUFFLE))
    cap = chunk + 64
    stride = (cap + 255) // 256 * 256
    comp = torch.zeros(nch * stride, dtype=torch.uint8, device="cuda")
    cb = torch.zeros(nch, dtype=torch.int32, device="cuda")
    B.compress_batch(cp, src.data_ptr(), chunk, nch, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
    out = torch.zeros(nch * chunk, dtype=torch.uint8, device="cuda")
    st = torch.zeros(nch, dtype=torch.int32, device="cuda")
    for _ in range(2):
        B.decompress_batch(comp.data_ptr(), stride, cb.data_ptr(), nch, out.data_ptr(), chunk, chunk, st.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out, src)
    n = nch * 16
    buf = np.zeros(2 * n, np.int64)
    got = B.lib().b2h_debug_decode_cycles(C.c_void_p(buf.ctypes.data), n)
    cyc, kind = buf[0::2][:got], buf[1::2][:got]
    by = collections.defaultdict(list)
    for i in range(got):
        by[(i % 16, int(kind[i]))].append(int(cyc[i]))
    tot = cyc.sum()
    for (j, k), v in sorted(by.items()):
        print(f"stream {j:2d} kind {k}: n {len(v):5d} mean {np.mean(v):10.0f} cycles  share {sum(v) / tot * 100:5.1f} %")


if __name__ == "__main__":
    main()
