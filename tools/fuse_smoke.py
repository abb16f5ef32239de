"""Quick GPU check of the fused fast-mode encode (k_encode_fast_fused) against the separate launches
(B2H_FUSE=0; 1 = finalize/scatter fused, 3 = + shuffle): one T chunk through blosc2_compress_ctx, then a 64-chunk T batch; byte comparison and
device round trip.  Usage: python tools/fuse_smoke.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "c-blosc2_amd"))
import torch  # noqa: E402

import blosc2_amd as B  # noqa: E402
from datagen import gen_f32  # noqa: E402

L = B.lib()
L.b2h_set_blosclz_mode(1)
src1 = gen_f32(0, 1 << 20)
for fuse in ("0", "83", "3"):
    os.environ["B2H_FUSE"] = fuse
    t = time.time()
    got = B.compress(src1, clevel=5, typesize=4)
    print(f"single chunk fuse={fuse}: {got.nbytes if isinstance(got, np.ndarray) else got} bytes "
          f"{time.time() - t:.3f}s", flush=True)
    assert isinstance(got, np.ndarray)
    assert np.array_equal(B.decompress(got, src1.nbytes), src1.view(np.uint8).reshape(-1)), fuse

dev = torch.device("cuda")
chunk, n = 4 << 20, 64
src = torch.from_numpy(gen_f32(7, n * chunk // 4).view(np.uint8)).to(dev)
cap = chunk + 64
stride = (cap + 255) // 256 * 256
cp = B.cparams(clevel=5, typesize=4)
res = {}
for fuse in ("0", "83", "3"):
    os.environ["B2H_FUSE"] = fuse
    comp = torch.zeros(n * stride, dtype=torch.uint8, device=dev)
    cb = torch.zeros(n, dtype=torch.int32, device=dev)
    for rep in range(3):
        torch.cuda.synchronize()
        t = time.time()
        B.compress_batch(cp, src.data_ptr(), chunk, n, chunk, comp.data_ptr(), stride, cap, cb.data_ptr(), 0)
        torch.cuda.synchronize()
        dt = time.time() - t
    out = torch.zeros_like(src)
    st = torch.zeros(n, dtype=torch.int32, device=dev)
    B.decompress_batch(comp.data_ptr(), stride, cb.data_ptr(), n, out.data_ptr(), chunk, chunk, st.data_ptr(), 0)
    torch.cuda.synchronize()
    ok = torch.equal(out, src) and bool((st == chunk).all())
    cbh = cb.cpu().numpy()
    res[fuse] = (cbh, comp.cpu().numpy().reshape(n, stride))
    print(f"batch fuse={fuse}: {dt * 1e3:.2f} ms, total {int(cbh.sum())} bytes, round trip {ok}", flush=True)
    assert ok
for fz in ("83", "3"):
    same = np.array_equal(res["0"][0], res[fz][0]) and all(
        np.array_equal(res["0"][1][i, :res["0"][0][i]], res[fz][1][i, :res[fz][0][i]]) for i in range(n))
    print(f"fused {fz} == separate:", same, flush=True)
    assert same
