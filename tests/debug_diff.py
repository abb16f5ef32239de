"""Ad-hoc GPU-vs-oracle diff report (debugging aid, not a test)."""
import os, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE); sys.path.insert(0, os.path.join(os.path.dirname(HERE), "c-blosc2_amd"))
import blosc2_amd as B
if os.environ.get("B2H_NO_TORCH"):
    B.lib()
    report_only = True
import torch
print("torch cuda:", torch.cuda.is_available())
B.lib()
print([l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l][:4])
from datagen import gen_f32, mixed_bytes
from oracle_lib import oracle_compress, oracle_decompress

def report(name, src, **kw):
    got = B.compress(src, **kw)
    want = oracle_compress(src, **kw)
    if isinstance(got, np.ndarray) and isinstance(want, np.ndarray) and np.array_equal(got, want):
        print(f"OK   {name}: {want.nbytes}")
        return
    print(f"DIFF {name}: got {getattr(got,'nbytes',got)} want {getattr(want,'nbytes',want)}")
    if isinstance(got, np.ndarray) and isinstance(want, np.ndarray):
        m = min(got.nbytes, want.nbytes)
        idx = np.nonzero(got[:m] != want[:m])[0]
        if len(idx):
            i = idx[0]
            print("   first diff at", i, "ndiff", len(idx))
            print("   got ", got[max(0,i-8):i+24].tolist())
            print("   want", want[max(0,i-8):i+24].tolist())
        print("   hdr got ", got[:48].tolist())
        print("   hdr want", want[:48].tolist())
    dec = B.decompress(want, src.nbytes) if isinstance(want, np.ndarray) else None
    if dec is not None:
        ok = isinstance(dec, np.ndarray) and np.array_equal(dec, src.view(np.uint8).reshape(-1))
        print("   decode of oracle chunk:", "OK" if ok else f"BAD {dec if not isinstance(dec, np.ndarray) else np.nonzero(dec != src.view(np.uint8).reshape(-1))[0][:5]}")

report("f32-1m-first", gen_f32(0, 1 << 18), typesize=4)
report("zeros", np.zeros(100000, np.uint8), typesize=4)
report("const", np.full(100000, 3, np.uint8), typesize=4)
report("ramp-1stream", np.arange(20000, dtype=np.int32), typesize=4, filters=(0,)*6, splitmode=2)
report("mixed-1stream-small", mixed_bytes(1, 3000), typesize=1, filters=(0,)*6, splitmode=2)
report("mixed-1stream", mixed_bytes(1, 60000), typesize=1, filters=(0,)*6, splitmode=2)
report("rand-1stream", np.random.default_rng(0).integers(0,256,60000,dtype=np.uint8), typesize=1, filters=(0,)*6, splitmode=2)
report("f32-64k", gen_f32(0, 16384), typesize=4)
report("f32-1m", gen_f32(0, 1 << 18), typesize=4)
for cl in (1, 2, 9):
    report(f"mixed-cl{cl}", mixed_bytes(2, 100000), clevel=cl, typesize=1, filters=(0,)*6, splitmode=2)

for r in range(3):
    report(f"f32-1m-rep{r}", gen_f32(r, 1 << 18), typesize=4)
