import os, sys, numpy as np
sys.path.insert(0, "c-blosc2_amd"); sys.path.insert(0, "tests")
os.environ["B2H_NO_TORCH"] = "1"
import blosc2_amd as B
L = B.lib()
print("devices", L.b2h_device_count())
from datagen import gen_f32
from oracle_lib import oracle_compress
src = gen_f32(0, 1 << 18)
got = B.compress(src, clevel=5, typesize=4)
print("got", getattr(got, "nbytes", got), L.b2h_last_error())
print("maps", sorted(set(l.split()[-1] for l in open('/proc/self/maps') if 'amdhip64' in l)))
want = oracle_compress(src, clevel=5, typesize=4)
print("equal", isinstance(got, np.ndarray) and np.array_equal(got, want))
