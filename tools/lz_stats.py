"""Token statistics of a BloscLZ stream (diagnostics): python tools/lz_stats.py stream.bin
Follows the token grammar of blosc/blosclz.c:685-795."""
import sys

import numpy as np

s = np.fromfile(sys.argv[1], np.uint8).tolist()
ip, op, nl, litb = 1, 0, 0, 0
mlens, dists = [], []
ctrl = s[0] & 31
while True:
    if ctrl >= 32:
        ln, ofs = (ctrl >> 5) - 1, (ctrl & 31) << 8
        if ln == 6:
            while True:
                c = s[ip]
                ip += 1
                ln += c
                if c != 255:
                    break
        code = s[ip]
        ip += 1
        ln += 3
        d = ofs + code + 1
        if code == 255 and ofs == (31 << 8):
            d = (s[ip] << 8 | s[ip + 1]) + 8191 + 1
            ip += 2
        mlens.append(ln)
        dists.append(d)
        op += ln
    else:
        r = ctrl + 1
        nl += 1
        litb += r
        ip += r
        op += r
    if ip >= len(s):
        break
    ctrl = s[ip]
    ip += 1
ml, ds = np.array(mlens), np.array(dists)
print("out", op, "matches", len(ml), "literal runs", nl, "literal bytes", litb)
print("match len percentiles 10/25/50/75/90/99:", np.percentile(ml, [10, 25, 50, 75, 90, 99]), "mean", ml.mean(),
      "frac >= 28:", (ml >= 28).mean())
vals, cnt = np.unique(ds, return_counts=True)
o = np.argsort(-cnt)[:10]
print("top distances", list(zip(vals[o].tolist(), cnt[o].tolist())))
