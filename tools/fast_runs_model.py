# Model count (diagnostics, not a test) of the fast matcher's runs per tile on a 64 KiB plane:
# runs of same-distance positions whose first four bytes match, and the compare points among their
# ends.  python tools/fast_runs_model.py tools/fixtures/f32_p2.bin
import numpy as np, sys
b = np.fromfile(sys.argv[1], np.uint8).astype(np.int64)
n = len(b)
tablog = 13
tab = np.zeros(1 << tablog, np.int64)  # u16 positions (<65536 here)
def h(q):
    v = int(b[q]) | int(b[q+1])<<8 | int(b[q+2])<<16 | int(b[q+3])<<24
    return ((v * 2654435761) & 0xffffffff) >> (32 - tablog)
loop_end = n - 12
cand = np.zeros(n, np.int64); cok = np.zeros(n, bool); x0z = np.zeros(n, bool); mm = np.zeros(n, np.int64)
for q in range(0, loop_end):
    k = h(q); c = tab[k]; tab[k] = q
    d = q - c
    ok = 0 < d < 8192
    cand[q] = c; cok[q] = ok
    if ok:
        m = 0
        while q + m < n and m < 200 and b[q+m] == b[c+m]: m += 1
        mm[q] = m; x0z[q] = m >= 4
T = 128
cps = []; runs=[]
for t in range(0, loop_end // T):
    P = t*T
    cnt = 0; nr=0
    for q in range(P, P+T):
        if not cok[q]: continue
        # run end: next position not same
        nxt = q+1
        same_next = nxt < P+T and cok[nxt] and (nxt-cand[nxt]) == (q-cand[q]) and x0z[q]
        if not same_next:
            nr+=1
            if x0z[q]: cnt += 1
    cps.append(cnt); runs.append(nr)
cps = np.array(cps)
print("tiles", len(cps), "compare points per tile mean %.2f max %d p99 %d" % (cps.mean(), cps.max(), np.percentile(cps, 99)), "runs mean %.1f" % np.mean(runs))
acc = cok & (mm >= 4)
print("mm>=60 among accepted: %.3f; 60<=mm<130: %.3f" % ((mm[acc] >= 60).mean(), ((mm[acc] >= 60) & (mm[acc] < 130)).mean()))
