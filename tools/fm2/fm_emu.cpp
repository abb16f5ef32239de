// fm_emu.cpp -- serial CPU emulation of the fast-mode kernel's pass (c-blosc2_amd/csrc/b2h_lzfast.h
// fm_pass / encode_stream_fast), lane by lane, with every LDS index and global address checked.
// Diagnostics only (test infrastructure): it finds out-of-range accesses, reads of stale LDS and
// lane-order dependences on the CPU, where a fault costs nothing.  The LDS arrays start filled
// with garbage (seeded) the way a workgroup finds them after a previous stream or kernel.
//
//   g++ -O2 -shared -fPIC -o tools/fm2/libfm_emu.so tools/fm2/fm_emu.cpp
//   int fm_emu_stream(in, n, avail, clevel, out, tablog, u16, seed, int64_t diag[8]) -> size (0 raw)
#include <stdint.h>
#include <string.h>
#include <algorithm>
#include <vector>

namespace {
constexpr int32_t kS = 1024, kHist = 32, kSeg = 32, kWin = kHist + kS, kWalk = kS / kSeg, kAhead = 64, kH = 16384;
constexpr int32_t kCmpCap = 256, kOpen = 0x7fffffff, kEoffLong = 0x7fff;
constexpr uint32_t kDMask = 0x1ffffu;
constexpr int kMaxCopy = 32;
constexpr uint32_t kNear = 8191, kFar = 65535 + 8191 - 1;

struct Emu {
  const uint8_t* in;
  int32_t avail;   // bytes readable from in (stream + slack)
  bool u16;
  int64_t* diag;
  std::vector<uint32_t> tab;
  uint32_t rec[kWin + 1];
  uint32_t mb[40], lb[40];
  uint8_t hist[kH];
  std::vector<uint8_t> ring;
  int32_t RM;
  struct {
    int32_t entry, open_q, open_d, o, lit, F, peak, fail, byte0, stop, pos;
  } sh;
  int32_t ringown[8192];
  uint64_t rng;

  void bad(int site, int64_t a, int64_t b, int64_t c) {
    if (diag[0] == 0) {
      diag[0] = site;
      diag[1] = a;
      diag[2] = b;
      diag[3] = c;
    }
    diag[7]++;
  }
  uint32_t rnd() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)rng;
  }
  void garbage() {
    for (auto& v : rec) v = rnd();
    for (auto& v : mb) v = rnd();
    for (auto& v : lb) v = rnd();
    for (auto& v : hist) v = (uint8_t)rnd();
    for (auto& v : ring) v = (uint8_t)rnd();
    for (auto& v : tab) v = rnd() & (u16 ? 0xffffu : 0xffffffffu);
    sh.entry = (int32_t)rnd();
    sh.open_q = (int32_t)rnd();
    sh.open_d = (int32_t)rnd();
  }
  // ---- global memory (checked: the aligned dwords read must lie in [0, avail))
  uint8_t gb(int64_t x) {
    if (x < 0 || x >= avail) {
      bad(100, x, avail, 0);
      return 0;
    }
    return in[x];
  }
  uint32_t gw(int64_t x) {   // aligned dword
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) v |= (uint32_t)gb(x + k) << (8 * k);
    return v;
  }
  static uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh) {
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * sh));
  }
  uint32_t ldu32(int64_t p) {
    const int64_t q = p & ~int64_t(3);
    return funnel(gw(q), gw(q + 4), (uint32_t)(p & 3));
  }
  void ld16(int64_t p, uint32_t (&w)[4]) {
    const int64_t q = p & ~int64_t(3);
    uint32_t d[5];
    for (int i = 0; i < 5; i++) d[i] = gw(q + 4 * i);
    for (int i = 0; i < 4; i++) w[i] = funnel(d[i], d[i + 1], (uint32_t)(p & 3));
  }
  // ---- LDS
  uint32_t hist32(int32_t x) {
    const uint32_t* w = (const uint32_t*)hist;
    constexpr int32_t M = kH / 4 - 1;
    const int32_t i = x >> 2;
    return funnel(w[i & M], w[(i + 1) & M], (uint32_t)(x & 3));
  }
  uint32_t& R(int32_t i) {
    if (i < 0 || i > kWin) {
      bad(200, i, 0, 0);
      static uint32_t dummy;
      return dummy;
    }
    return rec[i];
  }
  uint32_t LB(int32_t w) {
    if (w < 0 || w > kWin / 32) bad(201, w, 0, 0);
    return lb[w & 31 ? w : w];
  }

  int32_t lane_match_end(int32_t x, uint32_t d, int32_t bound) {
    if (!(x - (int32_t)d >= 0 && d > 0)) {
      bad(3, x, d, bound);
      return bound;
    }
    while (x < bound) {
      uint32_t a[4], b[4];
      ld16(x, a);
      ld16((int64_t)x - d, b);
      const int32_t nb = bound - x;
      for (int k = 0; k < 4; k++) {
        uint32_t diff = a[k] ^ b[k];
        const int32_t lo = 4 * k;
        if (nb <= lo) diff = 0;
        else if (nb < lo + 4) diff &= (1u << (8 * (nb - lo))) - 1u;
        if (diff) return x + lo + (int32_t)(__builtin_ctz(diff) >> 3) + 1;
      }
      x += 16;
    }
    return bound;
  }
  int32_t match_len(bool PROBE, int32_t q, uint32_t d, int32_t j0, int32_t W, int32_t bound) {
    int32_t j = j0;
    while (j < kWin) {
      const int32_t s = j & 31;
      const uint32_t nw = ~(LB(j >> 5) >> s);
      const int32_t ones = nw ? (int32_t)__builtin_ctz(nw) : 32;
      j += ones;
      if (ones < 32 - s) break;
    }
    if (j >= kWin) return kOpen;
    const int32_t qe = W + j - 1;
    const int32_t eo = (int32_t)(R(j) >> 17);
    int32_t e;
    if (eo == kEoffLong) e = lane_match_end(qe + 4, d, bound);
    else e = qe + eo;
    const int32_t len = e - 4 - q;
    if (len < 4 || (!PROBE && len <= 5 && d - 1 >= kNear)) return -1;
    return len;
  }
  static uint32_t from(int32_t lo) { return lo >= 32 ? 0u : (~0u << lo); }
  static uint32_t below(int32_t hi) { return hi >= 32 ? ~0u : ((1u << hi) - 1u); }
  void walk(bool PROBE, int32_t e, int32_t a, int32_t hi, uint32_t Mw, bool conv, uint32_t VISo, uint32_t MSo, int32_t xo,
            int32_t W, int32_t bound, int32_t& x, uint32_t& MS, uint32_t& VIS) {
    int32_t p = e;
    uint32_t ms = 0, vis = 0;
    while (p < hi) {
      const int32_t rel = p - a;
      if (rel < 0 || rel >= 32) bad(300, p, a, hi);
      const uint32_t mm = Mw & from(rel);
      const int32_t qrel = mm ? (int32_t)__builtin_ctz(mm) : hi - a;
      const uint32_t lits = from(rel) & below(qrel);
      const uint32_t starts = lits | (mm ? (1u << qrel) : 0u);
      if (conv && (starts & VISo)) {
        const int32_t c = (int32_t)__builtin_ctz(starts & VISo);
        const uint32_t lo = below(c);
        VIS = ((vis | starts) & lo) | (VISo & ~lo);
        MS = (ms & lo) | (MSo & ~lo);
        x = xo;
        return;
      }
      vis |= starts;
      if (!mm) {
        p = hi;
        break;
      }
      const int32_t q = a + qrel;
      const int32_t len = match_len(PROBE, q, R(1 + (q - W)) & kDMask, q - W + 1, W, bound);
      if (len < 0) {
        p = q + 1;
      } else {
        ms |= 1u << qrel;
        if (len == kOpen) {
          p = kOpen;
          break;
        }
        p = q + len + 2;
      }
    }
    MS = ms;
    VIS = vis;
    x = p;
  }

  struct PassOut {
    bool fail, early, sure;
    int32_t pos, o, peak;
  };

  PassOut pass(bool PROBE, int32_t base_off, int32_t length, int probe_hashlog, int tablog, uint8_t* out, int32_t maxout,
               int clevel) {
    const uint8_t* in0 = in;
    const int32_t avail0 = avail;
    in += base_off;
    avail -= base_off;
    int32_t limit = length;
    if (PROBE) limit = std::min(length, 1 << probe_hashlog);
    const int32_t bound = limit - 1, loop_end = limit - 12;
    std::fill(tab.begin(), tab.begin() + (1 << tablog), 0u);
    memset(hist, 0, sizeof hist);
    sh.entry = PROBE ? 0 : 4;
    sh.open_q = -1;
    sh.open_d = 0;
    sh.o = 5;
    sh.lit = 4;
    sh.F = 0;
    sh.peak = 0;
    sh.fail = 0;
    sh.byte0 = kMaxCopy - 1;
    sh.stop = 0;
    sh.pos = PROBE ? 0 : 4;
    if (!PROBE)
      for (int lane = 0; lane < 5; lane++) ring[lane] = lane == 0 ? (uint8_t)(kMaxCopy - 1) : gb(lane - 1);
    auto stage = [&](int32_t lo, int32_t hi) {
      if (hi <= limit && ((base_off + lo) & 15) == 0) {
        for (int32_t x = lo; x < hi; x += 16) {
          if (!(x >= 0 && x + 16 <= limit)) bad(7, x, lo, hi);
          for (int k = 0; k < 16; k++) hist[(x + k) & (kH - 1)] = gb(x + k);
        }
      } else {
        for (int32_t x = lo; x < hi; x += 4) {
          uint32_t w = 0;
          if (x + 4 <= limit) w = ldu32(x);
          else
            for (int k = 0; k < 4; k++)
              if (x + k < limit) w |= (uint32_t)gb(x + k) << (8 * k);
          memcpy(hist + (x & (kH - 1)), &w, 4);
        }
      }
    };
    stage(0, kS + kAhead);
    for (int32_t P = 0; P - kHist < loop_end; P += kS) {
      const int32_t W = P - kHist;
      const int32_t rlo = P + kS + kAhead - kH;
      const int32_t entry0 = sh.entry;
      const bool has_open = entry0 == kOpen;
      // ---- B
      {
        uint32_t hrec[kHist];
        for (int l = 0; l < kHist; l++) hrec[l] = P > 0 ? rec[1 + kS + l] : 0u;
        const uint32_t hm = P > 0 ? mb[kS / 32] : 0u, hl = P > 0 ? lb[kS / 32] : 0u;
        for (int l = 0; l < kHist; l++) rec[1 + l] = hrec[l];
        rec[0] = 0;
        mb[0] = hm;
        lb[0] = hl;
        const int32_t ntiles = std::max(0, std::min(kS, loop_end - P) + 63) / 64;
        for (int32_t t = 0; t < ntiles; t++)
          for (int lane = 0; lane < 64; lane++) {
            const int32_t p = P + t * 64 + lane;
            const bool valid = p < loop_end;
            uint32_t cand = 0;
            if (valid) {
              const uint32_t key = hist32(p);
              if (p + 4 <= limit && key != ldu32(p)) bad(400, p, key, ldu32(p));   // the ring holds p's bytes
              const uint32_t h = (key * 2654435761u) >> (32 - tablog);
              cand = tab[h];
              tab[h] = u16 ? ((uint32_t)p & 0xffffu) : (uint32_t)p;
            }
            const uint32_t d = (uint32_t)(p - (int32_t)cand);
            rec[1 + kHist + t * 64 + lane] = (valid && d != 0 && d < kFar) ? d : 0u;
          }
        for (int32_t i = ntiles * 64; i < kS; i++) rec[1 + kHist + i] = 0;
      }
      // ---- C
      for (int32_t t = 0; t < kS / 64; t++) {
        uint64_t mbits = 0, lbits = 0;
        for (int lane = 0; lane < 64; lane++) {
          const int32_t i = t * 64 + lane, q = P + i;
          const uint32_t key = hist32(q);
          const uint32_t d = rec[1 + kHist + i];
          const uint32_t dp = rec[kHist + i] & kDMask;
          const int32_t c = q - (int32_t)d;
          uint32_t cw = 0;
          if (d != 0) {
            if (c >= rlo) cw = hist32(c);
            else {
              if (!(c >= 0 && c < limit)) bad(1, c, d, q);
              cw = ldu32(c);
            }
          }
          const bool m4 = d != 0 && cw == key;
          if (m4 && q + 4 <= limit && ldu32(c) != ldu32(q)) bad(401, q, c, 0);
          if (m4) mbits |= 1ull << lane;
          if (m4 && d == dp) lbits |= 1ull << lane;
        }
        mb[1 + 2 * t] = (uint32_t)mbits;
        mb[2 + 2 * t] = (uint32_t)(mbits >> 32);
        lb[1 + 2 * t] = (uint32_t)lbits;
        lb[2 + 2 * t] = (uint32_t)(lbits >> 32);
      }
      // ---- C2
      for (int32_t j = kHist - 1; j < kWin - 1; j++) {
        const bool m4 = (mb[j >> 5] >> (j & 31)) & 1u;
        const bool next = (lb[(j + 1) >> 5] >> ((j + 1) & 31)) & 1u;
        if (!(m4 && !next)) continue;
        const uint32_t rw = rec[1 + j];
        const uint32_t d = rw & kDMask;
        const int32_t q = W + j;
        int32_t x = q + 4, e = -1;
        const int32_t xmax = std::min(bound, q + kCmpCap);
        while (x < xmax) {
          uint32_t a, b;
          if (x + 4 <= P + kS + kAhead && x - (int32_t)d >= rlo) {
            a = hist32(x);
            b = hist32(x - (int32_t)d);
          } else if (x - (int32_t)d >= 0 && x < limit) {
            a = ldu32(x);
            b = ldu32((int64_t)x - d);
          } else {
            bad(2, x, d, q);
            a = b = 0;
          }
          uint32_t diff = a ^ b;
          const int32_t nb = bound - x;
          if (nb < 4) diff &= (1u << (8 * nb)) - 1u;
          if (diff) {
            e = x + (int32_t)(__builtin_ctz(diff) >> 3) + 1;
            break;
          }
          x += 4;
        }
        const int32_t eo = e >= 0 ? e - q : (x >= bound ? bound - q : kEoffLong);
        if (eo < 0 || eo > kEoffLong) bad(402, eo, q, 0);
        rec[1 + j] = d | ((uint32_t)eo << 17);
      }
      // waves 1-3 stage the next super-tile while wave 0 parses: the two touch disjoint ring bytes
      if (P + kS - kHist < loop_end) stage(P + kS + kAhead, P + 2 * kS + kAhead);
      // ---- D + E
      if (has_open || entry0 < W + kS) {
        int32_t a[64], hi[64], e[64], x[64];
        uint32_t Mw[64], MS[64], VIS[64];
        int32_t cm_q = -1, cm_len = 0;
        uint32_t cm_d = 0;
        for (int l = 0; l < 64; l++) {
          a[l] = W + kSeg * l;
          hi[l] = std::min(std::min(a[l] + kSeg, loop_end), W + kS);
          Mw[l] = l < kWalk ? mb[l] : 0u;
          e[l] = l == 0 ? entry0 : a[l];
          MS[l] = VIS[l] = 0;
        }
        if (has_open) {
          cm_q = sh.open_q;
          cm_d = (uint32_t)sh.open_d;
          if (cm_q < W - 2 * kS || cm_q >= W + kHist || cm_d == 0 || cm_d >= kFar) bad(403, cm_q, cm_d, W);
          cm_len = match_len(PROBE, cm_q, cm_d, kHist, W, bound);
          if (cm_len != kOpen) e[0] = cm_q + cm_len + 2;
        }
        for (int l = 0; l < 64; l++) {
          if (e[l] >= hi[l]) x[l] = e[l];
          else walk(PROBE, e[l], a[l], hi[l], Mw[l], false, 0, 0, 0, W, bound, x[l], MS[l], VIS[l]);
        }
        int rounds = 0;
        for (;;) {
          rounds++;
          int32_t en[64];
          bool ch[64], any = false;
          for (int l = 0; l < 64; l++) {
            en[l] = l == 0 ? e[0] : x[l - 1];
            ch[l] = l < kWalk && en[l] != e[l];
            any |= ch[l];
          }
          if (!any) break;
          if (rounds > 200) {
            bad(404, rounds, P, 0);
            break;
          }
          for (int l = 0; l < 64; l++) {
            if (!ch[l]) continue;
            e[l] = en[l];
            if (en[l] >= hi[l]) {
              x[l] = en[l];
              MS[l] = VIS[l] = 0;
            } else {
              walk(PROBE, en[l], a[l], hi[l], Mw[l], true, VIS[l], MS[l], x[l], W, bound, x[l], MS[l], VIS[l]);
            }
          }
        }
        // per-lane elements
        struct El {
          bool match;
          uint32_t bits;
          int32_t len;
          uint32_t d;
        };
        std::vector<El> els[64];
        for (int l = 0; l < 64; l++) {
          const uint32_t LITS = VIS[l] & ~MS[l];
          const int32_t f = MS[l] ? (int32_t)__builtin_ctz(MS[l]) : 32;
          int32_t prev = -2;
          if (l == 0 && cm_q >= 0) {
            if (cm_len != kOpen) els[l].push_back({true, 0, cm_len, cm_d});
            prev = -1;
          } else {
            els[l].push_back({false, LITS & below(f), 0, 0});
          }
          uint32_t rem = MS[l];
          bool open = false;
          while (rem) {
            const int32_t m = (int32_t)__builtin_ctz(rem);
            rem &= rem - 1;
            if (prev != -2) els[l].push_back({false, LITS & from(prev + 1) & below(m), 0, 0});
            const int32_t q = a[l] + m;
            const uint32_t d = R(1 + (q - W)) & kDMask;
            const int32_t len = match_len(PROBE, q, d, q - W + 1, W, bound);
            if (len == kOpen) {
              open = true;
              break;
            }
            if (len < 0) bad(405, q, len, l);
            els[l].push_back({true, 0, len, d});
            prev = m;
          }
          if (!open && prev != -2) els[l].push_back({false, LITS & from(prev + 1), 0, 0});
        }
        auto tok = [](int32_t len, uint32_t d) { return (len >= 7 ? 1 + (len - 7) / 255 : 0) + ((d - 1) < kNear ? 2 : 4); };
        int32_t A[64], Bb[64], T[64];
        bool has[64];
        for (int l = 0; l < 64; l++) {
          int32_t t = 0;
          A[l] = Bb[l] = T[l] = 0;
          has[l] = false;
          for (auto& el : els[l]) {
            if (!el.match) {
              const int32_t n = __builtin_popcount(el.bits);
              if (has[l]) t += n;
              else A[l] += n;
            } else {
              if (has[l]) Bb[l] += t + t / 32 - ((t & 31) == 0 ? 1 : 0);
              has[l] = true;
              t = 0;
              Bb[l] += tok(el.len, el.d) + 1;
            }
          }
          if (has[l]) {
            Bb[l] += t + t / 32;
            T[l] = t & 31;
          }
        }
        const int32_t lit_in = sh.lit, o_in = sh.o;
        int32_t X[64], PX[64], mlast[64], size[64], incl[64], litk[64], s0[64];
        int32_t run = 0, mx = -1;
        for (int l = 0; l < 64; l++) {
          X[l] = has[l] ? 0 : A[l];
          run += X[l];
          PX[l] = run;
          mx = std::max(mx, has[l] ? l : -1);
          mlast[l] = mx;
        }
        int32_t tot = 0;
        for (int l = 0; l < 64; l++) {
          const int32_t mex = l == 0 ? -1 : mlast[l - 1];
          const int32_t src = std::max(mex, 0);
          const int32_t Ym = T[src] - PX[src];
          const int32_t Rr = (l > 0 && mex >= 0 ? Ym : lit_in) + (PX[l] - X[l]);
          litk[l] = Rr & 31;
          s0[l] = litk[l] + A[l];
          size[l] = A[l] + s0[l] / 32 + (has[l] ? Bb[l] - ((s0[l] & 31) == 0 ? 1 : 0) : 0);
          tot += size[l];
          incl[l] = tot;
        }
        const int32_t o_out = o_in + incl[63];
        const int32_t lit_out = has[63] ? T[63] : (s0[63] & 31);
        const int32_t x_out = x[kWalk - 1];
        int opener = -1;
        for (int l = 0; l < kWalk && opener < 0; l++)
          if (x[l] == kOpen && e[l] != kOpen) opener = l;
        int32_t stop = 0;
        if (!PROBE) {
          for (int32_t k = 0; k <= RM; k++) ringown[k] = -1;
          int32_t req = 0;
          struct Patch {
            int32_t pos;
            uint8_t v;
          };
          std::vector<Patch> patches;
          auto wr = [&](int32_t pos, uint8_t v, int l) {
            const int32_t k = pos & RM;
            if (ringown[k] >= 0 && ringown[k] != l) bad(500, pos, ringown[k], l);
            ringown[k] = l;
            ring[k] = v;
          };
          for (int l = 0; l < 64; l++) {
            int32_t o = o_in + incl[l] - size[l], lit = litk[l], dpos = -1;
            uint32_t dval = 0;
            bool first = true;
            for (auto& el : els[l]) {
              if (!el.match) {
                uint32_t bits = el.bits;
                while (bits) {
                  const int32_t j = (int32_t)__builtin_ctz(bits);
                  bits &= bits - 1;
                  req = std::max(req, o + 2);
                  wr(o, hist[(a[l] + j) & (kH - 1)], l);
                  if (hist[(a[l] + j) & (kH - 1)] != gb(a[l] + j)) bad(501, a[l] + j, 0, 0);
                  o++;
                  if (++lit == kMaxCopy) {
                    wr(o, (uint8_t)(kMaxCopy - 1), l);
                    o++;
                    lit = 0;
                  }
                }
              } else {
                const int32_t len = el.len;
                const uint32_t d = el.d;
                int32_t p0;
                uint32_t v0;
                const uint32_t bd = d - 1;
                const bool near = bd < kNear;
                const uint32_t fd = bd - kNear;
                const uint32_t b0 = (len >= 7 ? (7u << 5) : ((uint32_t)len << 5)) + (near ? (bd >> 8) : 31u);
                if (lit) {
                  p0 = o - lit - 1;
                  v0 = (uint32_t)(lit - 1);
                  wr(o, (uint8_t)b0, l);
                } else {
                  o--;
                  p0 = o;
                  v0 = b0;
                }
                if (first) {
                  dpos = p0;
                  dval = v0;
                } else {
                  wr(p0, (uint8_t)v0, l);
                }
                int32_t w = o + 1;
                if (len >= 7) {
                  uint32_t rem = (uint32_t)len - 7;
                  for (; rem >= 255; rem -= 255) wr(w++, 255, l);
                  wr(w++, (uint8_t)rem, l);
                }
                if (near) {
                  wr(w++, (uint8_t)(bd & 255), l);
                } else {
                  wr(w++, 255, l);
                  wr(w++, (uint8_t)(fd >> 8), l);
                  wr(w++, (uint8_t)(fd & 255), l);
                }
                wr(w++, (uint8_t)(kMaxCopy - 1), l);
                o = w;
                lit = 0;
                req = std::max(req, o);
                first = false;
              }
            }
            if (o != o_in + incl[l]) bad(502, l, o, o_in + incl[l]);
            if (dpos >= 0) patches.push_back({dpos, (uint8_t)dval});
          }
          for (auto& pt : patches) ring[pt.pos & RM] = pt.v;
          const int32_t peak = std::max(sh.peak, req);
          const bool fail = peak > maxout;
          int32_t F = sh.F, byte0 = sh.byte0;
          if (!fail) {
            if (o_out - F > RM + 1) bad(503, F, o_out, RM);   // unflushed bytes overrun the ring
            const int32_t fin = (o_out - lit_out - 1) & ~15;
            if (fin > F) {
              if (!(F >= 0 && fin <= maxout)) bad(5, F, fin, maxout);
              if (F == 0) byte0 = ring[0];
              for (int32_t y = F; y < fin && y < maxout; y++) out[y] = ring[y & RM];
              F = fin;
            }
          } else {
            stop = 1;
          }
          sh.peak = peak;
          sh.F = F;
          sh.byte0 = byte0;
        }
        sh.o = o_out;
        sh.lit = lit_out;
        sh.entry = x_out;
        if (x_out != kOpen) sh.pos = x_out;
        if (opener >= 0) {
          const uint32_t msk = MS[opener];
          if (msk == 0) bad(504, opener, P, 0);
          const int32_t q = W + kSeg * opener + 31 - (int32_t)__builtin_clz(msk | 1u);
          sh.open_q = q;
          sh.open_d = (int32_t)(R(1 + (q - W)) & kDMask);
        } else if (x_out == kOpen && !has_open) {
          bad(505, P, 0, 0);
        }
        if (PROBE && x_out != kOpen) {
          const double thr_o = 0.999 * (clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2
                                        : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0);
          const double thr_s = thr_o * (1.001 / 0.999);
          if ((double)(limit + 64) < thr_o * (double)o_out) stop = 2;
          else {
            const int32_t Rr = loop_end - x_out;
            if ((double)loop_end >= thr_s * (double)(o_out + Rr + Rr / 16 + 16)) stop = 3;
          }
        }
        if (stop) sh.stop = stop;
      }
      if (sh.stop || (sh.entry != kOpen && sh.entry >= loop_end)) break;
    }
    PassOut r;
    r.fail = sh.stop == 1;
    r.early = sh.stop == 2;
    r.sure = sh.stop == 3;
    r.pos = sh.pos;
    r.o = sh.o;
    r.peak = sh.peak;
    if (!PROBE) {
      if (sh.entry == kOpen) bad(506, 0, 0, 0);
      if (!r.fail) {
        int32_t o = r.o, lit = sh.lit, peak = r.peak;
        const int32_t pos = r.pos, F = sh.F;
        int32_t byte0 = sh.byte0;
        bool fail = false;
        if (pos <= bound) {
          const int32_t cnt = bound - pos + 1;
          if (cnt > 64) bad(507, pos, cnt, bound);
          const int32_t last = o + (cnt - 1) + (lit + cnt - 1) / 32;
          peak = std::max(peak, last + 2);
          if (last + 2 > maxout) fail = true;
          else {
            for (int lane = 0; lane < std::min(cnt, 64); lane++) {
              if (!(pos + lane >= 0 && pos + lane < limit)) bad(4, pos, cnt, bound);
              const int32_t off = o + lane + (lit + lane) / 32;
              ring[off & RM] = gb(pos + lane);
              if (((lit + lane + 1) & 31) == 0) ring[(off + 1) & RM] = (uint8_t)(kMaxCopy - 1);
            }
            o += cnt + (lit + cnt) / 32;
            lit = (lit + cnt) & 31;
          }
        }
        if (!fail) {
          if (lit) {
            const int32_t at = o - lit - 1;
            ring[at & RM] = (uint8_t)(lit - 1);
            if (at == 0) byte0 = lit - 1;
          } else {
            o--;
          }
          if (!(o >= 0 && o <= maxout && F <= o)) bad(6, F, o, maxout);
          else if (o - F > RM + 1) bad(508, F, o, RM);
          else if (F == 0) {
            byte0 = ring[0];
            ring[0] = (uint8_t)(byte0 | 0x20);
            for (int32_t y = 0; y < o; y++) out[y] = ring[y & RM];
          } else {
            for (int32_t y = F; y < o; y++) out[y] = ring[y & RM];
            out[0] = (uint8_t)(byte0 | 0x20);
          }
        }
        r.o = o;
        r.peak = peak;
        r.fail = fail;
      }
    }
    in = in0;
    avail = avail0;
    return r;
  }
};
}  // namespace

extern "C" int fm_emu_stream(const uint8_t* in, int32_t n, int32_t avail, int clevel, uint8_t* out, int tablog_max,
                             int u16, uint64_t seed, int64_t* diag) {
  Emu E;
  E.in = in;
  E.avail = avail;
  E.u16 = u16 != 0;
  E.diag = diag;
  E.tab.assign((size_t)1 << 14, 0);
  E.ring.assign(u16 ? 2048 : 4096, 0);
  E.RM = (int32_t)E.ring.size() - 1;
  E.rng = seed | 1;
  E.garbage();
  bool run = n > 0;
  for (int32_t i = 1; i < n && run; i++) run = in[i] == in[0];
  if (run) return -2;
  const int hashlog = clevel == 1 ? 12 : (clevel == 2 ? 13 : 14);
  const int tl = std::min(tablog_max, hashlog);
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  auto pr = E.pass(true, n - maxlen, maxlen, hashlog, tl, out, 0, clevel);
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  const bool go = !(pr.early || (!pr.sure && ratio < thr) || n < 66);
  if (!go) return 0;
  auto em = E.pass(false, 0, n, hashlog, tl, out, n, clevel);
  if (em.fail) return 0;
  diag[6] = em.peak;
  return em.o;
}
