// b2h_lzfast.h -- BloscLZ "fast mode" encoder for gfx950 (device code).
//
// Same token grammar, greedy rule, length / distance limits, entropy-probe thresholds and byte
// emission as blosclz_compress (blosc/blosclz.c:248-316, 320-419, 422-619); the ONE difference is
// which earlier position a hash bucket offers as a position's candidate.  The reference inserts
// only the positions its serial walk visits, so every candidate depends on the whole parse before
// it and the walk is a latency chain (exact mode, b2h_lz.h, ~9 000 cycles per 64 positions on T's
// smooth plane).  Fast mode inserts positions in TILES of 64, in tile order, independently of the
// parse (semantics and their CPU model: tools/fm_model.c):
//
//   * one LDS atomic exchange per lane swaps the lane's position into its bucket and returns the
//     bucket's previous position -- the most recent earlier position with that hash, earlier lanes
//     of the same tile included (LDS applies the lanes of one instruction in lane order);
//   * so a tile's candidates, their 60-byte compares and match lengths are known before the parse
//     reaches it: the kernel software-pipelines tiles T (compare + parse), T + 1 (table exchange +
//     candidate loads) and T + 2 (input loads), and the parse itself is the exact-mode window code
//     (ballot chain walk, DPP prefix-sum emission through the LDS output ring) started at the
//     parse position's lane;
//   * a match that jumps past tile T + 1 restarts the pipeline at its end (the tiles it covers are
//     never inserted, like the reference's skipped positions).
//
// Every match is verified byte for byte against its candidate, so any output decodes with
// blosclz_decompress; the ratio on T is the reference's (2^13 table) or better (2^14).
#pragma once
#include "b2h_lz.h"

namespace b2h {

constexpr int kFastTile = 64;

// Table exchange of one tile: the lanes with p < loop_end hash in[p..p+3] (v) and swap p into the
// bucket.  Returns the candidate (the bucket's previous position; 0 for an empty bucket).
// POS = uint32_t: one ds_wrxchg_rtn_b32.  POS = uint16_t (streams <= 64 KiB, half the LDS, twice
// the waves per CU): two buckets per dword, exchanged with ds_mskor_rtn_b32 -- the masked-or
// atomic replaces just the bucket's half ((old & ~mask) | p << sh) and returns the old dword.
template <typename POS>
__device__ __forceinline__ uint32_t fast_exchange(uint32_t v, int32_t p, bool valid, int tablog, B2H_LDS uint8_t* tab) {
  uint32_t old = 0;
  if (valid) {
    const uint32_t h = lz_hash(v, tablog);
    if (sizeof(POS) == 4) {
      old = __hip_atomic_exchange(&((B2H_LDS uint32_t*)tab)[h], (uint32_t)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      const uint32_t addr = (uint32_t)reinterpret_cast<uintptr_t>(tab) + ((h >> 1) << 2);
      const uint32_t sh = (h & 1u) << 4;
      const uint32_t mask = 0xffffu << sh, data = (uint32_t)p << sh;
      uint32_t w;
      asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(w) : "v"(addr), "v"(mask), "v"(data) : "memory");
      old = (w >> sh) & 0xffffu;
    }
  }
  return old;
}

// Candidate usable: 0 < distance < MAX_FARDISTANCE (blosc/blosclz.c:516-519).  Lanes without one
// load their own bytes (compares equal, flagged off).
__device__ __forceinline__ bool fast_cand_ok(int32_t p, uint32_t cand, bool valid) {
  const uint32_t d = (uint32_t)(p - (int32_t)cand);
  return valid && d != 0 && d < kLzFar;
}

// kCmpWords words (60 bytes) at p kept as the raw aligned dwords that hold them (+ the byte shift):
// the loads stay in flight across a whole tile of parsing and are only funnel-shifted when the
// bytes are used.  60 bytes up front: on T's smooth plane 32 % of the matches are >= 28 bytes but
// only 8 % >= 60, and every longer one costs a global round trip (or a neighbour-lane lookup).
constexpr int kCmpWords = 15, kCmpBytes = 4 * kCmpWords, kNbrStride = kCmpBytes - 4;
struct RawCmp {
  uint32_t d[kCmpWords + 1];
  uint32_t sh;
};
__device__ __forceinline__ void rawc_load(gin_t p, RawCmp& r) {
  const B2H_GLB uint32_t* q = align4(p);
  r.sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
#pragma unroll
  for (int i = 0; i < kCmpWords + 1; i++) r.d[i] = q[i];
}
__device__ __forceinline__ uint32_t rawc_word(const RawCmp& r, int i) { return funnel(r.d[i], r.d[i + 1], r.sh); }

template <bool PROBE, typename POS>
__device__ __forceinline__ LzPassOut lz_pass_fast(gin_t in, int32_t length, int probe_hashlog, int tablog, gout_t out,
                                                  int32_t maxout, B2H_LDS uint8_t* tab, B2H_LDS uint8_t* oring,
                                                  int clevel) {
  const int lane = lane_id();
  constexpr int32_t ORM = kOutRing - 1;
  int32_t F = 0;   // output [0, F) already in `out`
  auto flush = [&](int32_t to) {
    for (int32_t y = F + lane; y < to; y += 64) out[y] = oring[y & ORM];
    F = to;
  };
  int32_t limit = length;
  if (PROBE) {
    const int32_t hl = 1 << probe_hashlog;
    limit = length > hl ? hl : length;
  }
  const int32_t bound = limit - 1, loop_end = limit - 12;
  {  // clear the table (16-byte LDS stores)
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    B2H_LDS u32x4* t16 = (B2H_LDS u32x4*)tab;
    const int32_t n16 = (int32_t)((sizeof(POS) << tablog) / 16);
    for (int32_t i = lane; i < n16; i += 64) t16[i] = u32x4{0u, 0u, 0u, 0u};
    asm volatile("" ::: "memory");
  }
  LzPassOut r;
  int32_t windows = 0;
  int32_t o = 5, lit = 4, pos;
  uint32_t byte0 = kLzMaxCopy - 1;   // out[0] is patched at the end (marker bit)
  if (PROBE) {
    pos = 0;
  } else {
    pos = 4;
    if (lane < 5) oring[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : in[lane - 1];
  }
  int32_t peak = 0;
  bool fail = false;
  const double thr_o = PROBE ? 0.999 * (clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2
                                        : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0) : 0.0;
  const double thr_s = thr_o * (1.001 / 0.999);
  bool early = false, sure = false;
  EPROF_DECL;

  // ---- pipeline state: tile T (a, rr, cand), tiles T + 1 and T + 2 (a), the loads of T + 3 ----
  // Input loads are consumed two tiles after issue (an input line is an HBM miss every other
  // tile), candidate loads one tile after (recent positions: cache hits); vmcnt is in order, so
  // consuming tile T + 1's candidates leaves tile T + 3's input loads in flight.
  int32_t T = pos / kFastTile;
  RawCmp ca, crr, na, nna;
  uint32_t ccand = 0;
  auto load_a = [&](int32_t t, RawCmp& a) {
    const int32_t p = t * kFastTile + lane;
    rawc_load(in + (p < loop_end ? p : 0), a);
  };
  auto exchange_and_load = [&](int32_t t, const RawCmp& a, uint32_t& cand, RawCmp& rr) {
    const int32_t p = t * kFastTile + lane;
    const bool valid = p < loop_end;
    cand = fast_exchange<POS>(rawc_word(a, 0), p, valid, tablog, tab);
    const int32_t q = fast_cand_ok(p, cand, valid) ? (int32_t)cand : (valid ? p : 0);
    rawc_load(in + q, rr);
  };
  if (pos < loop_end) {
    load_a(T, ca);
    exchange_and_load(T, ca, ccand, crr);
    load_a(T + 1, na);
    load_a(T + 2, nna);
  }
  while (pos < loop_end) {
    if (PROBE) {
      if ((double)(limit + 64) < thr_o * (double)o) { early = true; break; }
      const int32_t R = loop_end - pos;
      if ((double)loop_end >= thr_s * (double)(o + R + R / 16 + 16)) { sure = true; break; }
    }
    windows++;
    EPROF_T(t0);
    if (!PROBE && o - F >= 1024) flush(F + 512);   // a tile emits < 512 bytes
    EPROF_T(t0f);
    EPROF_ADD(6, t0, t0f);
    const int32_t P = T * kFastTile;
    const int32_t p = P + lane;
    const bool valid = p < loop_end;
    const int32_t s0 = pos - P;                            // the parse enters the tile here
    const int32_t lim = min(kFastTile, loop_end - P);      // lanes below lim are main-loop positions
    // ---- stage B of tile T + 1 (table exchange, candidate loads) and stage A of tile T + 2: issued
    // first, consumed one tile later ----
    RawCmp nrr, n3a;
    uint32_t ncand = 0;
    exchange_and_load(T + 1, na, ncand, nrr);
    load_a(T + 3, n3a);
    EPROF_T(t1);
    EPROF_ADD(0, t0f, t1);
    // ---- stage C of tile T: candidate test (exactly as the serial loop decides) ----
    const uint32_t v = rawc_word(ca, 0);
    const uint32_t dist = (uint32_t)(p - (int32_t)ccand);
    // first mismatching byte of in[p..p+59] vs the candidate's (60: all equal), for every lane
    // with a usable candidate (mmd = -1 otherwise): the chain walk extends long matches from the
    // compares of later lanes that sit at the same distance
    const bool cok = fast_cand_ok(p, ccand, valid);
    int32_t mm = kCmpBytes;
#pragma unroll
    for (int i = kCmpWords - 1; i >= 0; i--) {
      const uint32_t x = rawc_word(ca, i) ^ rawc_word(crr, i);
      if (x) mm = 4 * i + (__builtin_ctz(x) >> 3);
    }
    const int32_t mmd = cok ? mm : -1;
    bool accept = false;
    int32_t lenx = 0;   // match length, or -1: the first kCmpBytes all match (extend later)
    if (lane >= s0 && cok && mm >= 4) {
      const int32_t e = min(mm < kCmpBytes ? p + mm + 1 : 0x7fffffff, bound);
      const int32_t len = e - 4 - p;
      accept = len >= 4 && (PROBE || !(len <= 5 && (dist - 1) >= kLzNear));
      lenx = (mm < kCmpBytes || p + kCmpBytes + 1 >= bound) ? len : -1;
    }

    const uint64_t am = __ballot(accept);
    EPROF_T(t2);
    EPROF_ADD(1, t1, t2);
    if (PROBE && am == 0) {
      // all-literal probe tile: closed-form count of lanes s0 .. lim-1
      const int32_t cnt = lim - s0;
      o += cnt + (lit + cnt) / 32;
      lit = (lit + cnt) & 31;
      pos = P + lim;
    } else {
      // ---- chain walk: the matches the greedy parse takes in this tile ----
      uint64_t chain = 0;
      int32_t ser = -1;    // a match with length-extension bytes (scalar token path)
      int32_t endc2 = -1;  // end + 2 of the last chain match, relative to P
      {
        uint64_t rem = am;
        while (rem) {
          const int32_t m = __builtin_ctzll(rem);
          int32_t lm = rdlane(lenx, m);
          if (lm < 0) {
            EPROF_T(te0);
            // bytes [p_m, p_m + L) are verified; lane m + 56 k compared the next 60 at the same
            // distance if its candidate sits there: follow those lanes, go to memory only past them
            const int32_t pm = P + m;
            const uint32_t dm = (uint32_t)rdlane((int32_t)dist, m);
            int32_t L = kCmpBytes, e = -1;
            for (int32_t j = m + kNbrStride; j < kFastTile; j += kNbrStride) {
              if (pm + L >= bound) { e = bound; break; }
              const int32_t mj = rdlane(mmd, j);
              if (mj < 0 || (uint32_t)rdlane((int32_t)dist, j) != dm) break;
              if (mj < kCmpBytes) { e = min(P + j + mj + 1, bound); break; }
              L = j - m + kCmpBytes;
            }
            if (e < 0) e = pm + L >= bound ? bound : wave_match_end(in, pm + L, dm, bound);
            lm = e - 4 - pm;
            lenx = lane == m ? lm : lenx;
            EPROF_T(te1);
            EPROF_ADD(5, te0, te1);
          }
          if (lm >= 262) { ser = m; break; }   // (len - 7) / 255 extension bytes
          chain |= 1ull << m;
          const int32_t c2 = m + lm + 2;         // the greedy parse resumes at the match end + 2
          endc2 = c2;
          if (c2 >= kFastTile) break;
          rem = am & (~0ull << c2);
        }
      }
      EPROF_T(t3);
      EPROF_ADD(2, t2, t3);
      // ---- all tokens of the tile at once (the exact-mode window emission, entered at s0) ----
      const bool ischain = (chain >> lane) & 1ull;
      // chain matches do not overlap, so their resume points c2 grow with the lane: the last one
      // strictly before each lane is a max-scan shifted by one lane (DPP wave_shr:1, lane 0: -1)
      const int32_t c2v = lane + lenx + 2;
      const int32_t c2incl = wave_scan_max(ischain ? c2v : -1);
      const int32_t pc2 = __builtin_amdgcn_update_dpp(-1, c2incl, 0x138, 0xf, 0xf, false);
      const bool hasprev = pc2 >= 0;
      const int32_t segstart = hasprev ? pc2 : s0;
      const int32_t lpos = (hasprev ? 0 : lit) + lane - segstart;
      const int32_t lit_end = ser >= 0 ? ser : lim;
      const bool islit = !ischain && lane >= segstart && lane < lit_end;
      const int32_t rr5 = lpos & 31;
      const uint32_t bd = dist - 1;
      const bool near = bd < kLzNear;
      const uint32_t ulen = (uint32_t)lenx;
      const int32_t tok = ulen < 7 ? (near ? 2 : 4) : (near ? 3 : 5);
      int32_t contrib = 0;
      if (islit) contrib = 1 + (rr5 == 31 ? 1 : 0);
      if (ischain) contrib = tok + 1 - (rr5 == 0 ? 1 : 0);
      const int32_t incl = wave_scan_add(contrib);
      const int32_t excl = incl - contrib;
      const uint64_t litm = __ballot(islit);
      const uint64_t elems = litm | chain;
      if (elems) {
        const int32_t le = 63 - __builtin_clzll(elems);
        const bool lelit = (litm >> le) & 1ull;
        if (!PROBE) {
          const int32_t base = o + excl;
          const int32_t ts = base - (rr5 == 0 ? 1 : 0);
          const int32_t req = lelit ? rdlane(base, le) + 2 : rdlane(ts + tok + 1, le);
          peak = max(peak, req);
          if (req > maxout) { fail = true; break; }
          // Every element writes a fixed 6-byte slot from its start in DESCENDING byte order: a
          // position's owner always has the lowest byte index among the elements that touch it
          // (the others start earlier), so the owner's byte lands last and the bytes past an
          // element's end need no masks: the next element's first byte replaces a literal's
          // pending run marker or a token's trailing marker exactly as the reference overwrites it.
          // Token bytes (MATCH_SHORT/LONG/_FAR, blosc/blosclz.c:270-316) + the marker opening the
          // next literal run, built without branches.
          if (islit || ischain) {
            const uint32_t fd = bd - kLzNear;
            const bool lng = ulen >= 7;
            const uint32_t b0 = (lng ? (7u << 5) : (ulen << 5)) + (near ? (bd >> 8) : 31u);
            const uint32_t dbytes = near ? (bd & 255u) : (255u | ((fd >> 8) << 8) | ((fd & 255u) << 16));
            uint64_t rest = (uint64_t)dbytes | (31ull << (near ? 8 : 24));
            if (lng) rest = (uint64_t)(ulen - 7) | (rest << 8);
            const uint64_t bytes = islit ? (uint64_t)((v & 0xffu) | ((uint32_t)(kLzMaxCopy - 1) << 8))
                                         : ((uint64_t)b0 | (rest << 8));
            const int32_t start = islit ? base : ts;
#pragma unroll
            for (int i = 5; i >= 0; i--) oring[(start + i) & ORM] = (uint8_t)(bytes >> (8 * i));
          }
          if (ischain && rr5 > 0) oring[(ts - rr5 - 1) & ORM] = (uint8_t)(rr5 - 1);
          const uint64_t z = __ballot(ischain && rr5 > 0 && ts - rr5 - 1 == 0);
          if (z) byte0 = (uint32_t)(rdlane(rr5, __builtin_ctzll(z)) - 1);
        }
        lit = lelit ? ((rdlane(lpos, le) + 1) & 31) : 0;
      }
      o += rdlane(incl, 63);
      EPROF_T(t4);
      EPROF_ADD(3, t3, t4);
      int32_t next_rel = max(endc2, lim);
      // ---- a match with extension bytes: the scalar token path ----
      if (ser >= 0) {
        const uint32_t dm = (uint32_t)rdlane((int32_t)dist, ser);
        const int32_t lm = rdlane(lenx, ser);
        const uint32_t sbd = dm - 1;
        const uint32_t sulen = (uint32_t)lm;
        const bool snear = sbd < kLzNear;
        int32_t at = -1;
        const uint32_t hdr = (uint32_t)(lit - 1);
        if (lit) {
          at = o - lit - 1;
          if (!PROBE && at == 0) byte0 = hdr;
        } else {
          o--;
        }
        lit = 0;
        const int32_t ext = (int32_t)((sulen - 7) / 255);
        const int32_t stok = 1 + ext + (snear ? 2 : 4);
        if (!PROBE) {
          peak = max(peak, o + stok + 1);
          if (o + stok + 1 > maxout) {
            fail = true;
          } else {
            if (lane == 0 && at >= 0) oring[at & ORM] = (uint8_t)hdr;
            const uint32_t remlen = (sulen - 7) - 255u * (uint32_t)ext;
            const uint32_t fd = sbd - kLzNear;
            if (lane == 0) oring[o & ORM] = (uint8_t)((7u << 5) + (snear ? (sbd >> 8) : 31u));
            for (int32_t i0 = 0; i0 < ext; i0 += 512) {
              if (o + 1 + i0 + 512 - F > kOutRing) flush(o + 1 + i0);
              for (int32_t i = i0 + lane; i < min(ext, i0 + 512); i += 64) oring[(o + 1 + i) & ORM] = 255;
            }
            if (o + 1 + ext + 5 - F > kOutRing) flush(o + 1 + ext);
            if (lane == 0) {
              const int32_t qq = o + 1 + ext;
              oring[qq & ORM] = (uint8_t)remlen;
              if (snear) { oring[(qq + 1) & ORM] = (uint8_t)(sbd & 255); oring[(qq + 2) & ORM] = (uint8_t)(kLzMaxCopy - 1); }
              else { oring[(qq + 1) & ORM] = 255; oring[(qq + 2) & ORM] = (uint8_t)(fd >> 8); oring[(qq + 3) & ORM] = (uint8_t)(fd & 255); oring[(qq + 4) & ORM] = (uint8_t)(kLzMaxCopy - 1); }
            }
          }
        }
        o += stok + 1;
        next_rel = ser + lm + 2;
      }
      if (fail) break;
      pos = P + next_rel;
    }
    // ---- advance the pipeline ----
    EPROF_T(t5);
    const int32_t NT = pos / kFastTile;
    if (pos >= loop_end) break;
    if (NT == T + 1) {
      ca = na;
      crr = nrr;
      na = nna;
      nna = n3a;
      ccand = ncand;
      T = NT;
    } else {   // a match jumped past tile T + 1: restart at its end
      T = NT;
      load_a(T, ca);
      exchange_and_load(T, ca, ccand, crr);
      load_a(T + 1, na);
      load_a(T + 2, nna);
    }
    EPROF_T(t6);
    EPROF_ADD(4, t5, t6);
  }
  EPROF_FLUSH;

  if (!PROBE && !fail) {
    // tail literals [pos, bound]
    while (pos <= bound) {
      if (o - F >= 1024) flush(F + 512);
      const int32_t cnt = min(64, bound - pos + 1);
      const int32_t last = o + (cnt - 1) + (lit + cnt - 1) / 32;
      peak = max(peak, last + 2);
      if (last + 2 > maxout) { fail = true; break; }
      if (lane < cnt) {
        const int32_t off = o + lane + (lit + lane) / 32;
        oring[off & ORM] = in[pos + lane];
        if (((lit + lane + 1) & 31) == 0) oring[(off + 1) & ORM] = (uint8_t)(kLzMaxCopy - 1);
      }
      o += cnt + (lit + cnt) / 32;
      lit = (lit + cnt) & 31;
      pos += cnt;
    }
    if (!fail) {
      if (lit) {
        const int32_t at = o - lit - 1;
        if (lane == 0) oring[at & ORM] = (uint8_t)(lit - 1);
        if (at == 0) byte0 = (uint32_t)(lit - 1);
      } else {
        o--;
      }
      if (F == 0) {
        if (lane == 0) oring[0] = (uint8_t)(byte0 | 0x20u);
        flush(o);
      } else {
        flush(o);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the flushed byte 0 first
        if (lane == 0) out[0] = (uint8_t)(byte0 | 0x20u);
      }
    }
  }
  r.o = o;
  r.pos = pos;
  r.peak = peak;
  r.fail = fail;
  r.early = early;
  r.sure = sure;
  r.windows = windows;
  return r;
}

// Fast-mode stream encode with maxout = neblock: run test, fast probe (the reference's decision
// rule over a fast-mode parse), fast main pass.  tablog: the LDS table (<= the clevel's hashlog).
template <typename POS>
__device__ __forceinline__ StreamResult encode_stream_fast(gin_t in, int32_t n, int clevel, gout_t out,
                                                           B2H_LDS uint8_t* tab, int tablog, B2H_LDS uint8_t* oring,
                                                           bool allow_runs) {
  StreamResult res;
  res.windows = 0;
  res.cycles = 0;
  res.peak = 0;
  if (allow_runs && wave_is_run(in, n)) {
    res.size = in[0];
    res.kind = res.size ? kStreamByteRun : kStreamZeroRun;
    return res;
  }
  res.kind = kStreamRaw;
  res.size = 0;
  const int hashlog = clevel == 1 ? 12 : (clevel == 2 ? 13 : 14);
  const int tl = min(tablog, hashlog);
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  const LzPassOut pr = lz_pass_fast<true, POS>(in + (n - maxlen), maxlen, hashlog, tl, out, 0, tab, oring, clevel);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (pr.early || (!pr.sure && ratio < thr) || n < 16 || n < 66) return res;
  const LzPassOut em = lz_pass_fast<false, POS>(in, n, hashlog, tl, out, n, tab, oring, clevel);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

}  // namespace b2h
