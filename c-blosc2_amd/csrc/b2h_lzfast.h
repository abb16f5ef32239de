// b2h_lzfast.h -- BloscLZ "fast mode" encoder for gfx950 (device code).
//
// Same token grammar, greedy rule, length / distance limits, entropy-probe thresholds and byte
// emission as blosclz_compress (blosc/blosclz.c:248-316, 320-419, 422-619); the ONE difference is
// which earlier position a hash bucket offers as a position's candidate.  The reference inserts
// only the positions its serial walk visits, so every candidate depends on the whole parse before
// it and the walk is a latency chain (exact mode, b2h_lz.h, ~9 000 cycles per 64 positions on T's
// smooth plane).  Fast mode inserts positions in TILES of 64, in tile order, independently of the
// parse (semantics and their CPU model: tools/fm_model.c): entering tile T, the parse inserts T
// (if a jump skipped it) and T + 1; tiles a long match jumps over are never inserted.
//
//   * one LDS atomic exchange per lane swaps the lane's position into its bucket and returns the
//     bucket's previous position -- the most recent earlier position with that hash, earlier lanes
//     of the same tile included (LDS applies the lanes of one instruction in lane order);
//   * so a tile's candidates, their 60-byte compares and match lengths are known before the parse
//     reaches it.  Two waves of a workgroup share one stream's table: the MATCHER exchanges and
//     compares tile T + 1 while the PARSER parses tile T with the exact-mode window code (ballot
//     chain walk, DPP prefix-sum emission through the LDS output ring), the two meeting at one
//     barrier per tile.
//
// Every match is verified byte for byte against its candidate, so any output decodes with
// blosclz_decompress; the ratio on T is within 0.1 % of the reference's.
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

// ============================================================ matcher / parser workgroup ====
// One stream per workgroup of two waves (k_encode_fast):
//   wave 0, the MATCHER: tile exchanges, candidate loads and 60-byte compares -- for each lane of a
//     tile its candidate distance, first mismatch and input byte, handed over through LDS;
//   wave 1, the PARSER: chain walk, token emission, output ring and flushes.
// Lockstep, one barrier per tile.  A match jumping past tile T + 1 costs one step in which the
// matcher produces the jump target and the parser waits.  The split keeps each wave within 128
// VGPRs, so a CU holds 8 streams x 2 waves (measured: the encoder is issue-bound at that
// occupancy, so a deeper matcher pipeline -- exchange T + 2 while comparing T + 1 -- ran slower).
struct FastShared {          // per workgroup, after the table and the output ring
  uint32_t dist[2][64];      // hand-over slots: candidate distance
  uint32_t aux[2][64];       //   (first mismatch + 1) | input byte << 8 (mismatch + 1 == 0: no candidate)
  int32_t ctrl[2];           // parser -> matcher: next tile, or -1 (stop); by iteration parity
  int32_t decide[2];         // the stream's probe decision / run verdict (parser -> both)
  int32_t pull;              // the stream index the workgroup pulled
  int32_t bcast;             // k_encode_fast_fused: claims and hand-off words, lane 0 -> workgroup
};

// Pass limits shared by both roles (blosc/blosclz.c:440-482, get_cratio 320-419).
template <bool PROBE>
__device__ __forceinline__ void fast_limits(int32_t length, int probe_hashlog, int32_t* limit, int32_t* bound,
                                            int32_t* loop_end) {
  int32_t lim = length;
  if (PROBE) {
    const int32_t hl = 1 << probe_hashlog;
    lim = length > hl ? hl : length;
  }
  *limit = lim;
  *bound = lim - 1;
  *loop_end = lim - 12;
}

// Clear one wave's half of the table (the matcher the first half, the parser the second).
template <typename POS>
__device__ __forceinline__ void fast_clear_half(B2H_LDS uint8_t* tab, int tablog, bool first) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  B2H_LDS u32x4* t16 = (B2H_LDS u32x4*)tab;
  const int32_t n16 = (int32_t)((sizeof(POS) << tablog) / 16);
  const int32_t h = n16 / 2;
  for (int32_t i = (first ? 0 : h) + lane_id(); i < (first ? h : n16); i += 64) t16[i] = u32x4{0u, 0u, 0u, 0u};
}

// The two roles of one pass run as two SEPARATE loops with the same barrier sequence (one barrier
// per step; the step's control word is read by both from LDS after it, as a uniform value): each
// role's loop-carried state is live in its own loop only, so the kernel's register allocation is
// the larger of the two, not their sum (one shared loop with a role branch inside kept both roles'
// state live everywhere and spilled ~170 SGPRs into VGPR lanes).
//
// MATCHER: tile exchanges, candidate loads and 60-byte compares -> the hand-over slots.
template <bool PROBE, typename POS>
__device__ __forceinline__ void lz_pass_fast_matcher(gin_t __restrict__ in, int32_t length, int probe_hashlog, int tablog,
                                                               B2H_LDS uint8_t* tab, B2H_LDS FastShared* sh) {
  const int lane = lane_id();
  int32_t limit, bound, loop_end;
  fast_limits<PROBE>(length, probe_hashlog, &limit, &bound, &loop_end);
  (void)bound;
  fast_clear_half<POS>(tab, tablog, true);
  // ---- matcher: the first input words of tile `ant` (prefetched one step ahead); the other 14
  // are loaded only when some lane's candidate matches its first 4 bytes, together with the
  // candidates' words (the same round trip): incompressible tiles issue 4 loads per lane, not 18 ----
  RawCmp na;
  int32_t ant = -1;
  auto load_a = [&](int32_t t, RawCmp& a) {
    const int32_t p = t * kFastTile + lane;
    gin_t q8 = in + (p < loop_end ? p : 0);
    const B2H_GLB uint32_t* q = align4(q8);
    a.sh = (uint32_t)(reinterpret_cast<uintptr_t>(q8) & 3);
    a.d[0] = q[0];
    a.d[1] = q[1];
  };
  // insert tile t, test every lane's candidate, hand the results over in slot `slot`
  auto produce = [&](int32_t t, int slot) {
    RawCmp a;
    if (t == ant) a = na;
    else load_a(t, a);
    const int32_t p = t * kFastTile + lane;
    const bool valid = p < loop_end;
    const uint32_t cand = fast_exchange<POS>(rawc_word(a, 0), p, valid, tablog, tab);
    const bool cok = fast_cand_ok(p, cand, valid);
    // the candidate's first word decides most tiles: when no lane's 4 bytes match, every first
    // mismatch lies in word 0 and the other 14 words are neither loaded nor compared
    gin_t cq = in + (cok ? (int32_t)cand : (valid ? p : 0));
    const B2H_GLB uint32_t* cw = align4(cq);
    const uint32_t csh = (uint32_t)(reinterpret_cast<uintptr_t>(cq) & 3);
    const uint32_t c0 = cw[0], c1 = cw[1];
    load_a(t + 1, na);   // issued after the candidate loads: the compare waits for those only
    ant = t + 1;
    const uint32_t x0 = rawc_word(a, 0) ^ funnel(c0, c1, csh);
    int32_t mm;
    if (__ballot(cok && x0 == 0) == 0) {
      mm = x0 ? (int32_t)(__builtin_ctz(x0) >> 3) : 4;
    } else {
      uint32_t c[kCmpWords + 1];
      c[0] = c0;
      c[1] = c1;
      const B2H_GLB uint32_t* aw = align4(in + (p < loop_end ? p : 0));
#pragma unroll
      for (int i = 2; i < kCmpWords + 1; i++) {
        c[i] = cw[i];
        a.d[i] = aw[i];
      }
      mm = kCmpBytes;
#pragma unroll
      for (int i = kCmpWords - 1; i >= 1; i--) {
        const uint32_t x = rawc_word(a, i) ^ funnel(c[i], c[i + 1], csh);
        if (x) mm = 4 * i + (__builtin_ctz(x) >> 3);
      }
      if (x0) mm = (int32_t)(__builtin_ctz(x0) >> 3);
    }
    sh->dist[slot][lane] = (uint32_t)(p - (int32_t)cand);
    sh->aux[slot][lane] = (uint32_t)(cok ? mm + 1 : 0) | ((rawc_word(a, 0) & 0xffu) << 8);
  };

  const int32_t pos = PROBE ? 0 : 4;
  int32_t T = pos / kFastTile, pend = -1;
  int cur = 0, it = 0;
  const bool any = pos < loop_end;
  __syncthreads();                           // table cleared
  if (any) produce(T, 0);                    // entering T: T and T + 1
  __syncthreads();
  while (any) {
    if (pend >= 0) produce(pend, cur ^ 1);               // the parser jumps to `pend`
    else if ((T + 1) * kFastTile < loop_end) produce(T + 1, cur ^ 1);
    __syncthreads();
    if (pend >= 0) {   // the matcher produced the jump target: the parser takes it next
      T = pend;
      cur ^= 1;
      pend = -1;
      continue;
    }
    const int32_t c = __builtin_amdgcn_readfirstlane(sh->ctrl[it & 1]);
    it++;
    if (c < 0) break;
    if (c == T + 1) {
      T = c;
      cur ^= 1;
    } else {
      pend = c;
    }
  }
}

// PARSER: chain walk, token emission, output ring and flushes, the tail.
template <bool PROBE, typename POS, bool WT>
__device__ __forceinline__ LzPassOut lz_pass_fast_parser(gin_t __restrict__ in, int32_t length, int probe_hashlog,
                                                                   int tablog, gout_t __restrict__ out, int32_t maxout,
                                                                   B2H_LDS uint8_t* tab, B2H_LDS uint8_t* oring,
                                                                   B2H_LDS FastShared* sh, int clevel) {
  const int lane = lane_id();
  constexpr int32_t ORM = kOutRing - 1;
  int32_t limit, bound, loop_end;
  fast_limits<PROBE>(length, probe_hashlog, &limit, &bound, &loop_end);
  fast_clear_half<POS>(tab, tablog, false);
  LzPassOut r;
  int32_t windows = 0;
  int32_t F = 0;   // output [0, F) already in `out`
  auto flush = [&](int32_t to) {
    ring_flush<WT>(out, oring, F, to);
    F = to;
  };
  int32_t o = 5, lit = 4, pos = PROBE ? 0 : 4;
  uint32_t byte0 = kLzMaxCopy - 1;
  if (!PROBE && lane < 5) oring[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : in[lane - 1];
  int32_t peak = 0;
  bool fail = false, early = false, sure = false;
  const double thr_o = PROBE ? 0.999 * (clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2
                                        : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0) : 0.0;
  const double thr_s = thr_o * (1.001 / 0.999);
  EPROF_DECL;
  int32_t T = pos / kFastTile, pend = -1;
  int cur = 0, it = 0;
  const bool any = pos < loop_end;
  __syncthreads();                           // table cleared
  __syncthreads();                           // the matcher produced the first tile
  while (any) {
    if (pend < 0) {
      int32_t nt = -1;
      do {
        if (PROBE) {
          if ((double)(limit + 64) < thr_o * (double)o) { early = true; break; }
          const int32_t R = loop_end - pos;
          if ((double)loop_end >= thr_s * (double)(o + R + R / 16 + 16)) { sure = true; break; }
        }
        windows++;
        EPROF_T(t0);
        if (!PROBE && o - F >= 1024) flush(F + 512);   // a tile emits < 512 bytes
        const int32_t P = T * kFastTile;
        const int32_t p = P + lane;
        const int32_t s0 = pos - P;
        const int32_t lim = min(kFastTile, loop_end - P);
        const uint32_t dist = sh->dist[cur][lane];
        const uint32_t ax = sh->aux[cur][lane];
        const int32_t mmd = (int32_t)(ax & 0xffu) - 1;   // -1: no usable candidate
        const uint32_t vbyte = (ax >> 8) & 0xffu;
        bool accept = false;
        int32_t lenx = 0;
        if (lane >= s0 && mmd >= 4) {
          const int32_t e = min(mmd < kCmpBytes ? p + mmd + 1 : 0x7fffffff, bound);
          const int32_t len = e - 4 - p;
          accept = len >= 4 && (PROBE || !(len <= 5 && (dist - 1) >= kLzNear));
          lenx = (mmd < kCmpBytes || p + kCmpBytes + 1 >= bound) ? len : -1;
        }
        const uint64_t am = __ballot(accept);
        EPROF_T(t2);
        EPROF_ADD(1, t0, t2);
        if (PROBE && am == 0) {
          const int32_t cnt = lim - s0;
          o += cnt + (lit + cnt) / 32;
          lit = (lit + cnt) & 31;
          pos = P + lim;
        } else {
          uint64_t chain = 0;
          int32_t ser = -1, endc2 = -1;
          {
            uint64_t rem = am;
            while (rem) {
              const int32_t m = __builtin_ctzll(rem);
              int32_t lm = rdlane(lenx, m);
              if (lm < 0) {
                EPROF_T(te0);
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
              if (lm >= 262) { ser = m; break; }
              chain |= 1ull << m;
              const int32_t c2 = m + lm + 2;
              endc2 = c2;
              if (c2 >= kFastTile) break;
              rem = am & (~0ull << c2);
            }
          }
          EPROF_T(t3);
          EPROF_ADD(2, t2, t3);
          const bool ischain = (chain >> lane) & 1ull;
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
                const uint64_t bytes = islit ? (uint64_t)(vbyte | ((uint32_t)(kLzMaxCopy - 1) << 8))
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
          if (ser >= 0) {   // a match with length-extension bytes: the scalar token path
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
        if (pos < loop_end) nt = pos / kFastTile;
      } while (false);
      if (lane == 0) sh->ctrl[it & 1] = nt;
    }
    EPROF_T(tb0);
    __syncthreads();
    EPROF_T(tb1);
    EPROF_ADD(6, tb0, tb1);
    if (pend >= 0) {   // the matcher produced the jump target: take it
      T = pend;
      cur ^= 1;
      pend = -1;
      continue;
    }
    const int32_t c = __builtin_amdgcn_readfirstlane(sh->ctrl[it & 1]);
    it++;
    if (c < 0) break;
    if (c == T + 1) {
      T = c;
      cur ^= 1;
    } else {
      pend = c;
    }
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
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) st8<WT>(out, wt_rsrc(out), 0, (uint8_t)(byte0 | 0x20u));
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

// One pass, both roles (the matcher's result is not used).
template <bool PROBE, typename POS, bool WT>
__device__ __forceinline__ LzPassOut lz_pass_fast(gin_t in, int32_t length, int probe_hashlog, int tablog, gout_t out,
                                                   int32_t maxout, B2H_LDS uint8_t* tab, B2H_LDS uint8_t* oring,
                                                   B2H_LDS FastShared* sh, int clevel, bool matcher) {
  if (matcher) {
    lz_pass_fast_matcher<PROBE, POS>(in, length, probe_hashlog, tablog, tab, sh);
    LzPassOut r;
    r.o = 1;
    r.pos = 0;
    r.peak = 0;
    r.fail = false;
    r.early = false;
    r.sure = false;
    r.windows = 0;
    return r;
  }
  return lz_pass_fast_parser<PROBE, POS, WT>(in, length, probe_hashlog, tablog, out, maxout, tab, oring, sh, clevel);
}

// Two-wave fast-mode stream encode: both waves run this; the parser's StreamResult is the one
// to keep.  The run test is split between the waves; decisions travel through sh->decide.
template <typename POS, bool WT = false>
__device__ __forceinline__ StreamResult encode_stream_fast(gin_t __restrict__ in, int32_t n, int clevel, gout_t __restrict__ out,
                                                            B2H_LDS uint8_t* tab, int tablog, B2H_LDS uint8_t* oring,
                                                            B2H_LDS FastShared* sh, bool allow_runs, bool matcher) {
  StreamResult res;
  res.windows = 0;
  res.cycles = 0;
  res.peak = 0;
  res.kind = kStreamRaw;
  res.size = 0;
  if (allow_runs) {
    // each wave tests its half against in[0]; both read both verdicts
    const int32_t h = (n / 2) & ~15;
    const bool half_run = matcher ? wave_is_run(in, h + 1) : wave_is_run_from(in, h, n, in[0]);
    if (lane_id() == 0) sh->decide[matcher ? 0 : 1] = half_run ? 1 : 0;
    __syncthreads();
    const bool run = sh->decide[0] && sh->decide[1];
    __syncthreads();   // both read before the next write
    if (run) {
      res.size = in[0];
      res.kind = res.size ? kStreamByteRun : kStreamZeroRun;
      return res;
    }
  }
  const int hashlog = clevel == 1 ? 12 : (clevel == 2 ? 13 : 14);
  const int tl = min(tablog, hashlog);
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  const LzPassOut pr = lz_pass_fast<true, POS, WT>(in + (n - maxlen), maxlen, hashlog, tl, out, 0, tab, oring, sh, clevel,
                                                matcher);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (!matcher && lane_id() == 0) sh->decide[0] = (pr.early || (!pr.sure && ratio < thr) || n < 66) ? 0 : 1;
  __syncthreads();
  const bool go = sh->decide[0] != 0;
  __syncthreads();
  if (!go) return res;
  const LzPassOut em = lz_pass_fast<false, POS, WT>(in, n, hashlog, tl, out, n, tab, oring, sh, clevel, matcher);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

}  // namespace b2h
