// b2h_lzfast.h -- BloscLZ "fast mode" encoder for gfx950 (device code).
//
// Same token grammar, greedy rule, length / distance limits, entropy-probe thresholds and byte
// emission as blosclz_compress (blosc/blosclz.c:248-316, 320-419, 422-619); the ONE difference is
// which earlier position a hash bucket offers as a position's candidate.  The reference inserts
// only the positions its serial walk visits, so every candidate depends on the whole parse before
// it and the walk is a latency chain (exact mode, b2h_lz.h, ~9 000 cycles per 64 positions on T's
// smooth plane).  Fast mode inserts positions in TILES of 128, in tile order, independently of the
// parse (semantics and their CPU model: tools/fm_model.c): entering tile T, the parse inserts T
// (if a jump skipped it) and T + 1; tiles a long match jumps over are never inserted.
//
//   * one LDS atomic exchange per lane and half swaps the position into its bucket and returns the
//     bucket's previous position -- the most recent earlier position with that hash, earlier
//     positions of the same tile included (LDS applies the lanes of one instruction in lane order,
//     and the wave's two exchanges in program order);
//   * so a tile's candidates, their 60-byte compares and match lengths are known before the parse
//     reaches it.  Two waves of a workgroup share one stream's table: the MATCHER exchanges and
//     compares tile T + 1 while the PARSER parses tile T with the exact-mode window code (ballot
//     chain walk, DPP prefix-sum emission through the LDS output ring), the two meeting at one
//     barrier per tile.
//
// Every match is verified byte for byte against its candidate, so any output decodes with
// blosclz_decompress; the ratio on T is within 0.1 % of the reference's.
//
// DEEP (BloscLZ mode 2): the candidate is the best of the bucket chain c1, prev[c1], ... (up to
// kDeepDepth links, by leading equal bytes up to kDeepSel, the newest on a tie -- tools/fm_model.c
// insert_tile).  The matcher records prev[p] = c1 in a per-workgroup global array (links into the
// tile being inserted come from the lanes' own exchange results) and walks the chains of a tile's
// 128 positions together, one load round trip per link.
#pragma once
#include "b2h_lz.h"

namespace b2h {

// Positions per parse step: two 64-lane HALVES.  The parser's per-step cost is mostly a fixed
// latency chain (LDS hand-over reads, two DPP scans, ballots, the ring writes, the barrier:
// measured 1 600 of 3 100 cycles per 64-position step on T's smooth plane, the chain walk the
// rest), so both halves go through the same instructions and their chains overlap.
constexpr int kFastTile = 128, kHalf = 64;
#ifndef B2H_PROBE_AHEAD
#define B2H_PROBE_AHEAD 0   // 1: the probe's matcher inserts T + 2 while the parser is on T (measured slower)
#endif
constexpr bool kProbeAhead = B2H_PROBE_AHEAD != 0;
#ifndef B2H_PASS_PRIO
#define B2H_PASS_PRIO 1   // 1: issue priority to the probe's matcher and the emitting pass's parser
#endif

// Table exchange of 64 positions: the lanes with p < loop_end hash in[p..p+3] (v) and swap p into
// the bucket.  Returns the candidate (the bucket's previous position; 0 for an empty bucket).
// POS = uint32_t: one ds_wrxchg_rtn_b32.  POS = uint16_t (half the LDS, twice the waves per CU):
// two buckets per dword, exchanged with ds_mskor_rtn_b32 -- the masked-or atomic replaces just the
// bucket's half ((old & ~mask) | p << sh) and returns the old dword.  A u16 bucket holds its
// position modulo 2^16 and the candidate is the latest position below p with those low bits: the
// bucket's own position while p < 2^16 (every stream of a split chunk), and past it the bucket's
// position or, for a bucket older than 2^16 positions, a nearer one with the same low bits -- a
// suggestion like any other, verified byte for byte (tools/fm_model.c, the same rule).  So streams
// longer than 64 KiB (unsplit blocks: BITSHUFFLE, leftovers) run at the u16 table's occupancy too.
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
      const uint32_t mask = 0xffffu << sh, data = ((uint32_t)p & 0xffffu) << sh;
      uint32_t w;
      asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                   : "=v"(w) : "v"(addr), "v"(mask), "v"(data) : "memory");
      old = (uint32_t)p - (((uint32_t)p - ((w >> sh) & 0xffffu)) & 0xffffu);
    }
  }
  return old;
}

// Both halves of a tile in one round trip (u16 buckets): the two ds_mskor_rtn_b32 go out back to
// back -- a wave's LDS instructions execute in order, so half 1's exchange still sees half 0's --
// and one wait covers both.  A lane past loop_end exchanges with an empty mask (a no-op).
template <typename POS>
__device__ __forceinline__ void fast_exchange2(const uint32_t (&v)[2], const int32_t (&p)[2], const bool (&valid)[2],
                                               int tablog, B2H_LDS uint8_t* tab, uint32_t (&cand)[2]) {
  if constexpr (sizeof(POS) == 4) {
#pragma unroll
    for (int h = 0; h < 2; h++) cand[h] = fast_exchange<POS>(v[h], p[h], valid[h], tablog, tab);
  } else {
    uint32_t addr[2], mask[2], data[2], sh[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t hh = lz_hash(v[h], tablog);
      addr[h] = (uint32_t)reinterpret_cast<uintptr_t>(tab) + ((hh >> 1) << 2);
      sh[h] = (hh & 1u) << 4;
      mask[h] = valid[h] ? 0xffffu << sh[h] : 0u;
      data[h] = valid[h] ? ((uint32_t)p[h] & 0xffffu) << sh[h] : 0u;
    }
    uint32_t w0, w1;
    asm volatile("ds_mskor_rtn_b32 %0, %2, %3, %4\n\tds_mskor_rtn_b32 %1, %5, %6, %7\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(w0), "=&v"(w1)
                 : "v"(addr[0]), "v"(mask[0]), "v"(data[0]), "v"(addr[1]), "v"(mask[1]), "v"(data[1])
                 : "memory");
    const uint32_t w[2] = {w0, w1};
#pragma unroll
    for (int h = 0; h < 2; h++)
      cand[h] = valid[h] ? (uint32_t)p[h] - (((uint32_t)p[h] - ((w[h] >> sh[h]) & 0xffffu)) & 0xffffu) : 0u;
  }
}

constexpr int kDeepDepth = 8, kDeepSel = 24;

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
__device__ __forceinline__ uint32_t rawc_word(const RawCmp& r, int i) { return funnel(r.d[i], r.d[i + 1], r.sh); }

// Hand-over record of one position, matcher -> parser: the match the serial loop would take there
// (L: 0 none, 4..57 its length, 127 longer than the 60-byte compare shows) | input byte << 7 |
// candidate distance << 15.  The matcher decides the position-local rules (distance range,
// minimum length, the far short-match rule, blosc/blosclz.c:516-540); the parser only masks the
// positions before its parse position.  A usable distance is < MAX_FARDISTANCE < 2^17.
constexpr int32_t kRecLong = 127;
__device__ __forceinline__ uint32_t rec_pack(int32_t L, uint32_t byte, uint32_t dist) {
  return (uint32_t)L | ((byte & 0xffu) << 7) | (dist << 15);
}
__device__ __forceinline__ int32_t rec_len(uint32_t w) { return (int32_t)(w & 127u); }
__device__ __forceinline__ uint32_t rec_byte(uint32_t w) { return (w >> 7) & 0xffu; }
__device__ __forceinline__ uint32_t rec_dist(uint32_t w) { return w >> 15; }

// ============================================================ matcher / parser workgroup ====
// One stream per workgroup of two waves (k_encode_fast):
//   wave 0, the MATCHER: tile exchanges, candidate loads and 60-byte compares -- for each position
//     of a tile its hand-over record, through LDS;
//   wave 1, the PARSER: chain walk, token emission, output ring and flushes.
// Lockstep, one barrier per tile.  A match jumping past tile T + 1 costs one step in which the
// matcher produces the jump target and the parser waits.  The split keeps each wave within 128
// VGPRs, so a CU holds 8 streams x 2 waves.
struct FastShared {          // per workgroup, after the table and the output ring
  uint32_t rec[2][kFastTile];   // hand-over records, by step parity
  int32_t ctrl[2];           // parser -> matcher: next tile, or -1 (stop); by iteration parity
  int32_t decide[2];         // the stream's probe decision / run verdict (parser -> both)
  int32_t pull;              // the stream index the workgroup pulled
  int32_t bcast;             // k_encode_fast_fused: claims and hand-off words, lane 0 -> workgroup
  uint32_t runred;           // k_encode_fast_fused: the (DELTA, SHUFFLE) job's plane-mismatch OR
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
// MATCHER: tile exchanges, candidate loads and 60-byte compares -> the hand-over records.
template <bool PROBE, typename POS, bool DEEP>
__device__ __forceinline__ void lz_pass_fast_matcher(gin_t __restrict__ in, int32_t length, int probe_hashlog, int tablog,
                                                               B2H_LDS uint8_t* tab, B2H_LDS FastShared* sh,
                                                               B2H_GLB POS* __restrict__ chain) {
  const int lane = lane_id();
  int32_t limit, bound, loop_end;
  fast_limits<PROBE>(length, probe_hashlog, &limit, &bound, &loop_end);
  fast_clear_half<POS>(tab, tablog, true);
  // ---- the first two input words of each half of tile `ant` (prefetched one step ahead); the
  // other 14 are loaded only when some lane's candidate matches its first 4 bytes, together with
  // the candidates' words (the same round trip): incompressible halves issue 4 loads per lane ----
  uint32_t na[2][2], nsh[2];
  int32_t ant = -1;
  auto load_a = [&](int32_t t, uint32_t (&w)[2][2], uint32_t (&s)[2]) {
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int32_t p = t * kFastTile + h * kHalf + lane;
      gin_t q8 = in + (p < loop_end ? p : 0);
      const B2H_GLB uint32_t* q = align4(q8);
      s[h] = (uint32_t)(reinterpret_cast<uintptr_t>(q8) & 3);
      w[h][0] = q[0];
      w[h][1] = q[1];
    }
  };
  // DEEP: record prev[p] = c1 and replace each position's candidate by the best of its chain
  // (tools/fm_model.c insert_tile; sel = equal leading bytes, at most kDeepSel, never at or past
  // `limit`; a link is followed while positive and within MAX_FARDISTANCE)
  auto deep_select = [&](int32_t t, const int32_t (&p)[2], const bool (&valid)[2], const uint32_t (&a0)[2][2],
                         const uint32_t (&ash)[2], uint32_t (&cand)[2], bool (&cok)[2]) {
    const int32_t P = t * kFastTile;
    uint32_t c1[2], aw[2][7];
    int32_t cc[2], best[2], bl[2], cap[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      c1[h] = cand[h];
      if (valid[h]) chain[p[h]] = (POS)c1[h];
      const B2H_GLB uint32_t* q = align4(in + (valid[h] ? p[h] : 0));
      aw[h][0] = a0[h][0];
      aw[h][1] = a0[h][1];
#pragma unroll
      for (int i = 2; i < 7; i++) aw[h][i] = q[i];
      cap[h] = min(kDeepSel, limit - p[h]);
      best[h] = (int32_t)c1[h];
      bl[h] = -1;
      cc[h] = (cok[h] && (int32_t)c1[h] > 0) ? (int32_t)c1[h] : 0;
    }
    for (int k = 0; k < kDeepDepth; k++) {
      if (__ballot(cc[0] > 0 || cc[1] > 0) == 0) break;   // wave-uniform
      int32_t nx[2];
      uint32_t cw7[2][7], csh[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        // the link: a position of this tile holds it in its lane's c1; an earlier one in `chain`
        const int32_t q = cc[h] - P;
        const int32_t l0 = __shfl((int)c1[0], q & 63), l1 = __shfl((int)c1[1], q & 63);
        const bool intile = q >= 0;
        nx[h] = (cc[h] > 0 && !intile && k + 1 < kDeepDepth) ? (int32_t)chain[cc[h]] : (q >= kHalf ? l1 : l0);
        gin_t cq = in + (cc[h] > 0 ? cc[h] : 0);
        const B2H_GLB uint32_t* cw = align4(cq);
        csh[h] = (uint32_t)(reinterpret_cast<uintptr_t>(cq) & 3);
#pragma unroll
        for (int i = 0; i < 7; i++) cw7[h][i] = cw[i];
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        int32_t n = kDeepSel;
#pragma unroll
        for (int i = 5; i >= 0; i--) {
          const uint32_t x = funnel(aw[h][i], aw[h][i + 1], ash[h]) ^ funnel(cw7[h][i], cw7[h][i + 1], csh[h]);
          if (x) n = 4 * i + (int32_t)(__builtin_ctz(x) >> 3);
        }
        n = min(n, cap[h]);
        if (cc[h] > 0 && n > bl[h]) { bl[h] = n; best[h] = cc[h]; }
        const bool more = cc[h] > 0 && bl[h] < cap[h] && k + 1 < kDeepDepth && nx[h] > 0 && p[h] - nx[h] < kLzFar;
        cc[h] = more ? nx[h] : 0;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      cand[h] = (uint32_t)best[h];
      cok[h] = fast_cand_ok(p[h], cand[h], valid[h]);
    }
  };
  // insert tile t (half 0, then half 1: position order), test every position's candidate, hand
  // the records over in slot `slot`
  EPROF_DECL;
  // Two phases per tile: AHEAD(t) inserts tile t and issues its candidates' first-word loads,
  // FINISH writes t's records.  (Measured and not kept, round 5: AHEAD one step before FINISH, so
  // the loads land across the barrier -- T 203.5 vs 203.2 GiB/s; and the two waves decoupled
  // through a 3-slot record ring with every tile inserted -- 203.6.  The matcher's step is not
  // load-latency-bound and the barrier is not the cost: both waves' chains share the SIMDs.)
  int32_t pti = 0;   // the tile AHEAD handled, for FINISH
  uint32_t pv[2], pcand[2], pc0[2], pc1[2], pa20[2] = {0u, 0u}, pa21[2] = {0u, 0u};
  bool pcok[2], palt[2] = {false, false};
  auto ahead = [&](int32_t t) {
    uint32_t a0[2][2], ash[2];
    if (t == ant) {
#pragma unroll
      for (int h = 0; h < 2; h++) { a0[h][0] = na[h][0]; a0[h][1] = na[h][1]; ash[h] = nsh[h]; }
    } else {
      load_a(t, a0, ash);
    }
    int32_t p[2];
    uint32_t cand[2];
    bool valid[2], cok[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      p[h] = t * kFastTile + h * kHalf + lane;
      valid[h] = p[h] < loop_end;
      pv[h] = funnel(a0[h][0], a0[h][1], ash[h]);
    }
    fast_exchange2<POS>(pv, p, valid, tablog, tab, cand);   // in order: half 1's positions follow half 0's
#pragma unroll
    for (int h = 0; h < 2; h++) cok[h] = fast_cand_ok(p[h], cand[h], valid[h]);
    if constexpr (DEEP) deep_select(t, p, valid, a0, ash, cand, cok);
    // every position's candidate words 0..1 (its first four bytes); lanes without a candidate load
    // their own bytes
#pragma unroll
    for (int h = 0; h < 2; h++) {
      gin_t cq = in + (cok[h] ? (int32_t)cand[h] : (valid[h] ? p[h] : 0));
      const B2H_GLB uint32_t* cw = align4(cq);
      pc0[h] = cw[0];
      pc1[h] = cw[1];
      // u16 buckets past 2^16 positions (fast_exchange): a near candidate may stand for one 2^16
      // positions further back (still within MAX_FARDISTANCE); when the near one's first 4 bytes
      // do not match, that one is offered instead (tools/fm_model.c insert_tile).  Its first words
      // come in the same round trip.  (Uniform: only streams longer than 2^16 positions.)
      if (sizeof(POS) == 2 && !DEEP && __builtin_amdgcn_readfirstlane(loop_end) > 65536) {
        palt[h] = cok[h] && cand[h] >= 65536u && (uint32_t)p[h] - cand[h] < kLzFar - 65536u;
        if (palt[h]) {
          pa20[h] = cw[-16384];   // 2^16 bytes back: the same alignment
          pa21[h] = cw[-16383];
        }
      }
      pcand[h] = cand[h];
      pcok[h] = cok[h];
    }
    load_a(t + 1, na, nsh);   // the next tile's own words, for the next AHEAD
    ant = t + 1;
    pti = t;
  };
  auto finish = [&](int slot) {
    const int32_t t = pti;
    int32_t p[2];
    uint32_t v[2], cand[2], c0[2], c1[2], csh[2];
    bool cok[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      p[h] = t * kFastTile + h * kHalf + lane;
      v[h] = pv[h];
      cand[h] = pcand[h];
      cok[h] = pcok[h];
      c0[h] = pc0[h];
      c1[h] = pc1[h];
      gin_t cq = in + (cok[h] ? (int32_t)cand[h] : (p[h] < loop_end ? p[h] : 0));
      csh[h] = (uint32_t)(reinterpret_cast<uintptr_t>(cq) & 3);
      if (palt[h] && (v[h] ^ funnel(c0[h], c1[h], csh[h])) != 0) {
        cand[h] -= 65536u;
        c0[h] = pa20[h];
        c1[h] = pa21[h];
      }
    }
    // ---- match ends by RUNS (the records are those of a 60-byte compare at every position) ----
    // E(q) = the first position >= q where in[x] != in[x - d(q)].  If q - 1 has the same distance
    // and its first four bytes match, E(q) = E(q - 1): a RUN of such positions shares one E, which
    // the run's LAST position determines -- from its first word when that mismatches (then it
    // ends the run), else by a 60-byte compare.  On T's smooth plane a tile holds ~23 runs, ~18 of
    // them needing the compare: one compacted 64-lane compare per tile instead of 128 lanes' worth,
    // and every position of a run whose end is known learns its exact length, past 60 bytes too
    // (up to the record's 126), which the parser would otherwise extend from memory.
    const int32_t P = t * kFastTile;
    uint32_t dd[2];
    int32_t mm0[2];
    bool zq[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t x0 = v[h] ^ funnel(c0[h], c1[h], csh[h]);
      zq[h] = cok[h] && x0 == 0;
      mm0[h] = x0 ? (int32_t)(__builtin_ctz(x0) >> 3) : 4;
      dd[h] = cok[h] ? (uint32_t)(p[h] - (int32_t)cand[h]) : 0u;
    }
    const uint64_t zm0 = __ballot(zq[0]), zm1 = __ballot(zq[1]);
    B2H_LDS uint32_t* scr = sh->rec[slot];   // scratch until the records are written
    if ((zm0 | zm1) == 0) {   // no position's first four bytes match (incompressible tiles): no match
#pragma unroll
      for (int h = 0; h < 2; h++) scr[h * kHalf + lane] = rec_pack(0, v[h], dd[h]);
      return;
    }
    const uint32_t d63 = (uint32_t)__builtin_amdgcn_readlane((int)dd[0], 63);
    uint64_t sm[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      // the previous position's distance and first-word verdict (tile position 0: none)
      const uint32_t dprev = (uint32_t)__builtin_amdgcn_update_dpp((int)(h ? d63 : 0xffffffffu), (int)dd[h], 0x138, 0xf, 0xf, false);
      const uint64_t zmh = h ? zm1 : zm0;
      const bool zprev = lane > 0 ? ((zmh >> (lane - 1)) & 1ull) != 0 : (h == 1 && (zm0 >> 63) != 0);
      sm[h] = __ballot(cok[h] && zprev && dprev == dd[h]);
    }
    // run ends (the successor does not continue the run; tile position 127 always ends one) and
    // the compare points among them (first four bytes equal)
    const uint64_t em0 = ~((sm[0] >> 1) | (sm[1] << 63)), em1 = ~(sm[1] >> 1);
    const uint64_t cp0 = em0 & zm0, cp1 = em1 & zm1;
    const int32_t n0 = __builtin_popcountll(cp0), ncp = n0 + __builtin_popcountll(cp1);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint64_t cpm = h ? cp1 : cp0;
      if ((cpm >> lane) & 1ull) {
        const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(cpm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)cpm, 0u));
        scr[(h ? n0 : 0) + (int32_t)below] = (uint32_t)(h * kHalf + lane) | (dd[h] << 8);
      }
    }
    uint32_t ent[2] = {0u, 0u};
    if (ncp > 0) {
      ent[0] = lane < ncp ? scr[lane] : 0u;
      if (ncp > kHalf) ent[1] = lane + kHalf < ncp ? scr[lane + kHalf] : 0u;
    }
    int32_t mmc[2] = {0, 0};
#pragma unroll
    for (int g = 0; g < 2; g++) {
      if (g == 1 && ncp <= kHalf) break;
      if (g == 0 && ncp == 0) break;
      const bool act = lane + g * kHalf < ncp;
      const int32_t pq = P + (int32_t)(ent[g] & 0xffu);
      const int32_t cqp = pq - (int32_t)(ent[g] >> 8);
      gin_t aq = in + (act ? pq : 0), cq = in + (act ? cqp : 0);
      const B2H_GLB uint32_t* awp = align4(aq);
      const B2H_GLB uint32_t* cwp = align4(cq);
      RawCmp a;
      uint32_t c[kCmpWords + 1];
      a.sh = (uint32_t)(reinterpret_cast<uintptr_t>(aq) & 3);
      const uint32_t sc = (uint32_t)(reinterpret_cast<uintptr_t>(cq) & 3);
#pragma unroll
      for (int i = 0; i < kCmpWords + 1; i++) {
        a.d[i] = awp[i];
        c[i] = cwp[i];
      }
      int32_t mm = kCmpBytes;
#pragma unroll
      for (int i = kCmpWords - 1; i >= 1; i--) {   // word 0 is equal at every compare point
        const uint32_t x = rawc_word(a, i) ^ funnel(c[i], c[i + 1], sc);
        if (x) mm = 4 * i + (__builtin_ctz(x) >> 3);
      }
      mmc[g] = mm;
    }
    // every position reads its run's end (the first run end at or after it): through LDS, unless
    // every position ends its own run and none needed the compare (incompressible tiles: each
    // position's verdict is its own first word)
    int32_t k[2], mk[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint64_t rem = (h ? em1 : em0) >> lane;
      k[h] = rem ? h * kHalf + lane + (int32_t)__builtin_ctzll(rem) : kHalf + (int32_t)__builtin_ctzll(em1);
      mk[h] = mm0[h];
    }
    if (ncp > 0 || (em0 & em1) != ~0ull) {
      // each run end's verdict at its position: compared, or its first word
      if (ncp > 0) {
        if (lane < ncp) scr[ent[0] & 0xffu] = (uint32_t)mmc[0];
        if (ncp > kHalf && lane + kHalf < ncp) scr[ent[1] & 0xffu] = (uint32_t)mmc[1];
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const uint64_t em = h ? em1 : em0, cpm = h ? cp1 : cp0;
        if (((em & ~cpm) >> lane) & 1ull) scr[h * kHalf + lane] = (uint32_t)mm0[h];
      }
#pragma unroll
      for (int h = 0; h < 2; h++) mk[h] = (int32_t)scr[k[h]];
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int32_t q = h * kHalf + lane;
      const bool ex = mk[h] < kCmpBytes;                 // E = P + k + mk exactly
      const int32_t mm = ex ? k[h] + mk[h] - q : kCmpBytes;   // (>= kCmpBytes: exact, or "at least")
      const uint32_t d = dd[h];
      const int32_t e = min(ex ? p[h] + mm + 1 : 0x7fffffff, bound);
      const int32_t len = e - 4 - p[h];
      const bool acc = zq[h] && len >= 4 && (PROBE || !(len <= 5 && d - 1 >= kLzNear));
      const bool known = (ex || p[h] + kCmpBytes + 1 >= bound) && len < kRecLong;
      scr[q] = rec_pack(acc ? (known ? len : kRecLong) : 0, v[h], d);
    }
  };

  const int32_t pos = PROBE ? 0 : 4;
  int32_t T = pos / kFastTile, pend = -1;
  int cur = 0, it = 0;
  const bool any = pos < loop_end;
  // B2H_PROBE_AHEAD: the probe's matcher -- its critical wave -- inserting one tile further ahead,
  // so AHEAD(t + 1)'s candidate loads land across the barrier (tools/fm_model.c
  // fm_set_ahead_probe(2)); same-box A/B T 209.6 -> 207.6 GiB/s, off
  constexpr bool LA = PROBE && kProbeAhead;
  int32_t pt = -1, hi = -1;
  __syncthreads();                           // table cleared
  if (any) {                                 // entering T: T and T + 1
    ahead(T);
    finish(0);
    hi = T;
    if (LA && (T + 1) * kFastTile < loop_end) { ahead(T + 1); pt = T + 1; hi = T + 1; }
  }
  __syncthreads();
  while (any) {
    EPROF_T(tm0);
    // the tile whose records are due at this step's barrier: the next one, or the jump target
    const int32_t X = pend >= 0 ? pend : T + 1;
    if (X * kFastTile < loop_end) {
      if (!LA || pt != X) { ahead(X); hi = X; }
      finish(cur ^ 1);
      pt = -1;
      if (LA && (X + 1) * kFastTile < loop_end && X + 1 > hi) { ahead(X + 1); pt = X + 1; hi = X + 1; }
    }
    EPROF_T(tm1);
    __syncthreads();
    EPROF_T(tm2);
    EPROF_ADD(0, tm0, tm1);
    EPROF_ADD(4, tm1, tm2);
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
  EPROF_FLUSH;
}

// value of per-half variable x[2] at tile position q (0..127), as a wave-uniform value
__device__ __forceinline__ int32_t rdq(const int32_t (&x)[2], int32_t q) {
  return q < kHalf ? rdlane(x[0], q) : rdlane(x[1], q - kHalf);
}

// Exact length of the match taken at tile position m whose 60-byte compare did not find its end
// (lenx == -1): the positions at +56, +112 at the same distance carry the next 60 bytes' compares
// (lenx -1: they match on; a known length: the match ends where theirs does), then 64 lanes x 16
// bytes per step from memory.
__device__ __forceinline__ int32_t fast_match_len(int32_t m, const int32_t (&lenx)[2], const int32_t (&dist)[2],
                                                  int32_t P, int32_t bound, gin_t in) {
  const int32_t known = rdq(lenx, m);
  if (known >= 0) return known;
  const int32_t pm = P + m;
  const int32_t dm = rdq(dist, m);
  int32_t L = kCmpBytes, e = -1;
  for (int32_t j = m + kNbrStride; j < kFastTile; j += kNbrStride) {
    if (pm + L >= bound) { e = bound; break; }
    const int32_t lj = rdq(lenx, j);
    if (lj == 0 || rdq(dist, j) != dm) break;
    if (lj > 0) { e = P + j + 4 + lj; break; }
    L = j - m + kCmpBytes;
  }
  if (e < 0) e = pm + L >= bound ? bound : wave_match_end(in, pm + L, (uint32_t)dm, bound);
  return e - 4 - pm;
}

// One counting step of the probe (get_cratio, blosc/blosclz.c:320-419) over a tile with accepted
// matches: the chain walk, then every element's output size through two 128-position DPP scans.
// Returns the next parse position relative to the tile.
__device__ __forceinline__ int32_t probe_step(const uint64_t (&am)[2], int32_t (&lenx)[2], const int32_t (&dist)[2],
                                              int32_t P, int32_t s0, int32_t lim,
                                              int32_t bound, gin_t in, int32_t& lit, int32_t& o) {
  const int lane = lane_id();
  uint64_t chain[2] = {0, 0};
  int32_t ser = -1, endc2 = -1;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    if (ser >= 0 || endc2 >= (h + 1) * kHalf) continue;
    uint64_t rem = endc2 > h * kHalf ? am[h] & (~0ull << (endc2 - h * kHalf)) : am[h];
    while (rem) {
      const int32_t m = h * kHalf + __builtin_ctzll(rem);
      int32_t lm = rdlane(lenx[h], m - h * kHalf);
      if (lm < 0) {
        lm = fast_match_len(m, lenx, dist, P, bound, in);
        lenx[h] = lane == m - h * kHalf ? lm : lenx[h];
      }
      if (lm >= 262) { ser = m; break; }
      chain[h] |= 1ull << (m - h * kHalf);
      const int32_t c2 = m + lm + 2;
      endc2 = c2;
      if (c2 >= (h + 1) * kHalf) break;
      rem = am[h] & (~0ull << (c2 - h * kHalf));
    }
  }
  bool ischain[2], islit[2];
  int32_t c2incl[2], lpos[2], contrib[2], incl[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    ischain[h] = (chain[h] >> lane) & 1ull;
    c2incl[h] = wave_scan_max(ischain[h] ? h * kHalf + lane + lenx[h] + 2 : -1);
  }
  const int32_t carry_c2 = rdlane(c2incl[0], 63);
  c2incl[1] = max(c2incl[1], carry_c2);
  const int32_t lit_end = ser >= 0 ? ser : lim;
#pragma unroll
  for (int h = 0; h < 2; h++) {
    const int32_t q = h * kHalf + lane;
    int32_t pc2 = __builtin_amdgcn_update_dpp(-1, c2incl[h], 0x138, 0xf, 0xf, false);   // wave_shr:1
    if (h == 1 && lane == 0) pc2 = carry_c2;
    const bool hasprev = pc2 >= 0;
    const int32_t segstart = hasprev ? pc2 : s0;
    lpos[h] = (hasprev ? 0 : lit) + q - segstart;
    islit[h] = !ischain[h] && q >= segstart && q < lit_end;
    const int32_t rr5 = lpos[h] & 31;
    const bool near = (uint32_t)dist[h] - 1 < kLzNear;
    const int32_t tok = (uint32_t)lenx[h] < 7 ? (near ? 2 : 4) : (near ? 3 : 5);
    contrib[h] = 0;
    if (islit[h]) contrib[h] = 1 + (rr5 == 31 ? 1 : 0);
    if (ischain[h]) contrib[h] = tok + 1 - (rr5 == 0 ? 1 : 0);
    incl[h] = wave_scan_add(contrib[h]);
  }
  const uint64_t litm0 = __ballot(islit[0]), litm1 = __ballot(islit[1]);
  const uint64_t elems0 = litm0 | chain[0], elems1 = litm1 | chain[1];
  if (elems0 | elems1) {
    const int32_t le = elems1 ? kHalf + 63 - __builtin_clzll(elems1) : 63 - __builtin_clzll(elems0);
    const bool lelit = le < kHalf ? ((litm0 >> le) & 1ull) : ((litm1 >> (le - kHalf)) & 1ull);
    lit = lelit ? ((rdq(lpos, le) + 1) & 31) : 0;
  }
  o += rdlane(incl[0], 63) + rdlane(incl[1], 63);
  int32_t next_rel = max(endc2, lim);
  if (ser >= 0) {   // a match with length-extension bytes
    const uint32_t sbd = (uint32_t)rdq(dist, ser) - 1;
    const int32_t lm = rdq(lenx, ser);
    if (!lit) o--;
    lit = 0;
    o += 1 + (int32_t)(((uint32_t)lm - 7) / 255) + (sbd < kLzNear ? 2 : 4) + 1;
    next_rel = ser + lm + 2;
  }
  return next_rel;
}

// PARSER: chain walk, token emission, output ring and flushes, the tail.  Position q of the tile
// (0..127) is lane q & 63 of half q >> 6; every per-position value is a pair [half].
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
  if (!PROBE && lane < 5) {   // marker + four literals; the load index never negative (in[-1] lies outside the image)
    const uint8_t b = in[lane > 0 ? lane - 1 : 0];
    oring[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : b;
  }
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
        const int32_t s0 = pos - P;
        const int32_t lim = min(kFastTile, loop_end - P);
        int32_t dist[2], lenx[2];
        uint32_t vbyte[2], wrec[2];
        uint64_t am[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
          const int32_t q = h * kHalf + lane;
          const uint32_t w = sh->rec[cur][q];
          wrec[h] = w;
          const int32_t L = rec_len(w);
          vbyte[h] = rec_byte(w);
          dist[h] = (int32_t)rec_dist(w);
          lenx[h] = L == kRecLong ? -1 : L;
          am[h] = __ballot(q >= s0 && L != 0);
        }
        EPROF_T(t2);
        EPROF_ADD(1, t0, t2);
        if constexpr (PROBE) {
          if ((am[0] | am[1]) == 0) {
            const int32_t cnt = lim - s0;
            o += cnt + (lit + cnt) / 32;
            lit = (lit + cnt) & 31;
            pos = P + lim;
          } else {
            pos = P + probe_step(am, lenx, dist, P, s0, lim, bound, in, lit, o);
          }
        } else {
          // ---- emitting pass: the chain walk emits each element as it takes it (literal runs by
          // the lanes that hold them, a token by lanes 0..5), so a step costs instructions per
          // ELEMENT, not per position: on T's smooth plane a 128-position step holds ~10 ----
          int32_t c = s0, ser = -1, ser_len = 0, endc2 = -1, req = -1;
          auto emit_lits = [&](int32_t a, int32_t e) {   // literals at tile positions [a, e), a < e
            const int32_t n = e - a;
#pragma unroll
            for (int h = 0; h < 2; h++) {
              if (a < (h + 1) * kHalf && e > h * kHalf) {
                const int32_t q = h * kHalf + lane, k = q - a;
                if (q >= a && q < e) {
                  const int32_t off = o + k + ((lit + k) >> 5);
                  oring[off & ORM] = (uint8_t)vbyte[h];
                  if (((lit + k + 1) & 31) == 0) oring[(off + 1) & ORM] = (uint8_t)(kLzMaxCopy - 1);
                }
              }
            }
            req = o + (n - 1) + ((lit + n - 1) >> 5) + 2;
            o += n + ((lit + n) >> 5);
            lit = (lit + n) & 31;
          };
          // MATCH_SHORT / MATCH_LONG (+ _FAR) token + the marker opening the next literal run
          // (blosc/blosclz.c:270-316); the run it ends gets its header (lane 8).
          // A token's place in the output is known in the walk (a scalar chain); its bytes are
          // written afterwards by one lane per token, all tokens of the step at once (the walk
          // records start, length, distance and the header it closes into lane k of e_*).
          int32_t nel = 0, e_ts = 0, e_len = 0, e_dist = 0, e_at = -1, e_hdr = 0;
          auto emit_token = [&](int32_t lm, uint32_t dm) {
            int32_t at = -1;
            const uint32_t hdr = (uint32_t)(lit - 1);
            if (lit) {
              at = o - lit - 1;
              if (at == 0) byte0 = hdr;
            } else {
              o--;
            }
            lit = 0;
            const uint32_t bd = dm - 1;
            const int32_t tok = (uint32_t)lm >= 7 ? (bd < kLzNear ? 3 : 5) : (bd < kLzNear ? 2 : 4);
            const bool me = lane == nel;
            e_ts = me ? o : e_ts;
            e_len = me ? lm : e_len;
            e_dist = me ? (int32_t)dm : e_dist;
            e_at = me ? at : e_at;
            e_hdr = me ? (int32_t)hdr : e_hdr;
            nel++;
            o += tok + 1;
            req = o;
          };
#pragma unroll
          for (int h = 0; h < 2; h++) {
            if (ser >= 0 || c >= (h + 1) * kHalf) continue;
            uint64_t rem = c > h * kHalf ? am[h] & (~0ull << (c - h * kHalf)) : am[h];
            while (rem) {
              const int32_t m = h * kHalf + __builtin_ctzll(rem);
              // the element's whole record in one readlane: length and distance unpacked on the
              // scalar side
              const uint32_t wm = (uint32_t)rdlane((int32_t)wrec[h], m - h * kHalf);
              int32_t lm = rec_len(wm);
              if (lm == kRecLong) {
                EPROF_T(te0);
                lm = fast_match_len(m, lenx, dist, P, bound, in);
                EPROF_T(te1);
                EPROF_ADD(5, te0, te1);
              }
              if (lm >= 262) { ser = m; ser_len = lm; break; }
              if (m > c) emit_lits(c, m);
              emit_token(lm, rec_dist(wm));
              c = m + lm + 2;
              endc2 = c;
              if (c >= (h + 1) * kHalf) break;
              rem = am[h] & (~0ull << (c - h * kHalf));
            }
          }
          const int32_t lit_end = ser >= 0 ? ser : lim;
          if (c < lit_end) emit_lits(c, lit_end);
          if (nel) {
            // the step's tokens (MATCH_SHORT / MATCH_LONG + _FAR, blosc/blosclz.c:270-316) + the
            // marker opening the next literal run, in DESCENDING byte order: a token right after
            // a marker (no literal between) overwrites it at its byte 0, written last; then the
            // headers of the literal runs the tokens close
            const bool el = lane < nel;
            const uint32_t bd = (uint32_t)e_dist - 1, ulen = (uint32_t)e_len, fd = bd - kLzNear;
            const bool near = bd < kLzNear, lng = ulen >= 7;
            const uint32_t b0 = (lng ? (7u << 5) : (ulen << 5)) + (near ? (bd >> 8) : 31u);
            const uint32_t dbytes = near ? (bd & 255u) : (255u | ((fd >> 8) << 8) | ((fd & 255u) << 16));
            uint64_t rest = (uint64_t)dbytes | (31ull << (near ? 8 : 24));
            if (lng) rest = (uint64_t)(ulen - 7) | (rest << 8);
            const uint64_t bytes = (uint64_t)b0 | (rest << 8);
            const int32_t tok = lng ? (near ? 3 : 5) : (near ? 2 : 4);
#pragma unroll
            for (int i = 5; i >= 0; i--)
              if (el && i <= tok) oring[(e_ts + i) & ORM] = (uint8_t)(bytes >> (8 * i));
            if (el && e_at >= 0) oring[e_at & ORM] = (uint8_t)e_hdr;
          }
          if (req >= 0) {
            peak = max(peak, req);
            if (req > maxout) { fail = true; break; }
          }
          EPROF_T(t3);
          EPROF_ADD(2, t2, t3);
          int32_t next_rel = max(endc2, lim);
          if (ser >= 0) {   // a match with length-extension bytes: the scalar token path
            const uint32_t dm = (uint32_t)rdq(dist, ser);
            const int32_t lm = ser_len;
            const uint32_t sbd = dm - 1;
            const uint32_t sulen = (uint32_t)lm;
            const bool snear = sbd < kLzNear;
            int32_t at = -1;
            const uint32_t hdr = (uint32_t)(lit - 1);
            if (lit) {
              at = o - lit - 1;
              if (at == 0) byte0 = hdr;
            } else {
              o--;
            }
            lit = 0;
            const int32_t ext = (int32_t)((sulen - 7) / 255);
            const int32_t stok = 1 + ext + (snear ? 2 : 4);
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
template <bool PROBE, typename POS, bool WT, bool DEEP>
__device__ __forceinline__ LzPassOut lz_pass_fast(gin_t in, int32_t length, int probe_hashlog, int tablog, gout_t out,
                                                   int32_t maxout, B2H_LDS uint8_t* tab, B2H_LDS uint8_t* oring,
                                                   B2H_LDS FastShared* sh, int clevel, bool matcher,
                                                   B2H_GLB POS* chain) {
  if (matcher) {
    lz_pass_fast_matcher<PROBE, POS, DEEP>(in, length, probe_hashlog, tablog, tab, sh, chain);
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
// DEEP: the chained candidates of BloscLZ mode 2; `chain` = this workgroup's prev[] array (one
// POS per position of the longest stream; unused otherwise).
template <typename POS, bool WT = false, bool DEEP = false>
__device__ __forceinline__ StreamResult encode_stream_fast(gin_t __restrict__ in, int32_t n, int clevel, gout_t __restrict__ out,
                                                            B2H_LDS uint8_t* tab, int tablog, B2H_LDS uint8_t* oring,
                                                            B2H_LDS FastShared* sh, bool allow_runs, bool matcher,
                                                            B2H_GLB POS* chain = nullptr) {
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
    // readfirstlane: branches around the passes' barriers must be seen as uniform (a divergent-looking
    // branch gets structurized into exec-masked paths that run s_barrier a different number of
    // times per wave)
    const bool run = (__builtin_amdgcn_readfirstlane(sh->decide[0]) & __builtin_amdgcn_readfirstlane(sh->decide[1])) != 0;
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
#if B2H_PASS_PRIO
  // the probe's critical wave is the matcher (few elements per tile to walk), the emitting
  // pass's the parser: the wave on the chain issues first on its SIMD
  if (matcher) __builtin_amdgcn_s_setprio(2); else __builtin_amdgcn_s_setprio(0);
#endif
  const LzPassOut pr = lz_pass_fast<true, POS, WT, DEEP>(in + (n - maxlen), maxlen, hashlog, tl, out, 0, tab, oring, sh,
                                                      clevel, matcher, chain);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (!matcher && lane_id() == 0) sh->decide[0] = (pr.early || (!pr.sure && ratio < thr) || n < 66) ? 0 : 1;
  __syncthreads();
  const bool go = __builtin_amdgcn_readfirstlane(sh->decide[0]) != 0;
  __syncthreads();
  if (!go) return res;
#if B2H_PASS_PRIO
  if (matcher) __builtin_amdgcn_s_setprio(0); else __builtin_amdgcn_s_setprio(2);
#endif
  const LzPassOut em = lz_pass_fast<false, POS, WT, DEEP>(in, n, hashlog, tl, out, n, tab, oring, sh, clevel, matcher, chain);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

}  // namespace b2h
