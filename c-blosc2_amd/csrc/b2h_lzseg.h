// b2h_lzseg.h -- BloscLZ mode 3, "segmented": the fast-mode parse with intra-stream parallelism
// (device code).
//
// Semantics (CPU model: tools/fm_model.c fm_parse with fm_set_noskip(1)): the reference's grammar,
// greedy rule, limits, probe thresholds and emission (blosc/blosclz.c:248-316, 320-419, 422-619),
// with one change -- the candidate a position's bucket offers is the most recent EARLIER POSITION
// with that hash, every position inserted in order (u16 buckets, the same rule as mode 1).  So a
// candidate is a function of the input alone, and the parse is the serial greedy walk over fixed
// candidates.  Ratio on T 1.0004 x exact's stream bytes (mode 1: 1.0004), C3 1.0019, C1 as mode 1
// (tools/fm3_ratio.py).
//
// Where mode 1 walks one stream with one wave (a matcher / parser pair, ~3 M cycles per 64 KiB
// stream on T's smooth plane, one element per scalar step), this mode splits a pass into:
//   1. candidates: one wave exchanges the stream's positions with the LDS table in order, 64 per
//      ds_mskor_rtn, eight half-tiles per round trip; every position whose candidate's first four
//      bytes equal its own gets its distance stored (global scratch) and a bit in a mask;
//   2. a segment-parallel greedy walk: the 64 lanes walk 64 segments of the pass at once, each from
//      an entry state (position, literal-run length).  The serial walk's state where it enters
//      segment k is only known once segments < k are walked, so the walk iterates: lane k's entry
//      = the furthest exit of lanes < k (a prefix max over packed (position, run) words) until no
//      entry moves -- the serial parse, reached in 2 rounds on T (the greedy walk resynchronises a
//      few elements after a wrong entry).  A lane steps from one masked position to the next
//      (positions without a 4-byte match are literals, skipped in bulk), loads the distance and
//      compares 28 + 32-byte windows of its own; matches running past 284 bytes are extended by
//      the whole wave (wave_match_end).  The counting walk gives every lane's output size and the
//      largest output requirement it meets (the reference's `maxout` checks, blosclz.c:548-610);
//   3. output offsets by a prefix sum, then one more walk writes every lane's bytes in place.  A
//      literal run's header is written by the lane whose walk closes the run (32 literals, a
//      match, the stream's end), so no byte has two writers.
// The probe (get_cratio) is the same counting walk over its window, ratio = position / count.
#pragma once
#include "b2h_lz.h"
#include "b2h_lzfast.h"

namespace b2h {

#ifdef B2H_SEG_PROF   // diagnostics build: per-phase s_memtime sums (b2h_debug_seg_prof)
__device__ unsigned long long g_seg_prof[32];
#define SPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define SPROF_ADD(i, a, b) \
  if (lane_id() == 0) atomicAdd(&g_seg_prof[(i)], (unsigned long long)((b) - (a)))
#define SPROF_CNT(i, n) \
  if (lane_id() == 0) atomicAdd(&g_seg_prof[(i)], (unsigned long long)(n))
#define SPROF_ACC(v, a, b) v += (b) - (a)
#define SPROF_DECL(v) uint64_t v = 0
#else
#define SPROF_ACC(v, a, b)
#define SPROF_DECL(v)
#define SPROF_T(v)
#define SPROF_ADD(i, a, b)
#define SPROF_CNT(i, n)
#endif

constexpr int kSegGroup = 8;          // half-tiles (64 positions) per candidate round trip
constexpr int32_t kSegMinLen = 256;   // smallest walk segment (bytes)
constexpr int32_t kSegLaneExt = 256;  // per-lane extension budget past the first 28 bytes

// ---- 1. candidates -------------------------------------------------------------------------
// Every position p < loop_end gets its record dist[p] (0: no usable candidate, else the distance to
// a candidate whose first four bytes equal p's) and its bit in mask.  Two groups of kSegGroup
// half-tiles are in flight: group g + 1 is exchanged and its candidates' words requested before
// group g's words are compared.
struct SegCand {
  uint32_t v[kSegGroup], cand[kSegGroup], c0[kSegGroup], c1[kSegGroup], csh[kSegGroup], x0[kSegGroup], x1[kSegGroup];
  bool cok[kSegGroup], alt[kSegGroup];
};
__device__ __forceinline__ void seg_cand_issue(gin_t __restrict__ in, int32_t loop_end, int tablog, B2H_LDS uint8_t* tab,
                                               bool far, int32_t t0, const uint32_t (&a0)[kSegGroup],
                                               const uint32_t (&a1)[kSegGroup], SegCand& C) {
  const int lane = lane_id();
  int32_t p[kSegGroup];
  bool valid[kSegGroup];
#pragma unroll
  for (int g = 0; g < kSegGroup; g++) {
    p[g] = (t0 + g) * 64 + lane;
    valid[g] = p[g] < loop_end;
    C.v[g] = funnel(a0[g], a1[g], (uint32_t)(reinterpret_cast<uintptr_t>(in + (valid[g] ? p[g] : 0)) & 3));
  }
  // the exchanges, in position order (a wave's LDS instructions execute in order)
#pragma unroll
  for (int g = 0; g < kSegGroup; g += 2) {
    const uint32_t vv[2] = {C.v[g], C.v[g + 1]};
    const int32_t pp[2] = {p[g], p[g + 1]};
    const bool va[2] = {valid[g], valid[g + 1]};
    uint32_t cc[2];
    fast_exchange2<uint16_t>(vv, pp, va, tablog, tab, cc);
    C.cand[g] = cc[0];
    C.cand[g + 1] = cc[1];
  }
  // every candidate's first four bytes (and, past 2^16 positions, those 2^16 further back)
#pragma unroll
  for (int g = 0; g < kSegGroup; g++) {
    C.cok[g] = fast_cand_ok(p[g], C.cand[g], valid[g]);
    gin_t cq = in + (C.cok[g] ? (int32_t)C.cand[g] : (valid[g] ? p[g] : 0));
    const B2H_GLB uint32_t* cw = align4(cq);
    C.csh[g] = (uint32_t)(reinterpret_cast<uintptr_t>(cq) & 3);
    C.c0[g] = cw[0];
    C.c1[g] = cw[1];
    C.alt[g] = far && C.cok[g] && C.cand[g] >= 65536u && (uint32_t)p[g] - C.cand[g] < kLzFar - 65536u;
    C.x0[g] = C.x1[g] = 0;
    if (C.alt[g]) {
      C.x0[g] = cw[-16384];
      C.x1[g] = cw[-16383];
    }
  }
}
__device__ __forceinline__ void seg_cand_finish(int32_t loop_end, int32_t nh, int32_t t0, const SegCand& C,
                                                B2H_GLB uint32_t* __restrict__ dist, B2H_GLB uint64_t* __restrict__ mask) {
  const int lane = lane_id();
  uint64_t bal[kSegGroup];
#pragma unroll
  for (int g = 0; g < kSegGroup; g++) {
    const int32_t p = (t0 + g) * 64 + lane;
    uint32_t c = C.cand[g];
    bool ok = C.cok[g] && funnel(C.c0[g], C.c1[g], C.csh[g]) == C.v[g];
    if (C.alt[g] && !ok) {   // the near candidate's first 4 bytes differ: the one 2^16 further back
      c -= 65536u;
      ok = funnel(C.x0[g], C.x1[g], C.csh[g]) == C.v[g];
    }
    bal[g] = __ballot(ok);
    if (ok) dist[p] = (uint32_t)p - c;
  }
#pragma unroll
  for (int g = 0; g < kSegGroup; g++)
    if (lane == g && t0 + g < nh) mask[t0 + g] = bal[g];
}

// Streams of at most 2^16 positions: the table holds u32 entries, position (16 bits) | a 16-bit check
// of the 4-byte value that position hashed (bits 3..18 of the product whose top bits are the
// bucket), so a candidate's first four bytes are compared without reading them: equal values give
// equal checks, and a check that matches unequal values (~2^-16) only marks a position whose walk
// step then finds the bytes differ -- a literal, as the model has it.  Empty buckets start as
// position 0 with position 0's check (the model's candidate of an empty bucket is position 0).
__device__ __forceinline__ uint32_t seg_chk(uint32_t v) { return ((v * 2654435761u) >> 3) & 0xffffu; }

__device__ __forceinline__ void seg_candidates_chk(gin_t __restrict__ in, int32_t loop_end, int tablog, B2H_LDS uint8_t* tab,
                                                   B2H_GLB uint32_t* __restrict__ dist, B2H_GLB uint64_t* __restrict__ mask) {
  const int lane = lane_id();
  const int32_t nh = loop_end > 0 ? (loop_end + 63) >> 6 : 0;
  {
    const uint32_t e0 = seg_chk(ldu32(in)) << 16;
    B2H_LDS u32x4* t16 = (B2H_LDS u32x4*)tab;
    const int32_t n16 = (int32_t)((4u << tablog) / 16);
    for (int32_t i = lane; i < n16; i += 64) t16[i] = u32x4{e0, e0, e0, e0};
  }
  if (nh == 0) return;
  constexpr int G = kSegGroup;
  const uint32_t base = (uint32_t)reinterpret_cast<uintptr_t>(tab);
  // the records as a buffer of loop_end entries: an offset past it is dropped by the hardware
  const __amdgpu_buffer_rsrc_t drs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)dist, (short)0, (int)(4u * (uint32_t)__builtin_amdgcn_readfirstlane(loop_end)), 0x00020000);
  uint32_t a0[G], a1[G];
  auto load_own = [&](int32_t t0) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      const int32_t p = (t0 + g) * 64 + lane;
      const B2H_GLB uint32_t* q = align4(in + (p < loop_end ? p : 0));
      a0[g] = q[0];
      a1[g] = q[1];
    }
  };
  load_own(0);
  for (int32_t t0 = 0; t0 < nh; t0 += G) {
    uint32_t addr[G], ent[G], old[G];
    int32_t p[G];
    bool valid[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
      p[g] = (t0 + g) * 64 + lane;
      valid[g] = p[g] < loop_end;
      const uint32_t v = funnel(a0[g], a1[g], (uint32_t)(reinterpret_cast<uintptr_t>(in + (valid[g] ? p[g] : 0)) & 3));
      const uint32_t prod = v * 2654435761u;
      addr[g] = base + ((prod >> (32 - tablog)) << 2);
      ent[g] = ((uint32_t)p[g] & 0xffffu) | (((prod >> 3) & 0xffffu) << 16);
    }
    if (t0 + G < nh) load_own(t0 + G);
    // the exchanges in position order (in-order LDS), one wait for all.  Lanes past loop_end come
    // after every valid position (higher lanes of the last half-tile, later half-tiles): what they
    // write is never read in this pass, and the next pass clears the table.
#pragma unroll
    for (int g = 0; g < G; g += 4) {
      uint32_t w0, w1, w2, w3;
      asm volatile(
          "ds_wrxchg_rtn_b32 %0, %4, %5\n\t"
          "ds_wrxchg_rtn_b32 %1, %6, %7\n\t"
          "ds_wrxchg_rtn_b32 %2, %8, %9\n\t"
          "ds_wrxchg_rtn_b32 %3, %10, %11\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(w0), "=&v"(w1), "=&v"(w2), "=&v"(w3)
          : "v"(addr[g]), "v"(ent[g]), "v"(addr[g + 1]), "v"(ent[g + 1]), "v"(addr[g + 2]), "v"(ent[g + 2]),
            "v"(addr[g + 3]), "v"(ent[g + 3])
          : "memory");
      old[g] = w0;
      old[g + 1] = w1;
      old[g + 2] = w2;
      old[g + 3] = w3;
    }
    // distance (p < 2^16: always below MAX_FARDISTANCE), record and mask: branch-free buffer
    // stores, a lane without a match storing out of range (dropped)
    uint64_t bal[G];
#pragma unroll
    for (int g = 0; g < G; g++) {
      const uint32_t pp = (uint32_t)p[g];
      const uint32_t d = (pp - old[g]) & 0xffffu;
      const bool ok = valid[g] && d != 0 && ((old[g] ^ ent[g]) >> 16) == 0;
      bal[g] = __ballot(ok);
      __builtin_amdgcn_raw_buffer_store_b32(d, drs, ok ? (int32_t)(pp << 2) : 0x7ffffff0, 0, 0);   // (>= 4 loop_end)
    }
#pragma unroll
    for (int g = 0; g < G; g++)
      if (lane == g && t0 + g < nh) mask[t0 + g] = bal[g];
  }
}

__device__ __forceinline__ void seg_candidates(gin_t __restrict__ in, int32_t loop_end, int tablog, B2H_LDS uint8_t* tab,
                                               B2H_GLB uint32_t* __restrict__ dist, B2H_GLB uint64_t* __restrict__ mask) {
  const int lane = lane_id();
  {
    B2H_LDS u32x4* t16 = (B2H_LDS u32x4*)tab;
    const int32_t n16 = (int32_t)((2u << tablog) / 16);
    for (int32_t i = lane; i < n16; i += 64) t16[i] = u32x4{0u, 0u, 0u, 0u};
  }
  const int32_t nh = loop_end > 0 ? (loop_end + 63) >> 6 : 0;
  if (nh == 0) return;
  const bool far = __builtin_amdgcn_readfirstlane(loop_end) > 65536;   // u16 aliases past 2^16 positions
  constexpr int G = kSegGroup;
  uint32_t a0[G], a1[G];   // own words of the next group (aligned dword pair)
  auto load_own = [&](int32_t t0) {
#pragma unroll
    for (int g = 0; g < G; g++) {
      const int32_t p = (t0 + g) * 64 + lane;
      const B2H_GLB uint32_t* q = align4(in + (p < loop_end ? p : 0));
      a0[g] = q[0];
      a1[g] = q[1];
    }
  };
  SegCand A, Bc;
  load_own(0);
  seg_cand_issue(in, loop_end, tablog, tab, far, 0, a0, a1, A);
  if (G < nh) load_own(G);
  for (int32_t t0 = 0; t0 < nh; t0 += 2 * G) {
    // A holds group t0 (issued); B: group t0 + G
    const bool more1 = t0 + G < nh;
    if (more1) {
      seg_cand_issue(in, loop_end, tablog, tab, far, t0 + G, a0, a1, Bc);
      if (t0 + 2 * G < nh) load_own(t0 + 2 * G);
    }
    seg_cand_finish(loop_end, nh, t0, A, dist, mask);
    if (!more1) break;
    if (t0 + 2 * G < nh) {
      seg_cand_issue(in, loop_end, tablog, tab, far, t0 + 2 * G, a0, a1, A);
      if (t0 + 3 * G < nh) load_own(t0 + 3 * G);
    }
    seg_cand_finish(loop_end, nh, t0 + G, Bc, dist, mask);
  }
}

// The candidate table is busy only during step 1 (a quarter of a smooth stream's time), so the
// waves of a workgroup share one: a wave takes the workgroup's lock word (global memory: the LDS is
// exactly five 32 KiB tables per CU) for step 1 and releases it after its last exchange completed.
__device__ __forceinline__ void seg_lock(int32_t* lock) {
  if (lane_id() == 0) {
    while (atomicCAS(lock, 0, 1) != 0) __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  __builtin_amdgcn_s_setprio(3);   // the workgroup's other waves wait for the table: issue first
}

__device__ __forceinline__ void seg_unlock(int32_t* lock) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the table's exchanges are complete
  if (lane_id() == 0) atomicExch(lock, 0);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_s_setprio(0);
}

// ---- 2./3. the segment walk ----------------------------------------------------------------
// One lane's match end at q against q - d: one past the first mismatch at or after q + 4, `bound`
// if none before it (blosclz.c:119-165 get_match), or q + 4 (length 0: a literal) when the first
// four bytes differ after all (a check collision of the candidate table).  `lng`: no mismatch in
// the lane's budget; the caller extends from *xnext.
__device__ __forceinline__ int32_t seg_lane_match_end(gin_t __restrict__ in, int32_t q, uint32_t d, int32_t bound,
                                                      bool* lng, int32_t* xnext) {
  {
    uint32_t a[8], b[8];
    ldw<8>(in + q, a);
    ldw<8>(in + q - d, b);
    if (a[0] != b[0]) return q + 4;
    int32_t f = 32;
#pragma unroll
    for (int i = 7; i >= 1; i--) {
      const uint32_t df = a[i] ^ b[i];
      if (df) f = 4 * i + (int32_t)(__builtin_ctz(df) >> 3);
    }
    if (f < 32) return q + f < bound ? q + f + 1 : bound;
  }
  int32_t x = q + 32;
  if (x >= bound) return bound;
  for (int32_t k = 0; k < kSegLaneExt; k += 32) {
    uint32_t a[8], b[8];
    ldw<8>(in + x, a);
    ldw<8>(in + x - d, b);
    int32_t f = 32;
#pragma unroll
    for (int i = 7; i >= 0; i--) {
      const uint32_t df = a[i] ^ b[i];
      if (df) f = 4 * i + (int32_t)(__builtin_ctz(df) >> 3);
    }
    if (f < 32) return x + f < bound ? x + f + 1 : bound;
    x += 32;
    if (x >= bound) return bound;
  }
  *lng = true;
  *xnext = x;
  return -1;
}

// The candidate record of a masked position: distance (17 bits) | (match length + 1) << 17 once a
// walk of this pass has measured it (0: not yet; lengths >= kSegLenCap are not kept).
constexpr uint32_t kSegDistMask = (1u << 17) - 1;
constexpr int32_t kSegLenCap = (1 << 15) - 2;

// Walk state of one lane (one segment).  Counting walks assume the literal run they enter is empty
// and count `lead` (the literals before the lane's first match) and `matched`; seg_pass corrects o
// for the real entry run (seg_corr).  The emitting walk knows its entry run and global offset.
// No running maximum of the reference's `maxout` checks is kept: o never drops between elements (a
// dropped marker is followed by a >= 2-byte token) and the tail always ends the stream with a
// literal, so the largest check is the last one, o_final + 1.
struct SegLane {
  int32_t pos, lit, o, lead;
  bool matched;
  int32_t steps;
};

// Output bytes of a walk entered with a run of L literals, minus those of the same walk entered with
// an empty run: the leading literals' run headers and the first match's header / dropped marker
// (blosclz.c:566-572, 598-610).
__device__ __forceinline__ int32_t seg_corr(int32_t L, int32_t lead, bool matched) {
  int32_t c = ((L + lead) >> 5) - (lead >> 5);
  if (matched) c += ((lead & 31) == 0 ? 1 : 0) - (((L + lead) & 31) == 0 ? 1 : 0);
  return c;
}

// The first walk of a lane records its first kSegSnap match starts (offsets from the segment start,
// two per word) and its state before each ((o << 5) | lit, in scratch).  When the lane's entry
// moves, the correcting walk from the new entry stops at the first of them it meets and takes the
// rest from the first walk: the greedy parse re-joins its path within a few elements (on T's smooth
// plane the new entry is one of the first 8 match starts for 80 % of the lanes, and the correcting
// walk meets one within 1.6 elements on average for the others: tools/fm3_merge notes in DESIGN §3).
constexpr int kSegSnap = 8;

enum SegMode { kSegFirst = 0, kSegFix = 1, kSegEmit = 2 };

template <bool PROBE, int MODE, bool WT>
__device__ __forceinline__ void seg_walk(gin_t __restrict__ in, int32_t bound, B2H_GLB uint32_t* __restrict__ dist,
                                         const B2H_GLB uint64_t* __restrict__ mask, int32_t wend, bool go, SegLane& L,
                                         gout_t __restrict__ out, int32_t s0, uint32_t (&snp)[kSegSnap / 2],
                                         int32_t& nsnap, B2H_GLB uint32_t* __restrict__ snv, int32_t& merged) {
  constexpr bool EMIT = MODE == kSegEmit;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(out);
  auto put = [&](int32_t at, uint32_t b) {
#ifndef B2H_SEG_NOSTORE   // diagnostics: the emitting walk without its stores (wrong output)
    if constexpr (EMIT) st8<WT>(out, r, at, (uint8_t)(at == 0 ? (b | 0x20u) : b));
#endif
  };
  // n literals at L.pos (the reference's literal path, blosclz.c:598-610)
  auto lits = [&](int32_t n) {
    if (n <= 0) return;
    if (!L.matched) L.lead += n;
    if constexpr (EMIT) {
      int32_t o = L.o, lit = L.lit;
      for (int32_t i = 0; i < n; i++) {
        put(o++, in[L.pos + i]);
        if (++lit == kLzMaxCopy) {   // a full run closes: its header is 31
          put(o - kLzMaxCopy - 1, kLzMaxCopy - 1);
          lit = 0;
          o++;
        }
      }
    }
    L.o += n + ((L.lit + n) >> 5);
    L.lit = (L.lit + n) & 31;
    L.pos += n;
  };
  bool act = go && L.pos < wend;
  [[maybe_unused]] constexpr int WB = EMIT ? 24 : 20;   // profile slots
  SPROF_DECL(pa);
  SPROF_DECL(pb);
  SPROF_DECL(pc);
  SPROF_DECL(pn);
  // The record at the walk position and its mask word come in one round trip, requested at the end
  // of the previous step BEFORE that step's stores (the length cache, the emitted bytes): loads and
  // stores share one in-order counter, and a load issued after a store cannot be waited for alone.
  uint32_t ent = 0;
  uint64_t mw = 0;
  if (act) {
    ent = dist[L.pos];   // (only read where the mask holds the position: records are not cleared)
    mw = mask[L.pos >> 6];
  }
  while (__ballot(act)) {
    SPROF_T(w0);
    // a position without a candidate starts a literal run that the mask skips
    if (act && ((mw >> (L.pos & 63)) & 1) == 0) {
      int32_t q = L.pos;
      uint64_t m = mw >> (q & 63);
      while (m == 0 && (q | 63) + 1 < wend) {
        q = (q | 63) + 1;
        m = mask[q >> 6];
      }
      q = m ? q + (int32_t)__builtin_ctzll(m) : wend;
      lits(min(q, wend) - L.pos);
      act = L.pos < wend;
      if (act) ent = dist[L.pos];
    }
    if constexpr (MODE == kSegFix) {   // back on the first walk's path?
      if (act) {
        const uint32_t off = (uint32_t)(L.pos - s0);
#pragma unroll
        for (int j = 0; j < kSegSnap; j++)
          if (merged < 0 && j < nsnap && ((snp[j >> 1] >> (16 * (j & 1))) & 0xffffu) == off) merged = j;
        if (merged >= 0) act = false;
      }
    }
    const uint32_t d = ent & kSegDistMask;
    int32_t e = -1, xn = 0;
    bool lng = false, fresh = false;
    SPROF_T(w1);
    SPROF_ACC(pa, w0, w1);
    if (act) {
      if (ent >> 17) {
        e = L.pos + 4 + (int32_t)(ent >> 17) - 1;
      } else {
        e = seg_lane_match_end(in, L.pos, d, bound, &lng, &xn);
        fresh = true;
      }
      L.steps++;
    }
    uint64_t lm = __ballot(act && lng);
    SPROF_T(w2);
    SPROF_ACC(pb, w1, w2);
    SPROF_ACC(pn, 0, __builtin_popcountll(lm));
    while (lm) {   // long matches: the whole wave extends them, one at a time
      const int l = __builtin_ctzll(lm);
      const int32_t ee = wave_match_end(in, rdlane(xn, l), (uint32_t)rdlane((int32_t)d, l), bound);
      if (lane_id() == l) e = ee;
      lm &= lm - 1;
    }
    SPROF_T(w3);
    SPROF_ACC(pc, w2, w3);
    // the element: its length decides the next position; the next step's loads go out first
    const int32_t at = L.pos;
    const int32_t len = act ? e - 4 - at : 0;
    const uint32_t bd = d - 1;
    const bool is_lit = act && (len < 4 || (!PROBE && len <= 5 && bd >= kLzNear));
    const bool is_match = act && !is_lit;
    const int32_t npos = is_lit ? at + 1 : (is_match ? at + len + 2 : at);
    const bool nact = act && npos < wend;
    uint32_t ent_n = 0;
    uint64_t mw_n = 0;
    if (nact) {
      ent_n = dist[npos];
      mw_n = mask[npos >> 6];
    }
    if (act && fresh && len < kSegLenCap) dist[at] = d | ((uint32_t)(len + 1) << 17);
    if (is_lit) {
      lits(1);
    } else if (is_match) {
      if constexpr (MODE == kSegFirst) {
        if (nsnap < kSegSnap) {   // a match start: remember where and in which state
          const uint32_t off = (uint32_t)(at - s0), sh = 16u * (uint32_t)(nsnap & 1);
          snp[nsnap >> 1] = (snp[nsnap >> 1] & ~(0xffffu << sh)) | (off << sh);
          snv[nsnap] = ((uint32_t)L.o << 5) | (uint32_t)L.lit;
          nsnap++;
        }
      }
      L.matched = true;
      if (L.lit) put(L.o - L.lit - 1, (uint32_t)(L.lit - 1));
      else L.o--;
      L.lit = 0;
      const uint32_t ulen = (uint32_t)len;
      const bool near = bd < kLzNear;
      const int32_t ext = ulen >= 7 ? (int32_t)((ulen - 7) / 255) : 0;
      const int32_t tok = ulen >= 7 ? 3 + ext + (near ? 0 : 2) : (near ? 2 : 4);
      if constexpr (EMIT) {
        int32_t o = L.o;
        const uint32_t fd = bd - kLzNear;
        put(o++, (ulen >= 7 ? (7u << 5) : (ulen << 5)) + (near ? (bd >> 8) : 31u));
        if (ulen >= 7) {
          for (int32_t i = 0; i < ext; i++) put(o++, 255u);
          put(o++, (ulen - 7) - 255u * (uint32_t)ext);
        }
        if (near) {
          put(o++, bd & 255u);
        } else {
          put(o++, 255u);
          put(o++, fd >> 8);
          put(o++, fd & 255u);
        }
      }
      L.o += tok + 1;   // the token + the header reserved for the next literal run
      L.pos = npos;
    }
    ent = ent_n;
    mw = mw_n;
    act = nact;
  }
  SPROF_ADD(WB + 0, 0, pa);
  SPROF_ADD(WB + 1, 0, pb);
  SPROF_ADD(WB + 2, 0, pc);
  SPROF_ADD(WB + 3, 0, pn);
}

// A workgroup wave's scratch: records (one u32 per position of the longest stream), mask words,
// the walk snapshots' states.
__host__ __device__ inline int64_t seg_dist_bytes(int64_t maxlen) { return ((maxlen + 64) * 4 + 255) & ~int64_t(255); }
__host__ __device__ inline int64_t seg_mask_bytes(int64_t maxlen) { return (((maxlen + 127) / 64) * 8 + 255) & ~int64_t(255); }
__host__ __device__ inline int64_t seg_scratch_bytes(int64_t maxlen) {
  return seg_dist_bytes(maxlen) + seg_mask_bytes(maxlen) + 64 * kSegSnap * 4;
}

// One pass (PROBE: get_cratio's count over min(length, 2^probe_hashlog); else the emitting parse
// with its tail), the serial parse's result: o, final position, peak requirement, fail.
template <bool PROBE, bool WT, bool CHK>
__device__ __forceinline__ LzPassOut seg_pass(gin_t __restrict__ in, int32_t length, int probe_hashlog, int tablog,
                                              gout_t __restrict__ out, int32_t maxout, B2H_LDS uint8_t* tab,
                                              B2H_GLB uint32_t* __restrict__ dist, B2H_GLB uint64_t* __restrict__ mask,
                                              B2H_GLB uint32_t* __restrict__ snv_all, int32_t* lock) {
  const int lane = lane_id();
  int32_t limit, bound, loop_end;
  fast_limits<PROBE>(length, probe_hashlog, &limit, &bound, &loop_end);
  LzPassOut res;
  res.early = res.sure = false;
  [[maybe_unused]] constexpr int PB = PROBE ? 0 : 8;   // profile slots of this pass
  SPROF_T(tp0);
  seg_lock(lock);
  if constexpr (CHK) seg_candidates_chk(in, loop_end, tablog, tab, dist, mask);
  else seg_candidates(in, loop_end, tablog, tab, dist, mask);
  seg_unlock(lock);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the records and masks, before the walks read them
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  SPROF_T(tp1);
  SPROF_ADD(PB + 0, tp0, tp1);
  const int32_t span = loop_end > 0 ? loop_end : 0;
  const int32_t S = max(kSegMinLen, ((span + 63) / 64 + 63) & ~63);
  const int32_t nseg = max(1, (span + S - 1) / S);
  const bool mine = lane < nseg;
  const int32_t s0 = lane * S, s1 = min((lane + 1) * S, span);
  const int32_t pos0 = PROBE ? 0 : 4;
  B2H_GLB uint32_t* snv = snv_all + lane * kSegSnap;
  uint32_t snp[kSegSnap / 2] = {0u, 0u, 0u, 0u};
  int32_t nsnap = 0, merged = -1;
  // the first walk of every lane, from its segment's start (lane 0: the parse's start)
  int32_t epos = lane == 0 ? pos0 : s0;
  SegLane L{epos, 0, 0, 0, false, 0};
  seg_walk<PROBE, kSegFirst, WT>(in, bound, dist, mask, s1, mine, L, out, s0, snp, nsnap, snv, merged);
  const int32_t r1_o = L.o, r1_lit = L.lit, r1_exit = max(L.pos, epos);
  int32_t xpos = r1_exit, x_o = L.o, x_lit = L.lit, x_lead = L.lead;
  bool x_matched = L.matched;
  // Settle every lane's entry POSITION: the parse path does not depend on literal-run lengths, so
  // lane k enters where the furthest walk of the lanes before it left off (a prefix max); a lane
  // whose entry moved walks again from it until it meets its first walk's path.
  for (int round = 0; round < 64; round++) {
    const int32_t incl = wave_scan_max(mine ? xpos : -1);
    const int32_t prev = __shfl(incl, lane > 0 ? lane - 1 : 0);
    const int32_t np = (lane > 0 && mine) ? max(prev, s0) : epos;
    const bool redo = mine && np != epos;
    epos = np;
    SPROF_CNT(PB + 3, 1);
    if (__ballot(redo) == 0) break;
    merged = -1;
    if (redo) L = SegLane{epos, 0, 0, 0, false, L.steps};
    seg_walk<PROBE, kSegFix, WT>(in, bound, dist, mask, s1, redo, L, out, s0, snp, nsnap, snv, merged);
    if (redo) {
      if (merged >= 0) {   // the rest is the first walk's, from snapshot `merged` on
        const uint32_t v = snv[merged];
        const int32_t oj = (int32_t)(v >> 5), lj = (int32_t)(v & 31u);
        x_o = L.o + (r1_o - oj) + (L.lit != 0 ? 1 : 0) - (lj != 0 ? 1 : 0);
        x_lit = r1_lit;
        x_lead = L.lead;
        x_matched = true;
        xpos = r1_exit;
      } else {
        x_o = L.o;
        x_lit = L.lit;
        x_lead = L.lead;
        x_matched = L.matched;
        xpos = max(L.pos, epos);
      }
    }
  }
  SPROF_T(tp2);
  SPROF_ADD(PB + 1, tp1, tp2);
  SPROF_CNT(PB + 4, 1);
  {
    int32_t mx = L.steps;
    for (int off = 32; off >= 1; off >>= 1) mx = max(mx, __shfl_xor(mx, off));
    SPROF_CNT(PB + 5, mx);
  }
  // Fold the literal runs in, lane by lane (a scalar chain of <= 64 steps): lane k's entry run
  // and output offset
  int32_t lit = 4, o = 5, my_lit = 0, my_o = 0;
  for (int32_t k = 0; k < nseg; k++) {
    const int32_t lead = rdlane(x_lead, k);
    const bool matched = rdlane(x_matched ? 1 : 0, k) != 0;
    if (lane == k) {
      my_lit = lit;
      my_o = o;
    }
    o += rdlane(x_o, k) + seg_corr(lit, lead, matched);
    lit = matched ? rdlane(x_lit, k) : ((lit + lead) & 31);
  }
  const int32_t fpos = rdlane(xpos, nseg - 1);
  if constexpr (!PROBE) {
    // tail literals [fpos, bound] and the close (blosclz.c:611-619)
    const int32_t n = bound - fpos + 1;
    if (n > 0) {
      o += n + ((lit + n) >> 5);
      lit = (lit + n) & 31;
    }
    if (!lit) o--;
  }
  res.o = o;
  res.pos = fpos;
  res.peak = PROBE ? 0 : o + 1;
  res.fail = !PROBE && o + 1 > maxout;
  res.windows = L.steps;
  if (PROBE || res.fail) return res;
  // the emitting walk, from the settled entries, at the settled offsets
  if (lane == 0 && pos0 < length) {
    for (int i = 0; i < 4 && i < length; i++) st8<WT>(out, wt_rsrc(out), 1 + i, in[i]);
  }
  SegLane E{epos, my_lit, my_o, 0, true, 0};
  SPROF_T(tp3);
  seg_walk<PROBE, kSegEmit, WT>(in, bound, dist, mask, s1, mine, E, out, s0, snp, nsnap, snv, merged);
  if (lane == nseg - 1) {
    // tail literals + close
    const __amdgpu_buffer_rsrc_t r = wt_rsrc(out);
    int32_t oo = E.o, ll = E.lit;
    for (int32_t p = E.pos; p <= bound; p++) {
      const uint8_t b = in[p];
      st8<WT>(out, r, oo, oo == 0 ? (uint8_t)(b | 0x20u) : b);
      oo++;
      if (++ll == kLzMaxCopy) {
        const int32_t h = oo - kLzMaxCopy - 1;
        st8<WT>(out, r, h, (uint8_t)(h == 0 ? (31u | 0x20u) : 31u));
        ll = 0;
        oo++;
      }
    }
    if (ll) {
      const int32_t h = oo - ll - 1;
      st8<WT>(out, r, h, (uint8_t)(h == 0 ? ((uint32_t)(ll - 1) | 0x20u) : (uint32_t)(ll - 1)));
    }
  }
  SPROF_T(tp4);
  SPROF_ADD(PB + 2, tp3, tp4);
  return res;
}

// Mode 3 stream encode (one wave): run test, probe, emitting pass -- encode_stream_fast's
// decisions (blosc/blosclz.c:440-468) over the segmented passes.
template <bool WT, bool CHK>
__device__ __forceinline__ StreamResult encode_stream_seg(gin_t __restrict__ in, int32_t n, int clevel, gout_t __restrict__ out,
                                                          B2H_LDS uint8_t* tab, int tablog, B2H_GLB uint32_t* __restrict__ dist,
                                                          B2H_GLB uint64_t* __restrict__ mask,
                                                          B2H_GLB uint32_t* __restrict__ snv, bool allow_runs,
                                                          int32_t* lock) {
  StreamResult res;
  res.windows = 0;
  res.cycles = 0;
  res.peak = 0;
  res.kind = kStreamRaw;
  res.size = 0;
  SPROF_T(tr0);
  const bool isrun = allow_runs && wave_is_run(in, n);
  SPROF_T(tr1);
  SPROF_ADD(16, tr0, tr1);
  SPROF_CNT(17, 1);
  if (isrun) {
    res.size = in[0];
    res.kind = res.size ? kStreamByteRun : kStreamZeroRun;
    return res;
  }
  const int hashlog = clevel == 1 ? 12 : (clevel == 2 ? 13 : 14);
  const int tl = min(tablog, hashlog);
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  const LzPassOut pr = seg_pass<true, WT, CHK>(in + (n - maxlen), maxlen, hashlog, tl, out, 0, tab, dist, mask, snv, lock);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (ratio < thr || n < 66) return res;
  const LzPassOut em = seg_pass<false, WT, CHK>(in, n, hashlog, tl, out, n, tab, dist, mask, snv, lock);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

}  // namespace b2h
