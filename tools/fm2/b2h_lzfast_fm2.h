// b2h_lzfast.h -- BloscLZ "fast mode" encoder for gfx950 (device code): a segment-parallel parse.
//
// Same token grammar, greedy rule, length / distance limits, entropy-probe thresholds and byte
// emission as blosclz_compress (blosc/blosclz.c:248-316, 320-419, 422-619); the ONE difference is
// which earlier position a hash bucket offers as a position's candidate.  The reference inserts
// only the positions its serial walk visits, so every candidate depends on the whole parse before
// it.  Fast mode inserts EVERY position of the pass, in position order (model: tools/fm_model.c):
//
//     cand[p] = tab[hash(in[p..p+3])];  tab[hash] = p          for p = 0 .. loop_end-1
//
// so the greedy parse is a walk over a successor function known before the walk starts:
// next(p) = p + 1 (literal) or p + len(p) + 2 (match).  A workgroup of four waves owns one stream
// and runs it in SUPER-TILES of kFmS positions, the input in a 16 KiB LDS ring:
//
//   B  wave 0      the table exchanges, in position order (one LDS atomic per 64 positions; LDS
//                  applies the lanes of one instruction in lane order) -> per position the
//                  candidate distance d(p);
//   C  all waves   per position the 4-byte check m4(p) and the chain bit L(p) = m4(p) && d(p) ==
//                  d(p-1) (bit maps, one bit per position): a run of L bits is a stretch of
//                  positions that match at one distance, all ending where its last one ends;
//   C2 all waves   for the last position of every such run, where its match ends (one compare);
//   D  wave 0      the parse, SEGMENT-PARALLEL: lane k walks the greedy chain of segment k (32
//                  positions) from the segment start; then, until nothing changes, every lane
//                  whose entry (the exit of lane k-1's walk) moved re-walks from it and stops as
//                  soon as it reaches a position its previous walk visited -- from there the two
//                  walks coincide.  A match's length is one scan of the L map to its run's end.
//                  Greedy paths converge within a few elements, so a few short rounds replace the
//                  serial walk; the result is exactly the serial parse;
//   E  wave 0      per-lane element counts, DPP scans for every lane's output offset and literal
//                  state, then every lane writes its segment's literals and tokens into the LDS
//                  output ring (headers another lane's run needs patched in a second write), one
//                  flush of the finished bytes per super-tile; waves 1-3 meanwhile stage the next
//                  super-tile's input.
//
// Every match is verified byte for byte, so any output decodes with blosclz_decompress; the CPU
// model (tools/fm_model.c) is the bit-exact reference of the kernel (tests/test_fast_mode.py).
#pragma once
#include "b2h_lz.h"

namespace b2h {

constexpr int kFmWaves = 4, kFmThreads = 64 * kFmWaves;
constexpr int32_t kFmS = 1024;              // positions exchanged per super-tile
constexpr int32_t kFmHist = 32;             // positions of the previous super-tile kept (see fm_pass)
constexpr int32_t kFmSeg = 32;              // positions per walking lane (one 32-bit map word)
constexpr int32_t kFmWin = kFmHist + kFmS;  // record window [W, W + kFmWin), W = P - kFmHist
constexpr int kFmWalk = kFmS / kFmSeg;      // walking lanes (segments of [W, W + kFmS))
constexpr int32_t kFmAhead = 64;            // input staged past the window (keys, compares)
constexpr int32_t kFmH = 16384;             // input ring: position x at byte x & (kFmH - 1)
constexpr int32_t kFmCmpCap = 256;          // match-end compares stop here (longer: resolved in the walk)
constexpr int32_t kFmOpen = 0x7fffffff;     // walk exit inside a match whose end lies beyond the window
// rec word of a position: candidate distance d (0: none usable) in bits 0..16; for the last
// position of an L run, where its match ends (e - p, kFmEoffLong: past the compare cap) in 17..31
constexpr uint32_t kFmDMask = 0x1ffffu;
constexpr int32_t kFmEoffLong = 0x7fff;
// A pass that runs longer than this (s_memrealtime, 100 MHz) gives up at the next super-tile: the
// stream is stored raw (a valid chunk either way) and the result carries kFmLateBit in `windows`.
// Streams take well under a millisecond; the watchdog bounds every workgroup's time on the card.
constexpr uint64_t kFmWatchdogTicks = 50000000;   // 0.5 s
constexpr int32_t kFmLateBit = 1 << 29;
static_assert(kFmS % 64 == 0 && kFmS / 64 % kFmWaves == 0, "whole tiles per wave");
static_assert(kFmWalk <= 64 && kFmHist == kFmSeg, "one walking lane per map word");
static_assert(kFmH >= 2 * kFmS + kFmAhead + kFmHist, "ring holds the window while the next one loads");

struct FmShared {           // per workgroup
  int32_t entry;            // parse position entering the next super-tile (kFmOpen: open match)
  int32_t open_q, open_d;   // the open match (start, distance)
  int32_t o, lit, F, peak, fail, byte0, stop, pos;
  int32_t decide[2];        // probe decision / run verdict (wave 0 -> all)
  int32_t pull;             // the stream index the workgroup pulled
  int32_t bcast;            // k_encode_fast_fused: claims and hand-off words, lane 0 -> workgroup
  int32_t pad[2];
};

// Output ring: a super-tile emits at most kFmS + kFmS / 32 literal bytes plus its tokens, and a
// token's length-extension bytes can reach neblock / 255 (1 KiB for 256 KiB streams).
template <typename POS>
__host__ __device__ constexpr int32_t fm_ring_bytes() { return sizeof(POS) == 2 ? 2048 : 4096; }

// LDS layout of one workgroup: [rec][M map][L map][input ring][shared][output ring][table].  All
// but the table have a fixed size: the kernels address them with constant offsets (no SGPRs).
__host__ __device__ constexpr size_t fm_al16(size_t x) { return (x + 15) & ~size_t(15); }
constexpr size_t kFmOffRec = 0;
constexpr size_t kFmOffMb = kFmOffRec + fm_al16(4 * (size_t)(kFmWin + 1));
constexpr size_t kFmOffLb = kFmOffMb + fm_al16(kFmWin / 8 + 4);
constexpr size_t kFmOffHist = kFmOffLb + fm_al16(kFmWin / 8 + 4);
constexpr size_t kFmOffSh = kFmOffHist + kFmH;
constexpr size_t kFmOffRing = kFmOffSh + fm_al16(sizeof(FmShared));
template <typename POS>
__host__ __device__ constexpr size_t fm_off_tab() { return kFmOffRing + fm_ring_bytes<POS>(); }
template <typename POS>
__host__ __device__ constexpr size_t fm_lds_bytes(int tablog) { return fm_off_tab<POS>() + fm_al16(sizeof(POS) << tablog); }

struct FmBufs {
  B2H_LDS uint8_t* tab;
  B2H_LDS uint32_t* rec;    // rec[1 + x - W]: position x of the window
  B2H_LDS uint32_t* mb;     // bit x - W: m4(x)
  B2H_LDS uint32_t* lb;     // bit x - W: L(x) = m4(x) && d(x) == d(x - 1)
  B2H_LDS uint8_t* hist;    // input ring
  B2H_LDS uint8_t* ring;    // output ring
  B2H_LDS FmShared* sh;
};
template <typename POS>
__device__ __forceinline__ FmBufs fm_bufs(B2H_LDS uint8_t* smem) {
  FmBufs b;
  b.tab = smem + fm_off_tab<POS>();
  b.rec = (B2H_LDS uint32_t*)(smem + kFmOffRec);
  b.mb = (B2H_LDS uint32_t*)(smem + kFmOffMb);
  b.lb = (B2H_LDS uint32_t*)(smem + kFmOffLb);
  b.hist = smem + kFmOffHist;
  b.ring = smem + kFmOffRing;
  b.sh = (B2H_LDS FmShared*)(smem + kFmOffSh);
  return b;
}

#ifdef B2H_ENC_PROF   // diagnostics build only (tools/fast_micro.hip): event counters
__device__ uint64_t g_fm_cnt[8];
#define FM_CNT(i, v) do { if (lane_id() == 0) atomicAdd((unsigned long long*)&g_fm_cnt[i], (unsigned long long)(v)); } while (0)
#else
#define FM_CNT(i, v)
#endif

#ifdef B2H_FM_CHECK   // debug build only (lib_dbg): global accesses bounds-checked, the first violation recorded
__device__ int64_t g_fm_bad[8];
__device__ __noinline__ void fm_bad(int site, int64_t a, int64_t b, int64_t c) {
  if (atomicCAS((unsigned long long*)&g_fm_bad[0], 0ull, (unsigned long long)site) == 0ull) {
    g_fm_bad[1] = a;
    g_fm_bad[2] = b;
    g_fm_bad[3] = c;
    g_fm_bad[4] = blockIdx.x;
    g_fm_bad[5] = threadIdx.x;
  }
}
#ifdef B2H_FM_CHECK_INLINE
#define FM_OK(cond, site, a, b, c)                                                                       \
  ((cond) ? true                                                                                         \
          : (atomicCAS((unsigned long long*)&g_fm_bad[0], 0ull, (unsigned long long)(site)), g_fm_bad[1] = (a), false))
#else
#define FM_OK(cond, site, a, b, c) ((cond) ? true : (fm_bad(site, (a), (b), (c)), false))
#endif
#else
#define FM_OK(cond, site, a, b, c) true
#endif

// Bounded global access.  A pass reads its stream and writes its output only through buffer
// resources whose num_records is the stream's extent: the hardware range check turns an offset
// outside it into a zero load or a dropped store, never a fault.  The input resource starts at
// the dword below the stream (offsets carry the stream's misalignment `sh`), so unaligned words
// are two aligned dword loads and a funnel shift, as ldu32.
struct FmIn {
  __amdgpu_buffer_rsrc_t r;
  int32_t sh;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t fm_rsrc(uint64_t base, int32_t bytes) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0,
                                           max(bytes, 0), 0x00020000);
}
__device__ __forceinline__ FmIn fm_in(gin_t in, int32_t bytes) {
  const uint64_t a = reinterpret_cast<uintptr_t>(in);
  FmIn g;
  g.sh = __builtin_amdgcn_readfirstlane((int32_t)(a & 3));
  g.r = fm_rsrc(a & ~uint64_t(3), bytes + g.sh);
  return g;
}
__device__ __forceinline__ uint32_t fm_dw(const FmIn& g, int32_t y) {   // y: a dword offset
  return __builtin_amdgcn_raw_buffer_load_b32(g.r, y, 0, 0);
}
__device__ __forceinline__ uint32_t fm_ldu32(const FmIn& g, int32_t x) {
  const int32_t y = x + g.sh, a = y & ~3;
  return funnel(fm_dw(g, a), fm_dw(g, a + 4), (uint32_t)(y & 3));
}
__device__ __forceinline__ void fm_ld16(const FmIn& g, int32_t x, uint32_t (&w)[4]) {
  const int32_t y = x + g.sh, a = y & ~3;
  const uint32_t sh = (uint32_t)(y & 3);
  const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(g.r, a, 0, 0);
  const uint32_t e = fm_dw(g, a + 16);
  w[0] = funnel(v.x, v.y, sh);
  w[1] = funnel(v.y, v.z, sh);
  w[2] = funnel(v.z, v.w, sh);
  w[3] = funnel(v.w, e, sh);
}
__device__ __forceinline__ uint8_t fm_ldb(const FmIn& g, int32_t x) {
  return __builtin_amdgcn_raw_buffer_load_b8(g.r, x + g.sh, 0, 0);
}
// Output ring -> bytes [F, to) of the stream's output through its bounded resource (one wave);
// WT: write-through (`sc1`) stores, for streams another workgroup copies in the same launch.
template <bool WT, int32_t RING>
__device__ __forceinline__ void fm_flush(__amdgpu_buffer_rsrc_t r, bool al16, const B2H_LDS uint8_t* oring, int32_t F,
                                         int32_t to) {
  constexpr int32_t ORM = RING - 1;
  constexpr int kAux = WT ? 16 : 0;
  const int lane = lane_id();
  if (!al16 || to - F < 32) {
    for (int32_t y = F + lane; y < to; y += 64) __builtin_amdgcn_raw_buffer_store_b8(oring[y & ORM], r, y, 0, kAux);
    return;
  }
  const int32_t a = (F + 15) & ~15, b = to & ~15;
  if (lane < a - F) __builtin_amdgcn_raw_buffer_store_b8(oring[(F + lane) & ORM], r, F + lane, 0, kAux);
  if (lane < to - b) __builtin_amdgcn_raw_buffer_store_b8(oring[(b + lane) & ORM], r, b + lane, 0, kAux);
  for (int32_t y = a + 16 * lane; y < b; y += 1024)
    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const B2H_LDS u32x4*>(oring + (y & ORM)), r, y, 0, kAux);
}

#if defined(B2H_FM_TRACE) || defined(B2H_FM_TRACE_LITE)   // diagnostics builds only: per-workgroup progress
                                                          // words in host-coherent memory
__device__ int32_t* g_fm_trace;
#define FM_TRACE_S(slot, v)                                                                                   \
  do {                                                                                                        \
    if (threadIdx.x == 0 && g_fm_trace)                                                                       \
      __hip_atomic_store(&g_fm_trace[blockIdx.x * 16 + (slot)], (int32_t)(v), __ATOMIC_RELAXED,               \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                                          \
  } while (0)
#else
#define FM_TRACE_S(slot, v)
#endif
#ifdef B2H_FM_TRACE   // the pass-internal points (the lite build keeps only the stream-level ones)
#define FM_TRACE(slot, v) FM_TRACE_S(slot, v)
#else
#define FM_TRACE(slot, v)
#endif

__device__ __forceinline__ uint32_t fm_from(int32_t lo) { return lo >= 32 ? 0u : (~0u << lo); }
__device__ __forceinline__ uint32_t fm_below(int32_t hi) { return hi >= 32 ? ~0u : ((1u << hi) - 1u); }

// little-endian u32 at position x of the input ring
__device__ __forceinline__ uint32_t fm_hist32(const B2H_LDS uint8_t* hist, int32_t x) {
  const B2H_LDS uint32_t* w = (const B2H_LDS uint32_t*)hist;
  constexpr int32_t M = kFmH / 4 - 1;
  const int32_t i = x >> 2;
  return funnel(w[i & M], w[(i + 1) & M], (uint32_t)(x & 3));
}

// Four table exchanges (positions in lane order within each, the four in program order): the
// bucket's previous occupant is returned and p stored.  u16 buckets (streams <= 64 KiB) share a
// dword two by two and go through ds_mskor_rtn_b32 ((old & ~mask) | p << sh, old returned); the
// four are issued back to back and waited for once.
template <typename POS>
__device__ __forceinline__ void fm_exchange4(const uint32_t (&key)[4], const int32_t (&p)[4], const bool (&valid)[4],
                                             int tablog, B2H_LDS uint8_t* tab, uint32_t (&cand)[4]) {
  if constexpr (sizeof(POS) == 4) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      cand[u] = 0;
      if (valid[u])
        cand[u] = __hip_atomic_exchange(&((B2H_LDS uint32_t*)tab)[lz_hash(key[u], tablog)], (uint32_t)p[u],
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  } else {
    uint32_t addr[4], mask[4], data[4], sh[4], w[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t h = lz_hash(key[u], tablog);
      // invalid lanes: a zero mask and zero data leave the dword unchanged
      addr[u] = (uint32_t)reinterpret_cast<uintptr_t>(tab) + ((h >> 1) << 2);
      sh[u] = (h & 1u) << 4;
      mask[u] = valid[u] ? (0xffffu << sh[u]) : 0u;
      data[u] = valid[u] ? ((uint32_t)p[u] << sh[u]) : 0u;
    }
    asm volatile(
        "ds_mskor_rtn_b32 %0, %4, %8, %12\n\t"
        "ds_mskor_rtn_b32 %1, %5, %9, %13\n\t"
        "ds_mskor_rtn_b32 %2, %6, %10, %14\n\t"
        "ds_mskor_rtn_b32 %3, %7, %11, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
        : "v"(addr[0]), "v"(addr[1]), "v"(addr[2]), "v"(addr[3]), "v"(mask[0]), "v"(mask[1]), "v"(mask[2]),
          "v"(mask[3]), "v"(data[0]), "v"(data[1]), "v"(data[2]), "v"(data[3])
        : "memory");
#pragma unroll
    for (int u = 0; u < 4; u++) cand[u] = valid[u] ? ((w[u] >> sh[u]) & 0xffffu) : 0u;
  }
}

// One past the first byte at or after x where in[] and in[-d] differ, capped at `bound` (get_match
// semantics, blosc/blosclz.c:148-165), one lane, 16 bytes per step from global memory.
__device__ __forceinline__ int32_t fm_lane_match_end(const FmIn& G, int32_t x, uint32_t d, int32_t bound) {
  if (!FM_OK(x - (int32_t)d >= 0 && d > 0, 3, x, d, bound)) return bound;
  while (x < bound) {
    uint32_t a[4], b[4];
    fm_ld16(G, x, a);
    fm_ld16(G, x - (int32_t)d, b);
    const int32_t nb = bound - x;
#pragma unroll
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

// Pass geometry (blosc/blosclz.c:440-482, get_cratio 320-419).
template <bool PROBE>
__device__ __forceinline__ void fm_limits(int32_t length, int probe_hashlog, int32_t* limit, int32_t* bound,
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

// Length of the match at q (d = its candidate distance, m4(q) set): the run of L bits after q,
// then where its last position's match ends (phase C2).  Returns the token length, -1 (literal)
// or kFmOpen (the run reaches the window's end: resolved in the next super-tile).  j0: window
// index where the run starts (q - W + 1; kFmHist for a match carried in from the last super-tile).
template <bool PROBE>
__device__ __forceinline__ int32_t fm_match_len(int32_t q, uint32_t d, int32_t j0, int32_t W, int32_t bound,
                                                const FmIn& in, const B2H_LDS uint32_t* rec, const B2H_LDS uint32_t* lb) {
  int32_t j = j0;
  while (j < kFmWin) {
    const int32_t s = j & 31;
    const uint32_t nw = ~(lb[j >> 5] >> s);   // the shifted-in bits read as "clear"
    const int32_t ones = nw ? (int32_t)__builtin_ctz(nw) : 32;
    j += ones;
    if (ones < 32 - s) break;
  }
  if (j >= kFmWin) return kFmOpen;
  const int32_t qe = W + j - 1;   // the run's last position
  const int32_t eo = (int32_t)(rec[j] >> 17);
  int32_t e;
  if (eo == kFmEoffLong) {
    FM_CNT(2, 1);
    e = fm_lane_match_end(in, qe + 4, d, bound);
  } else {
    e = qe + eo;
  }
  const int32_t len = e - 4 - q;
  if (len < 4 || (!PROBE && len <= 5 && d - 1 >= kLzNear)) return -1;
  return len;
}

// Token bytes of a match (MATCH_SHORT / MATCH_LONG (+ _FAR), blosc/blosclz.c:270-316).
__device__ __forceinline__ int32_t fm_tok(int32_t len, uint32_t d) {
  return (len >= 7 ? 1 + (len - 7) / 255 : 0) + ((d - 1) < kLzNear ? 2 : 4);
}

// Walk of one segment [a, hi) from e: element starts VIS (literals and match starts), match
// starts MS, exit x.  With `conv`, stops at the first position the previous walk (VISo, MSo, xo)
// visited: from there both walks coincide.
template <bool PROBE>
__device__ __forceinline__ void fm_walk(int32_t e, int32_t a, int32_t hi, uint32_t Mw, bool conv, uint32_t VISo,
                                        uint32_t MSo, int32_t xo, int32_t W, int32_t bound, const FmIn& in,
                                        const B2H_LDS uint32_t* rec, const B2H_LDS uint32_t* lb, int32_t& x,
                                        uint32_t& MS, uint32_t& VIS) {
  int32_t p = e;
  uint32_t ms = 0, vis = 0;
  while (p < hi) {
    const int32_t rel = p - a;
    const uint32_t mm = Mw & fm_from(rel);
    const int32_t qrel = mm ? (int32_t)__builtin_ctz(mm) : hi - a;
    const uint32_t lits = fm_from(rel) & fm_below(qrel);
    const uint32_t starts = lits | (mm ? (1u << qrel) : 0u);
    if (conv && (starts & VISo)) {
      const int32_t c = (int32_t)__builtin_ctz(starts & VISo);
      const uint32_t lo = fm_below(c);
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
    const int32_t len = fm_match_len<PROBE>(q, rec[1 + (q - W)] & kFmDMask, q - W + 1, W, bound, in, rec, lb);
    if (len < 0) {
      p = q + 1;
    } else {
      ms |= 1u << qrel;
      if (len == kFmOpen) {
        p = kFmOpen;
        break;
      }
      p = q + len + 2;
    }
  }
  MS = ms;
  VIS = vis;
  x = p;
}

// One pass of the workgroup over a stream (all four waves call it).  PROBE: get_cratio's count;
// else the emitting pass into `out` (maxout = length), the ring flushed per super-tile.
//
// Windows: super-tile P exchanges and checks positions [P, P + kFmS), and walks [W, W + kFmS) with
// W = P - kFmHist; the last kFmHist positions it checked are walked by the next super-tile, whose
// window starts with their records.  So a match whose L run reaches the window's end started at
// least kFmHist positions before it: it is accepted whatever its end, and is carried OPEN.
template <bool PROBE, typename POS, bool WT>
__device__ __forceinline__ LzPassOut fm_pass(gin_t __restrict__ in_ptr, int32_t length, int probe_hashlog, int tablog,
                                             gout_t __restrict__ out_ptr, int32_t maxout, const FmBufs& B, int clevel) {
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  constexpr int32_t RM = fm_ring_bytes<POS>() - 1;
  constexpr int kAux = WT ? 16 : 0;
  int32_t limit, bound, loop_end;
  fm_limits<PROBE>(length, probe_hashlog, &limit, &bound, &loop_end);
  const FmIn in = fm_in(in_ptr, length);
  const __amdgpu_buffer_rsrc_t out = fm_rsrc(reinterpret_cast<uintptr_t>(out_ptr), PROBE ? 0 : maxout);
  const bool out16 = (reinterpret_cast<uintptr_t>(out_ptr) & 15) == 0;
  {
    B2H_LDS u32x4* t16 = (B2H_LDS u32x4*)B.tab;
    const int32_t n16 = (int32_t)((sizeof(POS) << tablog) / 16);
    for (int32_t i = threadIdx.x; i < n16; i += kFmThreads) t16[i] = u32x4{0u, 0u, 0u, 0u};
    B2H_LDS u32x4* h16 = (B2H_LDS u32x4*)B.hist;
    for (int32_t i = threadIdx.x; i < kFmH / 16; i += kFmThreads) h16[i] = u32x4{0u, 0u, 0u, 0u};
  }
  if (threadIdx.x == 0) {
    B.sh->entry = PROBE ? 0 : 4;
    B.sh->open_q = -1;
    B.sh->open_d = 0;
    B.sh->o = 5;
    B.sh->lit = 4;
    B.sh->F = 0;
    B.sh->peak = 0;
    B.sh->fail = 0;
    B.sh->byte0 = kLzMaxCopy - 1;
    B.sh->stop = 0;
    B.sh->pos = PROBE ? 0 : 4;
  }
  if (!PROBE && wave == 0 && lane < 5) {
    // the stream starts with a marker and four literals
    const uint8_t b = fm_ldb(in, lane - 1);
    B.ring[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : b;
  }
  int32_t windows = 0;
  EPROF_DECL;
  // input positions [lo, hi) (multiples of 16) into the ring, zero at and past `limit`, by threads
  // [t0, t0 + nth)
  auto stage = [&](int32_t lo, int32_t hi, int32_t t0, int32_t nth) {
    const int32_t tid = (int32_t)threadIdx.x - t0;
    constexpr int32_t HM = kFmH - 1;
    if (hi <= limit && ((reinterpret_cast<uintptr_t>(in_ptr + lo) & 15) == 0)) {   // then in.sh == 0
      for (int32_t x = lo + 16 * tid; x < hi; x += 16 * nth)
        if (FM_OK(x >= 0 && x + 16 <= limit, 7, x, lo, hi))
          *(B2H_LDS u32x4*)(B.hist + (x & HM)) = __builtin_amdgcn_raw_buffer_load_b128(in.r, x, 0, 0);
    } else {
      for (int32_t x = lo + 4 * tid; x < hi; x += 4 * nth) {
        uint32_t w = 0;
        if (x + 4 <= limit) {
          w = fm_ldu32(in, x);
        } else {
          for (int k = 0; k < 4; k++)
            if (x + k < limit) w |= (uint32_t)fm_ldb(in, x + k) << (8 * k);
        }
        *(B2H_LDS uint32_t*)(B.hist + (x & HM)) = w;
      }
    }
  };
  __syncthreads();   // the ring is clear
  stage(0, kFmS + kFmAhead, 0, kFmThreads);
  __syncthreads();
  FM_TRACE(3, PROBE ? 1 : 2);
  FM_TRACE(9, loop_end);
  const uint64_t t_begin = __builtin_amdgcn_s_memrealtime();
  // one exit, decided last from broadcast values (see encode_stream_fast on uniform branches)
  bool more = -kFmHist < loop_end;
  for (int32_t P = 0; more; P += kFmS) {
    EPROF_T(tb0);
    FM_TRACE(4, P);
    const int32_t W = P - kFmHist;
    const int32_t rlo = P + kFmS + kFmAhead - kFmH;   // the ring holds [rlo, P + kFmS + kFmAhead)
    windows++;
    const int32_t entry0 = __builtin_amdgcn_readfirstlane(B.sh->entry);
    const bool has_open = entry0 == kFmOpen;
    FM_TRACE(5, entry0);
    FM_TRACE(6, 1);
    // ---- B: the history records move to the window's front; the exchanges of [P, P + kFmS) in
    // position order (wave 0)
    if (wave == 0) {
      const uint32_t hrec = (P > 0 && lane < kFmHist) ? B.rec[1 + kFmS + lane] : 0u;
      const uint32_t hm = P > 0 ? B.mb[kFmS / 32] : 0u, hl = P > 0 ? B.lb[kFmS / 32] : 0u;
      // lanes 32-63 of the exchanges below overwrite what lanes 0-31 just read: keep the reads
      // first (no lane aliases itself, so only a compiler memory barrier holds the order;
      // __builtin_amdgcn_wave_barrier does not order memory accesses)
      asm volatile("" ::: "memory");
      if (lane < kFmHist) B.rec[1 + lane] = hrec;
      if (lane == 0) {
        B.rec[0] = 0;
        B.mb[0] = hm;
        B.lb[0] = hl;
      }
      const int32_t ntiles = max(0, min(kFmS, loop_end - P) + 63) / 64;
      for (int32_t t0 = 0; t0 < ntiles; t0 += 4) {
        uint32_t key[4], cand[4];
        int32_t p[4];
        bool valid[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
          p[u] = P + (t0 + u) * 64 + lane;
          valid[u] = t0 + u < ntiles && p[u] < loop_end;
          key[u] = fm_hist32(B.hist, p[u]);
        }
        fm_exchange4<POS>(key, p, valid, tablog, B.tab, cand);
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const uint32_t d = (uint32_t)(p[u] - (int32_t)cand[u]);
          if (t0 + u < ntiles) B.rec[1 + kFmHist + (t0 + u) * 64 + lane] = (valid[u] && d != 0 && d < kLzFar) ? d : 0u;
        }
      }
      for (int32_t i = ntiles * 64 + lane; i < kFmS; i += 64) B.rec[1 + kFmHist + i] = 0;
    }
    EPROF_T(tb1);
    EPROF_ADD(1, tb0, tb1);
    FM_TRACE(6, 2);
    __syncthreads();
    EPROF_T(tc0);
    // ---- C: 4-byte checks and chain bits of [P, P + kFmS); every load of a wave's tiles issued
    // before the first compare
    {
      constexpr int NT = kFmS / 64 / kFmWaves;
      uint32_t key[NT], d[NT], dp[NT], cw[NT];
#pragma unroll
      for (int u = 0; u < NT; u++) {
        const int32_t i = (wave + kFmWaves * u) * 64 + lane;
        const int32_t q = P + i;
        key[u] = fm_hist32(B.hist, q);
        d[u] = B.rec[1 + kFmHist + i];
        dp[u] = B.rec[kFmHist + i] & kFmDMask;
        const int32_t c = q - (int32_t)d[u];
        cw[u] = d[u] == 0 ? 0u : (c >= rlo ? fm_hist32(B.hist, c) : (FM_OK(c >= 0 && c < limit, 1, c, d[u], q) ? fm_ldu32(in, c) : 0u));
      }
#pragma unroll
      for (int u = 0; u < NT; u++) {
        const int32_t t = wave + kFmWaves * u;
        const bool m4 = d[u] != 0 && cw[u] == key[u];
        const uint64_t mb = __ballot(m4), lbm = __ballot(m4 && d[u] == dp[u]);
        if (lane == 0) {
          B.mb[1 + 2 * t] = (uint32_t)mb;
          B.mb[2 + 2 * t] = (uint32_t)(mb >> 32);
          B.lb[1 + 2 * t] = (uint32_t)lbm;
          B.lb[2 + 2 * t] = (uint32_t)(lbm >> 32);
        }
      }
    }
    __syncthreads();
    // ---- C2: where the match of the last position of every L run ends (window indices
    // [kFmHist - 1, kFmWin - 1): the run ending at P - 1 could not be told from the last window)
    for (int32_t j = kFmHist - 1 + (int32_t)threadIdx.x; j < kFmWin - 1; j += kFmThreads) {
      const bool m4 = (B.mb[j >> 5] >> (j & 31)) & 1u;
      const bool next = (B.lb[(j + 1) >> 5] >> ((j + 1) & 31)) & 1u;
      if (m4 && !next) {
        const uint32_t rw = B.rec[1 + j];
        const uint32_t d = rw & kFmDMask;
        const int32_t q = W + j;
        int32_t x = q + 4, e = -1;
        const int32_t xmax = min(bound, q + kFmCmpCap);
        while (x < xmax) {
          uint32_t a, b;
          if (x + 4 <= P + kFmS + kFmAhead && x - (int32_t)d >= rlo) {
            a = fm_hist32(B.hist, x);
            b = fm_hist32(B.hist, x - (int32_t)d);
          } else if (FM_OK(x - (int32_t)d >= 0 && x < limit, 2, x, d, q)) {
            a = fm_ldu32(in, x);
            b = fm_ldu32(in, x - (int32_t)d);
          } else {
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
        const int32_t eo = e >= 0 ? e - q : (x >= bound ? bound - q : kFmEoffLong);
        B.rec[1 + j] = d | ((uint32_t)eo << 17);
      }
    }
    EPROF_T(tc1);
    EPROF_ADD(2, tc0, tc1);
    FM_TRACE(6, 3);
    __syncthreads();
    EPROF_T(td0);
    EPROF_ADD(7, tc1, td0);
    // the next super-tile's input, by waves 1-3 while wave 0 parses (it overwrites the oldest
    // kFmS bytes of the ring, which the parse no longer reads)
    if (wave != 0 && P + kFmS - kFmHist < loop_end)
      stage(P + kFmS + kFmAhead, P + 2 * kFmS + kFmAhead, 64, kFmThreads - 64);
    // ---- D + E (wave 0), unless a known match covers the whole walk region
    if (wave == 0 && (has_open || entry0 < W + kFmS)) {
      const int32_t a = W + kFmSeg * lane;
      const int32_t hi = min(min(a + kFmSeg, loop_end), W + kFmS);   // lanes >= kFmWalk: empty
      const uint32_t Mw = lane < kFmWalk ? B.mb[lane] : 0u;
      // lane 0: the carried entry (a position, or an open match resolved first)
      int32_t cm_q = -1, cm_len = 0;
      uint32_t cm_d = 0;
      int32_t e = lane == 0 ? entry0 : a;
      int32_t x;
      uint32_t MS = 0, VIS = 0;
      if (lane == 0 && has_open) {
        cm_q = B.sh->open_q;
        cm_d = (uint32_t)B.sh->open_d;
        cm_len = fm_match_len<PROBE>(cm_q, cm_d, kFmHist, W, bound, in, B.rec, B.lb);
        if (cm_len != kFmOpen) e = cm_q + cm_len + 2;   // an open match is always accepted
      }
      if (e >= hi) {
        x = e;
      } else {
        fm_walk<PROBE>(e, a, hi, Mw, false, 0u, 0u, 0, W, bound, in, B.rec, B.lb, x, MS, VIS);
      }
      EPROF_T(td1);
      EPROF_ADD(3, td0, td1);
      FM_TRACE(6, 4);
      // fixpoint: every lane's entry follows the exit of the lane below until nothing moves
      int32_t rounds = 0;
      for (;;) {
        rounds++;
        const int32_t xl = __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, false);   // wave_shr:1
        const int32_t en = lane == 0 ? e : xl;
        const bool changed = lane < kFmWalk && en != e;
        if (!__ballot(changed)) break;
        if (changed) {
          e = en;
          if (en >= hi) {
            x = en;
            MS = VIS = 0;
          } else {
            fm_walk<PROBE>(en, a, hi, Mw, true, VIS, MS, x, W, bound, in, B.rec, B.lb, x, MS, VIS);
          }
        }
      }
      EPROF_T(td2);
      EPROF_ADD(4, td1, td2);
      FM_TRACE(6, 5);
      FM_TRACE(8, rounds);
      FM_CNT(PROBE ? 4 : 0, rounds);
      FM_CNT(PROBE ? 5 : 1, 1);
      const uint32_t LITS = VIS & ~MS;
      // the lane's elements in order: literal runs (bit masks of the segment) and matches; an
      // open match (the lane's last) is left to the super-tile where it ends
      auto elements = [&](auto&& on_lits, auto&& on_match) {
        const int32_t f = MS ? (int32_t)__builtin_ctz(MS) : 32;
        int32_t prev = -2;
        if (cm_q >= 0) {
          if (cm_len != kFmOpen) on_match(cm_len, cm_d);
          prev = -1;
        } else {
          on_lits(LITS & fm_below(f));
        }
        uint32_t rem = MS;
        bool open = false;
        while (rem) {
          const int32_t m = (int32_t)__builtin_ctz(rem);
          rem &= rem - 1;
          if (prev != -2) on_lits(LITS & fm_from(prev + 1) & fm_below(m));
          const int32_t q = a + m;
          const uint32_t d = B.rec[1 + (q - W)] & kFmDMask;
          const int32_t len = fm_match_len<PROBE>(q, d, q - W + 1, W, bound, in, B.rec, B.lb);
          if (len == kFmOpen) {
            open = true;
            break;
          }
          on_match(len, d);
          prev = m;
        }
        if (!open && prev != -2) on_lits(LITS & fm_from(prev + 1));
      };
      // ---- per-lane summary: A literals before the first match, Bb bytes from the first match
      // on (literal state 0 after it), T the literal state at the end
      int32_t A = 0, Bb = 0, t = 0, T = 0;
      bool has = false;
      elements([&](uint32_t bits) {
                 const int32_t n = __builtin_popcount(bits);
                 if (has) t += n;
                 else A += n;
               },
               [&](int32_t len, uint32_t d) {
                 if (has) Bb += t + t / 32 - ((t & 31) == 0 ? 1 : 0);
                 has = true;
                 t = 0;
                 Bb += fm_tok(len, d) + 1;
               });
      if (has) {
        Bb += t + t / 32;
        T = t & 31;
      }
      // ---- scan: the literal state entering each lane (segmented at the lanes with a match),
      // then the output offsets
      const int32_t lit_in = __builtin_amdgcn_readfirstlane(B.sh->lit);
      const int32_t o_in = __builtin_amdgcn_readfirstlane(B.sh->o);
      const int32_t X = has ? 0 : A;
      const int32_t PX = wave_scan_add(X);
      const int32_t mlast = wave_scan_max(has ? lane : -1);
      const int32_t mex = __builtin_amdgcn_update_dpp(-1, mlast, 0x138, 0xf, 0xf, false);   // exclusive
      const int32_t Ym = __builtin_amdgcn_ds_bpermute(max(mex, 0) << 2, T - PX);
      const int32_t R = (lane > 0 && mex >= 0 ? Ym : lit_in) + (PX - X);
      const int32_t litk = R & 31;
      const int32_t s0 = litk + A;
      const int32_t size = A + s0 / 32 + (has ? Bb - ((s0 & 31) == 0 ? 1 : 0) : 0);
      const int32_t incl = wave_scan_add(size);
      const int32_t o_out = o_in + rdlane(incl, 63);
      const int32_t lit_out = rdlane(has ? T : (s0 & 31), 63);
      const int32_t x_out = rdlane(x, kFmWalk - 1);
      const bool opener = lane < kFmWalk && x == kFmOpen && e != kFmOpen;
      const uint64_t om = __ballot(opener);
      int32_t stop = 0;
      EPROF_T(td3);
      EPROF_ADD(5, td2, td3);
      if (!PROBE) {
        // ---- E: every lane writes its elements from (o, lit); the first match's header patch
        // (or, after a run of 0 mod 32 literals, its token's first byte, over the marker) lands
        // on a byte another lane wrote, so it is written after every lane's own bytes
        int32_t o = o_in + incl - size, lit = litk, req = 0, dpos = -1;
        uint32_t dval = 0;
        bool first = true;
        elements(
            [&](uint32_t bits) {
              while (bits) {
                const int32_t j = (int32_t)__builtin_ctz(bits);
                bits &= bits - 1;
                req = max(req, o + 2);
                B.ring[o & RM] = B.hist[(a + j) & (kFmH - 1)];
                o++;
                if (++lit == kLzMaxCopy) {
                  B.ring[o & RM] = (uint8_t)(kLzMaxCopy - 1);
                  o++;
                  lit = 0;
                }
              }
            },
            [&](int32_t len, uint32_t d) {
              int32_t p0;
              uint32_t v0;
              const uint32_t bd = d - 1;
              const bool near = bd < kLzNear;
              const uint32_t fd = bd - kLzNear;
              const uint32_t b0 = (len >= 7 ? (7u << 5) : ((uint32_t)len << 5)) + (near ? (bd >> 8) : 31u);
              if (lit) {
                p0 = o - lit - 1;
                v0 = (uint32_t)(lit - 1);
                B.ring[o & RM] = (uint8_t)b0;
              } else {
                o--;
                p0 = o;
                v0 = b0;
              }
              if (first) {
                dpos = p0;
                dval = v0;
              } else {
                B.ring[p0 & RM] = (uint8_t)v0;
              }
              int32_t w = o + 1;
              if (len >= 7) {
                uint32_t rem = (uint32_t)len - 7;
                for (; rem >= 255; rem -= 255) B.ring[(w++) & RM] = 255;
                B.ring[(w++) & RM] = (uint8_t)rem;
              }
              if (near) {
                B.ring[(w++) & RM] = (uint8_t)(bd & 255);
              } else {
                B.ring[(w++) & RM] = 255;
                B.ring[(w++) & RM] = (uint8_t)(fd >> 8);
                B.ring[(w++) & RM] = (uint8_t)(fd & 255);
              }
              B.ring[(w++) & RM] = (uint8_t)(kLzMaxCopy - 1);
              o = w;
              lit = 0;
              req = max(req, o);
              first = false;
            });
        asm volatile("" ::: "memory");
        if (dpos >= 0) B.ring[dpos & RM] = (uint8_t)dval;
        asm volatile("" ::: "memory");
        // the lanes' bound checks; a failure ends the pass (the stream is stored raw)
        int32_t rq = req;
#pragma unroll
        for (int sft = 32; sft >= 1; sft >>= 1) rq = max(rq, __shfl_xor(rq, sft));
        const int32_t peak = max(__builtin_amdgcn_readfirstlane(B.sh->peak), __builtin_amdgcn_readfirstlane(rq));
        const bool fail = peak > maxout;
        int32_t F = __builtin_amdgcn_readfirstlane(B.sh->F);
        int32_t byte0 = __builtin_amdgcn_readfirstlane(B.sh->byte0);
        if (!fail) {
          const int32_t fin = (o_out - lit_out - 1) & ~15;   // bytes below the pending header are final
          if (fin > F && FM_OK(F >= 0 && fin <= maxout, 5, F, fin, maxout)) {
            if (F == 0) byte0 = __builtin_amdgcn_readfirstlane((int32_t)B.ring[0]);
            fm_flush<WT, RM + 1>(out, out16, B.ring, F, fin);
            F = fin;
          }
        } else {
          stop = 1;
        }
        if (lane == 0) {
          B.sh->peak = peak;
          B.sh->F = F;
          B.sh->byte0 = byte0;
        }
      }
      if (lane == 0) {
        B.sh->o = o_out;
        B.sh->lit = lit_out;
        B.sh->entry = x_out;
        if (x_out != kFmOpen) B.sh->pos = x_out;
      }
      if (om) {   // the open match leaving this super-tile: its start and distance
        const int32_t k = (int32_t)__builtin_ctzll(om);
        const uint32_t msk = (uint32_t)__builtin_amdgcn_readlane((int32_t)MS, k);
        const int32_t q = W + kFmSeg * k + 31 - (int32_t)__builtin_clz(msk);
        if (lane == 0) {
          B.sh->open_q = q;
          B.sh->open_d = (int32_t)(B.rec[1 + (q - W)] & kFmDMask);
        }
      }
      if (PROBE && x_out != kFmOpen) {
        const double thr_o = 0.999 * (clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2
                                      : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0);
        const double thr_s = thr_o * (1.001 / 0.999);
        if ((double)(limit + 64) < thr_o * (double)o_out) {
          stop = 2;   // early: the ratio can no longer reach the threshold
        } else {
          const int32_t Rr = loop_end - x_out;
          if ((double)loop_end >= thr_s * (double)(o_out + Rr + Rr / 16 + 16)) stop = 3;   // sure
        }
      }
      if (lane == 0 && stop) B.sh->stop = stop;
      EPROF_T(td4);
      EPROF_ADD(6, td3, td4);
      FM_TRACE(7, o_out);
      FM_TRACE(6, 6);
    }
    FM_TRACE(6, 7);
    // the watchdog: one thread decides, every wave reads the verdict after the barrier
    if (threadIdx.x == 0 && __builtin_amdgcn_s_memrealtime() - t_begin > kFmWatchdogTicks) {
      B.sh->stop = PROBE ? 2 : 1;
      B.sh->fail = kFmLateBit;
      FM_TRACE(13, P);
      FM_TRACE(14, loop_end);
    }
    __syncthreads();
    const int32_t stop = __builtin_amdgcn_readfirstlane(B.sh->stop);
    const int32_t ent = __builtin_amdgcn_readfirstlane(B.sh->entry);
    FM_TRACE(10, windows);
    more = !stop && (ent == kFmOpen || ent < loop_end) && P + kFmS - kFmHist < loop_end;
  }
  if (wave == 0) {
    EPROF_FLUSH;
  }
  FM_TRACE(6, 8);
  LzPassOut r;
  const int32_t stop = __builtin_amdgcn_readfirstlane(B.sh->stop);
  r.fail = stop == 1;
  r.early = stop == 2;
  r.sure = stop == 3;
  r.pos = __builtin_amdgcn_readfirstlane(B.sh->pos);
  r.o = __builtin_amdgcn_readfirstlane(B.sh->o);
  r.peak = __builtin_amdgcn_readfirstlane(B.sh->peak);
  r.windows = windows | (__builtin_amdgcn_readfirstlane(B.sh->fail) & kFmLateBit);
  if (!PROBE) {
    if (!r.fail && wave == 0) {
      // tail literals [pos, bound] (blosc/blosclz.c:595-604), then the last run's header
      int32_t o = r.o, lit = __builtin_amdgcn_readfirstlane(B.sh->lit), peak = r.peak;
      const int32_t pos = r.pos;
      const int32_t F = __builtin_amdgcn_readfirstlane(B.sh->F);
      int32_t byte0 = __builtin_amdgcn_readfirstlane(B.sh->byte0);
      bool fail = false;
      if (pos <= bound) {
        const int32_t cnt = bound - pos + 1;   // <= 12: a match ends at most at bound - 2
        const int32_t last = o + (cnt - 1) + (lit + cnt - 1) / 32;
        peak = max(peak, last + 2);
        if (last + 2 > maxout) {
          fail = true;
        } else {
          if (lane < cnt && FM_OK(pos + lane >= 0 && pos + lane < limit, 4, pos, cnt, bound)) {
            const int32_t off = o + lane + (lit + lane) / 32;
            B.ring[off & RM] = fm_ldb(in, pos + lane);
            if (((lit + lane + 1) & 31) == 0) B.ring[(off + 1) & RM] = (uint8_t)(kLzMaxCopy - 1);
          }
          o += cnt + (lit + cnt) / 32;
          lit = (lit + cnt) & 31;
        }
      }
      if (!fail) {
        asm volatile("" ::: "memory");
        if (lit) {
          const int32_t at = o - lit - 1;
          if (lane == 0) B.ring[at & RM] = (uint8_t)(lit - 1);
          if (at == 0) byte0 = lit - 1;
        } else {
          o--;
        }
        asm volatile("" ::: "memory");
        if (!FM_OK(o >= 0 && o <= maxout && F <= o, 6, F, o, maxout)) {
        } else if (F == 0) {
          byte0 = __builtin_amdgcn_readfirstlane((int32_t)B.ring[0]);
          if (lane == 0) B.ring[0] = (uint8_t)(byte0 | 0x20);
          asm volatile("" ::: "memory");
          fm_flush<WT, RM + 1>(out, out16, B.ring, 0, o);
        } else {
          fm_flush<WT, RM + 1>(out, out16, B.ring, F, o);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(byte0 | 0x20), out, 0, 0, kAux);
        }
      }
      if (lane == 0) {
        B.sh->o = o;
        B.sh->peak = peak;
        B.sh->fail = fail ? 1 : 0;
      }
    } else if (wave == 0 && lane == 0) {
      B.sh->fail = 1;
    }
    // every wave returns wave 0's result
    __syncthreads();
    r.o = __builtin_amdgcn_readfirstlane(B.sh->o);
    r.peak = __builtin_amdgcn_readfirstlane(B.sh->peak);
    r.fail = __builtin_amdgcn_readfirstlane(B.sh->fail) != 0;
  }
  __syncthreads();   // the shared words are re-initialised by the next pass
  return r;
}

// Fast-mode stream encode (the whole workgroup): run test, entropy probe, main pass; maxout =
// neblock, `peak` for the chunk finaliser (b2h_lz.h).
template <typename POS, bool WT = false>
__device__ __forceinline__ StreamResult encode_stream_fast(gin_t __restrict__ in, int32_t n, int clevel, gout_t __restrict__ out,
                                                            const FmBufs& B, int tablog, bool allow_runs) {
  StreamResult res;
  res.windows = 0;
  res.cycles = 0;
  res.peak = 0;
  res.kind = kStreamRaw;
  res.size = 0;
  const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  if (allow_runs) {
    // waves 0 and 1 test one half each against in[0]
    const int32_t h = (n / 2) & ~15;
    bool half_run = true;
    if (wave == 0) half_run = wave_is_run(in, h + 1);
    else if (wave == 1) half_run = wave_is_run_from(in, h, n, in[0]);
    if (wave < 2 && lane_id() == 0) B.sh->decide[wave] = half_run ? 1 : 0;
    __syncthreads();
    // readfirstlane: a branch the compiler must see as uniform (a divergent-looking branch around the
    // passes' barriers gets structurized into exec-masked paths that run s_barrier a different
    // number of times per wave -- the stream loop then hangs or reads a stale stream index)
    const bool run = (__builtin_amdgcn_readfirstlane(B.sh->decide[0]) & __builtin_amdgcn_readfirstlane(B.sh->decide[1])) != 0;
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
  FM_TRACE_S(6, 20);
  const LzPassOut pr = fm_pass<true, POS, WT>(in + (n - maxlen), maxlen, hashlog, tl, out, 0, B, clevel);
  FM_TRACE_S(6, 21);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  const bool go = !(pr.early || (!pr.sure && ratio < thr) || n < 66);
  if (!go) return res;
  FM_TRACE_S(6, 22);
  const LzPassOut em = fm_pass<false, POS, WT>(in, n, hashlog, tl, out, n, B, clevel);
  FM_TRACE_S(6, 23);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

}  // namespace b2h
