// b2h_lz.h -- wave-cooperative BloscLZ encoder/decoder for gfx950 (device code).
//
// Encoder ("exact mode"): one wave64 owns one stream and reproduces blosclz_compress
// (blosc/blosclz.c:422-619, probe get_cratio 320-419) byte for byte.  The greedy parse is
// inherently serial, so the wave advances through the stream in WINDOWS of up to 64 positions:
//   * every lane hashes its own position and reads the hash table (LDS).  The value is the serial
//     loop's candidate for every lane below W, the first lane whose hash bucket already occurs at
//     an earlier lane of the window (found exactly with one LDS atomic-or per lane on a
//     one-bit-per-bucket table).
//   * every lane tests its candidate (a 60-byte compare) and decides literal / match exactly as
//     the serial loop would; `__ballot` yields the accepted-match mask.
//   * a short scalar chain walk picks the matches the serial loop takes (first accepted lane,
//     then the first accepted lane at or after that match's end + 2, ...) while they stay below
//     W -- the lanes after a match still hold their exact candidates because every position
//     inserted inside the window (literals, anchors, in-window rehash points) owns a distinct
//     bucket.  Matches longer than the up-front compare are extended cooperatively, 1 KiB per
//     step (64 lanes x 16 bytes).
//   * all tokens of the window are then emitted at once: per-lane output sizes (literal bytes,
//     32-literal run markers, match tokens) go through one DPP prefix sum, every lane writes its
//     bytes to an LDS output ring, and run headers are patched in a second write.
//   * the window's hash inserts are one LDS store per visited lane, then the out-of-window
//     rehash (if any) exactly in the serial order.
//
// The encoder runs with maxout = neblock and records `peak`, the largest `op + k` bound check the
// reference would have made.  A smaller maxout' (the serial reference's `destsize - ntbytes`,
// blosc/blosc2.c:1343-1350) then yields the same bytes iff peak <= maxout', else 0 -- so the chunk
// finaliser reproduces the serial layout without re-encoding.
//
// Decoder: one wave per stream, token cursor uniform across the wave, literal runs and matches
// copied by 64 lanes (overlapping matches replicate their period), same rejections as
// blosclz_decompress (blosc/blosclz.c:685-795).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "b2h_format.h"

namespace b2h {

constexpr int kOutRing = 2048;      // encoder output staging ring (LDS), flushed in 512 B pieces
// LDS per encoder wave: hash table + bucket bitset + output ring = 36 KiB for 64 KiB streams
// (4 waves per CU).  Layout: [htab: POS << hashlog][bits: 2^hashlog / 8][ring: kOutRing].
__host__ __device__ constexpr size_t enc_bits_offset(size_t pos_bytes, int hashlog) { return pos_bytes << hashlog; }
__host__ __device__ constexpr size_t enc_ring_offset(size_t pos_bytes, int hashlog) {
  return (pos_bytes << hashlog) + ((size_t(1) << hashlog) >> 3);
}
__host__ __device__ constexpr size_t enc_lds_bytes(size_t pos_bytes, int hashlog) {
  return enc_ring_offset(pos_bytes, hashlog) + kOutRing;
}

// Explicit address spaces: generic (flat) pointers would turn every access into a flat_* op,
// which couples vmcnt and lgkmcnt waits and serialises LDS behind global traffic.
#define B2H_LDS __attribute__((address_space(3)))
#define B2H_GLB __attribute__((address_space(1)))
typedef const B2H_GLB uint8_t* gin_t;
typedef B2H_GLB uint8_t* gout_t;

__device__ __forceinline__ uint32_t lz_hash(uint32_t seq, int hashlog) { return (seq * 2654435761u) >> (32 - hashlog); }

__device__ __forceinline__ const B2H_GLB uint32_t* align4(gin_t p) {
  return reinterpret_cast<const B2H_GLB uint32_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(3));
}
__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t sh_bytes) {
  return __builtin_amdgcn_alignbyte(hi, lo, sh_bytes);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// ---------------------------------------------------------------- plain / write-through stores ----
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(gout_t base) {
  const uint64_t a = reinterpret_cast<uintptr_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff,
                                           0x00020000);
}
template <bool WT>
__device__ __forceinline__ void st16(gout_t base, __amdgpu_buffer_rsrc_t r, int32_t off, u32x4 v) {
  if constexpr (WT) __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
  else *reinterpret_cast<B2H_GLB u32x4*>(base + off) = v;
}
template <bool WT>
__device__ __forceinline__ void st8(gout_t base, __amdgpu_buffer_rsrc_t r, int32_t off, uint8_t v) {
  if constexpr (WT) __builtin_amdgcn_raw_buffer_store_b8(v, r, off, 0, 16);
  else base[off] = v;
}

// Output ring -> global bytes [F, to) of `out` (one wave).  16-byte stores (the ring index of a
// byte is its output offset mod kOutRing, so a 16-aligned output offset is a 16-aligned ring
// offset when `out` is 16-aligned), bytes at the ends; WT: write-through (`sc1`) stores, for
// streams another workgroup copies inside the same launch (k_encode_fast_fused).
template <bool WT, int32_t RING = kOutRing>
__device__ __forceinline__ void ring_flush_n(gout_t out, const B2H_LDS uint8_t* oring, int32_t F, int32_t to) {
  constexpr int32_t ORM = RING - 1;
  const int lane = lane_id();
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(out);
  if ((reinterpret_cast<uintptr_t>(out) & 15) != 0 || to - F < 32) {
    for (int32_t y = F + lane; y < to; y += 64) st8<WT>(out, r, y, oring[y & ORM]);
    return;
  }
  const int32_t a = (F + 15) & ~15, b = to & ~15;
  if (lane < a - F) st8<WT>(out, r, F + lane, oring[(F + lane) & ORM]);
  if (lane < to - b) st8<WT>(out, r, b + lane, oring[(b + lane) & ORM]);
  for (int32_t y = a + 16 * lane; y < b; y += 1024)
    st16<WT>(out, r, y, *reinterpret_cast<const B2H_LDS u32x4*>(oring + (y & ORM)));
}
template <bool WT>
__device__ __forceinline__ void ring_flush(gout_t out, const B2H_LDS uint8_t* oring, int32_t F, int32_t to) {
  ring_flush_n<WT, kOutRing>(out, oring, F, to);
}


// Unaligned little-endian u32 from global memory: two aligned dword loads + funnel shift.
// Callers guarantee 8 readable bytes past p & ~3 (buffers carry slack).
__device__ __forceinline__ uint32_t ldu32(gin_t p) {
  const B2H_GLB uint32_t* q = align4(p);
  return funnel(q[0], q[1], (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3));
}

// 12 unaligned bytes as three words from one 16-byte aligned-to-4 window (4 dword loads).
__device__ __forceinline__ void ld12(gin_t p, uint32_t& w0, uint32_t& w1, uint32_t& w2) {
  const B2H_GLB uint32_t* q = align4(p);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t a = q[0], b = q[1], c = q[2], d = q[3];
  w0 = funnel(a, b, sh);
  w1 = funnel(b, c, sh);
  w2 = funnel(c, d, sh);
}

// 16 unaligned bytes as four words (5 dword loads).
__device__ __forceinline__ void ld16(gin_t p, uint32_t (&w)[4]) {
  const B2H_GLB uint32_t* q = align4(p);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  const uint32_t a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  w[0] = funnel(a, b, sh);
  w[1] = funnel(b, c, sh);
  w[2] = funnel(c, d, sh);
  w[3] = funnel(d, e, sh);
}

// 4N unaligned bytes as N words (N + 1 dword loads).
template <int N>
__device__ __forceinline__ void ldw(gin_t p, uint32_t (&w)[N]) {
  const B2H_GLB uint32_t* q = align4(p);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
  uint32_t d[N + 1];
#pragma unroll
  for (int i = 0; i < N + 1; i++) d[i] = q[i];
#pragma unroll
  for (int i = 0; i < N; i++) w[i] = funnel(d[i], d[i + 1], sh);
}
// Exact mode's up-front compare: kExWords words per lane and candidate.  60 bytes (15 words): a
// match the compare does not end needs a cooperative extension through memory (one round trip);
// with 28 bytes that was half of T's matches.  The wave can afford the registers: the encoder's
// workgroup shape is LDS-bound at 3 waves per SIMD (k_encode's waves_per_eu).
constexpr int kExWords = 15, kExBytes = 4 * kExWords;


__device__ __forceinline__ int32_t rdlane(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// Wave64 inclusive scans with DPP (row shifts inside 16-lane rows, then row broadcasts 15/31).
// Lanes whose DPP source is masked or out of row read the identity of the operation.
__device__ __forceinline__ int32_t wave_scan_add(int32_t v) {
  int32_t r = v;
  r += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  r += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  r += __builtin_amdgcn_update_dpp(0, v, 0x113, 0xf, 0xf, false);   // row_shr:3
  r += __builtin_amdgcn_update_dpp(0, r, 0x114, 0xf, 0xe, false);   // row_shr:4, banks 1-3
  r += __builtin_amdgcn_update_dpp(0, r, 0x118, 0xf, 0xc, false);   // row_shr:8, banks 2-3
  r += __builtin_amdgcn_update_dpp(0, r, 0x142, 0xa, 0xf, false);   // row_bcast:15, rows 1,3
  r += __builtin_amdgcn_update_dpp(0, r, 0x143, 0xc, 0xf, false);   // row_bcast:31, rows 2,3
  return r;
}
__device__ __forceinline__ int32_t wave_scan_max(int32_t v) {   // values >= -1
  int32_t r = v;
  r = max(r, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, v, 0x113, 0xf, 0xf, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, r, 0x114, 0xf, 0xe, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, r, 0x118, 0xf, 0xc, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, r, 0x142, 0xa, 0xf, false));
  r = max(r, __builtin_amdgcn_update_dpp(-1, r, 0x143, 0xc, 0xf, false));
  return r;
}

// The encoder's hash table (one per wave): in LDS, or in global memory.  LDS holds a 64 KiB
// stream's table (32 KiB) for only 4 waves per CU, one per SIMD, and a lone wave leaves its SIMD
// idle while it waits on memory; with the table in global memory a wave needs 4 KiB of LDS (bucket
// bitset + output ring) and 4 waves share each SIMD.  Global tables are accessed at workgroup
// scope: the table is private to the wave, and at agent scope the accesses bypass the XCD's L2
// (a lane then need not see what another lane stored in the previous window).
template <typename POS>
struct LdsTab {
  typedef POS pos_t;
  static constexpr bool kGlobal = false;
  volatile B2H_LDS POS* t;
  __device__ __forceinline__ uint32_t get(uint32_t h) const { return t[h]; }
  __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { t[h] = (POS)v; }
  __device__ __forceinline__ void clear(int hashlog) const {   // 8-byte LDS stores
    B2H_LDS uint64_t* h8 = (B2H_LDS uint64_t*)(t);
    const int32_t n8 = (int32_t)((sizeof(POS) << hashlog) / 8);
    for (int32_t i = lane_id(); i < n8; i += 64) h8[i] = 0;
  }
};
template <typename POS>
struct GlbTab {
  typedef POS pos_t;
  static constexpr bool kGlobal = true;
  B2H_GLB POS* t;
  __device__ __forceinline__ uint32_t get(uint32_t h) const {
    return __hip_atomic_load(t + h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
    __hip_atomic_store(t + h, (POS)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __device__ __forceinline__ void clear(int hashlog) const {   // 16-byte stores; they complete
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));   // before the first window's loads
    B2H_GLB u32x4* t16 = (B2H_GLB u32x4*)(t);
    const int32_t n16 = (int32_t)((sizeof(POS) << hashlog) / 16);
    const u32x4 z = {0u, 0u, 0u, 0u};
    for (int32_t i = lane_id(); i < n16; i += 64) t16[i] = z;
  }
};

// End of the common prefix of in[x..] and in[x-d..], one past the first mismatch, capped at
// `bound` (get_match / get_run semantics, blosc/blosclz.c:119-165).  64 lanes x 16 bytes per step.
#ifndef B2H_MATCH_U
#define B2H_MATCH_U 4   // 1 KiB sub-steps per round trip of a long match's extension
#endif
template <int U = B2H_MATCH_U>
__device__ __forceinline__ int32_t wave_match_end(gin_t in, int32_t x, uint32_t d, int32_t bound) {
  const int lane = lane_id();
  // first mismatch in 16 bytes at q (16: none; bytes at and after `bound` do not count)
  auto first16 = [&](int32_t q, const uint32_t (&a)[4], const uint32_t (&b)[4]) {
    int32_t first = 16;
    const int32_t nb = bound - q;
#pragma unroll
    for (int k = 3; k >= 0; k--) {
      uint32_t diff = a[k] ^ b[k];
      const int32_t lo = 4 * k;
      if (nb <= lo) diff = 0;
      else if (nb < lo + 4) diff &= (1u << (8 * (nb - lo))) - 1u;
      if (diff) first = lo + (__builtin_ctz(diff) >> 3);
    }
    return q < bound ? first : 16;
  };
  // 1 KiB per step first (most extensions end there); a match still running after it moves to
  // 4 KiB steps with every lane's four 16-byte pairs in flight at once -- a step is one memory
  // round trip, and long runs of repeats (C4's delta planes: one match per 64 KiB stream) would
  // otherwise pay 64 of them per stream
  if (x < bound) {
    const int32_t q = x + lane * 16;
    uint32_t a[4] = {0, 0, 0, 0}, b[4] = {0, 0, 0, 0};
    if (q < bound) { ld16(in + q, a); ld16(in + q - d, b); }
    const int32_t first = first16(q, a, b);
    const uint64_t mm = __ballot(first < 16);
    if (mm) {
      const int l = __builtin_ctzll(mm);
      return x + l * 16 + rdlane(first, l) + 1;
    }
    x += 1024;
  }
  while (x < bound) {
    uint32_t a[U][4], b[U][4];
    // unconditional loads (a lane past `bound` reads the step's first bytes instead, which
    // first16 ignores): a branch around each slice's loads had the compiler drain every slice
    // before the next one's issue -- U round trips per step instead of one
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t q = x + u * 1024 + lane * 16;
      const int32_t ql = q < bound ? q : x;
      ld16(in + ql, a[u]);
      ld16(in + ql - d, b[u]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t q = x + u * 1024 + lane * 16;
      const int32_t first = first16(q, a[u], b[u]);
      const uint64_t mm = __ballot(first < 16);
      if (mm) {
        const int l = __builtin_ctzll(mm);
        return x + u * 1024 + l * 16 + rdlane(first, l) + 1;
      }
    }
    x += U * 1024;
  }
  return bound;
}

struct LzPassOut {
  int32_t o;       // bytes emitted (emit) / counted (probe)
  int32_t pos;     // final parse position (probe ratio numerator)
  int32_t peak;
  bool fail;
  bool early;      // probe stopped once its ratio could no longer reach the threshold
  bool sure;       // probe stopped once its ratio could no longer fall below the threshold
  int32_t windows;
};

#ifdef B2H_ENC_PROF   // diagnostics build only (tools/enc_micro.hip): per-phase s_memtime sums
__device__ uint64_t g_enc_prof[16];
#define EPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define EPROF_USE(x) asm volatile("" :: "v"(x))
#define EPROF_DECL uint64_t eprof[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define EPROF_ADD(i, a, b) eprof[i] += (b) - (a)
#define EPROF_FLUSH                                                                            \
  if (lane == 0)                                                                               \
    for (int i_ = 0; i_ < 8; i_++) atomicAdd((unsigned long long*)&g_enc_prof[(PROBE ? 8 : 0) + i_], eprof[i_])
#else
#define EPROF_T(v)
#define EPROF_USE(x)
#define EPROF_DECL
#define EPROF_ADD(i, a, b)
#define EPROF_FLUSH
#endif

// One greedy parse.  PROBE: get_cratio (counts only, limit = min(length, 2^hashlog), no far
// short-match rule, no clevel-9 double rehash, no tail).  !PROBE: the emitting main loop + tail.
template <bool PROBE, typename TAB, bool WT = false>
__device__ __forceinline__ LzPassOut lz_pass(gin_t __restrict__ in, int32_t length, int hashlog, int clevel, gout_t __restrict__ out,
                                             int32_t maxout, TAB htab, B2H_LDS uint32_t* dbits,
                                             B2H_LDS uint8_t* oring) {
  const int lane = lane_id();
  // u16 positions (streams <= 64 KiB): kExWords; u32 (C3's 256 KiB streams): 28 bytes measured
  // faster there (the longer compare: C3 exact compress 27.4 -> 28.1 ms)
  constexpr int NW = sizeof(typename TAB::pos_t) == 2 ? kExWords : 7, NB = 4 * NW;
  // Output bytes are staged in an LDS ring and leave for `out` in 512-byte pieces once they are
  // final: global stores share vmcnt with loads on CDNA, so a byte store per token would make
  // every following input load wait for the store round trip.
  constexpr int32_t ORM = kOutRing - 1;
  int32_t F = 0;   // output [0, F) already in `out`
  auto flush = [&](int32_t to) {
    ring_flush<WT>(out, oring, F, to);
    F = to;
  };
  int32_t limit = length;
  if (PROBE) {
    const int32_t hl = 1 << hashlog;
    limit = length > hl ? hl : length;
  }
  const int32_t bound = limit - 1, loop_end = limit - 12;
  {  // clear the hash table and the bucket bitset
    htab.clear(hashlog);
    for (int32_t i = lane; i < (1 << hashlog) / 32; i += 64) dbits[i] = 0u;
    // the clear goes through a wider view: keep the compiler from sinking it below the
    // (differently typed) table reads that follow
    asm volatile("" ::: "memory");
  }
  // clevel 9 rehashes a second, differently hashed position after every match: keep one match
  // per window there so the insert order stays trivially serial
  const bool multi = PROBE || clevel != 9;
  LzPassOut r;
  int32_t windows = 0;
  int32_t o = 5, lit = 4, pos;
  uint32_t byte0 = kLzMaxCopy - 1;   // out[0] is patched at the end (marker bit)
  if (PROBE) {
    pos = 0;
  } else {
    pos = 4;
    if (lane < 5) {   // marker + four literals; the load index never negative (in[-1] lies outside the image)
      const uint8_t b = in[lane > 0 ? lane - 1 : 0];
      oring[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : b;
    }
  }
  int32_t peak = 0;
  bool fail = false;
  EPROF_DECL;

  // probe early exit: the final ratio is pos / o with pos <= limit + 2 and o never decreasing in
  // the probe, so once (limit + 64) / o < threshold (with margin) the stream is incompressible
  // whatever the rest of the probe finds (blosc/blosclz.c:463-468 decides on that ratio alone)
  const double thr_o = PROBE ? 0.999 * (clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2
                                        : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0) : 0.0;
  bool early = false, sure = false;
  // and the converse: the probe ends at pos >= loop_end, and the R positions left add at most
  // R + R/32 + 1 to o as literals (LITERAL2 of blosclz.c), less as matches (a match of len >= 4
  // consumes len + 2 positions for at most 5 + (len - 7)/255 + 1 bytes) except one final match
  // running past loop_end (at most 7 + (R + 12)/255): so once loop_end / (o + R + R/16 + 16) >=
  // threshold the stream is compressed whatever the rest of the probe finds
  const double thr_s = thr_o * (1.001 / 0.999);
  while (pos < loop_end) {
    if (PROBE) {
      if ((double)(limit + 64) < thr_o * (double)o) { early = true; break; }
      const int32_t R = loop_end - pos;
      if ((double)loop_end >= thr_s * (double)(o + R + R / 16 + 16)) { sure = true; break; }
    }
    windows++;
    if (!PROBE && o - F >= 1024) flush(F + 512);   // a window emits < 512 bytes
    EPROF_T(t0);
    const int32_t P = pos;
    const int32_t p = P + lane;
    const bool valid = p < loop_end;
    uint32_t a[NW] = {};   // in[p .. p + NB - 1]
    if (valid) ldw<NW>(in + p, a);
    const uint32_t v = a[0];
    EPROF_T(t1);
    const uint32_t h = lz_hash(v, hashlog);
    const uint32_t c0 = valid ? htab.get(h) : 0u;
    // W: first lane whose bucket already occurs at an earlier lane of the window.  One atomic-or
    // per lane on a bit-per-bucket table: the lanes that find their bit set are the repeats (LDS
    // applies the lanes of one instruction in lane order; any other order would only flag an
    // earlier lane of a repeated bucket -- a shorter window, still exact below W).  The words are
    // cleared right after: every bit set in them belongs to this window.
    uint32_t old = 0;
    if (valid) {
      old = __hip_atomic_fetch_or(&dbits[h >> 5], 1u << (h & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      dbits[h >> 5] = 0u;
    }
    const bool rep = valid && ((old >> (h & 31)) & 1u);
    // A lane whose left neighbour has the same hash (runs, short periods) knows its serial
    // candidate exactly: the neighbour, inserted just before it.  Other repeats end the window.
    const uint32_t hprev = (uint32_t)__shfl_up((int)h, 1);
    const bool same1 = valid && lane > 0 && hprev == h;
    const uint64_t s1mask = __ballot(same1);
    const uint64_t dup = __ballot(rep && !same1);
    int32_t W = dup ? __builtin_ctzll(dup) : 64;
    W = max(1, min(W, loop_end - P));   // lane 0's candidate is always exact
    EPROF_T(t2);

    // candidate test (lanes < W): literal or match, exactly as the serial loop decides
    const uint32_t cand = same1 ? (uint32_t)(p - 1) : c0;
    const uint32_t dist = (uint32_t)(p - (int32_t)cand);
    // NB bytes are compared up front; only longer matches need the cooperative extension
    bool accept = false;
    int32_t lenx = 0;   // match length, or -1: the first NB bytes all match (extend later)
    if (lane < W && dist != 0 && dist < kLzFar) {
      uint32_t rr[NW];
      ldw<NW>(in + cand, rr);
      if (rr[0] == v) {
        int32_t mm = NB;   // index of the first mismatching byte
#pragma unroll
        for (int i = NW - 1; i >= 1; i--) {
          const uint32_t x = a[i] ^ rr[i];
          if (x) mm = 4 * i + (__builtin_ctz(x) >> 3);
        }
        const int32_t e = min(mm < NB ? p + mm + 1 : 0x7fffffff, bound);
        const int32_t len = e - 4 - p;
        accept = len >= 4 && (PROBE || !(len <= 5 && (dist - 1) >= kLzNear));
        lenx = (mm < NB || p + NB + 1 >= bound) ? len : -1;
      }
    }
    const uint64_t am = __ballot(accept);
    EPROF_T(t3);

    if (PROBE && am == 0) {
      // ---- all-literal probe window (no match below W): the counting below in closed form ----
      // literal k of the window lands at o + k + (lit + k) / 32 (a run marker after every 32nd)
      if (!PROBE) {
        const int32_t last = o + (W - 1) + (lit + W - 1) / 32;
        peak = max(peak, last + 2);
        if (last + 2 > maxout) { fail = true; break; }
        if (lane < W) {
          const int32_t off = o + lane + (lit + lane) / 32;
          oring[off & ORM] = (uint8_t)(v & 0xffu);
          if (((lit + lane + 1) & 31) == 0) oring[(off + 1) & ORM] = (uint8_t)(kLzMaxCopy - 1);
        }
      }
      o += W + (lit + W) / 32;
      lit = (lit + W) & 31;
      {  // every lane below W is a visited literal (same run rule as the general insert below)
        const uint64_t visit = W >= 64 ? ~0ull : ((1ull << W) - 1ull);
        const uint64_t above = ~0ull << lane << 1;
        const uint64_t brk = ~s1mask & above;
        const uint64_t run = brk ? (above & ((1ull << __builtin_ctzll(brk)) - 1)) : above;
        if (((visit >> lane) & 1ull) && !(visit & run)) htab.put(h, (uint32_t)p);
      }
      EPROF_ADD(0, t0, t1);
      EPROF_ADD(1, t1, t2);
      EPROF_ADD(2, t2, t3);
      pos = P + W;
      continue;
    }

    // ---- chain walk: the matches the serial loop takes in this window ----
    uint64_t chain = 0;
    int32_t E = W;        // the window consumes positions P .. P+E-1 (E > 64 after a long match)
    int32_t ser = -1;     // a match with length-extension bytes, emitted by the scalar path below
    int32_t lastc2 = -1;  // end + 2 of the chain match that closes the window
    {
      uint64_t rem = am;
      while (rem) {
        const int32_t m = __builtin_ctzll(rem);
        int32_t lm = rdlane(lenx, m);
        if (lm < 0) {
          EPROF_T(te0);
          lm = wave_match_end(in, P + m + NB, (uint32_t)rdlane((int32_t)dist, m), bound) - 4 - (P + m);
          lenx = lane == m ? lm : lenx;
          EPROF_T(te1);
          EPROF_ADD(5, te0, te1);
        }
        if (lm >= 262) { ser = m; E = m; break; }   // (len - 7) / 255 extension bytes
        chain |= 1ull << m;
        const int32_t c2 = m + lm + 2;   // the serial loop resumes at the match end + 2
        // it stays in this window while the lane there holds an exact candidate: below W, and
        // not a left-neighbour candidate whose neighbour (end + 1) the match skipped
        if (!multi || c2 >= W || ((s1mask >> c2) & 1ull)) { E = c2; lastc2 = c2; break; }
        rem = am & (~0ull << c2);
      }
    }
    EPROF_T(t4);

    // ---- all tokens of the window at once ----
    // owner: the last chain match at or before the lane; prev: the last one strictly before
    const bool ischain = (chain >> lane) & 1ull;
    const int32_t own = wave_scan_max(ischain ? lane : -1);
    int32_t prev = __shfl_up(own, 1);
    if (lane == 0) prev = -1;
    const int32_t c2v = lane + lenx + 2;                        // chain lanes: where the walk resumes
    const int32_t pc2 = __shfl(c2v, prev < 0 ? 0 : prev);
    const int32_t segstart = prev >= 0 ? pc2 : 0;               // first lane after prev's match
    const int32_t lpos = (prev >= 0 ? 0 : lit) + lane - segstart;   // literals of the run before the lane
    const bool islit = !ischain && lane >= segstart && lane < min(E, W);
    const int32_t rr5 = lpos & 31;   // 32-literal runs: the run restarts after every marker
    const uint32_t bd = dist - 1;    // biased distance
    const bool near = bd < kLzNear;
    const uint32_t ulen = (uint32_t)lenx;
    const int32_t tok = ulen < 7 ? (near ? 2 : 4) : (near ? 3 : 5);   // no extension bytes here
    // output bytes per lane: a literal (+ the marker opening the next run after its 32nd), or a
    // match token + the marker opening the next run (- the pending marker it overwrites when no
    // literal precedes it)
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
        const int32_t ts = base - (rr5 == 0 ? 1 : 0);   // chain lanes: first token byte
        // every bound check grows with the output position: the window's last element makes
        // the largest (a literal checks op + 2, a match op + token + 1)
        const int32_t req = lelit ? rdlane(base, le) + 2 : rdlane(ts + tok + 1, le);
        peak = max(peak, req);
        if (req > maxout) { fail = true; break; }
        const bool nextchain = lane < 63 && ((chain >> (lane + 1)) & 1ull);
        if (islit) {
          oring[base & ORM] = (uint8_t)(v & 0xffu);
          // the marker after a 32nd literal is overwritten by a match right behind it
          if (rr5 == 31 && !nextchain) oring[(base + 1) & ORM] = (uint8_t)(kLzMaxCopy - 1);
        }
        if (ischain) {
          // token bytes + the marker that opens the next literal run, little-endian in a u64
          const uint32_t fd = bd - kLzNear;
          uint64_t tb;
          int32_t nb;
          if (ulen < 7) {
            if (near) { tb = (uint64_t)((ulen << 5) + (bd >> 8)) | ((uint64_t)(bd & 255) << 8) | (31ull << 16); nb = 3; }
            else { tb = (uint64_t)((ulen << 5) + 31) | (255ull << 8) | ((uint64_t)(fd >> 8) << 16) | ((uint64_t)(fd & 255) << 24) | (31ull << 32); nb = 5; }
          } else {
            const uint64_t rl = ulen - 7;
            if (near) { tb = (uint64_t)((7u << 5) + (bd >> 8)) | (rl << 8) | ((uint64_t)(bd & 255) << 16) | (31ull << 24); nb = 4; }
            else { tb = (uint64_t)((7u << 5) + 31) | (rl << 8) | (255ull << 16) | ((uint64_t)(fd >> 8) << 24) | ((uint64_t)(fd & 255) << 32) | (31ull << 40); nb = 6; }
          }
          if (c2v < 64 && ((chain >> c2v) & 1ull)) nb--;   // the next match overwrites the marker
#pragma unroll
          for (int i = 0; i < 6; i++)
            if (i < nb) oring[(ts + i) & ORM] = (uint8_t)(tb >> (8 * i));
        }
        // run headers closed by a match, after every byte of the window is in place
        if (ischain && rr5 > 0) oring[(ts - rr5 - 1) & ORM] = (uint8_t)(rr5 - 1);
        const uint64_t z = __ballot(ischain && rr5 > 0 && ts - rr5 - 1 == 0);
        if (z) byte0 = (uint32_t)(rdlane(rr5, __builtin_ctzll(z)) - 1);
      }
      lit = lelit ? ((rdlane(lpos, le) + 1) & 31) : 0;
    }
    o += rdlane(incl, 63);

    // visited positions: literals, match anchors, in-window rehash points (match end)
    uint64_t visit = elems | __ballot(!ischain && prev >= 0 && lane == pc2 - 2 && lane < W && multi);
    bool rehash_out = false;
    int32_t rq = 0;
    if (lastc2 >= 0 && (lastc2 - 2 >= W || !multi)) {
      rehash_out = true;
      rq = P + lastc2 - 2;
    }

    // ---- a match with extension bytes: the scalar token path ----
    if (ser >= 0) {
      visit |= 1ull << ser;
      const uint32_t dm = (uint32_t)rdlane((int32_t)dist, ser);
      const int32_t lm = rdlane(lenx, ser);
      const uint32_t sbd = dm - 1;
      const uint32_t sulen = (uint32_t)lm;
      const bool snear = sbd < kLzNear;
      int32_t at = -1;   // header of the literal run this match closes
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
          // a match of n bytes carries (n - 7) / 255 extension bytes (~2 KiB for a 512 KiB
          // stream): stream them through the ring in 512-byte slices
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
      o += stok + 1;   // token + the literal marker after it
      const int32_t ql = ser + lm;   // the match end, relative to P
      if (ql < W && multi) {
        visit |= 1ull << ql;         // lane ql holds hash(ld32(in + q)) already
      } else {
        rehash_out = true;
        rq = P + ql;
      }
      E = ql + 2;
    }
    if (fail) break;
    EPROF_T(t5);
    uint32_t rseq = 0;
    if (rehash_out) {
      // the four bytes at the match end: from the lane that loaded them, else from memory
      const int32_t ql = rq - P;
      rseq = (ql < 64 && rq < loop_end) ? (uint32_t)rdlane((int32_t)v, ql) : ldu32(in + rq);
    }
    // Below W a bucket repeats only inside a run of equal hashes (left-neighbour lanes); the
    // serial loop leaves the run's last visited position in it, so only that lane stores (in one
    // store instruction the surviving lane of a shared address is not specified).
    {
      const uint64_t above = ~0ull << lane << 1;                       // lanes > lane
      const uint64_t brk = ~s1mask & above;                            // lanes that start a new run
      const uint64_t run = brk ? (above & ((1ull << __builtin_ctzll(brk)) - 1)) : above;
      if (((visit >> lane) & 1ull) && !(visit & run)) htab.put(h, (uint32_t)p);
    }
    if (rehash_out && lane == 0) {
      htab.put(lz_hash(rseq, hashlog), (uint32_t)rq);
      if (!PROBE && clevel == 9) htab.put(lz_hash(rseq >> 8, hashlog), (uint32_t)(rq + 1));
    }
    EPROF_T(t6);
    EPROF_ADD(0, t0, t1);
    EPROF_ADD(1, t1, t2);
    EPROF_ADD(2, t2, t3);
    EPROF_ADD(3, t3, t4);
    EPROF_ADD(4, t4, t5);
    EPROF_ADD(6, t5, t6);
    pos = P + E;
  }

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
        if (lane == 0) st8<WT>(out, wt_rsrc(out), 0, (uint8_t)(byte0 | 0x20u));
      }
    }
  }
  EPROF_FLUSH;
  r.o = o;
  r.pos = pos;
  r.peak = peak;
  r.fail = fail;
  r.early = early;
  r.sure = sure;
  r.windows = windows;
  return r;
}

// Whether s[from, n) is all `first`: 4 KiB per step (64 lanes x 4 x 16 B).  A whole aligned step
// issues its four slices' loads unconditionally -- one round trip; under a branch per slice the
// compiler drained each slice before the next one's issue (four round trips per step)
__device__ __forceinline__ bool wave_run_span(gin_t s, int32_t from, int32_t n, uint8_t first) {
  const int lane = lane_id();
  const uint32_t rep = first * 0x01010101u;
  const bool aligned = (reinterpret_cast<uintptr_t>(s + from) & 15) == 0;
  for (int32_t base = from; base < n; base += 64 * 64) {
    bool bad = false;
    if (aligned && base + 64 * 64 <= n) {
      u32x4 w[4];
#pragma unroll
      for (int u = 0; u < 4; u++) w[u] = *reinterpret_cast<const B2H_GLB u32x4*>(s + base + (u * 64 + lane) * 16);
#pragma unroll
      for (int u = 0; u < 4; u++) bad |= (w[u].x != rep) | (w[u].y != rep) | (w[u].z != rep) | (w[u].w != rep);
    } else {
#pragma unroll
      for (int u = 0; u < 4; u++) {
        const int32_t i = base + (u * 64 + lane) * 16;
        if (aligned && i + 16 <= n) {
          const B2H_GLB uint32_t* w = reinterpret_cast<const B2H_GLB uint32_t*>(s + i);
          bad |= (w[0] != rep) | (w[1] != rep) | (w[2] != rep) | (w[3] != rep);
        } else {
          for (int32_t k = i; k < min(i + 16, n); k++) bad |= s[k] != first;
        }
      }
    }
    if (__ballot(bad)) return false;
  }
  return true;
}
// Is the whole stream one repeated byte? (blosc/blosc2.c:1184-1206)
__device__ __forceinline__ bool wave_is_run(gin_t s, int32_t n) { return wave_run_span(s, 0, n, s[0]); }
// Whether s[from, n) is all `first` (the second half of a split run test).
__device__ __forceinline__ bool wave_is_run_from(gin_t s, int32_t from, int32_t n, uint8_t first) {
  return wave_run_span(s, from, n, first);
}

// Full per-stream encode with maxout = neblock: run test, entropy probe, main pass.
template <typename TAB, bool WT = false>
__device__ __forceinline__ StreamResult encode_stream(gin_t __restrict__ in, int32_t n, int clevel, gout_t __restrict__ out,
                                                      TAB htab, B2H_LDS uint32_t* dbits,
                                                      B2H_LDS uint8_t* oring, bool allow_runs) {
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
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  const LzPassOut pr = lz_pass<true, TAB, WT>(in + (n - maxlen), maxlen, hashlog, clevel, out, 0, htab, dbits, oring);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  // cratio_ thresholds of blosc/blosclz.c:465 (compared in double, as the reference does)
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (pr.early || (!pr.sure && ratio < thr) || n < 16 || n < 66) return res;
  const LzPassOut em = lz_pass<false, TAB, WT>(in, n, hashlog, clevel, out, n, htab, dbits, oring);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

// ------------------------------------------------------------------ wave fills and copies ----
// Output stores, plain or write-through (WT: `sc1` buffer stores, MI355X_MICROARCH.md
// § inter-workgroup visibility, R1 payload).  The decoder writes its output write-through so the
// wave that completes a block can hand the block's planes to its own unshuffle inside the launch:
// every stream's bytes are in memory once its wave has drained them (vmcnt(0)), whichever XCD wrote
// them.  The descriptor is built from the wave-uniform base (no waterfall loops).
template <bool WT = false>
__device__ __forceinline__ void wave_fill(gout_t o, uint8_t v, int32_t n) {
  const int lane = lane_id();
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(o);
  const int32_t head = (int32_t)((16 - (reinterpret_cast<uintptr_t>(o) & 15)) & 15);
  const int32_t h = min(head, n);
  if (lane < h) st8<WT>(o, r, lane, v);
  const uint32_t w = v * 0x01010101u;
  const u32x4 w4 = {w, w, w, w};
  const int32_t n16 = (n - h) / 16;
  for (int32_t i = lane; i < n16; i += 64) st16<WT>(o, r, h + 16 * i, w4);
  for (int32_t i = h + n16 * 16 + lane; i < n; i += 64) st8<WT>(o, r, i, v);
}

// dst any alignment: 16-byte aligned stores of 16 funnel-shifted source bytes per lane, four
// 1 KiB rows in flight per step (the source is read with aligned dwords: never past the last
// dword that holds a source byte).
// NT: non-temporal loads and stores (a copy running beside latency-bound kernels: keeps their L2
// lines)
template <bool WT = false, bool NT = false>
__device__ __forceinline__ void wave_copy(gout_t o, gin_t s, int32_t n) {
  const int lane = lane_id();
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(o);
  const int32_t head = (int32_t)((16 - (reinterpret_cast<uintptr_t>(o) & 15)) & 15);
  const int32_t h = min(head, n);
  if (lane < h) st8<WT>(o, r, lane, s[lane]);
  const int32_t n16 = (n - h) / 16;
  gin_t s1 = s + h;
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(s1) & 3);
  const B2H_GLB uint32_t* q0 = align4(s1);
  // the 5th dword of the last 16-byte piece exists only if the source is misaligned
  int32_t i = lane;
  for (; i + 192 < n16; i += 256) {
    uint32_t w[4][5];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const B2H_GLB uint32_t* q = q0 + 4 * (i + 64 * u);
#pragma unroll
      for (int k = 0; k < 4; k++) w[u][k] = NT ? __builtin_nontemporal_load(q + k) : q[k];
      w[u][4] = sh ? (NT ? __builtin_nontemporal_load(q + 4) : q[4]) : 0u;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      u32x4 v;
      v.x = funnel(w[u][0], w[u][1], sh);
      v.y = funnel(w[u][1], w[u][2], sh);
      v.z = funnel(w[u][2], w[u][3], sh);
      v.w = funnel(w[u][3], w[u][4], sh);
      if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<B2H_GLB u32x4*>(o + h + 16 * (i + 64 * u)));
      else st16<WT>(o, r, h + 16 * (i + 64 * u), v);
    }
  }
  for (; i < n16; i += 64) {
    const B2H_GLB uint32_t* q = q0 + 4 * i;
    const uint32_t a = q[0], b = q[1], c = q[2], d = q[3], e = sh ? q[4] : 0u;
    u32x4 v;
    v.x = funnel(a, b, sh);
    v.y = funnel(b, c, sh);
    v.z = funnel(c, d, sh);
    v.w = funnel(d, e, sh);
    st16<WT>(o, r, h + 16 * i, v);
  }
  for (int32_t j = h + n16 * 16 + lane; j < n; j += 64) st8<WT>(o, r, j, s[j]);
}

// n bytes from a 16-byte aligned source to a destination of any alignment, with one 16-byte load
// and one 16-byte store per lane step (wave_copy's dword loads cost 4-5x the address work, which
// slows the latency-bound encoders sharing the CU when this runs inside their launch): the piece
// a lane stores straddles its own source chunk and the next lane's, fetched with DPP wave_shl:1
// (lane 63 loads it); sources are read up to 15 bytes past their end (scratch slack).
__device__ __forceinline__ u32x4 dpp_next_lane(u32x4 v) {   // lane l gets lane l + 1's value
  u32x4 r;
  r.x = __builtin_amdgcn_update_dpp(0, (int)v.x, 0x130, 0xf, 0xf, false);
  r.y = __builtin_amdgcn_update_dpp(0, (int)v.y, 0x130, 0xf, 0xf, false);
  r.z = __builtin_amdgcn_update_dpp(0, (int)v.z, 0x130, 0xf, 0xf, false);
  r.w = __builtin_amdgcn_update_dpp(0, (int)v.w, 0x130, 0xf, 0xf, false);
  return r;
}
__device__ void wave_copy_a16(gout_t o, gin_t s, int32_t n) {
  const int lane = lane_id();
  const int32_t head = (int32_t)((16 - (reinterpret_cast<uintptr_t>(o) & 15)) & 15);
  const int32_t h = min(head, n);
  auto ld16 = [&](int32_t i) -> u32x4 { return reinterpret_cast<const B2H_GLB u32x4*>(s)[i]; };
  auto ld8 = [&](int32_t j) -> uint8_t { return s[j]; };
  if (lane < h) o[lane] = ld8(lane);
  const int32_t n16 = (n - h) / 16;
  B2H_GLB u32x4* o16 = reinterpret_cast<B2H_GLB u32x4*>(o + h);
  if (h == 0) {
    for (int32_t i = lane; i < n16; i += 64) o16[i] = ld16(i);
  } else {
    const uint32_t ds = (uint32_t)h >> 2, bs = (uint32_t)h & 3;
    for (int32_t i0 = 0; i0 < n16; i0 += 64) {
      const int32_t i = i0 + lane;
      const u32x4 a = i <= n16 ? ld16(i) : u32x4{0, 0, 0, 0};   // chunk n16 still holds source bytes
      u32x4 b = dpp_next_lane(a);
      if (lane == 63 && i + 1 <= n16) b = ld16(i + 1);
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      u32x4 v;
      // bytes [h, h + 16) of a | b: dword shift ds (wave-uniform), byte shift bs
      if (ds == 0) v = {funnel(w[0], w[1], bs), funnel(w[1], w[2], bs), funnel(w[2], w[3], bs), funnel(w[3], w[4], bs)};
      else if (ds == 1) v = {funnel(w[1], w[2], bs), funnel(w[2], w[3], bs), funnel(w[3], w[4], bs), funnel(w[4], w[5], bs)};
      else if (ds == 2) v = {funnel(w[2], w[3], bs), funnel(w[3], w[4], bs), funnel(w[4], w[5], bs), funnel(w[5], w[6], bs)};
      else v = {funnel(w[3], w[4], bs), funnel(w[4], w[5], bs), funnel(w[5], w[6], bs), funnel(w[6], w[7], bs)};
      if (i < n16) o16[i] = v;
    }
  }
  for (int32_t j = h + n16 * 16 + lane; j < n; j += 64) o[j] = ld8(j);
}

// ------------------------------------------------------------------------------- decoder ----
// Double-buffered register window over the compressed stream.  w0 holds stream bytes
// [wpos, wpos + 256) (lane l: the aligned dword at wpos + 4 l), w1 the next 256; wpos is chosen so
// that in + wpos is 4-byte aligned (it may be -1..-3).  Token bytes are read with readlane (no
// memory round trip per token), literal runs with bpermute; w1 is loaded one window ahead.
// Dwords at or past the stream end read as 0; an aligned dword holding a stream byte never
// crosses a page, so the partial first/last dwords are safe to load.
struct InWin {
  uint32_t w0, w1;
  int32_t wpos;
};

__device__ __forceinline__ uint32_t inwin_dword(gin_t in, int32_t length, int32_t pos) {
  const int32_t mine = pos + 4 * lane_id();
  return mine < length ? *reinterpret_cast<const B2H_GLB uint32_t*>(in + mine) : 0u;
}

__device__ __forceinline__ void inwin_reload(InWin& W, gin_t in, int32_t length, int32_t pos) {
  W.wpos = pos - (int32_t)(reinterpret_cast<uintptr_t>(in + pos) & 3);
  W.w0 = inwin_dword(in, length, W.wpos);
  W.w1 = inwin_dword(in, length, W.wpos + 256);
}

// Make stream offset `pos` fall inside w0; returns its offset in w0 (0..255).
__device__ __forceinline__ int32_t inwin_seek(InWin& W, gin_t in, int32_t length, int32_t pos) {
  int32_t k = pos - W.wpos;
  if (k >= 256) {
    if (k < 512) {
      W.w0 = W.w1;
      W.wpos += 256;
      W.w1 = inwin_dword(in, length, W.wpos + 256);
    } else {
      inwin_reload(W, in, length, pos);
    }
    k = pos - W.wpos;
  }
  return k;
}

// Four stream bytes starting at w0 offset k (0..255), little-endian.
__device__ __forceinline__ uint32_t inwin_peek4(const InWin& W, int32_t k) {
  const int li = k >> 2;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)W.w0, li);
  const uint32_t hi = li < 63 ? (uint32_t)__builtin_amdgcn_readlane((int)W.w0, li + 1)
                              : (uint32_t)__builtin_amdgcn_readlane((int)W.w1, 0);
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> (8 * (k & 3)));
}

__device__ __forceinline__ uint32_t inwin_byte(InWin& W, gin_t in, int32_t length, int32_t pos) {
  const int32_t k = inwin_seek(W, in, length, pos);
  return ((uint32_t)__builtin_amdgcn_readlane((int)W.w0, k >> 2) >> (8 * (k & 3))) & 0xffu;
}

// Move output bytes [from, to) of the LDS ring to global memory (positions are stream offsets;
// ring slot = position mod R).  16 B per lane when both sides are 16-byte aligned.
// The decoders' output leaves write-through (see st16): 16 B per lane where out + x is 16-byte
// aligned (whole 1 KiB rows, then the 16-byte groups of the last row), bytes elsewhere.
template <int RLOG>
__device__ __forceinline__ void ring_flush(const B2H_LDS uint8_t* ring, gout_t out, int32_t from, int32_t to) {
  constexpr int32_t RM = (1 << RLOG) - 1;
  const int lane = lane_id();
  const __amdgpu_buffer_rsrc_t r = wt_rsrc(out);
  int32_t x = from;
  if (((reinterpret_cast<uintptr_t>(out + x) & 15) == 0) && ((x & 15) == 0)) {
    for (; x + 1024 <= to; x += 1024) {
      const int32_t y = x + lane * 16;
      st16<true>(out, r, y, *reinterpret_cast<const B2H_LDS u32x4*>(ring + (y & RM)));
    }
    const int32_t y = x + lane * 16;
    if (y + 16 <= to) st16<true>(out, r, y, *reinterpret_cast<const B2H_LDS u32x4*>(ring + (y & RM)));
    x += ((to - x) >> 4) << 4;
  }
  for (int32_t y = x + lane; y < to; y += 64) st8<true>(out, r, y, ring[y & RM]);
}


// The decoder's LDS ring leaves for global memory in pieces of ring_piece bytes, from the flush
// frontier F (a multiple of the piece) up to at most the current output position: a copy of n
// bytes at op may flush only while op + n - F > R, so R >= n + piece keeps every flushed byte final
// (copies go in steps of <= 1024, literal runs are <= 32).
__host__ __device__ constexpr int32_t ring_piece(int rlog) { return (1 << rlog) / 4 < 4096 ? (1 << rlog) / 4 : 4096; }

// Slow paths of the decoder, kept out of line on purpose: inlined, their loops and the flushes
// made the token loop irreducible (the backend then wraps every token in a guard-variable
// state machine, ~4x the instructions).  Called for copies longer than 64 bytes, sources older
// than the ring, and ring flushes.  Returns the new flush frontier F.
// A source before the stream start (src < 0, LZ4 with a dictionary) reads the dictionary's tail:
// position y < 0 is dict[dsz + y] (LZ4_decompress_safe_usingDict's external dictionary).
// B2H_FAR_COPY=1 (build option, off by default): a 1 KiB piece whose whole source has left the
// ring (C4's plane 1: 250-16 K byte matches 2-32 KiB back) is copied with sixteen byte loads per
// lane in flight -- one round trip per KiB instead of per 64 bytes -- then the ring writes.  It
// halves plane 1's decode (1.11 M -> 0.58 M cycles per stream) and C4 decompress gains 1-5 %, but
// with the call in copy_general, inline or not, the decoder's other paths lose: C1 decompress
// -3..-10 %, C3 -2 % (same-box A/B, profiles/r6_ab_far_copy.txt).  The source ends before the
// flush frontier <= the piece's destination, so no byte of it is written here.
#ifndef B2H_FAR_COPY
#define B2H_FAR_COPY 0
#endif
template <int RLOG>
__device__ __noinline__ void copy_far(B2H_LDS uint8_t* ring, gout_t out, int32_t dst, int32_t src, int32_t n) {
  constexpr int32_t RM = (1 << RLOG) - 1;
  const int lane = lane_id();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  uint8_t b[16];
#pragma unroll
  for (int k = 0; k < 16; k++) b[k] = lane + 64 * k < n ? out[src + lane + 64 * k] : (uint8_t)0;
#pragma unroll
  for (int k = 0; k < 16; k++)
    if (lane + 64 * k < n) ring[(dst + lane + 64 * k) & RM] = b[k];
}
template <int RLOG>
__device__ __noinline__ int32_t copy_general(B2H_LDS uint8_t* ring, gout_t out, int32_t op, int32_t src, int32_t len, int32_t dist, int32_t F,
                                             gin_t dict = nullptr, int32_t dsz = 0) {
  constexpr int32_t R = 1 << RLOG, RM = R - 1, PIECE = ring_piece(RLOG), STEP = 1024;
  const int lane = lane_id();
  const bool overlap = dist < len;
  const int32_t step = overlap ? 64 % dist : 0;
  int32_t r = overlap ? lane % dist : 0;
  // A long overlapping match repeats its period `dist`, so any multiple of it is a distance too:
  // once the first D = a multiple of lcm(dist, 16) >= 1 KiB bytes are out (byte by byte, below),
  // the rest copies 16 bytes per lane from D back -- 16-byte aligned on both sides of the ring,
  // one LDS round trip per KiB instead of sixteen (C4's int64 ramp: 64 KiB matches at distance
  // 256).  D stays within the ring (D + 1 KiB + PIECE <= R: the source slot is never overwritten).
  int32_t vec_from = len;   // relative output offset where the 16-byte copy takes over
  int32_t D = 0;
  if (overlap && len >= 4096 && src >= 0) {
    int32_t l16 = dist;
    while (l16 & 15) l16 += dist;   // lcm(dist, 16)
    D = ((STEP + l16 - 1) / l16) * l16;
    if (D + STEP + PIECE <= R) {
      const int32_t a = D + ((16 - ((op + D) & 15)) & 15);   // and the destination 16-byte aligned
      if (a + STEP < len) vec_from = a;
    }
  }
  for (int32_t done = 0; done < len; done += STEP) {
    if (vec_from < len && done + STEP > vec_from) {
      if (done < vec_from) {        // the bytes before the 16-byte copy takes over
        const int32_t n = vec_from - done;
        while (op + done + n - F > R) { ring_flush<RLOG>(ring, out, F, F + PIECE); F += PIECE; }
        if (src < F) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        r = (done + lane) % dist;
        for (int32_t i = done + lane; i < done + n; i += 64) {
          const int32_t y = src + r;
          ring[(op + i) & RM] = y >= F ? ring[y & RM] : out[y];
          r += step;
          if (r >= dist) r -= dist;
        }
        done = vec_from - STEP;   // (the loop adds STEP)
        continue;
      }
      const int32_t n = min(len - done, STEP);
      while (op + done + n - F > R) { ring_flush<RLOG>(ring, out, F, F + PIECE); F += PIECE; }
      const int32_t n16 = n >> 4;
      if (lane < n16) {
        const int32_t x = op + done + 16 * lane;
        *reinterpret_cast<B2H_LDS u32x4*>(ring + (x & RM)) = *reinterpret_cast<const B2H_LDS u32x4*>(ring + ((x - D) & RM));
      }
      for (int32_t i = (n16 << 4) + lane; i < n; i += 64) {
        const int32_t x = op + done + i;
        ring[x & RM] = ring[(x - D) & RM];
      }
      continue;
    }
    const int32_t n = min(len - done, STEP);
    while (op + done + n - F > R) { ring_flush<RLOG>(ring, out, F, F + PIECE); F += PIECE; }
    // a ring-resident source in slabs of S <= dist bytes (S = the chunk when the copy does not
    // overlap): within a slab every source byte precedes the slab, so all its reads go out before
    // its writes -- one LDS round trip per slab instead of one per 64 bytes (C4's delta planes:
    // runs of 255-511-byte matches at distance 256 / 512)
    const int32_t S = overlap ? (dist >= 64 ? min(dist & ~63, STEP) : 0) : STEP;
    if (S > 0 && src + done >= F) {
      for (int32_t sub = done; sub < done + n; sub += S) {
        const int32_t m = min(S, done + n - sub);
        uint8_t b[16];
#pragma unroll
        for (int k = 0; k < 4; k++) b[k] = ring[(src + sub + lane + 64 * k) & RM];
        if (m > 256) {
#pragma unroll
          for (int k = 4; k < 16; k++) b[k] = ring[(src + sub + lane + 64 * k) & RM];
        }
#pragma unroll
        for (int k = 0; k < 16; k++)
          if (lane + 64 * k < m) ring[(op + sub + lane + 64 * k) & RM] = b[k];
      }
      continue;
    }
    if (B2H_FAR_COPY && n == STEP && src + done >= 0 && src + done + n <= F) {
      copy_far<RLOG>(ring, out, op + done, src + done, n);
      continue;
    }
    if (src < F) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
    r = overlap ? (done + lane) % dist : 0;
    for (int32_t i = done + lane; i < done + n; i += 64) {
      const int32_t y = overlap ? src + r : src + i;
      const uint8_t b = y >= F ? ring[y & RM] : (y >= 0 ? out[y] : dict[dsz + y]);
      ring[(op + i) & RM] = b;
      if (overlap) { r += step; if (r >= dist) r -= dist; }
    }
  }
  return F;
}
// Ring-resident match of up to 256 bytes whose source ends before it starts (dist >= len):
// every source byte is final, so the four 64-byte slices' LDS reads are all issued before the
// first write.  Matches over 64 bytes are ~8 % of a float32 mantissa plane's tokens; through
// copy_general each cost a call and a dependent read->write per slice.
template <int RLOG>
__device__ __forceinline__ void ring_copy256(B2H_LDS uint8_t* ring, int32_t op, int32_t src, int32_t len) {
  constexpr int32_t RM = (1 << RLOG) - 1;
  const int lane = lane_id();
  uint8_t b[4];
#pragma unroll
  for (int u = 0; u < 4; u++) b[u] = lane + 64 * u < len ? ring[(src + lane + 64 * u) & RM] : (uint8_t)0;
#pragma unroll
  for (int u = 0; u < 4; u++)
    if (lane + 64 * u < len) ring[(op + lane + 64 * u) & RM] = b[u];
}
// Flush 4 KiB pieces until end - F <= ring size.
template <int RLOG>
__device__ __noinline__ int32_t flush_to(B2H_LDS uint8_t* ring, gout_t out, int32_t end, int32_t F) {
  constexpr int32_t R = 1 << RLOG, PIECE = ring_piece(RLOG);
  while (end - F > R) { ring_flush<RLOG>(ring, out, F, F + PIECE); F += PIECE; }
  return F;
}
// BloscLZ stream decode (blosc/blosclz.c:685-795).  Returns decoded bytes, or 0 on any violation
// (same conditions and order as the reference).  Output goes through an LDS ring of 2^RLOG bytes:
// matches read their source from the ring (in-order LDS per wave: no fences), and bytes leave for
// `out` in 4 KiB pieces once they are more than one ring behind.  A source older than the ring
// (distance > ring, rare) is read back from `out` after a fence.  One register peek per token;
// matches up to 64 bytes and literal runs are one LDS read + write per lane.
template <int RLOG>
__device__ __forceinline__ int32_t wave_lz_decode_ring(gin_t in, int32_t length, gout_t out, int32_t maxout,
                                                       B2H_LDS uint8_t* ring) {
  constexpr int32_t R = 1 << RLOG, RM = R - 1;
  const int lane = lane_id();
  if (length == 0) return 0;
  InWin W;
  inwin_reload(W, in, length, 0);
  int32_t ip = 0, op = 0, F = 0;   // ip: the current ctrl byte; output [0, F) already in `out`
  // the first ctrl is read as byte0 & 31 (blosc/blosclz.c:694): clear its top bits in the
  // register window (ip never returns to 0) instead of carrying a first-token flag, which the
  // compiler would thread into a second loop entry (irreducible -> state machine)
  if (lane == 0) W.w0 &= ~(0xe0u << (8 * (-W.wpos)));
  // make the entry values opaque: with ip = 0 known on the entry edge the compiler threads that
  // edge past the window check into the loop body (a second loop entry -> irreducible loop ->
  // guard-variable state machine around every token)
  asm volatile("" : "+s"(ip), "+s"(W.wpos));
  for (;;) {
    const int32_t k = inwin_seek(W, in, length, ip);
    const uint32_t t = inwin_peek4(W, k);
    const uint32_t ctrl = t & 0xffu;
    int32_t p = ip + 1;   // the reference's ip after reading ctrl
    if (ctrl >= 32) {
      int32_t len = (int32_t)(ctrl >> 5) + 2;
      const int32_t ofs = (int32_t)(ctrl & 31u) << 8;
      int32_t dist;
      if (len == 9) {   // length extension bytes
        uint32_t code;
        len = 6;
        do {
          if (p + 1 >= length) return 0;
          code = inwin_byte(W, in, length, p++);
          len += (int32_t)code;
        } while (code == 255);
        code = inwin_byte(W, in, length, p++);
        len += 3;
        dist = ofs + (int32_t)code + 1;
        if (code == 255 && ofs == (31 << 8)) {
          if (p + 1 >= length) return 0;
          const uint32_t hi = inwin_byte(W, in, length, p), lo = inwin_byte(W, in, length, p + 1);
          dist = (int32_t)((hi << 8) | lo) + (int32_t)kLzNear + 1;
          p += 2;
        }
      } else {
        if (p + 1 >= length) return 0;
        const uint32_t code = (t >> 8) & 0xffu;
        p += 1;
        dist = ofs + (int32_t)code + 1;   // op - ref after the reference's ref--
        if (code == 255 && ofs == (31 << 8)) {
          if (p + 1 >= length) return 0;
          dist = (int32_t)((((t >> 16) & 0xffu) << 8) | (t >> 24)) + (int32_t)kLzNear + 1;
          p += 2;
        }
      }
      if (op + len > maxout) return 0;
      if (op - dist < 0) return 0;
      if (p >= length) break;   // a trailing match is dropped (blosc/blosclz.c:742)
      const int32_t src = op - dist;
      if (len <= 64 && src >= F && op + len - F <= R) {
        // overlapping copies replicate the period `dist`: every source byte precedes this token
        const int32_t yl = dist < len ? lane % dist : lane;
        if (lane < len) ring[(op + lane) & RM] = ring[(src + yl) & RM];
      } else {
        F = copy_general<RLOG>(ring, out, op, src, len, dist, F);
      }
      op += len;
    } else {
      const int32_t run = (int32_t)ctrl + 1;
      if (op + run > maxout) return 0;
      if (p + run > length) return 0;
      if (op + run - F > R) F = flush_to<RLOG>(ring, out, op + run, F);
      // bytes [p, p + run) sit at w0 offsets k + 1 .. k + run (< 288): w0, spilling into w1
      const int32_t idx = k + 1 + lane;
      uint32_t v = (uint32_t)__shfl((int)W.w0, idx >> 2);
      if (k + 1 + run > 256) {
        const uint32_t v1 = (uint32_t)__shfl((int)W.w1, (idx >> 2) & 63);
        v = idx >= 256 ? v1 : v;
      }
      if (lane < run) ring[(op + lane) & RM] = (uint8_t)(v >> (8 * (idx & 3)));
      op += run;
      p += run;
      if (p >= length) break;
    }
    ip = p;
  }
  ring_flush<RLOG>(ring, out, F, op);
  return op;
}

// ------------------------------------------------------------------------ LZ4 decoder ----
// Bytes into the ring from global memory (`zero`: zero bytes), 1 KiB per step, flushing ahead.
template <int RLOG>
__device__ __noinline__ int32_t ring_put(B2H_LDS uint8_t* ring, gout_t out, int32_t op, gin_t src, int32_t len,
                                         bool zero, int32_t F) {
  constexpr int32_t RM = (1 << RLOG) - 1;
  const int lane = lane_id();
  for (int32_t done = 0; done < len; done += 1024) {
    const int32_t n = min(len - done, 1024);
    F = flush_to<RLOG>(ring, out, op + done + n, F);
    for (int32_t i = done + lane; i < done + n; i += 64) ring[(op + i) & RM] = zero ? (uint8_t)0 : src[i];
  }
  return F;
}

// LZ4 block decode, compformat 1 (blosc/blosc2.c:500-519 -> LZ4_decompress_safe of lz4 1.9.3;
// the grammar, bounds and rejections restated in oracle/blosc2_oracle.c or_lz4_decompress).
// Sequence = token (literal length << 4 | match length - 4, 15 = extension bytes until one != 255),
// literals, LE16 offset, match; the last sequence is literals only.  Same LDS-ring machinery as
// the BloscLZ decoder: token bytes by readlane from the register window, literal runs and matches
// copied by 64 lanes through the ring.  Returns decoded bytes, or -1.
// `dict` / `dsz`: the chunk's dictionary (BLOSC2_USEDICT, blosc/blosc2.c:504-508), matches may
// reach dsz bytes before the output start.
__device__ __forceinline__ uint32_t win_dword(const InWin& W, int32_t q);
#ifndef B2H_LZ4_PAR
#define B2H_LZ4_PAR 1
#endif
// (noinline: the LZ4 batch's registers would otherwise count against the BloscLZ decoder's
// 96-VGPR budget in k_decode -- 4 spills inlined)
template <int RLOG>
__device__ __noinline__ int32_t wave_lz4_decode_ring(gin_t in, int32_t length, gout_t out, int32_t maxout,
                                                        B2H_LDS uint8_t* ring, gin_t dict = nullptr, int32_t dsz = 0) {
  constexpr int32_t R = 1 << RLOG, RM = R - 1;
  constexpr int32_t kMfLimit = 12, kLastLit = 5;
  constexpr int32_t WMAX = R - ring_piece(RLOG) < 8192 ? R - ring_piece(RLOG) : 8192;
  const int lane = lane_id();
  // (a call's arguments arrive in VGPRs: make the wave-uniform ones scalar again)
  auto upt = [](const void* q) -> uint64_t {
    const uint64_t a = reinterpret_cast<uintptr_t>(q);
    return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(a >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)a);
  };
  in = (gin_t)upt((const void*)in);
  out = (gout_t)upt((const void*)out);
  dict = (gin_t)upt((const void*)dict);
  length = __builtin_amdgcn_readfirstlane(length);
  maxout = __builtin_amdgcn_readfirstlane(maxout);
  dsz = __builtin_amdgcn_readfirstlane(dsz);
  if (length <= 0) return -1;
  if (maxout == 0) return (length == 1 && in[0] == 0) ? 0 : -1;
  InWin W;
  inwin_reload(W, in, length, 0);
  int32_t ip = 0, op = 0, F = 0;
  asm volatile("" : "+s"(ip), "+s"(W.wpos));
  for (;;) {
#if B2H_LZ4_PAR
    // ---- window-parallel batch (as wave_lz_decode_par): every lane parses the sequence that would
    // start at its byte; the true chain from ip is walked; sequences with extension bytes, the
    // last (literals-only) sequence and any bound or offset the serial code rejects or treats
    // specially (offset 0, a dictionary source) end the batch and go through the serial code
    // below, one at a time.  Batched: <= 14 literals, matches with at most one extension byte.
    {
      const int32_t k = inwin_seek(W, in, length, ip);
      const int32_t P = ip + lane;
      const uint32_t lo32 = win_dword(W, k + lane);
      const uint32_t t = lo32 & 0xffu;
      const int32_t L = (int32_t)(t >> 4), M0 = (int32_t)(t & 15u);
      const uint32_t offw = win_dword(W, k + lane + 1 + L);   // offset (2 bytes) + a match extension byte
      const int32_t off = (int32_t)(offw & 0xffffu);
      const int32_t mx = (int32_t)((offw >> 16) & 0xffu);
      const bool mext = M0 == 15;                  // one extension byte (< 255) is taken in the batch
      const int32_t M = M0 + (mext ? mx : 0);
      const int32_t size = 1 + L + 2 + (mext ? 1 : 0), olen = L + M + 4;
      const bool special = L == 15 || (mext && mx == 255) || P + 1 + L > length - (2 + 1 + kLastLit);
      const int32_t step = special ? 128 : size;
      uint64_t chain = 0;
      int32_t sw = 0;
      do {
        chain |= 1ull << sw;
        sw += __builtin_amdgcn_readlane(step, sw);
      } while (sw < 64);
      const uint64_t spec = chain & __ballot(special);
      int32_t st = spec ? __builtin_ctzll(spec) : 64;
      uint64_t batch = chain & (st < 64 ? (1ull << st) - 1 : ~0ull);
      const bool inb = (batch >> lane) & 1ull;
      const int32_t v = inb ? olen : 0;
      const int32_t ex = wave_scan_add(v) - v;   // output offset of the lane's sequence - op
      const int32_t ol = op + ex + L;            // its match's output position
      const bool viol = inb && (op + ex + L > maxout - kMfLimit || off == 0 || off > ol ||
                                ol + M + 4 > maxout - kLastLit || ex + olen > WMAX);
      const uint64_t vm = __ballot(viol);
      if (vm) {
        st = min(st, (int32_t)__builtin_ctzll(vm));
        batch &= (1ull << __builtin_ctzll(vm)) - 1;
      }
      if (batch) {
        const int32_t last = 63 - __builtin_clzll(batch);
        const int32_t nip = ip + (st < 64 ? st : sw);
        const int32_t nop = op + __builtin_amdgcn_readlane(ex + v, last);
        if (nop - F > R) F = flush_to<RLOG>(ring, out, nop, F);
        // literal bytes: byte lane x belongs to the last batch sequence j <= x, a literal when
        // j < x <= j + L_j; the last sequence's literals may run past the 64 parsed bytes
        const bool inbt = (batch >> lane) & 1ull;
        const int32_t owner = wave_scan_max(inbt ? lane : -1);
        const uint32_t opk = (uint32_t)(ex << 6) | (uint32_t)L;   // ex < 2^13, L <= 14
        const uint32_t ow_pk = (uint32_t)__shfl((int)opk, owner & 63);
        const int32_t oL = (int32_t)(ow_pk & 63u), oex = (int32_t)(ow_pk >> 6);
        if (owner >= 0 && lane > owner && lane <= owner + oL)
          ring[(op + oex + (lane - owner - 1)) & RM] = (uint8_t)t;   // t = the byte at ip + lane
        const uint32_t last_pk = (uint32_t)__builtin_amdgcn_readlane((int)opk, last);
        const int32_t lL = (int32_t)(last_pk & 63u);
        if (last + lL >= 64) {
          const int32_t x = 64 + lane;
          const uint32_t byte = win_dword(W, k + x) & 0xffu;
          if (x <= last + lL) ring[(op + (int32_t)(last_pk >> 6) + (x - last - 1)) & RM] = (uint8_t)byte;
        }
        // matches: sources wholly before the batch (<= 64 bytes) eight at a time, reads before
        // writes; the others in order after
        const int32_t ml = M + 4;
        const int32_t srcv = ol - off;
        const bool indep = inbt && ml <= 64 && off >= ex + L + ml && (srcv >= F || srcv + ml <= F);
        uint64_t im = __ballot(indep);
        if (__ballot(indep && srcv < F)) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
        while (im) {
          int32_t oj[8], lj[8], sj[8];
          uint8_t vb[8];
#pragma unroll
          for (int u = 0; u < 8; u++) {
            lj[u] = 0;
            oj[u] = 0;
            sj[u] = 0;
            if (im) {
              const int j = __builtin_ctzll(im);
              im &= im - 1;
              oj[u] = __builtin_amdgcn_readlane(ol, j);
              lj[u] = __builtin_amdgcn_readlane(ml, j);
              sj[u] = oj[u] - __builtin_amdgcn_readlane(off, j);
            }
          }
#pragma unroll
          for (int u = 0; u < 8; u++)
            vb[u] = lane < lj[u] ? (sj[u] >= F ? ring[(sj[u] + lane) & RM] : out[sj[u] + lane]) : (uint8_t)0;
#pragma unroll
          for (int u = 0; u < 8; u++)
            if (lane < lj[u]) ring[(oj[u] + lane) & RM] = vb[u];
        }
        uint64_t mm = batch & ~__ballot(indep);
        while (mm) {
          const int j = __builtin_ctzll(mm);
          mm &= mm - 1;
          const int32_t oj = __builtin_amdgcn_readlane(ol, j);
          const int32_t lj = __builtin_amdgcn_readlane(ml, j);
          const int32_t dj = __builtin_amdgcn_readlane(off, j);
          const int32_t src = oj - dj;
          if (lj <= 64 && src >= F) {
            const int32_t yl = dj < lj ? lane % dj : lane;
            if (lane < lj) ring[(oj + lane) & RM] = ring[(src + yl) & RM];
          } else {
            F = copy_general<RLOG>(ring, out, oj, src, lj, dj, F, dict, dsz);
          }
        }
        ip = nip;
        op = nop;
      }
      if (st >= 64) continue;
    }
#endif
    if (ip >= length) return -1;
    const uint32_t token = inwin_byte(W, in, length, ip++);
    int32_t lit = (int32_t)(token >> 4);
    if (lit == 15) {
      uint32_t s;
      do {
        if (ip >= length) return -1;
        s = inwin_byte(W, in, length, ip++);
        lit += (int32_t)s;
        if (lit > maxout) return -1;
      } while (s == 255);
    }
    const bool last = op + lit > maxout - kMfLimit || ip + lit > length - (2 + 1 + kLastLit);
    if (last && (ip + lit != length || op + lit > maxout)) return -1;
    if (lit > 0) {
      if (lit <= 64 && op + lit - F <= R) {
        if (lane < lit) ring[(op + lane) & RM] = in[ip + lane];
      } else {
        F = ring_put<RLOG>(ring, out, op, in + ip, lit, false, F);
      }
    }
    op += lit;
    ip += lit;
    if (last) break;
    const int32_t off = (int32_t)(inwin_byte(W, in, length, ip) | (inwin_byte(W, in, length, ip + 1) << 8));
    ip += 2;
    if (off > op + dsz) return -1;
    int32_t ml = (int32_t)(token & 15u);
    if (ml == 15) {
      uint32_t s;
      do {
        if (ip >= length - kLastLit) return -1;
        s = inwin_byte(W, in, length, ip++);
        ml += (int32_t)s;
        if (ml > maxout) return -1;
      } while (s == 255);
    }
    ml += 4;
    if (op + ml > maxout - kLastLit) return -1;
    if (off == 0) {   // accepted by liblz4 1.9.3, which writes zeros (see or_lz4_decompress)
      F = ring_put<RLOG>(ring, out, op, in, ml, true, F);
    } else {
      const int32_t src = op - off;
      if (ml <= 64 && src >= F && op + ml - F <= R) {
        const int32_t yl = off < ml ? lane % off : lane;
        if (lane < ml) ring[(op + lane) & RM] = ring[(src + yl) & RM];
      } else {
        F = copy_general<RLOG>(ring, out, op, src, ml, off, F, dict, dsz);
      }
    }
    op += ml;
  }
  ring_flush<RLOG>(ring, out, F, op);
  return op;
}

// ------------------------------------------------------------- window-parallel decoder ----
// Four bytes at (lane-varying) offset q of the 512-byte register window w0|w1 (q <= 504).
__device__ __forceinline__ uint32_t win_dword(const InWin& W, int32_t q) {
  const int32_t d = q >> 2;
  const uint32_t a = (uint32_t)__shfl((int)W.w0, d), a1 = (uint32_t)__shfl((int)W.w1, d & 63);
  const uint32_t b = (uint32_t)__shfl((int)W.w0, (d + 1) & 63), b1 = (uint32_t)__shfl((int)W.w1, (d + 1) & 63);
  return funnel(d < 64 ? a : a1, d + 1 < 64 ? b : b1, (uint32_t)(q & 3));
}

// BloscLZ stream decode, window-parallel (same results and rejections as wave_lz_decode_ring,
// blosc/blosclz.c:685-795).  Per window of 64 candidate token starts ip + lane:
//   1. every lane parses the token that would start at its byte (2..5 header bytes from the
//      register window) -> kind, size, output length, distance;
//   2. the true token chain from ip is walked with one readlane per token (s += size[s]);
//   3. a DPP scan over the chain gives every token's output offset; bound violations (maxout,
//      distance before the output start), tokens near the stream end and multi-byte length
//      extensions end the batch and are decoded one at a time by the serial token code;
//   4. all literal bytes of the batch are written at once (each byte lane finds its token with a
//      max-scan), then the matches are copied in order (sources always precede the token, so
//      literals-first is safe).
// B2H_DEC_STRIP=1 (build option, off by default): the batch's dependent matches are copied one
// output byte per lane over 64-byte strips (pointer doubling for in-strip sources) instead of one
// match at a time.  Bit-exact (the whole decoder tier passes with it), measured slower on T
// (fast decode 4.1 -> 5.5 ms), kept for the record.
#ifndef B2H_DEC_STRIP
#define B2H_DEC_STRIP 0
#endif
#ifdef B2H_DEC_PROF   // diagnostics build only (tools/dec_micro.hip): per-phase s_memtime sums
__device__ uint64_t g_dec_prof[8];
#define DPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define DPROF_ADD(i, a, b) if (lane == 0) atomicAdd((unsigned long long*)&g_dec_prof[i], (unsigned long long)((b) - (a)))
#else
#define DPROF_T(v)
#define DPROF_ADD(i, a, b)
#endif

template <int RLOG>
__device__ __forceinline__ int32_t wave_lz_decode_par(gin_t in, int32_t length, gout_t out, int32_t maxout,
                                                      B2H_LDS uint8_t* ring) {
  // a batch's output must fit the ring next to the unflushed tail (F moves in whole pieces and
  // never past op): WMAX + PIECE <= R
  // (B2H_DEC_STRIP: kMk more bytes past the batch hold the strip markers, see 4b)
  // (and the strip keys hold (ex + 1) << 18 in a positive int: a batch's output stays < 8128)
  constexpr int32_t kMk = B2H_DEC_STRIP ? 260 : 0, kWcap = B2H_DEC_STRIP ? 8128 : 8192;
  constexpr int32_t R = 1 << RLOG, RM = R - 1,
                    WMAX = R - ring_piece(RLOG) - kMk < kWcap ? R - ring_piece(RLOG) - kMk : kWcap;
  const int lane = lane_id();
  if (length == 0) return 0;
  InWin W;
  inwin_reload(W, in, length, 0);
  int32_t ip = 0, op = 0, F = 0;
  int32_t result = -1;   // -1 running, 0 rejected
  if (lane == 0) W.w0 &= ~(0xe0u << (8 * (-W.wpos)));   // first ctrl is byte0 & 31
  asm volatile("" : "+s"(ip), "+s"(W.wpos));
  for (;;) {
    DPROF_T(t0);
    const int32_t k = inwin_seek(W, in, length, ip);
    // ---- 1. parse every candidate start ----
    const int32_t P = ip + lane;
    const uint32_t lo32 = win_dword(W, k + lane), hi32 = win_dword(W, k + lane + 4);
    const uint32_t ctrl = lo32 & 0xffu, b1 = (lo32 >> 8) & 0xffu, b2 = (lo32 >> 16) & 0xffu,
                   b3 = lo32 >> 24, b4 = hi32 & 0xffu;
    const bool lit = ctrl < 32;
    const bool ext = (ctrl >> 5) == 7;
    const uint32_t code = ext ? b2 : b1;
    const uint32_t ofs = (ctrl & 31u) << 8;
    const bool far = !lit && code == 255 && ofs == (31u << 8);
    const int32_t mlen = ext ? 9 + (int32_t)b1 : (int32_t)(ctrl >> 5) + 2;
    const int32_t dist = far ? (int32_t)(((ext ? b3 : b2) << 8) | (ext ? b4 : b3)) + (int32_t)kLzNear + 1
                             : (int32_t)(ofs + code) + 1;
    const int32_t size = lit ? (int32_t)ctrl + 2 : 2 + (ext ? 1 : 0) + (far ? 2 : 0);
    const int32_t olen = lit ? (int32_t)ctrl + 1 : mlen;
    const bool special = (ext && b1 == 255) || (P + 8 > length) || (P + size >= length);
    // ---- 2. chain walk ----
    const int32_t step = special ? 128 : size;
    DPROF_T(t1);
    uint64_t chain = 0;
    int32_t s = 0;
    do {
      chain |= 1ull << s;
      s += __builtin_amdgcn_readlane(step, s);
    } while (s < 64);
    DPROF_T(t2);
    const uint64_t spec = chain & __ballot(special);
    int32_t st = spec ? __builtin_ctzll(spec) : 64;   // first token for the serial path
    uint64_t batch = chain & (st < 64 ? (1ull << st) - 1 : ~0ull);
    // ---- 3. output offsets and bound checks ----
    const bool inb = (batch >> lane) & 1ull;
    const int32_t v = inb ? olen : 0;
    const int32_t ex = wave_scan_add(v) - v;   // exclusive: output offset of lane's token - op
    const bool viol = inb && (op + ex + olen > maxout || (!lit && op + ex < dist) || ex + olen > WMAX);
    const uint64_t vm = __ballot(viol);
    if (vm) {
      st = __builtin_ctzll(vm);
      batch &= (1ull << st) - 1;
    }
    int32_t nip, nop;
    if (st < 64) {
      nip = ip + st;
      nop = op + __builtin_amdgcn_readlane(ex, st);
    } else {
      nip = ip + s;
      nop = op + __builtin_amdgcn_readlane(ex + v, 63);
    }
    DPROF_T(t3);
    if (batch) {
      if (nop + kMk - F > R) F = flush_to<RLOG>(ring, out, nop + kMk, F);
      // ---- 4a. literal bytes: byte lane x belongs to the last batch token at or before it ----
      const bool inbt = (batch >> lane) & 1ull;   // `batch` after the violation cut (`inb` is before it)
      const int32_t owner = wave_scan_max(inbt ? lane : -1);
      const uint32_t opk = (uint32_t)(ex << 6) | (uint32_t)(lit ? olen : 0);   // ex < 2^13, run <= 32
      const uint32_t ow_pk = (uint32_t)__shfl((int)opk, owner & 63);
      const int32_t orun = (int32_t)(ow_pk & 63u), oex = (int32_t)(ow_pk >> 6);
      if (owner >= 0 && lane > owner && lane <= owner + orun)
        ring[(op + oex + (lane - owner - 1)) & RM] = (uint8_t)ctrl;   // ctrl = the byte at ip + lane
      const int32_t last = 63 - __builtin_clzll(batch);
      const uint32_t last_pk = (uint32_t)__builtin_amdgcn_readlane((int)opk, last);
      const int32_t lrun = (int32_t)(last_pk & 63u);
      if (last + lrun >= 64) {   // the last literal run spills past the 64 parsed bytes
        const int32_t x = 64 + lane;
        const uint32_t byte = win_dword(W, k + x) & 0xffu;
        if (x <= last + lrun) ring[(op + (int32_t)(last_pk >> 6) + (x - last - 1)) & RM] = (uint8_t)byte;
      }
      DPROF_T(t4);
#if B2H_DEC_STRIP
      // ---- 4b. matches ----
      // Matches whose whole source precedes the batch (src + len <= op, <= 64 bytes) read nothing
      // this batch writes: their reads go out eight at a time, ahead of the writes -- from the
      // ring (62 % of T's fast-mode matches), or from `out` when the source has already left the
      // ring (src + len <= F: far matches, 41 % of T's exact-mode matches, which one at a time
      // through copy_general cost a global round trip each); the others follow in order, after.
      const int32_t srcv = op + ex - dist;
      const bool indep = inbt && !lit && olen <= 64 && dist >= ex + olen && (srcv >= F || srcv + olen <= F);
      uint64_t im = __ballot(indep);
      if (__ballot(indep && srcv < F)) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // as copy_general
      while (im) {
        int32_t oj[8], lj[8], sj[8];
        uint8_t vb[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          lj[u] = 0;
          oj[u] = 0;
          sj[u] = 0;
          if (im) {
            const int j = __builtin_ctzll(im);
            im &= im - 1;
            oj[u] = op + __builtin_amdgcn_readlane(ex, j);
            lj[u] = __builtin_amdgcn_readlane(olen, j);
            sj[u] = oj[u] - __builtin_amdgcn_readlane(dist, j);
          }
        }
        // (measured round 5: every lane reading the ring for all eight, then the far ones from
        // memory together, was slower -- T decode 4.12 -> 4.29 ms fast, 4.33 -> 4.66 exact)
#pragma unroll
        for (int u = 0; u < 8; u++)
          vb[u] = lane < lj[u] ? (sj[u] >= F ? ring[(sj[u] + lane) & RM] : out[sj[u] + lane]) : (uint8_t)0;
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (lane < lj[u]) ring[(oj[u] + lane) & RM] = vb[u];
      }
      // Dependent matches (a source overlapping the batch's own output, longer than 64 bytes, or
      // straddling the flush frontier): one output byte per lane, 64 at a time, over the strips
      // that hold their bytes.  A byte's token is the last batch token starting at or before it:
      // every token starting in the strip drops its key ((ex + 1) << 18 | dependent << 17 | dist)
      // at its start in a 64-dword marker array, and a max-scan hands each byte the key of its
      // token (starts grow with the token order; the key of the last token before the strip seeds
      // the scan).  A dependent match byte at x copies x - dist; a source inside the strip that is
      // itself a dependent match byte is resolved by pointer doubling over the strip's lanes (each
      // round takes the source's own source), so every byte ends on a final one: a literal (4a), an
      // independent match byte (above), an earlier strip's byte or the bytes before the batch.  The
      // markers sit in the ring slots just past the batch, free by the flush above.
      const bool dep = inbt && !lit && !indep;
      if (__ballot(dep)) {
        const int32_t Lb = nop - op;
        const uint32_t key = inbt ? ((uint32_t)(ex + 1) << 18) | (dep ? 1u << 17 : 0u) | (lit ? 0u : (uint32_t)dist) : 0u;
        const int32_t mk0 = (nop + 3) & ~3;   // dword i at ring slot (mk0 + 4 i) & RM (it may wrap)
        auto mk = [&](int32_t i) -> B2H_LDS uint32_t& {
          return *reinterpret_cast<B2H_LDS uint32_t*>(ring + ((mk0 + 4 * i) & RM));
        };
        bool far = false;
        int32_t b = 0;
        for (;;) {
          // the next strip holding a dependent match byte
          const uint64_t nx = __ballot(dep && ex + olen > b);
          if (!nx) break;
          b = max(b, __builtin_amdgcn_readlane(ex, __builtin_ctzll(nx))) & ~63;
          const uint64_t bef = __ballot(inbt && ex < b);
          const uint32_t seed = bef ? (uint32_t)__builtin_amdgcn_readlane((int)key, 63 - __builtin_clzll(bef)) : 0u;
          mk(lane) = 0u;
          if (inbt && ex >= b && ex < b + 64) mk(ex - b) = key;
          asm volatile("" ::: "memory");   // other lanes' markers: no store-to-load forwarding
          const uint32_t own = (uint32_t)wave_scan_max((int32_t)max(mk(lane), seed));
          const int32_t x = b + lane;
          const bool mb = x < Lb && ((own >> 17) & 1u);
          int32_t sx = x - (int32_t)(own & 0x1ffffu);   // relative to op
          bool need = mb && sx >= b;
          while (__ballot(need)) {
            const int32_t w = mb ? (sx << 1) | 1 : (x << 1);
            const int32_t w2 = __shfl(w, need ? sx - b : lane);
            if (need) {
              if (w2 & 1) sx = w2 >> 1;
              else need = false;   // a final byte of this strip
            }
            need = need && sx >= b;
          }
          const int32_t y = op + sx;
          uint8_t vb = 0;
          if (mb && y >= F) vb = ring[y & RM];
          if (__ballot(mb && y < F)) {   // sources already flushed: read back from `out`
            if (!far) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            far = true;
            if (mb && y < F) vb = out[y];
          }
          if (mb) ring[(op + x) & RM] = vb;
          b += 64;
        }
      }
#else
      // ---- 4b. matches ----
      // Matches whose whole source precedes the batch (src + len <= op, <= 64 bytes) read nothing
      // this batch writes: their reads go out eight at a time, ahead of the writes -- from the
      // ring (62 % of T's fast-mode matches), or from `out` when the source has already left the
      // ring (src + len <= F: far matches, 41 % of T's exact-mode matches, which one at a time
      // through copy_general cost a global round trip each); the others follow in order, after.
      const int32_t srcv = op + ex - dist;
      const bool indep = inbt && !lit && olen <= 64 && dist >= ex + olen && (srcv >= F || srcv + olen <= F);
      uint64_t im = __ballot(indep);
      if (__ballot(indep && srcv < F)) __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");   // as copy_general
      while (im) {
        int32_t oj[8], lj[8], sj[8];
        uint8_t vb[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
          lj[u] = 0;
          oj[u] = 0;
          sj[u] = 0;
          if (im) {
            const int j = __builtin_ctzll(im);
            im &= im - 1;
            oj[u] = op + __builtin_amdgcn_readlane(ex, j);
            lj[u] = __builtin_amdgcn_readlane(olen, j);
            sj[u] = oj[u] - __builtin_amdgcn_readlane(dist, j);
          }
        }
        // (measured round 5: every lane reading the ring for all eight, then the far ones from
        // memory together, was slower -- T decode 4.12 -> 4.29 ms fast, 4.33 -> 4.66 exact)
#pragma unroll
        for (int u = 0; u < 8; u++)
          vb[u] = lane < lj[u] ? (sj[u] >= F ? ring[(sj[u] + lane) & RM] : out[sj[u] + lane]) : (uint8_t)0;
#pragma unroll
        for (int u = 0; u < 8; u++)
          if (lane < lj[u]) ring[(oj[u] + lane) & RM] = vb[u];
      }
      uint64_t mm = batch & ~__ballot(lit) & ~__ballot(indep);
      while (mm) {
        const int j = __builtin_ctzll(mm);
        mm &= mm - 1;
        const int32_t oj = op + __builtin_amdgcn_readlane(ex, j);
        const int32_t lj = __builtin_amdgcn_readlane(olen, j);
        const int32_t dj = __builtin_amdgcn_readlane(dist, j);
        const int32_t src = oj - dj;
        if (lj <= 64 && src >= F) {
          const int32_t yl = dj < lj ? lane % dj : lane;
          if (lane < lj) ring[(oj + lane) & RM] = ring[(src + yl) & RM];
        } else if (lj <= 256 && dj >= lj && src >= F) {
          ring_copy256<RLOG>(ring, oj, src, lj);
        } else {
          F = copy_general<RLOG>(ring, out, oj, src, lj, dj, F);
        }
      }
#endif
      DPROF_T(t5);
      DPROF_ADD(3, t3, t4);
      DPROF_ADD(4, t4, t5);
      ip = nip;
      op = nop;
    }
    DPROF_ADD(0, t0, t1);
    DPROF_ADD(1, t1, t2);
    DPROF_ADD(2, t2, t3);
    if (st >= 64) continue;
    DPROF_T(t6);
    // ---- one token the serial way (ip is its ctrl byte) ----
    {
      const int32_t k2 = inwin_seek(W, in, length, ip);
      const uint32_t t = inwin_peek4(W, k2);
      const uint32_t c = t & 0xffu;
      int32_t p = ip + 1;
      if (c >= 32) {
        int32_t len = (int32_t)(c >> 5) + 2;
        const int32_t of = (int32_t)(c & 31u) << 8;
        int32_t dd;
        bool bad = false;
        if (len == 9) {
          uint32_t cd;
          len = 6;
          do {
            if (p + 1 >= length) { bad = true; break; }
            cd = inwin_byte(W, in, length, p++);
            len += (int32_t)cd;
          } while (cd == 255);
          if (bad) { result = 0; break; }
          cd = inwin_byte(W, in, length, p++);
          len += 3;
          dd = of + (int32_t)cd + 1;
          if (cd == 255 && of == (31 << 8)) {
            if (p + 1 >= length) { result = 0; break; }
            const uint32_t hi = inwin_byte(W, in, length, p), lo = inwin_byte(W, in, length, p + 1);
            dd = (int32_t)((hi << 8) | lo) + (int32_t)kLzNear + 1;
            p += 2;
          }
        } else {
          if (p + 1 >= length) { result = 0; break; }
          const uint32_t cd = (t >> 8) & 0xffu;
          p += 1;
          dd = of + (int32_t)cd + 1;
          if (cd == 255 && of == (31 << 8)) {
            if (p + 1 >= length) { result = 0; break; }
            dd = (int32_t)((((t >> 16) & 0xffu) << 8) | (t >> 24)) + (int32_t)kLzNear + 1;
            p += 2;
          }
        }
        if (op + len > maxout || op - dd < 0) { result = 0; break; }
        if (p >= length) break;   // a trailing match is dropped (blosc/blosclz.c:742)
        const int32_t src = op - dd;
        if (len <= 64 && src >= F && op + len - F <= R) {
          const int32_t yl = dd < len ? lane % dd : lane;
          if (lane < len) ring[(op + lane) & RM] = ring[(src + yl) & RM];
        } else if (len <= 256 && dd >= len && src >= F && op + len - F <= R) {
          ring_copy256<RLOG>(ring, op, src, len);
        } else {
          F = copy_general<RLOG>(ring, out, op, src, len, dd, F);
        }
        op += len;
      } else {
        const int32_t run = (int32_t)c + 1;
        if (op + run > maxout || p + run > length) { result = 0; break; }
        if (op + run - F > R) F = flush_to<RLOG>(ring, out, op + run, F);
        const int32_t k3 = inwin_seek(W, in, length, p);
        const uint32_t byte = win_dword(W, k3 + lane) & 0xffu;
        if (lane < run) ring[(op + lane) & RM] = (uint8_t)byte;
        op += run;
        p += run;
        if (p >= length) break;
      }
      ip = p;
    }
    DPROF_T(t7);
    DPROF_ADD(5, t6, t7);
  }
  if (result == 0) return 0;
  ring_flush<RLOG>(ring, out, F, op);
  return op;
}

}  // namespace b2h
