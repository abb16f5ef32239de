// b2h_lz.h -- wave-cooperative BloscLZ encoder/decoder for gfx950 (device code).
//
// Encoder ("exact mode"): one wave64 owns one stream and reproduces blosclz_compress
// (blosc/blosclz.c:422-619, probe get_cratio 320-419) byte for byte.  The greedy parse is
// inherently serial, so the wave advances through the stream in WINDOWS of up to 64 positions:
//   * every lane hashes its own position and reads the hash table (LDS).  The value is the serial
//     loop's candidate for every lane below W, the first lane whose hash bucket already occurs at
//     an earlier lane of the window (found with one LDS atomic-min per lane).
//   * every lane tests its candidate (one 12-byte compare) and decides literal / match exactly as
//     the serial loop would; `__ballot` yields the accepted-match mask.
//   * a scalar scan then walks the window: literal runs are emitted in parallel (closed-form
//     offsets incl. the 32-literal run markers), each accepted match is emitted, and the scan
//     continues after the match while it stays below W -- the lanes after a match still hold
//     their exact candidates because every position inserted inside the window (literals,
//     anchors, in-window rehash points) owns a distinct bucket.  Long matches are extended
//     cooperatively, 1 KiB per step (64 lanes x 16 bytes).
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

constexpr int kTagBuckets = 2048;   // window bucket-repeat detector (u32 per bucket, LDS)

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

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int32_t rdlane(int32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }

// End of the common prefix of in[x..] and in[x-d..], one past the first mismatch, capped at
// `bound` (get_match / get_run semantics, blosc/blosclz.c:119-165).  64 lanes x 16 bytes per step.
__device__ __forceinline__ int32_t wave_match_end(gin_t in, int32_t x, uint32_t d, int32_t bound) {
  const int lane = lane_id();
  while (x < bound) {
    const int32_t q = x + lane * 16;
    int32_t first = 16;
    if (q < bound) {
      uint32_t a[4], b[4];
      ld16(in + q, a);
      ld16(in + q - d, b);
      const int32_t nb = bound - q;   // bytes at and after `bound` do not count
#pragma unroll
      for (int k = 3; k >= 0; k--) {
        uint32_t diff = a[k] ^ b[k];
        const int32_t lo = 4 * k;
        if (nb <= lo) diff = 0;
        else if (nb < lo + 4) diff &= (1u << (8 * (nb - lo))) - 1u;
        if (diff) first = lo + (__builtin_ctz(diff) >> 3);
      }
    }
    const uint64_t mm = __ballot(first < 16);
    if (mm) {
      const int l = __builtin_ctzll(mm);
      return x + l * 16 + rdlane(first, l) + 1;
    }
    x += 1024;
  }
  return bound;
}

struct LzPassOut {
  int32_t o;       // bytes emitted (emit) / counted (probe)
  int32_t pos;     // final parse position (probe ratio numerator)
  int32_t peak;
  bool fail;
  int32_t windows;
};

// One greedy parse.  PROBE: get_cratio (counts only, limit = min(length, 2^hashlog), no far
// short-match rule, no clevel-9 double rehash, no tail).  !PROBE: the emitting main loop + tail.
template <bool PROBE, typename POS>
__device__ __forceinline__ LzPassOut lz_pass(gin_t in, int32_t length, int hashlog, int clevel, gout_t out,
                                             int32_t maxout, volatile B2H_LDS POS* htab,
                                             volatile B2H_LDS uint32_t* tagm) {
  const int lane = lane_id();
  int32_t limit = length;
  if (PROBE) {
    const int32_t hl = 1 << hashlog;
    limit = length > hl ? hl : length;
  }
  const int32_t bound = limit - 1, loop_end = limit - 12;
  {  // clear the hash table with 8-byte LDS stores
    B2H_LDS uint64_t* h8 = (B2H_LDS uint64_t*)(htab);
    const int32_t n8 = (int32_t)((sizeof(POS) << hashlog) / 8);
    for (int32_t i = lane; i < n8; i += 64) h8[i] = 0;
    // the clear goes through a u64 view: keep the compiler from sinking it below the
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
    if (lane < 5) out[lane] = lane == 0 ? (uint8_t)(kLzMaxCopy - 1) : in[lane - 1];
  }
  int32_t peak = 0;
  bool fail = false;

  while (pos < loop_end) {
    windows++;
    const int32_t P = pos;
    const int32_t p = P + lane;
    const bool valid = p < loop_end;
    uint32_t v = 0, a1 = 0, a2 = 0;
    if (valid) ld12(in + p, v, a1, a2);
    const uint32_t h = lz_hash(v, hashlog);
    const uint32_t c0 = valid ? (uint32_t)htab[h] : 0u;
    // W: first lane whose bucket already occurs at an earlier lane of the window
    const uint32_t b = h & (kTagBuckets - 1);
    if (valid) __hip_atomic_fetch_min((B2H_LDS uint32_t*)&tagm[b], (uint32_t)lane, __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t minl = valid ? tagm[b] : (uint32_t)lane;
    if (valid) tagm[b] = 64u;
    // A lane whose left neighbour has the same hash (runs, short periods) knows its serial
    // candidate exactly: the neighbour, inserted just before it.  Other repeats end the window.
    const uint32_t hprev = (uint32_t)__shfl_up((int)h, 1);
    const bool same1 = valid && lane > 0 && hprev == h;
    const uint64_t s1mask = __ballot(same1);
    const uint64_t dup = __ballot(minl < (uint32_t)lane && !same1);
    int32_t W = dup ? __builtin_ctzll(dup) : 64;
    W = min(W, min(64, loop_end - P));

    // candidate test (lanes < W): literal or match, exactly as the serial loop decides
    const uint32_t cand = same1 ? (uint32_t)(p - 1) : c0;
    const uint32_t dist = (uint32_t)(p - (int32_t)cand);
    bool accept = false;
    int32_t m12 = 0, len = 0;
    if (lane < W && dist != 0 && dist < kLzFar) {
      uint32_t r0, r1, r2;
      ld12(in + cand, r0, r1, r2);
      if (r0 == v) {
        const uint32_t x1 = a1 ^ r1, x2 = a2 ^ r2;
        m12 = x1 ? 4 + (__builtin_ctz(x1) >> 3) : (x2 ? 8 + (__builtin_ctz(x2) >> 3) : 12);
        const int32_t e = min(m12 < 12 ? p + m12 + 1 : 0x7fffffff, bound);
        len = e - 4 - p;
        accept = len >= 4 && (PROBE || !(len <= 5 && (dist - 1) >= kLzNear));
      }
    }
    const uint64_t am = __ballot(accept);

    // scalar walk of the window
    int32_t cur = 0;
    uint64_t visit = 0;
    int32_t next_pos = P + W;
    bool rehash_out = false;
    int32_t rq = 0;
    uint32_t rseq = 0;
    for (;;) {
      const uint64_t rem = cur < 64 ? (am & (~0ull << cur)) : 0ull;
      const int32_t m = rem ? __builtin_ctzll(rem) : W;
      if (m > cur) {   // literals [cur, m)
        const int32_t cnt = m - cur;
        if (!PROBE) {
          const int32_t last = o + (cnt - 1) + (lit + cnt - 1) / 32;
          peak = max(peak, last + 2);
          if (last + 2 > maxout) { fail = true; break; }
          if (lane >= cur && lane < m) {
            const int32_t k = lane - cur;
            const int32_t off = o + k + (lit + k) / 32;
            out[off] = (uint8_t)(v & 0xffu);
            if (((lit + k + 1) & 31) == 0) out[off + 1] = (uint8_t)(kLzMaxCopy - 1);
          }
        }
        o += cnt + (lit + cnt) / 32;
        lit = (lit + cnt) & 31;
        visit |= (m >= 64 ? ~0ull : ((1ull << m) - 1)) & (~0ull << cur);
      }
      if (!rem) { next_pos = P + W; break; }
      // ---- the match of lane m ----
      visit |= 1ull << m;
      const int32_t pm = P + m;
      const uint32_t dm = (uint32_t)pm - (uint32_t)rdlane((int32_t)cand, m);
      int32_t lm = rdlane(len, m);
      if (rdlane(m12, m) == 12) lm = wave_match_end(in, pm + 12, dm, bound) - 4 - pm;
      const uint32_t bd = dm - 1;   // biased distance
      if (lit) {   // close the open literal run
        if (!PROBE) {
          const int32_t at = o - lit - 1;
          if (lane == 0) out[at] = (uint8_t)(lit - 1);
          if (at == 0) byte0 = (uint32_t)(lit - 1);
        }
      } else {
        o--;
      }
      lit = 0;
      const uint32_t ulen = (uint32_t)lm;
      if (PROBE) {
        if (ulen >= 7) o += (int32_t)((ulen - 7) / 255) + 1;
        o += bd < kLzNear ? 2 : 4;
      } else {
        const bool near = bd < kLzNear;
        const uint32_t fd = bd - kLzNear;
        const int32_t ext = ulen >= 7 ? (int32_t)((ulen - 7) / 255) : 0;   // 255 bytes
        const int32_t tok = ulen < 7 ? (near ? 2 : 4) : 1 + ext + (near ? 2 : 4);
        // every bound check of a token is <= the offset after the token: one check suffices
        peak = max(peak, o + tok);
        if (o + tok > maxout) { fail = true; break; }
        if (ulen < 7) {
          if (lane == 0) {
            if (near) { out[o] = (uint8_t)((ulen << 5) + (bd >> 8)); out[o + 1] = (uint8_t)(bd & 255); }
            else { out[o] = (uint8_t)((ulen << 5) + 31); out[o + 1] = 255; out[o + 2] = (uint8_t)(fd >> 8); out[o + 3] = (uint8_t)(fd & 255); }
          }
        } else {
          const uint32_t remlen = (ulen - 7) - 255u * (uint32_t)ext;
          if (lane == 0) out[o] = (uint8_t)((7u << 5) + (near ? (bd >> 8) : 31u));
          for (int32_t i = lane; i < ext; i += 64) out[o + 1 + i] = 255;
          if (lane == 0) {
            const int32_t qq = o + 1 + ext;
            out[qq] = (uint8_t)remlen;
            if (near) { out[qq + 1] = (uint8_t)(bd & 255); }
            else { out[qq + 1] = 255; out[qq + 2] = (uint8_t)(fd >> 8); out[qq + 3] = (uint8_t)(fd & 255); }
          }
        }
        o += tok;
      }
      // rehash at the match boundary q (and q+1 at clevel 9)
      const int32_t q = pm + lm;
      const int32_t ql = q - P;
      if (ql < W && !(!PROBE && clevel == 9)) {
        visit |= 1ull << ql;           // lane ql holds hash(ld32(in + q)) already
      } else {
        rehash_out = true;
        rq = q;
        rseq = ldu32(in + q);
      }
      if (!PROBE) {
        peak = max(peak, o + 1);
        if (o + 1 > maxout) { fail = true; break; }
        if (lane == 0) out[o] = (uint8_t)(kLzMaxCopy - 1);
      }
      o++;
      cur = q + 2 - P;
      next_pos = q + 2;
      // the lane after a match continues the window unless its neighbour-candidate (q + 1)
      // was skipped by the match
      if (!multi || rehash_out || cur >= W || ((s1mask >> cur) & 1ull)) break;
    }
    if (fail) break;
    if ((visit >> lane) & 1ull) htab[h] = (POS)p;   // buckets are distinct below W
    if (rehash_out && lane == 0) {
      htab[lz_hash(rseq, hashlog)] = (POS)rq;
      if (!PROBE && clevel == 9) htab[lz_hash(rseq >> 8, hashlog)] = (POS)(rq + 1);
    }
    pos = next_pos;
  }

  if (!PROBE && !fail) {
    // tail literals [pos, bound]
    while (pos <= bound) {
      const int32_t cnt = min(64, bound - pos + 1);
      const int32_t last = o + (cnt - 1) + (lit + cnt - 1) / 32;
      peak = max(peak, last + 2);
      if (last + 2 > maxout) { fail = true; break; }
      if (lane < cnt) {
        const int32_t off = o + lane + (lit + lane) / 32;
        out[off] = in[pos + lane];
        if (((lit + lane + 1) & 31) == 0) out[off + 1] = (uint8_t)(kLzMaxCopy - 1);
      }
      o += cnt + (lit + cnt) / 32;
      lit = (lit + cnt) & 31;
      pos += cnt;
    }
    if (!fail) {
      if (lit) {
        const int32_t at = o - lit - 1;
        if (lane == 0) out[at] = (uint8_t)(lit - 1);
        if (at == 0) byte0 = (uint32_t)(lit - 1);
      } else {
        o--;
      }
      if (lane == 0) out[0] = (uint8_t)(byte0 | 0x20u);
    }
  }
  r.o = o;
  r.pos = pos;
  r.peak = peak;
  r.fail = fail;
  r.windows = windows;
  return r;
}

// Is the whole stream one repeated byte? (blosc/blosc2.c:1184-1206)  4 KiB per step.
__device__ __forceinline__ bool wave_is_run(gin_t s, int32_t n) {
  const int lane = lane_id();
  const uint8_t first = s[0];
  const uint32_t rep = first * 0x01010101u;
  const bool aligned = (reinterpret_cast<uintptr_t>(s) & 15) == 0;
  for (int32_t base = 0; base < n; base += 64 * 64) {
    bool bad = false;
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
    if (__ballot(bad)) return false;
  }
  return true;
}

// Full per-stream encode with maxout = neblock: run test, entropy probe, main pass.
template <typename POS>
__device__ __forceinline__ StreamResult encode_stream(gin_t in, int32_t n, int clevel, gout_t out,
                                                      volatile B2H_LDS POS* htab, volatile B2H_LDS uint32_t* tagm,
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
  int32_t maxlen = n;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  const LzPassOut pr = lz_pass<true, POS>(in + (n - maxlen), maxlen, hashlog, clevel, out, 0, htab, tagm);
  res.windows = pr.windows;
  const double ratio = (double)pr.pos / (double)pr.o;
  // cratio_ thresholds of blosc/blosclz.c:465 (compared in double, as the reference does)
  const double thr = clevel == 1 ? 2.0 : clevel == 2 ? 1.5 : clevel <= 6 ? 1.2 : clevel == 7 ? 1.15 : clevel == 8 ? 1.1 : 1.0;
  if (ratio < thr || n < 16 || n < 66) return res;
  const LzPassOut em = lz_pass<false, POS>(in, n, hashlog, clevel, out, n, htab, tagm);
  res.windows += em.windows;
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

// ------------------------------------------------------------------ wave fills and copies ----
__device__ __forceinline__ void wave_fill(gout_t o, uint8_t v, int32_t n) {
  const int lane = lane_id();
  const int32_t head = (int32_t)((16 - (reinterpret_cast<uintptr_t>(o) & 15)) & 15);
  const int32_t h = min(head, n);
  if (lane < h) o[lane] = v;
  const uint32_t w = v * 0x01010101u;
  B2H_GLB uint4* o16 = reinterpret_cast<B2H_GLB uint4*>(o + h);
  const int32_t n16 = (n - h) / 16;
  for (int32_t i = lane; i < n16; i += 64) {
    B2H_GLB uint32_t* q = reinterpret_cast<B2H_GLB uint32_t*>(o16 + i);
    q[0] = w; q[1] = w; q[2] = w; q[3] = w;
  }
  for (int32_t i = h + n16 * 16 + lane; i < n; i += 64) o[i] = v;
}

// dst any alignment: aligned u32 stores, sources via ldu32 (8 readable slack bytes assumed).
__device__ __forceinline__ void wave_copy(gout_t o, gin_t s, int32_t n) {
  const int lane = lane_id();
  const int32_t head = (int32_t)((4 - (reinterpret_cast<uintptr_t>(o) & 3)) & 3);
  const int32_t h = min(head, n);
  if (lane < h) o[lane] = s[lane];
  B2H_GLB uint32_t* o4 = reinterpret_cast<B2H_GLB uint32_t*>(o + h);
  const int32_t n4 = (n - h) / 4;
  for (int32_t i = lane; i < n4; i += 64) o4[i] = ldu32(s + h + 4 * i);
  for (int32_t i = h + n4 * 4 + lane; i < n; i += 64) o[i] = s[i];
}

// ------------------------------------------------------------------------------- decoder ----
// Returns decoded bytes, or 0 on any violation (same conditions as the reference).  `out` is
// global memory written and re-read by this wave: every token that reads earlier output first
// waits for the wave's previous stores (workgroup-scope fence).
__device__ __forceinline__ int32_t wave_lz_decode(gin_t in, int32_t length, gout_t out, int32_t maxout) {
  const int lane = lane_id();
  if (length == 0) return 0;
  int32_t ip = 0, op = 0;
  uint32_t ctrl = in[ip++] & 31u;
  for (;;) {
    if (ctrl >= 32) {
      int32_t len = (int32_t)(ctrl >> 5) - 1;
      const int32_t ofs = (int32_t)(ctrl & 31u) << 8;
      uint32_t code;
      if (len == 6) {
        do {
          if (ip + 1 >= length) return 0;
          code = in[ip++];
          len += (int32_t)code;
        } while (code == 255);
      } else if (ip + 1 >= length) {
        return 0;
      }
      code = in[ip++];
      len += 3;
      int32_t dist = ofs + (int32_t)code + 1;   // op - ref after the reference's ref--
      if (code == 255 && ofs == (31 << 8)) {
        if (ip + 1 >= length) return 0;
        dist = (((int32_t)in[ip] << 8) | in[ip + 1]) + (int32_t)kLzNear + 1;
        ip += 2;
      }
      if (op + len > maxout) return 0;
      if (op - dist < 0) return 0;
      if (ip >= length) break;   // a trailing match is dropped (blosc/blosclz.c:742)
      ctrl = in[ip++];
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
      const int32_t src = op - dist;
      if (dist >= len) {
        for (int32_t i = lane; i < len; i += 64) out[op + i] = out[src + i];
      } else {
        // overlapping: period `dist`, every source byte precedes this token
        const int32_t step = 64 % dist;
        int32_t r = lane % dist;
        for (int32_t i = lane; i < len; i += 64) {
          out[op + i] = out[src + r];
          r += step;
          if (r >= dist) r -= dist;
        }
      }
      op += len;
    } else {
      const int32_t run = (int32_t)ctrl + 1;
      if (op + run > maxout) return 0;
      if (ip + run > length) return 0;
      if (lane < run) out[op + lane] = in[ip + lane];
      op += run;
      ip += run;
      if (ip >= length) break;
      ctrl = in[ip++];
    }
  }
  return op;
}

}  // namespace b2h
