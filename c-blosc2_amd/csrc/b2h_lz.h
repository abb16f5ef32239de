// b2h_lz.h -- wave-cooperative BloscLZ encoder/decoder for gfx950 (device code).
//
// Encoder ("exact mode"): one wave64 owns one stream and reproduces blosclz_compress
// (blosc/blosclz.c:422-619, probe get_cratio 320-419) byte for byte.  The greedy parse is
// inherently serial, so the wave advances through the stream in WINDOWS of up to 64 positions:
//   * every lane hashes its own position and reads the hash table (LDS) -- valid for all lanes
//     up to the first lane whose hash bucket repeats inside the window (the 2nd lane of a shared
//     bucket would have seen the 1st lane's insert).  A tiny LDS tag table detects repeats.
//   * every lane tests its candidate match (4-byte check + 12-byte prefix), `__ballot` picks the
//     first accepted match; all lanes before it are literals and are emitted in parallel (their
//     output offsets, incl. the 32-literal run markers, are closed-form).
//   * a long match is extended cooperatively, 256 bytes per step (64 lanes x 4 bytes).
// The window restarts after the match exactly where the serial loop would continue, so the
// hash-table state and the output are identical to the reference.
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

constexpr int kTagBuckets = 2048;   // window bucket-repeat detector (LDS bytes per wave)

__device__ __forceinline__ uint32_t lz_hash(uint32_t seq, int hashlog) { return (seq * 2654435761u) >> (32 - hashlog); }

// Unaligned little-endian u32 from global memory: two aligned dword loads + funnel shift.
// Callers guarantee 8 readable bytes past p & ~3 (buffers carry slack).
__device__ __forceinline__ uint32_t ldu32(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uintptr_t(3));
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const uint32_t lo = q[0], hi = q[1];
  return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T>
__device__ __forceinline__ T bcast(T v, int src_lane) {
  return (T)__builtin_amdgcn_readlane((int)v, src_lane);
}

// End of the common prefix of in[x..] and in[x-d..], one past the first mismatch, capped at
// `bound` (get_match / get_run semantics, blosc/blosclz.c:119-165).  Whole wave cooperates.
__device__ int32_t wave_match_end(const uint8_t* __restrict__ in, int32_t x, uint32_t d, int32_t bound) {
  const int lane = lane_id();
  while (x < bound) {
    const int32_t q = x + lane * 4;
    uint32_t diff = 0;
    if (q < bound) {
      diff = ldu32(in + q) ^ ldu32(in + q - d);
      const int32_t nb = bound - q;
      if (nb < 4) diff &= (1u << (8 * nb)) - 1u;
    }
    const uint64_t mm = __ballot(diff != 0);
    if (mm) {
      const int l = __builtin_ctzll(mm);
      const uint32_t dl = (uint32_t)__builtin_amdgcn_readlane((int)diff, l);
      return x + l * 4 + (__builtin_ctz(dl) >> 3) + 1;
    }
    x += 256;
  }
  return bound;
}

struct LzPassOut {
  int32_t o;       // bytes emitted (emit) / counted (probe)
  int32_t pos;     // final parse position (probe ratio numerator)
  int32_t peak;
  bool fail;
};

// One greedy parse.  PROBE: get_cratio (counts only, limit = min(length, 2^hashlog), no far
// short-match rule, no clevel-9 double rehash, no tail).  !PROBE: the emitting main loop + tail.
template <bool PROBE, typename POS>
__device__ LzPassOut lz_pass(const uint8_t* __restrict__ in, int32_t length, int hashlog, int clevel,
                             uint8_t* __restrict__ out, int32_t maxout, volatile POS* htab, volatile uint8_t* tag) {
  const int lane = lane_id();
  int32_t limit = length;
  if (PROBE) {
    const int32_t hl = 1 << hashlog;
    limit = length > hl ? hl : length;
  }
  const int32_t bound = limit - 1, loop_end = limit - 12;
  {  // clear the hash table (16-byte LDS stores)
    uint4* h4 = (uint4*)(htab);
    const int32_t n16 = (int32_t)((sizeof(POS) << hashlog) / 16);
    for (int32_t i = lane; i < n16; i += 64) h4[i] = make_uint4(0, 0, 0, 0);
    // the clear goes through a uint4 view: keep the compiler from sinking it below the
    // (differently typed) table reads that follow
    asm volatile("" ::: "memory");
  }
  LzPassOut r;
  r.peak = 0;
  r.fail = false;
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
    const int32_t p = pos + lane;
    const bool valid = p < loop_end;
    const uint32_t v = valid ? ldu32(in + p) : 0u;
    const uint32_t h = lz_hash(v, hashlog);
    const uint32_t c0 = valid ? (uint32_t)htab[h] : 0u;
    // bucket-repeat detection: winners keep their lane id, losers poison the bucket
    const uint32_t b = h & (kTagBuckets - 1);
    if (valid) tag[b] = (uint8_t)lane;
    const uint32_t t1 = valid ? tag[b] : (uint32_t)lane;
    if (valid && t1 != (uint32_t)lane) tag[b] = 0xFF;
    const bool conflicted = valid && tag[b] == 0xFF;
    const uint64_t cm = __ballot(conflicted);
    const uint64_t cm2 = cm & (cm - 1);
    int32_t W = cm2 ? __builtin_ctzll(cm2) : 64;
    const int32_t nvalid = min(64, loop_end - pos);
    W = min(W, nvalid);

    // candidate test for lanes < W
    const uint32_t dist = (uint32_t)(p - (int32_t)c0);
    bool cand = lane < W && dist != 0 && dist < kLzFar;
    int32_t m12 = 0;
    if (cand) {
      if (ldu32(in + c0) != v) {
        cand = false;
      } else {
        const uint32_t x1 = ldu32(in + p + 4) ^ ldu32(in + c0 + 4);
        const uint32_t x2 = ldu32(in + p + 8) ^ ldu32(in + c0 + 8);
        m12 = x1 ? 4 + (__builtin_ctz(x1) >> 3) : (x2 ? 8 + (__builtin_ctz(x2) >> 3) : 12);
      }
    }
    bool accept = false;
    if (cand) {
      int32_t e = m12 < 12 ? p + m12 + 1 : 0x7fffffff;
      e = min(e, bound);
      const int32_t len = e - 4 - p;
      accept = len >= 4 && (PROBE || !(len <= 5 && (dist - 1) >= kLzNear));
    }
    const uint64_t am = __ballot(accept);
    const int32_t m = am ? __builtin_ctzll(am) : W;   // literal lanes before the match

    // literals [0, m): closed-form offsets (a run marker follows every 32nd literal)
    if (m > 0) {
      if (!PROBE) {
        const int32_t last = o + (m - 1) + (lit + m - 1) / 32;
        peak = max(peak, last + 2);
        if (last + 2 > maxout) { fail = true; break; }
        if (lane < m) {
          const int32_t off = o + lane + (lit + lane) / 32;
          out[off] = (uint8_t)(v & 0xffu);
          if (((lit + lane + 1) & 31) == 0) out[off + 1] = (uint8_t)(kLzMaxCopy - 1);
        }
      }
      o += m + (lit + m) / 32;
      lit = (lit + m) & 31;
    }
    // hash inserts: every literal lane and the match anchor (buckets are unique below W)
    if (lane < m || (am && lane == m)) htab[h] = (POS)p;

    if (!am) {
      pos += m;
      continue;
    }
    // ---- the match of lane m ----
    const int32_t pm = pos + m;
    const uint32_t refm = (uint32_t)__builtin_amdgcn_readlane((int)c0, m);
    const int32_t m12m = __builtin_amdgcn_readlane(m12, m);
    const uint32_t dm = (uint32_t)pm - refm;
    int32_t end = (m12m < 12) ? min(pm + m12m + 1, bound) : wave_match_end(in, pm + 12, dm, bound);
    const int32_t len = end - 4 - pm;
    const uint32_t bd = dm - 1;   // biased distance
    // close the open literal run
    if (lit) {
      if (!PROBE) {
        const int32_t at = o - lit - 1;
        if (lane == 0) out[at] = (uint8_t)(lit - 1);
        if (at == 0) byte0 = (uint32_t)(lit - 1);
      }
    } else {
      o--;
    }
    lit = 0;
    const uint32_t ulen = (uint32_t)len;
    if (PROBE) {
      if (ulen >= 7) o += (int32_t)((ulen - 7) / 255) + 1;
      o += bd < kLzNear ? 2 : 4;
    } else {
      const bool near = bd < kLzNear;
      const uint32_t fd = bd - kLzNear;
      const int32_t ext = ulen >= 7 ? (int32_t)((ulen - 7) / 255) : 0;   // 255 bytes
      const int32_t tok = ulen < 7 ? (near ? 2 : 4) : 1 + ext + (near ? 2 : 4);
      // every check of a token is <= the offset after the token, so one check suffices
      peak = max(peak, o + tok);
      if (o + tok > maxout) { fail = true; break; }
      if (ulen < 7) {
        if (lane == 0) {
          if (near) { out[o] = (uint8_t)((ulen << 5) + (bd >> 8)); out[o + 1] = (uint8_t)(bd & 255); }
          else { out[o] = (uint8_t)((ulen << 5) + 31); out[o + 1] = 255; out[o + 2] = (uint8_t)(fd >> 8); out[o + 3] = (uint8_t)(fd & 255); }
        }
      } else {
        const uint32_t rem = (ulen - 7) - 255u * (uint32_t)ext;
        if (lane == 0) out[o] = (uint8_t)((7u << 5) + (near ? (bd >> 8) : 31u));
        for (int32_t i = lane; i < ext; i += 64) out[o + 1 + i] = 255;
        if (lane == 0) {
          const int32_t q = o + 1 + ext;
          out[q] = (uint8_t)rem;
          if (near) { out[q + 1] = (uint8_t)(bd & 255); }
          else { out[q + 1] = 255; out[q + 2] = (uint8_t)(fd >> 8); out[q + 3] = (uint8_t)(fd & 255); }
        }
      }
      o += tok;
    }
    // rehash at the match boundary
    pos = pm + len;
    const uint32_t seq = ldu32(in + pos);
    if (lane == 0) {
      htab[lz_hash(seq, hashlog)] = (POS)pos;
      if (!PROBE && clevel == 9) htab[lz_hash(seq >> 8, hashlog)] = (POS)(pos + 1);
    }
    pos += 2;
    if (!PROBE) {
      peak = max(peak, o + 1);
      if (o + 1 > maxout) { fail = true; break; }
      if (lane == 0) out[o] = (uint8_t)(kLzMaxCopy - 1);
    }
    o++;
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
  return r;
}

// Is the whole stream one repeated byte? (blosc/blosc2.c:1184-1206)
__device__ bool wave_is_run(const uint8_t* __restrict__ s, int32_t n) {
  const int lane = lane_id();
  const uint8_t first = s[0];
  const uint32_t rep = first * 0x01010101u;
  for (int32_t base = 0; base < n; base += 64 * 16) {
    bool bad = false;
    const int32_t i = base + lane * 16;
    if (i + 16 <= n && ((reinterpret_cast<uintptr_t>(s + i) & 15) == 0)) {
      const uint4 w = *reinterpret_cast<const uint4*>(s + i);
      bad = (w.x != rep) | (w.y != rep) | (w.z != rep) | (w.w != rep);
    } else {
      for (int32_t k = i; k < min(i + 16, n); k++) bad |= s[k] != first;
    }
    if (__ballot(bad)) return false;
  }
  return true;
}

// Full per-stream encode with maxout = neblock: run test, entropy probe, main pass.
template <typename POS>
__device__ StreamResult encode_stream(const uint8_t* __restrict__ in, int32_t n, int clevel, uint8_t* __restrict__ out,
                                      volatile POS* htab, volatile uint8_t* tag, bool allow_runs) {
  StreamResult res;
  res.pad = 0;
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
  const LzPassOut pr = lz_pass<true, POS>(in + (n - maxlen), maxlen, hashlog, clevel, nullptr, 0, htab, tag);
  const double ratio = (double)pr.pos / (double)pr.o;
  const double thr[10] = {0, 2, 1.5, 1.2, 1.2, 1.2, 1.2, 1.15, 1.1, 1.0};
  if (ratio < thr[clevel] || n < 16 || n < 66) return res;
  const LzPassOut em = lz_pass<false, POS>(in, n, hashlog, clevel, out, n, htab, tag);
  if (em.fail) return res;
  res.kind = kStreamLz;
  res.size = em.o;
  res.peak = em.peak;
  return res;
}

// ------------------------------------------------------------------------------- decoder ----
// Returns decoded bytes, or 0 on any violation (same conditions as the reference).  `out` is
// global memory written and re-read by this wave: every token that reads earlier output first
// waits for the wave's previous stores (workgroup-scope fence).
__device__ int32_t wave_lz_decode(const uint8_t* __restrict__ in, int32_t length, uint8_t* out, int32_t maxout) {
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
