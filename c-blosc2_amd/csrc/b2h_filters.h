// b2h_filters.h -- workgroup-level block filters for gfx950 (device code, included by
// b2h_engine.hip).  Each routine transforms ONE block `src -> dst` with the whole workgroup and
// reproduces the reference filter byte-for-byte:
//   shuffle / unshuffle      blosc/shuffle-generic.h:34-83, blosc/shuffle.c:416-449
//   bitshuffle / unshuffle   blosc/bitshuffle-generic.c:147-258, blosc/shuffle.c:454-521
//   delta encode / decode    blosc/delta.c:18-161
//   trunc-prec               blosc/trunc-prec.c:23-86
// Byte transposes move 16 B per lane on the element side and 4 B per lane per plane on the plane
// side, so both the HBM read and write streams are fully coalesced.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace b2h {

constexpr int kBlockThreads = 256;

__device__ __forceinline__ uint32_t byte_of(uint32_t w, int k) { return (w >> (8 * k)) & 0xffu; }

// ------------------------------------------------------------------------------- shuffle ----
// Fast path: TS in {2,4,8,16}, n % 4 == 0, 16-byte aligned src/dst.  A thread owns quads
// (4 elements = 4*TS contiguous bytes) q, q + T, q + 2T, q + 3T (T = threads): every load and
// store instruction stays coalesced across the wave, and the four quads' loads are issued before
// the first store, so 4x the bytes are in flight per lane (HBM latency x bandwidth wants
// ~64 KiB in flight per CU).  Quad q writes one u32 into each of the TS planes.
// `n` elements from `src`; plane p of `dst` starts at dst + p * pstride (pstride = n for a block).
constexpr int kQuadUnroll = 4;

template <int TS>
__device__ __forceinline__ void load_quad(const uint8_t* __restrict__ src, int32_t q, uint32_t (&w)[TS]) {
  const uint32_t* s32 = reinterpret_cast<const uint32_t*>(src + (int64_t)q * 4 * TS);
  if constexpr (TS % 4 == 0) {
#pragma unroll
    for (int k = 0; k < TS / 4; k++) {
      uint4 v = reinterpret_cast<const uint4*>(s32)[k];
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
  } else {  // TS == 2
    uint2 v = *reinterpret_cast<const uint2*>(s32);
    w[0] = v.x; w[1] = v.y;
  }
}

template <int TS>
__device__ __forceinline__ void store_planes(uint8_t* __restrict__ dst, int32_t q, int64_t pstride, const uint32_t (&w)[TS]) {
#pragma unroll
  for (int plane = 0; plane < TS; plane++) {
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int byte = e * TS + plane;     // byte index inside the 4*TS bytes
      o |= byte_of(w[byte / 4], byte % 4) << (8 * e);
    }
    reinterpret_cast<uint32_t*>(dst + (int64_t)plane * pstride)[q] = o;
  }
}

template <int TS>
__device__ void shuffle_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t n, int64_t pstride) {
  const int32_t quads = n / 4, T = blockDim.x;
  int32_t q = threadIdx.x;
  for (; q + (kQuadUnroll - 1) * T < quads; q += kQuadUnroll * T) {
    uint32_t w[kQuadUnroll][TS];
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) load_quad<TS>(src, q + u * T, w[u]);
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) store_planes<TS>(dst, q + u * T, pstride, w[u]);
  }
  for (; q < quads; q += T) {
    uint32_t w[TS];
    load_quad<TS>(src, q, w);
    store_planes<TS>(dst, q, pstride, w);
  }
}

template <int TS>
__device__ __forceinline__ void load_planes(const uint8_t* __restrict__ src, int32_t q, int64_t pstride, uint32_t (&p)[TS]) {
#pragma unroll
  for (int plane = 0; plane < TS; plane++) p[plane] = reinterpret_cast<const uint32_t*>(src + (int64_t)plane * pstride)[q];
}
// The same with run planes: plane j with bit j of `rm` (wave-uniform) is byte j of `rb` throughout
// and is not read (the decoder never staged it).
template <int TS>
__device__ __forceinline__ void load_planes_r(const uint8_t* __restrict__ src, int32_t q, int64_t pstride, uint32_t (&p)[TS],
                                              uint32_t rm, uint64_t rb) {
#pragma unroll
  for (int plane = 0; plane < TS; plane++) {
    if ((rm >> plane) & 1u) p[plane] = 0x01010101u * (uint32_t)((rb >> (8 * plane)) & 0xffu);
    else p[plane] = reinterpret_cast<const uint32_t*>(src + (int64_t)plane * pstride)[q];
  }
}

template <int TS>
__device__ __forceinline__ void store_quad(uint8_t* __restrict__ dst, int32_t q, const uint32_t (&p)[TS]) {
  uint32_t w[TS];
#pragma unroll
  for (int k = 0; k < TS; k++) {
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int byte = 4 * k + b;           // output byte inside the 4*TS bytes
      o |= byte_of(p[byte % TS], byte / TS) << (8 * b);
    }
    w[k] = o;
  }
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + (int64_t)q * 4 * TS);
  if constexpr (TS % 4 == 0) {
#pragma unroll
    for (int k = 0; k < TS / 4; k++) reinterpret_cast<uint4*>(d32)[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  } else {
    *reinterpret_cast<uint2*>(d32) = make_uint2(w[0], w[1]);
  }
}

template <int TS>
__device__ void unshuffle_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t n, int64_t pstride) {
  const int32_t quads = n / 4, T = blockDim.x;
  int32_t q = threadIdx.x;
  for (; q + (kQuadUnroll - 1) * T < quads; q += kQuadUnroll * T) {
    uint32_t p[kQuadUnroll][TS];
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) load_planes<TS>(src, q + u * T, pstride, p[u]);
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) store_quad<TS>(dst, q + u * T, p[u]);
  }
  for (; q < quads; q += T) {
    uint32_t p[TS];
    load_planes<TS>(src, q, pstride, p);
    store_quad<TS>(dst, q, p);
  }
}

__device__ __forceinline__ bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// Whole-block byte shuffle (any typesize 1..256), tail bytes copied verbatim.
__device__ void block_shuffle(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts) {
  const int32_t n = bsize / ts;
  const bool fast = (n % 4 == 0) && aligned16(src) && aligned16(dst);
  if (fast && ts == 4) shuffle_fast<4>(src, dst, n, n);
  else if (fast && ts == 8) shuffle_fast<8>(src, dst, n, n);
  else if (fast && ts == 2) shuffle_fast<2>(src, dst, n, n);
  else if (fast && ts == 16) shuffle_fast<16>(src, dst, n, n);
  else if (ts == 1) {
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
  } else {
    for (int64_t i = threadIdx.x; i < (int64_t)n * ts; i += blockDim.x) {
      const int32_t plane = (int32_t)(i / n), e = (int32_t)(i % n);
      dst[i] = src[(int64_t)e * ts + plane];
    }
  }
  for (int32_t i = n * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

__device__ void block_unshuffle(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts) {
  const int32_t n = bsize / ts;
  const bool fast = (n % 4 == 0) && aligned16(src) && aligned16(dst);
  if (fast && ts == 4) unshuffle_fast<4>(src, dst, n, n);
  else if (fast && ts == 8) unshuffle_fast<8>(src, dst, n, n);
  else if (fast && ts == 2) unshuffle_fast<2>(src, dst, n, n);
  else if (fast && ts == 16) unshuffle_fast<16>(src, dst, n, n);
  else if (ts == 1) {
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
  } else {
    for (int64_t i = threadIdx.x; i < (int64_t)n * ts; i += blockDim.x) {
      const int32_t e = (int32_t)(i / ts), plane = (int32_t)(i % ts);
      dst[i] = src[(int64_t)plane * n + e];
    }
  }
  for (int32_t i = n * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------------- bitshuffle ----
// 8x8 bit-matrix transpose of a u64 whose byte r is row r (bit c = column c): afterwards byte c
// holds column c, i.e. bit r of byte c = bit c of input byte r.  Three swap stages of 1/2/4.
__device__ __forceinline__ uint64_t bit_transpose8(uint64_t x) {
  const uint64_t m1 = 0x00AA00AA00AA00AAull, m2 = 0x0000CCCC0000CCCCull, m4 = 0x00000000F0F0F0F0ull;
  uint64_t t;
  t = (x ^ (x >> 7)) & m1;  x ^= t ^ (t << 7);
  t = (x ^ (x >> 14)) & m2; x ^= t ^ (t << 14);
  t = (x ^ (x >> 28)) & m4; x ^= t ^ (t << 28);
  return x;
}

// Fast bitshuffle, TS in {1,2,4,8}, m % 32 == 0, 16-byte aligned: a thread owns 32 consecutive
// elements (4 groups of 8), reads them with 16-byte loads and writes one u32 (4 group bytes) per
// bit row, so both sides are coalesced.
template <int TS>
__device__ void bitshuffle_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t m) {
  const int32_t rowlen = m / 8;
  for (int32_t t = threadIdx.x; t < m / 32; t += blockDim.x) {
    uint32_t w[8 * TS];   // 32 * TS bytes
    const uint4* s16 = reinterpret_cast<const uint4*>(src + (int64_t)t * 32 * TS);
#pragma unroll
    for (int k = 0; k < 2 * TS; k++) {
      const uint4 v = s16[k];
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
#pragma unroll
    for (int b = 0; b < TS; b++) {
      uint32_t o[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint64_t x = 0;
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const int byte = (8 * j + r) * TS + b;
          x |= (uint64_t)byte_of(w[byte / 4], byte % 4) << (8 * r);
        }
        x = bit_transpose8(x);
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] |= (uint32_t)((x >> (8 * k)) & 0xff) << (8 * j);
      }
#pragma unroll
      for (int k = 0; k < 8; k++) reinterpret_cast<uint32_t*>(dst + (int64_t)(8 * b + k) * rowlen)[t] = o[k];
    }
  }
}

template <int TS>
__device__ void bitunshuffle_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t m) {
  const int32_t rowlen = m / 8;
  for (int32_t t = threadIdx.x; t < m / 32; t += blockDim.x) {
    uint32_t w[8 * TS];
#pragma unroll
    for (int i = 0; i < 8 * TS; i++) w[i] = 0;
#pragma unroll
    for (int b = 0; b < TS; b++) {
      uint32_t rows[8];
#pragma unroll
      for (int k = 0; k < 8; k++) rows[k] = reinterpret_cast<const uint32_t*>(src + (int64_t)(8 * b + k) * rowlen)[t];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint64_t y = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) y |= (uint64_t)byte_of(rows[k], j) << (8 * k);
        y = bit_transpose8(y);
#pragma unroll
        for (int r = 0; r < 8; r++) {
          const int byte = (8 * j + r) * TS + b;
          w[byte / 4] |= (uint32_t)((y >> (8 * r)) & 0xff) << (8 * (byte % 4));
        }
      }
    }
    uint4* d16 = reinterpret_cast<uint4*>(dst + (int64_t)t * 32 * TS);
#pragma unroll
    for (int k = 0; k < 2 * TS; k++) d16[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  }
}

// Output row r = 8*b + k (b: byte of the element, k: bit) has m/8 bytes; byte g of row r packs
// bit k of byte b of elements 8g..8g+7 (element 8g+i in bit i).  Thread g owns one 8-element group.
__device__ void block_bitshuffle(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts) {
  const int32_t m = (bsize / ts) & ~7;
  const int32_t rowlen = m / 8;
  const bool fast = (m % 32) == 0 && aligned16(src) && aligned16(dst);
  if (fast && (ts == 1 || ts == 2 || ts == 4 || ts == 8)) {
    if (ts == 4) bitshuffle_fast<4>(src, dst, m);
    else if (ts == 8) bitshuffle_fast<8>(src, dst, m);
    else if (ts == 2) bitshuffle_fast<2>(src, dst, m);
    else bitshuffle_fast<1>(src, dst, m);
    for (int32_t i = m * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
    return;
  }
  for (int32_t g = threadIdx.x; g < rowlen; g += blockDim.x) {
    const uint8_t* e8 = src + (int64_t)g * 8 * ts;   // 8 consecutive elements
    for (int32_t b = 0; b < ts; b++) {
      uint64_t x = 0;
#pragma unroll
      for (int r = 0; r < 8; r++) x |= (uint64_t)e8[r * ts + b] << (8 * r);
      x = bit_transpose8(x);
#pragma unroll
      for (int k = 0; k < 8; k++) dst[(int64_t)(8 * b + k) * rowlen + g] = (uint8_t)(x >> (8 * k));
    }
  }
  for (int32_t i = m * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

// Inverse.  format_version == 2 (Blosc1 chunks): un-bitshuffle only if (bsize/ts) % 8 == 0,
// else plain copy (blosc/shuffle.c:489-505).
__device__ void block_bitunshuffle(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts,
                                   uint8_t format_version) {
  const int32_t n = bsize / ts;
  if (format_version == 2 && (n % 8) != 0) {
    for (int32_t i = threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
    return;
  }
  const int32_t m = n & ~7;
  const int32_t rowlen = m / 8;
  if ((m % 32) == 0 && aligned16(src) && aligned16(dst) && (ts == 1 || ts == 2 || ts == 4 || ts == 8)) {
    if (ts == 4) bitunshuffle_fast<4>(src, dst, m);
    else if (ts == 8) bitunshuffle_fast<8>(src, dst, m);
    else if (ts == 2) bitunshuffle_fast<2>(src, dst, m);
    else bitunshuffle_fast<1>(src, dst, m);
    for (int32_t i = m * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
    return;
  }
  for (int32_t g = threadIdx.x; g < rowlen; g += blockDim.x) {
    uint8_t* e8 = dst + (int64_t)g * 8 * ts;
    for (int32_t b = 0; b < ts; b++) {
      uint64_t y = 0;
#pragma unroll
      for (int k = 0; k < 8; k++) y |= (uint64_t)src[(int64_t)(8 * b + k) * rowlen + g] << (8 * k);
      y = bit_transpose8(y);
#pragma unroll
      for (int r = 0; r < 8; r++) e8[r * ts + b] = (uint8_t)(y >> (8 * r));
    }
  }
  for (int32_t i = m * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

// --------------------------------------------------------------------------------- delta ----
__device__ __forceinline__ int delta_width(int32_t ts) {
  if (ts == 1 || ts == 2 || ts == 4 || ts == 8) return ts;
  return (ts % 8 == 0) ? 8 : 1;
}

// XOR delta works on w-byte words, byte lanes independent: it is processed in 8-byte chunks
// (little-endian), every chunk holding 8 / w words.
// Prefix XOR of the words inside one chunk.
__device__ __forceinline__ uint64_t xor_prefix64(uint64_t x, int w) {
  if (w == 1) x ^= x << 8;
  if (w <= 2) x ^= x << 16;
  if (w <= 4) x ^= x << 32;
  return x;
}
// The chunk's last word, replicated over the 8 bytes (the carry into the next chunk).
__device__ __forceinline__ uint64_t xor_last_word64(uint64_t x, int w) {
  uint64_t t = w == 8 ? x : x >> (64 - 8 * w);
  if (w == 1) t |= t << 8;
  if (w <= 2) t |= t << 16;
  if (w <= 4) t |= t << 32;
  return t;
}
// The chunk shifted up by one word, the previous chunk's last word entering at the bottom.
__device__ __forceinline__ uint64_t shift_in_word64(uint64_t x, uint64_t prev, int w) {
  return w == 8 ? prev : (x << (8 * w)) | (prev >> (64 - 8 * w));
}

// Encoder.  Block 0: d[i] = s[i] ^ s[i-1] over w-byte words (d[0] = s[0]); `cur` is the stage
// input (the reference passes _src as dref for block 0).  Other blocks: d = s ^ dref where dref is
// the chunk's block-0 region of the pipeline input (blosc/blosc2.c:1126-1128).  Only
// (bsize / w) * w bytes are written, as in the reference.  16 B per lane when aligned.
__device__ void block_delta_encode(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ dref,
                                   uint8_t* __restrict__ dst, int32_t bsize, int32_t ts, bool first_block) {
  const int w = delta_width(ts);
  const int32_t nb = bsize / w * w;
  const bool vec = (nb % 16) == 0 && aligned16(cur) && aligned16(dst) && (first_block || aligned16(dref));
  if (vec && first_block) {
    const ulonglong2* c16 = reinterpret_cast<const ulonglong2*>(cur);
    for (int32_t i = threadIdx.x; i < nb / 16; i += blockDim.x) {
      const ulonglong2 v = c16[i];
      const uint64_t prev = i ? reinterpret_cast<const uint64_t*>(cur)[2 * i - 1] : 0ull;
      ulonglong2 o;
      o.x = v.x ^ shift_in_word64(v.x, prev, w);
      o.y = v.y ^ shift_in_word64(v.y, v.x, w);
      reinterpret_cast<ulonglong2*>(dst)[i] = o;
    }
  } else if (vec) {
    for (int32_t i = threadIdx.x; i < nb / 16; i += blockDim.x) {
      uint4 a = reinterpret_cast<const uint4*>(cur)[i], b = reinterpret_cast<const uint4*>(dref)[i];
      reinterpret_cast<uint4*>(dst)[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
    }
  } else if (first_block) {
    for (int32_t i = threadIdx.x; i < nb; i += blockDim.x) dst[i] = i < w ? cur[i] : (uint8_t)(cur[i] ^ cur[i - w]);
  } else {
    for (int32_t i = threadIdx.x; i < nb; i += blockDim.x) dst[i] = cur[i] ^ dref[i];
  }
}

// Decoder for blocks >= 1: d = s ^ decoded block 0 (bytes past (bsize / w) * w are copied).
__device__ void block_delta_decode_rest(const uint8_t* __restrict__ s, const uint8_t* __restrict__ dref,
                                        uint8_t* __restrict__ d, int32_t bsize, int32_t ts) {
  const int w = delta_width(ts);
  const int32_t nb = bsize / w * w;
  int32_t done = 0;
  if (aligned16(s) && aligned16(dref) && aligned16(d)) {
    done = nb / 16 * 16;
    for (int32_t i = threadIdx.x; i < nb / 16; i += blockDim.x) {
      uint4 a = reinterpret_cast<const uint4*>(s)[i], b = reinterpret_cast<const uint4*>(dref)[i];
      reinterpret_cast<uint4*>(d)[i] = make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
    }
  }
  for (int32_t i = done + threadIdx.x; i < bsize; i += blockDim.x) d[i] = i < nb ? (uint8_t)(s[i] ^ dref[i]) : s[i];
}

// Decoder for block 0: running XOR over w-byte words = inclusive XOR-scan (blosc/delta.c:96-161).
// Coalesced tiles: each pass the workgroup reads kDeltaScanU x blockDim 16-byte pieces (piece
// u * blockDim + tid of the tile, so every load instruction is contiguous across the wave), scans
// each piece's words in registers, XOR-scans the piece totals across the wave with shuffles and
// across waves through LDS (one barrier per tile: the wave totals are double-buffered), and adds
// the carry of all earlier tiles.  XOR of words replicated over a u64 (xor_last_word64) is
// linear, so carries combine by plain XOR.  Scalar word path when unaligned.
constexpr int kDeltaScanU = 4;

__device__ __forceinline__ uint64_t shfl_up64(uint64_t x, int d) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, d), hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}

__device__ void delta_scan_tiles(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int32_t n16, int w) {
  constexpr int U = kDeltaScanU;
  __shared__ uint64_t wt[2][U][kBlockThreads / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int32_t T = blockDim.x;
  const ulonglong2* s16 = reinterpret_cast<const ulonglong2*>(s);
  ulonglong2* d16 = reinterpret_cast<ulonglong2*>(d);
  uint64_t carry = 0;   // XOR of every word before this tile, replicated over the u64
  int buf = 0;
  for (int32_t base = 0; base < n16; base += U * T, buf ^= 1) {
    ulonglong2 v[U];
    uint64_t t[U], x[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t i = base + u * T + (int32_t)threadIdx.x;
      v[u] = i < n16 ? s16[i] : make_ulonglong2(0ull, 0ull);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      v[u].x = xor_prefix64(v[u].x, w);
      v[u].y = xor_prefix64(v[u].y, w) ^ xor_last_word64(v[u].x, w);
      t[u] = xor_last_word64(v[u].y, w);   // the piece's XOR, replicated
      x[u] = t[u];
    }
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t y = shfl_up64(x[u], dd);
        if (lane >= dd) x[u] ^= y;
      }
    }
    if (lane == 63) {
#pragma unroll
      for (int u = 0; u < U; u++) wt[buf][u][wv] = x[u];
    }
    __syncthreads();
    uint64_t c = carry;
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t before = 0, all = 0;
      for (int i = 0; i < nw; i++) {
        const uint64_t tt = wt[buf][u][i];
        before ^= i < wv ? tt : 0ull;
        all ^= tt;
      }
      const uint64_t ex = c ^ before ^ x[u] ^ t[u];   // everything before this piece
      const int32_t i = base + u * T + (int32_t)threadIdx.x;
      if (i < n16) d16[i] = make_ulonglong2(v[u].x ^ ex, v[u].y ^ ex);
      c ^= all;
    }
    carry = c;
  }
  __syncthreads();   // wt is reused by the next call
}

__device__ void block_delta_decode_first(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int32_t bsize,
                                         int32_t ts) {
  __shared__ uint64_t carry[kBlockThreads];
  const int w = delta_width(ts);
  const int32_t nb = bsize / w * w;
  if ((nb % 16) == 0 && aligned16(s) && aligned16(d)) {
    delta_scan_tiles(s, d, nb / 16, w);
    for (int32_t i = nb + threadIdx.x; i < bsize; i += blockDim.x) d[i] = s[i];   // past the last word
    __syncthreads();
    return;
  }
  const int32_t nw = bsize / w;
  const int32_t per = (nw + blockDim.x - 1) / blockDim.x;
  const int32_t lo = min(nw, (int32_t)threadIdx.x * per), hi = min(nw, lo + per);
  auto ldw = [&](int32_t i) { uint64_t v = 0; for (int k = 0; k < w; k++) v |= (uint64_t)s[(int64_t)i * w + k] << (8 * k); return v; };
  auto stw = [&](int32_t i, uint64_t v) { for (int k = 0; k < w; k++) d[(int64_t)i * w + k] = (uint8_t)(v >> (8 * k)); };
  uint64_t acc = 0;
  for (int32_t i = lo; i < hi; i++) acc ^= ldw(i);
  carry[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t r = 0;
    for (int t = 0; t < (int)blockDim.x; t++) { uint64_t v = carry[t]; carry[t] = r; r ^= v; }
  }
  __syncthreads();
  uint64_t r = carry[threadIdx.x];
  for (int32_t i = lo; i < hi; i++) { r ^= ldw(i); stw(i, r); }
  for (int32_t i = nb + threadIdx.x; i < bsize; i += blockDim.x) d[i] = s[i];
  __syncthreads();
}

// ------------------------------------------------- fused DELTA -> SHUFFLE (one pass per block) ----
// filters = (..., DELTA, SHUFFLE) with TS in {2,4,8}: the delta word is the element, so delta
// covers exactly the n * TS shuffled bytes and the (de)shuffle and the XOR run in registers on the
// same quad (4 elements = 4 * TS bytes), with no intermediate block in HBM.  Same results as the
// two stages one after the other (blosc/delta.c:18-161, blosc/shuffle-generic.h:34-83).

// Planes -> element-order u32 words of one quad (the byte permutation of store_quad).
template <int TS>
__device__ __forceinline__ void planes_to_words(const uint32_t (&p)[TS], uint32_t (&w)[TS]) {
#pragma unroll
  for (int k = 0; k < TS; k++) {
    uint32_t o = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int byte = 4 * k + b;
      o |= byte_of(p[byte % TS], byte / TS) << (8 * b);
    }
    w[k] = o;
  }
}

template <int TS>
__device__ __forceinline__ void load_words(const uint8_t* __restrict__ src, int32_t q, uint32_t (&w)[TS]) {
  load_quad<TS>(src, q, w);
}

template <int TS>
__device__ __forceinline__ void store_words(uint8_t* __restrict__ dst, int32_t q, const uint32_t (&w)[TS]) {
  uint32_t* d32 = reinterpret_cast<uint32_t*>(dst + (int64_t)q * 4 * TS);
  if constexpr (TS % 4 == 0) {
#pragma unroll
    for (int k = 0; k < TS / 4; k++) reinterpret_cast<uint4*>(d32)[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  } else {
    *reinterpret_cast<uint2*>(d32) = make_uint2(w[0], w[1]);
  }
}

// Decode, blocks >= 1: dst = unshuffle(src) ^ dref (dref = the chunk's decoded block 0).
template <int TS>
__device__ void unshuffle_xor_fast(const uint8_t* __restrict__ src, const uint8_t* __restrict__ dref,
                                   uint8_t* __restrict__ dst, int32_t n, uint32_t rm = 0, uint64_t rb = 0) {
  const int32_t quads = n / 4, T = blockDim.x;
  int32_t q = threadIdx.x;
  for (; q + (kQuadUnroll - 1) * T < quads; q += kQuadUnroll * T) {
    uint32_t p[kQuadUnroll][TS], r[kQuadUnroll][TS];
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) {
      load_planes_r<TS>(src, q + u * T, n, p[u], rm, rb);
      load_words<TS>(dref, q + u * T, r[u]);
    }
#pragma unroll
    for (int u = 0; u < kQuadUnroll; u++) {
      uint32_t w[TS];
      planes_to_words<TS>(p[u], w);
#pragma unroll
      for (int k = 0; k < TS; k++) w[k] ^= r[u][k];
      store_words<TS>(dst, q + u * T, w);
    }
  }
  for (; q < quads; q += T) {
    uint32_t p[TS], r[TS], w[TS];
    load_planes_r<TS>(src, q, n, p, rm, rb);
    load_words<TS>(dref, q, r);
    planes_to_words<TS>(p, w);
#pragma unroll
    for (int k = 0; k < TS; k++) w[k] ^= r[k];
    store_words<TS>(dst, q, w);
  }
}

// Decode, block 0: dst = inclusive XOR-scan over elements of unshuffle(src).  The tiles of
// delta_scan_tiles with a quad (TS / 2 u64 words) as each lane's piece.
template <int TS>
__device__ void unshuffle_scan_fast(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t n, uint32_t rm = 0,
                                    uint64_t rb = 0, int nx = 0, uint8_t* const* xout = nullptr,
                                    const uint64_t* xrb = nullptr) {
  // nx (<= 3) more outputs: blocks of the same chunk whose every plane is a run of xrb[i]'s bytes,
  // i.e. a constant element v_i after the un-shuffle, so their output is v_i ^ this block's
  // (delta_decoder's other-block rule) -- written here from registers instead of re-reading
  // this block in a second pass
  uint32_t xw[3][TS];
  for (int i = 0; i < 3; i++) {
    uint32_t pr[TS];
#pragma unroll
    for (int j = 0; j < TS; j++) pr[j] = i < nx ? 0x01010101u * (uint32_t)((xrb[i] >> (8 * j)) & 0xffu) : 0u;
    planes_to_words<TS>(pr, xw[i]);
  }
  constexpr int U = 2, K = TS / 2;
  __shared__ uint64_t wt[2][U][kBlockThreads / 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  const int32_t quads = n / 4, T = blockDim.x;
  uint64_t carry = 0;
  int buf = 0;
  // the next tile's planes are loaded before this tile's scan and barrier (the loads are the
  // latency this loop would otherwise expose once per tile)
  uint32_t pn[U][TS];
  auto load_tile = [&](int32_t base) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t q = base + u * T + (int32_t)threadIdx.x;
      if (q < quads) {
        load_planes_r<TS>(src, q, n, pn[u], rm, rb);
      } else {
#pragma unroll
        for (int k = 0; k < TS; k++) pn[u][k] = 0u;
      }
    }
  };
  load_tile(0);
  for (int32_t base = 0; base < quads; base += U * T, buf ^= 1) {
    uint64_t x[U][K], t[U], sc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint32_t w[TS];
      planes_to_words<TS>(pn[u], w);
#pragma unroll
      for (int k = 0; k < K; k++) x[u][k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
    }
    if (base + U * T < quads) load_tile(base + U * T);
#pragma unroll
    for (int u = 0; u < U; u++) {
      x[u][0] = xor_prefix64(x[u][0], TS);
#pragma unroll
      for (int k = 1; k < K; k++) x[u][k] = xor_prefix64(x[u][k], TS) ^ xor_last_word64(x[u][k - 1], TS);
      t[u] = xor_last_word64(x[u][K - 1], TS);
      sc[u] = t[u];
    }
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint64_t y = shfl_up64(sc[u], dd);
        if (lane >= dd) sc[u] ^= y;
      }
    }
    if (lane == 63) {
#pragma unroll
      for (int u = 0; u < U; u++) wt[buf][u][wv] = sc[u];
    }
    __syncthreads();
    uint64_t c = carry;
#pragma unroll
    for (int u = 0; u < U; u++) {
      uint64_t before = 0, all = 0;
      for (int i = 0; i < nw; i++) {
        const uint64_t tt = wt[buf][u][i];
        before ^= i < wv ? tt : 0ull;
        all ^= tt;
      }
      const uint64_t ex = c ^ before ^ sc[u] ^ t[u];
      const int32_t q = base + u * T + (int32_t)threadIdx.x;
      if (q < quads) {
        uint32_t w[TS];
#pragma unroll
        for (int k = 0; k < K; k++) {
          const uint64_t o = x[u][k] ^ ex;
          w[2 * k] = (uint32_t)o;
          w[2 * k + 1] = (uint32_t)(o >> 32);
        }
        store_words<TS>(dst, q, w);
        for (int i = 0; i < nx; i++) {
          uint32_t y[TS];
#pragma unroll
          for (int k = 0; k < TS; k++) y[k] = w[k] ^ xw[i][k];
          store_words<TS>(xout[i], q, y);
        }
      }
      c ^= all;
    }
    carry = c;
  }
  __syncthreads();
}

// Encode: dst = shuffle(delta(src)); block 0 XORs each element with the previous one, other
// blocks with the same element of dref (the chunk's block 0 of the pipeline input).
template <int TS>
__device__ void delta_shuffle_fast(const uint8_t* __restrict__ src, const uint8_t* __restrict__ dref,
                                   uint8_t* __restrict__ dst, int32_t n, bool first_block) {
  const int32_t quads = n / 4, T = blockDim.x;
  for (int32_t q = threadIdx.x; q < quads; q += T) {
    uint32_t w[TS], r[TS];
    load_words<TS>(src, q, w);
    if (first_block) {
      // previous element of every element of the quad: the quad shifted up by one element,
      // the element before the quad (0 for element 0) entering at the bottom
      uint32_t prev[TS / 4 > 0 ? TS / 4 : 1];
      constexpr int EW = TS / 4 > 0 ? TS / 4 : 1;   // u32 words per element (TS=2: half a word)
      if constexpr (TS == 2) {
        const uint32_t pe = q ? (uint32_t)reinterpret_cast<const uint16_t*>(src)[4 * (int64_t)q - 1] : 0u;
        r[0] = (w[0] << 16) | pe;
        r[1] = (w[1] << 16) | (w[0] >> 16);
      } else {
#pragma unroll
        for (int k = 0; k < EW; k++) prev[k] = q ? reinterpret_cast<const uint32_t*>(src)[(int64_t)q * TS - EW + k] : 0u;
#pragma unroll
        for (int k = 0; k < TS; k++) r[k] = k < EW ? prev[k] : w[k - EW];
      }
    } else {
      load_words<TS>(dref, q, r);
    }
#pragma unroll
    for (int k = 0; k < TS; k++) w[k] ^= r[k];
    store_planes<TS>(dst, q, n, w);
  }
}

// ---------------------------------------------------------------------------- trunc-prec ----
// dst = src & ~((1 << zeroed) - 1) per element; returns false on invalid parameters.
__device__ __forceinline__ bool trunc_zeroed_bits(int8_t prec, int32_t ts, int* zeroed) {
  const int mant = ts == 4 ? 23 : (ts == 8 ? 52 : -1);
  if (mant < 0) return false;
  const int p = prec;
  if ((p < 0 ? -p : p) > mant) return false;
  *zeroed = p >= 0 ? mant - p : -p;
  return *zeroed < mant;
}

__device__ void block_trunc(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts, int zeroed) {
  const int32_t n = bsize / ts;
  if (ts == 4) {
    const uint32_t mask = ~((1u << zeroed) - 1u);
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint32_t v; __builtin_memcpy(&v, src + 4 * (int64_t)i, 4); v &= mask; __builtin_memcpy(dst + 4 * (int64_t)i, &v, 4);
    }
  } else {
    const uint64_t mask = ~((1ull << zeroed) - 1ull);
    for (int32_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint64_t v; __builtin_memcpy(&v, src + 8 * (int64_t)i, 8); v &= mask; __builtin_memcpy(dst + 8 * (int64_t)i, &v, 8);
    }
  }
}

// ---------------------------------------------------------------------- bytedelta (35) ----
// plugins/filters/bytedelta/bytedelta.c:86-135 (forward) / 138-185 (backward).  The block is `ts`
// channels of n = bsize / ts bytes (the planes a preceding SHUFFLE produced): forward stores every
// byte minus its predecessor in the channel (the first minus 0), backward the running byte sum;
// the trailing bsize % ts bytes pass through.  Bytes are handled four to a u32 with SWAR add/sub.
__device__ __forceinline__ uint32_t swar_sub8(uint32_t a, uint32_t b) {
  return ((a | 0x80808080u) - (b & 0x7f7f7f7fu)) ^ ((a ^ ~b) & 0x80808080u);
}
__device__ __forceinline__ uint32_t swar_add8(uint32_t a, uint32_t b) {
  return ((a & 0x7f7f7f7fu) + (b & 0x7f7f7f7fu)) ^ ((a ^ b) & 0x80808080u);
}
// byte-wise inclusive prefix sum inside a u32 (little-endian byte order)
__device__ __forceinline__ uint32_t swar_prefix8(uint32_t x) {
  x = swar_add8(x, x << 8);
  return swar_add8(x, x << 16);
}

// Exclusive workgroup scan of per-thread values (sums taken mod 2^32); *total = the sum of all.
__device__ __forceinline__ uint32_t wg_excl_scan(uint32_t v, uint32_t* total) {
  __shared__ uint32_t wsum[kBlockThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = (int)blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
  for (int i = 0; i < nw; i++) {
    const uint32_t t = wsum[i];
    before += i < w ? t : 0u;
    all += t;
  }
  __syncthreads();   // wsum is reused by the next call
  *total = all;
  return before + x - v;
}

__device__ void block_bytedelta_encode(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts) {
  const int32_t n = bsize / ts;
  const bool fast = (n % 16 == 0) && aligned16(src) && aligned16(dst);
  for (int32_t ch = 0; ch < ts; ch++) {
    const uint8_t* s = src + (int64_t)ch * n;
    uint8_t* d = dst + (int64_t)ch * n;
    if (fast) {
      for (int32_t q = threadIdx.x; q < n / 16; q += blockDim.x) {
        const uint4 v = reinterpret_cast<const uint4*>(s)[q];
        const uint32_t prev = q ? (uint32_t)s[16 * (int64_t)q - 1] : 0u;
        uint4 o;
        o.x = swar_sub8(v.x, (v.x << 8) | prev);
        o.y = swar_sub8(v.y, (v.y << 8) | (v.x >> 24));
        o.z = swar_sub8(v.z, (v.z << 8) | (v.y >> 24));
        o.w = swar_sub8(v.w, (v.w << 8) | (v.z >> 24));
        reinterpret_cast<uint4*>(d)[q] = o;
      }
    } else {
      for (int32_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = (uint8_t)(s[i] - (i ? s[i - 1] : 0));
    }
  }
  for (int32_t i = n * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

__device__ void block_bytedelta_decode(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts) {
  const int32_t n = bsize / ts;
  const bool fast = (n % 16 == 0) && aligned16(src) && aligned16(dst);
  const int32_t T = (int32_t)blockDim.x;
  for (int32_t ch = 0; ch < ts; ch++) {
    const uint8_t* s = src + (int64_t)ch * n;
    uint8_t* d = dst + (int64_t)ch * n;
    uint32_t carry = 0;   // channel sum of the bytes before this round
    if (fast) {
      // a round: thread t owns bytes [16 (base + t), +16)
      for (int32_t base = 0; base < n / 16; base += T) {
        const int32_t q = base + (int32_t)threadIdx.x;
        uint4 v = q < n / 16 ? reinterpret_cast<const uint4*>(s)[q] : make_uint4(0u, 0u, 0u, 0u);
        v.x = swar_prefix8(v.x);
        v.y = swar_add8(swar_prefix8(v.y), (v.x >> 24) * 0x01010101u);
        v.z = swar_add8(swar_prefix8(v.z), (v.y >> 24) * 0x01010101u);
        v.w = swar_add8(swar_prefix8(v.w), (v.z >> 24) * 0x01010101u);
        uint32_t all;
        const uint32_t off = (carry + wg_excl_scan(v.w >> 24, &all)) & 0xffu;
        const uint32_t ob = off * 0x01010101u;
        v.x = swar_add8(v.x, ob); v.y = swar_add8(v.y, ob); v.z = swar_add8(v.z, ob); v.w = swar_add8(v.w, ob);
        if (q < n / 16) reinterpret_cast<uint4*>(d)[q] = v;
        carry = (carry + all) & 0xffu;
      }
    } else {
      // contiguous segments per thread: local sums, one scan, then the running sums
      const int32_t seg = (n + T - 1) / T;
      const int32_t lo = min(n, (int32_t)threadIdx.x * seg), hi = min(n, lo + seg);
      uint32_t local = 0;
      for (int32_t i = lo; i < hi; i++) local += s[i];
      uint32_t all;
      uint32_t run = wg_excl_scan(local & 0xffu, &all);
      for (int32_t i = lo; i < hi; i++) {
        run += s[i];
        d[i] = (uint8_t)run;
      }
    }
  }
  for (int32_t i = n * ts + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

// ---------------------------------------------------------------------- int_trunc (36) ----
// plugins/filters/int_trunc/int_trunc.c:18-114: elements of ts in {1, 2, 4, 8} bytes keep their top
// bits, x & ~((1 << zeroed) - 1).  The reference leaves the trailing bsize % ts bytes of its
// scratch buffer unwritten; they are copied here.  Backward is the identity (a copy, 116-125).
__device__ void block_int_trunc(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t bsize, int32_t ts, int zeroed) {
  const uint64_t m64 = ~((1ull << zeroed) - 1ull);
  // the element mask repeats every ts bytes: as u32 words it is m_lo (ts <= 4) or m_lo, m_hi (ts 8)
  uint32_t mlo, mhi;
  if (ts == 8) { mlo = (uint32_t)m64; mhi = (uint32_t)(m64 >> 32); }
  else {
    const uint32_t e = (uint32_t)m64 & (ts == 4 ? 0xffffffffu : ts == 2 ? 0xffffu : 0xffu);
    mlo = ts == 4 ? e : ts == 2 ? (e | (e << 16)) : e * 0x01010101u;
    mhi = mlo;
  }
  const int32_t body = bsize / ts * ts;
  int32_t done = 0;
  if (aligned16(src) && aligned16(dst)) {
    const int32_t n16 = body / 16;
    for (int32_t q = threadIdx.x; q < n16; q += blockDim.x) {
      uint4 v = reinterpret_cast<const uint4*>(src)[q];
      v.x &= mlo; v.y &= mhi; v.z &= mlo; v.w &= mhi;
      reinterpret_cast<uint4*>(dst)[q] = v;
    }
    done = n16 * 16;
  }
  for (int32_t i = done + threadIdx.x; i < body; i += blockDim.x)
    dst[i] = src[i] & (uint8_t)(m64 >> (8 * (i % ts)));
  for (int32_t i = body + threadIdx.x; i < bsize; i += blockDim.x) dst[i] = src[i];
}

}  // namespace b2h
