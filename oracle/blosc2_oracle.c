/*
 * blosc2_oracle.c -- clean-room CPU restatement of the c-blosc2 (3.3.3.dev) per-block
 * filter -> BloscLZ pipeline and its chunk framing, used ONLY as the parity checker.
 *
 * TEST INFRASTRUCTURE.  The product (c-blosc2_amd/) never links, loads or calls this file.
 * Pinned by the reference's own golden vectors (compat/ .cdata files) and by the reference library
 * compiled from its own sources (oracle/_ref), see tests/test_oracle_*.py.
 *
 * Every function cites the reference file:line whose behaviour it restates.  The code is written
 * index-based (no pointer walking) and the probe and the emitter of BloscLZ share one routine.
 */
#include "blosc2_oracle.h"

#include <stdlib.h>
#include <string.h>

enum {
  HDR_MIN = 16, HDR_EXT = 32,                 /* include/blosc2.h:177-180 */
  MIN_BUF = 32,                               /* BLOSC_MIN_BUFFERSIZE, include/blosc2.h:193 */
  F_SHUF = 1, F_MEMCPY = 2, F_BITSHUF = 4, F_DELTA = 8, /* include/blosc2.h:273-277 */
  FLT_NONE = 0, FLT_SHUFFLE = 1, FLT_BITSHUFFLE = 2, FLT_DELTA = 3, FLT_TRUNC = 4,
  FLT_BYTEDELTA = 35, FLT_INT_TRUNC = 36,     /* include/blosc2/filters-registry.h:27-28 */
  SPLIT_ALWAYS = 1, SPLIT_NEVER = 2, SPLIT_AUTO = 3, SPLIT_FWD = 4,
  SPECIAL_ZERO = 1, SPECIAL_NAN = 2, SPECIAL_VALUE = 3, SPECIAL_UNINIT = 4, USEDICT = 1,
  ERR_DATA = -3, ERR_READ = -5, ERR_WRITE = -6, ERR_PARAM = -12, ERR_CODEC = -7,
  ERR_RUNLEN = -17, ERR_FILTER = -18, ERR_HEADER = -11,
};

static inline uint32_t ld32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline void st32(uint8_t *p, int32_t v) {
  uint32_t u = (uint32_t)v;
  p[0] = (uint8_t)u; p[1] = (uint8_t)(u >> 8); p[2] = (uint8_t)(u >> 16); p[3] = (uint8_t)(u >> 24);
}

/* ------------------------------------------------------------------ shuffle / unshuffle ---- */
/* blosc/shuffle.c:416-430 (param check) + blosc/shuffle-generic.h:34-55 (dst[j*n+i]=src[i*ts+j],
 * tail bs%ts bytes copied verbatim). */
int32_t or_shuffle(int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  if (ts < 1 || ts > 256 || nbytes < 0) return ERR_PARAM;
  int32_t n = nbytes / ts, tail = nbytes % ts;
  for (int32_t plane = 0; plane < ts; plane++)
    for (int32_t e = 0; e < n; e++) dst[(int64_t)plane * n + e] = src[(int64_t)e * ts + plane];
  memcpy(dst + nbytes - tail, src + nbytes - tail, (size_t)tail);
  return nbytes;
}

/* blosc/shuffle.c:435-449 + blosc/shuffle-generic.h:62-83 */
int32_t or_unshuffle(int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  if (ts < 1 || ts > 256 || nbytes < 0) return ERR_PARAM;
  int32_t n = nbytes / ts, tail = nbytes % ts;
  for (int32_t e = 0; e < n; e++)
    for (int32_t plane = 0; plane < ts; plane++) dst[(int64_t)e * ts + plane] = src[(int64_t)plane * n + e];
  memcpy(dst + nbytes - tail, src + nbytes - tail, (size_t)tail);
  return nbytes;
}

/* ------------------------------------------------------------------------- bitshuffle ---- */
/* blosc/shuffle.c:454-478 (m = (bs/ts) rounded down to a multiple of 8, tail copied) and
 * blosc/bitshuffle-generic.c:147-167 (byte transpose, 8x8 bit transpose, bit-row transpose).
 * Net layout: out row r = 8*b + k (b = byte within element, k = bit) is m/8 bytes long and bit
 * (e % 8) of its byte (e / 8) is bit k of byte b of element e. */
static void bit_rows_forward(int32_t ts, int32_t m, const uint8_t *src, uint8_t *dst) {
  int32_t rowlen = m / 8;
  for (int32_t b = 0; b < ts; b++)
    for (int32_t k = 0; k < 8; k++) {
      uint8_t *row = dst + (int64_t)(8 * b + k) * rowlen;
      for (int32_t g = 0; g < rowlen; g++) {
        uint8_t v = 0;
        for (int32_t r = 0; r < 8; r++) v |= (uint8_t)(((src[(int64_t)(8 * g + r) * ts + b] >> k) & 1u) << r);
        row[g] = v;
      }
    }
}

static void bit_rows_inverse(int32_t ts, int32_t m, const uint8_t *src, uint8_t *dst) {
  int32_t rowlen = m / 8;
  memset(dst, 0, (size_t)m * (size_t)ts);
  for (int32_t b = 0; b < ts; b++)
    for (int32_t k = 0; k < 8; k++) {
      const uint8_t *row = src + (int64_t)(8 * b + k) * rowlen;
      for (int32_t g = 0; g < rowlen; g++)
        for (int32_t r = 0; r < 8; r++)
          dst[(int64_t)(8 * g + r) * ts + b] |= (uint8_t)(((row[g] >> r) & 1u) << k);
    }
}

int32_t or_bitshuffle(int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  if (ts < 1 || ts > 256 || nbytes < 0) return ERR_PARAM;
  int32_t m = (nbytes / ts) & ~7;
  bit_rows_forward(ts, m, src, dst);
  int32_t done = m * ts;
  memcpy(dst + done, src + done, (size_t)(nbytes - done));
  return nbytes;
}

/* blosc/shuffle.c:482-521: a chunk whose version byte is 2 (Blosc1) is un-bitshuffled only when
 * its element count is a multiple of 8 (else copied); newer formats work like or_bitshuffle. */
int32_t or_bitunshuffle(int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst,
                        uint8_t format_version) {
  if (ts < 1 || ts > 256 || nbytes < 0) return ERR_PARAM;
  int32_t n = nbytes / ts;
  if (format_version == 2) {
    if (n % 8 == 0) bit_rows_inverse(ts, n, src, dst);
    else memcpy(dst, src, (size_t)nbytes);
    return nbytes;
  }
  int32_t m = n & ~7;
  bit_rows_inverse(ts, m, src, dst);
  int32_t done = m * ts;
  memcpy(dst + done, src + done, (size_t)(nbytes - done));
  return nbytes;
}

/* ------------------------------------------------------------------------------ delta ---- */
/* blosc/delta.c:18-92.  Word width w = ts for ts in {1,2,4,8}, else 8 if ts%8==0, else 1.
 * Block 0 (offset 0): d[0]=ref[0], d[i]=s[i]^ref[i-1]; other blocks: d[i]=s[i]^ref[i].
 * Only nbytes/w words are written. */
static int delta_width(int32_t ts) {
  if (ts == 1 || ts == 2 || ts == 4 || ts == 8) return ts;
  return (ts % 8 == 0) ? 8 : 1;
}

static inline uint64_t ldw(const uint8_t *p, int w) {
  uint64_t v = 0;
  memcpy(&v, p, (size_t)w);
  return v;
}
static inline void stw(uint8_t *p, uint64_t v, int w) { memcpy(p, &v, (size_t)w); }

void or_delta_encode(const uint8_t *dref, int32_t offset, int32_t nbytes, int32_t ts,
                     const uint8_t *src, uint8_t *dst) {
  int w = delta_width(ts);
  int32_t nw = nbytes / w;
  if (nw <= 0) return;
  if (offset == 0) {
    /* Walk backwards so that dst may alias src (the reference works out of place). */
    uint64_t first = ldw(dref, w);
    for (int32_t i = nw - 1; i >= 1; i--) stw(dst + (int64_t)i * w, ldw(src + (int64_t)i * w, w) ^ ldw(dref + (int64_t)(i - 1) * w, w), w);
    stw(dst, first, w);
  } else {
    for (int32_t i = 0; i < nw; i++) stw(dst + (int64_t)i * w, ldw(src + (int64_t)i * w, w) ^ ldw(dref + (int64_t)i * w, w), w);
  }
}

/* blosc/delta.c:96-161: block 0 is an in-place running XOR (prefix scan over words, with
 * dref == dst); other blocks XOR with the decoded block 0. */
void or_delta_decode(const uint8_t *dref, int32_t offset, int32_t nbytes, int32_t ts, uint8_t *dst) {
  int w = delta_width(ts);
  int32_t nw = nbytes / w;
  if (offset == 0) {
    for (int32_t i = 1; i < nw; i++) stw(dst + (int64_t)i * w, ldw(dst + (int64_t)i * w, w) ^ ldw(dref + (int64_t)(i - 1) * w, w), w);
  } else {
    for (int32_t i = 0; i < nw; i++) stw(dst + (int64_t)i * w, ldw(dst + (int64_t)i * w, w) ^ ldw(dref + (int64_t)i * w, w), w);
  }
}

/* ------------------------------------------------------------------------- trunc-prec ---- */
/* blosc/trunc-prec.c:23-86 */
int or_trunc_prec(int8_t prec_bits, int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  int mant;
  if (ts == 4) mant = 23;
  else if (ts == 8) mant = 52;
  else return -1;
  int p = prec_bits;
  if ((p < 0 ? -p : p) > mant) return -1;
  int zeroed = p >= 0 ? mant - p : -p;
  if (zeroed >= mant) return -1;
  uint64_t mask = ~((1ULL << zeroed) - 1ULL);
  int32_t n = nbytes / ts;
  for (int32_t i = 0; i < n; i++) stw(dst + (int64_t)i * ts, ldw(src + (int64_t)i * ts, ts) & mask, ts);
  return 0;
}

/* ------------------------------------------------------------ registered plugin filters ---- */
/* plugins/filters/bytedelta/bytedelta.c:86-135: `channels` planes of nbytes / channels bytes, each
 * byte minus its predecessor in the plane (the first minus 0); the tail is copied. */
void or_bytedelta_encode(int32_t channels, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  int32_t n = nbytes / channels;
  for (int32_t c = 0; c < channels; c++)
    for (int32_t i = 0; i < n; i++) {
      int64_t k = (int64_t)c * n + i;
      dst[k] = (uint8_t)(src[k] - (i ? src[k - 1] : 0));
    }
  memcpy(dst + (int64_t)n * channels, src + (int64_t)n * channels, (size_t)(nbytes - n * channels));
}

/* bytedelta.c:138-185: the running byte sum of every plane */
void or_bytedelta_decode(int32_t channels, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  int32_t n = nbytes / channels;
  for (int32_t c = 0; c < channels; c++) {
    uint8_t acc = 0;
    for (int32_t i = 0; i < n; i++) {
      int64_t k = (int64_t)c * n + i;
      acc = (uint8_t)(acc + src[k]);
      dst[k] = acc;
    }
  }
  memcpy(dst + (int64_t)n * channels, src + (int64_t)n * channels, (size_t)(nbytes - n * channels));
}

/* plugins/filters/int_trunc/int_trunc.c:18-114: elements of 1/2/4/8 bytes keep their top bits; the
 * zeroed-bit count is computed in uint8 arithmetic.  The reference leaves the trailing
 * nbytes % ts bytes of its scratch buffer unwritten; this restatement copies them. */
int or_int_trunc(int8_t prec_bits, int32_t ts, int32_t nbytes, const uint8_t *src, uint8_t *dst) {
  if (ts != 1 && ts != 2 && ts != 4 && ts != 8) return -1;
  uint8_t bits = (uint8_t)(8 * ts);
  uint8_t zeroed = prec_bits >= 0 ? (uint8_t)(bits - prec_bits) : (uint8_t)(-prec_bits);
  if (zeroed >= bits) return -1;
  uint64_t mask = ~((1ULL << zeroed) - 1ULL);
  int32_t n = nbytes / ts;
  for (int32_t i = 0; i < n; i++) stw(dst + (int64_t)i * ts, ldw(src + (int64_t)i * ts, ts) & mask, ts);
  memcpy(dst + (int64_t)n * ts, src + (int64_t)n * ts, (size_t)(nbytes - n * ts));
  return 0;
}

/* ---------------------------------------------------------------------------- BloscLZ ---- */
enum { LZ_MAX_COPY = 32, LZ_NEAR = 8191, LZ_FAR = 65535 + 8191 - 1, LZ_SHIFT = 4, LZ_MINLEN = 4 };

static inline uint32_t lz_hash(uint32_t seq, int hashlog) { return (seq * 2654435761U) >> (32 - hashlog); }

/* End of the common prefix of in[p..] and in[r..] (p > r), as returned by the reference's
 * get_match / get_match_16 / get_run (blosc/blosclz.c:119-190): one past the first mismatching
 * byte, never beyond `bound`.  All three variants give this same answer (distance-1 runs too). */
static inline int32_t lz_match_end(const uint8_t *in, int32_t p, int32_t r, int32_t bound) {
  while (p < bound) {
    int same = in[p] == in[r];
    p++; r++;
    if (!same) return p;
  }
  return bound;
}

/* One greedy parse over in[0..length) (blosc/blosclz.c:422-619 main loop, or the probe
 * get_cratio at 320-419 when `probe` is set).  The probe only counts output bytes, uses
 * `limit` = min(length, 2^hashlog), stops at the main loop (no tail) and has neither the
 * far-distance short-match rule nor the clevel-9 double rehash.
 * Returns: probe -> writes *ratio; emit -> compressed size or 0 if it does not fit. */
static int lz_parse(const uint8_t *in, int32_t length, int hashlog, int clevel, int probe,
                    uint8_t *out, int32_t maxout, double *ratio, uint32_t *htab) {
  int32_t limit = length;
  if (probe) {
    int32_t hashlen = 1 << hashlog;
    limit = length > hashlen ? hashlen : length;
  }
  const int32_t bound = limit - 1, loop_end = limit - 12;
  memset(htab, 0, sizeof(uint32_t) << hashlog);

  int32_t o = 0;          /* output cursor (emit) or output byte count (probe) */
  int32_t lit = 4;        /* literals in the open literal run */
  int32_t pos = 4;
  if (probe) {
    o = 5;
  } else {
    out[0] = LZ_MAX_COPY - 1;
    for (int i = 0; i < 4; i++) out[1 + i] = in[i];
    o = 5;
  }
  if (probe) pos = 0;     /* get_cratio starts hashing at its first byte */
  if (probe) lit = 4;

  while (pos < loop_end) {
    const int32_t anchor = pos;
    const uint32_t h = lz_hash(ld32(in + anchor), hashlog);
    const int32_t ref = (int32_t)htab[h];
    uint32_t dist = (uint32_t)(anchor - ref);
    htab[h] = (uint32_t)anchor;

    int literal = (dist == 0 || dist >= LZ_FAR) || ld32(in + ref) != ld32(in + anchor);
    int32_t len = 0;
    if (!literal) {
      dist--;  /* biased distance */
      int32_t end = lz_match_end(in, anchor + 4, ref + 4, bound);
      len = end - LZ_SHIFT - anchor;
      if (len < LZ_MINLEN) literal = 1;
      else if (!probe && len <= 5 && dist >= LZ_NEAR) literal = 1;
    }
    if (literal) {
      /* LITERAL / LITERAL2 macros, blosc/blosclz.c:248-268 */
      if (probe) {
        o++;
      } else {
        if (o + 2 > maxout) return 0;
        out[o++] = in[anchor];
      }
      pos = anchor + 1;
      if (++lit == LZ_MAX_COPY) {
        lit = 0;
        if (probe) o++; else out[o++] = LZ_MAX_COPY - 1;
      }
      continue;
    }
    /* close the literal run (blosc/blosclz.c:546-554 / 387-391) */
    if (probe) {
      if (!lit) o--;
    } else {
      if (lit) out[o - lit - 1] = (uint8_t)(lit - 1);
      else o--;
    }
    lit = 0;
    pos = anchor + len;
    const uint32_t ulen = (uint32_t)len;
    if (probe) {
      if (ulen >= 7) o += (int32_t)((ulen - 7) / 255) + 1;
      o += dist < LZ_NEAR ? 2 : 4;
    } else if (dist < LZ_NEAR) {
      /* MATCH_SHORT / MATCH_LONG, blosc/blosclz.c:270-290 */
      if (ulen < 7) {
        if (o + 2 > maxout) return 0;
        out[o++] = (uint8_t)((ulen << 5) + (dist >> 8));
        out[o++] = (uint8_t)(dist & 255);
      } else {
        if (o + 1 > maxout) return 0;
        out[o++] = (uint8_t)((7u << 5) + (dist >> 8));
        uint32_t rem = ulen - 7;
        for (; rem >= 255; rem -= 255) {
          if (o + 1 > maxout) return 0;
          out[o++] = 255;
        }
        if (o + 2 > maxout) return 0;
        out[o++] = (uint8_t)rem;
        out[o++] = (uint8_t)(dist & 255);
      }
    } else {
      /* MATCH_SHORT_FAR / MATCH_LONG_FAR, blosc/blosclz.c:292-316 */
      uint32_t fd = dist - LZ_NEAR;
      if (ulen < 7) {
        if (o + 4 > maxout) return 0;
        out[o++] = (uint8_t)((ulen << 5) + 31);
        out[o++] = 255;
        out[o++] = (uint8_t)(fd >> 8);
        out[o++] = (uint8_t)(fd & 255);
      } else {
        if (o + 1 > maxout) return 0;
        out[o++] = (7u << 5) + 31;
        uint32_t rem = ulen - 7;
        for (; rem >= 255; rem -= 255) {
          if (o + 1 > maxout) return 0;
          out[o++] = 255;
        }
        if (o + 4 > maxout) return 0;
        out[o++] = (uint8_t)rem;
        out[o++] = 255;
        out[o++] = (uint8_t)(fd >> 8);
        out[o++] = (uint8_t)(fd & 255);
      }
    }
    /* rehash at the match boundary (blosc/blosclz.c:573-586 / 408-412) */
    const uint32_t seq = ld32(in + pos);
    htab[lz_hash(seq, hashlog)] = (uint32_t)pos;
    if (!probe && clevel == 9) htab[lz_hash(seq >> 8, hashlog)] = (uint32_t)(pos + 1);
    pos += 2;
    if (probe) {
      o++;
    } else {
      if (o + 1 > maxout) return 0;
      out[o++] = LZ_MAX_COPY - 1;
    }
  }
  if (probe) {
    *ratio = (double)pos / (double)o;
    return 0;
  }
  /* tail literals (blosc/blosclz.c:595-610) */
  for (; pos <= bound; pos++) {
    if (o + 2 > maxout) return 0;
    out[o++] = in[pos];
    if (++lit == LZ_MAX_COPY) {
      lit = 0;
      out[o++] = LZ_MAX_COPY - 1;
    }
  }
  if (lit) out[o - lit - 1] = (uint8_t)(lit - 1);
  else o--;
  out[0] |= 1u << 5;  /* blosc/blosclz.c:613 */
  return o;
}

/* blosc/blosclz.c:422-468: entropy probe over the last `maxlen` bytes, then the real pass. */
int or_blosclz_compress(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout) {
  static const uint8_t hashlogs[10] = {0, 12, 13, 14, 14, 14, 14, 14, 14, 14};
  static const double min_ratio[10] = {0, 2, 1.5, 1.2, 1.2, 1.2, 1.2, 1.15, 1.1, 1.0};
  if (clevel < 1 || clevel > 9) return 0;
  int hashlog = hashlogs[clevel];
  uint32_t *htab = (uint32_t *)malloc(sizeof(uint32_t) << 14);
  if (!htab) return -1;
  int32_t maxlen = length;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  double ratio = 0.0;
  lz_parse(in + (length - maxlen), maxlen, hashlog, clevel, 1, NULL, 0, &ratio, htab);
  int r = 0;
  if (!(ratio < min_ratio[clevel]) && length >= 16 && maxout >= 66)
    r = lz_parse(in, length, hashlog, clevel, 0, out, maxout, NULL, htab);
  free(htab);
  return r;
}

/* blosc/blosclz.c:685-795.  Returns the decoded size, 0 on any bound violation. */
int or_blosclz_decompress(const uint8_t *in, int length, uint8_t *out, int maxout) {
  if (length == 0) return 0;
  int32_t ip = 0, op = 0;
  uint32_t ctrl = in[ip++] & 31u;
  for (;;) {
    if (ctrl >= 32) {
      int32_t len = (int32_t)(ctrl >> 5) - 1;
      int32_t ofs = (int32_t)(ctrl & 31u) << 8;
      uint8_t code;
      if (len == 6) {
        do {
          if (ip + 1 >= length) return 0;
          code = in[ip++];
          len += code;
        } while (code == 255);
      } else if (ip + 1 >= length) {
        return 0;
      }
      code = in[ip++];
      len += 3;
      int64_t ref = (int64_t)op - ofs - code;
      if (code == 255 && ofs == (31 << 8)) {
        if (ip + 1 >= length) return 0;
        int32_t far = (int32_t)in[ip] << 8 | in[ip + 1];
        ip += 2;
        ref = (int64_t)op - far - LZ_NEAR;
      }
      if (op + len > maxout) return 0;
      if (ref - 1 < 0) return 0;
      /* a match that ends the input is dropped, not copied (blosc/blosclz.c:742) */
      if (ip >= length) break;
      ctrl = in[ip++];
      ref--;
      for (int32_t i = 0; i < len; i++) out[op + i] = out[ref + i];  /* forward, overlap-safe */
      op += len;
    } else {
      int32_t run = (int32_t)ctrl + 1;
      if (op + run > maxout) return 0;
      if (ip + run > length) return 0;
      memcpy(out + op, in + ip, (size_t)run);
      op += run;
      ip += run;
      if (ip >= length) break;
      ctrl = in[ip++];
    }
  }
  return op;
}

/* ------------------------------------------------------------------------------ LZ4 ---- */
/* LZ4 block format, compformat 1 (blosc/blosc2.c:450-469 lz4_wrap_compress -> LZ4_compress_fast,
 * 500-519 lz4_wrap_decompress -> LZ4_decompress_safe).  LZ4 is a third-party dependency, absent
 * from /root/reference: CMakeLists.txt:141 pins lz4 1.10.0; the image ships lz4 1.9.3
 * (/opt/conda/lib/liblz4.so, the library oracle/_ref links).  Restated from the published
 * algorithm of lz4.c LZ4_compress_generic (noDict, limitedOutput, byU16 table of 2^13 u16
 * positions with hash4 when the input is < 64 KiB + 11, else byU32 of 2^12 with the 5-byte hash)
 * and pinned byte-for-byte against liblz4 itself (tests/test_oracle.py::test_lz4_*). */
enum { LZ4_MINMATCH = 4, LZ4_MFLIMIT = 12, LZ4_LASTLIT = 5, LZ4_SKIP = 6, LZ4_RUN_MASK = 15,
       LZ4_ML_MASK = 15, LZ4_64K = 65536 + 11, LZ4_DMAX = 65535 };

static inline uint32_t lz4_hash_at(const uint8_t *p, int u16tab) {
  if (u16tab) return (ld32(p) * 2654435761U) >> (32 - 13);                  /* LZ4_hash4, log 12+1 */
  uint64_t v; memcpy(&v, p, 8);
  return (uint32_t)(((v << 24) * 889523592379ULL) >> (64 - 12));            /* LZ4_hash5, log 12 */
}

/* LZ4_count: equal bytes of in[a..] and in[b..] before `limit` */
static inline int32_t lz4_count(const uint8_t *in, int32_t a, int32_t b, int32_t limit) {
  int32_t n = 0;
  while (a + n < limit && in[a + n] == in[b + n]) n++;
  return n;
}

/* LZ4_compress_fast(in, out, length, maxout, accel) for maxout < LZ4_compressBound(length) (the
 * only case blosc reaches: maxout <= neblock).  Returns the compressed size, 0 if it does not
 * fit.  *peak (optional) = the largest `op + need` of the output checks relative to out. */
int or_lz4_compress(int accel, const uint8_t *in, int length, uint8_t *out, int maxout) {
  if (accel < 1) accel = 1;
  if (accel > 65537) accel = 65537;
  if (length < 0 || length > 0x7E000000) return 0;
  if (length == 0) { if (maxout <= 0) return 0; out[0] = 0; return 1; }
  const int u16tab = length < LZ4_64K;
  uint32_t *tab = (uint32_t *)calloc(1u << 13, sizeof(uint32_t));
  if (!tab) return -1;
  const int32_t iend = length, mflimit1 = length - LZ4_MFLIMIT + 1, matchlimit = length - LZ4_LASTLIT;
  int32_t ip = 0, anchor = 0, op = 0, match = 0;
  int rc = 0;
  if (length < LZ4_MFLIMIT + 1) goto last_literals;
  tab[lz4_hash_at(in, u16tab)] = 0;
  ip = 1;
  uint32_t fwdh = lz4_hash_at(in + ip, u16tab);
  for (;;) {
    /* find a match: step grows by one every 2^LZ4_SKIP failed probes */
    int32_t fwd = ip, step = 1, nb = accel << LZ4_SKIP;
    for (;;) {
      uint32_t h = fwdh;
      int32_t cur = fwd;
      int32_t mi = (int32_t)tab[h];
      ip = fwd;
      fwd += step;
      step = nb++ >> LZ4_SKIP;
      if (fwd > mflimit1) goto last_literals;
      match = mi;
      fwdh = lz4_hash_at(in + fwd, u16tab);
      tab[h] = (uint32_t)cur;
      if (!u16tab && mi + LZ4_DMAX < cur) continue;   /* too far (byU32 only) */
      if (ld32(in + match) == ld32(in + ip)) break;
    }
    /* catch up */
    while (ip > anchor && match > 0 && in[ip - 1] == in[match - 1]) { ip--; match--; }
    int32_t token;
    {
      int32_t lit = ip - anchor;
      token = op++;
      if (op + lit + (2 + 1 + LZ4_LASTLIT) + lit / 255 > maxout) goto fail;
      if (lit >= LZ4_RUN_MASK) {
        int32_t len = lit - LZ4_RUN_MASK;
        out[token] = LZ4_RUN_MASK << 4;
        for (; len >= 255; len -= 255) out[op++] = 255;
        out[op++] = (uint8_t)len;
      } else {
        out[token] = (uint8_t)(lit << 4);
      }
      memcpy(out + op, in + anchor, (size_t)lit);
      op += lit;
    }
    for (;;) {   /* _next_match */
      out[op] = (uint8_t)(ip - match); out[op + 1] = (uint8_t)((ip - match) >> 8);
      op += 2;
      int32_t mc = lz4_count(in, ip + LZ4_MINMATCH, match + LZ4_MINMATCH, matchlimit);
      ip += mc + LZ4_MINMATCH;
      if (op + (1 + LZ4_LASTLIT) + (mc + 240) / 255 > maxout) goto fail;
      if (mc >= LZ4_ML_MASK) {
        out[token] += LZ4_ML_MASK;
        mc -= LZ4_ML_MASK;
        for (; mc >= 255; mc -= 255) out[op++] = 255;
        out[op++] = (uint8_t)mc;
      } else {
        out[token] += (uint8_t)mc;
      }
      anchor = ip;
      if (ip >= mflimit1) goto last_literals;
      tab[lz4_hash_at(in + ip - 2, u16tab)] = (uint32_t)(ip - 2);
      /* test the next position for an immediate match */
      uint32_t h = lz4_hash_at(in + ip, u16tab);
      int32_t mi = (int32_t)tab[h];
      tab[h] = (uint32_t)ip;
      if ((u16tab || mi + LZ4_DMAX >= ip) && ld32(in + mi) == ld32(in + ip)) {
        match = mi;
        token = op++;
        out[token] = 0;
        continue;
      }
      break;
    }
    fwdh = lz4_hash_at(in + ++ip, u16tab);
  }
last_literals:
  {
    int32_t last = iend - anchor;
    if (op + last + 1 + (last + 255 - LZ4_RUN_MASK) / 255 > maxout) goto fail;
    if (last >= LZ4_RUN_MASK) {
      int32_t acc = last - LZ4_RUN_MASK;
      out[op++] = LZ4_RUN_MASK << 4;
      for (; acc >= 255; acc -= 255) out[op++] = 255;
      out[op++] = (uint8_t)acc;
    } else {
      out[op++] = (uint8_t)(last << 4);
    }
    memcpy(out + op, in + anchor, (size_t)last);
    op += last;
  }
  rc = op;
fail:
  free(tab);
  return rc;
}

/* LZ4_loadDict + LZ4_compress_fast_continue in external-dictionary mode (lz4 1.9.3), the call
 * sequence of lz4_wrap_compress with a dictionary (blosc/blosc2.c:455-465).  Restated from the
 * published algorithm and pinned against liblz4 through the reference build
 * (tests/test_oracle.py::test_lz4_dict_chunks_match_reference).  Positions are 32-bit indices:
 * loadDict starts the stream at currentOffset = 64 KiB, so the dictionary's last byte is index
 * 65535 and the input starts at startIndex = 65536; the dictionary's positions 0, 3, 6, ... (up to
 * its last 8 bytes) are pre-inserted in the byU32 table (hash5, log 12).  Candidates below
 * startIndex - dictSize are empty slots (dictSmall), farther than 65535 are too far; a match that
 * starts in the dictionary may run on into the input (LZ4_count up to the dictionary's end, then
 * from the input's start); offsets are index differences. */
int or_lz4_compress_dict(int accel, const uint8_t *in, int length, uint8_t *out, int maxout,
                         const uint8_t *dict, int dsz) {
  if (accel < 1) accel = 1;
  if (accel > 65537) accel = 65537;
  if (length < 0 || length > 0x7E000000) return 0;
  if (length == 0) { if (maxout <= 0) return 0; out[0] = 0; return 1; }
  if (dsz < 8) return or_lz4_compress(accel, in, length, out, maxout);   /* loadDict keeps no dictionary */
  if (dsz > 65536) { dict += dsz - 65536; dsz = 65536; }
  uint32_t *tab = (uint32_t *)calloc(1u << 12, sizeof(uint32_t));
  if (!tab) return -1;
  const uint32_t start = 65536, dict0 = start - (uint32_t)dsz;   /* index of dict[0] */
  for (int32_t p = 0; p <= dsz - 8; p += 3) tab[lz4_hash_at(dict + p, 0)] = dict0 + (uint32_t)p;
  const uint32_t prefix_lim = dict0;   /* dictSmall: startIndex - dictSize */
  const int32_t iend = length, mflimit1 = length - LZ4_MFLIMIT + 1, matchlimit = length - LZ4_LASTLIT;
  int32_t ip = 0, anchor = 0, op = 0;
  int rc = 0;
  /* the match: in the dictionary (mdict, at dict[mpos]) or in the input (at in[mpos]) */
  int mdict = 0;
  int32_t mpos = 0;
  uint32_t offset = 0;
#define LZ4D_BYTE(isd, q) ((isd) ? dict[(q)] : in[(q)])
  if (length < LZ4_MFLIMIT + 1) goto last_literals;
  tab[lz4_hash_at(in, 0)] = start;
  ip = 1;
  uint32_t fwdh = lz4_hash_at(in + ip, 0);
  for (;;) {
    int32_t fwd = ip, step = 1, nb = accel << LZ4_SKIP;
    for (;;) {
      uint32_t h = fwdh;
      uint32_t cur = start + (uint32_t)fwd;
      uint32_t mi = tab[h];
      ip = fwd;
      fwd += step;
      step = nb++ >> LZ4_SKIP;
      if (fwd > mflimit1) goto last_literals;
      mdict = mi < start;
      mpos = mdict ? (int32_t)(mi - dict0) : (int32_t)(mi - start);
      fwdh = lz4_hash_at(in + fwd, 0);
      tab[h] = cur;
      if (mi < prefix_lim) continue;                 /* outside the valid area */
      if (mi + LZ4_DMAX < cur) continue;             /* too far */
      if (ld32(mdict ? dict + mpos : in + mpos) == ld32(in + ip)) { offset = cur - mi; break; }
    }
    /* catch up, not below the match's segment start (lowLimit) */
    while (ip > anchor && mpos > 0 && in[ip - 1] == LZ4D_BYTE(mdict, mpos - 1)) { ip--; mpos--; }
    int32_t token;
    {
      int32_t lit = ip - anchor;
      token = op++;
      if (op + lit + (2 + 1 + LZ4_LASTLIT) + lit / 255 > maxout) goto fail;
      if (lit >= LZ4_RUN_MASK) {
        int32_t len = lit - LZ4_RUN_MASK;
        out[token] = LZ4_RUN_MASK << 4;
        for (; len >= 255; len -= 255) out[op++] = 255;
        out[op++] = (uint8_t)len;
      } else {
        out[token] = (uint8_t)(lit << 4);
      }
      memcpy(out + op, in + anchor, (size_t)lit);
      op += lit;
    }
    for (;;) {   /* _next_match */
      out[op] = (uint8_t)offset; out[op + 1] = (uint8_t)(offset >> 8);
      op += 2;
      int32_t mc;
      if (mdict) {
        int32_t limit = ip + (dsz - mpos);
        if (limit > matchlimit) limit = matchlimit;
        mc = 0;
        while (ip + LZ4_MINMATCH + mc < limit && in[ip + LZ4_MINMATCH + mc] == dict[mpos + LZ4_MINMATCH + mc]) mc++;
        ip += mc + LZ4_MINMATCH;
        if (ip == limit) {   /* the match runs on from the dictionary's end into the input */
          int32_t more = 0;
          while (limit + more < matchlimit && in[limit + more] == in[more]) more++;
          mc += more;
          ip += more;
        }
      } else {
        mc = lz4_count(in, ip + LZ4_MINMATCH, mpos + LZ4_MINMATCH, matchlimit);
        ip += mc + LZ4_MINMATCH;
      }
      if (op + (1 + LZ4_LASTLIT) + (mc + 240) / 255 > maxout) goto fail;
      if (mc >= LZ4_ML_MASK) {
        out[token] += LZ4_ML_MASK;
        mc -= LZ4_ML_MASK;
        for (; mc >= 255; mc -= 255) out[op++] = 255;
        out[op++] = (uint8_t)mc;
      } else {
        out[token] += (uint8_t)mc;
      }
      anchor = ip;
      if (ip >= mflimit1) goto last_literals;
      tab[lz4_hash_at(in + ip - 2, 0)] = start + (uint32_t)(ip - 2);
      /* test the next position for an immediate match */
      uint32_t h = lz4_hash_at(in + ip, 0);
      uint32_t cur = start + (uint32_t)ip;
      uint32_t mi = tab[h];
      mdict = mi < start;
      mpos = mdict ? (int32_t)(mi - dict0) : (int32_t)(mi - start);
      tab[h] = cur;
      if (mi >= prefix_lim && mi + LZ4_DMAX >= cur &&
          ld32(mdict ? dict + mpos : in + mpos) == ld32(in + ip)) {
        token = op++;
        out[token] = 0;
        offset = cur - mi;
        continue;
      }
      break;
    }
    fwdh = lz4_hash_at(in + ++ip, 0);
  }
last_literals:
  {
    int32_t last = iend - anchor;
    if (op + last + 1 + (last + 255 - LZ4_RUN_MASK) / 255 > maxout) goto fail;
    if (last >= LZ4_RUN_MASK) {
      int32_t acc = last - LZ4_RUN_MASK;
      out[op++] = LZ4_RUN_MASK << 4;
      for (; acc >= 255; acc -= 255) out[op++] = 255;
      out[op++] = (uint8_t)acc;
    } else {
      out[op++] = (uint8_t)(last << 4);
    }
    memcpy(out + op, in + anchor, (size_t)last);
    op += last;
  }
  rc = op;
fail:
#undef LZ4D_BYTE
  free(tab);
  return rc;
}

/* LZ4_decompress_safe: the decoded size, or < 0 for a malformed stream.  Rejections: truncated
 * input, output overflow, a reference before the output start, a match reaching into the last
 * LASTLITERALS bytes of the output, a stream that does not end on a literal run. */
int or_lz4_decompress(const uint8_t *in, int length, uint8_t *out, int maxout) {
  return or_lz4_decompress_dict(in, length, out, maxout, NULL, 0);
}

/* LZ4_decompress_safe_usingDict (lz4_wrap_decompress with a dictionary, blosc/blosc2.c:504-508):
 * a match may reach dsz bytes before the output start, into the dictionary's tail. */
int or_lz4_decompress_dict(const uint8_t *in, int length, uint8_t *out, int maxout, const uint8_t *dict,
                           int dsz) {
  if (length <= 0) return -1;
  if (maxout == 0) return (length == 1 && in[0] == 0) ? 0 : -1;
  int32_t ip = 0, op = 0;
  for (;;) {
    if (ip >= length) return -1;
    uint32_t token = in[ip++];
    int32_t lit = (int32_t)(token >> 4);
    if (lit == LZ4_RUN_MASK) {
      uint32_t s;
      do {
        if (ip >= length) return -1;
        s = in[ip++];
        lit += (int32_t)s;
        if (lit > maxout) return -1;
      } while (s == 255);
    }
    if (op + lit > maxout - LZ4_MFLIMIT || ip + lit > length - (2 + 1 + LZ4_LASTLIT)) {
      /* the last sequence: literals only, consuming the input exactly */
      if (ip + lit != length || op + lit > maxout) return -1;
      memcpy(out + op, in + ip, (size_t)lit);
      return op + lit;
    }
    memcpy(out + op, in + ip, (size_t)lit);
    op += lit; ip += lit;
    int32_t off = in[ip] | (in[ip + 1] << 8);
    ip += 2;
    if (off > op + dsz) return -1;   /* offset 0 is accepted by liblz4 1.9.3 (it copies zeros) */
    int32_t ml = (int32_t)(token & 15u);
    if (ml == LZ4_ML_MASK) {
      uint32_t s;
      do {
        if (ip >= length - LZ4_LASTLIT) return -1;
        s = in[ip++];
        ml += (int32_t)s;
        if (ml > maxout) return -1;
      } while (s == 255);
    }
    ml += LZ4_MINMATCH;
    if (op + ml > maxout - LZ4_LASTLIT) return -1;
    if (off == 0) memset(out + op, 0, (size_t)ml);
    else
      for (int32_t i = 0; i < ml; i++) {
        const int32_t q = op - off + i;
        out[op + i] = q >= 0 ? out[q] : dict[dsz + q];
      }
    op += ml;
  }
}

/* ----------------------------------------------------------------------- chunk framing ---- */
/* blosc/stune.c:186-215 */
int or_split_block(const or_cparams *cp, int32_t typesize, int32_t blocksize) {
  if (cp->splitmode == SPLIT_ALWAYS) return 1;
  if (cp->splitmode == SPLIT_NEVER) return 0;
  int shuffle_on = 0;
  for (int i = 0; i < 6; i++) shuffle_on |= cp->filters[i] == FLT_SHUFFLE;
  return (cp->compcode == 0 || cp->compcode == 1) && shuffle_on && typesize <= 16 && (blocksize / typesize) >= MIN_BUF;
}

static int32_t eff_typesize(const or_cparams *cp) { return cp->typesize > 255 ? 1 : cp->typesize; }

/* blosc/stune.c:47-165 (BloscLZ is not an HCR codec) */
int32_t or_compute_blocksize(const or_cparams *cp, int32_t nbytes) {
  int32_t ts = cp->typesize;   /* stune runs before the >255 typesize cap (blosc2.c:2468, 2530) */
  int32_t clevel = cp->clevel;
  if (nbytes < ts) return 1;
  int split = or_split_block(cp, ts, nbytes);
  int32_t bs = nbytes;
  if (cp->blocksize) {
    bs = cp->blocksize;
  } else {
    if (nbytes >= 32 * 1024) {
      static const int32_t scale[10] = {8 * 1024, 16 * 1024, 32 * 1024, 64 * 1024, 128 * 1024,
                                        128 * 1024, 256 * 1024, 256 * 1024, 256 * 1024, 256 * 1024};
      bs = scale[clevel];
    }
    if (clevel > 0 && split) {
      static const int32_t per_ts[10] = {0, 32, 32, 32, 64, 64, 64, 128, 256, 512};
      bs = per_ts[clevel] * 1024 * ts;
      if (bs > 4 * 1024 * 1024) bs = 4 * 1024 * 1024;
      if (bs < 32 * 1024) bs = 32 * 1024;
    }
  }
  if (bs > nbytes) bs = nbytes;
  if (bs > ts) bs = bs / ts * ts;
  return bs;
}

/* blosc/blosc2.c:1184-1206: the whole stream is a single repeated byte. */
static int whole_run(const uint8_t *p, int32_t n) {
  for (int32_t i = 1; i < n; i++)
    if (p[i] != p[0]) return 0;
  return 1;
}

/* pipeline_forward, blosc/blosc2.c:1055-1180 (no prefilter, built-in filters only).
 * The reference rotates three buffers with _cycle_buffers (blosc2.c:1048): the k-th active
 * filter (0-based) writes into tmp, tmp2, then the caller's own source block, cyclically.  So a
 * 3rd (or 6th) active filter overwrites the input chunk in place, and DELTA on later blocks then
 * XORs against that rewritten block 0.  `chunk` is therefore a private, writable copy here.
 * Returns the buffer holding the filtered block, NULL on filter error. */
static const uint8_t *pipe_forward(const or_cparams *cp, int32_t ts, uint8_t *chunk,
                                   int32_t offset, int32_t bsize, uint8_t *t1, uint8_t *t2) {
  uint8_t *cur = chunk + offset;
  uint8_t *ring[3] = {t1, t2, chunk + offset};
  int k = 0;
  for (int i = 0; i < 6; i++) {
    uint8_t f = cp->filters[i];
    if (f == FLT_NONE) continue;
    uint8_t *dst = ring[k % 3];
    uint8_t meta = cp->filters_meta[i];
    switch (f) {
      case FLT_SHUFFLE: or_shuffle(meta ? meta : ts, bsize, cur, dst); break;
      case FLT_BITSHUFFLE: or_bitshuffle(ts, bsize, cur, dst); break;
      case FLT_DELTA: or_delta_encode(offset == 0 ? cur : chunk, offset, bsize, ts, cur, dst); break;
      case FLT_TRUNC:
        if (or_trunc_prec((int8_t)meta, ts, bsize, cur, dst) < 0) return NULL;
        break;
      case FLT_BYTEDELTA: or_bytedelta_encode(meta ? meta : ts, bsize, cur, dst); break;
      case FLT_INT_TRUNC:
        if (or_int_trunc((int8_t)meta, cp->typesize, bsize, cur, dst) < 0) return NULL;
        break;
      default: return NULL;
    }
    cur = dst;
    k++;
  }
  return cur;
}

typedef struct {
  uint8_t flags, typesize;
  int32_t nbytes, blocksize, cbytes, nblocks, leftover, overhead;
  uint8_t filters[6], filters_meta[6];
  uint8_t version, bflags;
} or_hdr;

static void flags_to_filter_list(uint8_t flags, uint8_t *filters) {
  memset(filters, 0, 6);
  if (flags & F_SHUF) filters[5] = FLT_SHUFFLE;
  if (flags & F_BITSHUF) filters[5] = FLT_BITSHUFFLE;
  if (flags & F_DELTA) filters[4] = FLT_DELTA;
}

/* blosc_c for one block, serial mode: blosc/blosc2.c:1210-1469.  Returns the bytes written
 * (>0), 0 when the chunk does not fit, <0 on error. */
static int32_t compress_block(const or_cparams *cp, int32_t ts, int split, uint8_t *chunk,
                              int32_t offset, int32_t bsize, int leftover, uint8_t *dest,
                              int32_t ntbytes, int32_t destsize, uint8_t *t1, uint8_t *t2,
                              const uint8_t *dict, int dsz) {
  const uint8_t *blk = pipe_forward(cp, ts, chunk, offset, bsize, t1, t2);
  if (!blk) return ERR_FILTER;
  int32_t nstreams = (split && !leftover) ? ts : 1;
  int32_t neblock = bsize / nstreams;
  int32_t written = 0;
  for (int32_t j = 0; j < nstreams; j++) {
    const uint8_t *s = blk + (int64_t)j * neblock;
    uint8_t *csize_at = dest + written;
    written += 4; ntbytes += 4;
    if (whole_run(s, neblock)) {
      if (ntbytes > destsize) return 0;
      st32(csize_at, -(int32_t)s[0]);
      if (s[0]) {
        ntbytes++;
        if (ntbytes > destsize) return 0;
        dest[written++] = 0x1;
      }
      continue;
    }
    int32_t maxout = neblock;
    if (ntbytes + maxout > destsize) {
      maxout = destsize - ntbytes;
      if (maxout <= 0) return 0;
    }
    /* the codec call (blosc/blosc2.c:1357-1366); LZ4's acceleration is 10 - clevel (get_accel 619-629) */
    int32_t cb = cp->compcode == 1
                     ? (dict ? or_lz4_compress_dict(10 - cp->clevel, s, neblock, dest + written, maxout, dict, dsz)
                             : or_lz4_compress(10 - cp->clevel, s, neblock, dest + written, maxout))
                     : or_blosclz_compress(cp->clevel, s, neblock, dest + written, maxout);
    if (cb < 0) return ERR_DATA;
    if (cb == 0) cb = neblock;
    if (cb == neblock) {
      if (ntbytes + neblock > destsize) return 0;
      memcpy(dest + written, s, (size_t)neblock);
    }
    st32(csize_at, cb);
    written += cb; ntbytes += cb;
  }
  return written;
}

/* blosc2_compress_ctx with nthreads == 1 (blosc/blosc2.c:3121-3148, header 2911-3001,
 * body 3004-3107, per-block loop serial_blosc 2161-2228). */
int or_compress_chunk(const or_cparams *cp, const void *src_, int32_t srcsize, void *dest_,
                      int32_t destsize) {
  const uint8_t *src = (const uint8_t *)src_;
  uint8_t *dest = (uint8_t *)dest_;
  if (cp->compcode != 0 && cp->compcode != 1) return ERR_CODEC;   /* BloscLZ, LZ4 */
  /* buffer size limits (blosc/blosc2.c:2492-2504): BLOSC2_ERROR_MAX_BUFSIZE_EXCEEDED */
  if (srcsize > 0x7fffffff - 32) return -35;
  if (destsize < 32) return -35;
  if (cp->clevel < 0 || cp->clevel > 9) return -10;
  int32_t ts = eff_typesize(cp);
  int32_t bs = or_compute_blocksize(cp, srcsize);
  int32_t nblocks = bs ? srcsize / bs : 0, leftover = bs ? srcsize % bs : 0;
  if (leftover) nblocks++;

  /* dictionaries: LZ4 only (blosc/blosc2.c:2514-2521); clevel 0 drops them (2916-2919) */
  if (cp->use_dict && cp->compcode != 1) return -8;
  const int use_dict = cp->use_dict && cp->clevel > 0 && srcsize >= MIN_BUF;
  uint8_t flags = F_SHUF | F_BITSHUF;   /* extended-header marker */
  int memcpyed = cp->clevel == 0 || srcsize < MIN_BUF;
  int32_t out = HDR_EXT + (memcpyed ? 0 : 4 * nblocks);
  /* a dictionary's training pass writes no bstarts: only the header must fit (2940-2942, 2960) */
  if (!memcpyed && (use_dict ? HDR_EXT : out) > destsize) { memcpyed = 1; out = HDR_EXT; }
  int split = 0;
  if (memcpyed) {
    flags |= F_MEMCPY;
  } else {
    for (int i = 0; i < 6; i++) {
      if (cp->filters[i] == FLT_SHUFFLE) flags |= F_SHUF;
      if (cp->filters[i] == FLT_BITSHUFFLE) flags |= F_BITSHUF;
      if (cp->filters[i] == FLT_DELTA) flags |= F_DELTA;
    }
    split = or_split_block(cp, ts, bs);
    flags |= (uint8_t)((!split) << 4);       /* dont_split, bit 4 */
    flags |= (uint8_t)(cp->compcode << 5);  /* compformat: BLOSCLZ 0, LZ4 1 (blosc2.c:2990-2991) */
  }
  /* header: blosc2_initialize_header_from_context, blosc/blosc2.c:1000-1046 */
  memset(dest, 0, HDR_EXT);
  dest[0] = 5; dest[1] = 1; dest[2] = flags; dest[3] = (uint8_t)ts;
  st32(dest + 4, srcsize);
  /* the header carries the context's incoming blocksize when it is set (header_blocksize,
   * blosc/blosc2.c:2414 and 1001-1005), else the computed one; clamped to nbytes */
  int32_t hb = cp->blocksize > 0 ? cp->blocksize : bs;
  st32(dest + 8, (srcsize > 0 && hb > srcsize) ? srcsize : hb);
  for (int i = 0; i < 6; i++) { dest[16 + i] = cp->filters[i]; dest[24 + i] = cp->filters_meta[i]; }
  dest[22] = (uint8_t)cp->compcode;
  if (use_dict) dest[31] |= USEDICT;   /* blosc2_initialize_header_from_context, 1037-1039 */

  int32_t ntbytes = 0;
  /* private copy of the input: the reference may rewrite it (see pipe_forward), and a later
   * memcpy fallback copies whatever the input holds by then (blosc/blosc2.c:2185-2189) */
  uint8_t *work = (uint8_t *)malloc((size_t)srcsize + 64);
  if (!work) return -1;
  memcpy(work, src, (size_t)srcsize);
  uint8_t *dict = NULL;
  int32_t dsz = 0;
  if (use_dict) {
    /* blosc2_compress_ctx with use_dict (blosc/blosc2.c:3140-3235): a training pass runs the
     * filters over every block and stores the filtered blocks in order (blosc_c with
     * dict_training: one stream per block, no csize words, 1270-1356); when they do not fit the
     * chunk is given up (the memcpy bit stays set, 3036-3052, and the second pass returns 0).
     * The dictionary is the first bytes of that image: min(nblocks' * (nbytes / nblocks' / 16),
     * min(32 KiB, nbytes / 20)), nblocks' = nblocks * typesize when split, at least 8; below
     * 256 bytes (or a zero sample) the chunk is compressed without one (the flag cleared).
     * A training block that does not fit: with no room left at all the pass gives up (0, and the
     * chunk is 0); with some room, the block is stored anyway and blosc_c reports a codec overrun
     * (BLOSC2_ERROR_WRITE_BUFFER, 1343-1356 and 1417-1420). */
    if (HDR_EXT > destsize) { free(work); memset(dest, 0, HDR_EXT); return 0; }
    uint8_t *img = (uint8_t *)malloc((size_t)srcsize + 64);
    uint8_t *t1 = (uint8_t *)malloc((size_t)bs + 64), *t2 = (uint8_t *)malloc((size_t)bs + 64);
    if (!img || !t1 || !t2) { free(img); free(t1); free(t2); free(work); return -1; }
    for (int32_t j = 0; j < nblocks; j++) {
      int lo = (j == nblocks - 1) && leftover;
      int32_t bsize = lo ? leftover : bs;
      const uint8_t *blk = pipe_forward(cp, ts, work, j * bs, bsize, t1, t2);
      if (!blk) { free(img); free(t1); free(t2); free(work); return ERR_FILTER; }
      const int64_t at = (int64_t)HDR_EXT + (int64_t)j * bs;
      if (at + bsize > destsize) {
        free(img); free(t1); free(t2); free(work);
        if (destsize - at <= 0) { memset(dest, 0, HDR_EXT); return 0; }
        return ERR_WRITE;
      }
      memcpy(img + (int64_t)j * bs, blk, (size_t)bsize);
    }
    free(t1); free(t2);
    int32_t nbe = split ? nblocks * ts : nblocks;
    if (nbe < 8) nbe = 8;
    const int32_t sample = srcsize / nbe / 16;
    int32_t dmax = srcsize / 20 < 32 * 1024 ? srcsize / 20 : 32 * 1024;
    if (dmax < 256 || sample == 0) {
      dest[31] &= (uint8_t)~USEDICT;
      free(img);
    } else {
      dsz = nbe * sample < dmax ? nbe * sample : dmax;
      dict = img;   /* its first dsz bytes ... */
      /* ... as they lie in the output when they are moved behind the size word: the samples start
       * at the bstarts (dest + 32) and the size word is stored at dest + 32 + 4 * nblocks before the
       * move (3205-3210), so it replaces those four sample bytes */
      for (int32_t k = 0; k < 4; k++)
        if (4 * nblocks + k < dsz) dict[4 * nblocks + k] = (uint8_t)((uint32_t)dsz >> (8 * k));
    }
  }
  if (!memcpyed) {
    uint8_t *t1 = (uint8_t *)malloc((size_t)bs + 64), *t2 = (uint8_t *)malloc((size_t)bs + 64);
    if (!t1 || !t2) { free(t1); free(t2); free(work); free(dict); return -1; }
    ntbytes = out;
    if (dict) {   /* [int32 dsz | dictionary] after the bstarts (3202-3221) */
      st32(dest + ntbytes, dsz);
      memcpy(dest + ntbytes + 4, dict, (size_t)dsz);
      ntbytes += 4 + dsz;
    }
    for (int32_t j = 0; j < nblocks; j++) {
      st32(dest + HDR_EXT + 4 * j, ntbytes);
      int lo = (j == nblocks - 1) && leftover;
      int32_t bsize = lo ? leftover : bs;
      int32_t cb = compress_block(cp, ts, split, work, j * bs, bsize, lo, dest + ntbytes, ntbytes,
                                  destsize, t1, t2, dict, dsz);
      if (cb < 0) { free(t1); free(t2); free(work); free(dict); return cb; }
      if (cb == 0) { ntbytes = 0; break; }
      ntbytes += cb;
    }
    free(t1); free(t2);
    if (ntbytes == 0) memcpyed = 2;   /* fall back to a plain copy (blosc/blosc2.c:3017-3051) */
  }
  const int dict_used = dict != NULL;
  free(dict);
  if (memcpyed) {
    if (srcsize + HDR_EXT > destsize) {
      ntbytes = 0;
    } else {
      memcpy(dest + HDR_EXT, work, (size_t)srcsize);
      ntbytes = HDR_EXT + srcsize;
      dest[2] = flags | F_MEMCPY;
    }
  } else if (!dict_used) {
    /* all streams zero runs -> SPECIAL_ZERO chunk (blosc/blosc2.c:3054-3063) */
    int32_t nstreams = nblocks;
    if (split) nstreams = leftover ? (nblocks - 1) * ts + 1 : nblocks * ts;
    if (ntbytes == HDR_EXT + 4 * nblocks + 4 * nstreams) {
      dest[31] |= SPECIAL_ZERO << 4;
      ntbytes = HDR_EXT;
    }
  }
  free(work);
  st32(dest + 12, ntbytes);
  return ntbytes;
}

/* read_chunk_header + initialize_context_decompression (blosc/blosc2.c:738-852, 2688-2909),
 * restricted to non-VL, non-lazy chunks. */
static int parse_header(const uint8_t *src, int32_t srcsize, or_hdr *h) {
  memset(h, 0, sizeof *h);
  if (srcsize < HDR_MIN) return ERR_READ;
  h->version = src[0]; h->flags = src[2]; h->typesize = src[3];
  h->nbytes = (int32_t)ld32(src + 4); h->blocksize = (int32_t)ld32(src + 8); h->cbytes = (int32_t)ld32(src + 12);
  if (h->cbytes < HDR_MIN || h->blocksize <= 0 || h->blocksize > 536866816 || h->typesize == 0) return ERR_HEADER;
  if ((h->flags & F_SHUF) && (h->flags & F_BITSHUF)) {
    if (h->cbytes < HDR_EXT || srcsize < HDR_EXT) return ERR_HEADER;
    memcpy(h->filters, src + 16, 6);
    memcpy(h->filters_meta, src + 24, 6);
    h->bflags = src[31];
    if (src[30] != 0) return ERR_HEADER;      /* VL blocks: not part of this oracle */
    if (h->version == 3) { h->filters[5] = 0; h->filters_meta[5] = 0; }
    h->overhead = HDR_EXT;
  } else {
    flags_to_filter_list(h->flags, h->filters);
    if ((h->flags & F_SHUF) && h->typesize <= 1) h->filters[5] = 0;  /* get_filter_flags */
    h->overhead = HDR_MIN;
  }
  if (h->nbytes > 0 && h->blocksize > h->nbytes) h->blocksize = h->nbytes;
  h->nblocks = h->nbytes / h->blocksize;
  h->leftover = h->nbytes % h->blocksize;
  if (h->leftover) h->nblocks++;
  if (h->cbytes > srcsize) return ERR_HEADER;
  return 0;
}

/* pipeline_backward, blosc/blosc2.c:1473-1609 (serial mode, built-in filters). `cur` holds the
 * decoded streams of block nblock; the result lands in out + offset. */
static int pipe_backward(const or_hdr *h, uint8_t *out, int32_t offset, int32_t bsize,
                         uint8_t *cur, uint8_t *t1, uint8_t *t2) {
  int32_t ts = h->typesize;
  uint8_t *bufs[2] = {t1, t2};
  int nb = 0;
  for (int i = 5; i >= 0; i--) {
    uint8_t f = h->filters[i];
    if (f == FLT_NONE || f == FLT_TRUNC || f == FLT_INT_TRUNC) continue;   /* int_trunc.c:116-125 copies */
    uint8_t *dst = bufs[nb];
    uint8_t meta = h->filters_meta[i];
    switch (f) {
      case FLT_SHUFFLE: or_unshuffle(meta ? meta : ts, bsize, cur, dst); break;
      case FLT_BITSHUFFLE: or_bitunshuffle(ts, bsize, cur, dst, h->version); break;
      case FLT_BYTEDELTA: or_bytedelta_decode(meta ? meta : ts, bsize, cur, dst); break;
      case FLT_DELTA:
        memcpy(dst, cur, (size_t)bsize);
        if (offset == 0) {
          /* block 0 decodes in place inside the output chunk */
          memcpy(out, dst, (size_t)bsize);
          or_delta_decode(out, 0, bsize, ts, out);
          memcpy(dst, out, (size_t)bsize);
        } else {
          or_delta_decode(out, offset, bsize, ts, dst);
        }
        break;
      default: return ERR_FILTER;
    }
    cur = dst;
    nb ^= 1;
  }
  memcpy(out + offset, cur, (size_t)bsize);
  return 0;
}

int or_decompress_chunk(const void *src_, int32_t srcsize, void *dest_, int32_t destsize) {
  const uint8_t *src = (const uint8_t *)src_;
  uint8_t *dest = (uint8_t *)dest_;
  or_hdr h;
  int rc = parse_header(src, srcsize, &h);
  if (rc < 0) return rc;
  if (h.nbytes > destsize) return ERR_WRITE;
  int special = (h.overhead == HDR_EXT) ? (h.bflags >> 4) & 7 : 0;
  int memcpyed = (h.flags & F_MEMCPY) != 0;
  if (memcpyed && h.cbytes != h.nbytes + h.overhead) return ERR_DATA;
  if (h.nbytes == 0 && h.cbytes == h.overhead && !special) return 0;
  if ((h.bflags & USEDICT) && (special || memcpyed)) {
    /* the dictionary section is looked for right after the header (no bstarts), as the reference
     * does (blosc/blosc2.c:2754-2809): its own memcpyed fallback chunks with the flag set fail */
    if (srcsize - h.overhead < 4) return ERR_READ;
    const int32_t dsz = (int32_t)ld32(src + h.overhead);
    if (dsz <= 0 || dsz > 32 * 1024) return -9;
    if (srcsize - h.overhead - 4 < dsz) return ERR_READ;
  }
  if (special) {
    /* blosc_d special fills (blosc/blosc2.c:1865-1935): set_values 1644-1700 repeats the typesize
       bytes stored after the 32-byte header; set_nans 1612-1641 writes quiet NaNs (ts 4/8 only). */
    int32_t ts = h.typesize;
    if (special == SPECIAL_ZERO) memset(dest, 0, (size_t)h.nbytes);
    else if (special == SPECIAL_UNINIT) { /* nothing */ }
    else if (special == SPECIAL_VALUE) {
      if (h.nbytes % ts != 0 || srcsize < h.overhead + ts) return ERR_DATA;
      for (int32_t i = 0; i < h.nbytes; i += ts) memcpy(dest + i, src + h.overhead, (size_t)ts);
    } else if (special == SPECIAL_NAN) {
      if (h.nbytes % ts != 0 || (ts != 4 && ts != 8)) return ERR_DATA;
      static const uint8_t nan4[4] = {0, 0, 0xc0, 0x7f}, nan8[8] = {0, 0, 0, 0, 0, 0, 0xf8, 0x7f};
      for (int32_t i = 0; i < h.nbytes; i += ts) memcpy(dest + i, ts == 4 ? nan4 : nan8, (size_t)ts);
    } else return ERR_DATA;
    return h.nbytes;
  }
  if (memcpyed) {
    memcpy(dest, src + h.overhead, (size_t)h.nbytes);
    return h.nbytes;
  }
  const int compformat = h.flags >> 5;
  if (compformat > 1) return ERR_CODEC;   /* BloscLZ and LZ4 */
  int32_t bstarts_end = h.overhead + 4 * h.nblocks;
  if (srcsize < bstarts_end) return ERR_READ;
  const uint8_t *dict = NULL;
  int32_t dsz = 0;
  if (h.bflags & USEDICT) {   /* [int32 size | bytes] after the bstarts (blosc/blosc2.c:2790-2825) */
    if (srcsize - bstarts_end < 4) return ERR_READ;
    dsz = (int32_t)ld32(src + bstarts_end);
    if (dsz <= 0 || dsz > 32 * 1024) return -9;
    if (srcsize - bstarts_end - 4 < dsz) return ERR_READ;
    dict = src + bstarts_end + 4;
  }
  int dont_split = (h.flags >> 4) & 1;
  int32_t bs = h.blocksize;
  uint8_t *t0 = (uint8_t *)malloc((size_t)bs + 64), *t1 = (uint8_t *)malloc((size_t)bs + 64),
          *t2 = (uint8_t *)malloc((size_t)bs + 64);
  if (!t0 || !t1 || !t2) { free(t0); free(t1); free(t2); return -1; }
  int32_t total = 0;
  rc = 0;
  for (int32_t j = 0; j < h.nblocks && rc == 0; j++) {
    int lo = (j == h.nblocks - 1) && h.leftover;
    int32_t bsize = lo ? h.leftover : bs;
    int32_t off = (int32_t)ld32(src + h.overhead + 4 * j);
    if (off <= 0 || off >= srcsize) { rc = ERR_DATA; break; }
    int32_t avail = srcsize - off;
    const uint8_t *p = src + off;
    int32_t nstreams = (!dont_split && !lo) ? h.typesize : 1;
    int32_t neblock = bsize / nstreams;
    if (neblock == 0) { rc = ERR_WRITE; break; }
    int has_filters = 0;
    for (int i = 0; i < 6; i++)
      has_filters |= h.filters[i] != FLT_NONE && h.filters[i] != FLT_TRUNC && h.filters[i] != FLT_INT_TRUNC;
    uint8_t *stage = has_filters ? t0 : dest + (int64_t)j * bs;
    for (int32_t s = 0; s < nstreams; s++) {
      if (avail < 4) { rc = ERR_READ; break; }
      int32_t cb = (int32_t)ld32(p);
      p += 4; avail -= 4;
      uint8_t *d = stage + (int64_t)s * neblock;
      if (cb == 0) {
        memset(d, 0, (size_t)neblock);
      } else if (cb < 0) {
        if (avail < 1) { rc = ERR_READ; break; }
        uint8_t token = *p++; avail--;
        if (!(token & 1) || cb < -255) { rc = ERR_RUNLEN; break; }
        memset(d, (uint8_t)(-cb), (size_t)neblock);
      } else {
        if (avail < cb) { rc = ERR_READ; break; }
        if (cb == neblock) {
          memcpy(d, p, (size_t)neblock);
        } else if ((compformat == 1 ? or_lz4_decompress_dict(p, cb, d, neblock, dict, dsz)
                                    : or_blosclz_decompress(p, cb, d, neblock)) != neblock) {
          rc = ERR_DATA; break;
        }
        p += cb; avail -= cb;
      }
    }
    if (rc) break;
    if (has_filters) rc = pipe_backward(&h, dest, j * bs, bsize, t0, t1, t2);
    total += bsize;
  }
  free(t0); free(t1); free(t2);
  return rc < 0 ? rc : total;
}
