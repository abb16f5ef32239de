/* fm_model.c -- CPU model of the engine's BloscLZ "fast mode" encoder (test infrastructure only;
 * built into oracle/libfm_model.so by oracle/Makefile, never linked into the product).
 *
 * Fast mode keeps the reference's token grammar, greedy rule, length/distance limits, entropy
 * probe thresholds and emission byte for byte (blosc/blosclz.c:248-316, 422-619), and changes one
 * thing: which earlier position a position's hash bucket offers as its candidate.  The reference
 * inserts only the positions its serial walk visits (literals, match starts, the match-end rehash),
 * so every candidate depends on the whole parse before it.  Fast mode inserts EVERY position of the
 * pass, in position order, independently of the parse:
 *
 *   for p = 0 .. loop_end-1:  cand[p] = tab[hash(in[p..p+3])];  tab[hash] = p
 *
 * so a position's candidate is the most recent earlier position with the same hash, and the
 * greedy parse becomes a walk over a successor function fixed before it starts (next(p) = p + 1 for
 * a literal, p + len + 2 after a match) -- the kernel (b2h_lzfast.h) walks it segment-parallel.
 * A candidate is only a suggestion: every match is verified byte for byte and bounded exactly as in
 * the reference, so any stream this produces decodes with blosclz_decompress (blosclz.c:685-795).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { LZ_MAX_COPY = 32, LZ_NEAR = 8191, LZ_FAR = 65535 + 8191 - 1, LZ_SHIFT = 4, LZ_MINLEN = 4 };

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint32_t lz_hash(uint32_t seq, int hashlog) { return (seq * 2654435761U) >> (32 - hashlog); }

static inline int32_t lz_match_end(const uint8_t *in, int32_t p, int32_t r, int32_t bound) {
  while (p < bound) {
    int same = in[p] == in[r];
    p++; r++;
    if (!same) return p;
  }
  return bound;
}

/* Candidates of every position p in [0, loop_end), inserted in position order: the bucket's previous
 * occupant (0 for an empty bucket, as the reference's zeroed htab), then p. */
static void insert_all(const uint8_t *in, int32_t loop_end, int tablog, uint32_t *tab, int32_t *cand) {
  for (int32_t p = 0; p < loop_end; p++) {
    const uint32_t h = lz_hash(ld32(in + p), tablog);
    cand[p] = (int32_t)tab[h];
    tab[h] = (uint32_t)p;
  }
}

/* One fast-mode greedy parse (probe: counts only over limit = min(length, probe_limit), no tail,
 * no far short-match rule -- the same differences get_cratio has).  Returns the emitted size (0:
 * does not fit) or, for the probe, writes *ratio.  *peak: the largest `o + k` bound check made
 * (the `op + k > op_limit` tests of blosc/blosclz.c:248-316, 588-604), as the kernel records it. */
static int fm_parse(const uint8_t *in, int32_t length, int tablog, int probe, int32_t probe_limit, uint8_t *out,
                    int32_t maxout, double *ratio, int32_t *peak_out) {
  int32_t limit = length;
  if (probe && limit > probe_limit) limit = probe_limit;
  const int32_t bound = limit - 1, loop_end = limit - 12;
  uint32_t *tab = (uint32_t *)calloc((size_t)1 << tablog, sizeof(uint32_t));
  int32_t *cand = (int32_t *)calloc((size_t)(limit > 0 ? limit : 1), sizeof(int32_t));
  insert_all(in, loop_end, tablog, tab, cand);
  int32_t o = 5, lit = 4, pos = probe ? 0 : 4, peak = 0;
#define REQ(x) do { const int32_t r_ = (x); if (r_ > peak) peak = r_; if (r_ > maxout) { fail = 1; } } while (0)
  if (!probe) {
    out[0] = LZ_MAX_COPY - 1;
    for (int i = 0; i < 4; i++) out[1 + i] = in[i];
  }
  int fail = 0;
  while (pos < loop_end && !fail) {
    const int32_t anchor = pos;
    const int32_t ref = cand[anchor];
    uint32_t dist = (uint32_t)(anchor - ref);
    int literal = (dist == 0 || dist >= LZ_FAR) || ld32(in + ref) != ld32(in + anchor);
    int32_t len = 0;
    if (!literal) {
      dist--;
      len = lz_match_end(in, anchor + 4, ref + 4, bound) - LZ_SHIFT - anchor;
      if (len < LZ_MINLEN) literal = 1;
      else if (!probe && len <= 5 && dist >= LZ_NEAR) literal = 1;
    }
    if (literal) {
      if (probe) {
        o++;
      } else {
        REQ(o + 2);
        if (fail) break;
        out[o++] = in[anchor];
      }
      pos = anchor + 1;
      if (++lit == LZ_MAX_COPY) {
        lit = 0;
        if (probe) o++; else out[o++] = LZ_MAX_COPY - 1;
      }
      continue;
    }
    if (probe) {
      if (!lit) o--;
    } else {
      if (lit) out[o - lit - 1] = (uint8_t)(lit - 1);
      else o--;
    }
    lit = 0;
    const uint32_t ulen = (uint32_t)len;
    if (probe) {
      if (ulen >= 7) o += (int32_t)((ulen - 7) / 255) + 1;
      o += dist < LZ_NEAR ? 2 : 4;
    } else {
      /* every check of the token and the marker after it is bounded by the marker's end */
      const int far = dist >= LZ_NEAR;
      const uint32_t d = far ? dist - LZ_NEAR : dist;
      const int32_t tok = (ulen >= 7 ? 1 + (int32_t)((ulen - 7) / 255) : 0) + (far ? 4 : 2);
      REQ(o + tok + 1);
      if (fail) break;
      if (ulen < 7) {
        out[o++] = (uint8_t)((ulen << 5) + (far ? 31 : (d >> 8)));
      } else {
        out[o++] = (uint8_t)((7u << 5) + (far ? 31 : (d >> 8)));
        uint32_t rem = ulen - 7;
        for (; rem >= 255; rem -= 255) out[o++] = 255;
        out[o++] = (uint8_t)rem;
      }
      if (far) { out[o++] = 255; out[o++] = (uint8_t)(d >> 8); }
      out[o++] = (uint8_t)(d & 255);
    }
    pos = anchor + len + 2;
    if (probe) o++;
    else out[o++] = LZ_MAX_COPY - 1;
  }
  free(tab);
  free(cand);
  if (fail) return 0;
  if (probe) {
    *ratio = (double)pos / (double)o;
    return 0;
  }
  for (; pos <= bound; pos++) {
    REQ(o + 2);
    if (fail) return 0;
    out[o++] = in[pos];
    if (++lit == LZ_MAX_COPY) {
      lit = 0;
      out[o++] = LZ_MAX_COPY - 1;
    }
  }
#undef REQ
  if (lit) out[o - lit - 1] = (uint8_t)(lit - 1);
  else o--;
  out[0] |= 1u << 5;
  if (peak_out) *peak_out = peak;
  return o;
}

/* Fast-mode blosclz_compress: the reference's entropy-probe decision (blosc/blosclz.c:440-468:
 * maxlen per clevel, limit min(maxlen, 2^hashlog), cratio_ thresholds) over a fast-mode probe,
 * then the fast-mode pass.  tablog_max caps the table size (the kernel's LDS budget). */
int fm_blosclz_compress_peak(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout, int tablog_max,
                             int32_t *peak) {
  static const uint8_t hashlogs[10] = {0, 12, 13, 14, 14, 14, 14, 14, 14, 14};
  static const double min_ratio[10] = {0, 2, 1.5, 1.2, 1.2, 1.2, 1.2, 1.15, 1.1, 1.0};
  if (clevel < 1 || clevel > 9) return 0;
  const int hashlog = hashlogs[clevel];
  const int tablog = hashlog < tablog_max ? hashlog : tablog_max;
  int32_t maxlen = length;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  double ratio = 0.0;
  fm_parse(in + (length - maxlen), maxlen, tablog, 1, 1 << hashlog, NULL, 0, &ratio, NULL);
  if (ratio < min_ratio[clevel] || length < 16 || maxout < 66) return 0;
  return fm_parse(in, length, tablog, 0, 0, out, maxout, NULL, peak);
}

int fm_blosclz_compress(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout, int tablog_max) {
  return fm_blosclz_compress_peak(clevel, in, length, out, maxout, tablog_max, NULL);
}

/* Diagnostics: the matches of a main-pass parse (no emission, no bound checks): start, length,
 * distance per match; returns how many (at most maxtok stored). */
int fm_parse_matches(const uint8_t *in, int length, int tablog, int32_t *q, int32_t *len, int32_t *dist, int maxtok) {
  const int32_t bound = length - 1, loop_end = length - 12;
  if (loop_end <= 0) return 0;
  uint32_t *tab = (uint32_t *)calloc((size_t)1 << tablog, sizeof(uint32_t));
  int32_t *cand = (int32_t *)calloc((size_t)length, sizeof(int32_t));
  insert_all(in, loop_end, tablog, tab, cand);
  int n = 0;
  int32_t pos = 4;
  while (pos < loop_end) {
    const int32_t ref = cand[pos];
    const uint32_t d = (uint32_t)(pos - ref);
    int32_t l = -1;
    if (d != 0 && d < LZ_FAR && ld32(in + ref) == ld32(in + pos)) {
      l = lz_match_end(in, pos + 4, ref + 4, bound) - LZ_SHIFT - pos;
      if (l < LZ_MINLEN || (l <= 5 && d - 1 >= LZ_NEAR)) l = -1;
    }
    if (l < 0) { pos++; continue; }
    if (n < maxtok) { q[n] = pos; len[n] = l; dist[n] = (int32_t)d; }
    n++;
    pos += l + 2;
  }
  free(tab);
  free(cand);
  return n;
}

/* The probe ratio alone (diagnostics: decision agreement with the exact probe). */
double fm_probe_ratio(int clevel, const uint8_t *in, int length, int tablog_max) {
  static const uint8_t hashlogs[10] = {0, 12, 13, 14, 14, 14, 14, 14, 14, 14};
  const int hashlog = hashlogs[clevel];
  const int tablog = hashlog < tablog_max ? hashlog : tablog_max;
  int32_t maxlen = length;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  double ratio = 0.0;
  fm_parse(in + (length - maxlen), maxlen, tablog, 1, 1 << hashlog, NULL, 0, &ratio, NULL);
  return ratio;
}
