/* fm_model.c -- CPU model of the engine's BloscLZ "fast mode" encoder (test infrastructure only;
 * built into oracle/libfm_model.so by oracle/Makefile, never linked into the product).
 *
 * Fast mode keeps the reference's token grammar, greedy rule, length/distance limits, entropy
 * probe thresholds and emission byte for byte (blosc/blosclz.c:248-316, 422-619), and changes one
 * thing: which earlier position a position's hash bucket offers as its candidate.  The reference
 * inserts only the positions its serial walk visits (literals, match starts, the match-end rehash),
 * so every candidate depends on the whole parse before it.  Fast mode inserts positions in TILES of
 * 128 consecutive positions, in tile order, independently of the parse:
 *
 *   insert_tile(t): for i = 0..127 (p = 128 t + i < loop_end, in order):
 *                     cand[p] = tab[hash(in[p..p+3])]; tab[hash] = p
 *                   (mode 1 keeps p mod 2^16 per bucket: cand = the latest position below p with
 *                   the bucket's low 16 bits -- the same while p < 2^16)
 *
 * and the parse consumes tiles: entering tile T (the one holding the parse position) it inserts
 * whichever of T, T + 1 are above the highest tile inserted so far, in order (the GPU kernel's
 * matcher wave exchanges and compares T + 1 while the parser wave parses T; fm_set_ahead(2): T + 2
 * as well, the kernel built with B2H_FAST_AHEAD=2); tiles a long match jumps over are never
 * inserted.  A
 * candidate is only a suggestion: every match is verified byte for byte and bounded exactly as in
 * the reference, so any stream this produces decodes with blosclz_decompress (blosclz.c:685-795).
 *
 * The GPU kernel (b2h_lzfast.h lz_pass_fast) runs the tile inserts as one LDS atomic exchange per
 * lane; LDS applies the lanes of one instruction in lane order, so it reproduces this model byte
 * for byte (tests/test_fast_mode.py checks both that and the reference decoder round trip).
 *
 * Deep candidates (fm_set_depth(d), d > 1; the engine's BloscLZ mode 2): the most recent position
 * of a bucket is often a short repeat inside a long-period pattern, where the reference's sparse
 * table happens to keep an older, longer one (b2bench's data: ratio 12.2 vs 20.6).  So every
 * inserted position also records its bucket predecessor, prev[p] = cand[p], and the candidate
 * offered at p is the best of the chain cand[p], prev[cand[p]], ... (at most d positions, while
 * positive and within MAX_FARDISTANCE): the one with the most equal leading bytes, counted up to
 * KSEL and never past the pass's limit, the most recent one on a tie.  Still a function of the
 * input alone, so the kernel's matcher computes it a tile ahead like the plain candidate.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* TILE = the kernel's parse step: 128 positions, two 64-lane halves exchanged in order */
enum { LZ_MAX_COPY = 32, LZ_NEAR = 8191, LZ_FAR = 65535 + 8191 - 1, LZ_SHIFT = 4, LZ_MINLEN = 4, TILE = 128, KSEL = 24 };

static int fm_depth = 1;
void fm_set_depth(int d) { fm_depth = d < 1 ? 1 : d; }
/* tiles inserted ahead of the parse (entering T: T .. T + fm_ahead; the kernel's B2H_FAST_AHEAD) */
static int fm_ahead = 1;
/* the probe pass's (2: the kernel built with B2H_PROBE_AHEAD=1) */
static int fm_ahead_probe = 1;
void fm_set_ahead_probe(int a) { fm_ahead_probe = a < 1 ? 1 : a; }
static int fm_noskip = 0;
/* fast mode's probe window cap (positions; the reference's is 1 << hashlog) */
static int fm_probe_cap = 1 << 30;
void fm_set_probe_cap(int c) { fm_probe_cap = c < 64 ? 64 : c; }
void fm_set_noskip(int v) { fm_noskip = v; }
void fm_set_ahead(int a) { fm_ahead = a < 1 ? 1 : a; }

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

/* equal leading bytes of in[p..] and in[c..], at most KSEL and never at or past `limit` */
static int32_t sel_len(const uint8_t *in, int32_t p, int32_t c, int32_t limit) {
  const int32_t cap = limit - p < KSEL ? limit - p : KSEL;
  int32_t n = 0;
  while (n < cap && in[p + n] == in[c + n]) n++;
  return n;
}

static void insert_tile(const uint8_t *in, int32_t t, int32_t loop_end, int32_t limit, int tablog, uint32_t *tab,
                        int32_t *prev, int32_t *cand) {
  for (int32_t i = 0; i < TILE; i++) {
    const int32_t p = t * TILE + i;
    if (p >= loop_end) break;
    const uint32_t h = lz_hash(ld32(in + p), tablog);
    int32_t c1;
    if (fm_depth < 2) {
      /* 16-bit buckets (the kernel's u16 table at any stream length): a bucket keeps p mod 2^16 and
       * offers the latest position below p with those low bits -- its own position while
       * p < 2^16, a nearer alias for a bucket older than 2^16 positions */
      c1 = p - (int32_t)(((uint32_t)p - tab[h]) & 0xffffu);
      tab[h] = (uint32_t)p & 0xffffu;
      /* a near candidate may stand for one 2^16 positions further back: offered instead when the
       * near one's first 4 bytes differ (and the far one is within MAX_FARDISTANCE) */
      if (c1 >= 65536 && p - c1 < LZ_FAR - 65536 && ld32(in + c1) != ld32(in + p)) c1 -= 65536;
    } else {
      c1 = (int32_t)tab[h];
      tab[h] = (uint32_t)p;
    }
    prev[p] = c1;
    cand[p] = c1;
    /* a usable first candidate (0 < p - c1 < MAX_FARDISTANCE, the parse's own test) opens the chain;
     * older links are only farther */
    if (fm_depth < 2 || c1 <= 0 || p - c1 >= LZ_FAR) continue;
    int32_t best = c1, bl = sel_len(in, p, c1, limit), c = c1;
    for (int k = 1; k < fm_depth; k++) {
      c = prev[c];
      if (c <= 0 || p - c >= LZ_FAR) break;
      const int32_t l = sel_len(in, p, c, limit);
      if (l > bl) { bl = l; best = c; }
    }
    cand[p] = best;
  }
}

/* One fast-mode greedy parse (probe: counts only over limit = min(length, probe_limit), no tail,
 * no far short-match rule -- the same differences get_cratio has).  Returns the emitted size (0:
 * does not fit) or, for the probe, writes *ratio. */
static int fm_parse(const uint8_t *in, int32_t length, int tablog, int probe, int32_t probe_limit, uint8_t *out,
                    int32_t maxout, double *ratio) {
  int32_t limit = length;
  if (probe && limit > probe_limit) limit = probe_limit;
  const int32_t bound = limit - 1, loop_end = limit - 12;
  uint32_t *tab = (uint32_t *)calloc((size_t)1 << tablog, sizeof(uint32_t));
  int32_t *cand = (int32_t *)calloc((size_t)(limit > 0 ? limit : 1) + TILE, sizeof(int32_t));
  int32_t *prev = (int32_t *)calloc((size_t)(limit > 0 ? limit : 1) + TILE, sizeof(int32_t));
  int32_t o = 5, lit = 4, pos = probe ? 0 : 4;
  if (!probe) {
    out[0] = LZ_MAX_COPY - 1;
    for (int i = 0; i < 4; i++) out[1 + i] = in[i];
  }
  int32_t hi = -1;   /* highest inserted tile */
  int fail = 0;
  while (pos < loop_end && !fail) {
    const int32_t T = pos / TILE;
    if (fm_noskip) {   /* every tile up to T + fm_ahead, jumped over or not, in order */
      for (int32_t u = hi + 1; u <= T + (probe ? fm_ahead_probe : fm_ahead); u++)
        if (u * TILE < loop_end) { insert_tile(in, u, loop_end, limit, tablog, tab, prev, cand); hi = u; }
    }
    if (T > hi) { insert_tile(in, T, loop_end, limit, tablog, tab, prev, cand); hi = T; }
    for (int32_t u = T + 1; u <= T + (probe ? fm_ahead_probe : fm_ahead); u++)
      if (u > hi && u * TILE < loop_end) { insert_tile(in, u, loop_end, limit, tablog, tab, prev, cand); hi = u; }
    while (pos < loop_end && pos < (T + 1) * TILE) {
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
          if (o + 2 > maxout) { fail = 1; break; }
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
        const int far = dist >= LZ_NEAR;
        const uint32_t d = far ? dist - LZ_NEAR : dist;
        if (ulen < 7) {
          if (o + (far ? 4 : 2) > maxout) { fail = 1; break; }
          out[o++] = (uint8_t)((ulen << 5) + (far ? 31 : (d >> 8)));
          if (far) { out[o++] = 255; out[o++] = (uint8_t)(d >> 8); }
          out[o++] = (uint8_t)(d & 255);
        } else {
          if (o + 1 > maxout) { fail = 1; break; }
          out[o++] = (uint8_t)((7u << 5) + (far ? 31 : (d >> 8)));
          uint32_t rem = ulen - 7;
          for (; rem >= 255; rem -= 255) {
            if (o + 1 > maxout) { fail = 1; break; }
            out[o++] = 255;
          }
          if (fail) break;
          if (o + (far ? 4 : 2) > maxout) { fail = 1; break; }
          out[o++] = (uint8_t)rem;
          if (far) { out[o++] = 255; out[o++] = (uint8_t)(d >> 8); }
          out[o++] = (uint8_t)(d & 255);
        }
      }
      pos = anchor + len + 2;
      if (probe) {
        o++;
      } else {
        if (o + 1 > maxout) { fail = 1; break; }
        out[o++] = LZ_MAX_COPY - 1;
      }
    }
  }
  free(tab);
  free(cand);
  free(prev);
  if (fail) return 0;
  if (probe) {
    *ratio = (double)pos / (double)o;
    return 0;
  }
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
  out[0] |= 1u << 5;
  return o;
}

/* Fast-mode blosclz_compress: the reference's entropy-probe decision (blosc/blosclz.c:440-468:
 * maxlen per clevel, limit min(maxlen, 2^hashlog), cratio_ thresholds) over a fast-mode probe,
 * then the fast-mode pass.  tablog_max caps the table size (the kernel's LDS budget). */
int fm_blosclz_compress(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout, int tablog_max) {
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
  fm_parse(in + (length - maxlen), maxlen, tablog, 1, (1 << hashlog) < fm_probe_cap ? (1 << hashlog) : fm_probe_cap, NULL, 0, &ratio);
  if (ratio < min_ratio[clevel] || length < 16 || maxout < 66) return 0;
  return fm_parse(in, length, tablog, 0, 0, out, maxout, NULL);
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
  fm_parse(in + (length - maxlen), maxlen, tablog, 1, 1 << hashlog, NULL, 0, &ratio);
  return ratio;
}

/* ==================================================================== segmented fast mode ====
 * fm_set_segment(S), S > 0 (the engine's BloscLZ mode 3, "segmented"): the parse no longer walks
 * the stream as one greedy chain.  Candidates: EVERY position p < loop_end is inserted in order
 * (cand[p] = the bucket's previous position, the u16 rule above), so the candidate array is a
 * function of the input alone.  The stream is cut into segments of S bytes; segment k covers
 * [k S, min((k + 1) S, limit)) and is parsed greedily on its own (the GPU kernel gives each
 * segment a lane): it starts a fresh literal run at its first byte (segment 0: the reference's
 * four initial literals), a match never covers bytes past the segment's end (its length is cut
 * there: e <= seg_end + 2, and a cut match shorter than LZ_MINLEN becomes a literal), and every
 * rule inside a segment is fm_parse's.  The segments' token streams, each closed as the reference
 * closes a stream (an open literal run's header written, an unused reserved header dropped), are
 * concatenated: BloscLZ tokens are self-delimiting and a match may reference any earlier byte, so
 * blosclz_decompress decodes the result (a literal run may now be followed by another one).
 * The probe counts the same way per segment over the probe window; its ratio is the window's
 * parsed length over the summed counts.  Output: 0 when the concatenation is longer than maxout. */
static int fm_segment = 0;
void fm_set_segment(int s) { fm_segment = s < 0 ? 0 : s; }

static int fm3_parse(const uint8_t *in, int32_t length, int tablog, int probe, int32_t probe_limit, uint8_t *out,
                     int32_t maxout, double *ratio) {
  int32_t limit = length;
  if (probe && limit > probe_limit) limit = probe_limit;
  const int32_t bound = limit - 1, loop_end = limit - 12, S = fm_segment;
  uint32_t *tab = (uint32_t *)calloc((size_t)1 << tablog, sizeof(uint32_t));
  int32_t *cand = (int32_t *)calloc((size_t)(limit > 0 ? limit : 1), sizeof(int32_t));
  for (int32_t p = 0; p < loop_end; p++) {   /* every position, in order */
    const uint32_t h = lz_hash(ld32(in + p), tablog);
    int32_t c1 = p - (int32_t)(((uint32_t)p - tab[h]) & 0xffffu);
    tab[h] = (uint32_t)p & 0xffffu;
    if (c1 >= 65536 && p - c1 < LZ_FAR - 65536 && ld32(in + c1) != ld32(in + p)) c1 -= 65536;
    cand[p] = c1;
  }
  free(tab);
  uint8_t *seg = probe ? NULL : (uint8_t *)malloc((size_t)S + (size_t)S / 16 + 64);
  int64_t total = 0;
  int32_t last_pos = 0;
  int fail = 0;
  const int32_t nseg = limit > 0 ? (limit + S - 1) / S : 0;
  for (int32_t k = 0; k < nseg && !fail; k++) {
    const int32_t s0 = k * S, s1 = (k + 1) * S < limit ? (k + 1) * S : limit;
    const int32_t walk_end = s1 < loop_end ? s1 : loop_end;
    const int32_t emax = s1 + 2 < bound ? s1 + 2 : bound;
    int32_t o, lit, pos;
    if (k == 0) {
      o = 5; lit = 4; pos = probe ? 0 : 4;
      if (!probe) { seg[0] = LZ_MAX_COPY - 1; for (int i = 0; i < 4; i++) seg[1 + i] = in[i]; }
    } else {
      o = 1; lit = 0; pos = s0;
      if (!probe) seg[0] = LZ_MAX_COPY - 1;
    }
    while (pos < walk_end) {
      const int32_t anchor = pos;
      const int32_t ref = cand[anchor];
      uint32_t dist = (uint32_t)(anchor - ref);
      int literal = (dist == 0 || dist >= LZ_FAR) || ld32(in + ref) != ld32(in + anchor);
      int32_t len = 0;
      if (!literal) {
        dist--;
        len = lz_match_end(in, anchor + 4, ref + 4, emax) - LZ_SHIFT - anchor;
        if (len < LZ_MINLEN) literal = 1;
        else if (!probe && len <= 5 && dist >= LZ_NEAR) literal = 1;
      }
      if (literal) {
        if (probe) o++; else seg[o++] = in[anchor];
        pos = anchor + 1;
        if (++lit == LZ_MAX_COPY) {
          lit = 0;
          if (probe) o++; else seg[o++] = LZ_MAX_COPY - 1;
        }
        continue;
      }
      if (probe) {
        if (!lit) o--;
      } else {
        if (lit) seg[o - lit - 1] = (uint8_t)(lit - 1);
        else o--;
      }
      lit = 0;
      const uint32_t ulen = (uint32_t)len;
      if (probe) {
        if (ulen >= 7) o += (int32_t)((ulen - 7) / 255) + 1;
        o += dist < LZ_NEAR ? 2 : 4;
        o++;
      } else {
        const int far = dist >= LZ_NEAR;
        const uint32_t d = far ? dist - LZ_NEAR : dist;
        if (ulen < 7) {
          seg[o++] = (uint8_t)((ulen << 5) + (far ? 31 : (d >> 8)));
        } else {
          seg[o++] = (uint8_t)((7u << 5) + (far ? 31 : (d >> 8)));
          uint32_t rem = ulen - 7;
          for (; rem >= 255; rem -= 255) seg[o++] = 255;
          seg[o++] = (uint8_t)rem;
        }
        if (far) { seg[o++] = 255; seg[o++] = (uint8_t)(d >> 8); }
        seg[o++] = (uint8_t)(d & 255);
        seg[o++] = LZ_MAX_COPY - 1;
      }
      pos = anchor + len + 2;
    }
    if (probe) {
      total += o;
      last_pos = pos;
      continue;
    }
    for (; pos < s1; pos++) {   /* the stream's tail (past loop_end): literals */
      seg[o++] = in[pos];
      if (++lit == LZ_MAX_COPY) { lit = 0; seg[o++] = LZ_MAX_COPY - 1; }
    }
    if (lit) seg[o - lit - 1] = (uint8_t)(lit - 1);
    else o--;
    if (total + o > maxout) { fail = 1; break; }
    memcpy(out + total, seg, (size_t)o);
    total += o;
  }
  free(cand);
  free(seg);
  if (probe) {
    *ratio = total > 0 ? (double)last_pos / (double)total : 0.0;
    return 0;
  }
  if (fail || total == 0) return 0;
  out[0] |= 1u << 5;
  return (int)total;
}

/* fm_blosclz_compress with the segmented parse (fm_set_segment(S) first). */
int fm3_blosclz_compress(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout, int tablog_max) {
  static const uint8_t hashlogs[10] = {0, 12, 13, 14, 14, 14, 14, 14, 14, 14};
  static const double min_ratio[10] = {0, 2, 1.5, 1.2, 1.2, 1.2, 1.2, 1.15, 1.1, 1.0};
  if (clevel < 1 || clevel > 9 || fm_segment <= 0) return 0;
  const int hashlog = hashlogs[clevel];
  const int tablog = hashlog < tablog_max ? hashlog : tablog_max;
  int32_t maxlen = length;
  if (clevel < 2) maxlen /= 8;
  else if (clevel < 4) maxlen /= 4;
  else if (clevel < 7) maxlen /= 2;
  double ratio = 0.0;
  fm3_parse(in + (length - maxlen), maxlen, tablog, 1, (1 << hashlog) < fm_probe_cap ? (1 << hashlog) : fm_probe_cap, NULL, 0, &ratio);
  if (ratio < min_ratio[clevel] || length < 16 || maxout < 66) return 0;
  return fm3_parse(in, length, tablog, 0, 0, out, maxout, NULL);
}
