/* b2h_prepost.c -- prefilter / postfilter callbacks for the pre/postfilter parity tests (test
 * infrastructure only; built by oracle/Makefile into tests/plugins/libb2h_prepost.so).
 *
 * The same functions are handed to this engine and to the reference build (oracle/_ref) through
 * cparams.prefilter / dparams.postfilter, like the callbacks of the reference's own tests
 * (tests/test_prefilter.c, tests/test_postfilter.c).  Each call appends one record of the params
 * it was given to the user data, so a test compares the call sequence as well as the bytes.
 *
 *   mode 0: out = in * 2             (int32 items, test_postfilter.c:62-67)
 *   mode 1: out = inputs[0][off] * 3 (int32 items read at the block's offset, :69-74)
 *   mode 2: out = inputs[0][off] + inputs[1][off]                           (:76-82)
 *   mode 3: out[i] = in[i] + 7 * nblock + i   (bytes: any typesize)
 * A call for block `fail_block` returns 1 (the reference maps it to FILTER_PIPELINE / POSTFILTER).
 */
#include <stdint.h>
#include <string.h>

#include "blosc2.h"

typedef struct {
  int32_t mode;
  int32_t fail_block;
  const uint8_t *inputs[2];
  int32_t nrec;
  int32_t cap;
  int64_t *rec;   /* 8 per call */
} b2h_pp_user;

static void record(b2h_pp_user *u, int64_t a, int64_t b, int64_t c, int64_t d, int64_t e, int64_t f, int64_t g) {
  if (!u->rec || u->nrec >= u->cap) return;
  int64_t *r = u->rec + 8 * (int64_t)u->nrec++;
  r[0] = a; r[1] = b; r[2] = c; r[3] = d; r[4] = e; r[5] = f; r[6] = g; r[7] = 0;
}

static void apply(const b2h_pp_user *u, const uint8_t *in, uint8_t *out, int32_t nbytes, int32_t itemsize,
                  int32_t offset, int32_t nblock) {
  const int32_t n = nbytes / itemsize;
  if (u->mode == 0) {
    for (int32_t i = 0; i < n; i++) {
      int32_t x;
      memcpy(&x, in + 4 * (int64_t)i, 4);
      x = (int32_t)((uint32_t)x * 2u);
      memcpy(out + 4 * (int64_t)i, &x, 4);
    }
  } else if (u->mode == 1 || u->mode == 2) {
    for (int32_t i = 0; i < n; i++) {
      int32_t x, y = 0;
      memcpy(&x, u->inputs[0] + offset + 4 * (int64_t)i, 4);
      if (u->mode == 2) memcpy(&y, u->inputs[1] + offset + 4 * (int64_t)i, 4);
      x = u->mode == 1 ? (int32_t)((uint32_t)x * 3u) : (int32_t)((uint32_t)x + (uint32_t)y);
      memcpy(out + 4 * (int64_t)i, &x, 4);
    }
  } else {
    for (int32_t i = 0; i < nbytes; i++) out[i] = (uint8_t)(in[i] + 7 * nblock + i);
  }
}

int b2h_prefilter(blosc2_prefilter_params *p) {
  b2h_pp_user *u = (b2h_pp_user *)p->user_data;
  record(u, p->nblock, p->output_size, p->output_typesize, p->output_offset, p->nchunk, (int64_t)p->ttmp_nbytes,
         p->output_is_disposable);
  if (p->nblock == u->fail_block) return 1;
  apply(u, p->input, p->output, p->output_size, u->mode == 3 ? 1 : p->output_typesize, p->output_offset, p->nblock);
  return 0;
}

int b2h_postfilter(blosc2_postfilter_params *p) {
  b2h_pp_user *u = (b2h_pp_user *)p->user_data;
  record(u, p->nblock, p->size, p->typesize, p->offset, p->nchunk, (int64_t)p->ttmp_nbytes, 0);
  if (p->nblock == u->fail_block) return 1;
  apply(u, p->input, p->output, p->size, u->mode == 3 ? 1 : p->typesize, p->offset, p->nblock);
  return 0;
}
