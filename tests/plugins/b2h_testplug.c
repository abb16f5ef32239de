/* b2h_testplug.c -- user plugins for the host-callback pipeline tests (test infrastructure only).
 *
 * Built twice by oracle/Makefile: with -DB2H_FILTER into libblosc2_b2hfilt.so and with
 * -DB2H_CODEC into libblosc2_b2hcodec.so.  Each library exports its callbacks and the `info`
 * symbol the reference's lazy loader reads (blosc/blosc2.c:913-971, blosc-private.h:317-360), so
 * the same .so serves as (a) explicit callbacks registered in both the engine and the reference
 * build, and (b) a plugin registered by name only and dlopen'ed on first use.
 *
 *   filter "b2hfilt":  dst[i] = src[i] - src[i-1] + meta (byte delta within one block); backward
 *                      is the running sum.  Block-local, so the block order of the pipeline shows.
 *   codec  "b2hcodec": byte run-length pairs (count 1..255, value); 0 when it does not fit.
 *                      The compcode_meta byte is XORed into every value so the meta travels.
 */
#include <stdbool.h>
#include <stdint.h>
#include <string.h>

typedef struct blosc2_cparams blosc2_cparams;   /* opaque here: only passed through */
typedef struct blosc2_dparams blosc2_dparams;

#ifdef B2H_FILTER
typedef struct { char *forward; char *backward; } filter_info;

int b2h_filt_forward(const uint8_t *src, uint8_t *dst, int32_t size, uint8_t meta, blosc2_cparams *cp, uint8_t id) {
  (void)cp;
  if (id < 160) return -1;
  uint8_t prev = 0;
  for (int32_t i = 0; i < size; i++) {
    dst[i] = (uint8_t)(src[i] - prev + meta);
    prev = src[i];
  }
  return 0;
}

int b2h_filt_backward(const uint8_t *src, uint8_t *dst, int32_t size, uint8_t meta, blosc2_dparams *dp, uint8_t id) {
  (void)dp;
  if (id < 160) return -1;
  uint8_t acc = 0;
  for (int32_t i = 0; i < size; i++) {
    acc = (uint8_t)(acc + (uint8_t)(src[i] - meta));
    dst[i] = acc;
  }
  return 0;
}

filter_info info = {"b2h_filt_forward", "b2h_filt_backward"};
#endif

#ifdef B2H_CODEC
typedef struct { char *encoder; char *decoder; } codec_info;

int b2h_codec_encoder(const uint8_t *in, int32_t len, uint8_t *out, int32_t maxout, uint8_t meta, blosc2_cparams *cp,
                      const void *chunk) {
  (void)cp;
  (void)chunk;
  int32_t o = 0;
  for (int32_t i = 0; i < len;) {
    int32_t r = 1;
    while (i + r < len && r < 255 && in[i + r] == in[i]) r++;
    if (o + 2 > maxout) return 0;
    out[o++] = (uint8_t)r;
    out[o++] = (uint8_t)(in[i] ^ meta);
    i += r;
  }
  return o;
}

int b2h_codec_decoder(const uint8_t *in, int32_t len, uint8_t *out, int32_t maxout, uint8_t meta, blosc2_dparams *dp,
                      const void *chunk) {
  (void)dp;
  (void)chunk;
  int32_t o = 0;
  for (int32_t i = 0; i + 1 < len; i += 2) {
    const int32_t r = in[i];
    if (o + r > maxout) return -1;
    memset(out + o, in[i + 1] ^ meta, (size_t)r);
    o += r;
  }
  return o;
}

codec_info info = {"b2h_codec_encoder", "b2h_codec_decoder"};
#endif
