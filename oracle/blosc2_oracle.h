/*
 * blosc2_oracle.h -- CPU restatement of the c-blosc2 block pipeline.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into, loaded by or called from
 * the product library (c-blosc2_amd/lib/libblosc2.so).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * Parity pinning: the restatement is checked (tests/test_oracle_golden.py) against the four
 * known-answer vectors in /root/reference/compat (shuffle-2.20.0, bitshuffle-2.20.0,
 * blosc-blosclz-3.0.0, the blosc-1.x-blosclz decode fixtures) and, where the reference is built
 * (oracle/_ref/libblosc2_ref.so, see oracle/Makefile), against the reference itself on seeded
 * grids (tests/test_oracle_vs_ref.py).
 */
#ifndef B2_ORACLE_H
#define B2_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Byte transpose (reference: blosc/shuffle-generic.h:34-55, API blosc/shuffle.c:416-430). */
int32_t or_shuffle(int32_t typesize, int32_t nbytes, const uint8_t *src, uint8_t *dst);
/* Inverse byte transpose (reference: blosc/shuffle-generic.h:62-83, blosc/shuffle.c:435-449). */
int32_t or_unshuffle(int32_t typesize, int32_t nbytes, const uint8_t *src, uint8_t *dst);
/* Bit transpose (reference: blosc/bitshuffle-generic.c:147-167, blosc/shuffle.c:454-478). */
int32_t or_bitshuffle(int32_t typesize, int32_t nbytes, const uint8_t *src, uint8_t *dst);
/* Inverse bit transpose incl. the format-version-2 rule (reference: blosc/shuffle.c:482-521). */
int32_t or_bitunshuffle(int32_t typesize, int32_t nbytes, const uint8_t *src, uint8_t *dst,
                        uint8_t format_version);
/* XOR delta (reference: blosc/delta.c:18-92 and 96-161). */
void or_delta_encode(const uint8_t *dref, int32_t offset, int32_t nbytes, int32_t typesize,
                     const uint8_t *src, uint8_t *dst);
void or_delta_decode(const uint8_t *dref, int32_t offset, int32_t nbytes, int32_t typesize,
                     uint8_t *dst);
/* Mantissa truncation (reference: blosc/trunc-prec.c:23-86).  Returns <0 on bad params. */
void or_bytedelta_encode(int32_t channels, int32_t nbytes, const uint8_t *src, uint8_t *dst);
void or_bytedelta_decode(int32_t channels, int32_t nbytes, const uint8_t *src, uint8_t *dst);
int or_int_trunc(int8_t prec_bits, int32_t typesize, int32_t nbytes, const uint8_t *src, uint8_t *dst);
int or_trunc_prec(int8_t prec_bits, int32_t typesize, int32_t nbytes, const uint8_t *src,
                  uint8_t *dst);
/* BloscLZ codec (reference: blosc/blosclz.c:320-619 encoder, 685-795 decoder). */
int or_blosclz_compress(int clevel, const uint8_t *in, int length, uint8_t *out, int maxout);
int or_blosclz_decompress(const uint8_t *in, int length, uint8_t *out, int maxout);

/* LZ4 block codec, compformat 1 (blosc/blosc2.c:450-519 -> lz4 1.9.3 LZ4_compress_fast /
 * LZ4_decompress_safe).  compress returns 0 when the output does not fit in maxout. */
int or_lz4_compress(int accel, const uint8_t *in, int length, uint8_t *out, int maxout);
/* LZ4_loadDict(dict, dsz) + LZ4_compress_fast_continue (external-dictionary mode), as
 * lz4_wrap_compress does per stream when the context has a dictionary (blosc2.c:455-465). */
int or_lz4_compress_dict(int accel, const uint8_t *in, int length, uint8_t *out, int maxout,
                         const uint8_t *dict, int dsz);
int or_lz4_decompress(const uint8_t *in, int length, uint8_t *out, int maxout);
int or_lz4_decompress_dict(const uint8_t *in, int length, uint8_t *out, int maxout, const uint8_t *dict,
                           int dsz);

/* Chunk engine, serial (nthreads == 1) layout, BloscLZ codec only.
 * cparams mirror blosc2_cparams (include/blosc2.h of the reference, 1173-1211). */
typedef struct {
  int compcode;        /* 0 = BLOSCLZ (only one supported here) */
  int clevel;          /* 0..9 */
  int typesize;        /* 1..255 (>255 treated like the reference: split machinery sees 1) */
  int blocksize;       /* 0 = automatic (stune) */
  int splitmode;       /* BLOSC_ALWAYS_SPLIT=1, NEVER=2, AUTO=3, FORWARD_COMPAT=4 */
  uint8_t filters[6];
  uint8_t filters_meta[6];
  int use_dict;        /* LZ4 only: a dictionary from the filtered chunk (blosc2.c:3151-3235) */
} or_cparams;

/* Automatic blocksize (reference: blosc/stune.c:47-165 + split_block 186-215). */
int32_t or_compute_blocksize(const or_cparams *cp, int32_t nbytes);
int or_split_block(const or_cparams *cp, int32_t typesize, int32_t blocksize);
/* Compress one chunk with the extended (32-byte) header, as blosc2_compress_ctx does
 * (reference: blosc/blosc2.c:3121-3148 -> 2911-3107).  Returns cbytes, 0 if it does not fit,
 * <0 on error. */
int or_compress_chunk(const or_cparams *cp, const void *src, int32_t srcsize, void *dest,
                      int32_t destsize);
/* Decompress one chunk (extended or Blosc1 16-byte header), as blosc2_decompress_ctx does
 * (reference: blosc/blosc2.c:3943 -> 3910, 2688, 1710). */
int or_decompress_chunk(const void *src, int32_t srcsize, void *dest, int32_t destsize);

#ifdef __cplusplus
}
#endif
#endif
