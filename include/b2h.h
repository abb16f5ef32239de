/*
 * b2h.h -- device-resident batch interface of the MI355X Blosc2 engine (new; no reference
 * counterpart).  This is the "thin device interface called by the drop-in" of SURVEY.md §8b:
 * descriptors + device pointers in, chunks in the reference's exact format out.  All buffers
 * are device memory; every call is asynchronous on `stream` (a hipStream_t; NULL = default
 * stream) unless stated otherwise.
 *
 * The batch form replaces the reference's per-chunk loops (blosc/schunk.c:1459-1530 call
 * blosc2_compress_ctx / blosc2_decompress_ctx once per chunk; blosc/blosc2.c:2161-2228 and
 * 4898-5075 walk the blocks of one chunk on host threads): one launch sequence covers every
 * (chunk, block, stream) of the batch.
 */
#ifndef BLOSC2_AMD_B2H_H
#define BLOSC2_AMD_B2H_H

#include <stdint.h>

#include "blosc2.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Compress `nchunks` equally sized chunks: chunk i = d_src + i*src_stride (chunk_nbytes bytes),
 * output at d_dst + i*dst_stride with capacity dst_capacity (the reference's `destsize`),
 * d_cbytes[i] = compressed size (0: does not fit).  Output is byte-identical to
 * blosc2_compress_ctx(cctx(cparams), ...) with nthreads = 1 for every chunk.
 * Returns 0 or a BLOSC2_ERROR_* code (parameter errors). */
BLOSC_EXPORT int b2h_compress_batch(const blosc2_cparams *cparams, const void *d_src, int32_t chunk_nbytes,
                                    int32_t nchunks, int64_t src_stride, void *d_dst, int64_t dst_stride,
                                    int32_t dst_capacity, int32_t *d_cbytes, void *stream);

/* Decompress chunk i = d_src + i*src_stride (d_cbytes[i] bytes) into d_dst + i*dst_stride
 * (capacity dst_capacity).  d_status[i] = decompressed bytes or BLOSC2_ERROR_*.
 * Synchronises `stream` once (plan totals).  Returns 0 or a BLOSC2_ERROR_* code. */
BLOSC_EXPORT int b2h_decompress_batch(const void *d_src, int64_t src_stride, const int32_t *d_cbytes,
                                      int32_t nchunks, void *d_dst, int64_t dst_stride, int32_t dst_capacity,
                                      int32_t *d_status, void *stream);

/* Same with device arrays of chunk pointers/sizes (arbitrary, mixed chunks). */
BLOSC_EXPORT int b2h_decompress_ptrs(const void *const *d_srcs, const int32_t *d_srcsizes, void *const *d_dsts,
                                     const int32_t *d_dstsizes, int32_t n, int64_t dst_bound, int32_t *d_status,
                                     void *stream);

/* Raw byte/bit (un)shuffle of a device buffer (blosc2_shuffle semantics). */
BLOSC_EXPORT int32_t b2h_shuffle(int32_t typesize, int32_t nbytes, const void *d_src, void *d_dst, int inverse,
                                 void *stream);
BLOSC_EXPORT int32_t b2h_bitshuffle(int32_t typesize, int32_t nbytes, const void *d_src, void *d_dst, int inverse,
                                    void *stream);

/* Per-phase HIP-event timings of the last batch on this process (ms): filter, encode, finalize,
 * decode, unfilter.  Enabling adds event records only (no extra synchronisation until read). */
BLOSC_EXPORT void b2h_enable_timing(int on);
BLOSC_EXPORT void b2h_last_times(float out[5]);

BLOSC_EXPORT const char *b2h_last_error(void);
/* Diagnostics: per-stream encoder records of the last compression batch on this device
 * ({kind, size, peak, windows, int64 cycles} x n). Returns n or < 0. Synchronous. */
BLOSC_EXPORT int b2h_debug_stream_results(void *host, int32_t n);
/* Diagnostics (B2H_DECODE_DEBUG=1 only): {int64 cycles, int64 kind} per stream of the last
 * decompression batch.  Returns n or < 0. Synchronous. */
BLOSC_EXPORT int b2h_debug_decode_cycles(void *host, int32_t n);
BLOSC_EXPORT int b2h_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* BLOSC2_AMD_B2H_H */
