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

/* Chunks of per-chunk sizes nbytes[i] (HOST array), e.g. a super-chunk whose last chunk is short:
 * chunk i = d_src + i*src_stride, output at d_dst + i*dst_stride, capacity dst_capacity (<= 0:
 * nbytes[i] + BLOSC2_MAX_OVERHEAD, the destsize blosc2_schunk_append_buffer uses, ref
 * blosc/schunk.c:1459-1477).  Runs of equal sizes go through one engine batch each, queued back
 * to back on `stream` without any host wait.  Byte-identical per chunk to blosc2_compress_ctx. */
BLOSC_EXPORT int b2h_compress_batch_sizes(const blosc2_cparams *cparams, const void *d_src, const int32_t *nbytes,
                                          int32_t nchunks, int64_t src_stride, void *d_dst, int64_t dst_stride,
                                          int32_t dst_capacity, int32_t *d_cbytes, void *stream);

/* Decompress chunk i = d_src + i*src_stride (d_cbytes[i] bytes, at most src_stride: chunks do not
 * overlap) into d_dst + i*dst_stride (capacity dst_capacity).  d_status[i] = decompressed bytes or
 * BLOSC2_ERROR_*.  Stream-ordered: never waits on the host (the plan tables are sized from
 * nchunks*src_stride).  Returns 0 or a BLOSC2_ERROR_* code. */
BLOSC_EXPORT int b2h_decompress_batch(const void *d_src, int64_t src_stride, const int32_t *d_cbytes,
                                      int32_t nchunks, void *d_dst, int64_t dst_stride, int32_t dst_capacity,
                                      int32_t *d_status, void *stream);

/* Same with device arrays of chunk pointers/sizes (arbitrary, mixed chunks).  Synchronises `stream`
 * once to size the plan tables exactly. */
BLOSC_EXPORT int b2h_decompress_ptrs(const void *const *d_srcs, const int32_t *d_srcsizes, void *const *d_dsts,
                                     const int32_t *d_dstsizes, int32_t n, int64_t dst_bound, int32_t *d_status,
                                     void *stream);

/* Chunk packing for the multi-GPU super-chunk scheduler (SURVEY.md §8e gatherv staging; replaces
 * the per-chunk appends of blosc/schunk.c:1459-1477 into a contiguous, chunk-ordered buffer).
 * pack:   chunk i (d_src + i*src_stride, d_sizes[i] bytes) -> d_dst at d_offsets[i];
 *         d_offsets[0..n] = exclusive prefix sum of d_sizes (d_offsets[n] = total bytes).
 * unpack: d_src[d_offsets[i], d_offsets[i+1]) -> d_dst + i*dst_stride; d_sizes[i] (optional) = size.
 * Both asynchronous on `stream`.  Return 0 or a BLOSC2_ERROR_* code. */
BLOSC_EXPORT int b2h_pack_chunks(const void *d_src, int64_t src_stride, const int32_t *d_sizes, int32_t n, void *d_dst,
                                 int64_t *d_offsets, void *stream);
BLOSC_EXPORT int b2h_unpack_chunks(const void *d_src, const int64_t *d_offsets, int32_t n, void *d_dst,
                                   int64_t dst_stride, int32_t *d_sizes, void *stream);

/* Plain device-to-device copy with the engine's streaming kernel (the achievable copy bandwidth
 * bench.py reports next to the HBM spec).  Asynchronous on `stream`. */
BLOSC_EXPORT int b2h_device_copy(void *d_dst, const void *d_src, int64_t nbytes, void *stream);

/* Raw byte/bit (un)shuffle of a device buffer (blosc2_shuffle semantics). */
BLOSC_EXPORT int32_t b2h_shuffle(int32_t typesize, int32_t nbytes, const void *d_src, void *d_dst, int inverse,
                                 void *stream);
BLOSC_EXPORT int32_t b2h_bitshuffle(int32_t typesize, int32_t nbytes, const void *d_src, void *d_dst, int inverse,
                                    void *stream);

/* ---- contiguous-frame read path ----
 * Replaces, for contiguous in-memory / on-disk frames (README_CFRAME_FORMAT.rst):
 *   blosc2_schunk_open / blosc2_schunk_from_buffer (blosc/schunk.c) + frame_get_chunk / get_coffset
 *   (blosc/frame.c:3283-3480) + blosc2_schunk_decompress_chunk -> frame_decompress_chunk
 *   (blosc/frame.c:5248-5290), with the stdio backend's reads (blosc/blosc2-stdio.c:241-276).
 * The frame is read once into pinned memory and copied to HBM; the offsets index is decoded on the
 * device; b2h_frame_decompress decodes every chunk in one device batch.  Read-only: frames must be
 * contiguous, 64-bit offsets, fixed chunk size, regular blocks, device-pipeline codecs/filters.
 * Errors: NULL + *err = BLOSC2_ERROR_* (FILE_OPEN, FILE_READ, FRAME_TYPE, VERSION_SUPPORT,
 * INVALID_HEADER, DATA, MEMORY_ALLOC).
 * Device destinations are written on the frame's own non-blocking HIP stream, and the calls return
 * after that stream has drained: work that produces a d_dst buffer on another stream must be
 * finished (or synchronised) before the call. */
typedef struct b2h_frame b2h_frame;
typedef struct {
  int64_t nbytes, cbytes, nchunks;
  int32_t typesize, blocksize, chunksize;
  uint8_t compcode, clevel;
  uint8_t filters[6], filters_meta[6];
} b2h_frame_info;
BLOSC_EXPORT b2h_frame *b2h_frame_open(const char *urlpath, int *err);
BLOSC_EXPORT b2h_frame *b2h_frame_from_buffer(const void *cframe, int64_t len, int *err);
BLOSC_EXPORT void b2h_frame_free(b2h_frame *frame);
BLOSC_EXPORT int b2h_frame_get_info(const b2h_frame *frame, b2h_frame_info *info);
/* Every chunk of the frame into device memory d_dst (chunk i at i * chunksize).  Returns nbytes or
 * a BLOSC2_ERROR_* code.  Synchronous. */
BLOSC_EXPORT int64_t b2h_frame_decompress(b2h_frame *frame, void *d_dst, int64_t dst_capacity);
/* One chunk into a host buffer: blosc2_schunk_decompress_chunk semantics (returns the chunk's
 * nbytes, BLOSC2_ERROR_WRITE_BUFFER when `nbytes` is too small). */
BLOSC_EXPORT int b2h_frame_decompress_chunk(b2h_frame *frame, int64_t nchunk, void *dest, int32_t nbytes);
/* Items [start, stop) (typesize units) of the frame into device memory d_dst: replaces
 * blosc2_schunk_get_slice_buffer (blosc/schunk.c:1662-1760).  Chunks inside the slice decode in
 * place, partial edge chunks through scratch, all in one device batch.  Returns 0 or a
 * BLOSC2_ERROR_* code (INVALID_PARAM for a range outside the frame).  Synchronous. */
BLOSC_EXPORT int b2h_frame_get_slice(b2h_frame *frame, int64_t start, int64_t stop, void *d_dst);

/* blosc2_schunk_get_sparse_buffer (ref blosc/schunk.c:1921-2110, include/blosc2.h): the items at
 * coords[0 .. ncoords) (item indices), in that order, into the HOST buffer (ncoords * typesize
 * bytes).  Only the blocks holding a coordinate (plus block 0 under DELTA) are decoded, all touched
 * chunks in one device batch per group.  Errors as the reference: BLOSC2_ERROR_INVALID_PARAM for
 * negative ncoords, NULL coords/buffer, out-of-range coordinates, non-positive typesize /
 * chunksize / blocksize, or sizes that are not multiples of typesize. */
BLOSC_EXPORT int b2h_frame_get_sparse_buffer(b2h_frame *frame, int64_t ncoords, const int64_t *coords, void *buffer);

/* ---- super-chunk device batches (include/blosc2.h blosc2_schunk, in-memory sparse storage) ----
 * The reference walks a super-chunk one chunk per call (blosc2_schunk_append_buffer,
 * blosc/schunk.c:1459-1477; blosc2_schunk_decompress_chunk, 1481-1530; blosc2_schunk_get_slice_buffer,
 * 1662-1783).  These run many of those calls as one device batch, with the super-chunk's own
 * contexts, and leave the super-chunk exactly as the serial calls leave it (chunk bytes, nbytes,
 * cbytes, chunksize, the cctx's sticky blocksize).  Synchronous.
 *
 * append: chunk i = d_src + i*src_stride (device), nbytes[i] bytes (HOST array), appended in order.
 *   Returns the new nchunks or BLOSC2_ERROR_*.  Pipelines with user-registered filters / codecs
 *   run the serial appends (through host memory).  On an error return the chunks appended before
 *   the failing one stay, and the cctx's sticky blocksize is unspecified (it has advanced over all
 *   n chunks, the serial walk's only up to the failing one).
 * decompress: chunks [nchunk, nchunk + n) into d_dst + i*dst_stride (device, capacity dst_capacity);
 *   status[i] (HOST, optional) = blosc2_schunk_decompress_chunk's return for chunk nchunk + i.
 *   Returns 0 or the first chunk error; BLOSC2_ERROR_INVALID_PARAM for a range outside the schunk.
 * get_slice: items [start, stop) into device memory d_dst (blosc2_schunk_get_slice_buffer).
 * set_slice: items [start, stop) from device memory d_src (blosc2_schunk_set_slice_buffer): the chunks
 *   wholly inside the range are compressed in one device batch, the edge chunks one by one, all in
 *   the serial calls' order (the cctx's sticky blocksize moves as theirs does). */
BLOSC_EXPORT int64_t b2h_schunk_append_device(blosc2_schunk *schunk, const void *d_src, const int32_t *nbytes,
                                              int32_t n, int64_t src_stride);
BLOSC_EXPORT int b2h_schunk_decompress_device(blosc2_schunk *schunk, int64_t nchunk, int32_t n, void *d_dst,
                                              int64_t dst_stride, int32_t dst_capacity, int32_t *status);
BLOSC_EXPORT int b2h_schunk_get_slice_device(blosc2_schunk *schunk, int64_t start, int64_t stop, void *d_dst);
BLOSC_EXPORT int b2h_schunk_set_slice_device(blosc2_schunk *schunk, int64_t start, int64_t stop, const void *d_src);

/* Multi-GPU fan-out from C.  n blosc2_schunk_append_buffer calls (reference blosc/schunk.c:1459-1477)
 * from HOST buffers (chunk i = src + i * src_stride, nbytes[i] bytes), spread over the node's GPUs:
 * `ndevices` workers (<= 0: one per visible device; more workers than devices share them round
 * robin), worker k compressing a contiguous range of the chunks on device k % count with its own
 * stream and workspace.  The chunks are appended in order and equal the serial calls' bytes (each
 * worker starts from the sticky blocksize the serial walk reaches at its first chunk).  Each worker
 * streams its range through pinned memory in groups of <= 128 MiB (host copy, H2D and compression of
 * three groups overlapped); every worker runs on a thread of its own, so the caller's current device
 * is unchanged.  Returns the new number of chunks, or a negative error: nothing is appended when a
 * worker fails; if the final appends fail at chunk i, chunks before i stay appended and the context
 * holds the blocksize the serial calls leave after chunk i - 1. */
BLOSC_EXPORT int64_t b2h_schunk_append_buffers(blosc2_schunk *schunk, const void *src, const int32_t *nbytes,
                                               int32_t n, int64_t src_stride, int32_t ndevices);
/* Chunks [nchunk, nchunk + n) into HOST dst + i * dst_stride (capacity dst_capacity each), spread the
 * same way; status[i] (optional) = what blosc2_schunk_decompress_chunk (schunk.c:1481-1530) returns
 * for chunk nchunk + i.  Decoded groups come back through pinned memory while the next group
 * decodes.  Returns 0 or the first worker's error. */
BLOSC_EXPORT int b2h_schunk_decompress_buffers(blosc2_schunk *schunk, int64_t nchunk, int32_t n, void *dst,
                                               int64_t dst_stride, int32_t dst_capacity, int32_t *status,
                                               int32_t ndevices);

/* Per-context BloscLZ encoder mode.  Built-in BloscLZ does not read blosc2_cparams.codec_params
 * (reference include/blosc2.h:1207; only user codecs receive it), so a context selects its encoder
 * by pointing codec_params at one of these when it is created (blosc2_create_cctx copies the mode;
 * the b2h_compress_batch* entry points read it from their cparams).  No chunk byte changes with the
 * carrier: the mode only picks which encoder writes the streams.  Anything else in codec_params
 * (a NULL pointer, a user codec's own struct) leaves the process default (b2h_set_blosclz_mode). */
#define B2H_CODEC_PARAMS_MAGIC 0x68623262u /* "b2bh" */
typedef struct {
  uint32_t magic;       /* B2H_CODEC_PARAMS_MAGIC */
  int32_t blosclz_mode; /* 0 exact (byte-identical to the reference), 1 fast, 2 fast + deep candidates */
} b2h_codec_params;

/* BloscLZ encoder mode, the process-wide default of contexts that do not choose one through
 * codec_params (above); returns the previous one.
 *   0 exact (default): byte-identical to blosclz_compress (blosc/blosclz.c:422-619).
 *   1 fast: same token grammar, greedy rule, limits, entropy-probe thresholds and emission, but the
 *     hash-table candidates come from positions inserted in 128-position tiles independently of the
 *     parse (c-blosc2_amd/csrc/b2h_lzfast.h, model tools/fm_model.c); every stream decodes with the
 *     reference's blosclz_decompress and the chunk format is unchanged.  Also B2H_LZ_MODE=fast.
 *   2 fast with deep candidates: as 1, but a position's candidate is the best of its hash bucket's
 *     last 8 positions (by up to 24 leading equal bytes; tools/fm_model.c fm_set_depth), which
 *     brings the ratio to the reference's or above on its benchmark data at the
 *     cost of a longer matcher step.  Also B2H_LZ_MODE=deep.
 * Any other value only queries. */
BLOSC_EXPORT int b2h_set_blosclz_mode(int mode);

/* Exact-mode encoder workgroup shape, process-wide (diagnostics and tests; B2H_ENC_MODE sets it at
 * start-up): (-1, -1) auto -- batches that fit the LDS-only shape's resident waves run one
 * LDS-table wave per workgroup, larger ones 1 LDS-table + 3 global-table waves; (1, n) one
 * LDS-table wave + n (0..4) global-table waves; (0, 1) global tables only; (-2, x) only queries.
 * Same bytes in every shape.  Returns the previous shape as 16 * nlds + nglb (-1: auto), or -1 for
 * an invalid one. */
BLOSC_EXPORT int b2h_set_encode_shape(int nlds, int nglb);

/* Per-phase HIP-event timings (ms): filter, encode, finalize, decode, unfilter.  Enabling
 * (re)starts the log and adds event records only: the batch calls never wait on the host; the
 * times are read after the timed work.  last: the latest batch; mean: every batch since enabled. */
BLOSC_EXPORT void b2h_enable_timing(int on);
BLOSC_EXPORT void b2h_last_times(float out[5]);
BLOSC_EXPORT void b2h_mean_times(float out[5]);

BLOSC_EXPORT const char *b2h_last_error(void);
/* Diagnostics: per-stream encoder records of the last compression batch on this device
 * ({kind, size, peak, windows, int64 cycles} x n). Returns n or < 0. Synchronous. */
BLOSC_EXPORT int b2h_debug_stream_results(void *host, int32_t n);
/* Diagnostics: BloscLZ mode 3's per-phase cycle sums since the last call (32 x uint64; zeros unless
 * the library was built with -DB2H_SEG_PROF).  Returns 32. Synchronous. */
BLOSC_EXPORT int b2h_debug_seg_prof(uint64_t *host);
/* Diagnostics (B2H_DECODE_DEBUG=1 only): {int64 cycles, int64 kind} per stream of the last
 * decompression batch.  Returns n or < 0. Synchronous. */
BLOSC_EXPORT int b2h_debug_decode_cycles(void *host, int32_t n);
/* 1 if the last fused encode launch of the current device's default workspace timed out in a
 * hand-off wait (its batch was then redone by the gated separate launches), else 0. */
BLOSC_EXPORT int b2h_debug_fuse_timed_out(void);
BLOSC_EXPORT int b2h_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* BLOSC2_AMD_B2H_H */
