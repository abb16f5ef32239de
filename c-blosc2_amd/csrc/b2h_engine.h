// b2h_engine.h -- host-side interface of the MI355X batch engine (C++, internal).
// The public C-ABI wrappers live in blosc2_api.cpp (include/blosc2.h) and b2h_api.cpp
// (include/b2h.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct blosc2_context_s;   // include/blosc2.h (opaque blosc2_context)

namespace b2h {

// Device scratch of one user (the process-wide default of a device, a blosc2 context, a frame).
// Every batch call is stream-ordered on it: the call waits (hipStreamWaitEvent) for the previous
// user's last kernel when that ran on another stream, and records an event after its own, so
// independent contexts on different threads or streams never overwrite each other's plan tables
// or staging (the reference's contexts are independent, include/blosc2.h:1462-1466).  Scratch is
// freed by workspace_destroy (blosc2_free_ctx) or release_device_workspaces (blosc2_destroy).
struct Workspace;
Workspace* workspace_create();
void workspace_destroy(Workspace* ws);
void release_device_workspaces();

// Uniform compression batch: every chunk has `nbytes` bytes and the same cparams, which is what
// a super-chunk's shared cctx produces (blosc/schunk.c:1459-1477).
struct CompressPlan {
  int32_t nbytes;          // bytes per chunk
  int32_t typesize;        // effective typesize (the reference caps > 255 to 1)
  int32_t clevel;
  int32_t blocksize;       // computed (stune)
  int32_t header_blocksize;
  int32_t destsize;        // per-chunk output capacity (serial-mode bound checks use it)
  bool split;              // streams per block = typesize
  bool memcpyed;           // chunk-level memcpy decided before compressing (clevel 0, tiny, no room)
  int32_t overhead;        // 32 (extended header, blosc2_compress_ctx) or 16 (BLOSC_BLOSC1_COMPAT)
  uint8_t filters[6];
  uint8_t filters_meta[6];
  uint8_t header[32];      // header template (cbytes patched per chunk)
  int32_t compcode;        // BLOSC_BLOSCLZ (0) or BLOSC_LZ4 (1)
  bool use_dict;           // LZ4 with a dictionary requested and in force (clevel > 0, not memcpyed)
  int32_t dict_size;       // its size (0: the reference falls back to no dictionary)
  int32_t lz_mode = -1;    // BloscLZ encoder: 0 exact, 1 fast, 2 fast + deep candidates, -1 the process default
};

// Fill the plan from cparams-level values the way blosc2_compress_ctx does (initialize_context_
// compression + write_compression_header, blosc/blosc2.c:2385-2533, 2911-3001).  Returns < 0 on
// invalid parameters.  `ctx_blocksize` is the blocksize the context currently holds (0 = auto).
// compcode: BloscLZ (0), LZ4 (1), or a user-registered codec id (> 31: compformat
// BLOSC_UDCODEC_FORMAT, versionlz = user_version -- encoded by the host callback path).
int make_compress_plan(CompressPlan* p, int32_t nbytes, int32_t destsize, int clevel, int32_t typesize,
                       int32_t ctx_blocksize, int32_t splitmode, const uint8_t* filters,
                       const uint8_t* filters_meta, int32_t* computed_blocksize, bool extended = true,
                       int compcode = 0, int compcode_meta = 0, int user_version = 1, int use_dict = 0);

// Compress `nchunks` chunks: chunk i is d_src + i*src_stride, its output goes to
// d_dst + i*dst_stride (capacity plan.destsize), its cbytes (>0, 0 = does not fit) to d_cbytes[i].
// Asynchronous on `stream`.
int compress_batch(const CompressPlan& plan, const uint8_t* d_src, int64_t src_stride, int32_t nchunks,
                   uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes, hipStream_t stream,
                   Workspace* ws = nullptr);

// Decompress `n` arbitrary chunks (device pointer arrays).  d_status[i] = nbytes or BLOSC2_ERROR_*.
// `dst_bound` is an upper bound of the sum of decompressed sizes (sizes the staging scratch).
// d_maskout (optional): one byte per block, nonzero = skip (blosc2_set_maskout); chunk c's mask
// starts at d_maskout + c * mask_stride (mask_stride 0: one mask shared by every chunk).
// `src_bound` >= 0: an upper bound of the sum of the chunks' compressed sizes; the block and stream
// tables are then sized from it (every block has a 4-byte bstart, every stream a 4-byte csize word)
// and the call never waits on the host (a batch that exceeds the bounds fails per chunk with
// BLOSC2_ERROR_MEMORY_ALLOC).  src_bound < 0: the tables are sized exactly, which costs one
// synchronisation of `stream`.  `mode`: kDecRawStreams (decode the streams only) | kDecDeltaSelf
// (every block un-deltas against itself, as blosc_d with dest_offset 0 does for getitem /
// decompress_block) | kDecNoDict (the dictionary flag is not read: those entry points never parse
// the dictionary section).  Errors are the reference's for the same chunk: its chunk-level checks in
// order, then the first failure of its serial block walk (blosc/blosc2.c:2177-2225).
enum { kDecRawStreams = 1, kDecDeltaSelf = 2, kDecNoDict = 4 };
int decompress_batch(const uint8_t* const* d_src, const int32_t* d_srcsize, uint8_t* const* d_dst,
                     const int32_t* d_dstsize, int32_t n, int64_t dst_bound, int32_t* d_status,
                     const uint8_t* d_maskout, hipStream_t stream, Workspace* ws = nullptr,
                     int64_t src_bound = -1, int mode = 0, int32_t mask_stride = 0);

// Strided convenience form: chunk i at d_src + i*src_stride with cbytes d_cbytes[i], output at
// d_dst + i*dst_stride with capacity dst_cap.
// with d_cbytes[i] <= src_stride (chunks do not overlap), so this form never synchronises.
int decompress_batch_strided(const uint8_t* d_src, int64_t src_stride, const int32_t* d_cbytes, int32_t n,
                             uint8_t* d_dst, int64_t dst_stride, int32_t dst_cap, int32_t* d_status,
                             hipStream_t stream, Workspace* ws = nullptr);

// Concatenate chunk i (d_src + i*src_stride, d_sizes[i] bytes) into d_dst in chunk order;
// d_offsets[0..n] = exclusive prefix sum of the sizes (d_offsets[n] = total).  And the inverse:
// chunk i = d_src[d_offsets[i], d_offsets[i+1]) to d_dst + i*dst_stride, d_sizes[i] = its size.
// Asynchronous on `stream` (the multi-GPU scheduler's gatherv staging).
int pack_chunks(const uint8_t* d_src, int64_t src_stride, const int32_t* d_sizes, int32_t n, uint8_t* d_dst,
                int64_t* d_offsets, hipStream_t stream);
int unpack_chunks(const uint8_t* d_src, const int64_t* d_offsets, int32_t n, uint8_t* d_dst, int64_t dst_stride,
                  int32_t* d_sizes, hipStream_t stream);

// Single-chunk stages of host-driven pipelines (chunks with user-registered filters / codecs):
// one forward filter slot of P over the blocks of `pass` (0 all, 1 block 0, 2 blocks >= 1); the
// built-in codec stage from an already-filtered image; one backward filter over a pass (0 all
// blocks, 1 block 0, 2 blocks >= 1, 3 all blocks with DELTA decoded per block against itself).  Device
// buffers need >= 256 bytes of slack.  decompress_batch(..., kDecRawStreams) decodes the streams
// only, leaving the backward filters to the caller.
int forward_filter_chunk(const CompressPlan& P, int slot, int pass, const uint8_t* d_in, uint8_t* d_out,
                         const uint8_t* d_raw, hipStream_t stream);
int encode_chunk_filtered(const CompressPlan& P, const uint8_t* d_filt, const uint8_t* d_raw, uint8_t* d_dst,
                          int32_t* d_cbytes, hipStream_t stream, Workspace* ws = nullptr);
int backward_filter_chunk(uint8_t filter, uint8_t meta, int32_t typesize, int32_t nbytes, int32_t blocksize,
                          uint8_t version, int pass, const uint8_t* d_in, uint8_t* d_out, const uint8_t* d_final,
                          hipStream_t stream);

// Streaming D2D copy (bench.py's measured copy peak).
int device_copy(uint8_t* d_dst, const uint8_t* d_src, int64_t nbytes, hipStream_t stream);

// Raw filters on device buffers (blosc2_shuffle & co. use these on staged copies).
int shuffle_dev(int32_t typesize, int32_t nbytes, const uint8_t* d_src, uint8_t* d_dst, bool inverse, hipStream_t s);
int bitshuffle_dev(int32_t typesize, int32_t nbytes, const uint8_t* d_src, uint8_t* d_dst, bool inverse,
                   uint8_t format_version, hipStream_t s);

// BloscLZ encoder mode, process-wide default: 0 exact (default), 1 fast.  Returns the previous
// mode.  A plan's own lz_mode (a context's cparams.codec_params, see include/b2h.h) overrides it.
// Exact encoder workgroup shape (b2h_set_encode_shape): -1,-1 auto; 1,N one LDS-table wave + N
// global-table waves; 0,1 global-table only.  Returns the previous shape (16 nlds + nglb, -1 auto).
int set_encode_shape(int nlds, int nglb);
int set_blosclz_mode(int mode);
// Fused launches (k_encode_fast_fused / k_encode_fused) off for the calling host thread: a caller
// that saw a fused launch's hand-off wait time out (BLOSC2_ERROR_FAILURE for the whole batch, e.g.
// on a time-sliced GPU) re-runs the batch with the separate shuffle / encode / layout launches.
void set_fuse_disabled(bool off);
// The BloscLZ mode a cparams.codec_params selects (b2h_codec_params), or -1 (none / not ours).
int codec_params_lz_mode(const void* codec_params);

// Kernel timing hook for bench.py (HIP events around the dominant kernels of the last batch).
struct KernelTimes { float filter_ms, encode_ms, finalize_ms, decode_ms, unfilter_ms; };
void enable_timing(bool on);
int debug_stream_results(void* host, int32_t n);
int debug_decode_cycles(void* host, int32_t n);
int debug_fuse_timed_out();
int debug_seg_prof(uint64_t* host);
KernelTimes last_times();   // the latest batch (waits for its events)
KernelTimes mean_times();   // mean over every batch since enable_timing(true)

// The super-chunk layer's device batches over a context (blosc2_api.cpp; used by b2h_schunk.cpp).
// ctx_compress_device: n consecutive blosc2_compress_ctx calls (chunk i = d_src + i*src_stride,
//   nbytes[i] bytes, destsize nbytes[i] + 32) into d_dst + i*dst_stride, as device batches.  Async.
// ctx_append_device: the same, returning each chunk as a malloc'd host buffer of exactly its cbytes
//   (what blosc2_schunk_append_buffer hands to blosc2_schunk_append_chunk).  Synchronous.
// ctx_decompress_device: n host chunks decoded into d_dst + i*dst_stride (capacity dst_cap) in one
//   device batch; status[i] = blosc2_schunk_decompress_chunk's return for that chunk.  Synchronous.
int ctx_compress_device(::blosc2_context_s* ctx, const uint8_t* d_src, const int32_t* nbytes, int32_t n,
                        int64_t src_stride, uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes);
int ctx_append_device(::blosc2_context_s* ctx, const uint8_t* d_src, const int32_t* nbytes, int32_t n,
                      int64_t src_stride, uint8_t** chunks_out);
int ctx_decompress_device(::blosc2_context_s* ctx, const uint8_t* const* chunks, int32_t n, uint8_t* d_dst,
                          int64_t dst_stride, int32_t dst_cap, int32_t* status);
// The staged fan-out decode (b2h_schunk_decompress_buffers) takes a chunk itself when this holds:
// no postfilter on ctx, no user filter / codec in the chunk, a readable header (sizes returned).
bool ctx_chunk_on_device(const ::blosc2_context_s* ctx, const uint8_t* chunk, int32_t* nbytes, int32_t* cbytes);
// The multi-device fan-out (b2h_schunk_append_buffers): a context with ctx's parameters, sticky
// blocksize and encoder mode, but device state of its own (created on the calling thread's device);
// and the sticky-blocksize walk of n consecutive compressions, before[i] = the state chunk i starts
// from (before[n] = the state after the last), ctx itself unchanged.
::blosc2_context_s* ctx_clone(const ::blosc2_context_s* ctx);
int ctx_blocksize_walk(const ::blosc2_context_s* ctx, const int32_t* nbytes, int32_t n, int32_t* before);
void ctx_set_blocksize(::blosc2_context_s* ctx, int32_t blocksize);

// Device bookkeeping
int device_count();
const char* last_error();

}  // namespace b2h
