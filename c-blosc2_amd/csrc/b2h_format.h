// b2h_format.h -- chunk-format constants and plan records shared by the HIP engine and the host
// C-ABI.  Values follow the reference's on-disk format (README_CHUNK_FORMAT.rst and
// include/blosc2.h:128-300 of c-blosc2); the plan records are this engine's own.
#pragma once
#include <stdint.h>

namespace b2h {

constexpr int kHdrMin = 16;        // BLOSC_MIN_HEADER_LENGTH   (include/blosc2.h:177)
constexpr int kHdrExt = 32;        // BLOSC_EXTENDED_HEADER_LENGTH (include/blosc2.h:180)
constexpr int kMinBuffer = 32;     // BLOSC_MIN_BUFFERSIZE      (include/blosc2.h:193)
constexpr int kMaxFilters = 6;     // BLOSC2_MAX_FILTERS
constexpr int kMaxStreams = 16;    // MAX_STREAMS               (blosc/stune.h:24)

// header flag bits (include/blosc2.h:273-277)
constexpr uint8_t kFlagShuffle = 0x1, kFlagMemcpy = 0x2, kFlagBitshuffle = 0x4, kFlagDelta = 0x8,
                  kFlagDontSplit = 0x10;
// filter ids (include/blosc2.h:248-259)
constexpr uint8_t kNoFilter = 0, kShuffle = 1, kBitshuffle = 2, kDelta = 3, kTruncPrec = 4;
// Registered plugin filters (include/blosc2/filters-registry.h:27-28, registered at blosc2_init by
// plugins/filters/filters-registry.c:43-57) that the device pipeline also runs.
constexpr uint8_t kBytedelta = 35, kIntTrunc = 36;
constexpr uint8_t kSpecialZero = 1, kSpecialNan = 2, kSpecialValue = 3, kSpecialUninit = 4;

// BloscLZ constants (blosc/blosclz.c:45-47, 442-465)
constexpr int kLzMaxCopy = 32;
constexpr uint32_t kLzNear = 8191;
constexpr uint32_t kLzFar = 65535 + 8191 - 1;

// Result of encoding one stream with maxout == neblock, enough to reproduce the serial
// reference decision for any smaller maxout (see b2h_lz.h: peak).
enum StreamKind : int32_t { kStreamZeroRun = 0, kStreamByteRun = 1, kStreamRaw = 2, kStreamLz = 3 };

struct StreamResult {
  int32_t kind;   // StreamKind
  int32_t size;   // LZ: encoded bytes; run: the repeated byte
  int32_t peak;   // LZ: largest `op + k` bound check made while encoding (<= neblock)
  int32_t windows;   // diagnostics: parse windows executed (probe + main pass)
  int64_t cycles;    // diagnostics: s_memtime ticks spent on this stream
  int64_t t_start;   // diagnostics: s_memtime at start (occupancy reconstruction)
};

// One chunk of a decompression batch after header parsing (device-side plan).
struct DChunk {
  int64_t stage_off;     // offset of this chunk's staging area (sum of previous nbytes)
  // First error of the block walk in the reference's serial order (blosc/blosc2.c:2177-2225):
  // (block << 20 | step << 8 | -code), step 0 = the block's bstart / size checks, 1 + j = stream
  // j, kStepFilters = the backward pipeline; atomicMin keeps the earliest.  kNoErr: none.
  uint64_t errkey;
  int32_t status;        // >= 0: nbytes; < 0: BLOSC2_ERROR_* (header-level checks)
  int32_t nbytes;
  int32_t blocksize;
  int32_t nblocks;
  int32_t leftover;
  int32_t nstreams;      // total streams (0 for memcpyed / special chunks)
  int32_t block_base;    // first block index in the batch block table
  int32_t stream_base;   // first stream index in the batch stream table
  uint8_t typesize, flags, version, special;
  uint8_t overhead, dont_split, nfilters_bwd, has_delta;
  uint8_t filters[kMaxFilters];
  uint8_t filters_meta[kMaxFilters];
  uint8_t fsrc[kMaxFilters];   // per backward slot: buffer the stage reads (0 stage,1 tmp,2 dst)
  uint8_t fdst[kMaxFilters];   // per backward slot: buffer the stage writes
  uint8_t codec, delta_self;   // delta_self: every block un-deltas against itself (dest_offset 0)
  int8_t ferr;                 // backward-pipeline error of every decoded block (0, -1, -18)
  uint8_t fuse_unshuffle;      // the lone backward filter is SHUFFLE: undone inside the decode launch
  uint8_t fuse_ds;             // (DELTA, SHUFFLE) at typesize 2/4/8: undone inside the decode launch
  uint8_t ds_runs;             // (DELTA, SHUFFLE) undone by k_dfilter, whose planes of run streams it
                               // synthesises from the csize word: k_decode leaves them unwritten
  uint8_t unshuf_direct;       // fuse_unshuffle with planes = streams: raw planes are read in place
                               // from the chunk and run planes synthesised, neither staged
  int32_t dict_off, dict_size; // LZ4 dictionary section (BLOSC2_USEDICT): offset in the chunk, bytes
};

constexpr uint64_t kNoErr = ~0ull;
constexpr int32_t kStepFilters = 4095;
constexpr uint64_t err_key(int32_t block, int32_t step, int32_t code) {
  return ((uint64_t)(uint32_t)block << 20) | ((uint64_t)step << 8) | (uint64_t)(uint8_t)(-code);
}

// One LZ/raw/run stream of a decompression batch.
struct DStream {
  int64_t src;       // byte offset of the payload inside the chunk (after the csize word)
  int32_t csize;     // the csize word as written by the encoder
  int32_t neblock;   // decoded bytes
  int32_t chunk;
  int32_t dst_off;   // offset of the decoded bytes inside the chunk's uncompressed image
};

}  // namespace b2h
