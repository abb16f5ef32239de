/*
 * blosc2.h -- drop-in C ABI of the MI355X-native Blosc2 chunk engine (libblosc2.so from
 * c-blosc2_amd/).  Binary compatible with the c-blosc2 3.3.3 entry points listed here: same
 * names, same struct layouts, same argument meaning, same return / error conventions.  Each
 * declaration cites the reference declaration it replaces (c-blosc2 include/blosc2.h:line).
 *
 * What runs where: every built-in filter (SHUFFLE, BITSHUFFLE, DELTA, TRUNC_PREC), the registered
 * filters bytedelta (35) and int_trunc (36), and the BloscLZ and LZ4 codecs execute as HIP kernels
 * on the GPU; host code only parses/writes headers, stages buffers and keeps context state.
 * User-registered filters and codecs, and cparams.prefilter / dparams.postfilter, run as host
 * callbacks per block (per stream for codecs) between the device stages, with the reference's
 * params and return codes (blosc/blosc2.c:1069-1110, 1586-1606, 1910-1931).  Chunks needing
 * LZ4HC, ZLIB or ZSTD return BLOSC2_ERROR_CODEC_SUPPORT; the device batch entry points of b2h.h
 * refuse prefilters and user callbacks with BLOSC2_ERROR_FILTER_PIPELINE.
 */
#ifndef BLOSC2_AMD_BLOSC2_H
#define BLOSC2_AMD_BLOSC2_H

#include <limits.h>
#include <stdbool.h>
#include <stdint.h>
#include <stddef.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLOSC_EXPORT __attribute__((visibility("default")))

/* ---- version (include/blosc2.h:84-89) ---- */
#define BLOSC2_VERSION_MAJOR 3
#define BLOSC2_VERSION_MINOR 3
#define BLOSC2_VERSION_RELEASE 3
#define BLOSC2_VERSION_STRING "3.3.3.dev"
#define BLOSC2_VERSION_DATE "$Date:: 2026-08-06 #$"

/* ---- the Blosc 1.x spellings (include/blosc2.h:43-80): macros onto the exported names ---- */
#ifdef BLOSC1_COMPAT
#define BLOSC_VERSION_MAJOR BLOSC2_VERSION_MAJOR
#define BLOSC_VERSION_MINOR BLOSC2_VERSION_MINOR
#define BLOSC_VERSION_RELEASE BLOSC2_VERSION_RELEASE
#define BLOSC_VERSION_STRING BLOSC2_VERSION_STRING
#define BLOSC_VERSION_DATE BLOSC2_VERSION_DATE
#define blosc_compress blosc1_compress
#define blosc_decompress blosc1_decompress
#define blosc_getitem blosc1_getitem
#define blosc_get_compressor blosc1_get_compressor
#define blosc_set_compressor blosc1_set_compressor
#define blosc_cbuffer_sizes blosc1_cbuffer_sizes
#define blosc_cbuffer_validate blosc1_cbuffer_validate
#define blosc_cbuffer_metainfo blosc1_cbuffer_metainfo
#define blosc_get_blocksize blosc1_get_blocksize
#define blosc_set_blocksize blosc1_set_blocksize
#define blosc_set_splitmode blosc1_set_splitmode
#define blosc_init blosc2_init
#define blosc_destroy blosc2_destroy
#define blosc_free_resources blosc2_free_resources
#define blosc_get_nthreads blosc2_get_nthreads
#define blosc_set_nthreads blosc2_set_nthreads
#define blosc_compcode_to_compname blosc2_compcode_to_compname
#define blosc_compname_to_compcode blosc2_compname_to_compcode
#define blosc_list_compressors blosc2_list_compressors
#define blosc_get_version_string blosc2_get_version_string
#define blosc_get_complib_info blosc2_get_complib_info
#define blosc_cbuffer_versions blosc2_cbuffer_versions
#define blosc_cbuffer_complib blosc2_cbuffer_complib
#endif

/* ---- tracing / error macros user code (plugins, examples) expands (include/blosc2.h:92-125,
 * include/blosc2/blosc2-common.h:28) ---- */
#define BLOSC_UNUSED_PARAM(x) ((void)(x))
#define BLOSC_ATTRIBUTE_UNUSED __attribute__((unused))
#define BLOSC_TRACE(cat, msg, ...)                                                        \
  do {                                                                                    \
    const char *__e = getenv("BLOSC_TRACE");                                              \
    if (!__e) { break; }                                                                  \
    fprintf(stderr, "[%s] - " msg " (%s:%d)\n", #cat, ##__VA_ARGS__, __FILE__, __LINE__); \
  } while (0)
#define BLOSC_TRACE_ERROR(msg, ...) BLOSC_TRACE(error, msg, ##__VA_ARGS__)
#define BLOSC_TRACE_WARNING(msg, ...) BLOSC_TRACE(warning, msg, ##__VA_ARGS__)
#define BLOSC_TRACE_INFO(msg, ...) BLOSC_TRACE(info, msg, ##__VA_ARGS__)
#define BLOSC_ERROR_NULL(pointer, rc)           \
  do {                                          \
    if ((pointer) == NULL) {                    \
      BLOSC_TRACE_ERROR("Pointer is null");     \
      return (rc);                              \
    }                                           \
  } while (0)
#define BLOSC_ERROR(rc)                          \
  do {                                           \
    int rc_ = (rc);                              \
    if (rc_ < BLOSC2_ERROR_SUCCESS) {            \
      char *error_msg = print_error(rc_);        \
      BLOSC_TRACE_ERROR("%s", error_msg);        \
      return rc_;                                \
    }                                            \
  } while (0)
#define BLOSC_INFO(msg, ...)                              \
  do {                                                    \
    const char *__e = getenv("BLOSC_INFO");               \
    if (!__e) { break; }                                  \
    fprintf(stderr, "[INFO] - " msg "\n", ##__VA_ARGS__); \
  } while (0)

/* ---- format constants (include/blosc2.h:128-196) ---- */
enum {
  BLOSC1_VERSION_FORMAT_PRE1 = 1,
  BLOSC1_VERSION_FORMAT = 2,
  BLOSC2_VERSION_FORMAT_ALPHA = 3,
  BLOSC2_VERSION_FORMAT_BETA1 = 4,
  BLOSC2_VERSION_FORMAT_STABLE = 5,
  BLOSC2_VERSION_FORMAT_VL_BLOCKS = 6,
  BLOSC2_VERSION_FORMAT = BLOSC2_VERSION_FORMAT_VL_BLOCKS,
};

enum {
  BLOSC_MIN_HEADER_LENGTH = 16,
  BLOSC_EXTENDED_HEADER_LENGTH = 32,
  BLOSC2_MAX_OVERHEAD = BLOSC_EXTENDED_HEADER_LENGTH,
  BLOSC2_MAX_BUFFERSIZE = (INT_MAX - BLOSC2_MAX_OVERHEAD),
  BLOSC_MAX_TYPESIZE = UINT8_MAX,
  BLOSC_MIN_BUFFERSIZE = 32,
};
#define BLOSC_MAX_OVERHEAD BLOSC2_MAX_OVERHEAD
#define BLOSC_MAX_BUFFERSIZE BLOSC2_MAX_BUFFERSIZE

/* filters (include/blosc2.h:221-264) */
enum {
  BLOSC2_DEFINED_FILTERS_START = 0,
  BLOSC2_DEFINED_FILTERS_STOP = 31,
  BLOSC2_GLOBAL_REGISTERED_FILTERS_START = 32,
  BLOSC2_GLOBAL_REGISTERED_FILTERS_STOP = 159,
  BLOSC2_GLOBAL_REGISTERED_FILTERS = 5,
  BLOSC2_USER_REGISTERED_FILTERS_START = 160,
  BLOSC2_USER_REGISTERED_FILTERS_STOP = 255,
  BLOSC2_MAX_FILTERS = 6,
  BLOSC2_MAX_UDFILTERS = 16,
};
enum {
  BLOSC_NOSHUFFLE = 0,
  BLOSC_NOFILTER = 0,
  BLOSC_SHUFFLE = 1,
  BLOSC_BITSHUFFLE = 2,
  BLOSC_DELTA = 3,
  BLOSC_TRUNC_PREC = 4,
  BLOSC_LAST_FILTER = 5,
  BLOSC_LAST_REGISTERED_FILTER = BLOSC2_GLOBAL_REGISTERED_FILTERS_START + BLOSC2_GLOBAL_REGISTERED_FILTERS - 1,
};

/* header flags (include/blosc2.h:270-295) */
enum {
  BLOSC_DOSHUFFLE = 0x1,
  BLOSC_MEMCPYED = 0x2,
  BLOSC_DOBITSHUFFLE = 0x4,
  BLOSC_DODELTA = 0x8,
};
enum {
  BLOSC2_USEDICT = 0x1,
  BLOSC2_BIGENDIAN = 0x2,
  BLOSC2_INSTR_CODEC = 0x80,
};
enum {
  BLOSC2_VL_BLOCKS = 0x1,
};
enum {
  BLOSC2_MAXDICTSIZE = 128 * 1024,
  BLOSC2_MINUSEFULDICT = 256,
  BLOSC2_MAXBLOCKSIZE = 536866816,
  BLOSC2_MAXTYPESIZE = BLOSC2_MAXBLOCKSIZE,
};

/* codecs (include/blosc2.h:306-400) */
enum {
  BLOSC2_DEFINED_CODECS_START = 0,
  BLOSC2_DEFINED_CODECS_STOP = 31,
  BLOSC2_GLOBAL_REGISTERED_CODECS_START = 32,
  BLOSC2_GLOBAL_REGISTERED_CODECS_STOP = 159,
  BLOSC2_GLOBAL_REGISTERED_CODECS = 5,
  BLOSC2_USER_REGISTERED_CODECS_START = 160,
  BLOSC2_USER_REGISTERED_CODECS_STOP = 255,
};
enum {
  BLOSC_BLOSCLZ = 0,
  BLOSC_LZ4 = 1,
  BLOSC_LZ4HC = 2,
  BLOSC_ZLIB = 4,
  BLOSC_ZSTD = 5,
  BLOSC_LAST_CODEC = 6,
  BLOSC_LAST_REGISTERED_CODEC = BLOSC2_GLOBAL_REGISTERED_CODECS_START + BLOSC2_GLOBAL_REGISTERED_CODECS - 1,
};
#define BLOSC_BLOSCLZ_COMPNAME "blosclz"
#define BLOSC_LZ4_COMPNAME "lz4"
#define BLOSC_LZ4HC_COMPNAME "lz4hc"
#define BLOSC_ZLIB_COMPNAME "zlib"
#define BLOSC_ZSTD_COMPNAME "zstd"
enum {
  BLOSC_BLOSCLZ_LIB = 0,
  BLOSC_LZ4_LIB = 1,
  BLOSC_ZLIB_LIB = 3,
  BLOSC_ZSTD_LIB = 4,
  BLOSC_UDCODEC_LIB = 6,
  BLOSC_SCHUNK_LIB = 7,
};
#define BLOSC_BLOSCLZ_LIBNAME "BloscLZ"
#define BLOSC_LZ4_LIBNAME "LZ4"
#define BLOSC_ZLIB_LIBNAME "Zlib"
#define BLOSC_ZSTD_LIBNAME "Zstd"
enum {
  BLOSC_BLOSCLZ_FORMAT = BLOSC_BLOSCLZ_LIB,
  BLOSC_LZ4_FORMAT = BLOSC_LZ4_LIB,
  BLOSC_LZ4HC_FORMAT = BLOSC_LZ4_LIB,
  BLOSC_ZLIB_FORMAT = BLOSC_ZLIB_LIB,
  BLOSC_ZSTD_FORMAT = BLOSC_ZSTD_LIB,
  BLOSC_UDCODEC_FORMAT = BLOSC_UDCODEC_LIB,
};
enum {
  BLOSC_BLOSCLZ_VERSION_FORMAT = 1,
  BLOSC_LZ4_VERSION_FORMAT = 1,
  BLOSC_LZ4HC_VERSION_FORMAT = 1,
  BLOSC_ZLIB_VERSION_FORMAT = 1,
  BLOSC_ZSTD_VERSION_FORMAT = 1,
  BLOSC_UDCODEC_VERSION_FORMAT = 1,
};
/* split modes (include/blosc2.h:410-415) */
enum {
  BLOSC_ALWAYS_SPLIT = 1,
  BLOSC_NEVER_SPLIT = 2,
  BLOSC_AUTO_SPLIT = 3,
  BLOSC_FORWARD_COMPAT_SPLIT = 4,
};
/* chunk header offsets (include/blosc2.h:420-433) */
enum {
  BLOSC2_CHUNK_VERSION = 0x0,
  BLOSC2_CHUNK_VERSIONLZ = 0x1,
  BLOSC2_CHUNK_FLAGS = 0x2,
  BLOSC2_CHUNK_TYPESIZE = 0x3,
  BLOSC2_CHUNK_NBYTES = 0x4,
  BLOSC2_CHUNK_BLOCKSIZE = 0x8,
  BLOSC2_CHUNK_CBYTES = 0xc,
  BLOSC2_CHUNK_FILTER_CODES = 0x10,
  BLOSC2_CHUNK_FILTER_META = 0x18,
  BLOSC2_CHUNK_BLOSC2_FLAGS2 = 0x1e,
  BLOSC2_CHUNK_BLOSC2_FLAGS = 0x1F,
};
/* special values (include/blosc2.h:438-446) */
enum {
  BLOSC2_NO_SPECIAL = 0x0,
  BLOSC2_SPECIAL_ZERO = 0x1,
  BLOSC2_SPECIAL_NAN = 0x2,
  BLOSC2_SPECIAL_VALUE = 0x3,
  BLOSC2_SPECIAL_UNINIT = 0x4,
  BLOSC2_SPECIAL_LASTID = 0x4,
  BLOSC2_SPECIAL_MASK = 0x7,
};
/* error codes (include/blosc2.h:453-492) */
enum {
  BLOSC2_ERROR_SUCCESS = 0,
  BLOSC2_ERROR_FAILURE = -1,
  BLOSC2_ERROR_STREAM = -2,
  BLOSC2_ERROR_DATA = -3,
  BLOSC2_ERROR_MEMORY_ALLOC = -4,
  BLOSC2_ERROR_READ_BUFFER = -5,
  BLOSC2_ERROR_WRITE_BUFFER = -6,
  BLOSC2_ERROR_CODEC_SUPPORT = -7,
  BLOSC2_ERROR_CODEC_PARAM = -8,
  BLOSC2_ERROR_CODEC_DICT = -9,
  BLOSC2_ERROR_VERSION_SUPPORT = -10,
  BLOSC2_ERROR_INVALID_HEADER = -11,
  BLOSC2_ERROR_INVALID_PARAM = -12,
  BLOSC2_ERROR_FILE_READ = -13,
  BLOSC2_ERROR_FILE_WRITE = -14,
  BLOSC2_ERROR_FILE_OPEN = -15,
  BLOSC2_ERROR_NOT_FOUND = -16,
  BLOSC2_ERROR_RUN_LENGTH = -17,
  BLOSC2_ERROR_FILTER_PIPELINE = -18,
  BLOSC2_ERROR_CHUNK_INSERT = -19,
  BLOSC2_ERROR_CHUNK_APPEND = -20,
  BLOSC2_ERROR_CHUNK_UPDATE = -21,
  BLOSC2_ERROR_2GB_LIMIT = -22,
  BLOSC2_ERROR_SCHUNK_COPY = -23,
  BLOSC2_ERROR_FRAME_TYPE = -24,
  BLOSC2_ERROR_FILE_TRUNCATE = -25,
  BLOSC2_ERROR_THREAD_CREATE = -26,
  BLOSC2_ERROR_POSTFILTER = -27,
  BLOSC2_ERROR_FRAME_SPECIAL = -28,
  BLOSC2_ERROR_SCHUNK_SPECIAL = -29,
  BLOSC2_ERROR_PLUGIN_IO = -30,
  BLOSC2_ERROR_FILE_REMOVE = -31,
  BLOSC2_ERROR_NULL_POINTER = -32,
  BLOSC2_ERROR_INVALID_INDEX = -33,
  BLOSC2_ERROR_METALAYER_NOT_FOUND = -34,
  BLOSC2_ERROR_MAX_BUFSIZE_EXCEEDED = -35,
  BLOSC2_ERROR_TUNER = -36,
  BLOSC2_ERROR_LOCK = -37,
};

/* include/blosc2.h:510 (blosc2_error_string, blosc/blosc2.c:6916-6995): a static string for every
 * BLOSC2_ERROR_* code, "Unknown error" for anything else. */
BLOSC_EXPORT const char *blosc2_error_string(int error_code);
/* include/blosc2.h:524-528: the legacy spelling, header-inline as in the reference. */
static char *print_error(int rc) __attribute__((unused));
static char *print_error(int rc) { return (char *)blosc2_error_string(rc); }

/* ---- timing helpers the reference's benchmarks use (include/blosc2.h:2600-2636,
 * blosc/timestamp.c): a CLOCK_MONOTONIC timestamp and differences in ns / s. ---- */
typedef struct timespec blosc_timestamp_t;
BLOSC_EXPORT void blosc_set_timestamp(blosc_timestamp_t *timestamp);
BLOSC_EXPORT double blosc_elapsed_nsecs(blosc_timestamp_t start_time, blosc_timestamp_t end_time);
BLOSC_EXPORT double blosc_elapsed_secs(blosc_timestamp_t start_time, blosc_timestamp_t end_time);

/* ---- context and parameter structs (ABI-identical to include/blosc2.h:1125-1248) ---- */
typedef struct blosc2_context_s blosc2_context;

typedef struct {
  void *user_data;
  const uint8_t *input;
  uint8_t *output;
  int32_t output_size;
  int32_t output_typesize;
  int32_t output_offset;
  int64_t nchunk;
  int32_t nblock;
  int32_t tid;
  uint8_t *ttmp;
  size_t ttmp_nbytes;
  blosc2_context *ctx;
  bool output_is_disposable;
} blosc2_prefilter_params;

typedef struct {
  void *user_data;
  const uint8_t *input;
  uint8_t *output;
  int32_t size;
  int32_t typesize;
  int32_t offset;
  int64_t nchunk;
  int32_t nblock;
  int32_t tid;
  uint8_t *ttmp;
  size_t ttmp_nbytes;
  blosc2_context *ctx;
} blosc2_postfilter_params;

typedef int (*blosc2_prefilter_fn)(blosc2_prefilter_params *params);
typedef int (*blosc2_postfilter_fn)(blosc2_postfilter_params *params);

/* include/blosc2.h:1173-1211 */
typedef struct {
  uint8_t compcode;
  uint8_t compcode_meta;
  uint8_t clevel;
  int use_dict;
  int32_t typesize;
  int16_t nthreads;
  int32_t blocksize;
  int32_t splitmode;
  void *schunk;
  uint8_t filters[BLOSC2_MAX_FILTERS];
  uint8_t filters_meta[BLOSC2_MAX_FILTERS];
  blosc2_prefilter_fn prefilter;
  blosc2_prefilter_params *preparams;
  void *tuner_params;
  int tuner_id;
  bool instr_codec;
  void *codec_params;
  void *filter_params[BLOSC2_MAX_FILTERS];
} blosc2_cparams;

/* include/blosc2.h:1216-1223 */
static const blosc2_cparams BLOSC2_CPARAMS_DEFAULTS = {
    BLOSC_BLOSCLZ, 0, 5, 0, 8, 1, 0, BLOSC_FORWARD_COMPAT_SPLIT, NULL,
    {0, 0, 0, 0, 0, BLOSC_SHUFFLE}, {0, 0, 0, 0, 0, 0},
    NULL, NULL, NULL, 0, 0, NULL, {NULL, NULL, NULL, NULL, NULL, NULL}};

/* include/blosc2.h:1232-1243 */
typedef struct {
  int16_t nthreads;
  void *schunk;
  blosc2_postfilter_fn postfilter;
  blosc2_postfilter_params *postparams;
  int32_t typesize;
} blosc2_dparams;

/* include/blosc2.h:1248 */
static const blosc2_dparams BLOSC2_DPARAMS_DEFAULTS = {1, NULL, NULL, NULL, 8};

/* ---- codec / filter plugin registry (include/blosc2.h:2698-2762) ---- */
typedef int (*blosc2_codec_encoder_cb)(const uint8_t *input, int32_t input_len, uint8_t *output, int32_t output_len,
                                       uint8_t meta, blosc2_cparams *cparams, const void *chunk);
typedef int (*blosc2_codec_decoder_cb)(const uint8_t *input, int32_t input_len, uint8_t *output, int32_t output_len,
                                       uint8_t meta, blosc2_dparams *dparams, const void *chunk);
typedef struct {
  uint8_t compcode;
  char *compname;
  uint8_t complib;
  uint8_t version;
  blosc2_codec_encoder_cb encoder;
  blosc2_codec_decoder_cb decoder;
} blosc2_codec;

typedef int (*blosc2_filter_forward_cb)(const uint8_t *, uint8_t *, int32_t, uint8_t, blosc2_cparams *, uint8_t);
typedef int (*blosc2_filter_backward_cb)(const uint8_t *, uint8_t *, int32_t, uint8_t, blosc2_dparams *, uint8_t);
typedef struct {
  uint8_t id;
  char *name;
  uint8_t version;
  blosc2_filter_forward_cb forward;
  blosc2_filter_backward_cb backward;
} blosc2_filter;

/* ================================================================ entry points ========= */
/* library lifetime: include/blosc2.h:540 (blosc2_init), 551 (blosc2_destroy) */
BLOSC_EXPORT void blosc2_init(void);
BLOSC_EXPORT void blosc2_destroy(void);
/* include/blosc2.h:872 (blosc2_free_resources, blosc/blosc2.c:6001-6006): releases the engine's
 * device scratch (per-device workspaces, the global contexts' staging); they are re-created on
 * the next call.  BLOSC2_ERROR_FAILURE when the library is not initialised. */
BLOSC_EXPORT int blosc2_free_resources(void);
/* include/blosc2.h:843 (blosc2_get_version_string) */
BLOSC_EXPORT const char *blosc2_get_version_string(void);

/* contexts: include/blosc2.h:1263-1328 */
BLOSC_EXPORT blosc2_context *blosc2_create_cctx(blosc2_cparams cparams);
BLOSC_EXPORT blosc2_context *blosc2_create_dctx(blosc2_dparams dparams);
BLOSC_EXPORT void blosc2_free_ctx(blosc2_context *context);
BLOSC_EXPORT int blosc2_ctx_get_cparams(blosc2_context *ctx, blosc2_cparams *cparams);
BLOSC_EXPORT int blosc2_ctx_get_dparams(blosc2_context *ctx, blosc2_dparams *dparams);
/* Special chunks (reference include/blosc2.h:1616-1668, blosc/blosc2.c:6452-6637): header-only chunks
 * that decompress to zeros / NaNs / uninitialised bytes / one repeated value. */
BLOSC_EXPORT int blosc2_chunk_zeros(blosc2_cparams cparams, int32_t nbytes, void *dest, int32_t destsize);
BLOSC_EXPORT int blosc2_chunk_uninit(blosc2_cparams cparams, int32_t nbytes, void *dest, int32_t destsize);
BLOSC_EXPORT int blosc2_chunk_nans(blosc2_cparams cparams, int32_t nbytes, void *dest, int32_t destsize);
BLOSC_EXPORT int blosc2_chunk_repeatval(blosc2_cparams cparams, int32_t nbytes, void *dest, int32_t destsize,
                                        const void *repeatval);
BLOSC_EXPORT int blosc2_set_maskout(blosc2_context *ctx, bool *maskout, int nblocks);

/* the hot path: include/blosc2.h:1482-1484 and 1538-1539 */
BLOSC_EXPORT int blosc2_compress_ctx(blosc2_context *context, const void *src, int32_t srcsize, void *dest,
                                     int32_t destsize);
BLOSC_EXPORT int blosc2_decompress_ctx(blosc2_context *context, const void *src, int32_t srcsize, void *dest,
                                       int32_t destsize);
/* one block of a chunk (ref blosc/blosc2.c:4580-4687; declared in blosc/blosc-private.h:29 and
 * exported by the reference library; the sparse reader's per-block decode, schunk.c:1858).
 * Returns the block's size or a BLOSC2_ERROR_* code. */
BLOSC_EXPORT int blosc2_decompress_block_ctx(blosc2_context *context, const void *src, int32_t srcsize, int32_t nblock,
                                             void *dest, int32_t destsize);
/* partial decode: include/blosc2.h:1698 (blosc2_getitem_ctx), 722 (blosc2_getitem) */
BLOSC_EXPORT int blosc2_getitem_ctx(blosc2_context *context, const void *src, int32_t srcsize, int start, int nitems,
                                    void *dest, int32_t destsize);
BLOSC_EXPORT int blosc2_getitem(const void *src, int32_t srcsize, int start, int nitems, void *dest,
                                int32_t destsize);

/* global-context API: include/blosc2.h:1413 (blosc2_compress), 1459 (blosc2_decompress),
 * 638-704 (blosc1_compress / blosc1_decompress / blosc1_getitem) */
BLOSC_EXPORT int blosc2_compress(int clevel, int doshuffle, int32_t typesize, const void *src, int32_t srcsize,
                                 void *dest, int32_t destsize);
BLOSC_EXPORT int blosc2_decompress(const void *src, int32_t srcsize, void *dest, int32_t destsize);
BLOSC_EXPORT int blosc1_compress(int clevel, int doshuffle, size_t typesize, size_t nbytes, const void *src,
                                 void *dest, size_t destsize);
BLOSC_EXPORT int blosc1_decompress(const void *src, void *dest, size_t destsize);
BLOSC_EXPORT int blosc1_getitem(const void *src, int start, int nitems, void *dest);

/* global settings: include/blosc2.h:751-797, 2649-2679 */
BLOSC_EXPORT int16_t blosc2_get_nthreads(void);
BLOSC_EXPORT int16_t blosc2_set_nthreads(int16_t nthreads);
/* Caller-managed threading backend (include/blosc2.h:731-744 of the reference, blosc/blosc2.c:181):
 * `callback` runs dojob(jobdata + i*jobdata_elsize) for i in [0, numjobs).  The device pipeline has
 * no host worker pool; the callback dispatches the per-block / per-stream host callbacks of
 * user-registered filters and codecs when nthreads > 1, as the reference's pool would. */
typedef void (*blosc_threads_callback)(void *callback_data, void (*dojob)(void *), int numjobs, size_t jobdata_elsize,
                                       void *jobdata);
BLOSC_EXPORT void blosc2_set_threads_callback(blosc_threads_callback callback, void *callback_data);
BLOSC_EXPORT const char *blosc1_get_compressor(void);
BLOSC_EXPORT int blosc1_set_compressor(const char *compname);
BLOSC_EXPORT void blosc2_set_delta(int dodelta);
BLOSC_EXPORT int blosc1_get_blocksize(void);
BLOSC_EXPORT void blosc1_set_blocksize(size_t blocksize);
BLOSC_EXPORT void blosc1_set_splitmode(int splitmode);

/* codec names: include/blosc2.h:809-861 */
BLOSC_EXPORT int blosc2_compcode_to_compname(int compcode, const char **compname);
BLOSC_EXPORT int blosc2_compname_to_compcode(const char *compname);
BLOSC_EXPORT const char *blosc2_list_compressors(void);
BLOSC_EXPORT int blosc2_get_complib_info(const char *compname, char **complib, char **version);

/* chunk inspection: include/blosc2.h:893-988 */
BLOSC_EXPORT int blosc2_cbuffer_sizes(const void *cbuffer, int32_t *nbytes, int32_t *cbytes, int32_t *blocksize);
BLOSC_EXPORT void blosc1_cbuffer_sizes(const void *cbuffer, size_t *nbytes, size_t *cbytes, size_t *blocksize);
BLOSC_EXPORT int blosc1_cbuffer_validate(const void *cbuffer, size_t cbytes, size_t *nbytes);
BLOSC_EXPORT void blosc2_cbuffer_versions(const void *cbuffer, int *version, int *versionlz);
BLOSC_EXPORT const char *blosc2_cbuffer_complib(const void *cbuffer);
BLOSC_EXPORT void blosc1_cbuffer_metainfo(const void *cbuffer, size_t *typesize, int *flags);

/* plugin registry: include/blosc2.h:2727 (codec), 2762 (filter) */
BLOSC_EXPORT int blosc2_register_codec(blosc2_codec *codec);
BLOSC_EXPORT int blosc2_register_filter(blosc2_filter *filter);

/* raw filters on host buffers (executed by the GPU kernels): include/blosc2.h:2845-2900 */
BLOSC_EXPORT int32_t blosc2_shuffle(int32_t typesize, int32_t blocksize, const void *src, void *dest);
BLOSC_EXPORT int32_t blosc2_unshuffle(int32_t typesize, int32_t blocksize, const void *src, void *dest);
BLOSC_EXPORT int32_t blosc2_bitshuffle(int32_t typesize, int32_t blocksize, const void *src, void *dest);
BLOSC_EXPORT int32_t blosc2_bitunshuffle(int32_t typesize, int32_t blocksize, const void *src, void *dest);

/* partial decode by bytes: include/blosc2.h:1735 (blosc2_getitem_bytes_ctx, blosc/blosc2.c:4552-4577):
 * `start` and `nbytes` count bytes and must be multiples of the chunk's stored typesize. */
BLOSC_EXPORT int blosc2_getitem_bytes_ctx(blosc2_context *context, const void *src, int32_t srcsize, int32_t start,
                                          int32_t nbytes, void *dest, int32_t destsize);

/* ---- super-chunks (include/blosc2.h:1740-2362): the container the reference's callers reach the
 * chunk engine through (blosc/schunk.c).  Structs ABI-identical; the engine keeps IN-MEMORY, SPARSE
 * super-chunks (storage.contiguous == false, urlpath == NULL): chunks are malloc'd host buffers
 * indexed by schunk->data, exactly as the reference's frame-less schunk.  New frame-backed storage
 * (contiguous frames, files, directories) is outside the device engine:
 * blosc2_schunk_new returns NULL for it.  Existing contiguous frames OPEN through the reference's
 * entry points (blosc2_schunk_open* / _from_buffer below) as read-only, frame-attached handles:
 * a frame file is read through its IO backend (blosc2_io_cb) lazily, a chunk or a run of adjacent
 * chunks at a time, as frame_get_chunk reads it; an in-memory frame is used in place.  Any
 * super-chunk is written out as a contiguous frame with blosc2_schunk_to_buffer / _to_file /
 * _append_file.  The device-batch forms (b2h_schunk_append_device / b2h_schunk_decompress_device
 * in include/b2h.h) run one engine launch over many chunks of a super-chunk. ---- */
enum {   /* include/blosc2.h:994-1005 */
  BLOSC2_IO_FILESYSTEM = 0,
  BLOSC2_IO_FILESYSTEM_MMAP = 1,
  BLOSC_IO_LAST_BLOSC_DEFINED = 2,
  BLOSC_IO_LAST_REGISTERED = 32,
};
enum {
  BLOSC2_IO_BLOSC_DEFINED = 32,
  BLOSC2_IO_REGISTERED = 160,
  BLOSC2_IO_USER_DEFINED = 256
};
/* include/blosc2.h:1047-1059 */
typedef struct {
  uint8_t id;
  const char *name;
  void *params;
} blosc2_io;
static const blosc2_io BLOSC2_IO_DEFAULTS = {BLOSC2_IO_FILESYSTEM, "filesystem", NULL};

/* IO backends: include/blosc2.h:1007-1078 (registry blosc/blosc2.c:6784-6847).  The registry holds
 * the filesystem backend (id 0, blosc2_stdio_*) and the memory-mapped one (id 1,
 * blosc2_stdio_mmap_*); users register ids >= BLOSC2_IO_REGISTERED. */
typedef void*   (*blosc2_open_cb)(const char *urlpath, const char *mode, void *params);
typedef int     (*blosc2_close_cb)(void *stream);
typedef int64_t (*blosc2_size_cb)(void *stream);
typedef int64_t (*blosc2_write_cb)(const void *ptr, int64_t size, int64_t nitems, int64_t position, void *stream);
typedef int64_t (*blosc2_read_cb)(void **ptr, int64_t size, int64_t nitems, int64_t position, void *stream);
typedef int     (*blosc2_truncate_cb)(void *stream, int64_t size);
typedef int     (*blosc2_destroy_cb)(void *params);
typedef struct {
  uint8_t id;
  char *name;
  bool is_allocation_necessary;   /* true: read() fills the caller's buffer; false: it returns a pointer */
  blosc2_open_cb open;
  blosc2_close_cb close;
  blosc2_size_cb size;
  blosc2_write_cb write;
  blosc2_read_cb read;
  blosc2_truncate_cb truncate;
  blosc2_destroy_cb destroy;
} blosc2_io_cb;
BLOSC_EXPORT int blosc2_register_io_cb(const blosc2_io_cb *io);
BLOSC_EXPORT blosc2_io_cb *blosc2_get_io_cb(uint8_t id);

/* The filesystem backend: include/blosc2/blosc2-stdio.h:25-69 (blosc/blosc2-stdio.c:120-300).
 * Positioned reads and writes (pread / pwrite), so one open handle serves concurrent readers. */
typedef struct {
  FILE *file;
} blosc2_stdio_file;
typedef struct {
  bool locking;   /* accepted; the sidecar lock file is not implemented */
} blosc2_stdio_params;
static const blosc2_stdio_params BLOSC2_STDIO_PARAMS_DEFAULTS = {false};
BLOSC_EXPORT void *blosc2_stdio_open(const char *urlpath, const char *mode, void *params);
BLOSC_EXPORT int blosc2_stdio_close(void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_size(void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_write(const void *ptr, int64_t size, int64_t nitems, int64_t position, void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_read(void **ptr, int64_t size, int64_t nitems, int64_t position, void *stream);
BLOSC_EXPORT int blosc2_stdio_truncate(void *stream, int64_t size);
BLOSC_EXPORT int blosc2_stdio_destroy(void *params);

/* The memory-mapped backend: include/blosc2/blosc2-stdio.h:76-135.  Read modes ("r", "c") map the
 * file; read() hands out pointers into the mapping (no copy).  The writable modes ("r+", "w+")
 * back frame-backed storage that the engine does not create; open refuses them. */
typedef struct {
  const char *mode;
  size_t initial_mapping_size;
  bool needs_free;
  char *addr;
  char *urlpath;
  size_t file_size;
  size_t mapping_size;
  bool is_memory_only;
  FILE *file;
  int fd;
  int64_t access_flags;
  int64_t map_flags;
} blosc2_stdio_mmap;
static const blosc2_stdio_mmap BLOSC2_STDIO_MMAP_DEFAULTS = {
  "r", ((size_t)1 << 30), false, NULL, NULL, 0, 0, false, NULL, -1, -1, -1};
BLOSC_EXPORT blosc2_stdio_mmap blosc2_get_blosc2_stdio_mmap_defaults(void);
BLOSC_EXPORT void *blosc2_stdio_mmap_open(const char *urlpath, const char *mode, void *params);
BLOSC_EXPORT int blosc2_stdio_mmap_close(void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_mmap_size(void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_mmap_write(const void *ptr, int64_t size, int64_t nitems, int64_t position,
                                             void *stream);
BLOSC_EXPORT int64_t blosc2_stdio_mmap_read(void **ptr, int64_t size, int64_t nitems, int64_t position, void *stream);
BLOSC_EXPORT int blosc2_stdio_mmap_truncate(void *stream, int64_t size);
BLOSC_EXPORT int blosc2_stdio_mmap_destroy(void *params);

#define BLOSC2_MAX_METALAYERS 16                  /* include/blosc2.h:1744 */
#define BLOSC2_METALAYER_NAME_MAXLEN 31
#define BLOSC2_MAX_VLMETALAYERS (8 * 1024)        /* include/blosc2.h:1750 */
#define BLOSC2_VLMETALAYERS_NAME_MAXLEN BLOSC2_METALAYER_NAME_MAXLEN

/* include/blosc2.h:1758-1776 */
typedef struct {
  bool contiguous;
  char *urlpath;
  blosc2_cparams *cparams;
  blosc2_dparams *dparams;
  blosc2_io *io;
} blosc2_storage;
static const blosc2_storage BLOSC2_STORAGE_DEFAULTS = {false, NULL, NULL, NULL, NULL};

/* defaults getters: include/blosc2.h:1781-1796 (blosc/blosc2.c:6896-6911) */
BLOSC_EXPORT blosc2_cparams blosc2_get_blosc2_cparams_defaults(void);
BLOSC_EXPORT blosc2_dparams blosc2_get_blosc2_dparams_defaults(void);
BLOSC_EXPORT blosc2_storage blosc2_get_blosc2_storage_defaults(void);
BLOSC_EXPORT blosc2_io blosc2_get_blosc2_io_defaults(void);

typedef struct blosc2_frame_s blosc2_frame;   /* opaque (include/blosc2.h:1803) */

/* include/blosc2.h:1810-1814 */
typedef struct blosc2_metalayer {
  char *name;
  uint8_t *content;
  int32_t content_len;
} blosc2_metalayer;

/* include/blosc2.h:1823-1892 */
typedef struct blosc2_schunk {
  uint8_t version;
  uint8_t compcode;
  uint8_t compcode_meta;
  uint8_t clevel;
  uint8_t splitmode;
  int32_t typesize;
  int32_t blocksize;
  int32_t chunksize;
  uint8_t flags2;
  uint8_t use_dict;
  uint8_t filters[BLOSC2_MAX_FILTERS];
  uint8_t filters_meta[BLOSC2_MAX_FILTERS];
  int64_t nchunks;
  int64_t current_nchunk;
  int64_t nbytes;
  int64_t cbytes;
  uint8_t **data;
  size_t data_len;
  blosc2_storage *storage;
  blosc2_frame *frame;
  blosc2_context *cctx;
  blosc2_context *dctx;
  struct blosc2_metalayer *metalayers[BLOSC2_MAX_METALAYERS];
  uint16_t nmetalayers;
  struct blosc2_metalayer *vlmetalayers[BLOSC2_MAX_VLMETALAYERS];
  int16_t nvlmetalayers;
  void *tuner_params;
  int tuner_id;
  int8_t ndim;
  int64_t *blockshape;
  bool view;
  int64_t change_tick;
} blosc2_schunk;

/* include/blosc2.h:1905 (blosc/schunk.c:163-242) */
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_new(blosc2_storage *storage);
/* include/blosc2.h:2088 (blosc/schunk.c:679-729) */
BLOSC_EXPORT int blosc2_schunk_free(blosc2_schunk *schunk);
/* include/blosc2.h:1934 (blosc/schunk.c:731-750, frame_to_schunk frame.c:2941-3245): a contiguous
 * frame in memory; `copy` false gives the frame-attached flavour (storage.contiguous, the header's
 * cbytes and blocksize; the chunks are read in place from `cframe`, which must outlive the handle),
 * true the copy (sum of the chunks' cbytes, their common blocksize, chunks in malloc'd buffers).
 * Frame-attached handles are read-only (their mutators return BLOSC2_ERROR_INVALID_PARAM). */
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_from_buffer(uint8_t *cframe, int64_t len, bool copy);
/* include/blosc2.h:2008, 2019, 2030, 2043 (blosc/schunk.c:366-470, frame_from_file_offset
 * frame.c:1720-1870): a contiguous frame file (at `offset`) through the IO backend `udio->id`
 * (registry above; NULL udio = the filesystem backend).  Open reads the header, the trailer and
 * the offsets index only; chunks are read when used, through the backend's read callback, which
 * stays open for the handle's life.  Unlike the reference's, the handle is READ-ONLY: append /
 * insert / update / delete chunk, append_buffer and set_slice_buffer return
 * BLOSC2_ERROR_INVALID_PARAM on it (copy the chunks into a blosc2_schunk_new super-chunk and write
 * that out with blosc2_schunk_to_file to modify a frame). */
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_open(const char *urlpath);
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_open_offset(const char *urlpath, int64_t offset);
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_open_udio(const char *urlpath, const blosc2_io *udio);
BLOSC_EXPORT blosc2_schunk *blosc2_schunk_open_offset_udio(const char *urlpath, int64_t offset, const blosc2_io *udio);
/* include/blosc2.h:1946, 1957, 1968 (blosc/schunk.c:481-650; frame_from_schunk frame.c:1926-2100,
 * new_header_frame 591-889, frame_update_trailer 1422-1640): the super-chunk as one contiguous
 * frame -- header (fields, metalayers), the chunks in order, the offsets index (a Blosc chunk of
 * int64 offsets, compressed as frame_append_chunk compresses it: BloscLZ, typesize 8, 16 KiB
 * blocks, no split) and the trailer (vlmetalayers).  to_buffer hands out a malloc'd frame
 * (*needs_free true), or the attached frame itself for a handle on an in-memory frame; to_file
 * writes through the filesystem backend and returns the frame length; append_file writes the frame
 * at the end of the file and returns the offset it starts at (for blosc2_schunk_open_offset). */
BLOSC_EXPORT int64_t blosc2_schunk_to_buffer(blosc2_schunk *schunk, uint8_t **cframe, bool *needs_free);
BLOSC_EXPORT int64_t blosc2_schunk_to_file(blosc2_schunk *schunk, const char *urlpath);
BLOSC_EXPORT int64_t blosc2_schunk_append_file(blosc2_schunk *schunk, const char *urlpath);
/* include/blosc2.h:2101, 2115, 2129, 2140 (blosc/schunk.c:975-1457) */
BLOSC_EXPORT int64_t blosc2_schunk_append_chunk(blosc2_schunk *schunk, uint8_t *chunk, bool copy);
BLOSC_EXPORT int64_t blosc2_schunk_update_chunk(blosc2_schunk *schunk, int64_t nchunk, uint8_t *chunk, bool copy);
BLOSC_EXPORT int64_t blosc2_schunk_insert_chunk(blosc2_schunk *schunk, int64_t nchunk, uint8_t *chunk, bool copy);
BLOSC_EXPORT int64_t blosc2_schunk_delete_chunk(blosc2_schunk *schunk, int64_t nchunk);
/* include/blosc2.h:2152 (blosc/schunk.c:1459-1477) */
BLOSC_EXPORT int64_t blosc2_schunk_append_buffer(blosc2_schunk *schunk, const void *src, int32_t nbytes);
/* include/blosc2.h:2171 (blosc/schunk.c:1481-1530) */
BLOSC_EXPORT int blosc2_schunk_decompress_chunk(blosc2_schunk *schunk, int64_t nchunk, void *dest, int32_t nbytes);
/* include/blosc2.h:2196, 2236 (blosc/schunk.c:1543-1631) */
BLOSC_EXPORT int blosc2_schunk_get_chunk(blosc2_schunk *schunk, int64_t nchunk, uint8_t **chunk, bool *needs_free);
BLOSC_EXPORT int blosc2_schunk_get_lazychunk(blosc2_schunk *schunk, int64_t nchunk, uint8_t **chunk,
                                             bool *needs_free);
/* include/blosc2.h:2275 (blosc/schunk.c:1662-1783) */
BLOSC_EXPORT int blosc2_schunk_get_slice_buffer(blosc2_schunk *schunk, int64_t start, int64_t stop, void *buffer);
/* include/blosc2.h:2290 (blosc/schunk.c:1922-2110): the items at `coords` (any order, repeats
 * allowed) into buffer[i * typesize].  Same argument checks and error codes as the reference;
 * under DELTA, a postfilter or one coordinate, one getitem per coordinate (schunk.c:1866-1900),
 * otherwise every touched chunk is decoded once -- only its touched blocks, through a block mask
 * (one device call per chunk instead of one per block). */
BLOSC_EXPORT int blosc2_schunk_get_sparse_buffer(blosc2_schunk *schunk, int64_t ncoords, const int64_t *coords,
                                                 void *buffer);
/* include/blosc2.h:2304 (blosc/schunk.c:2146-2216): items [start, stop) of the super-chunk replaced by
 * `buffer`, every touched chunk recompressed through the super-chunk's cctx and updated in place. */
BLOSC_EXPORT int blosc2_schunk_set_slice_buffer(blosc2_schunk *schunk, int64_t start, int64_t stop, void *buffer);
/* include/blosc2.h:2316, 2328 (blosc/schunk.c:70-105) */
BLOSC_EXPORT int blosc2_schunk_get_cparams(blosc2_schunk *schunk, blosc2_cparams **cparams);
BLOSC_EXPORT int blosc2_schunk_get_dparams(blosc2_schunk *schunk, blosc2_dparams **dparams);

#ifdef __cplusplus
}
#endif
#endif /* BLOSC2_AMD_BLOSC2_H */
