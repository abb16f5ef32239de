// blosc2_api.cpp -- the drop-in C ABI (include/blosc2.h) on top of the MI355X batch engine.
//
// Host responsibilities only: context state (incl. the reference's sticky context blocksize,
// blosc/blosc2.c:2414-2416 + stune.c:54-60), environment overrides, header parsing for the
// inspection API, H<->D staging of caller buffers, and the plugin registry.  Every byte of
// filter / codec work is done by the HIP kernels in b2h_engine.hip; there is no CPU fallback --
// without a usable GPU the compute entry points return BLOSC2_ERROR_FAILURE loudly.
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/b2h.h"
#include "../../include/blosc2.h"
#include "b2h_engine.h"
#include "b2h_format.h"

namespace {

bool trace_on() {
  static int on = -1;
  if (on < 0) on = getenv("BLOSC_TRACE") != nullptr;
  return on;
}
#define TRACE_ERROR(...)                                                   \
  do {                                                                     \
    if (trace_on()) {                                                      \
      fprintf(stderr, "[error] - ");                                       \
      fprintf(stderr, __VA_ARGS__);                                        \
      fprintf(stderr, " (%s:%d)\n", __FILE__, __LINE__);                   \
    }                                                                      \
  } while (0)

int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// ---------------------------------------------------------------- device staging buffers ----
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    n += 256;
    if (n <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) return false;
    cap = n;
    static const bool poison = getenv("B2H_POISON") != nullptr;   // debug: expose unwritten bytes
    if (poison) (void)hipMemset(p, 0xA5, n);
    return true;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

// Pinned host staging of the super-chunk batches (one DMA per direction instead of one per chunk).
struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool ensure(size_t n) {
    if (n <= cap) return true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    n = std::max<size_t>(n, 1 << 20);
    if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return false;
    cap = n;
    return true;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

// Per-context device state: its own stream, staging buffers and engine workspace, so distinct
// contexts run concurrently (include/blosc2.h:1462-1466); all of it is freed by blosc2_free_ctx
// (the reference frees its context scratch there, blosc/blosc2.c:6290).
struct Device {
  int dev = -1;
  hipStream_t stream = nullptr;
  DevBuf in, out, small;
  PinnedBuf host;   // super-chunk batches only
  b2h::Workspace* ws = nullptr;
  bool init() {
    if (stream) return true;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
      TRACE_ERROR("no HIP device available: the MI355X engine has no CPU fallback");
      return false;
    }
    if (hipGetDevice(&dev) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return false;
    ws = b2h::workspace_create();
    return true;
  }
  void release() {
    if (stream) (void)hipStreamSynchronize(stream);
    b2h::workspace_destroy(ws);
    ws = nullptr;
    in.release();
    out.release();
    small.release();
    host.release();
    if (stream) (void)hipStreamDestroy(stream);
    stream = nullptr;
  }
};

// --------------------------------------------------------------------- plugin registry ----
std::mutex g_reg_mu;
std::vector<blosc2_codec> g_codecs;
std::vector<blosc2_filter> g_filters;

// ------------------------------------------------------------------------ global state ----
std::mutex g_global_mu;
bool g_initlib = false;
int16_t g_nthreads = 1;
int g_compressor = BLOSC_BLOSCLZ;
int g_delta = 0;
int32_t g_force_blocksize = 0;
int32_t g_splitmode = BLOSC_FORWARD_COMPAT_SPLIT;
blosc_threads_callback g_threads_cb = nullptr;
void* g_threads_cb_data = nullptr;

}  // namespace

struct blosc2_context_s {
  int do_compress = 0;
  // compression parameters (blosc2_cparams)
  uint8_t compcode = 0, compcode_meta = 0;
  int clevel = 5;
  int use_dict = 0;
  int32_t typesize = 8;
  int16_t nthreads = 1;
  int32_t blocksize = 0;     // sticky: overwritten by every compression (see header comment)
  int32_t splitmode = BLOSC_FORWARD_COMPAT_SPLIT;
  void* schunk = nullptr;
  uint8_t filters[6] = {0, 0, 0, 0, 0, BLOSC_SHUFFLE};
  uint8_t filters_meta[6] = {0};
  blosc2_prefilter_fn prefilter = nullptr;
  blosc2_prefilter_params* preparams = nullptr;   // -> pre_copy when a prefilter is set
  blosc2_prefilter_params pre_copy{};             // the context's own copy (blosc/blosc2.c:6215-6219)
  blosc2_postfilter_params post_copy{};           // dparams.postparams points here (6279-6283)
  std::vector<uint8_t> ttmp;                      // the callbacks' `ttmp` (a thread context's 4 x ebsize tmp)
  void* tuner_params = nullptr;
  int tuner_id = 0;
  bool instr_codec = false;
  void* codec_params = nullptr;
  int lz_mode = -1;          // BloscLZ encoder chosen through codec_params at creation (-1: process default)
  void* filter_params[6] = {nullptr};
  // decompression parameters
  blosc2_dparams dparams = BLOSC2_DPARAMS_DEFAULTS;
  // block mask for the next decompression (blosc2_set_maskout)
  std::vector<uint8_t> maskout;
  // device side
  Device dev;
  std::mutex mu;
};

namespace b2h {
// cparams.codec_params -> BloscLZ encoder mode (include/b2h.h b2h_codec_params), or -1.  Only a
// struct carrying the magic word is ours: a user codec's own parameters are left alone.
int codec_params_lz_mode(const void* codec_params) {
  if (!codec_params) return -1;
  const b2h_codec_params* p = static_cast<const b2h_codec_params*>(codec_params);
  if (p->magic != B2H_CODEC_PARAMS_MAGIC) return -1;
  return (p->blosclz_mode >= 0 && p->blosclz_mode <= 3) ? p->blosclz_mode : -1;
}
}  // namespace b2h

namespace {

bool env_long(const char* name, long* out) {
  const char* v = getenv(name);
  if (!v) return false;
  errno = 0;
  long x = strtol(v, nullptr, 10);
  if (errno == EINVAL) return false;
  *out = x;
  return true;
}

void build_filters(int doshuffle, int delta, int32_t typesize, uint8_t* filters) {
  // blosc/blosc2.c:3686-3698
  if (doshuffle == BLOSC_SHUFFLE && typesize > 1) filters[5] = BLOSC_SHUFFLE;
  if (doshuffle == BLOSC_BITSHUFFLE) filters[5] = BLOSC_BITSHUFFLE;
  if (doshuffle == BLOSC_NOSHUFFLE) filters[5] = BLOSC_NOSHUFFLE;
  if (delta) filters[4] = BLOSC_DELTA;
}

int compname_to_code(const char* name) {
  if (!name) return -1;
  if (!strcmp(name, BLOSC_BLOSCLZ_COMPNAME)) return BLOSC_BLOSCLZ;
  if (!strcmp(name, BLOSC_LZ4_COMPNAME)) return BLOSC_LZ4;
  if (!strcmp(name, BLOSC_LZ4HC_COMPNAME)) return BLOSC_LZ4HC;
  if (!strcmp(name, BLOSC_ZLIB_COMPNAME)) return BLOSC_ZLIB;
  if (!strcmp(name, BLOSC_ZSTD_COMPNAME)) return BLOSC_ZSTD;
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (auto& c : g_codecs)
    if (c.compname && !strcmp(c.compname, name)) return c.compcode;
  return -1;
}

// Pipelines the device path executes: built-in filters and BloscLZ.
// User-registered filters and codecs run through the host-callback pipelines below.
int check_supported(const blosc2_context* c, bool host_pipeline = false) {
  if (c->compcode != BLOSC_BLOSCLZ && c->compcode != BLOSC_LZ4 && c->compcode <= BLOSC2_DEFINED_CODECS_STOP) {
    TRACE_ERROR("codec %d is not implemented by the MI355X engine (BloscLZ, LZ4 and user codecs)", c->compcode);
    return BLOSC2_ERROR_CODEC_SUPPORT;
  }
  // blosc/blosc2.c:2514-2521 (ZSTD and LZ4HC are refused above as codecs)
  if (c->use_dict && c->compcode != BLOSC_LZ4) {
    TRACE_ERROR("`use_dict` is only supported for ZSTD, LZ4, and LZ4HC codecs.");
    return BLOSC2_ERROR_CODEC_PARAM;
  }
  for (int i = 0; i < 6; i++) {
    const uint8_t f = c->filters[i];
    // bytedelta with meta 0 takes the super-chunk's typesize and fails without one
    // (plugins/filters/bytedelta/bytedelta.c:90-98 -> pipeline_forward returns NULL)
    if (f == b2h::kBytedelta && c->filters_meta[i] == 0 && c->schunk == nullptr) {
      TRACE_ERROR("When meta is 0, you need to be on a schunk!");
      return BLOSC2_ERROR_FILTER_PIPELINE;
    }
  }
  if (c->prefilter && !host_pipeline) {
    TRACE_ERROR("prefilters run per chunk through blosc2_compress_ctx, not the device batch");
    return BLOSC2_ERROR_FILTER_PIPELINE;
  }
  if (c->instr_codec || c->tuner_params || c->tuner_id != 0) {
    TRACE_ERROR("instrumented codecs / tuners are not supported by the device pipeline");
    return BLOSC2_ERROR_FILTER_PIPELINE;
  }
  return 0;
}

bool needs_host_callbacks(const uint8_t* filters, int compcode);
bool device_filter(uint8_t f);
bool lookup_filter(uint8_t id, blosc2_filter* out);
bool lookup_codec(int compcode, blosc2_codec* out);
int compress_hybrid(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                    int32_t blocksize_in, bool sticky, bool extended);
int decompress_hybrid(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                      const std::vector<uint8_t>* mask, int mode);

// Compress one host buffer through the engine (n = 1 batch).
int compress_host(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                  int32_t blocksize_in, bool sticky, bool extended) {
  if (srcsize < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (ctx->prefilter || needs_host_callbacks(ctx->filters, ctx->compcode))
    return compress_hybrid(ctx, src, srcsize, dest, destsize, blocksize_in, sticky, extended);
  b2h::CompressPlan plan;
  int32_t computed = 0;
  int rc = b2h::make_compress_plan(&plan, srcsize, destsize, ctx->clevel, ctx->typesize, blocksize_in, ctx->splitmode,
                                   ctx->filters, ctx->filters_meta, &computed, extended, ctx->compcode,
                                   ctx->compcode_meta, 1, ctx->use_dict);
  if (rc < 0) return rc;
  plan.lz_mode = ctx->lz_mode;
  if (sticky) ctx->blocksize = computed;
  if ((rc = check_supported(ctx)) < 0) return rc;
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  if (!d.in.ensure((size_t)srcsize) || !d.out.ensure((size_t)destsize) || !d.small.ensure(64)) return BLOSC2_ERROR_MEMORY_ALLOC;
  if (srcsize && hipMemcpyAsync(d.in.p, src, (size_t)srcsize, hipMemcpyHostToDevice, d.stream) != hipSuccess)
    return BLOSC2_ERROR_FAILURE;
  int32_t* d_cb = reinterpret_cast<int32_t*>(d.small.p);
  int32_t cb = 0;
  // a fused launch whose hand-off wait timed out fails the batch with FAILURE: run it once more
  // with the separate launches (the chunk bytes are the same either way)
  for (int attempt = 0; attempt < 2; attempt++) {
    b2h::set_fuse_disabled(attempt > 0);
    rc = b2h::compress_batch(plan, d.in.u8(), 0, 1, d.out.u8(), 0, d_cb, d.stream, d.ws);
    b2h::set_fuse_disabled(false);
    if (rc < 0) {
      TRACE_ERROR("device compression failed: %s", b2h::last_error());
      return rc;
    }
    if (hipMemcpyAsync(&cb, d_cb, 4, hipMemcpyDeviceToHost, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
    if (hipStreamSynchronize(d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
    if (cb != BLOSC2_ERROR_FAILURE) break;
  }
  const int32_t ncopy = cb > 0 ? cb : (destsize < plan.overhead ? destsize : plan.overhead);
  if (hipMemcpy(dest, d.out.p, (size_t)ncopy, hipMemcpyDeviceToHost) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  return cb;
}

// Host mirror of read_chunk_header (blosc/blosc2.c:738-852, extended headers read) and
// blosc2_initialize_context_from_header (862-910): the same checks, order and codes as the
// reference and as the device planner (b2h_engine.hip k_dplan_chunks), for the entry points that
// need the geometry on the host (staging sizes, masks, getitem, decompress_block).
struct ChunkHdr {
  int32_t nbytes, blocksize, cbytes;   // blocksize clamped to nbytes as the reference does
  uint8_t version, flags, typesize, flags2, bflags, special;
  bool ext, vl, memcpyed, lazy;
  int32_t overhead, nblocks, leftover;
};

int read_header(const void* src, int32_t srcsize, ChunkHdr* h) {
  memset(h, 0, sizeof *h);
  if (srcsize < BLOSC_MIN_HEADER_LENGTH) return BLOSC2_ERROR_READ_BUFFER;
  const uint8_t* s = static_cast<const uint8_t*>(src);
  h->version = s[0];
  h->flags = s[2];
  h->typesize = s[3];
  h->nbytes = rd32(s + 4);
  h->blocksize = rd32(s + 8);
  h->cbytes = rd32(s + 12);
  if (h->cbytes < BLOSC_MIN_HEADER_LENGTH) return BLOSC2_ERROR_INVALID_HEADER;
  if (h->blocksize <= 0 || h->blocksize > BLOSC2_MAXBLOCKSIZE) return BLOSC2_ERROR_INVALID_HEADER;
  if (h->typesize == 0) return BLOSC2_ERROR_INVALID_HEADER;
  h->ext = (h->flags & BLOSC_DOSHUFFLE) && (h->flags & BLOSC_DOBITSHUFFLE);
  if (h->ext) {
    if (h->cbytes < BLOSC_EXTENDED_HEADER_LENGTH) return BLOSC2_ERROR_INVALID_HEADER;
    if (srcsize < BLOSC_EXTENDED_HEADER_LENGTH) return BLOSC2_ERROR_READ_BUFFER;
    h->flags2 = s[BLOSC2_CHUNK_BLOSC2_FLAGS2];
    h->bflags = s[BLOSC2_CHUNK_BLOSC2_FLAGS];
    h->special = (h->bflags >> 4) & BLOSC2_SPECIAL_MASK;
    if ((h->flags2 & BLOSC2_VL_BLOCKS) && h->special != 0) return BLOSC2_ERROR_INVALID_HEADER;
    if (h->special == BLOSC2_SPECIAL_VALUE) {
      const int32_t vts = h->cbytes - BLOSC_EXTENDED_HEADER_LENGTH;
      if (vts <= 0 || vts > BLOSC2_MAXTYPESIZE || vts > h->nbytes || h->nbytes % vts != 0)
        return BLOSC2_ERROR_INVALID_HEADER;
    } else if (h->special != 0 && h->special != BLOSC2_SPECIAL_ZERO && h->nbytes % h->typesize != 0) {
      return BLOSC2_ERROR_INVALID_HEADER;
    }
  }
  if (h->version > BLOSC2_VERSION_FORMAT && (h->flags2 & (uint8_t)~BLOSC2_VL_BLOCKS) != 0)
    return BLOSC2_ERROR_VERSION_SUPPORT;
  h->vl = h->flags2 & BLOSC2_VL_BLOCKS;
  h->memcpyed = h->flags & BLOSC_MEMCPYED;
  if (h->vl && h->memcpyed) return BLOSC2_ERROR_INVALID_HEADER;
  if (!h->vl && h->nbytes > 0 && h->blocksize > h->nbytes) h->blocksize = h->nbytes;
  return 0;
}

int init_from_header(ChunkHdr* h, int32_t srcsize) {
  if (h->vl) {
    h->nblocks = h->blocksize;
    h->leftover = 0;
  } else {
    h->nblocks = h->nbytes / h->blocksize;
    h->leftover = h->nbytes % h->blocksize;
    if (h->leftover > 0) h->nblocks++;
  }
  h->overhead = h->ext ? BLOSC_EXTENDED_HEADER_LENGTH : BLOSC_MIN_HEADER_LENGTH;
  h->lazy = h->ext && (h->bflags & 0x08);
  if (!h->lazy && h->cbytes > srcsize) return BLOSC2_ERROR_INVALID_HEADER;
  return 0;
}

// User filters / codecs in an extended header (not memcpyed, not special) -> host callbacks.
// Unknown ids <= BLOSC2_DEFINED_FILTERS_STOP stay on the device, which fails them as
// pipeline_backward does (blosc/blosc2.c:1534-1539); so does a plugin that is neither registered
// nor loadable: it fails where the reference's block walk meets it (the codec at its first stream,
// a filter after the block's streams), and the device planner keys those failures in order.
bool chunk_needs_host(const uint8_t* s, const ChunkHdr& H) {
  if (!H.ext || H.memcpyed || H.special != 0 || H.nbytes <= 0) return false;
  uint8_t fl[6];
  for (int i = 0; i < 6; i++) {
    fl[i] = s[16 + i];
    if (fl[i] <= BLOSC2_DEFINED_FILTERS_STOP) fl[i] = 0;
  }
  if (s[0] == BLOSC2_VERSION_FORMAT_ALPHA) fl[5] = 0;
  const bool udcodec = (s[2] >> 5) == BLOSC_UDCODEC_FORMAT;
  if (!needs_host_callbacks(fl, udcodec ? 255 : 0)) return false;
  blosc2_filter fi;
  blosc2_codec co;
  for (int i = 0; i < 6; i++)
    if (!device_filter(fl[i]) && !lookup_filter(fl[i], &fi)) return false;
  if (udcodec && !lookup_codec(s[22], &co)) return false;
  return true;
}

uint8_t* ctx_ttmp(blosc2_context* ctx, int32_t blocksize, int32_t typesize, size_t* nbytes);

// pipeline_backward's postfilter step for block `nblock` (blosc/blosc2.c:1586-1606; for memcpyed
// and special chunks 1910-1931): `in` is the block as the backward filters leave it, the
// callback writes `out`.  A special-value chunk passes its value's width as the typesize
// (blosc_d 1743-1746).
int call_postfilter(blosc2_context* ctx, const ChunkHdr& H, const uint8_t* in, uint8_t* out, int32_t nblock) {
  blosc2_postfilter_params pp;
  memcpy(&pp, ctx->dparams.postparams, sizeof pp);
  const int32_t off = nblock * H.blocksize;
  pp.input = in;
  pp.output = out;
  pp.size = std::min(H.blocksize, H.nbytes - off);
  pp.typesize = H.special == BLOSC2_SPECIAL_VALUE ? H.cbytes - H.overhead : H.typesize;
  pp.offset = off;
  pp.nchunk = ctx->schunk ? static_cast<blosc2_schunk*>(ctx->schunk)->current_nchunk : -1;
  pp.nblock = nblock;
  pp.tid = 0;
  pp.ttmp = ctx_ttmp(ctx, H.blocksize, H.typesize, &pp.ttmp_nbytes);
  pp.ctx = ctx;
  if (ctx->dparams.postfilter(&pp) != 0) {
    TRACE_ERROR("Execution of postfilter function failed");
    return BLOSC2_ERROR_POSTFILTER;
  }
  return 0;
}

// decompress_host mode bit (host only, never reaches the device): decode the chunk's block images
// without running the postfilter.  A flag instead of clearing ctx->dparams.postfilter for the call:
// other threads read that field (the fan-out's staged decode classifies chunks concurrently).
constexpr int kHostNoPost = 1 << 16;

// Decompress one host chunk through the engine.  With a block mask only unmasked blocks are
// copied back so masked regions of `dest` keep the caller's bytes (blosc/blosc2.c:1734-1737).
// `mode`: b2h::kDecDeltaSelf for the per-block entry points (getitem, decompress_block).
int decompress_host(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                    const std::vector<uint8_t>* mask, int mode = 0) {
  const bool run_post = ctx->dparams.postfilter && !(mode & kHostNoPost);
  mode &= ~kHostNoPost;
  ChunkHdr H;
  int rc = read_header(src, srcsize, &H);
  if (rc < 0) return rc;
  if (H.nbytes > destsize) return BLOSC2_ERROR_WRITE_BUFFER;
  if ((rc = init_from_header(&H, srcsize)) < 0) return rc;
  const int32_t nbytes = H.nbytes, bs = H.blocksize, nblocks = H.nblocks;
  if (mask && (int32_t)mask->size() != nblocks) {
    TRACE_ERROR("The number of items in block_maskout (%zu) must match the number of blocks in chunk (%d).",
                mask->size(), nblocks);
    return BLOSC2_ERROR_DATA;
  }
  if (run_post) {
    // The engine decodes the chunk (every backward filter) into a host image; the callback then
    // runs per unmasked block, in block order, writing `dest` (blosc_d with a postfilter never
    // writes dest itself: 1880-1883, 1960-1965, 1489, 1581).
    std::vector<uint8_t> img((size_t)std::max(nbytes, 1));
    rc = decompress_host(ctx, src, srcsize, img.data(), nbytes, mask, mode | kHostNoPost);
    if (rc < 0) return rc;
    for (int32_t b = 0; b < nblocks; b++) {
      if (mask && (*mask)[(size_t)b]) continue;
      const int64_t off = (int64_t)b * bs;
      if ((rc = call_postfilter(ctx, H, img.data() + off, static_cast<uint8_t*>(dest) + off, b)) < 0) return rc;
    }
    return nbytes;
  }
  if (chunk_needs_host(static_cast<const uint8_t*>(src), H))
    return decompress_hybrid(ctx, src, srcsize, dest, destsize, mask, mode);
  // The device reads what the reference may read: srcsize bytes (the blosc1 entry points pass
  // INT32_MAX for "unknown": the chunk's own cbytes then).
  const int32_t ss = srcsize == INT32_MAX ? std::max<int32_t>(H.cbytes, BLOSC_EXTENDED_HEADER_LENGTH) : srcsize;
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  const size_t mask_bytes = mask ? mask->size() : 0;
  if (!d.in.ensure((size_t)ss) || !d.out.ensure((size_t)(nbytes > 0 ? nbytes : 1)) ||
      !d.small.ensure(64 + mask_bytes))
    return BLOSC2_ERROR_MEMORY_ALLOC;
  struct Ptrs { const uint8_t* s; uint8_t* o; int32_t ss, ds, status, pad; } h;
  h.s = d.in.u8();
  h.o = d.out.u8();
  h.ss = ss;
  h.ds = destsize;
  uint8_t* sm = d.small.u8();
  if (hipMemcpyAsync(d.in.p, src, (size_t)ss, hipMemcpyHostToDevice, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  if (hipMemcpyAsync(sm, &h, sizeof h, hipMemcpyHostToDevice, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  const uint8_t* d_mask = nullptr;
  if (mask) {
    if (hipMemcpyAsync(sm + 64, mask->data(), mask_bytes, hipMemcpyHostToDevice, d.stream) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
    d_mask = sm + 64;
  }
  Ptrs* dp = reinterpret_cast<Ptrs*>(sm);
  // exact tables (src_bound -1): a malformed chunk may claim more streams than its bytes hold and
  // still be decoded by the reference (bstarts sharing stream data); one extra sync, host call
  rc = b2h::decompress_batch(reinterpret_cast<const uint8_t* const*>(&dp->s), &dp->ss,
                             reinterpret_cast<uint8_t* const*>(&dp->o), &dp->ds, 1, std::max(nbytes, 0), &dp->status,
                             d_mask, d.stream, d.ws, -1, mode);
  if (rc < 0) {
    TRACE_ERROR("device decompression failed: %s", b2h::last_error());
    return rc;
  }
  int32_t status = 0;
  if (hipMemcpyAsync(&status, &dp->status, 4, hipMemcpyDeviceToHost, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  if (hipStreamSynchronize(d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  if (status <= 0) return status;
  if (H.special == BLOSC2_SPECIAL_UNINIT) return status;   // nothing written (blosc/blosc2.c:1904-1906)
  if (!mask) {
    if (hipMemcpy(dest, d.out.p, (size_t)status, hipMemcpyDeviceToHost) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  } else {
    for (int32_t b = 0; b < nblocks; b++) {
      if ((*mask)[b]) continue;
      const int64_t off = (int64_t)b * bs;
      const int64_t len = std::min<int64_t>(bs, nbytes - off);
      if (hipMemcpy(static_cast<uint8_t*>(dest) + off, d.out.u8() + off, (size_t)len, hipMemcpyDeviceToHost) != hipSuccess)
        return BLOSC2_ERROR_FAILURE;
    }
  }
  return status;
}


// ============================================================= host-callback pipelines ====
// Chunks whose pipeline holds a user-registered filter (id > BLOSC2_DEFINED_FILTERS_STOP other
// than the device plugins 35 / 36) or a user-registered codec (compcode > 31) run the reference's
// semantics with the user's callbacks on host buffers and the built-in stages on the device:
//   compress   pipeline_forward (blosc/blosc2.c:1055-1180): the active slots in order, buffers
//              cycled src -> tmp -> tmp2 (the >= 3-filter rewrite of the input included), block 0
//              first when DELTA is present (its reference is the input's block 0 as the serial
//              walk leaves it); user forward(src, dst, bsize, meta, cparams*, id) per block;
//              then blosc_c / serial_blosc / blosc_compress_context (2161-2228, 1210-1469,
//              3004-3107): BloscLZ / LZ4 on the device, a user encoder(in, neblock, out, maxout,
//              meta, cparams*, chunk) per stream with the same run detection, maxout, raw and
//              memcpy / special-zero fallbacks;
//   decompress blosc_d (1710-2157) with the user decoder per stream (or the device decoder for
//              built-in codecs, streams only), then pipeline_backward (1473-1609) slot 5 -> 0 with
//              user backward(...) per block and device un-filters, block 0 first with DELTA.
// Callbacks run on the calling thread; with nthreads > 1 and blosc2_set_threads_callback, the
// per-block filter callbacks and per-stream decoder callbacks go through the caller's backend.

struct FilterInfo { char* forward; char* backward; };   // blosc-private.h filter_info
struct CodecInfo { char* encoder; char* decoder; };     // blosc-private.h codec_info

bool valid_plugin_name(const char* n) {
  if (!n || !*n) return false;
  for (const char* c = n; *c; c++)
    if (!((*c >= 'a' && *c <= 'z') || (*c >= 'A' && *c <= 'Z') || (*c >= '0' && *c <= '9') || *c == '_')) return false;
  return true;
}

// fill_filter / fill_codec (blosc/blosc2.c:913-971): lazy dlopen of libblosc2_<name>.so, symbol
// `info` naming the callbacks (the python-path fallback of load_lib is not reproduced).
void* load_plugin(const char* name) {
  if (!valid_plugin_name(name)) return nullptr;
  char path[512];
  snprintf(path, sizeof path, "libblosc2_%s.so", name);
  return dlopen(path, RTLD_LAZY);
}

bool lookup_filter(uint8_t id, blosc2_filter* out) {
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (auto& f : g_filters) {
    if (f.id != id) continue;
    if (f.forward == nullptr || f.backward == nullptr) {
      void* lib = load_plugin(f.name);
      FilterInfo* info = lib ? static_cast<FilterInfo*>(dlsym(lib, "info")) : nullptr;
      if (!info) { TRACE_ERROR("Could not load filter %d", id); return false; }
      f.forward = reinterpret_cast<blosc2_filter_forward_cb>(dlsym(lib, info->forward));
      f.backward = reinterpret_cast<blosc2_filter_backward_cb>(dlsym(lib, info->backward));
      if (!f.forward || !f.backward) { TRACE_ERROR("Wrong library loaded"); return false; }
    }
    *out = f;
    return true;
  }
  return false;
}

bool lookup_codec(int compcode, blosc2_codec* out) {
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (auto& c : g_codecs) {
    if (c.compcode != compcode) continue;
    if (c.encoder == nullptr || c.decoder == nullptr) {
      void* lib = load_plugin(c.compname);
      CodecInfo* info = lib ? static_cast<CodecInfo*>(dlsym(lib, "info")) : nullptr;
      if (!info) { TRACE_ERROR("Could not load codec %d.", compcode); return false; }
      c.encoder = reinterpret_cast<blosc2_codec_encoder_cb>(dlsym(lib, info->encoder));
      c.decoder = reinterpret_cast<blosc2_codec_decoder_cb>(dlsym(lib, info->decoder));
      if (!c.encoder || !c.decoder) { TRACE_ERROR("encoder or decoder cannot be loaded"); return false; }
    }
    *out = c;
    return true;
  }
  return false;
}

bool device_filter(uint8_t f) { return f <= BLOSC_TRUNC_PREC || f == b2h::kBytedelta || f == b2h::kIntTrunc; }

bool needs_host_callbacks(const uint8_t* filters, int compcode) {
  if (compcode > BLOSC2_DEFINED_CODECS_STOP) return true;
  for (int i = 0; i < 6; i++)
    if (!device_filter(filters[i])) return true;
  return false;
}

// Runs job(i) for i in [0, n): through the caller's threads callback when one is set and the
// context asks for threads (blosc2.c:181-185, 5399-5414), else in order.  Returns the first error.
template <typename F>
int run_jobs(int16_t nthreads, int n, F&& job) {
  std::vector<int> rcs((size_t)std::max(n, 0), 0);
  struct Job { F* fn; int i; int* rc; };
  if (g_threads_cb && nthreads > 1 && n > 1) {
    std::vector<Job> jobs((size_t)n);
    for (int i = 0; i < n; i++) jobs[(size_t)i] = Job{&job, i, &rcs[(size_t)i]};
    g_threads_cb(g_threads_cb_data, [](void* p) { Job* j = static_cast<Job*>(p); *j->rc = (*j->fn)(j->i); }, n,
                 sizeof(Job), jobs.data());
  } else {
    for (int i = 0; i < n; i++) {
      rcs[(size_t)i] = job(i);
      if (rcs[(size_t)i]) break;
    }
  }
  for (int r : rcs) if (r) return r;
  return 0;
}

void cycle(uint8_t*& src, uint8_t*& dst, uint8_t*& tmp) {   // _cycle_buffers (blosc/blosc2.c:1048)
  uint8_t* t = src;
  src = dst;
  dst = tmp;
  tmp = t;
}

struct HybridBufs {   // per-call device buffers of the host-callback pipelines
  DevBuf a, b, c, out;
  ~HybridBufs() { a.release(); b.release(); c.release(); out.release(); }
};

int sync_to_host(hipStream_t st, void* h, const void* d, size_t n) {
  if (n && hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, st) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
}
int to_device(hipStream_t st, void* d, const void* h, size_t n) {
  if (n && hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, st) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  return 0;
}

// The callbacks' `ttmp`: a thread context's temporaries, 4 x (blocksize + 4 * typesize) bytes
// (blosc/blosc2.c:2233-2261, 4663-4673).
uint8_t* ctx_ttmp(blosc2_context* ctx, int32_t blocksize, int32_t typesize, size_t* nbytes) {
  const size_t need = (size_t)4 * ((size_t)blocksize + 4 * (size_t)typesize);
  if (ctx->ttmp.size() < need) ctx->ttmp.assign(need, 0);
  *nbytes = need;
  return ctx->ttmp.data();
}

// pipeline_forward's prefilter step for the block at `offset` (blosc/blosc2.c:1066-1103): a copy
// of the context's params completed for the block, the output zeroed first unless disposable.
// Returns 0, 1 (the callback failed on a disposable output: the block's pipeline ends at the
// prefilter output, 1096-1099) or BLOSC2_ERROR_FILTER_PIPELINE.  `out` holds >= the output size.
int call_prefilter(blosc2_context* ctx, const b2h::CompressPlan& P, const uint8_t* in, uint8_t* out, int32_t bsize,
                   int32_t offset) {
  blosc2_prefilter_params pp;
  memcpy(&pp, ctx->preparams, sizeof pp);
  const bool disposable = ctx->preparams->output_is_disposable;
  const int32_t ts = P.typesize;
  const int32_t ots = pp.output_typesize > 0 ? pp.output_typesize : ts;
  const int32_t osize = bsize / ts * ots;
  pp.output_typesize = ots;
  if (!disposable) memset(out, 0, (size_t)osize);
  pp.input = in;
  pp.output = out;
  pp.output_size = osize;
  pp.output_offset = offset;
  pp.nblock = offset / P.blocksize;
  pp.nchunk = ctx->schunk ? static_cast<blosc2_schunk*>(ctx->schunk)->current_nchunk : -1;
  pp.tid = 0;
  pp.ttmp = ctx_ttmp(ctx, P.blocksize, ts, &pp.ttmp_nbytes);
  pp.ctx = ctx;
  pp.output_is_disposable = disposable;
  if (ctx->prefilter(&pp) != 0) {
    if (disposable) return 1;
    TRACE_ERROR("Execution of prefilter function failed");
    return BLOSC2_ERROR_FILTER_PIPELINE;
  }
  return 0;
}

// Bytes a prefilter may write for one block (its output size, or the block).
size_t prefilter_span(const blosc2_context* ctx, const b2h::CompressPlan& P) {
  const int32_t ots = ctx->preparams->output_typesize > 0 ? ctx->preparams->output_typesize : P.typesize;
  return (size_t)std::max<int64_t>(P.blocksize, (int64_t)(P.blocksize / P.typesize) * ots) + 64;
}

// A memcpyed chunk compressed with a prefilter holds the prefilter's outputs, block by block
// (serial_blosc 2188-2200 -> blosc_c 1241-1248: the prefilter writes straight into the chunk).
// `raw` is the input as the pipeline leaves it; the chunk's payload in `dest` is rewritten.
int prefilter_memcpyed(blosc2_context* ctx, const b2h::CompressPlan& P, const uint8_t* raw, int32_t n, uint8_t* dest,
                       int32_t destsize, int32_t ovh) {
  std::vector<uint8_t> blk(prefilter_span(ctx, P));
  for (int64_t off = 0; off < n; off += P.blocksize) {
    const int32_t bsize = (int32_t)std::min<int64_t>(P.blocksize, n - off);
    uint8_t* o = dest + ovh + off;
    memcpy(blk.data(), o, (size_t)std::min<int64_t>(bsize, destsize - ovh - off));   // bytes left unwritten stay
    const int r = call_prefilter(ctx, P, raw + off, blk.data(), bsize, (int32_t)off);
    if (r < 0) return r;
    memcpy(o, blk.data(), (size_t)std::min<int64_t>(bsize, destsize - ovh - off));
  }
  return 0;
}

int compress_hybrid(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                    int32_t blocksize_in, bool sticky, bool extended) {
  blosc2_codec codec{};
  const bool ucodec = ctx->compcode > BLOSC2_DEFINED_CODECS_STOP;
  if (ucodec && !lookup_codec(ctx->compcode, &codec)) {
    TRACE_ERROR("User-defined compressor codec %d not found during compression", ctx->compcode);
    return BLOSC2_ERROR_CODEC_SUPPORT;
  }
  b2h::CompressPlan P;
  int32_t computed = 0;
  int rc = b2h::make_compress_plan(&P, srcsize, destsize, ctx->clevel, ctx->typesize, blocksize_in, ctx->splitmode,
                                   ctx->filters, ctx->filters_meta, &computed, extended, ctx->compcode,
                                   ctx->compcode_meta, ucodec ? codec.version : 1);
  if (rc < 0) return rc;
  P.lz_mode = ctx->lz_mode;
  if (sticky) ctx->blocksize = computed;
  if ((rc = check_supported(ctx, true)) < 0) return rc;
  if (P.use_dict) {
    // the dictionary's training pass is a device-pipeline feature (compress_batch); host-callback
    // pipelines (user filters, prefilters) do not run it
    TRACE_ERROR("`use_dict` with user-registered filters is not supported by the MI355X engine");
    return BLOSC2_ERROR_CODEC_PARAM;
  }
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  const int32_t n = srcsize, ovh = P.overhead;
  HybridBufs hb;
  if (!hb.a.ensure((size_t)n) || !hb.b.ensure((size_t)n) || !hb.c.ensure((size_t)n) ||
      !hb.out.ensure((size_t)destsize) || !d.small.ensure(64))
    return BLOSC2_ERROR_MEMORY_ALLOC;
  if ((rc = to_device(d.stream, hb.a.p, src, (size_t)n))) return rc;
  int32_t* d_cb = reinterpret_cast<int32_t*>(d.small.p);
  blosc2_cparams cp;
  blosc2_ctx_get_cparams(ctx, &cp);
  if (P.memcpyed) {   // chunk-level memcpy: no filter or codec runs (a prefilter does)
    rc = b2h::compress_batch(P, hb.a.u8(), 0, 1, hb.out.u8(), 0, d_cb, d.stream, d.ws);
    if (rc < 0) return rc;
    int32_t cb = 0;
    if ((rc = sync_to_host(d.stream, &cb, d_cb, 4))) return rc;
    const int32_t ncopy = cb > 0 ? cb : std::min(destsize, ovh);
    if (hipMemcpy(dest, hb.out.p, (size_t)ncopy, hipMemcpyDeviceToHost) != hipSuccess) return BLOSC2_ERROR_FAILURE;
    if (cb > 0 && ctx->prefilter &&
        (rc = prefilter_memcpyed(ctx, P, static_cast<const uint8_t*>(src), n, static_cast<uint8_t*>(dest), destsize, ovh)))
      return rc;
    return cb;
  }
  const int32_t bs = P.blocksize, nblocks = n / bs + (n % bs ? 1 : 0);
  if (ctx->prefilter && ctx->preparams->output_is_disposable && extended) {
    // A disposable output: blosc_c writes every stream as a run of zeros whatever the pipeline
    // produced (blosc/blosc2.c:1286-1291), so the chunk ends as SPECIAL_ZERO (3054-3063); the
    // prefilter still runs once per block, in block order
    std::vector<uint8_t> blk(prefilter_span(ctx, P));
    for (int32_t b = 0; b < nblocks; b++)
      (void)call_prefilter(ctx, P, static_cast<const uint8_t*>(src) + (int64_t)b * bs, blk.data(),
                           std::min<int32_t>(bs, n - b * bs), b * bs);
    if (destsize < ovh) return 0;
    uint8_t hdr[BLOSC_EXTENDED_HEADER_LENGTH];
    memcpy(hdr, P.header, sizeof hdr);
    hdr[31] |= (uint8_t)(BLOSC2_SPECIAL_ZERO << 4);
    const int32_t cb = ovh;
    memcpy(hdr + 12, &cb, 4);
    memcpy(dest, hdr, sizeof hdr);
    return cb;
  }
  bool has_delta = false;
  for (int i = 0; i < 6; i++) has_delta |= P.filters[i] == BLOSC_DELTA;
  // ---- forward pipeline (block 0 first with DELTA: the serial walk's order) ----
  std::vector<uint8_t> hs, hd;
  std::vector<std::pair<int32_t, std::vector<uint8_t>>> disposed;   // blocks whose pipeline ended at the prefilter
  uint8_t* fsrc = hb.a.u8();
  for (int pass = (has_delta && nblocks > 1) ? 1 : 0; pass <= ((has_delta && nblocks > 1) ? 2 : 0); pass++) {
    uint8_t *s = hb.a.u8(), *t = hb.b.u8(), *u = hb.c.u8();
    const int32_t b0 = pass == 2 ? 1 : 0, b1 = pass == 1 ? 1 : nblocks;
    const int64_t lo = (int64_t)b0 * bs, hi = std::min<int64_t>((int64_t)b1 * bs, n);
    if (ctx->prefilter) {   // pipeline_forward's prefilter, before slot 0 (blosc/blosc2.c:1069-1110)
      hs.resize((size_t)n);
      hd.resize((size_t)n);
      std::vector<uint8_t> blk(prefilter_span(ctx, P));
      if ((rc = sync_to_host(d.stream, hs.data() + lo, s + lo, (size_t)(hi - lo)))) return rc;
      for (int32_t b = b0; b < b1; b++) {
        const int32_t bsize = std::min<int32_t>(bs, n - b * bs);
        const int r = call_prefilter(ctx, P, hs.data() + (int64_t)b * bs, blk.data(), bsize, b * bs);
        if (r < 0) return r;
        memcpy(hd.data() + (int64_t)b * bs, blk.data(), (size_t)bsize);
        if (r == 1) disposed.emplace_back(b, std::vector<uint8_t>(blk.data(), blk.data() + bsize));
      }
      if ((rc = to_device(d.stream, t + lo, hd.data() + lo, (size_t)(hi - lo)))) return rc;
      cycle(s, t, u);
    }
    for (int i = 0; i < 6; i++) {
      const uint8_t f = P.filters[i];
      if (f == BLOSC_NOFILTER) continue;
      if (device_filter(f)) {
        if ((rc = b2h::forward_filter_chunk(P, i, pass, s, t, hb.a.u8(), d.stream)) < 0) return rc;
      } else {
        blosc2_filter flt{};
        if (!lookup_filter(f, &flt)) {
          TRACE_ERROR("User-defined filter %d not found during compression", f);
          return BLOSC2_ERROR_FILTER_PIPELINE;
        }
        hs.resize((size_t)n);
        hd.resize((size_t)n);
        if ((rc = sync_to_host(d.stream, hs.data() + lo, s + lo, (size_t)(hi - lo)))) return rc;
        rc = run_jobs(ctx->nthreads, b1 - b0, [&](int k) {
          const int32_t b = b0 + k;
          const int32_t bsize = std::min<int32_t>(bs, n - b * bs);
          blosc2_cparams cpl = cp;
          const int r = flt.forward(hs.data() + (int64_t)b * bs, hd.data() + (int64_t)b * bs, bsize,
                                    P.filters_meta[i], &cpl, f);
          return r != BLOSC2_ERROR_SUCCESS ? (int)BLOSC2_ERROR_FILTER_PIPELINE : 0;
        });
        if (rc) { TRACE_ERROR("User-defined filter %d failed during compression", f); return rc; }
        if ((rc = to_device(d.stream, t + lo, hd.data() + lo, (size_t)(hi - lo)))) return rc;
      }
      cycle(s, t, u);
    }
    fsrc = s;
  }
  for (auto& db : disposed)   // 1096-1099: no filter ran after a disposable prefilter failure
    if ((rc = to_device(d.stream, fsrc + (int64_t)db.first * bs, db.second.data(), db.second.size()))) return rc;
  // ---- codec ----
  int32_t cb = 0;
  if (!ucodec) {
    rc = b2h::encode_chunk_filtered(P, fsrc, hb.a.u8(), hb.out.u8(), d_cb, d.stream, d.ws);
    if (rc < 0) return rc;
    if ((rc = sync_to_host(d.stream, &cb, d_cb, 4))) return rc;
    const int32_t ncopy = cb > 0 ? cb : std::min(destsize, ovh);
    if (hipMemcpy(dest, hb.out.p, (size_t)ncopy, hipMemcpyDeviceToHost) != hipSuccess) return BLOSC2_ERROR_FAILURE;
    // the memcpy fallback re-runs the pipeline as a memcpyed chunk: the prefilter again, over
    // the input as the first pass left it (blosc_compress_context 3017-3051)
    if (cb > 0 && ctx->prefilter && (static_cast<uint8_t*>(dest)[2] & BLOSC_MEMCPYED)) {
      std::vector<uint8_t> raw((size_t)n);
      if ((rc = sync_to_host(d.stream, raw.data(), hb.a.p, (size_t)n))) return rc;
      if ((rc = prefilter_memcpyed(ctx, P, raw.data(), n, static_cast<uint8_t*>(dest), destsize, ovh))) return rc;
    }
    return cb;
  }
  // user encoder per stream, serial layout (blosc_c / serial_blosc / blosc_compress_context)
  std::vector<uint8_t> filt((size_t)n + 1), raw((size_t)n + 1), out((size_t)destsize + 1);
  if ((rc = sync_to_host(d.stream, filt.data(), fsrc, (size_t)n))) return rc;
  if ((rc = sync_to_host(d.stream, raw.data(), hb.a.p, (size_t)n))) return rc;   // memcpy source
  uint8_t* o = out.data();
  memcpy(o, P.header, (size_t)ovh);
  int32_t ntbytes = ovh + 4 * nblocks;
  const bool split = !((P.header[2] >> 4) & 1);
  bool ok = ntbytes <= destsize;
  for (int32_t b = 0; b < nblocks && ok; b++) {
    const int32_t bsize = std::min<int32_t>(bs, n - b * bs);
    const bool leftover = bsize < bs;
    const int32_t ns = (split && !leftover) ? P.typesize : 1, neblock = bsize / ns;
    const int32_t bstart = ntbytes;
    memcpy(o + ovh + 4 * b, &bstart, 4);
    for (int32_t j = 0; j < ns && ok; j++) {
      const uint8_t* ip = filt.data() + (int64_t)b * bs + (int64_t)j * neblock;
      ntbytes += 4;
      if (extended && std::all_of(ip, ip + neblock, [&](uint8_t x) { return x == ip[0]; })) {
        if (ntbytes > destsize) { ok = false; break; }
        const int32_t v = -(int32_t)ip[0];
        memcpy(o + ntbytes - 4, &v, 4);
        if (ip[0]) {
          ntbytes += 1;
          if (ntbytes > destsize) { ok = false; break; }
          o[ntbytes - 1] = 0x1;
        }
        continue;
      }
      int32_t maxout = neblock;
      if (ntbytes + maxout > destsize) {
        maxout = destsize - ntbytes;
        if (maxout <= 0) { ok = false; break; }
      }
      blosc2_cparams cpl = cp;
      int32_t c = codec.encoder(ip, neblock, o + ntbytes, maxout, ctx->compcode_meta, &cpl, raw.data());
      if (c > maxout) return BLOSC2_ERROR_WRITE_BUFFER;
      if (c < 0) return BLOSC2_ERROR_DATA;
      if (c == 0) c = neblock;
      if (c == neblock) {
        if (ntbytes + neblock > destsize) { ok = false; break; }
        memcpy(o + ntbytes, ip, (size_t)neblock);
      }
      memcpy(o + ntbytes - 4, &c, 4);
      ntbytes += c;
    }
  }
  if (ok) {
    int32_t nstreams = nblocks;
    if (split) nstreams = (n % bs) ? (nblocks - 1) * P.typesize + 1 : nblocks * P.typesize;
    if (ntbytes == ovh + 4 * nblocks + 4 * nstreams) {   // every stream a zero run: SPECIAL_ZERO
      o[31] |= (uint8_t)(BLOSC2_SPECIAL_ZERO << 4);
      ntbytes = ovh;
    }
    cb = ntbytes;
  } else if (n + ovh <= destsize) {   // memcpy fallback: the (possibly rewritten) input
    o[2] |= BLOSC_MEMCPYED;
    memcpy(o + ovh, raw.data(), (size_t)n);
    cb = n + ovh;
    if (ctx->prefilter && (rc = prefilter_memcpyed(ctx, P, raw.data(), n, o, destsize, ovh))) return rc;
  } else {
    cb = 0;
  }
  memcpy(o + 12, &cb, 4);
  memcpy(dest, o, (size_t)(cb > 0 ? cb : std::min(destsize, ovh)));
  return cb;
}

int decompress_hybrid(blosc2_context* ctx, const void* src, int32_t srcsize, void* dest, int32_t destsize,
                      const std::vector<uint8_t>* mask, int mode) {
  const uint8_t* s = static_cast<const uint8_t*>(src);
  const int32_t nbytes = rd32(s + 4), cbytes = rd32(s + 12);
  // lazy chunks (their blocks live in a frame) are not read here: init_from_header skips their
  // cbytes <= srcsize check, and the copy below reads cbytes bytes of `src`
  if (cbytes > srcsize) return BLOSC2_ERROR_INVALID_PARAM;
  int32_t bs = rd32(s + 8);
  const int ts = s[3];
  if (nbytes > 0 && bs > nbytes) bs = nbytes;
  const int32_t nblocks = nbytes > 0 ? nbytes / bs + (nbytes % bs ? 1 : 0) : 0;
  const bool ucodec = (s[2] >> 5) == BLOSC_UDCODEC_FORMAT;
  const int ccode = s[22], cmeta = s[23];
  const int32_t ovh = BLOSC_EXTENDED_HEADER_LENGTH;
  if (srcsize < ovh + 4 * nblocks) return BLOSC2_ERROR_READ_BUFFER;
  blosc2_codec codec{};
  if (ucodec && !lookup_codec(ccode, &codec)) {
    TRACE_ERROR("User-defined compressor codec %d not found during decompression", ccode);
    return BLOSC2_ERROR_CODEC_SUPPORT;
  }
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  HybridBufs hb;
  if (!hb.a.ensure((size_t)std::max(cbytes, nbytes)) || !hb.b.ensure((size_t)nbytes) || !hb.c.ensure((size_t)nbytes) ||
      !hb.out.ensure((size_t)nbytes) || !d.small.ensure(64))
    return BLOSC2_ERROR_MEMORY_ALLOC;
  blosc2_dparams dp;
  blosc2_ctx_get_dparams(ctx, &dp);
  int rc = 0;
  uint8_t* unf = hb.b.u8();   // the decoded, still filtered image
  if (ucodec) {
    // blosc_d per stream with the user decoder (blosc/blosc2.c:1987-2136)
    std::vector<uint8_t> img((size_t)nbytes + 1);
    const bool split = !((s[2] >> 4) & 1);
    std::vector<std::pair<int32_t, int32_t>> streams;   // (src offset of the csize word, dst offset)
    for (int32_t b = 0; b < nblocks; b++) {
      const int32_t bsize = std::min<int32_t>(bs, nbytes - b * bs);
      const int32_t ns = (split && bsize == bs) ? ts : 1, neblock = bsize / ns;
      int32_t pos = rd32(s + ovh + 4 * b);
      for (int32_t j = 0; j < ns; j++) {
        if (pos < 0 || pos > srcsize - 4) return BLOSC2_ERROR_READ_BUFFER;
        const int32_t cs = rd32(s + pos);
        streams.push_back({pos, b * bs + j * neblock});
        // 64-bit: a csize near INT32_MAX must not wrap the cursor back into the buffer
        const int64_t next = (int64_t)pos + 4 + (cs > 0 ? cs : (cs < 0 ? 1 : 0));
        pos = next > srcsize ? srcsize : (int32_t)next;
        (void)neblock;
      }
    }
    rc = run_jobs(ctx->nthreads, (int)streams.size(), [&](int k) {
      const int32_t pos = streams[(size_t)k].first, off = streams[(size_t)k].second;
      const int32_t b = off / bs;
      const int32_t bsize = std::min<int32_t>(bs, nbytes - b * bs);
      const int32_t ns = (split && bsize == bs) ? ts : 1, neblock = bsize / ns;
      const int32_t cs = rd32(s + pos);
      const uint8_t* in = s + pos + 4;
      uint8_t* o = img.data() + off;
      if (cs == 0) { memset(o, 0, (size_t)neblock); return 0; }
      if (cs < 0) {
        if (!(in[0] & 1) || cs < -255) return (int)BLOSC2_ERROR_RUN_LENGTH;
        memset(o, -cs, (size_t)neblock);
        return 0;
      }
      if (cs > srcsize - pos - 4) return (int)BLOSC2_ERROR_READ_BUFFER;   // subtraction form: no int32 overflow
      if (cs == neblock) { memcpy(o, in, (size_t)neblock); return 0; }
      blosc2_dparams dpl = dp;
      const int r = codec.decoder(in, cs, o, neblock, (uint8_t)cmeta, &dpl, src);
      return r != neblock ? (int)BLOSC2_ERROR_DATA : 0;
    });
    if (rc) return rc;
    if ((rc = to_device(d.stream, unf, img.data(), (size_t)nbytes))) return rc;
  } else {
    // device decode of the streams only (the filters follow below)
    struct Ptrs { const uint8_t* s; uint8_t* o; int32_t ss, ds, status, pad; } h{hb.a.u8(), unf, cbytes, nbytes, 0, 0};
    uint8_t* sm = d.small.u8();
    if ((rc = to_device(d.stream, hb.a.p, src, (size_t)cbytes)) || (rc = to_device(d.stream, sm, &h, sizeof h))) return rc;
    Ptrs* dptr = reinterpret_cast<Ptrs*>(sm);
    rc = b2h::decompress_batch(reinterpret_cast<const uint8_t* const*>(&dptr->s), &dptr->ss,
                               reinterpret_cast<uint8_t* const*>(&dptr->o), &dptr->ds, 1, nbytes, &dptr->status, nullptr,
                               d.stream, d.ws, cbytes, 1);
    if (rc < 0) return rc;
    int32_t status = 0;
    if ((rc = sync_to_host(d.stream, &status, &dptr->status, 4))) return rc;
    if (status != nbytes) return status < 0 ? status : BLOSC2_ERROR_DATA;
  }
  // ---- pipeline_backward, slots 5 -> 0, block 0 first with DELTA ----
  uint8_t filters[6], fmeta[6];
  for (int i = 0; i < 6; i++) { filters[i] = s[16 + i]; fmeta[i] = s[24 + i]; }
  if (s[0] == BLOSC2_VERSION_FORMAT_ALPHA) { filters[5] = 0; fmeta[5] = 0; }
  bool has_delta = false;
  for (int i = 0; i < 6; i++) has_delta |= filters[i] == BLOSC_DELTA;
  std::vector<uint8_t> hs, hd;
  uint8_t* fin = hb.out.u8();
  // DELTA: block 0 first, then the others against the final block 0 (blosc/blosc2.c:1505-1529);
  // kDecDeltaSelf (getitem / decompress_block): every block un-deltas against itself, as blosc_d
  // does with dest_offset 0 -- one pass, backward_filter_chunk's pass 3
  const bool self = (mode & b2h::kDecDeltaSelf) != 0;
  const bool two = has_delta && nblocks > 1 && !self;
  const int pfirst = two ? 1 : (self && has_delta ? 3 : 0), plast = two ? 2 : pfirst;
  for (int pass = pfirst; pass <= plast; pass++) {
    uint8_t *cur = unf, *nxt = hb.c.u8();
    const int32_t b0 = pass == 2 ? 1 : 0, b1 = pass == 1 ? 1 : nblocks;
    const int64_t lo = (int64_t)b0 * bs, hi = std::min<int64_t>((int64_t)b1 * bs, nbytes);
    for (int i = 5; i >= 0; i--) {
      const uint8_t f = filters[i];
      if (f == BLOSC_NOFILTER || f == BLOSC_TRUNC_PREC || f == b2h::kIntTrunc) continue;   // nothing to undo
      if (device_filter(f)) {
        if ((rc = b2h::backward_filter_chunk(f, fmeta[i], ts, nbytes, bs, s[0], pass, cur, nxt, fin, d.stream)) < 0)
          return rc;
      } else {
        blosc2_filter flt{};
        if (!lookup_filter(f, &flt)) {
          TRACE_ERROR("User-defined filter %d not found during decompression.", f);
          return BLOSC2_ERROR_FILTER_PIPELINE;
        }
        hs.resize((size_t)nbytes);
        hd.resize((size_t)nbytes);
        if ((rc = sync_to_host(d.stream, hs.data() + lo, cur + lo, (size_t)(hi - lo)))) return rc;
        rc = run_jobs(ctx->nthreads, b1 - b0, [&](int k) {
          const int32_t b = b0 + k;
          const int32_t bsize = std::min<int32_t>(bs, nbytes - b * bs);
          blosc2_dparams dpl = dp;
          return flt.backward(hs.data() + (int64_t)b * bs, hd.data() + (int64_t)b * bs, bsize, fmeta[i], &dpl, f);
        });
        if (rc) { TRACE_ERROR("User-defined filter %d failed during decompression.", f); return rc; }
        if ((rc = to_device(d.stream, nxt + lo, hd.data() + lo, (size_t)(hi - lo)))) return rc;
      }
      std::swap(cur, nxt);
    }
    if (hipMemcpyAsync(fin + lo, cur + lo, (size_t)(hi - lo), hipMemcpyDeviceToDevice, d.stream) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
  }
  if (nbytes > destsize) return BLOSC2_ERROR_WRITE_BUFFER;
  if (hipStreamSynchronize(d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  for (int32_t b = 0; b < nblocks; b++) {
    if (mask && (*mask)[(size_t)b]) continue;
    const int64_t off = (int64_t)b * bs, len = std::min<int64_t>(bs, nbytes - off);
    if (hipMemcpy(static_cast<uint8_t*>(dest) + off, fin + off, (size_t)len, hipMemcpyDeviceToHost) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
  }
  return nbytes;
}

}  // namespace

// --------------------------------------------------- super-chunk layer helpers (b2h_schunk.cpp) ----
namespace b2h {
// Consecutive blosc2_compress_ctx calls on one context, as ONE queue of device batches: chunk i =
// d_src + i * src_stride (nbytes[i] bytes) into d_dst + i * dst_stride with destsize nbytes[i] + 32
// (blosc2_schunk_append_buffer, blosc/schunk.c:1459-1477).  The context's sticky blocksize is
// carried from chunk to chunk exactly as the serial calls carry it (blosc/blosc2.c:3130-3133: the
// previous call's blocksize is the next call's request), so runs of chunks whose plans agree share
// one launch and every chunk equals the serial call's bytes.  Asynchronous on the context's stream.
// Caller holds ctx->mu.
static int compress_device_locked(blosc2_context* ctx, const uint8_t* d_src, const int32_t* nbytes, int32_t n,
                                  int64_t src_stride, uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes) {
  if (n > 0 && (!nbytes || !d_src || !d_dst || !d_cbytes)) return BLOSC2_ERROR_NULL_POINTER;
  if (ctx->do_compress != 1) return BLOSC2_ERROR_INVALID_PARAM;
  int rc = check_supported(ctx);
  if (rc < 0) return rc;
  if (needs_host_callbacks(ctx->filters, ctx->compcode)) {
    TRACE_ERROR("user filters / codecs run per chunk through blosc2_compress_ctx, not the device batch");
    return BLOSC2_ERROR_FILTER_PIPELINE;
  }
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  int32_t i = 0;
  while (i < n) {
    if (nbytes[i] < 0 || (int64_t)nbytes[i] > src_stride || (int64_t)nbytes[i] + BLOSC2_MAX_OVERHEAD > dst_stride)
      return BLOSC2_ERROR_INVALID_PARAM;
    b2h::CompressPlan plan;
    int32_t computed = 0;
    rc = b2h::make_compress_plan(&plan, nbytes[i], nbytes[i] + BLOSC2_MAX_OVERHEAD, ctx->clevel, ctx->typesize,
                                 ctx->blocksize, ctx->splitmode, ctx->filters, ctx->filters_meta, &computed, true,
                                 ctx->compcode, ctx->compcode_meta, 1, ctx->use_dict);
    if (rc < 0) return rc;
    plan.lz_mode = ctx->lz_mode;
    ctx->blocksize = computed;
    // the following chunks of the same size request `computed`: same plan while it stays put
    int32_t j = i + 1;
    while (j < n && nbytes[j] == nbytes[i]) {
      b2h::CompressPlan q;
      int32_t c2 = 0;
      if (b2h::make_compress_plan(&q, nbytes[j], nbytes[j] + BLOSC2_MAX_OVERHEAD, ctx->clevel, ctx->typesize,
                                  ctx->blocksize, ctx->splitmode, ctx->filters, ctx->filters_meta, &c2, true,
                                  ctx->compcode, ctx->compcode_meta, 1, ctx->use_dict) < 0 ||
          c2 != computed || q.blocksize != plan.blocksize || q.split != plan.split || q.memcpyed != plan.memcpyed ||
          memcmp(q.header, plan.header, sizeof q.header) != 0)
        break;
      j++;
    }
    rc = b2h::compress_batch(plan, d_src + (int64_t)i * src_stride, src_stride, j - i, d_dst + (int64_t)i * dst_stride,
                             dst_stride, d_cbytes + i, d.stream, d.ws);
    if (rc < 0) {
      TRACE_ERROR("device compression failed: %s", b2h::last_error());
      return rc;
    }
    i = j;
  }
  return 0;
}

blosc2_context* ctx_clone(const blosc2_context* ctx) {
  if (!ctx) return nullptr;
  blosc2_context* c = new (std::nothrow) blosc2_context();
  if (!c) return nullptr;
  c->do_compress = ctx->do_compress;
  c->compcode = ctx->compcode;
  c->compcode_meta = ctx->compcode_meta;
  c->clevel = ctx->clevel;
  c->use_dict = ctx->use_dict;
  c->typesize = ctx->typesize;
  c->nthreads = ctx->nthreads;
  c->blocksize = ctx->blocksize;
  c->splitmode = ctx->splitmode;
  c->schunk = ctx->schunk;
  memcpy(c->filters, ctx->filters, sizeof c->filters);
  memcpy(c->filters_meta, ctx->filters_meta, sizeof c->filters_meta);
  c->prefilter = ctx->prefilter;
  c->pre_copy = ctx->pre_copy;
  c->preparams = ctx->prefilter ? &c->pre_copy : nullptr;
  c->post_copy = ctx->post_copy;
  c->tuner_params = ctx->tuner_params;
  c->tuner_id = ctx->tuner_id;
  c->instr_codec = ctx->instr_codec;
  c->codec_params = ctx->codec_params;
  c->lz_mode = ctx->lz_mode;
  memcpy(c->filter_params, ctx->filter_params, sizeof c->filter_params);
  c->dparams = ctx->dparams;
  if (c->dparams.postfilter) c->dparams.postparams = &c->post_copy;
  return c;
}

int ctx_blocksize_walk(const blosc2_context* ctx, const int32_t* nbytes, int32_t n, int32_t* before) {
  if (!ctx || !before || (n > 0 && !nbytes)) return BLOSC2_ERROR_NULL_POINTER;
  int32_t state = ctx->blocksize;
  for (int32_t i = 0; i < n; i++) {
    before[i] = state;
    b2h::CompressPlan plan;
    int32_t computed = 0;
    const int rc = b2h::make_compress_plan(&plan, nbytes[i], nbytes[i] + BLOSC2_MAX_OVERHEAD, ctx->clevel, ctx->typesize,
                                           state, ctx->splitmode, ctx->filters, ctx->filters_meta, &computed, true,
                                           ctx->compcode, ctx->compcode_meta, 1, ctx->use_dict);
    if (rc < 0) return rc;
    state = computed;
  }
  before[n] = state;
  return 0;
}

void ctx_set_blocksize(blosc2_context* ctx, int32_t blocksize) {
  std::lock_guard<std::mutex> g(ctx->mu);
  ctx->blocksize = blocksize;
}

int ctx_compress_device(blosc2_context* ctx, const uint8_t* d_src, const int32_t* nbytes, int32_t n,
                        int64_t src_stride, uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes) {
  if (!ctx) return BLOSC2_ERROR_NULL_POINTER;
  std::lock_guard<std::mutex> g(ctx->mu);
  return compress_device_locked(ctx, d_src, nbytes, n, src_stride, d_dst, dst_stride, d_cbytes);
}

// n appends' worth of chunks: compressed in groups of <= 512 MiB of output slots, each group
// packed on the device (pack_chunks) and brought back in ONE copy through pinned memory, then split
// into malloc'd chunks of exactly cbytes bytes (the shrunk chunk blosc2_schunk_append_chunk keeps,
// blosc/schunk.c:1055-1058).  On failure nothing is returned (every chunk produced so far is freed).
// The context's sticky blocksize advances over all n chunks here; when the caller's append of
// chunk i then fails (b2h_schunk_append_device), the context's blocksize is the one after chunk
// n-1, not after chunk i as in the serial walk: after a failed device append the context state is
// unspecified (include/b2h.h).
int ctx_append_device(blosc2_context* ctx, const uint8_t* d_src, const int32_t* nbytes, int32_t n,
                      int64_t src_stride, uint8_t** chunks_out) {
  if (!ctx || (n > 0 && (!nbytes || !d_src || !chunks_out))) return BLOSC2_ERROR_NULL_POINTER;
  if (n < 0) return BLOSC2_ERROR_INVALID_PARAM;
  int32_t maxnb = 0;
  for (int32_t i = 0; i < n; i++) {
    chunks_out[i] = nullptr;
    if (nbytes[i] < 0 || nbytes[i] > BLOSC2_MAX_BUFFERSIZE || (int64_t)nbytes[i] > src_stride)
      return BLOSC2_ERROR_INVALID_PARAM;
    maxnb = std::max(maxnb, nbytes[i]);
  }
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(ctx->mu);
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  const int64_t dst_stride = ((int64_t)maxnb + BLOSC2_MAX_OVERHEAD + 255) & ~int64_t(255);
  const int32_t group = (int32_t)std::max<int64_t>(1, std::min<int64_t>(n, (int64_t(512) << 20) / dst_stride));
  const size_t cb_bytes = ((size_t)group * 4 + 63) & ~size_t(63);
  if (!d.out.ensure((size_t)(group * dst_stride)) || !d.in.ensure((size_t)(group * dst_stride)) ||
      !d.small.ensure(cb_bytes + 8 * ((size_t)group + 1)))
    return BLOSC2_ERROR_MEMORY_ALLOC;
  int32_t* d_cb = reinterpret_cast<int32_t*>(d.small.p);
  int64_t* d_off = reinterpret_cast<int64_t*>(d.small.u8() + cb_bytes);
  std::vector<int64_t> off((size_t)group + 1);
  auto fail = [&](int rc) {
    for (int32_t i = 0; i < n; i++) {
      free(chunks_out[i]);
      chunks_out[i] = nullptr;
    }
    return rc;
  };
  std::vector<int32_t> cbh((size_t)group);
  for (int32_t g0 = 0; g0 < n; g0 += group) {
    const int32_t m = std::min(group, n - g0);
    // a fused launch whose hand-off wait timed out fails its whole batch with FAILURE (b2h.h): the
    // group runs once more with the separate launches, from the sticky blocksize it started with,
    // so every chunk is still the serial blosc2_schunk_append_buffer's
    const int32_t blocksize0 = ctx->blocksize;
    for (int attempt = 0; attempt < 2; attempt++) {
      ctx->blocksize = blocksize0;
      b2h::set_fuse_disabled(attempt > 0);
      int rc = compress_device_locked(ctx, d_src + (int64_t)g0 * src_stride, nbytes + g0, m, src_stride, d.out.u8(),
                                      dst_stride, d_cb);
      b2h::set_fuse_disabled(false);
      if (rc < 0) return fail(rc);
      if (hipMemcpyAsync(cbh.data(), d_cb, 4 * (size_t)m, hipMemcpyDeviceToHost, d.stream) != hipSuccess ||
          hipStreamSynchronize(d.stream) != hipSuccess)
        return fail(BLOSC2_ERROR_FAILURE);
      if (std::find(cbh.begin(), cbh.begin() + m, (int32_t)BLOSC2_ERROR_FAILURE) == cbh.begin() + m) break;
    }
    if (b2h::pack_chunks(d.out.u8(), dst_stride, d_cb, m, d.in.u8(), d_off, d.stream) < 0) return fail(BLOSC2_ERROR_FAILURE);
    if (hipMemcpyAsync(off.data(), d_off, 8 * ((size_t)m + 1), hipMemcpyDeviceToHost, d.stream) != hipSuccess ||
        hipStreamSynchronize(d.stream) != hipSuccess)
      return fail(BLOSC2_ERROR_FAILURE);
    for (int32_t k = 0; k < m; k++)
      if (off[k + 1] - off[k] < BLOSC_MIN_HEADER_LENGTH) return fail(BLOSC2_ERROR_FAILURE);   // never with destsize nbytes + 32
    const int64_t total = off[m];
    if (!d.host.ensure((size_t)total)) return fail(BLOSC2_ERROR_MEMORY_ALLOC);
    if (hipMemcpyAsync(d.host.p, d.in.p, (size_t)total, hipMemcpyDeviceToHost, d.stream) != hipSuccess ||
        hipStreamSynchronize(d.stream) != hipSuccess)
      return fail(BLOSC2_ERROR_FAILURE);
    // one malloc'd buffer per chunk (the super-chunk owns them); fresh pages fault in on the first
    // write, so the copies are split over a few threads
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>({8, total >> 23, m}));
    std::vector<char> ok((size_t)T, 1);
    auto part = [&](int t) {
      for (int32_t k = m * t / T; k < m * (t + 1) / T; k++) {
        const size_t sz = (size_t)(off[k + 1] - off[k]);
        uint8_t* c = static_cast<uint8_t*>(malloc(sz));
        if (!c) { ok[(size_t)t] = 0; continue; }
        memcpy(c, d.host.u8() + off[k], sz);
        chunks_out[g0 + k] = c;
      }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; t++) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
    for (char c : ok)
      if (!c) return fail(BLOSC2_ERROR_MEMORY_ALLOC);
  }
  return 0;
}

// True when `ctx` decodes chunk `c` entirely on the device -- no postfilter, no user filter or
// codec -- and its header reads; *nbytes / *cbytes from the header.  The fan-out's staged
// pipeline (b2h_schunk.cpp) queues only such chunks itself and hands the others to
// ctx_decompress_device.
bool ctx_chunk_on_device(const blosc2_context* ctx, const uint8_t* c, int32_t* nbytes, int32_t* cbytes) {
  if (!ctx || !c || ctx->dparams.postfilter) return false;
  if (blosc2_cbuffer_sizes(c, nbytes, cbytes, nullptr) < 0) return false;
  ChunkHdr H;
  if (read_header(c, *cbytes, &H) != 0) return false;
  return !chunk_needs_host(c, H);
}

// n host chunks (what blosc2_schunk_decompress_chunk would be handed one by one, schunk.c:1481-1530)
// staged into pinned memory, copied to HBM in one DMA and decoded by one device batch straight into
// d_dst + i * dst_stride.  Chunks with user-registered filters / codecs run the host-callback pipeline
// one by one and are copied up afterwards.  A pending blosc2_set_maskout is not applied (it stays
// for the next blosc2_decompress_ctx).  Returns 0 or the first chunk's error (status[] has them all).
int ctx_decompress_device(blosc2_context* ctx, const uint8_t* const* chunks, int32_t n, uint8_t* d_dst,
                          int64_t dst_stride, int32_t dst_cap, int32_t* status) {
  if (!ctx || (n > 0 && (!chunks || !status || !d_dst))) return BLOSC2_ERROR_NULL_POINTER;
  if (n < 0 || dst_cap < 0 || (n > 1 && dst_stride < dst_cap)) return BLOSC2_ERROR_INVALID_PARAM;
  if (ctx->do_compress != 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (n == 0) return 0;
  std::lock_guard<std::mutex> g(ctx->mu);
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  std::vector<int32_t> dev_idx, host_idx, nb((size_t)n, 0), cb((size_t)n, 0);
  std::vector<int64_t> at;
  int64_t total_c = 0, total_d = 0;
  for (int32_t i = 0; i < n; i++) {
    status[i] = 0;
    const uint8_t* c = chunks[i];
    if (!c) continue;   // an empty slot decompresses to nothing (schunk.c:1495-1498)
    int rc = blosc2_cbuffer_sizes(c, &nb[i], &cb[i], nullptr);
    if (rc < 0) {
      status[i] = rc;
      continue;
    }
    if (dst_cap < nb[i]) {   // schunk.c:1505-1509
      status[i] = BLOSC2_ERROR_INVALID_PARAM;
      continue;
    }
    ChunkHdr H;
    if (ctx->dparams.postfilter || (read_header(c, cb[i], &H) == 0 && chunk_needs_host(c, H))) {
      host_idx.push_back(i);   // user callbacks (filters, codecs, a postfilter) run on the host
      continue;
    }
    dev_idx.push_back(i);
    at.push_back(total_c);
    total_c += ((int64_t)cb[i] + 63) & ~int64_t(63);
    total_d += std::max(nb[i], 0);
  }
  const int32_t m = (int32_t)dev_idx.size();
  if (m > 0) {
    const size_t tbytes = (size_t)m * (8 + 8 + 4 + 4);
    if (!d.host.ensure((size_t)total_c + tbytes) || !d.in.ensure((size_t)total_c) || !d.small.ensure(tbytes + 4 * (size_t)m))
      return BLOSC2_ERROR_MEMORY_ALLOC;
    // one SoA table in the small buffer: src ptrs | dst ptrs | srcsizes | dstsizes | status
    uint8_t* sm = d.small.u8();
    const uint8_t** h_s = reinterpret_cast<const uint8_t**>(d.host.u8() + total_c);
    uint8_t** h_o = reinterpret_cast<uint8_t**>(d.host.u8() + total_c + 8 * (size_t)m);
    int32_t* h_ss = reinterpret_cast<int32_t*>(h_o + m);
    int32_t* h_ds = h_ss + m;
    for (int32_t k = 0; k < m; k++) {
      const int32_t i = dev_idx[k];
      memcpy(d.host.u8() + at[k], chunks[i], (size_t)cb[i]);
      h_s[k] = d.in.u8() + at[k];
      h_o[k] = d_dst + (int64_t)i * dst_stride;
      h_ss[k] = cb[i];
      h_ds[k] = dst_cap;
    }
    // every early return below drains the stream first: the copies read the pinned staging
    // buffer, which the next call on this context rewrites (or frees when it grows)
    auto drained = [&](int rc) {
      (void)hipStreamSynchronize(d.stream);
      return rc;
    };
    if (hipMemcpyAsync(d.in.p, d.host.p, (size_t)total_c, hipMemcpyHostToDevice, d.stream) != hipSuccess ||
        hipMemcpyAsync(sm, h_s, tbytes, hipMemcpyHostToDevice, d.stream) != hipSuccess)
      return drained(BLOSC2_ERROR_FAILURE);
    const uint8_t* const* d_s = reinterpret_cast<const uint8_t* const*>(sm);
    uint8_t* const* d_o = reinterpret_cast<uint8_t* const*>(sm + 8 * (size_t)m);
    const int32_t* d_ss = reinterpret_cast<const int32_t*>(sm + 16 * (size_t)m);
    const int32_t* d_ds = d_ss + m;
    int32_t* d_st = const_cast<int32_t*>(d_ds + m);
    int rc = b2h::decompress_batch(d_s, d_ss, d_o, d_ds, m, total_d, d_st, nullptr, d.stream, d.ws, total_c, 0);
    if (rc < 0) {
      TRACE_ERROR("device decompression failed: %s", b2h::last_error());
      return drained(rc);
    }
    std::vector<int32_t> st((size_t)m);
    if (hipMemcpyAsync(st.data(), d_st, 4 * (size_t)m, hipMemcpyDeviceToHost, d.stream) != hipSuccess ||
        hipStreamSynchronize(d.stream) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
    for (int32_t k = 0; k < m; k++) {
      const int32_t i = dev_idx[k];
      status[i] = st[k] < 0 ? st[k] : (st[k] != nb[i] ? BLOSC2_ERROR_FAILURE : st[k]);   // schunk.c:1511-1517
    }
  }
  std::vector<uint8_t> tmp;
  for (int32_t i : host_idx) {
    tmp.resize((size_t)std::max(nb[i], 1));
    int r = decompress_host(ctx, chunks[i], cb[i], tmp.data(), nb[i], nullptr);
    if (r >= 0 && r != nb[i]) r = BLOSC2_ERROR_FAILURE;
    if (r > 0 && hipMemcpy(d_dst + (int64_t)i * dst_stride, tmp.data(), (size_t)r, hipMemcpyHostToDevice) != hipSuccess)
      r = BLOSC2_ERROR_FAILURE;
    status[i] = r;
  }
  for (int32_t i = 0; i < n; i++)
    if (status[i] < 0) return status[i];
  return 0;
}
}  // namespace b2h

namespace {

blosc2_context* g_global_cctx = nullptr;
blosc2_context* g_global_dctx = nullptr;

}  // namespace

extern "C" {

void blosc2_init(void) {
  std::lock_guard<std::mutex> g(g_global_mu);
  if (g_initlib) return;
  g_initlib = true;
}

// blosc/blosc2.c:6009-6036: the global contexts and every device's default workspace go
void blosc2_destroy(void) {
  std::lock_guard<std::mutex> g(g_global_mu);
  if (g_global_cctx) { g_global_cctx->dev.release(); delete g_global_cctx; g_global_cctx = nullptr; }
  if (g_global_dctx) { g_global_dctx->dev.release(); delete g_global_dctx; g_global_dctx = nullptr; }
  b2h::release_device_workspaces();
  g_initlib = false;
}

int blosc2_free_resources(void) {
  std::lock_guard<std::mutex> g(g_global_mu);
  if (!g_initlib) return BLOSC2_ERROR_FAILURE;
  if (g_global_cctx) g_global_cctx->dev.release();
  if (g_global_dctx) g_global_dctx->dev.release();
  b2h::release_device_workspaces();
  return 0;
}

const char* blosc2_get_version_string(void) { return BLOSC2_VERSION_STRING; }

// blosc/blosc2.c:6916-6995
const char* blosc2_error_string(int error_code) {
  static const char* const msg[] = {
      "Success",   // (never returned: 0 is not an error, see below)
      "Generic failure", "Bad stream", "Invalid data", "Memory alloc/realloc failure", "Not enough space to read",
      "Not enough space to write", "Codec not supported", "Invalid parameter supplied to codec",
      "Codec dictionary error", "Version not supported", "Invalid value in header",
      "Invalid parameter supplied to function", "File read failure", "File write failure", "File open failure",
      "Not found", "Bad run length encoding", "Filter pipeline error", "Chunk insert failure",
      "Chunk append failure", "Chunk update failure", "Sizes larger than 2gb not supported",
      "Super-chunk copy failure", "Wrong type for frame", "File truncate failure",
      "Thread or thread context creation failure", "Postfilter failure", "Special frame failure",
      "Special super-chunk failure", "IO plugin error", "Remove file failure", "Pointer is null", "Invalid index",
      "Metalayer has not been found", "Maximum buffersize exceeded", "Tuner failure", "Frame lock failure"};
  // codes -1 .. -37 index the table; BLOSC2_ERROR_SUCCESS has no case in the reference's switch
  if (error_code < 0 && error_code >= BLOSC2_ERROR_LOCK) return msg[-error_code];
  return "Unknown error";
}

// blosc/timestamp.c (the POSIX branch): CLOCK_MONOTONIC, differences in ns and s
void blosc_set_timestamp(blosc_timestamp_t* timestamp) { clock_gettime(CLOCK_MONOTONIC, timestamp); }

double blosc_elapsed_nsecs(blosc_timestamp_t start_time, blosc_timestamp_t end_time) {
  return 1e9 * (double)(end_time.tv_sec - start_time.tv_sec) + (double)(end_time.tv_nsec - start_time.tv_nsec);
}

double blosc_elapsed_secs(blosc_timestamp_t start_time, blosc_timestamp_t end_time) {
  return 1e-9 * blosc_elapsed_nsecs(start_time, end_time);
}

// blosc/blosc2.c:6040-6251 (validation + environment overrides)
blosc2_context* blosc2_create_cctx(blosc2_cparams cparams) {
  blosc2_context* c = new blosc2_context_s();
  c->do_compress = 1;
  c->use_dict = cparams.use_dict;
  c->instr_codec = cparams.instr_codec;
  for (int i = 0; i < 6; i++) {
    c->filters[i] = cparams.filters[i];
    c->filters_meta[i] = cparams.filters_meta[i];
    const uint8_t f = c->filters[i];
    if ((f >= BLOSC_LAST_FILTER && f <= BLOSC2_DEFINED_FILTERS_STOP) ||
        (f > BLOSC_LAST_REGISTERED_FILTER && f <= BLOSC2_GLOBAL_REGISTERED_FILTERS_STOP)) {
      TRACE_ERROR("filter (%d) is not yet defined", f);
      delete c;
      return nullptr;
    }
  }
  int doshuffle = -1, dodelta = BLOSC_NOFILTER;
  if (const char* v = getenv("BLOSC_SHUFFLE")) {
    if (!strcmp(v, "NOSHUFFLE")) doshuffle = BLOSC_NOSHUFFLE;
    else if (!strcmp(v, "SHUFFLE")) doshuffle = BLOSC_SHUFFLE;
    else if (!strcmp(v, "BITSHUFFLE")) doshuffle = BLOSC_BITSHUFFLE;
  }
  if (const char* v = getenv("BLOSC_DELTA")) {
    if (!strcmp(v, "1")) dodelta = BLOSC_DELTA;
    else if (!strcmp(v, "0")) dodelta = BLOSC_NOFILTER;
  }
  long x;
  c->typesize = cparams.typesize;
  if (env_long("BLOSC_TYPESIZE", &x) && x > 0) c->typesize = (int32_t)x;
  build_filters(doshuffle, dodelta, c->typesize, c->filters);
  c->clevel = cparams.clevel;
  if (env_long("BLOSC_CLEVEL", &x) && x >= 0) c->clevel = (int)x;
  c->compcode = cparams.compcode;
  if (const char* v = getenv("BLOSC_COMPRESSOR")) {
    const int code = compname_to_code(v);
    if (code >= BLOSC_LAST_CODEC) {
      TRACE_ERROR("User defined codecs cannot be set here. Use Blosc2 mechanism instead.");
      delete c;
      return nullptr;
    }
    c->compcode = (uint8_t)code;
  }
  c->compcode_meta = cparams.compcode_meta;
  c->blocksize = cparams.blocksize;
  if (env_long("BLOSC_BLOCKSIZE", &x) && x > 0) c->blocksize = (int32_t)x;
  c->nthreads = cparams.nthreads;
  if (env_long("BLOSC_NTHREADS", &x) && x > 0) c->nthreads = (int16_t)x;
  c->splitmode = cparams.splitmode;
  if (const char* v = getenv("BLOSC_SPLITMODE")) {
    if (!strcmp(v, "ALWAYS")) c->splitmode = BLOSC_ALWAYS_SPLIT;
    else if (!strcmp(v, "NEVER")) c->splitmode = BLOSC_NEVER_SPLIT;
    else if (!strcmp(v, "AUTO")) c->splitmode = BLOSC_AUTO_SPLIT;
    else if (!strcmp(v, "FORWARD_COMPAT")) c->splitmode = BLOSC_FORWARD_COMPAT_SPLIT;
  }
  c->schunk = cparams.schunk;
  if (cparams.prefilter) {   // blosc/blosc2.c:6215-6219: the context keeps a copy of the params
    c->prefilter = cparams.prefilter;
    if (cparams.preparams) memcpy(&c->pre_copy, cparams.preparams, sizeof c->pre_copy);
    c->preparams = &c->pre_copy;
  }
  c->tuner_params = cparams.tuner_params;
  c->tuner_id = cparams.tuner_id;
  c->codec_params = cparams.codec_params;
  c->lz_mode = b2h::codec_params_lz_mode(cparams.codec_params);
  for (int i = 0; i < 6; i++) c->filter_params[i] = cparams.filter_params[i];
  return c;
}

blosc2_context* blosc2_create_dctx(blosc2_dparams dparams) {
  blosc2_context* c = new blosc2_context_s();
  c->do_compress = 0;
  c->dparams = dparams;
  if (dparams.postfilter) {   // blosc/blosc2.c:6279-6283: the context keeps a copy of the params
    if (dparams.postparams) memcpy(&c->post_copy, dparams.postparams, sizeof c->post_copy);
    c->dparams.postparams = &c->post_copy;
  } else {
    c->dparams.postparams = nullptr;
  }
  c->nthreads = dparams.nthreads;
  long x;
  if (env_long("BLOSC_NTHREADS", &x) && x > 0) c->nthreads = (int16_t)x;
  c->schunk = dparams.schunk;
  return c;
}

void blosc2_free_ctx(blosc2_context* context) {
  if (!context) return;
  context->dev.release();
  delete context;
}

int blosc2_ctx_get_cparams(blosc2_context* ctx, blosc2_cparams* cparams) {
  if (!ctx || !cparams) return BLOSC2_ERROR_NULL_POINTER;
  *cparams = BLOSC2_CPARAMS_DEFAULTS;
  cparams->compcode = ctx->compcode;
  cparams->compcode_meta = ctx->compcode_meta;
  cparams->clevel = (uint8_t)ctx->clevel;
  cparams->use_dict = ctx->use_dict;
  cparams->instr_codec = ctx->instr_codec;
  cparams->typesize = ctx->typesize;
  cparams->nthreads = ctx->nthreads;
  cparams->blocksize = ctx->blocksize;
  cparams->splitmode = ctx->splitmode;
  cparams->schunk = ctx->schunk;
  for (int i = 0; i < 6; i++) {
    cparams->filters[i] = ctx->filters[i];
    cparams->filters_meta[i] = ctx->filters_meta[i];
    cparams->filter_params[i] = ctx->filter_params[i];
  }
  cparams->prefilter = ctx->prefilter;
  cparams->preparams = ctx->preparams;
  cparams->tuner_id = ctx->tuner_id;
  cparams->tuner_params = ctx->tuner_params;
  cparams->codec_params = ctx->codec_params;
  return BLOSC2_ERROR_SUCCESS;
}

int blosc2_ctx_get_dparams(blosc2_context* ctx, blosc2_dparams* dparams) {
  if (!ctx || !dparams) return BLOSC2_ERROR_NULL_POINTER;
  *dparams = ctx->dparams;
  dparams->nthreads = ctx->nthreads;
  dparams->schunk = ctx->schunk;
  return BLOSC2_ERROR_SUCCESS;
}

int blosc2_set_maskout(blosc2_context* ctx, bool* maskout, int nblocks) {
  if (!ctx) return BLOSC2_ERROR_NULL_POINTER;
  ctx->maskout.assign(maskout, maskout + nblocks);
  return 0;
}

// blosc/blosc2.c:3121-3148
int blosc2_compress_ctx(blosc2_context* context, const void* src, int32_t srcsize, void* dest, int32_t destsize) {
  if (!context) return BLOSC2_ERROR_NULL_POINTER;
  if (context->do_compress != 1) {
    TRACE_ERROR("Context is not meant for compression.  Giving up.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  std::lock_guard<std::mutex> g(context->mu);
  return compress_host(context, src, srcsize, dest, destsize, context->blocksize, true, true);
}

// blosc/blosc2.c:3943-3962
int blosc2_decompress_ctx(blosc2_context* context, const void* src, int32_t srcsize, void* dest, int32_t destsize) {
  if (!context) return BLOSC2_ERROR_NULL_POINTER;
  if (context->do_compress != 0) {
    TRACE_ERROR("Context is not meant for decompression.  Giving up.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  std::lock_guard<std::mutex> g(context->mu);
  std::vector<uint8_t> mask;
  const bool has_mask = !context->maskout.empty();
  if (has_mask) mask.swap(context->maskout);   // a mask applies to one call (blosc2.c:3954-3959)
  return decompress_host(context, src, srcsize, dest, destsize, has_mask ? &mask : nullptr);
}

// A memcpyed or special chunk's items [off, off + len) as a stand-alone chunk of the same kind
// (header with nbytes = blocksize = len, no dictionary / lazy / VL bits; the raw bytes, or the
// repeated value), decoded by the device's memcpyed / special path.
static void carve_items(const uint8_t* s, const ChunkHdr& H, int64_t off, int32_t len, std::vector<uint8_t>& one) {
  auto put32 = [&](size_t at, int32_t v) { memcpy(one.data() + at, &v, 4); };
  if (H.special) {
    // the special kind decides, whatever the memcpyed bit and cbytes say (blosc_d 1865-1909)
    one.assign(s, s + (H.special == BLOSC2_SPECIAL_VALUE ? H.cbytes : BLOSC_EXTENDED_HEADER_LENGTH));
    one[2] &= (uint8_t)~BLOSC_MEMCPYED;
    put32(12, (int32_t)one.size());
  } else {
    one.assign(s, s + H.overhead);
    one.insert(one.end(), s + H.overhead + off, s + H.overhead + off + len);
    put32(12, (int32_t)one.size());
  }
  put32(4, len);
  put32(8, len);
  if (H.ext) {
    one[BLOSC2_CHUNK_BLOSC2_FLAGS2] = 0;
    one[BLOSC2_CHUNK_BLOSC2_FLAGS] = (uint8_t)(H.special << 4);
  }
}

static int blosc2_decompress_block_unlocked(blosc2_context* context, const void* src, int32_t srcsize, int32_t nblock,
                                            void* dest, int32_t destsize, const ChunkHdr& H, int host_mode);

// blosc2_decompress_block_ctx (blosc/blosc2.c:4580-4687; declared in blosc-private.h:29 and used
// by the sparse reader, schunk.c:1858): block `nblock` of a chunk into dest, returning its size.
// Checks in the reference's order; then the chunk is decoded on the device with every other block
// masked and the block un-deltaed against itself, as blosc_d with dest_offset 0 leaves it
// (delta_decoder's offset == 0 branch, delta.c:96-100).  Memcpyed / special blocks are carved out
// as stand-alone chunks of the same kind (blosc_d's memcpyed path, 1865-1935).
int blosc2_decompress_block_ctx(blosc2_context* context, const void* src, int32_t srcsize, int32_t nblock, void* dest,
                                int32_t destsize) {
  if (!context || !src) return BLOSC2_ERROR_NULL_POINTER;
  ChunkHdr H;
  int rc = read_header(src, srcsize, &H);
  if (rc < 0) return rc;
  if (H.vl) {
    TRACE_ERROR("block decompression is not supported for VL-block chunks.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if ((rc = init_from_header(&H, srcsize)) < 0) return rc;
  if (H.special > BLOSC2_SPECIAL_LASTID) {
    TRACE_ERROR("Unknown special values ID (%d) ", H.special);
    return BLOSC2_ERROR_DATA;
  }
  if (nblock < 0 || nblock >= H.nblocks) {
    TRACE_ERROR("`nblock` out of bounds.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if (!H.special && !H.memcpyed && (int64_t)H.overhead + 4 * (int64_t)H.nblocks > srcsize) {
    TRACE_ERROR("`bstarts` out of bounds.");
    return BLOSC2_ERROR_READ_BUFFER;
  }
  const bool leftover = nblock == H.nblocks - 1 && H.leftover > 0;
  const int32_t bsize = leftover ? H.leftover : H.blocksize;
  if (destsize < bsize) {
    TRACE_ERROR("Destination is too small for block.");
    return BLOSC2_ERROR_WRITE_BUFFER;
  }
  if (H.lazy && !H.special) return BLOSC2_ERROR_INVALID_PARAM;   // lazy chunks need their frame
  std::lock_guard<std::mutex> g(context->mu);
  if (context->dparams.postfilter) {
    // blosc_d(dest, dest_offset 0) with the postfilter: the block's image, then the callback
    // writes dest (blosc/blosc2.c:4678-4682, 1586-1606, 1910-1931)
    std::vector<uint8_t> blk((size_t)bsize);
    rc = blosc2_decompress_block_unlocked(context, src, srcsize, nblock, blk.data(), bsize, H, kHostNoPost);
    if (rc < 0) return rc;
    if ((rc = call_postfilter(context, H, blk.data(), static_cast<uint8_t*>(dest), nblock)) < 0) return rc;
    return bsize;
  }
  return blosc2_decompress_block_unlocked(context, src, srcsize, nblock, dest, destsize, H, 0);
}

static int blosc2_decompress_block_unlocked(blosc2_context* context, const void* src, int32_t srcsize, int32_t nblock,
                                            void* dest, int32_t destsize, const ChunkHdr& H, int host_mode) {
  const uint8_t* s = static_cast<const uint8_t*>(src);
  const bool leftover = nblock == H.nblocks - 1 && H.leftover > 0;
  const int32_t bsize = leftover ? H.leftover : H.blocksize;
  int rc;
  if (H.memcpyed || H.special) {
    if (!H.special) {
      if (H.nbytes + H.overhead != H.cbytes) return BLOSC2_ERROR_WRITE_BUFFER;
      if (H.cbytes < H.overhead + (int64_t)nblock * H.blocksize + bsize) return BLOSC2_ERROR_READ_BUFFER;
    }
    const int32_t its = H.special == BLOSC2_SPECIAL_VALUE ? H.cbytes - H.overhead : H.typesize;
    if ((H.special == BLOSC2_SPECIAL_VALUE || H.special == BLOSC2_SPECIAL_NAN) && bsize % its) return BLOSC2_ERROR_DATA;
    if (H.special == BLOSC2_SPECIAL_NAN && its != 4 && its != 8) return BLOSC2_ERROR_DATA;
    if (H.special == BLOSC2_SPECIAL_UNINIT) return bsize;
    std::vector<uint8_t> one;
    carve_items(s, H, (int64_t)nblock * H.blocksize, bsize, one);
    rc = decompress_host(context, one.data(), (int32_t)one.size(), dest, destsize, nullptr, host_mode);
    return rc < 0 ? rc : bsize;
  }
  std::vector<uint8_t> mask((size_t)H.nblocks, 1);
  mask[nblock] = 0;
  std::vector<uint8_t> full((size_t)H.nbytes);
  rc = decompress_host(context, src, srcsize, full.data(), H.nbytes, &mask,
                       b2h::kDecDeltaSelf | b2h::kDecNoDict | host_mode);
  if (rc < 0) return rc;
  memcpy(dest, full.data() + (int64_t)nblock * H.blocksize, (size_t)bsize);
  return bsize;
}

// blosc/blosc2.c:4265-4474 / 4541-4550: the reference's checks in order, then the blocks
// overlapping [start, start + nitems) decoded on the device (the rest masked), each un-deltaed
// against itself as _blosc_getitem's blosc_d(dest_offset 0) leaves it; memcpyed / special chunks
// through a carved stand-alone chunk (the reference's short-circuit, 4321-4383).
int blosc2_getitem_ctx(blosc2_context* context, const void* src, int32_t srcsize, int start, int nitems, void* dest,
                       int32_t destsize) {
  if (!context) return BLOSC2_ERROR_NULL_POINTER;
  ChunkHdr H;
  int rc = read_header(src, srcsize, &H);
  if (rc < 0) return rc;
  if (H.vl) {
    TRACE_ERROR("getitem is not supported for VL-block chunks.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if ((rc = init_from_header(&H, srcsize)) < 0) return rc;
  if (nitems == 0) return 0;
  if (nitems < 0) return BLOSC2_ERROR_INVALID_PARAM;
  const int64_t ts = H.typesize;
  const int64_t nib = (int64_t)nitems * ts;
  if (nib > INT32_MAX || nib > destsize) return BLOSC2_ERROR_WRITE_BUFFER;
  const int64_t sb = (int64_t)start * ts;
  if (start < 0 || sb > H.nbytes) return BLOSC2_ERROR_INVALID_PARAM;
  const int64_t stop = (int64_t)start + nitems;
  if (stop > INT32_MAX || stop * ts > H.nbytes) return BLOSC2_ERROR_INVALID_PARAM;
  if (!H.special && !H.memcpyed && (int64_t)H.overhead + 4 * (int64_t)H.nblocks > srcsize) {
    TRACE_ERROR("`bstarts` out of bounds.");
    return BLOSC2_ERROR_READ_BUFFER;
  }
  const uint8_t* s = static_cast<const uint8_t*>(src);
  const bool lazy = H.lazy && !H.special;
  std::lock_guard<std::mutex> g(context->mu);
  if (context->dparams.postfilter && !lazy) {
    // With a postfilter there is no memcpyed / special short-circuit (blosc/blosc2.c:4336): every
    // touched block is decoded as blosc_d(dest_offset 0) leaves it, the callback writes the whole
    // block, and the slice is copied out (4399-4461)
    std::vector<uint8_t> mask((size_t)H.nblocks, 1);
    for (int32_t b = 0; b < H.nblocks; b++) {
      const int64_t lo = (int64_t)b * H.blocksize, hi = lo + H.blocksize;
      if (hi > sb && lo < stop * ts) mask[b] = 0;
    }
    std::vector<uint8_t> full((size_t)std::max(H.nbytes, 1)), blk((size_t)H.blocksize);
    rc = decompress_host(context, src, srcsize, full.data(), H.nbytes, &mask,
                         b2h::kDecDeltaSelf | b2h::kDecNoDict | kHostNoPost);
    if (rc < 0) return rc;
    int64_t nt = 0;
    for (int32_t b = 0; b < H.nblocks; b++) {
      if (mask[b]) continue;
      const int64_t lo = (int64_t)b * H.blocksize;
      const int64_t startb = std::max<int64_t>(sb - lo, 0), stopb = std::min<int64_t>(stop * ts - lo, H.blocksize);
      if ((rc = call_postfilter(context, H, full.data() + lo, blk.data(), b)) < 0) return rc;
      memcpy(static_cast<uint8_t*>(dest) + nt, blk.data() + startb, (size_t)(stopb - startb));
      nt += stopb - startb;
    }
    return (int)nib;
  }
  if ((H.memcpyed || H.special) && !lazy) {
    if (H.special > BLOSC2_SPECIAL_LASTID) return BLOSC2_ERROR_SCHUNK_SPECIAL;
    const int32_t its = H.special == BLOSC2_SPECIAL_VALUE ? H.cbytes - H.overhead : H.typesize;
    if ((H.special == BLOSC2_SPECIAL_VALUE || H.special == BLOSC2_SPECIAL_NAN) && nib % its) return BLOSC2_ERROR_DATA;
    if (H.special == BLOSC2_SPECIAL_NAN && its != 4 && its != 8) return BLOSC2_ERROR_DATA;
    if (!H.special && H.overhead + sb + nib > srcsize) return BLOSC2_ERROR_READ_BUFFER;
    if (H.special == BLOSC2_SPECIAL_UNINIT) return (int)nib;
    std::vector<uint8_t> one;
    carve_items(s, H, sb, (int32_t)nib, one);
    rc = decompress_host(context, one.data(), (int32_t)one.size(), dest, destsize, nullptr);
    return rc < 0 ? rc : (int)nib;
  }
  if (lazy) return BLOSC2_ERROR_INVALID_PARAM;   // lazy chunks need their frame (blosc_d 1757-1766)
  std::vector<uint8_t> mask((size_t)H.nblocks, 1);
  for (int32_t b = 0; b < H.nblocks; b++) {
    const int64_t lo = (int64_t)b * H.blocksize, hi = lo + H.blocksize;
    if (hi > sb && lo < stop * ts) mask[b] = 0;
  }
  std::vector<uint8_t> full((size_t)H.nbytes);
  rc = decompress_host(context, src, srcsize, full.data(), H.nbytes, &mask, b2h::kDecDeltaSelf | b2h::kDecNoDict);
  if (rc < 0) return rc;
  memcpy(dest, full.data() + sb, (size_t)nib);
  return (int)nib;
}

// blosc/blosc2.c:4552-4578: byte offsets, checked against the chunk's stored typesize, then getitem.
int blosc2_getitem_bytes_ctx(blosc2_context* context, const void* src, int32_t srcsize, int32_t start, int32_t nbytes,
                             void* dest, int32_t destsize) {
  if (!context) return BLOSC2_ERROR_NULL_POINTER;
  ChunkHdr H;
  int rc = read_header(src, srcsize, &H);
  if (rc < 0) return rc;
  if (start < 0 || nbytes < 0) {
    TRACE_ERROR("`start` and `nbytes` must not be negative.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  const int32_t ts = H.typesize;
  if (start % ts != 0 || nbytes % ts != 0) {
    TRACE_ERROR("`start` (%d) and `nbytes` (%d) must both be multiples of the typesize stored in the chunk (%d).",
                start, nbytes, ts);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  return blosc2_getitem_ctx(context, src, srcsize, start / ts, nbytes / ts, dest, destsize);
}

int blosc2_getitem(const void* src, int32_t srcsize, int start, int nitems, void* dest, int32_t destsize) {
  blosc2_context* c = blosc2_create_dctx(BLOSC2_DPARAMS_DEFAULTS);
  const int r = blosc2_getitem_ctx(c, src, srcsize, start, nitems, dest, destsize);
  blosc2_free_ctx(c);
  return r;
}

int blosc1_getitem(const void* src, int start, int nitems, void* dest) {
  return blosc2_getitem(src, INT32_MAX, start, nitems, dest, INT32_MAX);
}

// blosc/blosc2.c:3701-3897 (environment overrides, global context)
int blosc2_compress(int clevel, int doshuffle, int32_t typesize, const void* src, int32_t srcsize, void* dest,
                    int32_t destsize) {
  if (!g_initlib) blosc2_init();
  long x;
  if (env_long("BLOSC_CLEVEL", &x) && x >= 0) clevel = (int)x;
  if (const char* v = getenv("BLOSC_SHUFFLE")) {
    if (!strcmp(v, "NOSHUFFLE")) doshuffle = BLOSC_NOSHUFFLE;
    else if (!strcmp(v, "SHUFFLE")) doshuffle = BLOSC_SHUFFLE;
    else if (!strcmp(v, "BITSHUFFLE")) doshuffle = BLOSC_BITSHUFFLE;
  }
  if (const char* v = getenv("BLOSC_DELTA")) {
    if (!strcmp(v, "1")) blosc2_set_delta(1);
    else if (!strcmp(v, "0")) blosc2_set_delta(0);
  }
  if (env_long("BLOSC_TYPESIZE", &x) && x > 0) typesize = (int32_t)x;
  if (const char* v = getenv("BLOSC_COMPRESSOR")) (void)blosc1_set_compressor(v);
  if (env_long("BLOSC_BLOCKSIZE", &x) && x > 0) blosc1_set_blocksize((size_t)x);
  if (env_long("BLOSC_NTHREADS", &x) && x > 0) (void)blosc2_set_nthreads((int16_t)x);
  if (const char* v = getenv("BLOSC_SPLITMODE")) {
    int sm = -1;
    if (!strcmp(v, "ALWAYS")) sm = BLOSC_ALWAYS_SPLIT;
    else if (!strcmp(v, "NEVER")) sm = BLOSC_NEVER_SPLIT;
    else if (!strcmp(v, "AUTO")) sm = BLOSC_AUTO_SPLIT;
    else if (!strcmp(v, "FORWARD_COMPAT")) sm = BLOSC_FORWARD_COMPAT_SPLIT;
    if (sm >= 0) blosc1_set_splitmode(sm);
  }
  std::lock_guard<std::mutex> g(g_global_mu);
  if (!g_global_cctx) {
    g_global_cctx = new blosc2_context_s();
    g_global_cctx->do_compress = 1;
  }
  blosc2_context* c = g_global_cctx;
  memset(c->filters, 0, 6);
  memset(c->filters_meta, 0, 6);
  build_filters(doshuffle, g_delta, typesize, c->filters);
  c->clevel = clevel;
  c->typesize = typesize;
  c->compcode = (uint8_t)g_compressor;
  c->splitmode = g_splitmode;
  c->nthreads = g_nthreads;
  const bool blosc1_compat = getenv("BLOSC_BLOSC1_COMPAT") != nullptr && getenv("BLOSC_NOLOCK") == nullptr;
  // the global path passes g_force_blocksize every call (no sticky blocksize)
  return compress_host(c, src, srcsize, dest, destsize, g_force_blocksize, false, !blosc1_compat);
}

int blosc2_decompress(const void* src, int32_t srcsize, void* dest, int32_t destsize) {
  if (!g_initlib) blosc2_init();
  std::lock_guard<std::mutex> g(g_global_mu);
  if (!g_global_dctx) g_global_dctx = new blosc2_context_s();
  return decompress_host(g_global_dctx, src, srcsize, dest, destsize, nullptr);
}

int blosc1_compress(int clevel, int doshuffle, size_t typesize, size_t nbytes, const void* src, void* dest,
                    size_t destsize) {
  return blosc2_compress(clevel, doshuffle, (int32_t)typesize, src, (int32_t)nbytes, dest, (int32_t)destsize);
}

int blosc1_decompress(const void* src, void* dest, size_t destsize) {
  return blosc2_decompress(src, INT32_MAX, dest, (int32_t)destsize);
}

int16_t blosc2_get_nthreads(void) { return g_nthreads; }

// blosc/blosc2.c:181-185: not thread-safe by contract, affects every context
void blosc2_set_threads_callback(blosc_threads_callback callback, void* callback_data) {
  g_threads_cb = callback;
  g_threads_cb_data = callback_data;
}
int16_t blosc2_set_nthreads(int16_t nthreads) {
  const int16_t old = g_nthreads;
  if (nthreads <= 0) return BLOSC2_ERROR_INVALID_PARAM;
  g_nthreads = nthreads;   // only recorded: the device path has no host worker pool
  return old;
}

const char* blosc1_get_compressor(void) {
  const char* name = nullptr;
  blosc2_compcode_to_compname(g_compressor, &name);
  return name;
}

int blosc1_set_compressor(const char* compname) {
  const int code = compname_to_code(compname);
  if (code >= BLOSC_LAST_CODEC) {
    TRACE_ERROR("User defined codecs cannot be set here. Use Blosc2 mechanism instead.");
    return BLOSC2_ERROR_CODEC_SUPPORT;
  }
  if (code >= 0) g_compressor = code;
  if (!g_initlib) blosc2_init();
  return code;
}

void blosc2_set_delta(int dodelta) { g_delta = dodelta; }
int blosc1_get_blocksize(void) { return g_force_blocksize; }
void blosc1_set_blocksize(size_t blocksize) { g_force_blocksize = (int32_t)blocksize; }
void blosc1_set_splitmode(int splitmode) { g_splitmode = splitmode; }

int blosc2_compcode_to_compname(int compcode, const char** compname) {
  const char* name = nullptr;
  switch (compcode) {
    case BLOSC_BLOSCLZ: name = BLOSC_BLOSCLZ_COMPNAME; break;
    case BLOSC_LZ4: name = BLOSC_LZ4_COMPNAME; break;
    case BLOSC_LZ4HC: name = BLOSC_LZ4HC_COMPNAME; break;
    case BLOSC_ZLIB: name = BLOSC_ZLIB_COMPNAME; break;
    case BLOSC_ZSTD: name = BLOSC_ZSTD_COMPNAME; break;
    default: {
      std::lock_guard<std::mutex> g(g_reg_mu);
      for (auto& c : g_codecs)
        if (c.compcode == compcode) name = c.compname;
    }
  }
  *compname = name;
  if (compcode == BLOSC_BLOSCLZ || compcode == BLOSC_LZ4) return compcode;
  // other built-in codecs exist in the format but are not implemented by this engine
  return name ? (compcode < BLOSC_LAST_CODEC ? -1 : compcode) : -1;
}

int blosc2_compname_to_compcode(const char* compname) { return compname_to_code(compname); }

const char* blosc2_list_compressors(void) { return BLOSC_BLOSCLZ_COMPNAME "," BLOSC_LZ4_COMPNAME; }

int blosc2_get_complib_info(const char* compname, char** complib, char** version) {
  const int code = compname_to_code(compname);
  if (code == BLOSC_LZ4) {   // the LZ4 block format as produced by lz4 1.9.3 (the image's liblz4)
    if (complib) *complib = strdup(BLOSC_LZ4_LIBNAME);
    if (version) *version = strdup("1.9.3");
    return BLOSC_LZ4_LIB;
  }
  if (code != BLOSC_BLOSCLZ) {
    if (complib) *complib = nullptr;
    if (version) *version = nullptr;
    return -1;
  }
  if (complib) *complib = strdup(BLOSC_BLOSCLZ_LIBNAME);
  if (version) *version = strdup("2.5.3");
  return BLOSC_BLOSCLZ_LIB;
}

// blosc/blosc2.c:4702-4760 (cbuffer inspection)
int blosc2_cbuffer_sizes(const void* cbuffer, int32_t* nbytes, int32_t* cbytes, int32_t* blocksize) {
  const uint8_t* s = static_cast<const uint8_t*>(cbuffer);
  int32_t nb = rd32(s + 4), bs = rd32(s + 8), cb = rd32(s + 12);
  if (cb < BLOSC_MIN_HEADER_LENGTH || bs <= 0 || bs > BLOSC2_MAXBLOCKSIZE || s[3] == 0) {
    if (nbytes) *nbytes = 0;
    if (cbytes) *cbytes = 0;
    if (blocksize) *blocksize = 0;
    return BLOSC2_ERROR_INVALID_HEADER;
  }
  if (nb > 0 && bs > nb) bs = nb;
  if (nbytes) *nbytes = nb;
  if (cbytes) *cbytes = cb;
  if (blocksize) *blocksize = bs;
  return 0;
}

void blosc1_cbuffer_sizes(const void* cbuffer, size_t* nbytes, size_t* cbytes, size_t* blocksize) {
  int32_t nb = 0, cb = 0, bs = 0;
  blosc2_cbuffer_sizes(cbuffer, &nb, &cb, &bs);
  if (nbytes) *nbytes = (size_t)nb;
  if (cbytes) *cbytes = (size_t)cb;
  if (blocksize) *blocksize = (size_t)bs;
}

int blosc1_cbuffer_validate(const void* cbuffer, size_t cbytes, size_t* nbytes) {
  int32_t header_cbytes, nb, bs;
  if (cbytes < BLOSC_MIN_HEADER_LENGTH) { *nbytes = 0; return BLOSC2_ERROR_WRITE_BUFFER; }
  int rc = blosc2_cbuffer_sizes(cbuffer, &nb, &header_cbytes, &bs);
  if (rc < 0) { *nbytes = 0; return rc; }
  *nbytes = (size_t)nb;
  if ((size_t)header_cbytes != cbytes) return BLOSC2_ERROR_INVALID_HEADER;
  if (nb > BLOSC2_MAX_BUFFERSIZE) return BLOSC2_ERROR_MEMORY_ALLOC;
  return 0;
}

void blosc1_cbuffer_metainfo(const void* cbuffer, size_t* typesize, int* flags) {
  const uint8_t* s = static_cast<const uint8_t*>(cbuffer);
  if (typesize) *typesize = s[3];
  if (flags) *flags = s[2];
}

void blosc2_cbuffer_versions(const void* cbuffer, int* version, int* versionlz) {
  const uint8_t* s = static_cast<const uint8_t*>(cbuffer);
  if (version) *version = s[0];
  if (versionlz) *versionlz = s[1];
}

const char* blosc2_cbuffer_complib(const void* cbuffer) {
  const uint8_t* s = static_cast<const uint8_t*>(cbuffer);
  switch (s[2] >> 5) {
    case BLOSC_BLOSCLZ_FORMAT: return BLOSC_BLOSCLZ_LIBNAME;
    case BLOSC_LZ4_FORMAT: return BLOSC_LZ4_LIBNAME;
    case BLOSC_ZLIB_FORMAT: return BLOSC_ZLIB_LIBNAME;
    case BLOSC_ZSTD_FORMAT: return BLOSC_ZSTD_LIBNAME;
    case BLOSC_UDCODEC_FORMAT: return "User-defined";
    default: return "Unknown";
  }
}

// blosc/blosc2.c:6692-6737 (register_codec_private + blosc2_register_codec)
int blosc2_register_codec(blosc2_codec* codec) {
  if (!codec) return BLOSC2_ERROR_NULL_POINTER;
  if (codec->compcode < BLOSC2_USER_REGISTERED_CODECS_START) {
    TRACE_ERROR("The id must be greater or equal to %d", BLOSC2_USER_REGISTERED_CODECS_START);
    return BLOSC2_ERROR_FAILURE;
  }
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (g_codecs.size() >= 256) return BLOSC2_ERROR_CODEC_SUPPORT;
  for (auto& c : g_codecs)
    if (c.compcode == codec->compcode) {
      if (c.compname && codec->compname && !strcmp(c.compname, codec->compname)) return 0;
      TRACE_ERROR("The codec is already registered!");
      return BLOSC2_ERROR_CODEC_PARAM;
    }
  g_codecs.push_back(*codec);
  return 0;
}

// blosc/blosc2.c:6642-6687 (register_filter_private + blosc2_register_filter)
int blosc2_register_filter(blosc2_filter* filter) {
  if (!filter) return BLOSC2_ERROR_NULL_POINTER;
  if (filter->id < BLOSC2_USER_REGISTERED_FILTERS_START) {
    TRACE_ERROR("The id must be greater or equal to %d", BLOSC2_USER_REGISTERED_FILTERS_START);
    return BLOSC2_ERROR_FAILURE;
  }
  std::lock_guard<std::mutex> g(g_reg_mu);
  if (g_filters.size() >= 256) return BLOSC2_ERROR_CODEC_SUPPORT;
  for (auto& f : g_filters)
    if (f.id == filter->id) {
      if (f.name && filter->name && !strcmp(f.name, filter->name)) return 0;
      TRACE_ERROR("The filter is already registered!");
      return BLOSC2_ERROR_FAILURE;
    }
  g_filters.push_back(*filter);
  return 0;
}

// ------------------------------------------------------------------ special chunks ----
// blosc2_chunk_zeros / _nans / _uninit / _repeatval (blosc/blosc2.c:6452-6637): a 32-byte header
// (plus the value) whose blosc2_flags carry the special kind; the blocksize is the one
// initialize_context_compression computes for these cparams.  Host-only: no data moves.
static int special_chunk(const blosc2_cparams& cp, int32_t nbytes, void* dest, int32_t destsize, int kind,
                         const void* value) {
  const int32_t need = BLOSC_EXTENDED_HEADER_LENGTH + (kind == BLOSC2_SPECIAL_VALUE ? cp.typesize : 0);
  if (destsize < need) {
    TRACE_ERROR("dest buffer is not long enough");
    return BLOSC2_ERROR_DATA;
  }
  if (cp.typesize <= 0) return BLOSC2_ERROR_INVALID_PARAM;
  if ((kind != BLOSC2_SPECIAL_ZERO || nbytes > 0) && nbytes % cp.typesize) {
    TRACE_ERROR("nbytes must be a multiple of typesize");
    return BLOSC2_ERROR_DATA;
  }
  b2h::CompressPlan plan;
  int32_t bs = 0;
  const int rc = b2h::make_compress_plan(&plan, nbytes, destsize, cp.clevel, cp.typesize, cp.blocksize, cp.splitmode,
                                         cp.filters, cp.filters_meta, &bs, true, cp.compcode, cp.compcode_meta);
  if (rc < 0) return rc;
  uint8_t h[BLOSC_EXTENDED_HEADER_LENGTH];
  memset(h, 0, sizeof h);
  h[0] = BLOSC2_VERSION_FORMAT_STABLE;
  h[1] = BLOSC_BLOSCLZ_VERSION_FORMAT;
  h[2] = BLOSC_DOSHUFFLE | BLOSC_DOBITSHUFFLE;   // extended header
  h[3] = (uint8_t)(cp.typesize > 255 ? 1 : cp.typesize);
  const int32_t cb = need;
  memcpy(h + 4, &nbytes, 4);
  memcpy(h + 8, &bs, 4);
  memcpy(h + 12, &cb, 4);
  h[31] = (uint8_t)(kind << 4);
  memcpy(dest, h, sizeof h);
  if (kind == BLOSC2_SPECIAL_VALUE) memcpy(static_cast<uint8_t*>(dest) + sizeof h, value, (size_t)cp.typesize);
  return cb;
}

int blosc2_chunk_zeros(blosc2_cparams cparams, const int32_t nbytes, void* dest, int32_t destsize) {
  return special_chunk(cparams, nbytes, dest, destsize, BLOSC2_SPECIAL_ZERO, nullptr);
}
int blosc2_chunk_uninit(blosc2_cparams cparams, const int32_t nbytes, void* dest, int32_t destsize) {
  return special_chunk(cparams, nbytes, dest, destsize, BLOSC2_SPECIAL_UNINIT, nullptr);
}
int blosc2_chunk_nans(blosc2_cparams cparams, const int32_t nbytes, void* dest, int32_t destsize) {
  return special_chunk(cparams, nbytes, dest, destsize, BLOSC2_SPECIAL_NAN, nullptr);
}
int blosc2_chunk_repeatval(blosc2_cparams cparams, const int32_t nbytes, void* dest, int32_t destsize,
                           const void* repeatval) {
  if (!repeatval) return BLOSC2_ERROR_NULL_POINTER;
  return special_chunk(cparams, nbytes, dest, destsize, BLOSC2_SPECIAL_VALUE, repeatval);
}

// ------------------------------------------------------------------- raw filter API ----
static int32_t raw_filter(int kind, int32_t typesize, int32_t blocksize, const void* src, void* dest) {
  if (typesize < 1 || typesize > 256 || blocksize < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (blocksize == 0) return 0;
  static blosc2_context* ctx = nullptr;
  static std::mutex m;
  std::lock_guard<std::mutex> g(m);
  if (!ctx) ctx = new blosc2_context_s();
  Device& d = ctx->dev;
  if (!d.init()) return BLOSC2_ERROR_FAILURE;
  if (!d.in.ensure((size_t)blocksize) || !d.out.ensure((size_t)blocksize)) return BLOSC2_ERROR_MEMORY_ALLOC;
  if (hipMemcpyAsync(d.in.p, src, (size_t)blocksize, hipMemcpyHostToDevice, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  int rc;
  switch (kind) {
    case 0: rc = b2h::shuffle_dev(typesize, blocksize, d.in.u8(), d.out.u8(), false, d.stream); break;
    case 1: rc = b2h::shuffle_dev(typesize, blocksize, d.in.u8(), d.out.u8(), true, d.stream); break;
    case 2: rc = b2h::bitshuffle_dev(typesize, blocksize, d.in.u8(), d.out.u8(), false, 0, d.stream); break;
    default: rc = b2h::bitshuffle_dev(typesize, blocksize, d.in.u8(), d.out.u8(), true, BLOSC2_VERSION_FORMAT, d.stream); break;
  }
  if (rc < 0) return rc;
  if (hipMemcpyAsync(dest, d.out.p, (size_t)blocksize, hipMemcpyDeviceToHost, d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  if (hipStreamSynchronize(d.stream) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  return blocksize;
}

int32_t blosc2_shuffle(int32_t typesize, int32_t blocksize, const void* src, void* dest) {
  return raw_filter(0, typesize, blocksize, src, dest);
}
int32_t blosc2_unshuffle(int32_t typesize, int32_t blocksize, const void* src, void* dest) {
  return raw_filter(1, typesize, blocksize, src, dest);
}
int32_t blosc2_bitshuffle(int32_t typesize, int32_t blocksize, const void* src, void* dest) {
  return raw_filter(2, typesize, blocksize, src, dest);
}
int32_t blosc2_bitunshuffle(int32_t typesize, int32_t blocksize, const void* src, void* dest) {
  return raw_filter(3, typesize, blocksize, src, dest);
}

// ------------------------------------------------------------------ b2h batch C-ABI ----
int b2h_compress_batch(const blosc2_cparams* cp, const void* d_src, int32_t chunk_nbytes, int32_t nchunks,
                       int64_t src_stride, void* d_dst, int64_t dst_stride, int32_t dst_capacity, int32_t* d_cbytes,
                       void* stream) {
  if (!cp) return BLOSC2_ERROR_NULL_POINTER;
  blosc2_context tmp;
  tmp.compcode = cp->compcode;
  tmp.use_dict = cp->use_dict;
  tmp.filters[5] = 0;
  for (int i = 0; i < 6; i++) { tmp.filters[i] = cp->filters[i]; tmp.filters_meta[i] = cp->filters_meta[i]; }
  tmp.prefilter = cp->prefilter;
  tmp.instr_codec = cp->instr_codec;
  tmp.tuner_params = cp->tuner_params;
  tmp.tuner_id = cp->tuner_id;
  int rc = check_supported(&tmp);
  if (rc < 0) return rc;
  if (needs_host_callbacks(cp->filters, cp->compcode)) {
    TRACE_ERROR("user filters / codecs run per chunk through blosc2_compress_ctx, not the device batch API");
    return BLOSC2_ERROR_FILTER_PIPELINE;
  }
  b2h::CompressPlan plan;
  int32_t computed = 0;
  rc = b2h::make_compress_plan(&plan, chunk_nbytes, dst_capacity, cp->clevel, cp->typesize, cp->blocksize,
                               cp->splitmode, cp->filters, cp->filters_meta, &computed, true, cp->compcode, cp->compcode_meta,
                               1, cp->use_dict);
  if (rc < 0) return rc;
  plan.lz_mode = b2h::codec_params_lz_mode(cp->codec_params);
  return b2h::compress_batch(plan, static_cast<const uint8_t*>(d_src), src_stride, nchunks,
                             static_cast<uint8_t*>(d_dst), dst_stride, d_cbytes, static_cast<hipStream_t>(stream));
}

// Chunks of per-chunk sizes (a super-chunk's ragged last chunk: blosc2_schunk_append_buffer,
// blosc/schunk.c:1459-1477, compresses every chunk into nbytes + BLOSC2_MAX_OVERHEAD).  Runs of
// equal sizes share one plan and one engine batch; all batches are queued on `stream` back to
// back with no host wait.  dst_capacity <= 0: each chunk's own nbytes + BLOSC2_MAX_OVERHEAD.
int b2h_compress_batch_sizes(const blosc2_cparams* cp, const void* d_src, const int32_t* nbytes, int32_t nchunks,
                             int64_t src_stride, void* d_dst, int64_t dst_stride, int32_t dst_capacity,
                             int32_t* d_cbytes, void* stream) {
  if (!cp || (nchunks > 0 && !nbytes)) return BLOSC2_ERROR_NULL_POINTER;
  if (nchunks < 0) return BLOSC2_ERROR_INVALID_PARAM;
  for (int32_t i = 0; i < nchunks; i++) {
    if (nbytes[i] < 0 || (int64_t)nbytes[i] > src_stride) return BLOSC2_ERROR_INVALID_PARAM;
    const int64_t cap = dst_capacity > 0 ? dst_capacity : (int64_t)nbytes[i] + BLOSC2_MAX_OVERHEAD;
    if (cap > dst_stride && nchunks > 1) return BLOSC2_ERROR_INVALID_PARAM;   // outputs would overlap
  }
  const uint8_t* src = static_cast<const uint8_t*>(d_src);
  uint8_t* dst = static_cast<uint8_t*>(d_dst);
  for (int32_t i = 0; i < nchunks;) {
    int32_t j = i + 1;
    while (j < nchunks && nbytes[j] == nbytes[i]) j++;
    const int32_t cap = dst_capacity > 0 ? dst_capacity : nbytes[i] + BLOSC2_MAX_OVERHEAD;
    const int rc = b2h_compress_batch(cp, src + (int64_t)i * src_stride, nbytes[i], j - i, src_stride,
                                      dst + (int64_t)i * dst_stride, dst_stride, cap, d_cbytes + i, stream);
    if (rc < 0) return rc;
    i = j;
  }
  return 0;
}

int b2h_decompress_batch(const void* d_src, int64_t src_stride, const int32_t* d_cbytes, int32_t nchunks, void* d_dst,
                         int64_t dst_stride, int32_t dst_capacity, int32_t* d_status, void* stream) {
  return b2h::decompress_batch_strided(static_cast<const uint8_t*>(d_src), src_stride, d_cbytes, nchunks,
                                       static_cast<uint8_t*>(d_dst), dst_stride, dst_capacity, d_status,
                                       static_cast<hipStream_t>(stream));
}

int b2h_decompress_ptrs(const void* const* d_srcs, const int32_t* d_srcsizes, void* const* d_dsts,
                        const int32_t* d_dstsizes, int32_t n, int64_t dst_bound, int32_t* d_status, void* stream) {
  return b2h::decompress_batch(reinterpret_cast<const uint8_t* const*>(d_srcs), d_srcsizes,
                               reinterpret_cast<uint8_t* const*>(d_dsts), d_dstsizes, n, dst_bound, d_status, nullptr,
                               static_cast<hipStream_t>(stream));
}

int b2h_pack_chunks(const void* d_src, int64_t src_stride, const int32_t* d_sizes, int32_t n, void* d_dst,
                    int64_t* d_offsets, void* stream) {
  if (n < 0 || !d_offsets || (n > 0 && (!d_src || !d_sizes || !d_dst))) return BLOSC2_ERROR_INVALID_PARAM;
  return b2h::pack_chunks(static_cast<const uint8_t*>(d_src), src_stride, d_sizes, n, static_cast<uint8_t*>(d_dst),
                          d_offsets, static_cast<hipStream_t>(stream));
}

int b2h_unpack_chunks(const void* d_src, const int64_t* d_offsets, int32_t n, void* d_dst, int64_t dst_stride,
                      int32_t* d_sizes, void* stream) {
  if (n < 0 || (n > 0 && (!d_src || !d_offsets || !d_dst))) return BLOSC2_ERROR_INVALID_PARAM;
  return b2h::unpack_chunks(static_cast<const uint8_t*>(d_src), d_offsets, n, static_cast<uint8_t*>(d_dst), dst_stride,
                            d_sizes, static_cast<hipStream_t>(stream));
}

int b2h_device_copy(void* d_dst, const void* d_src, int64_t nbytes, void* stream) {
  if (nbytes < 0 || (nbytes > 0 && (!d_dst || !d_src))) return BLOSC2_ERROR_INVALID_PARAM;
  return b2h::device_copy(static_cast<uint8_t*>(d_dst), static_cast<const uint8_t*>(d_src), nbytes,
                          static_cast<hipStream_t>(stream));
}

int32_t b2h_shuffle(int32_t typesize, int32_t nbytes, const void* d_src, void* d_dst, int inverse, void* stream) {
  return b2h::shuffle_dev(typesize, nbytes, static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst),
                          inverse != 0, static_cast<hipStream_t>(stream));
}

int32_t b2h_bitshuffle(int32_t typesize, int32_t nbytes, const void* d_src, void* d_dst, int inverse, void* stream) {
  return b2h::bitshuffle_dev(typesize, nbytes, static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst),
                             inverse != 0, BLOSC2_VERSION_FORMAT, static_cast<hipStream_t>(stream));
}

int b2h_set_blosclz_mode(int mode) { return b2h::set_blosclz_mode(mode); }
int b2h_set_encode_shape(int nlds, int nglb) { return b2h::set_encode_shape(nlds, nglb); }
void b2h_enable_timing(int on) { b2h::enable_timing(on != 0); }
void b2h_last_times(float out[5]) {
  const b2h::KernelTimes t = b2h::last_times();
  out[0] = t.filter_ms; out[1] = t.encode_ms; out[2] = t.finalize_ms; out[3] = t.decode_ms; out[4] = t.unfilter_ms;
}
void b2h_mean_times(float out[5]) {
  const b2h::KernelTimes t = b2h::mean_times();
  out[0] = t.filter_ms; out[1] = t.encode_ms; out[2] = t.finalize_ms; out[3] = t.decode_ms; out[4] = t.unfilter_ms;
}
const char* b2h_last_error(void) { return b2h::last_error(); }
int b2h_debug_stream_results(void* host, int32_t n) { return b2h::debug_stream_results(host, n); }
int b2h_debug_seg_prof(uint64_t* host) { return b2h::debug_seg_prof(host); }
int b2h_debug_decode_cycles(void* host, int32_t n) { return b2h::debug_decode_cycles(host, n); }
int b2h_debug_fuse_timed_out(void) { return b2h::debug_fuse_timed_out(); }
int b2h_device_count(void) { return b2h::device_count(); }

}  // extern "C"
