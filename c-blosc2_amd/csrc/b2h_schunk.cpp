// b2h_schunk.cpp -- in-memory super-chunks (include/blosc2.h blosc2_schunk) over the MI355X engine.
//
// The super-chunk is the container the reference's callers reach the chunk engine through
// (blosc/schunk.c): a list of compressed chunks plus counters, one compression and one
// decompression context.  This file is host bookkeeping only -- every chunk is compressed and
// decompressed by the device engine through the contexts (blosc2_api.cpp).  It keeps the
// reference's frame-less (sparse, in-memory) super-chunk: chunks are malloc'd buffers indexed by
// schunk->data, and the counters (nbytes, cbytes, chunksize, flags2, current_nchunk) move exactly
// as blosc/schunk.c moves them, quirks included (a 32-byte chunk is counted when appended but not
// when replaced or deleted, schunk.c:1300-1302), so a caller sees the same numbers.  Frame-backed
// storage (contiguous frames, files, directories) is outside the device engine: blosc2_schunk_new
// returns NULL for it (the read side of contiguous frames is b2h_frame_* in b2h.h).
//
// The b2h_schunk_* entry points (include/b2h.h) are the batch forms: many appends / decompressions
// of one super-chunk as one device batch, chunk-for-chunk identical to the serial calls.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/b2h.h"
#include "../../include/blosc2.h"
#include "b2h_engine.h"
#include "b2h_frame.h"

namespace {

bool trace_on() {
  static int on = -1;
  if (on < 0) on = getenv("BLOSC_TRACE") != nullptr;
  return on;
}
#define TRACE_ERROR(...)                                 \
  do {                                                   \
    if (trace_on()) {                                    \
      fprintf(stderr, "[error] - ");                     \
      fprintf(stderr, __VA_ARGS__);                      \
      fprintf(stderr, " (%s:%d)\n", __FILE__, __LINE__); \
    }                                                    \
  } while (0)

// Sizes and the flags2 byte of a chunk.  flags2 exists only in an extended header, which the flags
// byte announces (both shuffle bits set); the size bound keeps a short chunk from being over-read
// (get_chunk_flags2, schunk.c:942-949).
struct ChunkInfo {
  int32_t nbytes = 0, cbytes = 0;
  uint8_t flags2 = 0;
  bool vl() const { return (flags2 & BLOSC2_VL_BLOCKS) != 0; }
};

int chunk_info(const uint8_t* c, ChunkInfo* ci) {
  const int rc = blosc2_cbuffer_sizes(c, &ci->nbytes, &ci->cbytes, nullptr);
  if (rc < 0) return rc;
  const uint8_t fl = c[BLOSC2_CHUNK_FLAGS];
  const bool ext = (fl & BLOSC_DOSHUFFLE) && (fl & BLOSC_DOBITSHUFFLE);
  ci->flags2 = (ext && ci->cbytes >= BLOSC_EXTENDED_HEADER_LENGTH) ? c[BLOSC2_CHUNK_BLOSC2_FLAGS2] : 0;
  return 0;
}

// A replaced / deleted chunk's sizes; a header-only chunk (32 bytes) counts 0 compressed bytes
// (schunk.c:1295-1303, 1392-1400).
void old_sizes(const uint8_t* c, int32_t* nb, int32_t* cb) {
  *nb = *cb = 0;
  if (!c) return;
  if (blosc2_cbuffer_sizes(c, nb, cb, nullptr) < 0) *nb = *cb = 0;
  if (*cb == BLOSC2_MAX_OVERHEAD) *cb = 0;
}

int validate_nchunk(const blosc2_schunk* s, int64_t nchunk, bool allow_end, const char* fn) {   // schunk.c:44-66
  if (nchunk < 0) {
    TRACE_ERROR("nchunk ('%lld') is negative in %s.", (long long)nchunk, fn);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if (allow_end ? nchunk > s->nchunks : nchunk >= s->nchunks) {
    TRACE_ERROR("nchunk ('%lld') is out of range (%lld chunks) in %s.", (long long)nchunk, (long long)s->nchunks, fn);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  return 0;
}

enum Op { kAppend, kInsert, kUpdate };

// A super-chunk holds regular chunks or VL-block chunks, never both: the new chunk is checked
// against chunk `ref` (< 0: none left to compare with, the super-chunk adopts its flags2).
// schunk.c:985-1000 (append), 1114-1129 (insert), 1248-1264 (update).
int check_kind(blosc2_schunk* s, int64_t ref, const ChunkInfo& ci, int err) {
  if (ref < 0) {
    s->flags2 = ci.flags2;
    return 0;
  }
  ChunkInfo r;
  const int rc = chunk_info(s->data[ref], &r);
  if (rc < 0) return rc;
  if (r.vl() != ci.vl()) {
    TRACE_ERROR("schunks cannot mix regular chunks and VL-block chunks.");
    return err;
  }
  return 0;
}

// The fixed-chunksize bookkeeping: -1 until the first chunk, then that chunk's nbytes while every
// chunk but the last has it; 0 (variable) from the first chunk that breaks the pattern.
// schunk.c:1002-1023 (append), 1131-1154 (insert), 1266-1282 (update).
int settle_chunksize(blosc2_schunk* s, Op op, int64_t nchunk, int32_t nb, int err) {
  const bool variable = s->chunksize == 0;
  if (s->chunksize == -1) s->chunksize = nb;
  const int32_t cs = s->chunksize;
  if (variable) return 0;
  bool breaks = false;
  if (op == kUpdate) {
    breaks = nb > cs || (nchunk != s->nchunks - 1 && nb != cs);
  } else if (s->nchunks > 0) {
    int32_t last_nb = 0;
    const int rc = blosc2_cbuffer_sizes(s->data[s->nchunks - 1], &last_nb, nullptr, nullptr);
    if (rc < 0) return rc;
    breaks = last_nb < cs || nb > cs || (op == kInsert && nchunk != s->nchunks && nb != cs);
  }
  if (breaks) {
    s->chunksize = 0;
    return 0;
  }
  if (cs > 0 && nb > cs) {
    TRACE_ERROR("Chunks of different lengths in the same schunk are not supported yet: %d > %d.", nb, cs);
    return err;
  }
  return 0;
}

// The chunk the super-chunk keeps: a copy, or the caller's buffer shrunk to its cbytes
// (schunk.c:1045-1058).
uint8_t* keep_chunk(uint8_t* chunk, const ChunkInfo& ci, bool copy) {
  if (copy) {
    uint8_t* c = static_cast<uint8_t*>(malloc((size_t)ci.cbytes));
    if (c) memcpy(c, chunk, (size_t)ci.cbytes);
    return c;
  }
  if (ci.cbytes < ci.nbytes) {
    uint8_t* c = static_cast<uint8_t*>(realloc(chunk, (size_t)ci.cbytes));
    return c ? c : chunk;
  }
  return chunk;
}

// Room for one more slot: the index grows one 4 KiB page at a time (schunk.c:1060-1065).
bool grow_index(blosc2_schunk* s) {
  if ((size_t)(s->nchunks + 1) * sizeof(void*) <= s->data_len) return true;
  uint8_t** d = static_cast<uint8_t**>(realloc(s->data, s->data_len + 4096));
  if (!d) return false;
  s->data = d;
  s->data_len += 4096;
  return true;
}

// blosc2_schunk_insert_chunk / append_chunk on a frame-less super-chunk (schunk.c:976-1075,
// 1100-1212): nchunk == nchunks appends.
int64_t put_chunk(blosc2_schunk* s, Op op, int64_t nchunk, uint8_t* chunk, bool copy) {
  const int err = op == kAppend ? BLOSC2_ERROR_CHUNK_APPEND : BLOSC2_ERROR_CHUNK_INSERT;
  if (!s || !chunk) return BLOSC2_ERROR_NULL_POINTER;
  ChunkInfo ci;
  int rc = chunk_info(chunk, &ci);
  if (rc < 0) return rc;
  if ((rc = check_kind(s, s->nchunks > 0 ? 0 : -1, ci, err)) < 0) return rc;
  if ((rc = settle_chunksize(s, op, nchunk, ci.nbytes, err)) < 0) return rc;
  if (!grow_index(s)) return BLOSC2_ERROR_MEMORY_ALLOC;
  uint8_t* kept = keep_chunk(chunk, ci, copy);
  if (!kept) return BLOSC2_ERROR_MEMORY_ALLOC;
  const int64_t n = s->nchunks;
  s->current_nchunk = op == kAppend ? n : nchunk;
  s->nchunks = n + 1;
  s->nbytes += ci.nbytes;
  s->cbytes += ci.cbytes;
  if (nchunk < n) memmove(s->data + nchunk + 1, s->data + nchunk, (size_t)(n - nchunk) * sizeof(uint8_t*));
  s->data[nchunk] = kept;
  return s->nchunks;
}

// The super-chunk's copies of its storage's parameters and its two contexts (the fields
// blosc/schunk.c:108-153 derives): the per-chunk knobs come from cparams, chunksize and flags2 are
// unknown until the first chunk, and each context is told which super-chunk it serves.
int adopt_params(blosc2_schunk* s) {
  const blosc2_cparams& cp = *s->storage->cparams;
  s->compcode = cp.compcode;
  s->compcode_meta = cp.compcode_meta;
  s->clevel = cp.clevel;
  s->splitmode = (uint8_t)cp.splitmode;
  s->use_dict = (uint8_t)cp.use_dict;
  s->typesize = cp.typesize;
  s->blocksize = cp.blocksize;
  memcpy(s->filters, cp.filters, BLOSC2_MAX_FILTERS);
  memcpy(s->filters_meta, cp.filters_meta, BLOSC2_MAX_FILTERS);
  s->tuner_params = cp.tuner_params;
  s->tuner_id = cp.tuner_id;
  s->chunksize = -1;
  s->flags2 = 0;
  blosc2_context* made[2] = {nullptr, nullptr};
  s->storage->cparams->schunk = s;
  s->storage->dparams->schunk = s;
  made[0] = blosc2_create_cctx(*s->storage->cparams);
  made[1] = blosc2_create_dctx(*s->storage->dparams);
  if (s->cctx) blosc2_free_ctx(s->cctx);
  if (s->dctx) blosc2_free_ctx(s->dctx);
  s->cctx = made[0];
  s->dctx = made[1];
  if (!made[0] || !made[1]) {
    TRACE_ERROR("super-chunk: %s context not created", made[0] ? "decompression" : "compression");
    return BLOSC2_ERROR_NULL_POINTER;
  }
  return 0;
}

void free_layers(blosc2_metalayer** layers, int n) {   // schunk.c:653-676
  for (int i = 0; i < n; i++) {
    if (!layers[i]) continue;
    free(layers[i]->name);
    free(layers[i]->content);
    free(layers[i]);
    layers[i] = nullptr;
  }
}

}  // namespace

// ------------------------------------------------------------------------ defaults getters ----
// blosc/blosc2.c:6896-6911
blosc2_cparams blosc2_get_blosc2_cparams_defaults(void) { return BLOSC2_CPARAMS_DEFAULTS; }
blosc2_dparams blosc2_get_blosc2_dparams_defaults(void) { return BLOSC2_DPARAMS_DEFAULTS; }
blosc2_storage blosc2_get_blosc2_storage_defaults(void) { return BLOSC2_STORAGE_DEFAULTS; }
blosc2_io blosc2_get_blosc2_io_defaults(void) { return BLOSC2_IO_DEFAULTS; }

// ------------------------------------------------------------------------------ lifetime ----
// schunk.c:163-242 with get_new_storage (frame.c:2834-2877): the storage, its cparams, dparams and
// io are private copies (defaults where the caller passed NULL).
blosc2_schunk* blosc2_schunk_new(blosc2_storage* storage) {
  const blosc2_storage st = storage ? *storage : BLOSC2_STORAGE_DEFAULTS;
  if (st.contiguous || st.urlpath) {
    TRACE_ERROR("frame-backed super-chunks (contiguous / urlpath) are outside the device engine; "
                "use an in-memory sparse storage (contiguous = false, urlpath = NULL)");
    return nullptr;
  }
  blosc2_schunk* s = static_cast<blosc2_schunk*>(calloc(1, sizeof(blosc2_schunk)));
  blosc2_storage* ns = static_cast<blosc2_storage*>(calloc(1, sizeof(blosc2_storage)));
  blosc2_cparams* cp = static_cast<blosc2_cparams*>(malloc(sizeof(blosc2_cparams)));
  blosc2_dparams* dp = static_cast<blosc2_dparams*>(malloc(sizeof(blosc2_dparams)));
  blosc2_io* io = static_cast<blosc2_io*>(malloc(sizeof(blosc2_io)));
  if (!s || !ns || !cp || !dp || !io) {
    free(s);
    free(ns);
    free(cp);
    free(dp);
    free(io);
    return nullptr;
  }
  *ns = st;
  *cp = st.cparams ? *st.cparams : BLOSC2_CPARAMS_DEFAULTS;
  *dp = st.dparams ? *st.dparams : BLOSC2_DPARAMS_DEFAULTS;
  *io = st.io ? *st.io : BLOSC2_IO_DEFAULTS;
  ns->cparams = cp;
  ns->dparams = dp;
  ns->io = io;
  s->storage = ns;
  s->version = 0;   // pre-first version
  s->view = false;
  if (adopt_params(s) < 0) {
    blosc2_schunk_free(s);
    return nullptr;
  }
  return s;
}

// schunk.c:679-727
int blosc2_schunk_free(blosc2_schunk* schunk) {
  if (!schunk) return 0;
  if (schunk->frame) b2h::link_free(schunk);   // an attached handle: its index and its frame link
  if (schunk->data && !schunk->view) {
    for (int64_t i = 0; i < schunk->nchunks; i++) free(schunk->data[i]);
    free(schunk->data);
  }
  if (schunk->cctx) blosc2_free_ctx(schunk->cctx);
  if (schunk->dctx) blosc2_free_ctx(schunk->dctx);
  free(schunk->blockshape);
  free_layers(schunk->metalayers, schunk->nmetalayers);
  schunk->nmetalayers = 0;
  if (schunk->storage) {
    free(schunk->storage->urlpath);
    free(schunk->storage->cparams);
    free(schunk->storage->dparams);
    free(schunk->storage->io);
    free(schunk->storage);
  }
  free_layers(schunk->vlmetalayers, schunk->nvlmetalayers);
  schunk->nvlmetalayers = 0;
  free(schunk);
  return 0;
}

// ---------------------------------------------------------------------- chunk index ops ----
// A handle attached to a contiguous frame (blosc2_schunk_open / _from_buffer(copy = false),
// b2h_frame.cpp) reads its chunks from the frame; the reference's writes go back to the frame
// (frame_append_chunk etc.), which this engine does not write in place.  Such handles are
// read-only: every write entry point refuses them (blosc2_schunk_to_buffer / _to_file write a
// new frame instead).
static int refuse_if_attached(const blosc2_schunk* s, const char* fn) {
  if (s->storage && (s->storage->contiguous || s->storage->urlpath)) {
    TRACE_ERROR("%s: super-chunks attached to a frame are read-only in the MI355X engine", fn);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  return 0;
}

int64_t blosc2_schunk_append_chunk(blosc2_schunk* schunk, uint8_t* chunk, bool copy) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_append_chunk")) return rc0;
  return put_chunk(schunk, kAppend, schunk->nchunks, chunk, copy);
}

int64_t blosc2_schunk_insert_chunk(blosc2_schunk* schunk, int64_t nchunk, uint8_t* chunk, bool copy) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_insert_chunk")) return rc0;
  const int rc = validate_nchunk(schunk, nchunk, true, "blosc2_schunk_insert_chunk");
  if (rc < 0) return rc;
  return put_chunk(schunk, kInsert, nchunk, chunk, copy);
}

// schunk.c:1235-1360
int64_t blosc2_schunk_update_chunk(blosc2_schunk* schunk, int64_t nchunk, uint8_t* chunk, bool copy) {
  if (!schunk || !chunk) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_update_chunk")) return rc0;
  int rc = validate_nchunk(schunk, nchunk, false, "blosc2_schunk_update_chunk");
  if (rc < 0) return rc;
  ChunkInfo ci;
  if ((rc = chunk_info(chunk, &ci)) < 0) return rc;
  // compared with another chunk when there is one (chunk 1 when chunk 0 itself is replaced)
  const int64_t ref = (schunk->nchunks > 1 || nchunk != 0) ? (nchunk == 0 ? 1 : 0) : -1;
  if ((rc = check_kind(schunk, ref, ci, BLOSC2_ERROR_CHUNK_UPDATE)) < 0) return rc;
  if ((rc = settle_chunksize(schunk, kUpdate, nchunk, ci.nbytes, BLOSC2_ERROR_CHUNK_UPDATE)) < 0) return rc;
  int32_t nb_old, cb_old;
  old_sizes(schunk->data[nchunk], &nb_old, &cb_old);
  schunk->current_nchunk = nchunk;
  uint8_t* kept = keep_chunk(chunk, ci, copy);
  if (!kept) return BLOSC2_ERROR_MEMORY_ALLOC;
  schunk->nbytes += (int64_t)ci.nbytes - nb_old;
  schunk->cbytes += (int64_t)ci.cbytes - cb_old;
  free(schunk->data[nchunk]);
  schunk->data[nchunk] = kept;
  return schunk->nchunks;
}

// schunk.c:1375-1442
int64_t blosc2_schunk_delete_chunk(blosc2_schunk* schunk, int64_t nchunk) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_delete_chunk")) return rc0;
  const int rc = validate_nchunk(schunk, nchunk, false, "blosc2_schunk_delete_chunk");
  if (rc < 0) return rc;
  int32_t nb_old, cb_old;
  old_sizes(schunk->data[nchunk], &nb_old, &cb_old);
  schunk->current_nchunk = nchunk;
  schunk->nchunks -= 1;
  if (schunk->nchunks == 0) schunk->flags2 = 0;
  schunk->nbytes -= nb_old;
  schunk->cbytes -= cb_old;
  free(schunk->data[nchunk]);
  memmove(schunk->data + nchunk, schunk->data + nchunk + 1, (size_t)(schunk->nchunks - nchunk) * sizeof(uint8_t*));
  schunk->data[schunk->nchunks] = nullptr;
  return schunk->nchunks;
}

// ---------------------------------------------------------------------- compress / decode ----
// schunk.c:1459-1477
int64_t blosc2_schunk_append_buffer(blosc2_schunk* schunk, const void* src, int32_t nbytes) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_append_buffer")) return rc0;
  if (nbytes < 0 || nbytes > BLOSC2_MAX_BUFFERSIZE) return BLOSC2_ERROR_INVALID_PARAM;
  uint8_t* chunk = static_cast<uint8_t*>(malloc((size_t)nbytes + BLOSC2_MAX_OVERHEAD));
  if (!chunk) return BLOSC2_ERROR_MEMORY_ALLOC;
  schunk->current_nchunk = schunk->nchunks;
  const int cbytes = blosc2_compress_ctx(schunk->cctx, src, nbytes, chunk, nbytes + BLOSC2_MAX_OVERHEAD);
  if (cbytes < 0) {
    free(chunk);
    return cbytes;
  }
  const int64_t n = blosc2_schunk_append_chunk(schunk, chunk, false);
  if (n < 0) {
    TRACE_ERROR("Error appending a buffer in super-chunk");
    free(chunk);
  }
  return n;
}

// schunk.c:1481-1530
int blosc2_schunk_decompress_chunk(blosc2_schunk* schunk, int64_t nchunk, void* dest, int32_t nbytes) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  int rc = validate_nchunk(schunk, nchunk, false, "blosc2_schunk_decompress_chunk");
  if (rc < 0) return rc;
  schunk->current_nchunk = nchunk;
  uint8_t* src = schunk->data[nchunk];
  bool needs_free = false;
  if (!src && schunk->frame) {   // frame_decompress_chunk (frame.c:5248-5290): the chunk off the frame
    if ((rc = b2h::link_get_chunk(schunk, nchunk, &src, &needs_free)) < 0) return rc;
  }
  if (!src) return 0;
  struct Freer {
    uint8_t* p;
    ~Freer() { free(p); }
  } freer{needs_free ? src : nullptr};
  int32_t chunk_nbytes, chunk_cbytes;
  if ((rc = blosc2_cbuffer_sizes(src, &chunk_nbytes, &chunk_cbytes, nullptr)) < 0) return rc;
  if (nbytes < chunk_nbytes) {
    TRACE_ERROR("Buffer size is too small for the decompressed buffer ('%d' bytes, but '%d' are needed).", nbytes,
                chunk_nbytes);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  const int got = blosc2_decompress_ctx(schunk->dctx, src, chunk_cbytes, dest, nbytes);
  if (got < 0) return got;
  if (got != chunk_nbytes) {
    TRACE_ERROR("Error in decompressing chunk.");
    return BLOSC2_ERROR_FAILURE;
  }
  return got;
}

// schunk.c:1543-1632 (frame-less: the chunk is the super-chunk's own buffer, never to be freed;
// frame-attached: frame_get_chunk, a chunk read off a frame file is the caller's to free)
static int get_chunk(blosc2_schunk* schunk, int64_t nchunk, uint8_t** chunk, bool* needs_free, const char* fn) {
  if (!schunk || !chunk || !needs_free) return BLOSC2_ERROR_NULL_POINTER;
  int rc = validate_nchunk(schunk, nchunk, false, fn);
  if (rc < 0) return rc;
  schunk->current_nchunk = nchunk;
  if (schunk->frame) return b2h::link_get_chunk(schunk, nchunk, chunk, needs_free);
  *chunk = schunk->data[nchunk];
  *needs_free = false;
  if (!*chunk) return 0;
  int32_t cbytes;
  if ((rc = blosc2_cbuffer_sizes(*chunk, nullptr, &cbytes, nullptr)) < 0) return rc;
  return cbytes;
}

int blosc2_schunk_get_chunk(blosc2_schunk* schunk, int64_t nchunk, uint8_t** chunk, bool* needs_free) {
  return get_chunk(schunk, nchunk, chunk, needs_free, "blosc2_schunk_get_chunk");
}

int blosc2_schunk_get_lazychunk(blosc2_schunk* schunk, int64_t nchunk, uint8_t** chunk, bool* needs_free) {
  return get_chunk(schunk, nchunk, chunk, needs_free, "blosc2_schunk_get_lazychunk");
}

// Items [start, stop) of the super-chunk.  The range is checked (the reference reads past the
// super-chunk for a range outside it); chunks are walked as schunk.c:1662-1783 walks them: a chunk
// wholly inside the range decompresses straight into the buffer, an edge chunk goes through
// blosc2_getitem_bytes_ctx.
int blosc2_schunk_get_slice_buffer(blosc2_schunk* schunk, int64_t start, int64_t stop, void* buffer) {
  if (!schunk || !buffer) return BLOSC2_ERROR_NULL_POINTER;
  const int64_t ts = schunk->typesize;
  if (start < 0 || stop < start || ts <= 0 || stop * ts > schunk->nbytes || schunk->chunksize <= 0) {
    TRACE_ERROR("slice [%lld, %lld) is outside the super-chunk (or the super-chunk has no fixed chunksize)",
                (long long)start, (long long)stop);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  const int64_t cs = schunk->chunksize, b0 = start * ts, b1 = stop * ts;
  uint8_t* dst = static_cast<uint8_t*>(buffer);
  for (int64_t k = b0 / cs; k * cs < b1; k++) {
    uint8_t* chunk;
    bool needs_free;
    const int cbytes = blosc2_schunk_get_lazychunk(schunk, k, &chunk, &needs_free);
    if (cbytes < 0) {
      TRACE_ERROR("Cannot get lazychunk ('%lld').", (long long)k);
      return BLOSC2_ERROR_FAILURE;
    }
    const int64_t len = (k == schunk->nchunks - 1 && schunk->nbytes % cs) ? schunk->nbytes % cs : cs;
    const int32_t lo = (int32_t)(std::max(b0, k * cs) - k * cs), hi = (int32_t)(std::min(b1, k * cs + len) - k * cs);
    int got;
    if (lo == 0 && hi == len) {
      got = blosc2_decompress_ctx(schunk->dctx, chunk, cbytes, dst, (int32_t)len);
      if (got < 0) {
        TRACE_ERROR("Cannot decompress chunk ('%lld').", (long long)k);
        return BLOSC2_ERROR_FAILURE;
      }
    } else {
      got = blosc2_getitem_bytes_ctx(schunk->dctx, chunk, cbytes, lo, hi - lo, dst, hi - lo);
      if (got != hi - lo) {
        TRACE_ERROR("Cannot get items from ('%lld') chunk (%d of %d bytes).", (long long)k, got, hi - lo);
        return BLOSC2_ERROR_FAILURE;
      }
    }
    dst += got;
  }
  return BLOSC2_ERROR_SUCCESS;
}

// blosc2_schunk_get_sparse_buffer (blosc/schunk.c:1922-2110).  The argument checks are the
// reference's, in its order.  Under DELTA, with a postfilter, or for a single coordinate it takes
// one getitem per coordinate (schunk_get_sparse_getitem, schunk.c:1866-1900): the bounds check
// of a coordinate only when its turn comes.  Otherwise every coordinate is checked first, the
// coordinates are sorted by (coord, output index) and grouped by chunk and block, every touched
// chunk is fetched, and then -- where the reference decodes each touched block with
// blosc2_decompress_block_ctx on its thread pool -- a chunk with several touched blocks is decoded
// once on the device with the other blocks masked (one device call per chunk).  A chunk whose
// masked decode fails, or whose own blocksize is not the super-chunk's, takes the reference's
// per-block calls, so the error code is the one its serial walk meets first.
int blosc2_schunk_get_sparse_buffer(blosc2_schunk* schunk, int64_t ncoords, const int64_t* coords, void* buffer) {
  if (!schunk) return BLOSC2_ERROR_INVALID_PARAM;
  if (ncoords < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (ncoords == 0) return BLOSC2_ERROR_SUCCESS;
  if (!coords || !buffer) return BLOSC2_ERROR_INVALID_PARAM;
  if (schunk->typesize <= 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (schunk->chunksize <= 0) {
    TRACE_ERROR("blosc2_schunk_get_sparse_buffer does not support variable-length chunks yet.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if (schunk->blocksize <= 0 || (schunk->flags2 & BLOSC2_VL_BLOCKS)) {
    TRACE_ERROR("blosc2_schunk_get_sparse_buffer does not support variable-length blocks yet.");
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  const int64_t ts = schunk->typesize, cs = schunk->chunksize, bs = schunk->blocksize;
  if (cs % ts || bs % ts) return BLOSC2_ERROR_INVALID_PARAM;
  const int64_t nitems = schunk->nbytes / ts, chunk_nitems = cs / ts;
  uint8_t* out = static_cast<uint8_t*>(buffer);

  bool per_item = ncoords <= 1;
  for (int i = 0; i < BLOSC2_MAX_FILTERS; i++) per_item |= schunk->filters[i] == BLOSC_DELTA;
  blosc2_dparams dp;
  per_item |= schunk->dctx && blosc2_ctx_get_dparams(schunk->dctx, &dp) == 0 && dp.postfilter;
  if (per_item) {
    for (int64_t i = 0; i < ncoords; i++) {
      const int64_t coord = coords[i];
      if (coord < 0 || coord >= nitems) return BLOSC2_ERROR_INVALID_PARAM;
      uint8_t* chunk;
      bool needs_free = false;
      const int cbytes = blosc2_schunk_get_lazychunk(schunk, coord / chunk_nitems, &chunk, &needs_free);
      if (cbytes <= 0) return BLOSC2_ERROR_FAILURE;
      const int got = blosc2_getitem_bytes_ctx(schunk->dctx, chunk, cbytes, (int32_t)((coord % chunk_nitems) * ts),
                                               (int32_t)ts, out + i * ts, (int32_t)ts);
      if (needs_free) free(chunk);
      if (got != ts) return BLOSC2_ERROR_FAILURE;
    }
    return BLOSC2_ERROR_SUCCESS;
  }

  for (int64_t i = 0; i < ncoords; i++)
    if (coords[i] < 0 || coords[i] >= nitems) return BLOSC2_ERROR_INVALID_PARAM;
  if (chunk_nitems > INT32_MAX) return BLOSC2_ERROR_INVALID_PARAM;
  std::vector<std::pair<int64_t, int64_t>> e((size_t)ncoords);   // (coord, output index)
  for (int64_t i = 0; i < ncoords; i++) e[(size_t)i] = {coords[i], i};
  std::sort(e.begin(), e.end());
  struct Fetched {
    uint8_t* chunk;
    int cbytes;
    bool needs_free;
    size_t first, last;   // its entries [first, last)
  };
  std::vector<Fetched> chunks;
  struct Freer {
    std::vector<Fetched>* v;
    ~Freer() {
      for (auto& f : *v)
        if (f.needs_free) free(f.chunk);
    }
  } freer{&chunks};
  for (size_t i = 0; i < e.size();) {   // every touched chunk fetched before any decode
    const int64_t nchunk = e[i].first / chunk_nitems;
    size_t j = i;
    while (j < e.size() && e[j].first / chunk_nitems == nchunk) j++;
    Fetched f{nullptr, 0, false, i, j};
    f.cbytes = blosc2_schunk_get_lazychunk(schunk, nchunk, &f.chunk, &f.needs_free);
    if (f.cbytes <= 0) {
      TRACE_ERROR("Cannot get lazychunk ('%lld').", (long long)nchunk);
      return BLOSC2_ERROR_FAILURE;
    }
    chunks.push_back(f);
    i = j;
  }
  std::vector<uint8_t> img, blk((size_t)bs);
  auto block_of = [&](int64_t coord) { return (int32_t)(((coord % chunk_nitems) * ts) / bs); };
  auto put = [&](const uint8_t* b, int32_t nbytes, size_t first, size_t last) {
    for (size_t k = first; k < last; k++) {
      const int32_t off = (int32_t)(((e[k].first % chunk_nitems) * ts) % bs);
      if (off > nbytes - ts) return (int)BLOSC2_ERROR_DATA;
      memcpy(out + e[k].second * ts, b + off, (size_t)ts);
    }
    return 0;
  };
  for (const Fetched& f : chunks) {
    int32_t nblocks_touched = 0;
    for (size_t k = f.first; k < f.last; k++)
      nblocks_touched += k == f.first || block_of(e[k].first) != block_of(e[k - 1].first);
    int32_t c_nbytes = 0, c_bs = 0;
    bool whole = nblocks_touched > 1 && blosc2_cbuffer_sizes(f.chunk, &c_nbytes, nullptr, &c_bs) >= 0 &&
                 c_bs == bs && c_nbytes > 0;
    if (whole) {
      const int32_t nb = (int32_t)((c_nbytes + bs - 1) / bs);
      std::vector<uint8_t> mask((size_t)nb, 1);
      bool fits = true;
      for (size_t k = f.first; k < f.last; k++) {
        const int32_t b = block_of(e[k].first);
        fits &= b < nb;
        if (b < nb) mask[(size_t)b] = 0;
      }
      img.resize((size_t)c_nbytes);
      whole = fits && blosc2_set_maskout(schunk->dctx, reinterpret_cast<bool*>(mask.data()), nb) == 0 &&
              blosc2_decompress_ctx(schunk->dctx, f.chunk, f.cbytes, img.data(), c_nbytes) == c_nbytes;
    }
    for (size_t k = f.first; k < f.last;) {   // one task per touched block, in order
      const int32_t b = block_of(e[k].first);
      size_t k2 = k;
      while (k2 < f.last && block_of(e[k2].first) == b) k2++;
      int rc;
      if (whole) {
        rc = put(img.data() + (int64_t)b * bs, (int32_t)std::min<int64_t>(bs, c_nbytes - (int64_t)b * bs), k, k2);
      } else {
        const int nbytes = blosc2_decompress_block_ctx(schunk->dctx, f.chunk, f.cbytes, b, blk.data(), (int32_t)bs);
        rc = nbytes < 0 ? nbytes : put(blk.data(), nbytes, k, k2);
      }
      if (rc < 0) return rc;
      k = k2;
    }
  }
  return BLOSC2_ERROR_SUCCESS;
}

// schunk.c:70-105
int blosc2_schunk_get_cparams(blosc2_schunk* schunk, blosc2_cparams** cparams) {
  if (!schunk || !cparams) return BLOSC2_ERROR_NULL_POINTER;
  blosc2_cparams* cp = static_cast<blosc2_cparams*>(calloc(1, sizeof(blosc2_cparams)));
  if (!cp) return BLOSC2_ERROR_MEMORY_ALLOC;
  cp->schunk = schunk;
  memcpy(cp->filters, schunk->filters, BLOSC2_MAX_FILTERS);
  memcpy(cp->filters_meta, schunk->filters_meta, BLOSC2_MAX_FILTERS);
  cp->compcode = schunk->compcode;
  cp->compcode_meta = schunk->compcode_meta;
  cp->clevel = schunk->clevel;
  cp->typesize = schunk->typesize;
  cp->blocksize = schunk->blocksize;
  cp->splitmode = schunk->splitmode;
  cp->use_dict = schunk->use_dict;
  blosc2_cparams ctx_cp;
  cp->nthreads = (schunk->cctx && blosc2_ctx_get_cparams(schunk->cctx, &ctx_cp) == 0) ? ctx_cp.nthreads
                                                                                      : blosc2_get_nthreads();
  *cparams = cp;
  return 0;
}

int blosc2_schunk_get_dparams(blosc2_schunk* schunk, blosc2_dparams** dparams) {
  if (!schunk || !dparams) return BLOSC2_ERROR_NULL_POINTER;
  blosc2_dparams* dp = static_cast<blosc2_dparams*>(calloc(1, sizeof(blosc2_dparams)));
  if (!dp) return BLOSC2_ERROR_MEMORY_ALLOC;
  dp->schunk = schunk;
  blosc2_dparams ctx_dp;
  dp->nthreads = (schunk->dctx && blosc2_ctx_get_dparams(schunk->dctx, &ctx_dp) == 0) ? ctx_dp.nthreads
                                                                                      : blosc2_get_nthreads();
  *dparams = dp;
  return 0;
}

// ------------------------------------------------------------------ device batch forms ----
// n blosc2_schunk_append_buffer calls in one: the chunks are compressed by device batches on the
// super-chunk's cctx (its sticky blocksize carried as the serial calls carry it), brought back in one
// copy per group and appended in order.  A pipeline with user-registered filters / codecs runs the
// serial calls instead (chunk by chunk through host memory).
int64_t b2h_schunk_append_device(blosc2_schunk* schunk, const void* d_src, const int32_t* nbytes, int32_t n,
                                 int64_t src_stride) {
  if (!schunk || (n > 0 && (!d_src || !nbytes))) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "b2h_schunk_append_device")) return rc0;
  if (n < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (n == 0) return schunk->nchunks;
  const uint8_t* src = static_cast<const uint8_t*>(d_src);
  std::vector<uint8_t*> chunks((size_t)n, nullptr);
  int rc = b2h::ctx_append_device(schunk->cctx, src, nbytes, n, src_stride, chunks.data());
  if (rc == BLOSC2_ERROR_FILTER_PIPELINE) {
    std::vector<uint8_t> host;
    int64_t r = schunk->nchunks;
    for (int32_t i = 0; i < n && r >= 0; i++) {
      host.resize((size_t)std::max(nbytes[i], 1));
      if (hipMemcpy(host.data(), src + (int64_t)i * src_stride, (size_t)nbytes[i], hipMemcpyDeviceToHost) != hipSuccess)
        return BLOSC2_ERROR_FAILURE;
      r = blosc2_schunk_append_buffer(schunk, host.data(), nbytes[i]);
    }
    return r;
  }
  if (rc < 0) return rc;
  int64_t r = schunk->nchunks;
  for (int32_t i = 0; i < n; i++) {
    r = blosc2_schunk_append_chunk(schunk, chunks[i], false);
    if (r < 0) {
      for (int32_t j = i; j < n; j++) free(chunks[j]);
      return r;
    }
  }
  return r;
}

// Chunks [nchunk, nchunk + n) into d_dst + i * dst_stride in one device batch; status[i] (optional)
// = what blosc2_schunk_decompress_chunk(schunk, nchunk + i, ., dst_capacity) returns.
namespace {
int staged_decode(blosc2_schunk* schunk, blosc2_context* ctx, int device, int64_t c0, int32_t n, uint8_t* out_host,
                  uint8_t* out_dev, int64_t dst_stride, int32_t dst_capacity, int32_t* st);
}  // namespace

int b2h_schunk_decompress_device(blosc2_schunk* schunk, int64_t nchunk, int32_t n, void* d_dst, int64_t dst_stride,
                                 int32_t dst_capacity, int32_t* status) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (n < 0 || nchunk < 0 || nchunk + n > schunk->nchunks) {
    TRACE_ERROR("chunks [%lld, %lld) are outside the super-chunk (%lld chunks)", (long long)nchunk,
                (long long)(nchunk + n), (long long)schunk->nchunks);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if (n == 0) return 0;
  std::vector<int32_t> st((size_t)n);
  schunk->current_nchunk = nchunk + n - 1;
  int device = 0;
  if (hipGetDevice(&device) != hipSuccess) return BLOSC2_ERROR_FAILURE;
  const int rc = staged_decode(schunk, schunk->dctx, device, nchunk, n, nullptr, static_cast<uint8_t*>(d_dst),
                               dst_stride, dst_capacity, st.data());
  if (status) memcpy(status, st.data(), sizeof(int32_t) * (size_t)n);
  return rc;
}

// blosc2_schunk_get_slice_buffer into device memory: the chunks wholly inside [start, stop) decode
// in one device batch straight into place, the (at most two) edge chunks through getitem.
int b2h_schunk_get_slice_device(blosc2_schunk* schunk, int64_t start, int64_t stop, void* d_dst) {
  if (!schunk || !d_dst) return BLOSC2_ERROR_NULL_POINTER;
  const int64_t ts = schunk->typesize;
  if (start < 0 || stop < start || ts <= 0 || stop * ts > schunk->nbytes || schunk->chunksize <= 0)
    return BLOSC2_ERROR_INVALID_PARAM;
  if (start == stop) return 0;
  const int64_t cs = schunk->chunksize, b0 = start * ts, b1 = stop * ts;
  uint8_t* dst = static_cast<uint8_t*>(d_dst);
  int64_t f0 = -1, f1 = -1;   // the run of whole chunks
  std::vector<uint8_t> edge;
  for (int64_t k = b0 / cs; k * cs < b1; k++) {
    const int64_t len = (k == schunk->nchunks - 1 && schunk->nbytes % cs) ? schunk->nbytes % cs : cs;
    const int32_t lo = (int32_t)(std::max(b0, k * cs) - k * cs), hi = (int32_t)(std::min(b1, k * cs + len) - k * cs);
    if (lo == 0 && hi == len) {
      if (f0 < 0) f0 = k;
      f1 = k;
      continue;
    }
    uint8_t* chunk;
    bool needs_free;
    const int cbytes = blosc2_schunk_get_lazychunk(schunk, k, &chunk, &needs_free);
    if (cbytes <= 0) return BLOSC2_ERROR_FAILURE;
    edge.resize((size_t)(hi - lo));
    if (blosc2_getitem_bytes_ctx(schunk->dctx, chunk, cbytes, lo, hi - lo, edge.data(), hi - lo) != hi - lo)
      return BLOSC2_ERROR_FAILURE;
    if (hipMemcpy(dst + (k * cs + lo - b0), edge.data(), edge.size(), hipMemcpyHostToDevice) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
  }
  if (f0 >= 0) {
    const int32_t m = (int32_t)(f1 - f0 + 1);
    std::vector<int32_t> st((size_t)m);
    std::vector<const uint8_t*> ptrs;
    b2h::ReadBuf hold;
    int rc = b2h::chunk_ptrs(schunk, f0, m, &ptrs, &hold);
    if (rc < 0) return rc;
    rc = b2h::ctx_decompress_device(schunk->dctx, ptrs.data(), m, dst + (f0 * cs - b0), cs, (int32_t)cs, st.data());
    if (rc < 0) return BLOSC2_ERROR_FAILURE;
    schunk->current_nchunk = f1;
  }
  return 0;
}

// ------------------------------------------------------------ multi-device fan-out ----
// The reference's C callers loop over chunks (blosc2_schunk_append_buffer /
// blosc2_schunk_decompress_chunk, blosc/schunk.c:1459-1530) and its thread pool spreads each chunk's
// blocks over cores.  Here a C caller hands over many chunks at once and they are spread over the
// node's GPUs: `workers` host threads, worker k on device k % device_count, each with its own
// contexts (stream, workspace) and a contiguous range of the chunks.  No collective: chunks are
// independent.  Worker k's compression context starts from the sticky blocksize the serial calls
// would have reached at its first chunk (ctx_blocksize_walk), so every chunk equals the serial
// call's bytes and the super-chunk's context ends in the serial state.
namespace {
int fanout_workers(int32_t ndevices, int32_t n) {
  const int nd = b2h::device_count();
  if (nd <= 0) return 0;
  const int w = ndevices > 0 ? ndevices : nd;
  return std::max(1, std::min(w, (int)std::max<int32_t>(n, 1)));
}

// Bytes of one staging group: the device batches move through host memory in groups of this
// size, so a range larger than HBM streams through instead of failing its allocation.
constexpr int64_t kGroupBytes = int64_t(128) << 20;

// Host copies between the caller's (pageable) buffers and a pinned staging buffer, split over a
// few threads: one thread's memcpy (~10 GB/s) would otherwise bound the whole fan-out.
void par_copy(uint8_t* dst, int64_t dst_stride, const uint8_t* src, int64_t src_stride, int32_t rows, int64_t row_bytes) {
  const int64_t total = (int64_t)rows * row_bytes;
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(4, total >> 24));
  auto part = [&](int t) {
    for (int32_t r = (int32_t)((int64_t)rows * t / T); r < (int32_t)((int64_t)rows * (t + 1) / T); r++)
      memcpy(dst + (int64_t)r * dst_stride, src + (int64_t)r * src_stride, (size_t)row_bytes);
  };
  if (T == 1) return part(0);
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
}

// One fan-out worker's staging: three pinned host buffers (a ring: one being filled by the host
// copy, one in flight over PCIe, one spare) and two device buffers (one being copied into while
// the engine works on the other), a copy stream and an event per device buffer.
struct Stage {
  void* pin[3] = {nullptr, nullptr, nullptr};
  uint8_t* dev[2] = {nullptr, nullptr};
  hipStream_t cs = nullptr;
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool init(size_t bytes) {
    for (auto& x : pin)
      if (hipHostMalloc(&x, std::max<size_t>(bytes, 1), hipHostMallocDefault) != hipSuccess) return false;
    for (auto& x : dev)
      if (hipMalloc(&x, std::max<size_t>(bytes, 1)) != hipSuccess) return false;
    if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return false;
    for (auto& e : ev)
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return false;
    return true;
  }
  ~Stage() {
    if (cs) (void)hipStreamSynchronize(cs);
    for (auto& e : ev) if (e) (void)hipEventDestroy(e);
    if (cs) (void)hipStreamDestroy(cs);
    for (auto& x : dev) if (x) (void)hipFree(x);
    for (auto& x : pin) if (x) (void)hipHostFree(x);
  }
  uint8_t* p(int i) const { return static_cast<uint8_t*>(pin[i % 3]); }
};
}  // namespace

// Worker threads are spawned for every device, the caller's thread included none: its current
// device is never changed (a torch rank bound to device d keeps d).
int64_t b2h_schunk_append_buffers(blosc2_schunk* schunk, const void* src, const int32_t* nbytes, int32_t n,
                                  int64_t src_stride, int32_t ndevices) {
  if (!schunk || (n > 0 && (!src || !nbytes))) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "b2h_schunk_append_buffers")) return rc0;
  if (n < 0 || src_stride < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (n == 0) return schunk->nchunks;
  for (int32_t i = 0; i < n; i++)
    if (nbytes[i] < 0 || nbytes[i] > BLOSC2_MAX_BUFFERSIZE || (int64_t)nbytes[i] > src_stride)
      return BLOSC2_ERROR_INVALID_PARAM;
  const int W = fanout_workers(ndevices, n);
  if (W == 0) {
    TRACE_ERROR("no HIP device available: the MI355X engine has no CPU fallback");
    return BLOSC2_ERROR_FAILURE;
  }
  const uint8_t* h = static_cast<const uint8_t*>(src);
  std::vector<int32_t> before((size_t)n + 1);
  int rc = b2h::ctx_blocksize_walk(schunk->cctx, nbytes, n, before.data());
  if (rc < 0) return rc;
  std::vector<uint8_t*> chunks((size_t)n, nullptr);
  std::vector<int> wrc((size_t)W, 0);
  const int32_t maxnb = *std::max_element(nbytes, nbytes + n);
  auto work = [&](int k) {
    const int32_t i0 = (int32_t)((int64_t)n * k / W), i1 = (int32_t)((int64_t)n * (k + 1) / W);
    if (i1 <= i0) return;
    if (hipSetDevice(k % b2h::device_count()) != hipSuccess) { wrc[k] = BLOSC2_ERROR_FAILURE; return; }
    blosc2_context* ctx = b2h::ctx_clone(schunk->cctx);
    if (!ctx) { wrc[k] = BLOSC2_ERROR_MEMORY_ALLOC; return; }
    b2h::ctx_set_blocksize(ctx, before[i0]);
    // groups of G chunks: host copy of group g + 2, H2D of group g + 1 and the engine on group g
    // run at once (the copy on helper threads, the H2D on the copy stream)
    const int32_t G = (int32_t)std::max<int64_t>(1, std::min<int64_t>(i1 - i0, kGroupBytes / std::max<int64_t>(src_stride, 1)));
    const int32_t ng = (i1 - i0 + G - 1) / G;
    const int64_t row = std::min<int64_t>(src_stride, maxnb);
    Stage S;
    auto lo = [&](int32_t g) { return i0 + g * G; };
    auto cnt = [&](int32_t g) { return std::min(G, i1 - lo(g)); };
    auto stage = [&](int32_t g) { par_copy(S.p(g), src_stride, h + (int64_t)lo(g) * src_stride, src_stride, cnt(g), row); };
    auto h2d = [&](int32_t g) {
      return hipMemcpyAsync(S.dev[g % 2], S.p(g), (size_t)cnt(g) * (size_t)src_stride, hipMemcpyHostToDevice, S.cs) ==
                 hipSuccess &&
             hipEventRecord(S.ev[g % 2], S.cs) == hipSuccess;
    };
    int r = S.init((size_t)G * (size_t)src_stride) ? 0 : BLOSC2_ERROR_MEMORY_ALLOC;
    if (r == 0) {
      stage(0);
      if (ng > 1) stage(1);
      if (!h2d(0)) r = BLOSC2_ERROR_FAILURE;
    }
    for (int32_t g = 0; g < ng && r == 0; g++) {
      std::thread ahead;
      if (g + 2 < ng) ahead = std::thread(stage, g + 2);   // its buffer's H2D (group g - 1) completed
      if (hipEventSynchronize(S.ev[g % 2]) != hipSuccess) r = BLOSC2_ERROR_FAILURE;
      if (r == 0 && g + 1 < ng && !h2d(g + 1)) r = BLOSC2_ERROR_FAILURE;
      if (r == 0) r = b2h::ctx_append_device(ctx, S.dev[g % 2], nbytes + lo(g), cnt(g), src_stride, chunks.data() + lo(g));
      if (ahead.joinable()) ahead.join();
    }
    wrc[k] = r;
    blosc2_free_ctx(ctx);
  };
  std::vector<std::thread> th;
  for (int k = 0; k < W; k++) th.emplace_back(work, k);
  for (auto& t : th) t.join();
  rc = 0;
  for (int k = 0; k < W && rc == 0; k++) rc = wrc[k];
  if (rc == BLOSC2_ERROR_FILTER_PIPELINE) {   // user callbacks, prefilters: the serial calls, through host memory
    for (uint8_t* c : chunks) free(c);
    int64_t r = schunk->nchunks;
    for (int32_t i = 0; i < n && r >= 0; i++) r = blosc2_schunk_append_buffer(schunk, h + (int64_t)i * src_stride, nbytes[i]);
    return r;
  }
  if (rc < 0) {
    for (uint8_t* c : chunks) free(c);
    return rc;
  }
  int64_t r = schunk->nchunks;
  for (int32_t i = 0; i < n; i++) {
    r = blosc2_schunk_append_chunk(schunk, chunks[i], false);
    if (r < 0) {
      // chunks [0, i) stay appended (include/b2h.h); the context is left where the serial calls
      // would have left it after chunk i - 1
      for (int32_t j = i; j < n; j++) free(chunks[j]);
      b2h::ctx_set_blocksize(schunk->cctx, before[i]);
      return r;
    }
  }
  b2h::ctx_set_blocksize(schunk->cctx, before[n]);
  return r;
}

namespace {

// A decode worker's staging, kept per device between calls (pinned allocations of a few hundred
// MiB cost tens of ms each): two input slots (packed compressed chunks in pinned and device memory,
// with the batch's pointer / size tables), two device output slots, three pinned output slots with
// their status words, a stream per direction plus the compute stream, the events that order them,
// and the engine workspace.
struct DecodeStage {
  int device = -1;
  size_t in_cap = 0, out_cap = 0, tab_cap = 0;
  uint8_t *pin_in[2] = {}, *dev_in[2] = {}, *pin_tab[2] = {}, *dev_tab[2] = {}, *dev_out[2] = {};
  uint8_t* pin_out[3] = {};
  int32_t* pin_st[3] = {};
  hipStream_t s_in = nullptr, s_out = nullptr, s_k = nullptr;
  hipEvent_t e_in[2] = {}, e_dec[2] = {}, e_dout[2] = {}, e_out[3] = {};
  b2h::Workspace* ws = nullptr;
  b2h::ReadBuf hold[2] = {b2h::ReadBuf(true), b2h::ReadBuf(true)};   // chunks read off a frame file
  bool init() {
    auto ev = [](hipEvent_t* e) { return hipEventCreateWithFlags(e, hipEventDisableTiming) == hipSuccess; };
    if (hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&s_k, hipStreamNonBlocking) != hipSuccess)
      return false;
    for (int i = 0; i < 2; i++)
      if (!ev(&e_in[i]) || !ev(&e_dec[i]) || !ev(&e_dout[i])) return false;
    for (int i = 0; i < 3; i++)
      if (!ev(&e_out[i])) return false;
    ws = b2h::workspace_create();
    return ws != nullptr;
  }
  static bool grow_pin(uint8_t** p, size_t n) {
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    return hipHostMalloc(reinterpret_cast<void**>(p), n, hipHostMallocDefault) == hipSuccess;
  }
  static bool grow_dev(uint8_t** p, size_t n) {
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    return hipMalloc(reinterpret_cast<void**>(p), n) == hipSuccess;
  }
  // Frees every slot and zeroes the capacities: after a failed grow some slots are freed or null,
  // and a stage going back to the pool must not claim room it no longer has.
  void drop() {
    for (int i = 0; i < 2; i++) {
      for (uint8_t** p : {&pin_in[i], &pin_tab[i]}) {
        if (*p) (void)hipHostFree(*p);
        *p = nullptr;
      }
      for (uint8_t** p : {&dev_in[i], &dev_tab[i], &dev_out[i]}) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
      }
    }
    for (int i = 0; i < 3; i++) {
      if (pin_out[i]) (void)hipHostFree(pin_out[i]);
      if (pin_st[i]) (void)hipHostFree(pin_st[i]);
      pin_out[i] = nullptr;
      pin_st[i] = nullptr;
    }
    in_cap = out_cap = tab_cap = 0;
  }
  bool ensure(size_t in, size_t out, size_t tab) {   // (an idle stage has nothing in flight)
    auto fail = [&] {
      drop();
      return false;
    };
    if (in > in_cap) {
      for (int i = 0; i < 2; i++)
        if (!grow_pin(&pin_in[i], in) || !grow_dev(&dev_in[i], in)) return fail();
      in_cap = in;
    }
    if (out > out_cap) {
      for (int i = 0; i < 2; i++)
        if (!grow_dev(&dev_out[i], out)) return fail();
      for (int i = 0; i < 3; i++)
        if (!grow_pin(&pin_out[i], out)) return fail();
      out_cap = out;
    }
    if (tab > tab_cap) {
      for (int i = 0; i < 2; i++)
        if (!grow_pin(&pin_tab[i], tab) || !grow_dev(&dev_tab[i], tab)) return fail();
      for (int i = 0; i < 3; i++)
        if (!grow_pin(reinterpret_cast<uint8_t**>(&pin_st[i]), tab)) return fail();
      tab_cap = tab;
    }
    return true;
  }
};

std::mutex g_stage_mu;
std::vector<DecodeStage*> g_stages;   // idle stages, any device

DecodeStage* stage_acquire(int device) {
  {
    std::lock_guard<std::mutex> g(g_stage_mu);
    for (size_t i = 0; i < g_stages.size(); i++) {
      if (g_stages[i]->device != device) continue;
      DecodeStage* st = g_stages[i];
      g_stages.erase(g_stages.begin() + (long)i);
      return st;
    }
  }
  DecodeStage* st = new DecodeStage();
  st->device = device;
  if (!st->init()) {
    delete st;   // (its streams / events leak: a failed init means a broken device anyway)
    return nullptr;
  }
  return st;
}

void stage_release(DecodeStage* st) {
  std::lock_guard<std::mutex> g(g_stage_mu);
  g_stages.push_back(st);
}

// Host copies of many separate chunks into one packed buffer, split over a few threads.
void par_pack(uint8_t* dst, const std::vector<int64_t>& at, const std::vector<const uint8_t*>& src,
              const std::vector<int32_t>& len, int64_t total) {
  const int n = (int)src.size();
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>({8, total >> 23, n}));
  auto part = [&](int t) {
    for (int i = n * t / T; i < n * (t + 1) / T; i++) memcpy(dst + at[(size_t)i], src[(size_t)i], (size_t)len[(size_t)i]);
  };
  if (T == 1) return part(0);
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
}

// The staged decode of chunks [c0, c0 + n) of `schunk` on the current device, through `ctx` (a
// decompression context with the super-chunk's dparams), in groups of chunks through a pipeline
// whose stages each hold their own resource: (1) the host gathers group g + 1's chunks (reading
// them off the frame file for an attached handle) into a pinned slot and queues their H2D on the
// input stream; (2) the engine decodes group g on the compute stream -- into a device slot, or
// straight into `out_dev`; (3) the output stream brings the group's statuses (and, for host
// output, its bytes) back into a pinned slot; (4) a helper thread copies group g - 1 from pinned
// memory into `out_host`.  A group holding a chunk the device path does not take (user filters /
// codecs, a postfilter, a bad header, too small a destination) goes through ctx_decompress_device
// instead.  st[i] = what blosc2_schunk_decompress_chunk returns for chunk c0 + i.  Returns 0, the
// first chunk's error, or the pipeline's.
int staged_decode(blosc2_schunk* schunk, blosc2_context* ctx, int device, int64_t c0, int32_t n, uint8_t* out_host,
                  uint8_t* out_dev, int64_t dst_stride, int32_t dst_capacity, int32_t* st) {
  for (int32_t i = 0; i < n; i++) st[i] = BLOSC2_ERROR_FAILURE;
  const int32_t G = (int32_t)std::max<int64_t>(1, std::min<int64_t>(n, kGroupBytes / std::max<int64_t>(dst_stride, 1)));
  const int32_t ng = (n + G - 1) / G;
  auto lo = [&](int32_t g) { return g * G; };
  auto cnt = [&](int32_t g) { return std::min(G, n - lo(g)); };
  const size_t tab = (size_t)G * (8 + 8 + 4 + 4 + 4);
  const size_t in_cap = (size_t)G * ((size_t)dst_capacity + BLOSC2_MAX_OVERHEAD + 64);
  DecodeStage* S = stage_acquire(device);
  if (!S) return BLOSC2_ERROR_FAILURE;
  int r = S->ensure(in_cap, out_dev ? 0 : (size_t)G * (size_t)dst_stride, tab) ? 0 : BLOSC2_ERROR_MEMORY_ALLOC;
  std::vector<char> staged((size_t)ng, 0);   // per group: the device path took it
  std::vector<int32_t> nbs((size_t)n, 0);
  b2h::ReadBuf* hold = S->hold;
  std::vector<const uint8_t*> ptrs_of[2];      // a fallback group's chunks (held until it ran)
  auto dst_of = [&](int32_t g, int slot) {
    return out_dev ? out_dev + (int64_t)lo(g) * dst_stride : S->dev_out[slot];
  };
  auto prep = [&](int32_t g) -> int {   // (1)
    const int slot = g % 2;
    const int32_t m = cnt(g);
    if (hipEventSynchronize(S->e_dec[slot]) != hipSuccess) return BLOSC2_ERROR_FAILURE;   // group g - 2 left the slot
    std::vector<const uint8_t*>& ptrs = ptrs_of[slot];
    int rr = b2h::chunk_ptrs(schunk, c0 + lo(g), m, &ptrs, &hold[slot]);
    if (rr < 0) return rr;
    std::vector<int64_t> at((size_t)m);
    std::vector<int32_t> cbs((size_t)m);
    int64_t total = 0;
    bool ok = true;
    for (int32_t i = 0; i < m && ok; i++) {
      int32_t nb = 0, cb = 0;
      ok = ptrs[(size_t)i] && b2h::ctx_chunk_on_device(ctx, ptrs[(size_t)i], &nb, &cb) && nb <= dst_capacity && nb >= 0;
      nbs[(size_t)(lo(g) + i)] = nb;
      cbs[(size_t)i] = cb;
      at[(size_t)i] = total;
      total += ((int64_t)cb + 63) & ~int64_t(63);
    }
    staged[(size_t)g] = ok && (size_t)total <= S->in_cap;
    if (!staged[(size_t)g]) return 0;
    // chunks read off a frame file sit in the pinned read buffer already: its used span goes up
    // as it is, the chunks keep their places in it; anything else is packed into the pinned slot
    const uint8_t* hb = hold[slot].p;
    bool in_hold = hb != nullptr;
    int64_t span = 0;
    for (int32_t i = 0; i < m && in_hold; i++) {
      const uint8_t* c = ptrs[(size_t)i];
      in_hold = c >= hb && c + cbs[(size_t)i] <= hb + hold[slot].cap;
      if (in_hold) span = std::max<int64_t>(span, (c - hb) + cbs[(size_t)i]);
    }
    in_hold = in_hold && (size_t)span <= S->in_cap;
    const uint8_t* h2d_src = S->pin_in[slot];
    if (in_hold) {
      for (int32_t i = 0; i < m; i++) at[(size_t)i] = ptrs[(size_t)i] - hb;
      h2d_src = hb;
      total = span;
    } else {
      par_pack(S->pin_in[slot], at, ptrs, cbs, total);
    }
    uint8_t* t = S->pin_tab[slot];
    const uint8_t** h_s = reinterpret_cast<const uint8_t**>(t);
    uint8_t** h_d = reinterpret_cast<uint8_t**>(t + 8 * (size_t)m);
    int32_t* h_ss = reinterpret_cast<int32_t*>(t + 16 * (size_t)m);
    int32_t* h_ds = h_ss + m;
    uint8_t* base = dst_of(g, slot);
    for (int32_t i = 0; i < m; i++) {
      h_s[i] = S->dev_in[slot] + at[(size_t)i];
      h_d[i] = base + (int64_t)i * dst_stride;
      h_ss[i] = cbs[(size_t)i];
      h_ds[i] = dst_capacity;
    }
    if (hipMemcpyAsync(S->dev_in[slot], h2d_src, (size_t)total, hipMemcpyHostToDevice, S->s_in) != hipSuccess ||
        hipMemcpyAsync(S->dev_tab[slot], t, 24 * (size_t)m, hipMemcpyHostToDevice, S->s_in) != hipSuccess ||
        hipEventRecord(S->e_in[slot], S->s_in) != hipSuccess)
      return BLOSC2_ERROR_FAILURE;
    ptrs.clear();   // packed: the chunk bytes are no longer needed
    return 0;
  };
  auto run = [&](int32_t g) -> int {   // (2) + (3)
    const int slot = g % 2, o = g % 3;
    const int32_t m = cnt(g);
    uint8_t* d_out = dst_of(g, slot);
    if (staged[(size_t)g]) {
      uint8_t* dt = S->dev_tab[slot];
      const uint8_t* const* d_s = reinterpret_cast<const uint8_t* const*>(dt);
      uint8_t* const* d_d = reinterpret_cast<uint8_t* const*>(dt + 8 * (size_t)m);
      const int32_t* d_ss = reinterpret_cast<const int32_t*>(dt + 16 * (size_t)m);
      int32_t* d_st = const_cast<int32_t*>(d_ss) + 2 * m;
      int64_t bound = 0;
      for (int32_t i = 0; i < m; i++) bound += nbs[(size_t)(lo(g) + i)];
      if (hipStreamWaitEvent(S->s_k, S->e_in[slot], 0) != hipSuccess ||
          (!out_dev && hipStreamWaitEvent(S->s_k, S->e_dout[slot], 0) != hipSuccess))
        return BLOSC2_ERROR_FAILURE;
      const int rr = b2h::decompress_batch(d_s, d_ss, d_d, d_ss + m, m, bound, d_st, nullptr, S->s_k, S->ws,
                                           (int64_t)S->in_cap, 0);
      if (rr < 0) return rr;
      if (hipEventRecord(S->e_dec[slot], S->s_k) != hipSuccess ||
          hipStreamWaitEvent(S->s_out, S->e_dec[slot], 0) != hipSuccess ||
          hipMemcpyAsync(S->pin_st[o], d_st, 4 * (size_t)m, hipMemcpyDeviceToHost, S->s_out) != hipSuccess)
        return BLOSC2_ERROR_FAILURE;
    } else {
      // the context path (synchronous): a device slot's previous output must have left first
      if (!out_dev && hipEventSynchronize(S->e_dout[slot]) != hipSuccess) return BLOSC2_ERROR_FAILURE;
      const int rr = b2h::ctx_decompress_device(ctx, ptrs_of[slot].data(), m, d_out, dst_stride, dst_capacity,
                                                st + lo(g));
      if (rr < 0) {
        bool chunk_error = false;   // a chunk's own error is in st[]; anything else stops the pipeline
        for (int32_t i = 0; i < m; i++) chunk_error |= st[lo(g) + i] == rr;
        if (!chunk_error) return rr;
      }
      ptrs_of[slot].clear();
    }
    if (!out_dev &&
        (hipMemcpyAsync(S->pin_out[o], d_out, (size_t)m * (size_t)dst_stride, hipMemcpyDeviceToHost, S->s_out) != hipSuccess ||
         hipEventRecord(S->e_dout[slot], S->s_out) != hipSuccess))
      return BLOSC2_ERROR_FAILURE;
    return hipEventRecord(S->e_out[o], S->s_out) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  };
  auto unstage = [&](int32_t g) -> int {   // (4)
    const int o = g % 3;
    if (hipEventSynchronize(S->e_out[o]) != hipSuccess) return BLOSC2_ERROR_FAILURE;
    if (staged[(size_t)g]) {
      for (int32_t i = 0; i < cnt(g); i++) {   // schunk.c:1511-1517
        const int32_t v = S->pin_st[o][i], nb = nbs[(size_t)(lo(g) + i)];
        st[lo(g) + i] = v < 0 ? v : (v != nb ? BLOSC2_ERROR_FAILURE : v);
      }
    }
    if (out_host) par_copy(out_host + (int64_t)lo(g) * dst_stride, dst_stride, S->pin_out[o], dst_stride, cnt(g), dst_capacity);
    return 0;
  };
  int behind_rc = 0;
  std::thread behind;
  if (r == 0) r = prep(0);
  for (int32_t g = 0; g < ng && r == 0; g++) {
    int ahead_rc = 0;
    std::thread ahead;
    if (g + 1 < ng) ahead = std::thread([&, g] { ahead_rc = prep(g + 1); });
    r = run(g);
    if (behind.joinable()) behind.join();   // group g - 1's copy-out: pinned slot (g + 2) % 3 is free
    if (r == 0 && behind_rc) r = behind_rc;
    if (r == 0) behind = std::thread([&, g] { behind_rc = unstage(g); });
    if (ahead.joinable()) ahead.join();
    if (r == 0 && ahead_rc) r = ahead_rc;
  }
  if (behind.joinable()) behind.join();
  if (r == 0 && behind_rc) r = behind_rc;
  (void)hipStreamSynchronize(S->s_in);
  (void)hipStreamSynchronize(S->s_k);
  (void)hipStreamSynchronize(S->s_out);
  stage_release(S);
  for (int32_t i = 0; i < n && r == 0; i++)
    if (st[i] < 0) r = st[i];
  return r;
}

}  // namespace

// Each worker decodes its contiguous range with staged_decode (above) on its device.
int b2h_schunk_decompress_buffers(blosc2_schunk* schunk, int64_t nchunk, int32_t n, void* dst, int64_t dst_stride,
                                  int32_t dst_capacity, int32_t* status, int32_t ndevices) {
  if (!schunk || (n > 0 && !dst)) return BLOSC2_ERROR_NULL_POINTER;
  if (n < 0 || nchunk < 0 || nchunk + n > schunk->nchunks || dst_capacity < 0 || dst_stride < dst_capacity) {
    TRACE_ERROR("chunks [%lld, %lld) are outside the super-chunk (%lld chunks) or the strides do not fit",
                (long long)nchunk, (long long)(nchunk + n), (long long)schunk->nchunks);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  if (n == 0) return 0;
  const int W = fanout_workers(ndevices, n);
  if (W == 0) {
    TRACE_ERROR("no HIP device available: the MI355X engine has no CPU fallback");
    return BLOSC2_ERROR_FAILURE;
  }
  uint8_t* out = static_cast<uint8_t*>(dst);
  blosc2_dparams dp;
  int rc = blosc2_ctx_get_dparams(schunk->dctx, &dp);
  if (rc < 0) return rc;
  std::vector<int32_t> st((size_t)n, BLOSC2_ERROR_FAILURE);
  std::vector<int> wrc((size_t)W, 0);
  auto work = [&](int k) {
    const int32_t i0 = (int32_t)((int64_t)n * k / W), i1 = (int32_t)((int64_t)n * (k + 1) / W);
    if (i1 <= i0) return;
    const int device = k % b2h::device_count();
    if (hipSetDevice(device) != hipSuccess) { wrc[k] = BLOSC2_ERROR_FAILURE; return; }
    blosc2_context* ctx = blosc2_create_dctx(dp);
    if (!ctx) { wrc[k] = BLOSC2_ERROR_MEMORY_ALLOC; return; }
    wrc[k] = staged_decode(schunk, ctx, device, nchunk + i0, i1 - i0, out + (int64_t)i0 * dst_stride, nullptr,
                           dst_stride, dst_capacity, st.data() + i0);
    blosc2_free_ctx(ctx);
  };
  std::vector<std::thread> th;
  for (int k = 0; k < W; k++) th.emplace_back(work, k);
  for (auto& t : th) t.join();
  rc = 0;
  for (int k = 0; k < W && rc == 0; k++) rc = wrc[k];
  if (status) memcpy(status, st.data(), sizeof(int32_t) * (size_t)n);
  schunk->current_nchunk = nchunk + n - 1;
  return rc;
}

// ------------------------------------------------------------------------ slice writes ----
namespace {
// The chunk walk of blosc2_schunk_set_slice_buffer (schunk.c:2146-2216): chunk k takes the range's
// bytes [lo, hi) of it; `whole` chunks are compressed straight from the caller's bytes with `n`
// = the byte count the reference compresses, the others are decompressed, patched and recompressed.
// Quirk kept: a range that starts a chunk and ends nbytes % chunksize bytes into it counts as a
// whole chunk of that many bytes, even in the middle of the super-chunk, where the chunk then
// shrinks (the reference's `chunksize` local, 2165-2172).
struct SliceStep {
  int64_t k;
  int32_t lo, hi, n;
  bool whole;
};
std::vector<SliceStep> slice_walk(const blosc2_schunk* s, int64_t b0, int64_t b1) {
  std::vector<SliceStep> v;
  const int64_t cs = s->chunksize;
  int64_t k = b0 / cs;
  int32_t lo = (int32_t)(b0 % cs), hi = b1 >= (k + 1) * cs ? (int32_t)cs : (int32_t)(b1 % cs);
  int32_t csz = (int32_t)cs;
  for (int64_t done = 0; done < b1 - b0;) {
    const int32_t tail = (int32_t)(s->nbytes % cs);
    SliceStep st{k, lo, hi, 0, lo == 0 && (hi == cs || hi == tail)};
    if (st.whole && hi == tail) csz = hi;
    st.n = st.whole ? csz : 0;
    v.push_back(st);
    done += hi - lo;
    k++;
    lo = 0;
    hi = b1 >= (k + 1) * cs ? (int32_t)cs : (int32_t)(b1 % cs);
  }
  return v;
}

int check_slice(const blosc2_schunk* s, int64_t start, int64_t stop) {
  const int64_t ts = s->typesize;
  if (start < 0 || stop < start || ts <= 0 || stop * ts > s->nbytes || s->chunksize <= 0) {
    TRACE_ERROR("slice [%lld, %lld) is outside the super-chunk (or the super-chunk has no fixed chunksize)",
                (long long)start, (long long)stop);
    return BLOSC2_ERROR_INVALID_PARAM;
  }
  return 0;
}

// One chunk of the walk from host bytes `src` (the range's bytes for this chunk).
int set_one(blosc2_schunk* s, const SliceStep& st, const uint8_t* src, std::vector<uint8_t>& data) {
  uint8_t* chunk;
  if (st.whole) {
    chunk = static_cast<uint8_t*>(malloc((size_t)st.n + BLOSC2_MAX_OVERHEAD));
    if (!chunk) return BLOSC2_ERROR_MEMORY_ALLOC;
    if (blosc2_compress_ctx(s->cctx, src, st.n, chunk, st.n + BLOSC2_MAX_OVERHEAD) < 0) {
      TRACE_ERROR("Cannot compress data of chunk ('%lld').", (long long)st.k);
      free(chunk);
      return BLOSC2_ERROR_FAILURE;
    }
  } else {
    data.resize((size_t)s->chunksize);
    const int got = blosc2_schunk_decompress_chunk(s, st.k, data.data(), s->chunksize);
    if (got < 0) {
      TRACE_ERROR("Cannot decompress chunk ('%lld').", (long long)st.k);
      return BLOSC2_ERROR_FAILURE;
    }
    memcpy(data.data() + st.lo, src, (size_t)(st.hi - st.lo));
    chunk = static_cast<uint8_t*>(malloc((size_t)got + BLOSC2_MAX_OVERHEAD));
    if (!chunk) return BLOSC2_ERROR_MEMORY_ALLOC;
    if (blosc2_compress_ctx(s->cctx, data.data(), got, chunk, got + BLOSC2_MAX_OVERHEAD) < 0) {
      TRACE_ERROR("Cannot compress data of chunk ('%lld').", (long long)st.k);
      free(chunk);
      return BLOSC2_ERROR_FAILURE;
    }
  }
  if (blosc2_schunk_update_chunk(s, st.k, chunk, false) != s->nchunks) {
    TRACE_ERROR("Cannot update chunk ('%lld').", (long long)st.k);
    free(chunk);
    return BLOSC2_ERROR_CHUNK_UPDATE;
  }
  return 0;
}
}  // namespace

int blosc2_schunk_set_slice_buffer(blosc2_schunk* schunk, int64_t start, int64_t stop, void* buffer) {
  if (!schunk || !buffer) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "blosc2_schunk_set_slice_buffer")) return rc0;
  int rc = check_slice(schunk, start, stop);
  if (rc < 0) return rc;
  const uint8_t* src = static_cast<const uint8_t*>(buffer);
  std::vector<uint8_t> data;
  for (const SliceStep& st : slice_walk(schunk, start * schunk->typesize, stop * schunk->typesize)) {
    if ((rc = set_one(schunk, st, src, data)) < 0) return rc;
    src += st.hi - st.lo;
  }
  return BLOSC2_ERROR_SUCCESS;
}

// The same walk from device bytes: each run of whole chunks is compressed by one device batch on the
// super-chunk's cctx (ctx_append_device, the sticky blocksize carried as the serial calls carry it),
// then updated in order; the (at most two) edge chunks go through the host walk above.
int b2h_schunk_set_slice_device(blosc2_schunk* schunk, int64_t start, int64_t stop, const void* d_src) {
  if (!schunk || !d_src) return BLOSC2_ERROR_NULL_POINTER;
  if (int rc0 = refuse_if_attached(schunk, "b2h_schunk_set_slice_device")) return rc0;
  int rc = check_slice(schunk, start, stop);
  if (rc < 0) return rc;
  const uint8_t* src = static_cast<const uint8_t*>(d_src);
  const std::vector<SliceStep> walk = slice_walk(schunk, start * schunk->typesize, stop * schunk->typesize);
  std::vector<uint8_t> data, piece;
  int64_t off = 0;
  for (size_t i = 0; i < walk.size();) {
    if (!walk[i].whole) {
      const SliceStep& st = walk[i];
      piece.resize((size_t)(st.hi - st.lo));
      if (hipMemcpy(piece.data(), src + off, piece.size(), hipMemcpyDeviceToHost) != hipSuccess) return BLOSC2_ERROR_FAILURE;
      if ((rc = set_one(schunk, st, piece.data(), data)) < 0) return rc;
      off += st.hi - st.lo;
      i++;
      continue;
    }
    size_t j = i;
    std::vector<int32_t> sizes;
    for (; j < walk.size() && walk[j].whole; j++) sizes.push_back(walk[j].n);
    // the whole chunks of a run sit back to back in the range, chunksize apart
    std::vector<uint8_t*> chunks(sizes.size(), nullptr);
    rc = b2h::ctx_append_device(schunk->cctx, src + off, sizes.data(), (int32_t)sizes.size(), schunk->chunksize,
                                chunks.data());
    if (rc == BLOSC2_ERROR_FILTER_PIPELINE) {   // user filters / codecs: the host walk
      for (; i < j; i++) {
        piece.resize((size_t)walk[i].n);
        if (hipMemcpy(piece.data(), src + off, piece.size(), hipMemcpyDeviceToHost) != hipSuccess)
          return BLOSC2_ERROR_FAILURE;
        if ((rc = set_one(schunk, walk[i], piece.data(), data)) < 0) return rc;
        off += walk[i].hi - walk[i].lo;
      }
      continue;
    }
    if (rc < 0) return rc;
    for (size_t q = 0; i < j; i++, q++) {
      if (blosc2_schunk_update_chunk(schunk, walk[i].k, chunks[q], false) != schunk->nchunks) {
        for (size_t r = q; r < chunks.size(); r++) free(chunks[r]);
        return BLOSC2_ERROR_CHUNK_UPDATE;
      }
      off += walk[i].hi - walk[i].lo;
    }
  }
  return BLOSC2_ERROR_SUCCESS;
}
