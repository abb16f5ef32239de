// b2h_frame.cpp -- contiguous-frame read path on the MI355X engine.
//
// The reference reads a frame chunk by chunk: blosc2_schunk_decompress_chunk -> frame_decompress_chunk
// (blosc/frame.c:5248-5290) -> frame_get_chunk (3378-3480) -> get_coffset (3283-3318, the offsets
// index is itself a Blosc chunk read with blosc2_getitem) -> a read through the stdio backend
// (blosc/blosc2-stdio.c:241-276) -> blosc2_decompress_ctx.  Here the whole frame is read once into
// pinned host memory, copied to HBM in one transfer, the offsets chunk is decoded on the device,
// and every data chunk of the frame goes through ONE device decompression batch.
//
// Supported: contiguous frames (frame_type 0) of format version <= 3 with 64-bit offsets and
// regular (non-VL) blocks, whose chunks use the device pipeline (BloscLZ, built-in and plugin
// filters).  Special offsets (runs of zeros / NaNs / uninitialised values, frame.c:3320-3365)
// are materialised with fills.  Frame layout: README_CFRAME_FORMAT.rst.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/b2h.h"
#include "../../include/blosc2.h"
#include "b2h_engine.h"

namespace {

// Field offsets of the msgpack header (blosc/frame.h:29-49).
constexpr int kMagic = 2, kHeaderLen = 11, kFrameLen = 16, kFlags = 25, kType = 26, kCodecs = 27,
              kNbytes = 30, kCbytes = 39, kTypesize = 48, kBlocksize = 53, kChunksize = 58,
              kFilters = 70, kHeaderMin = 87, kChunkHdr = 32;
constexpr int kFrameFormatMax = 3;   // BLOSC2_VERSION_FRAME_FORMAT (include/blosc2.h:159)

int64_t be(const uint8_t* p, int n) {   // big-endian msgpack integers (frame.c from_big)
  uint64_t v = 0;
  for (int i = 0; i < n; i++) v = (v << 8) | p[i];
  if (n == 4) return (int64_t)(int32_t)(uint32_t)v;
  return (int64_t)v;
}
int32_t le32(const uint8_t* p) { int32_t v; memcpy(&v, p, 4); return v; }

__global__ void k_fill_pattern(uint8_t* dst, int64_t nbytes, uint64_t pattern, int width) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (uint8_t)(pattern >> (8 * (i % width)));
}

}  // namespace

struct b2h_frame {
  uint8_t* host = nullptr;      // pinned copy of the whole frame
  int64_t len = 0;
  uint8_t* dev = nullptr;       // HBM copy (uploaded on first use)
  int32_t header_len = 0;
  int64_t nbytes = 0, cbytes = 0, nchunks = 0;
  int32_t typesize = 0, blocksize = 0, chunksize = 0;
  uint8_t compcode = 0, clevel = 0;
  uint8_t filters[6] = {0}, filters_meta[6] = {0};
  std::vector<int64_t> offsets;  // per chunk: >= 0 offset from the header start, < 0 special
  hipStream_t stream = nullptr;
  b2h::Workspace* ws = nullptr;  // the frame's own engine scratch (stream-ordered on `stream`)
};

namespace {

void frame_release(b2h_frame* f) {
  if (!f) return;
  if (f->stream) (void)hipStreamSynchronize(f->stream);
  b2h::workspace_destroy(f->ws);
  if (f->host) (void)hipHostFree(f->host);
  if (f->dev) (void)hipFree(f->dev);
  if (f->stream) (void)hipStreamDestroy(f->stream);
  delete f;
}

int32_t chunk_nbytes(const b2h_frame* f, int64_t i) {
  if (i == f->nchunks - 1 && f->chunksize > 0 && f->nbytes % f->chunksize) return (int32_t)(f->nbytes % f->chunksize);
  return f->chunksize;
}

int upload(b2h_frame* f) {
  if (f->dev) return 0;
  if (hipMalloc(&f->dev, (size_t)f->len) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  if (hipMemcpyAsync(f->dev, f->host, (size_t)f->len, hipMemcpyHostToDevice, f->stream) != hipSuccess)
    return BLOSC2_ERROR_FAILURE;
  return 0;
}

// Decode `n` chunks of the frame (device copy) into device outputs; status per chunk.
// With `masks` (n * mask_stride bytes, nonzero = skip the block), only the unmasked blocks of each
// chunk are decoded (blosc2_set_maskout per chunk, blosc/blosc2.c:1734-1737).
int decode_chunks(b2h_frame* f, const std::vector<int64_t>& idx, const std::vector<uint8_t*>& outs,
                  const std::vector<int32_t>& caps, std::vector<int32_t>* status,
                  const std::vector<uint8_t>* masks = nullptr, int32_t mask_stride = 0) {
  const int32_t n = (int32_t)idx.size();
  if (n == 0) return 0;
  std::vector<const uint8_t*> srcs(n);
  std::vector<int32_t> sizes(n);
  int64_t bound = 0;
  for (int32_t k = 0; k < n; k++) {
    const int64_t pos = f->header_len + f->offsets[idx[k]];
    srcs[k] = f->dev + pos;
    sizes[k] = le32(f->host + pos + 12);   // the chunk's own cbytes field
    if (sizes[k] < 16 || pos + sizes[k] > f->header_len + f->cbytes) return BLOSC2_ERROR_INVALID_HEADER;
    bound += caps[k];
  }
  void* blob = nullptr;
  const size_t mask_bytes = masks ? masks->size() : 0;
  const size_t bytes = (size_t)n * (2 * sizeof(void*) + 3 * sizeof(int32_t)) + mask_bytes;
  if (hipMalloc(&blob, bytes) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  uint8_t* b = static_cast<uint8_t*>(blob);
  const uint8_t** d_srcs = reinterpret_cast<const uint8_t**>(b);
  uint8_t** d_dsts = reinterpret_cast<uint8_t**>(b + (size_t)n * sizeof(void*));
  int32_t* d_sizes = reinterpret_cast<int32_t*>(b + (size_t)n * 2 * sizeof(void*));
  int32_t* d_caps = d_sizes + n;
  int32_t* d_status = d_caps + n;
  uint8_t* d_masks = masks ? reinterpret_cast<uint8_t*>(d_status + n) : nullptr;
  int rc = 0;
  if (masks && hipMemcpyAsync(d_masks, masks->data(), mask_bytes, hipMemcpyHostToDevice, f->stream) != hipSuccess)
    rc = BLOSC2_ERROR_FAILURE;
  if (hipMemcpyAsync(d_srcs, srcs.data(), n * sizeof(void*), hipMemcpyHostToDevice, f->stream) != hipSuccess ||
      hipMemcpyAsync(d_dsts, outs.data(), n * sizeof(void*), hipMemcpyHostToDevice, f->stream) != hipSuccess ||
      hipMemcpyAsync(d_sizes, sizes.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, f->stream) != hipSuccess ||
      hipMemcpyAsync(d_caps, caps.data(), n * sizeof(int32_t), hipMemcpyHostToDevice, f->stream) != hipSuccess) {
    rc = BLOSC2_ERROR_FAILURE;
  }
  int64_t src_bound = 0;
  for (int32_t k = 0; k < n; k++) src_bound += sizes[k];
  if (!rc) rc = b2h::decompress_batch(d_srcs, d_sizes, d_dsts, d_caps, n, bound, d_status, d_masks, f->stream, f->ws,
                                      src_bound, 0, mask_stride);
  status->assign(n, 0);
  if (!rc && hipMemcpyAsync(status->data(), d_status, n * sizeof(int32_t), hipMemcpyDeviceToHost, f->stream) != hipSuccess)
    rc = BLOSC2_ERROR_FAILURE;
  if (hipStreamSynchronize(f->stream) != hipSuccess && !rc) rc = BLOSC2_ERROR_FAILURE;
  (void)hipFree(blob);
  return rc;
}

// get_header_info (blosc/frame.c:895-1060) for an in-memory contiguous frame, then the offsets
// index (get_coffsets, 2102-2155) decoded on the device.
int parse(b2h_frame* f) {
  const uint8_t* h = f->host;
  if (f->len < kHeaderMin) return BLOSC2_ERROR_READ_BUFFER;
  if (h[0] < 0x90 || h[0] > 0x9f || memcmp(h + kMagic, "b2frame", 8) != 0) return BLOSC2_ERROR_INVALID_HEADER;
  if ((h[kType] & 0x0f) != 0) return BLOSC2_ERROR_FRAME_TYPE;                  // contiguous only
  if ((h[kFlags] & 0x0f) > kFrameFormatMax) return BLOSC2_ERROR_VERSION_SUPPORT;
  if (((h[kFlags] >> 4) & 3) != 1) return BLOSC2_ERROR_VERSION_SUPPORT;         // 64-bit offsets
  if (h[kFlags] & 0x80) return BLOSC2_ERROR_VERSION_SUPPORT;                    // VL blocks
  f->header_len = (int32_t)be(h + kHeaderLen, 4);
  const int64_t frame_len = be(h + kFrameLen, 8);
  if (f->header_len < kHeaderMin || f->header_len > frame_len || frame_len > f->len) return BLOSC2_ERROR_INVALID_HEADER;
  f->nbytes = be(h + kNbytes, 8);
  f->cbytes = be(h + kCbytes, 8);
  f->typesize = (int32_t)be(h + kTypesize, 4);
  f->blocksize = (int32_t)be(h + kBlocksize, 4);
  f->chunksize = (int32_t)be(h + kChunksize, 4);
  if (f->typesize <= 0 || f->nbytes < 0 || f->cbytes < 0) return BLOSC2_ERROR_INVALID_HEADER;
  f->compcode = h[kCodecs] & 0x0f;
  f->clevel = h[kCodecs] >> 4;
  const uint8_t nf = h[kFilters];
  if (nf > 6) return BLOSC2_ERROR_INVALID_HEADER;
  for (int i = 0; i < nf; i++) { f->filters[i] = h[kFilters + 1 + i]; f->filters_meta[i] = h[kFilters + 1 + 8 + i]; }
  if (f->nbytes == 0) { f->nchunks = 0; return 0; }
  if (f->chunksize <= 0) return BLOSC2_ERROR_VERSION_SUPPORT;                   // variable chunk sizes
  f->nchunks = f->nbytes / f->chunksize + (f->nbytes % f->chunksize ? 1 : 0);
  // offsets index: a Blosc chunk right after the data chunks
  const int64_t off_pos = (int64_t)f->header_len + f->cbytes;
  if (off_pos + kChunkHdr > f->len) return BLOSC2_ERROR_INVALID_HEADER;
  const int32_t off_nbytes = le32(h + off_pos + 4), off_cbytes = le32(h + off_pos + 12);
  if (off_nbytes != f->nchunks * 8 || off_cbytes < 16 || off_pos + off_cbytes > f->len) return BLOSC2_ERROR_INVALID_HEADER;
  int rc = upload(f);
  if (rc) return rc;
  uint8_t* d_off = nullptr;
  if (hipMalloc(&d_off, (size_t)off_nbytes) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  // decode the index chunk as a one-chunk batch (its offset relative to the header start is cbytes)
  f->offsets.assign(1, f->cbytes);
  std::vector<int32_t> st;
  rc = [&]() {
    // the index lies past the data section: widen the bounds check for this one call
    const int64_t saved = f->cbytes;
    f->cbytes = f->len - f->header_len;
    const int r = decode_chunks(f, {0}, {d_off}, {off_nbytes}, &st);
    f->cbytes = saved;
    return r;
  }();
  if (!rc && st[0] != off_nbytes) rc = st[0] < 0 ? st[0] : BLOSC2_ERROR_DATA;
  if (!rc) {
    f->offsets.resize((size_t)f->nchunks);
    if (hipMemcpy(f->offsets.data(), d_off, (size_t)off_nbytes, hipMemcpyDeviceToHost) != hipSuccess) rc = BLOSC2_ERROR_FAILURE;
  }
  (void)hipFree(d_off);
  if (rc) return rc;
  for (int64_t i = 0; i < f->nchunks; i++) {   // get_coffset bounds (frame.c:3297-3313)
    const int64_t o = f->offsets[i];
    if (o >= 0 && (f->header_len + o > f->header_len + f->cbytes - kChunkHdr || f->header_len + o > f->len - kChunkHdr))
      return BLOSC2_ERROR_INVALID_HEADER;
  }
  return 0;
}

b2h_frame* open_pinned(uint8_t* host, int64_t len, int* err) {
  b2h_frame* f = new b2h_frame();
  f->host = host;
  f->len = len;
  int rc = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  if (!rc) f->ws = b2h::workspace_create();
  if (!rc) rc = parse(f);
  if (rc) { frame_release(f); f = nullptr; }
  if (err) *err = rc;
  return f;
}

// Special offset (frame.c:3320-3365): byte 7 bit 7 set, kind in bits 0-2 of byte 7.
int fill_special(b2h_frame* f, int64_t special, uint8_t* d_dst, int32_t nbytes) {
  const int kind = (int)(((uint64_t)special >> 56) & 0x7);
  if (kind == BLOSC2_SPECIAL_ZERO) return hipMemsetAsync(d_dst, 0, (size_t)nbytes, f->stream) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  if (kind == BLOSC2_SPECIAL_UNINIT) return 0;
  if (kind == BLOSC2_SPECIAL_NAN) {   // set_nans (blosc/blosc2.c:1612-1636): f32 / f64 quiet NaN
    if (f->typesize != 4 && f->typesize != 8) return BLOSC2_ERROR_DATA;
    const uint64_t pat = f->typesize == 4 ? 0x7fc00000ull : 0x7ff8000000000000ull;
    k_fill_pattern<<<256, 256, 0, f->stream>>>(d_dst, nbytes, pat, f->typesize);
    return hipGetLastError() == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  }
  return BLOSC2_ERROR_DATA;
}

// Geometry of a stored chunk from its own header: blocksize, block count, and whether its
// pipeline holds DELTA (whose blocks >= 1 XOR with block 0, so block 0 is always decoded).
struct ChunkGeom { int32_t blocksize = 0, nblocks = 0; bool delta = false; };
ChunkGeom chunk_geom(const b2h_frame* f, int64_t i) {
  ChunkGeom g;
  const uint8_t* h = f->host + f->header_len + f->offsets[i];
  const int32_t nb = le32(h + 4), bs = le32(h + 8);
  if (bs <= 0 || nb <= 0) return g;
  g.blocksize = std::min(bs, nb);
  g.nblocks = nb / g.blocksize + (nb % g.blocksize ? 1 : 0);
  if ((h[2] & BLOSC_DOSHUFFLE) && (h[2] & BLOSC_DOBITSHUFFLE)) {
    for (int k = 0; k < 6; k++) g.delta |= h[16 + k] == BLOSC_DELTA;
  } else {
    g.delta = (h[2] & BLOSC_DODELTA) != 0;
  }
  return g;
}

// Unmask the blocks of chunk i holding bytes [a, b) (chunk-relative) in m[0 .. stride).
void unmask_range(const ChunkGeom& g, int64_t a, int64_t b, uint8_t* m) {
  if (g.blocksize <= 0) return;
  for (int64_t k = a / g.blocksize; k <= (b - 1) / g.blocksize && k < g.nblocks; k++) m[k] = 0;
  if (g.delta) m[0] = 0;
}

// out[dst[k] * ts + j] = scratch[src[k] + j]: the sparse reader's item gather.
__global__ void k_gather_items(const uint8_t* __restrict__ scratch, const int64_t* __restrict__ src,
                               const int64_t* __restrict__ dst, int64_t n, int32_t ts, uint8_t* __restrict__ out) {
  const int64_t total = n * ts;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / ts, j = i - k * ts;
    out[dst[k] * ts + j] = scratch[src[k] + j];
  }
}

}  // namespace

extern "C" {

b2h_frame* b2h_frame_from_buffer(const void* cframe, int64_t len, int* err) {
  if (!cframe || len <= 0) { if (err) *err = BLOSC2_ERROR_READ_BUFFER; return nullptr; }
  uint8_t* host = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&host), (size_t)len, hipHostMallocDefault) != hipSuccess) {
    if (err) *err = BLOSC2_ERROR_MEMORY_ALLOC;
    return nullptr;
  }
  memcpy(host, cframe, (size_t)len);
  return open_pinned(host, len, err);
}

// The stdio backend's read path (blosc/blosc2-stdio.c:241-276), one read of the whole file.
b2h_frame* b2h_frame_open(const char* urlpath, int* err) {
  FILE* fp = urlpath ? fopen(urlpath, "rb") : nullptr;
  if (!fp) { if (err) *err = BLOSC2_ERROR_FILE_OPEN; return nullptr; }
  int64_t len = -1;
  if (fseek(fp, 0, SEEK_END) == 0) len = (int64_t)ftell(fp);
  uint8_t* host = nullptr;
  int rc = len > 0 ? 0 : BLOSC2_ERROR_FILE_READ;
  if (!rc && (fseek(fp, 0, SEEK_SET) != 0 || hipHostMalloc(reinterpret_cast<void**>(&host), (size_t)len, hipHostMallocDefault) != hipSuccess))
    rc = BLOSC2_ERROR_MEMORY_ALLOC;
  if (!rc && fread(host, 1, (size_t)len, fp) != (size_t)len) rc = BLOSC2_ERROR_FILE_READ;
  fclose(fp);
  if (rc) {
    if (host) (void)hipHostFree(host);
    if (err) *err = rc;
    return nullptr;
  }
  return open_pinned(host, len, err);
}

void b2h_frame_free(b2h_frame* f) { frame_release(f); }

int b2h_frame_get_info(const b2h_frame* f, b2h_frame_info* info) {
  if (!f || !info) return BLOSC2_ERROR_NULL_POINTER;
  info->nbytes = f->nbytes;
  info->cbytes = f->cbytes;
  info->nchunks = f->nchunks;
  info->typesize = f->typesize;
  info->blocksize = f->blocksize;
  info->chunksize = f->chunksize;
  info->compcode = f->compcode;
  info->clevel = f->clevel;
  memcpy(info->filters, f->filters, 6);
  memcpy(info->filters_meta, f->filters_meta, 6);
  return 0;
}

int64_t b2h_frame_decompress(b2h_frame* f, void* d_dst, int64_t dst_capacity) {
  if (!f || (!d_dst && f->nbytes)) return BLOSC2_ERROR_NULL_POINTER;
  if (dst_capacity < f->nbytes) return BLOSC2_ERROR_WRITE_BUFFER;
  uint8_t* out = static_cast<uint8_t*>(d_dst);
  std::vector<int64_t> idx;
  std::vector<uint8_t*> outs;
  std::vector<int32_t> caps, st;
  int rc = 0;
  for (int64_t i = 0; i < f->nchunks && !rc; i++) {
    uint8_t* o = out + i * (int64_t)f->chunksize;
    if (f->offsets[i] < 0) {
      rc = fill_special(f, f->offsets[i], o, chunk_nbytes(f, i));
      continue;
    }
    idx.push_back(i);
    outs.push_back(o);
    caps.push_back(chunk_nbytes(f, i));
  }
  if (!rc) rc = decode_chunks(f, idx, outs, caps, &st);
  // the fills are queued on the frame's stream too: drained before returning on every path
  // (decode_chunks has nothing to wait for when every chunk is special)
  if (hipStreamSynchronize(f->stream) != hipSuccess && !rc) rc = BLOSC2_ERROR_FAILURE;
  if (rc) return rc;
  for (size_t k = 0; k < idx.size(); k++)
    if (st[k] != caps[k]) return st[k] < 0 ? st[k] : BLOSC2_ERROR_DATA;
  return f->nbytes;
}

int b2h_frame_decompress_chunk(b2h_frame* f, int64_t nchunk, void* dest, int32_t nbytes) {
  if (!f || !dest) return BLOSC2_ERROR_NULL_POINTER;
  if (nchunk < 0 || nchunk >= f->nchunks) return BLOSC2_ERROR_INVALID_PARAM;
  const int32_t need = chunk_nbytes(f, nchunk);
  if (nbytes < need) return BLOSC2_ERROR_WRITE_BUFFER;
  uint8_t* d_out = nullptr;
  if (hipMalloc(&d_out, (size_t)need) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  int rc = 0;
  std::vector<int32_t> st;
  if (f->offsets[nchunk] < 0) {
    rc = fill_special(f, f->offsets[nchunk], d_out, need);
  } else {
    rc = decode_chunks(f, {nchunk}, {d_out}, {need}, &st);
    if (!rc && st[0] != need) rc = st[0] < 0 ? st[0] : BLOSC2_ERROR_DATA;
  }
  if (!rc && hipMemcpyAsync(dest, d_out, (size_t)need, hipMemcpyDeviceToHost, f->stream) != hipSuccess) rc = BLOSC2_ERROR_FAILURE;
  if (hipStreamSynchronize(f->stream) != hipSuccess && !rc) rc = BLOSC2_ERROR_FAILURE;
  (void)hipFree(d_out);
  return rc ? rc : need;
}

// blosc2_schunk_get_slice_buffer (blosc/schunk.c:1662-1760): items [start, stop) of the frame into
// device memory.  The reference decodes chunks wholly inside the slice and getitem's the partial
// edge chunks (which decodes only the touched blocks).  Here the whole chunks decode straight into
// place and the (at most two) edge chunks decode only their touched blocks (plus block 0 under
// DELTA) into scratch, all in ONE device batch with per-chunk block masks; the edges are then
// copied in.
int b2h_frame_get_slice(b2h_frame* f, int64_t start, int64_t stop, void* d_dst) {
  if (!f || !d_dst) return BLOSC2_ERROR_NULL_POINTER;
  const int64_t ts = f->typesize > 0 ? f->typesize : 1;
  if (start < 0 || stop < start || stop * ts > f->nbytes) return BLOSC2_ERROR_INVALID_PARAM;
  if (stop == start) return 0;
  const int64_t b0 = start * ts, b1 = stop * ts, cs = f->chunksize;
  const int64_t c0 = b0 / cs, c1 = (b1 - 1) / cs;
  uint8_t* out = static_cast<uint8_t*>(d_dst);
  uint8_t* scratch = nullptr;
  if (hipMalloc(&scratch, (size_t)(2 * cs)) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  std::vector<int64_t> idx;
  std::vector<uint8_t*> outs;
  std::vector<int32_t> caps, st;
  struct Edge { uint8_t* from; uint8_t* to; int64_t n; };
  std::vector<Edge> edges;
  struct Part { int64_t a, b; bool whole; ChunkGeom g; };
  std::vector<Part> parts;
  int32_t stride = 0;
  int rc = 0;
  for (int64_t i = c0; i <= c1 && !rc; i++) {
    const int64_t lo = i * cs, n = chunk_nbytes(f, i);
    const int64_t a = std::max(b0, lo), b = std::min(b1, lo + n);
    const bool whole = a == lo && b == lo + n;
    if (f->offsets[i] < 0) {   // special chunk: fill the touched range directly
      rc = fill_special(f, f->offsets[i], out + (a - b0), (int32_t)(b - a));
      continue;
    }
    uint8_t* o = whole ? out + (lo - b0) : scratch + (i == c0 ? 0 : cs);
    if (!whole) edges.push_back({o + (a - lo), out + (a - b0), b - a});
    const ChunkGeom g = chunk_geom(f, i);
    stride = std::max(stride, g.nblocks);
    parts.push_back({a - lo, b - lo, whole, g});
    idx.push_back(i);
    outs.push_back(o);
    caps.push_back((int32_t)n);
  }
  std::vector<uint8_t> masks((size_t)stride * parts.size(), 0);
  bool any_masked = false;
  for (size_t k = 0; k < parts.size(); k++) {
    if (parts[k].whole || parts[k].g.blocksize <= 0) continue;
    uint8_t* m = masks.data() + k * (size_t)stride;
    memset(m, 1, (size_t)parts[k].g.nblocks);
    unmask_range(parts[k].g, parts[k].a, parts[k].b, m);
    any_masked = true;
  }
  if (!rc) rc = decode_chunks(f, idx, outs, caps, &st, any_masked ? &masks : nullptr, stride);
  for (size_t k = 0; !rc && k < idx.size(); k++)
    if (st[k] != caps[k]) rc = st[k] < 0 ? st[k] : BLOSC2_ERROR_DATA;
  for (const Edge& e : edges) {
    if (rc) break;
    if (hipMemcpyAsync(e.to, e.from, (size_t)e.n, hipMemcpyDeviceToDevice, f->stream) != hipSuccess) rc = BLOSC2_ERROR_FAILURE;
  }
  if (hipStreamSynchronize(f->stream) != hipSuccess && !rc) rc = BLOSC2_ERROR_FAILURE;
  (void)hipFree(scratch);
  return rc;
}

// blosc2_schunk_get_sparse_buffer (blosc/schunk.c:1921-2110): items at arbitrary coordinates, in
// coordinate order, into a host buffer.  The reference sorts the coordinates, groups them by
// (chunk, block) and decodes each touched block with blosc2_decompress_block_ctx on a thread pool
// (getitem per coordinate under DELTA).  Here every touched chunk of a group goes through ONE
// device batch with per-chunk block masks (only touched blocks, plus block 0 under DELTA, are
// decoded), and one gather kernel pulls the items.  Groups bound the scratch to ~1 GiB.
int b2h_frame_get_sparse_buffer(b2h_frame* f, int64_t ncoords, const int64_t* coords, void* buffer) {
  if (!f) return BLOSC2_ERROR_INVALID_PARAM;
  if (ncoords < 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (ncoords == 0) return BLOSC2_ERROR_SUCCESS;
  if (!coords || !buffer) return BLOSC2_ERROR_INVALID_PARAM;
  if (f->typesize <= 0 || f->chunksize <= 0 || f->blocksize <= 0) return BLOSC2_ERROR_INVALID_PARAM;
  if (f->chunksize % f->typesize || f->blocksize % f->typesize) return BLOSC2_ERROR_INVALID_PARAM;
  const int64_t ts = f->typesize, cs = f->chunksize, nitems = f->nbytes / ts, chunk_nitems = cs / ts;
  for (int64_t i = 0; i < ncoords; i++)
    if (coords[i] < 0 || coords[i] >= nitems) return BLOSC2_ERROR_INVALID_PARAM;
  // coordinate order sorted by chunk (stable: equal chunks keep the caller's order)
  std::vector<int64_t> order((size_t)ncoords);
  for (int64_t i = 0; i < ncoords; i++) order[(size_t)i] = i;
  std::stable_sort(order.begin(), order.end(),
                   [&](int64_t x, int64_t y) { return coords[x] / chunk_nitems < coords[y] / chunk_nitems; });
  const int64_t group_max = std::max<int64_t>(1, std::min<int64_t>(4096, (int64_t(1) << 30) / cs));
  uint8_t *scratch = nullptr, *d_out = nullptr;
  int64_t* d_idx = nullptr;
  int rc = 0;
  if (hipMalloc(&d_out, (size_t)(ncoords * ts)) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  size_t scratch_bytes = 0, idx_cap = 0;
  for (size_t pos = 0; pos < order.size() && !rc;) {
    // one group: up to group_max distinct chunks
    std::vector<int64_t> idx;
    std::vector<uint8_t*> outs;
    std::vector<int32_t> caps, st;
    std::vector<ChunkGeom> geo;
    std::vector<int64_t> src, dst;
    std::vector<int32_t> kof;                              // per item: decoded-chunk index, -1 special
    std::vector<int64_t> dslot;                            // per decoded chunk: its scratch slot
    std::vector<std::pair<int64_t, int64_t>> specials;   // (chunk, slot)
    size_t end = pos;
    int64_t nslots = 0;
    while (end < order.size()) {
      const int64_t c = coords[order[end]] / chunk_nitems;
      if (nslots == group_max) break;
      size_t e2 = end;
      while (e2 < order.size() && coords[order[e2]] / chunk_nitems == c) e2++;
      const int64_t slot = nslots++;
      int32_t kk = -1;
      if (f->offsets[c] < 0) {
        specials.push_back({c, slot});
      } else {
        kk = (int32_t)idx.size();
        idx.push_back(c);
        caps.push_back(chunk_nbytes(f, c));
        geo.push_back(chunk_geom(f, c));
        dslot.push_back(slot);
      }
      for (size_t k = end; k < e2; k++) {
        src.push_back(slot * cs + (coords[order[k]] % chunk_nitems) * ts);
        dst.push_back(order[k]);
        kof.push_back(kk);
      }
      end = e2;
    }
    if ((size_t)(nslots * cs) > scratch_bytes) {
      if (scratch) (void)hipFree(scratch);
      scratch_bytes = (size_t)(nslots * cs);
      if (hipMalloc(&scratch, scratch_bytes) != hipSuccess) { scratch = nullptr; rc = BLOSC2_ERROR_MEMORY_ALLOC; break; }
    }
    for (int64_t sl : dslot) outs.push_back(scratch + sl * cs);
    for (auto& sp : specials) {
      if (rc) break;
      rc = fill_special(f, f->offsets[sp.first], scratch + sp.second * cs, chunk_nbytes(f, sp.first));
    }
    int32_t stride = 0;
    for (auto& g : geo) stride = std::max(stride, g.nblocks);
    std::vector<uint8_t> masks((size_t)stride * idx.size(), 1);
    for (size_t q = 0; q < kof.size(); q++) {   // touched blocks, per decoded chunk
      if (kof[q] < 0) continue;                  // special chunk: filled whole
      const int64_t byte = src[q] % cs;
      unmask_range(geo[(size_t)kof[q]], byte, byte + ts, masks.data() + (size_t)kof[q] * (size_t)stride);
    }
    if (!rc) rc = decode_chunks(f, idx, outs, caps, &st, &masks, stride);
    for (size_t k = 0; !rc && k < idx.size(); k++)
      if (st[k] != caps[k]) rc = st[k] < 0 ? st[k] : BLOSC2_ERROR_FAILURE;
    const int64_t n = (int64_t)src.size();
    if (!rc && (size_t)(2 * n) > idx_cap) {
      if (d_idx) (void)hipFree(d_idx);
      idx_cap = (size_t)(2 * n);
      if (hipMalloc(reinterpret_cast<void**>(&d_idx), idx_cap * sizeof(int64_t)) != hipSuccess) {
        d_idx = nullptr;
        rc = BLOSC2_ERROR_MEMORY_ALLOC;
      }
    }
    if (!rc && (hipMemcpyAsync(d_idx, src.data(), (size_t)n * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
                hipMemcpyAsync(d_idx + n, dst.data(), (size_t)n * 8, hipMemcpyHostToDevice, f->stream) != hipSuccess))
      rc = BLOSC2_ERROR_FAILURE;
    if (!rc) {
      const int64_t total = n * ts;
      const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 4096));
      k_gather_items<<<grid, 256, 0, f->stream>>>(scratch, d_idx, d_idx + n, n, (int32_t)ts, d_out);
      if (hipGetLastError() != hipSuccess) rc = BLOSC2_ERROR_FAILURE;
    }
    // the host vectors of this group are re-used next round: drain the stream first
    if (hipStreamSynchronize(f->stream) != hipSuccess && !rc) rc = BLOSC2_ERROR_FAILURE;
    pos = end;
  }
  if (!rc && hipMemcpy(buffer, d_out, (size_t)(ncoords * ts), hipMemcpyDeviceToHost) != hipSuccess) rc = BLOSC2_ERROR_FAILURE;
  if (scratch) (void)hipFree(scratch);
  if (d_idx) (void)hipFree(d_idx);
  (void)hipFree(d_out);
  return rc;
}

}  // extern "C"

// ------------------------------------------------------------ frame -> super-chunk ----
namespace {

// One metalayer index (msgpack): be16 idx_size, 0xde map16 (be16 count), then per layer a fixstr
// name and 0xd2 + be32 offset of its content (0xc6 bin32: be32 length, bytes), offsets from `base`.
// `idx` is where idx_size sits: FRAME_IDX_SIZE (89) for the header metalayers (get_meta_from_header,
// blosc/frame.c:2388-2500), FRAME_TRAILER_VLMETALAYERS + 2 (4) for the trailer's vlmetalayers
// (get_vlmeta_from_trailer, 2591-2720).
int read_layers(const uint8_t* base, int64_t len, int64_t idx, int max, blosc2_metalayer** out, int* count) {
  int64_t pos = idx + 2 + 1 + 2;
  if (len < pos) return BLOSC2_ERROR_READ_BUFFER;
  const uint8_t* p = base + idx + 2;
  if (p[0] != 0xde) return BLOSC2_ERROR_DATA;
  const int n = (int)be(p + 1, 2);
  p += 3;
  if (n > max) return BLOSC2_ERROR_DATA;
  for (int k = 0; k < n; k++) {
    if (len < ++pos) return BLOSC2_ERROR_READ_BUFFER;
    if ((*p & 0xe0u) != 0xa0u) return BLOSC2_ERROR_DATA;
    const int nslen = *p & 0x1f;
    p++;
    if (len < (pos += nslen)) return BLOSC2_ERROR_READ_BUFFER;
    blosc2_metalayer* m = static_cast<blosc2_metalayer*>(calloc(1, sizeof(blosc2_metalayer)));
    if (!m) return BLOSC2_ERROR_MEMORY_ALLOC;
    out[k] = m;
    *count = k + 1;
    m->name = static_cast<char*>(malloc((size_t)nslen + 1));
    if (!m->name) return BLOSC2_ERROR_MEMORY_ALLOC;
    memcpy(m->name, p, (size_t)nslen);
    m->name[nslen] = '\0';
    p += nslen;
    if (len < (pos += 1 + 4)) return BLOSC2_ERROR_READ_BUFFER;
    if (*p != 0xd2) return BLOSC2_ERROR_DATA;
    const int64_t off = be(p + 1, 4);
    p += 5;
    if (off < 0 || off >= len) return BLOSC2_ERROR_DATA;
    if (len < off + 5) return BLOSC2_ERROR_READ_BUFFER;
    if (base[off] != 0xc6) return BLOSC2_ERROR_DATA;
    const int64_t clen = be(base + off + 1, 4);
    if (clen < 0) return BLOSC2_ERROR_DATA;
    if (len < off + 5 + clen) return BLOSC2_ERROR_READ_BUFFER;
    m->content_len = (int32_t)clen;
    m->content = static_cast<uint8_t*>(malloc(clen > 0 ? (size_t)clen : 1));
    if (!m->content) return BLOSC2_ERROR_MEMORY_ALLOC;
    if (clen > 0) memcpy(m->content, base + off + 5, (size_t)clen);
  }
  return 0;
}

// frame_to_schunk (blosc/frame.c:2941-3245): header fields -> cparams, every chunk into the
// in-memory index (special offsets become 32-byte special chunks, frame_special_chunk 3321-3365),
// counters, metalayers and vlmetalayers.  `copy` selects the reference's two flavours: a copy
// (storage not contiguous, cbytes = sum of the chunks, blocksize = the chunks' common one) or a
// frame-attached handle (contiguous, header cbytes and blocksize).  Either way the chunks live in
// host memory here; writes to the handle do not go back to the frame.
blosc2_schunk* schunk_from_frame(b2h_frame* f, bool copy, const char* urlpath) {
  const uint8_t* h = f->host;
  blosc2_cparams cp = BLOSC2_CPARAMS_DEFAULTS;
  cp.typesize = f->typesize;
  cp.clevel = f->clevel;
  cp.compcode = f->compcode == BLOSC_UDCODEC_FORMAT ? h[77] : f->compcode;   // FRAME_UDCODEC
  cp.compcode_meta = h[78];                                                    // FRAME_CODEC_META
  cp.splitmode = (h[28] & 0x03) + 1;                                           // FRAME_OTHER_FLAGS
  cp.use_dict = h[85] & 1;                                                     // FRAME_OTHER_FLAGS2
  cp.blocksize = f->blocksize;
  memcpy(cp.filters, f->filters, 6);
  memcpy(cp.filters_meta, f->filters_meta, 6);
  blosc2_dparams dp = BLOSC2_DPARAMS_DEFAULTS;
  blosc2_storage st = BLOSC2_STORAGE_DEFAULTS;
  st.contiguous = false;
  st.urlpath = nullptr;
  st.cparams = &cp;
  st.dparams = &dp;
  blosc2_schunk* s = blosc2_schunk_new(&st);
  if (!s) return nullptr;
  int rc = 0;
  int32_t common_bs = 0;
  for (int64_t i = 0; i < f->nchunks && rc >= 0; i++) {
    uint8_t special[BLOSC_EXTENDED_HEADER_LENGTH];
    uint8_t* c;
    if (f->offsets[i] >= 0) {
      c = f->host + f->header_len + f->offsets[i];
      const int32_t cb = le32(c + 12);
      if (cb < BLOSC_EXTENDED_HEADER_LENGTH || f->offsets[i] + cb > f->cbytes) rc = BLOSC2_ERROR_INVALID_HEADER;
    } else {
      blosc2_cparams scp = BLOSC2_CPARAMS_DEFAULTS;
      scp.typesize = f->typesize;
      scp.blocksize = f->blocksize;
      const uint64_t v = (uint64_t)f->offsets[i];
      const int32_t nb = chunk_nbytes(f, i);
      if (v & ((uint64_t)BLOSC2_SPECIAL_ZERO << 56)) rc = blosc2_chunk_zeros(scp, nb, special, sizeof special);
      else if (v & ((uint64_t)BLOSC2_SPECIAL_UNINIT << 56)) rc = blosc2_chunk_uninit(scp, nb, special, sizeof special);
      else if (v & ((uint64_t)BLOSC2_SPECIAL_NAN << 56)) rc = blosc2_chunk_nans(scp, nb, special, sizeof special);
      else rc = BLOSC2_ERROR_DATA;
      c = special;
    }
    if (rc < 0) break;
    const int32_t bs = le32(c + 8);
    common_bs = i == 0 ? bs : (common_bs == bs ? bs : 0);
    const int64_t r = blosc2_schunk_append_chunk(s, c, true);
    if (r < 0) rc = (int)r;
  }
  if (rc >= 0 && s->nbytes != f->nbytes) rc = BLOSC2_ERROR_INVALID_HEADER;
  if (rc >= 0 && f->nchunks > 0) s->flags2 = s->data[0][BLOSC2_CHUNK_BLOSC2_FLAGS2];
  s->current_nchunk = 0;
  if (rc >= 0) {
    s->chunksize = f->chunksize;
    if (copy) {
      s->blocksize = common_bs;   // cbytes: the appended chunks' sum already
    } else {
      s->cbytes = f->cbytes;
      s->blocksize = f->blocksize;
      s->storage->contiguous = true;
      if (urlpath) s->storage->urlpath = strdup(urlpath);
    }
  }
  int nm = 0;
  if (rc >= 0) {
    rc = read_layers(h, f->header_len, 89, BLOSC2_MAX_METALAYERS, s->metalayers, &nm);   // FRAME_IDX_SIZE
    s->nmetalayers = (uint16_t)nm;
  }
  if (rc >= 0 && f->len >= 25) {   // the trailer (frame_from_cframe, frame.c:1893-1910)
    const uint8_t* t = h + f->len - 25;   // FRAME_TRAILER_MINLEN
    const int64_t tlen = t[25 - 22 - 1] == 0xce ? be(t + 25 - 22, 4) : -1;
    if (tlen < 25 || tlen > f->len - kHeaderMin) {
      rc = BLOSC2_ERROR_READ_BUFFER;
    } else {
      const int64_t toff = f->nbytes > 0 ? f->len - tlen : f->header_len;   // get_trailer_offset
      if (toff < BLOSC_EXTENDED_HEADER_LENGTH || toff + tlen > f->len) {
        rc = BLOSC2_ERROR_READ_BUFFER;
      } else {
        int nv = 0;
        rc = read_layers(h + toff, tlen, 4, BLOSC2_MAX_VLMETALAYERS, s->vlmetalayers, &nv);   // FRAME_TRAILER_VLMETALAYERS + 2
        s->nvlmetalayers = (int16_t)nv;
      }
    }
  }
  if (rc < 0) {
    blosc2_schunk_free(s);
    return nullptr;
  }
  return s;
}

std::vector<uint8_t> read_file(const char* path, int64_t offset, int* err) {
  std::vector<uint8_t> v;
  FILE* fp = path ? fopen(path, "rb") : nullptr;
  if (!fp) { *err = BLOSC2_ERROR_FILE_OPEN; return v; }
  int64_t len = -1;
  if (fseek(fp, 0, SEEK_END) == 0) len = (int64_t)ftell(fp);
  if (len <= offset || offset < 0 || fseek(fp, (long)offset, SEEK_SET) != 0) {
    *err = BLOSC2_ERROR_FILE_READ;
  } else {
    v.resize((size_t)(len - offset));
    if (fread(v.data(), 1, v.size(), fp) != v.size()) { *err = BLOSC2_ERROR_FILE_READ; v.clear(); }
  }
  fclose(fp);
  return v;
}

}  // namespace

extern "C" {

// blosc2_schunk_from_buffer (blosc/schunk.c:731-750): a contiguous frame in memory.
blosc2_schunk* blosc2_schunk_from_buffer(uint8_t* cframe, int64_t len, bool copy) {
  if (!cframe || len < kHeaderMin || memcmp(cframe + kMagic, "b2frame", 8) != 0) return nullptr;
  int err = 0;
  b2h_frame* f = b2h_frame_from_buffer(cframe, len, &err);
  if (!f) return nullptr;
  blosc2_schunk* s = schunk_from_frame(f, copy, nullptr);
  frame_release(f);
  return s;
}

// blosc2_schunk_open_offset_udio (blosc/schunk.c:405-470) for the filesystem backend: the frame
// starting `offset` bytes into the file, attached (contiguous, urlpath kept).
blosc2_schunk* blosc2_schunk_open_offset_udio(const char* urlpath, int64_t offset, const blosc2_io* udio) {
  if (!urlpath) return nullptr;
  if (udio && udio->id != BLOSC2_IO_FILESYSTEM) return nullptr;   // user I/O backends: not in the engine
  int err = 0;
  std::vector<uint8_t> bytes = read_file(urlpath, offset, &err);
  if (err || bytes.size() < (size_t)kHeaderMin) return nullptr;
  b2h_frame* f = b2h_frame_from_buffer(bytes.data(), (int64_t)bytes.size(), &err);
  if (!f) return nullptr;
  blosc2_schunk* s = schunk_from_frame(f, false, urlpath);
  frame_release(f);
  return s;
}
blosc2_schunk* blosc2_schunk_open_udio(const char* urlpath, const blosc2_io* udio) {   // schunk.c:371-373
  return blosc2_schunk_open_offset_udio(urlpath, 0, udio);
}
blosc2_schunk* blosc2_schunk_open_offset(const char* urlpath, int64_t offset) {
  return blosc2_schunk_open_offset_udio(urlpath, offset, &BLOSC2_IO_DEFAULTS);
}
blosc2_schunk* blosc2_schunk_open(const char* urlpath) {
  return blosc2_schunk_open_offset_udio(urlpath, 0, &BLOSC2_IO_DEFAULTS);
}

}  // extern "C"
