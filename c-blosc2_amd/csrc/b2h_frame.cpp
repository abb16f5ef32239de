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
//
// The second half of the file is the reference's own frame API over super-chunks: read-only
// frame-attached handles (blosc2_schunk_open*, _from_buffer) whose chunks are read lazily through
// the frame's IO backend (b2h_io.cpp), and the frame writer (blosc2_schunk_to_buffer / _to_file /
// _append_file).
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/b2h.h"
#include "../../include/blosc2.h"
#include "b2h_engine.h"
#include "b2h_frame.h"

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

// out[i * 32 + j] = the j-th header byte of chunk i (zeros for a special offset).
__global__ void k_gather_hdrs(const uint8_t* __restrict__ frame, int32_t header_len, const int64_t* __restrict__ offsets,
                              int64_t n, uint8_t* __restrict__ out) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * 32; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = offsets[t >> 5];
    out[t] = o >= 0 ? frame[header_len + o + (t & 31)] : 0;
  }
}

__global__ void k_fill_pattern(uint8_t* dst, int64_t nbytes, uint64_t pattern, int width) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = (uint8_t)(pattern >> (8 * (i % width)));
}

}  // namespace

struct b2h_frame {
  uint8_t* host = nullptr;      // pinned host copy of the whole frame (from_buffer), or none (open)
  std::vector<uint8_t> chdr;    // per chunk: its 32-byte header (zeros for a special chunk)
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
    sizes[k] = le32(f->chdr.data() + idx[k] * kChunkHdr + 12);   // the chunk's own cbytes field
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

// get_header_info (blosc/frame.c:895-1060): the fixed part of a frame header (kHeaderMin bytes).
struct FrameHead {
  int32_t header_len = 0;
  int64_t frame_len = 0, nbytes = 0, cbytes = 0, nchunks = 0;
  int32_t typesize = 0, blocksize = 0, chunksize = 0;
  uint8_t compcode = 0, clevel = 0, udcodec = 0, codec_meta = 0, other = 0, other2 = 0;
  uint8_t filters[6] = {0}, filters_meta[6] = {0};
};

int parse_head(const uint8_t* h, FrameHead* H) {
  if (h[0] < 0x90 || h[0] > 0x9f || memcmp(h + kMagic, "b2frame", 8) != 0) return BLOSC2_ERROR_INVALID_HEADER;
  if ((h[kType] & 0x0f) != 0) return BLOSC2_ERROR_FRAME_TYPE;                  // contiguous only
  if ((h[kFlags] & 0x0f) > kFrameFormatMax) return BLOSC2_ERROR_VERSION_SUPPORT;
  if (((h[kFlags] >> 4) & 3) != 1) return BLOSC2_ERROR_VERSION_SUPPORT;         // 64-bit offsets
  if (h[kFlags] & 0x80) return BLOSC2_ERROR_VERSION_SUPPORT;                    // VL blocks
  H->header_len = (int32_t)be(h + kHeaderLen, 4);
  H->frame_len = be(h + kFrameLen, 8);
  if (H->header_len < kHeaderMin || H->header_len > H->frame_len) return BLOSC2_ERROR_INVALID_HEADER;
  H->nbytes = be(h + kNbytes, 8);
  H->cbytes = be(h + kCbytes, 8);
  H->typesize = (int32_t)be(h + kTypesize, 4);
  H->blocksize = (int32_t)be(h + kBlocksize, 4);
  H->chunksize = (int32_t)be(h + kChunksize, 4);
  if (H->typesize <= 0 || H->nbytes < 0 || H->cbytes < 0) return BLOSC2_ERROR_INVALID_HEADER;
  H->compcode = h[kCodecs] & 0x0f;
  H->clevel = h[kCodecs] >> 4;
  H->other = h[kFlags + 3];          // FRAME_OTHER_FLAGS
  H->udcodec = h[77];                // FRAME_UDCODEC
  H->codec_meta = h[78];             // FRAME_CODEC_META
  H->other2 = h[85];                 // FRAME_OTHER_FLAGS2
  const uint8_t nf = h[kFilters];
  if (nf > 6) return BLOSC2_ERROR_INVALID_HEADER;
  for (int i = 0; i < nf; i++) { H->filters[i] = h[kFilters + 1 + i]; H->filters_meta[i] = h[kFilters + 1 + 8 + i]; }
  if (H->nbytes == 0) { H->nchunks = 0; return 0; }
  if (H->chunksize == 0) { H->nchunks = -1; return 0; }   // variable chunk sizes: the offsets index tells
  if (H->chunksize < 0) return BLOSC2_ERROR_INVALID_HEADER;
  H->nchunks = H->nbytes / H->chunksize + (H->nbytes % H->chunksize ? 1 : 0);
  return 0;
}

// The in-memory frame's header, then the offsets index (get_coffsets, 2102-2155) decoded on the
// device.
int parse(b2h_frame* f) {
  if (f->len < kHeaderMin) return BLOSC2_ERROR_READ_BUFFER;
  int rc = upload(f);
  if (rc) return rc;
  // `len` bytes at `pos`: the host copy's, or fetched from the device copy
  auto bytes_at = [&](int64_t pos, int32_t len, uint8_t* out) {
    if (f->host) {
      memcpy(out, f->host + pos, (size_t)len);
      return 0;
    }
    return hipMemcpy(out, f->dev + pos, (size_t)len, hipMemcpyDeviceToHost) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  };
  uint8_t h[kHeaderMin];
  if ((rc = bytes_at(0, kHeaderMin, h))) return rc;
  FrameHead H;
  int rc0 = parse_head(h, &H);
  if (rc0) return rc0;
  if (H.frame_len > f->len) return BLOSC2_ERROR_INVALID_HEADER;
  if (H.nchunks < 0) return BLOSC2_ERROR_VERSION_SUPPORT;   // variable chunk sizes: not in the device reader
  f->header_len = H.header_len;
  f->nbytes = H.nbytes;
  f->cbytes = H.cbytes;
  f->typesize = H.typesize;
  f->blocksize = H.blocksize;
  f->chunksize = H.chunksize;
  f->compcode = H.compcode;
  f->clevel = H.clevel;
  memcpy(f->filters, H.filters, 6);
  memcpy(f->filters_meta, H.filters_meta, 6);
  f->nchunks = H.nchunks;
  if (f->nbytes == 0) return 0;
  // offsets index: a Blosc chunk right after the data chunks
  const int64_t off_pos = (int64_t)f->header_len + f->cbytes;
  if (off_pos + kChunkHdr > f->len) return BLOSC2_ERROR_INVALID_HEADER;
  f->chdr.assign(kChunkHdr, 0);   // the index chunk's header, as "chunk 0" for one decode call
  if ((rc = bytes_at(off_pos, kChunkHdr, f->chdr.data()))) return rc;
  const int32_t off_nbytes = le32(f->chdr.data() + 4), off_cbytes = le32(f->chdr.data() + 12);
  if (off_nbytes != f->nchunks * 8 || off_cbytes < 16 || off_pos + off_cbytes > f->len) return BLOSC2_ERROR_INVALID_HEADER;
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
  for (int64_t i = 0; i < f->nchunks && !rc; i++) {   // get_coffset bounds (frame.c:3297-3313)
    const int64_t o = f->offsets[i];
    if (o >= 0 && (f->header_len + o > f->header_len + f->cbytes - kChunkHdr || f->header_len + o > f->len - kChunkHdr))
      rc = BLOSC2_ERROR_INVALID_HEADER;
  }
  // every chunk's header: from the host copy, or gathered on the device in one kernel
  f->chdr.assign((size_t)f->nchunks * kChunkHdr, 0);
  if (!rc && f->host) {
    for (int64_t i = 0; i < f->nchunks; i++)
      if (f->offsets[i] >= 0) memcpy(f->chdr.data() + i * kChunkHdr, f->host + f->header_len + f->offsets[i], kChunkHdr);
  } else if (!rc && f->nchunks > 0) {
    uint8_t* d_hdr = nullptr;
    if (hipMalloc(&d_hdr, f->chdr.size()) != hipSuccess) rc = BLOSC2_ERROR_MEMORY_ALLOC;
    if (!rc) {
      const uint32_t grid = (uint32_t)std::min<int64_t>((f->nchunks * kChunkHdr + 255) / 256, 4096);
      k_gather_hdrs<<<grid, 256, 0, f->stream>>>(f->dev, f->header_len, reinterpret_cast<const int64_t*>(d_off),
                                                 f->nchunks, d_hdr);
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(f->chdr.data(), d_hdr, f->chdr.size(), hipMemcpyDeviceToHost, f->stream) != hipSuccess ||
          hipStreamSynchronize(f->stream) != hipSuccess)
        rc = BLOSC2_ERROR_FAILURE;
      (void)hipFree(d_hdr);
    }
  }
  (void)hipFree(d_off);
  return rc;
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

// A ring of pinned slots the file loader reads through (kept for the process: pinning memory
// costs far more than reading it).
constexpr int kLoadSlots = 8;
constexpr int64_t kLoadPiece = int64_t(32) << 20;
std::mutex g_load_mu;
uint8_t* g_load_ring = nullptr;

// Reads [0, len) of an open filesystem-backend stream into HBM (f->dev): kLoadSlots threads each
// read a piece into their pinned slot and queue its H2D, then wait for the slot's DMA before
// reading their next piece.  No host copy: parse() fetches the header bytes it needs from HBM.
int load_file(b2h_frame* f, const blosc2_io_cb* io, void* fp) {
  std::lock_guard<std::mutex> g(g_load_mu);   // one loader at a time owns the ring
  if (!g_load_ring && hipHostMalloc(reinterpret_cast<void**>(&g_load_ring), (size_t)(kLoadSlots * kLoadPiece),
                                    hipHostMallocDefault) != hipSuccess) {
    g_load_ring = nullptr;
    return BLOSC2_ERROR_MEMORY_ALLOC;
  }
  if (hipMalloc(&f->dev, (size_t)f->len) != hipSuccess) return BLOSC2_ERROR_MEMORY_ALLOC;
  const int64_t npieces = (f->len + kLoadPiece - 1) / kLoadPiece;
  const int T = (int)std::min<int64_t>(kLoadSlots, npieces);
  std::vector<int> trc((size_t)T, 0);
  auto worker = [&](int t) {
    uint8_t* slot = g_load_ring + t * kLoadPiece;
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) { trc[(size_t)t] = BLOSC2_ERROR_FAILURE; return; }
    for (int64_t i = t; i < npieces && !trc[(size_t)t]; i += T) {
      const int64_t off = i * kLoadPiece, n = std::min(kLoadPiece, f->len - off);
      if (hipEventSynchronize(ev) != hipSuccess) { trc[(size_t)t] = BLOSC2_ERROR_FAILURE; break; }
      void* q = slot;
      if (io->read(&q, 1, n, off, fp) != n) { trc[(size_t)t] = BLOSC2_ERROR_FILE_READ; break; }
      if (hipMemcpyAsync(f->dev + off, slot, (size_t)n, hipMemcpyHostToDevice, f->stream) != hipSuccess ||
          hipEventRecord(ev, f->stream) != hipSuccess) {
        trc[(size_t)t] = BLOSC2_ERROR_FAILURE;
        break;
      }
    }
    (void)hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(worker, t);
  worker(0);
  for (auto& x : th) x.join();
  for (int r : trc)
    if (r) return r;
  return hipStreamSynchronize(f->stream) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
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
  const uint8_t* h = f->chdr.data() + i * kChunkHdr;
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

// The whole file through the filesystem backend (blosc/blosc2-stdio.c:241-276) into pinned memory:
// positioned reads, a few in flight at once.
b2h_frame* b2h_frame_open(const char* urlpath, int* err) {
  const blosc2_io_cb* io = blosc2_get_io_cb(BLOSC2_IO_FILESYSTEM);
  void* fp = urlpath && io ? io->open(urlpath, "rb", nullptr) : nullptr;
  if (!fp) { if (err) *err = BLOSC2_ERROR_FILE_OPEN; return nullptr; }
  const int64_t len = io->size(fp);
  b2h_frame* f = new b2h_frame();
  f->len = len;
  int rc = len > 0 ? 0 : BLOSC2_ERROR_FILE_READ;
  if (!rc) rc = hipStreamCreateWithFlags(&f->stream, hipStreamNonBlocking) == hipSuccess ? 0 : BLOSC2_ERROR_FAILURE;
  if (!rc) rc = load_file(f, io, fp);
  io->close(fp);
  if (!rc) {
    f->ws = b2h::workspace_create();
    rc = parse(f);   // the device copy is already there (upload() keeps it)
  }
  if (rc) {
    frame_release(f);
    if (err) *err = rc;
    return nullptr;
  }
  if (err) *err = 0;
  return f;
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

// Big-endian stores for the frame writer (frame.c to_big).
void put_be(uint8_t* p, uint64_t v, int n) {
  for (int i = n - 1; i >= 0; i--, v >>= 8) p[i] = (uint8_t)v;
}

}  // namespace

// ------------------------------------------------------------ the frame link ----
namespace b2h {

// The reference's blosc2_frame_s (blosc/frame.h:50-75) for a read-only handle: where the frame's
// bytes are (an in-memory frame, or a stream of an IO backend kept open for the handle's life, as
// frame_reader_acquire keeps one, frame.c:157-216), its header and its decoded offsets index.
struct FrameLink {
  const uint8_t* cframe = nullptr;    // in-memory frame, read in place (not owned)
  const blosc2_io_cb* io = nullptr;   // else: the file's backend ...
  void* params = nullptr;             // ... its udio params ...
  void* fp = nullptr;                 // ... and its open stream
  int64_t file_offset = 0;            // where the frame starts in the file
  FrameHead H;
  std::vector<int64_t> offsets;       // per chunk, from the header end; < 0: special
  std::vector<int64_t> next;          // per stored chunk: where the next stored chunk (or the offsets index) starts
  uint8_t* specials = nullptr;        // the special chunks' 32-byte bodies (schunk->data points in)
  std::mutex mu;                      // serialises the reads of a user backend
  bool serial = false;
  ~FrameLink() {
    if (fp) io->close(fp);
    free(specials);
  }
};

namespace {
FrameLink* link_of(const blosc2_schunk* s) { return reinterpret_cast<FrameLink*>(s->frame); }
}  // namespace

int io_read_par(const blosc2_io_cb* io, void* fp, int64_t pos, int64_t n, uint8_t* dst, std::mutex* mu) {
  if (n <= 0) return 0;
  auto one = [&](int64_t at, int64_t len) {
    void* q = dst + (at - pos);
    std::unique_lock<std::mutex> g;
    if (mu) g = std::unique_lock<std::mutex>(*mu);
    return io->read(&q, 1, len, at, fp) == len;
  };
  constexpr int64_t kPart = int64_t(16) << 20;
  const int T = mu ? 1 : (int)std::max<int64_t>(1, std::min<int64_t>(4, n / kPart));
  if (T == 1) return one(pos, n) ? 0 : BLOSC2_ERROR_FILE_READ;
  std::vector<char> ok((size_t)T, 0);
  std::vector<std::thread> th;
  auto part = [&](int t) {
    const int64_t a = pos + n * t / T, b = pos + n * (t + 1) / T;
    ok[(size_t)t] = one(a, b - a);
  };
  for (int t = 1; t < T; t++) th.emplace_back(part, t);
  part(0);
  for (auto& x : th) x.join();
  for (char c : ok)
    if (!c) return BLOSC2_ERROR_FILE_READ;
  return 0;
}

namespace {

// `n` bytes at frame position `pos` (from the frame start): a buffer backend fills *p, an
// in-memory frame or a mapping backend points it at the bytes.
int link_read(FrameLink* L, int64_t pos, int64_t n, uint8_t** p) {
  if (n == 0) return 0;
  if (pos < 0 || n < 0 || pos + n > L->H.frame_len) return BLOSC2_ERROR_READ_BUFFER;
  if (L->cframe) {
    *p = const_cast<uint8_t*>(L->cframe) + pos;
    return 0;
  }
  if (L->io->is_allocation_necessary) return io_read_par(L->io, L->fp, L->file_offset + pos, n, *p, L->serial ? &L->mu : nullptr);
  std::unique_lock<std::mutex> g;
  if (L->serial) g = std::unique_lock<std::mutex>(L->mu);
  void* q = nullptr;
  if (L->io->read(&q, 1, n, L->file_offset + pos, L->fp) != n || !q) return BLOSC2_ERROR_FILE_READ;
  *p = static_cast<uint8_t*>(q);
  return 0;
}

// `n` bytes at `pos` into `out` whatever the backend.
int link_read_copy(FrameLink* L, int64_t pos, int64_t n, std::vector<uint8_t>* out) {
  out->resize((size_t)n);
  uint8_t* p = out->data();
  const int rc = link_read(L, pos, n, &p);
  if (!rc && p != out->data()) memcpy(out->data(), p, (size_t)n);
  return rc;
}

}  // namespace

bool frame_attached(const blosc2_schunk* s) { return s && s->frame; }

int chunk_ptrs(blosc2_schunk* s, int64_t c0, int32_t n, std::vector<const uint8_t*>* ptrs, ReadBuf* hold) {
  ptrs->assign((size_t)n, nullptr);
  FrameLink* L = link_of(s);
  std::vector<std::pair<int64_t, int32_t>> lazy;   // (offset, k) of the chunks still on the file
  for (int32_t k = 0; k < n; k++) {
    const int64_t i = c0 + k;
    if (s->data && s->data[i]) (*ptrs)[(size_t)k] = s->data[i];
    else if (L && L->offsets[(size_t)i] >= 0) lazy.push_back({L->offsets[(size_t)i], k});
  }
  if (lazy.empty()) return 0;
  std::sort(lazy.begin(), lazy.end());
  // runs of adjacent chunks: [start, end) of the data section, read at once
  struct Run { int64_t start, end; size_t first, last; };
  std::vector<Run> runs;
  for (size_t q = 0; q < lazy.size(); q++) {
    const int64_t o = lazy[q].first, e = L->next[(size_t)(c0 + lazy[q].second)];
    if (!runs.empty() && o <= runs.back().end) {
      runs.back().end = std::max(runs.back().end, e);
      runs.back().last = q;
    } else {
      runs.push_back({o, e, q, q});
    }
  }
  size_t total = 0;
  for (const Run& r : runs) total += (size_t)(r.end - r.start);
  const bool buffered = L->io->is_allocation_necessary;
  if (buffered && !hold->ensure(total)) return BLOSC2_ERROR_MEMORY_ALLOC;
  size_t at = 0;
  for (const Run& r : runs) {
    uint8_t* p = buffered ? hold->p + at : nullptr;
    at += (size_t)(r.end - r.start);
    int rc = link_read(L, (int64_t)L->H.header_len + r.start, r.end - r.start, &p);
    if (rc) return rc;
    for (size_t q = r.first; q <= r.last; q++) {
      const uint8_t* c = p + (lazy[q].first - r.start);
      const int64_t room = L->next[(size_t)(c0 + lazy[q].second)] - lazy[q].first;
      const int32_t cb = room >= BLOSC_MIN_HEADER_LENGTH ? le32(c + 12) : -1;
      if (cb < BLOSC_EXTENDED_HEADER_LENGTH || cb > room) return BLOSC2_ERROR_INVALID_HEADER;   // frame.c:3474-3481
      (*ptrs)[(size_t)lazy[q].second] = c;
    }
  }
  return 0;
}

int link_get_chunk(blosc2_schunk* s, int64_t i, uint8_t** chunk, bool* needs_free) {
  *chunk = nullptr;
  *needs_free = false;
  FrameLink* L = link_of(s);
  if (s->data && s->data[i]) {
    int32_t cb;
    const int rc = blosc2_cbuffer_sizes(s->data[i], nullptr, &cb, nullptr);
    *chunk = s->data[i];
    return rc < 0 ? rc : cb;
  }
  const int64_t o = L->offsets[(size_t)i];
  const int64_t pos = (int64_t)L->H.header_len + o;
  uint8_t hdr[BLOSC_EXTENDED_HEADER_LENGTH];
  uint8_t* p = hdr;
  int rc = link_read(L, pos, BLOSC_EXTENDED_HEADER_LENGTH, &p);
  if (rc) return rc;
  const int32_t cb = le32(p + 12);
  if (cb < BLOSC_EXTENDED_HEADER_LENGTH || o + cb > L->H.cbytes) return BLOSC2_ERROR_INVALID_HEADER;
  if (!L->io->is_allocation_necessary) {
    uint8_t* q = nullptr;
    if ((rc = link_read(L, pos, cb, &q))) return rc;
    *chunk = q;
    return cb;
  }
  uint8_t* q = static_cast<uint8_t*>(malloc((size_t)cb));
  if (!q) return BLOSC2_ERROR_MEMORY_ALLOC;
  if ((rc = link_read(L, pos, cb, &q))) {
    free(q);
    return rc;
  }
  *chunk = q;
  *needs_free = true;
  return cb;
}

void link_free(blosc2_schunk* s) {
  FrameLink* L = link_of(s);
  if (!L) return;
  free(s->data);   // the index only: its chunks live in the frame or in L->specials
  s->data = nullptr;
  s->data_len = 0;
  const blosc2_io_cb* io = L->io;
  void* params = L->params;
  delete L;   // closes the stream
  s->frame = nullptr;
  if (io && io->destroy) (void)io->destroy(params);   // schunk.c:698-705
}

}  // namespace b2h

namespace {

using b2h::FrameLink;
using b2h::link_read_copy;

// frame_from_file_offset (frame.c:1720-1870) / frame_from_cframe (1873-1925) and the header,
// trailer and offsets-index part of frame_to_schunk (2941-3245): everything but the chunks.
// `avail` is the bytes there are from the frame start (the buffer, or the file past `offset`).
int link_open(FrameLink* L, int64_t avail, std::vector<uint8_t>* head, std::vector<uint8_t>* trailer) {
  if (avail < kHeaderMin) return BLOSC2_ERROR_READ_BUFFER;
  L->H.frame_len = avail;   // bounds for the first read only
  std::vector<uint8_t> fixed;
  int rc = link_read_copy(L, 0, kHeaderMin, &fixed);
  if (rc) return rc;
  if ((rc = parse_head(fixed.data(), &L->H))) return rc;
  FrameHead& H = L->H;
  if (H.frame_len < kHeaderMin + 25 || H.frame_len > avail) return BLOSC2_ERROR_INVALID_HEADER;
  if ((rc = link_read_copy(L, 0, H.header_len, head))) return rc;
  // the trailer: its length sits 22 bytes from the frame end (FRAME_TRAILER_LEN_OFFSET)
  std::vector<uint8_t> tail;
  if ((rc = link_read_copy(L, H.frame_len - 25, 25, &tail))) return rc;
  const int64_t tlen = tail[25 - 22 - 1] == 0xce ? be(tail.data() + 25 - 22, 4) : -1;
  if (tlen < 25 || tlen > H.frame_len - kHeaderMin) return BLOSC2_ERROR_READ_BUFFER;
  const int64_t toff = H.nbytes > 0 ? H.frame_len - tlen : H.header_len;   // get_trailer_offset
  if (toff < BLOSC_EXTENDED_HEADER_LENGTH || toff + tlen > H.frame_len) return BLOSC2_ERROR_READ_BUFFER;
  if ((rc = link_read_copy(L, toff, tlen, trailer))) return rc;
  if (H.nchunks == 0 || H.nbytes == 0) {
    H.nchunks = 0;
    return 0;
  }
  // the offsets index: a Blosc chunk right after the data section, decoded by the engine
  const int64_t off_pos = (int64_t)H.header_len + H.cbytes;
  if (off_pos + kChunkHdr > H.frame_len) return BLOSC2_ERROR_INVALID_HEADER;
  std::vector<uint8_t> oc;
  if ((rc = link_read_copy(L, off_pos, kChunkHdr, &oc))) return rc;
  const int32_t off_nbytes = le32(oc.data() + 4), off_cbytes = le32(oc.data() + 12);
  if (H.nchunks < 0) {   // variable chunk sizes (get_header_info, frame.c:1010-1030): count from the index
    if (off_nbytes <= 0 || off_nbytes % 8) return BLOSC2_ERROR_INVALID_HEADER;
    H.nchunks = off_nbytes / 8;
  }
  if (off_nbytes != H.nchunks * 8 || off_cbytes < 16 || off_pos + off_cbytes > H.frame_len) return BLOSC2_ERROR_INVALID_HEADER;
  if ((rc = link_read_copy(L, off_pos, off_cbytes, &oc))) return rc;
  L->offsets.resize((size_t)H.nchunks);
  blosc2_context* dctx = blosc2_create_dctx(BLOSC2_DPARAMS_DEFAULTS);
  if (!dctx) return BLOSC2_ERROR_MEMORY_ALLOC;
  const int got = blosc2_decompress_ctx(dctx, oc.data(), off_cbytes, L->offsets.data(), off_nbytes);
  blosc2_free_ctx(dctx);
  if (got != off_nbytes) return got < 0 ? got : BLOSC2_ERROR_DATA;
  // get_coffset's bounds (frame.c:3297-3313), then each stored chunk's room: up to the next one
  std::vector<int64_t> starts;
  for (int64_t o : L->offsets) {
    if (o >= 0 && o > H.cbytes - kChunkHdr) return BLOSC2_ERROR_INVALID_HEADER;
    if (o >= 0) starts.push_back(o);
  }
  std::sort(starts.begin(), starts.end());
  L->next.assign((size_t)H.nchunks, 0);
  for (size_t i = 0; i < L->offsets.size(); i++) {
    if (L->offsets[i] < 0) continue;
    auto it = std::upper_bound(starts.begin(), starts.end(), L->offsets[i]);
    L->next[i] = it == starts.end() ? H.cbytes : *it;
  }
  return 0;
}

int32_t link_chunk_nbytes(const FrameHead& H, int64_t i) {
  if (H.chunksize <= 0) return 0;   // variable chunk sizes: a special chunk stands for 0 bytes (frame.c:3430-3437)
  if (i == H.nchunks - 1 && H.chunksize > 0 && H.nbytes % H.chunksize) return (int32_t)(H.nbytes % H.chunksize);
  return H.chunksize;
}

// frame_special_chunk (frame.c:3321-3365): the 32-byte chunk a special offset stands for.
int special_chunk(const FrameHead& H, int64_t i, uint64_t v, uint8_t* out) {
  blosc2_cparams scp = BLOSC2_CPARAMS_DEFAULTS;
  scp.typesize = H.typesize;
  scp.blocksize = H.blocksize;
  const int32_t nb = link_chunk_nbytes(H, i);
  const int kind = (int)((v >> 56) & BLOSC2_SPECIAL_MASK);
  if (kind == BLOSC2_SPECIAL_ZERO) return blosc2_chunk_zeros(scp, nb, out, BLOSC_EXTENDED_HEADER_LENGTH);
  if (kind == BLOSC2_SPECIAL_UNINIT) return blosc2_chunk_uninit(scp, nb, out, BLOSC_EXTENDED_HEADER_LENGTH);
  if (kind == BLOSC2_SPECIAL_NAN) return blosc2_chunk_nans(scp, nb, out, BLOSC_EXTENDED_HEADER_LENGTH);
  return BLOSC2_ERROR_DATA;
}

// frame_to_schunk (blosc/frame.c:2941-3245): header fields -> cparams, counters, metalayers and
// vlmetalayers.  `copy` selects the reference's two flavours: a copy (frame-less; every chunk read
// once into a malloc'd buffer; cbytes = the chunks' sum, blocksize = their common one) or a
// frame-attached handle (contiguous; the header's cbytes and blocksize; chunks read when used).
blosc2_schunk* schunk_from_link(std::unique_ptr<FrameLink> L, bool copy, const char* urlpath, const blosc2_io* udio,
                                const std::vector<uint8_t>& head, const std::vector<uint8_t>& trailer) {
  const FrameHead& H = L->H;
  const blosc2_destroy_cb io_destroy = L->io ? L->io->destroy : nullptr;
  void* const io_params = L->params;
  blosc2_cparams cp = BLOSC2_CPARAMS_DEFAULTS;
  cp.typesize = H.typesize;
  cp.clevel = H.clevel;
  cp.compcode = H.compcode == BLOSC_UDCODEC_FORMAT ? H.udcodec : H.compcode;
  cp.compcode_meta = H.codec_meta;
  cp.splitmode = (H.other & 0x03) + 1;
  cp.use_dict = H.other2 & 1;
  cp.blocksize = H.blocksize;
  memcpy(cp.filters, H.filters, 6);
  memcpy(cp.filters_meta, H.filters_meta, 6);
  blosc2_dparams dp = BLOSC2_DPARAMS_DEFAULTS;
  blosc2_storage st = BLOSC2_STORAGE_DEFAULTS;
  st.contiguous = false;
  st.urlpath = nullptr;
  st.cparams = &cp;
  st.dparams = &dp;
  if (udio) st.io = const_cast<blosc2_io*>(udio);
  blosc2_schunk* s = blosc2_schunk_new(&st);
  if (!s) {
    if (io_destroy) io_destroy(io_params);
    return nullptr;
  }
  int rc = 0;
  // the special chunks, built once (their 32 bytes stand in the index for either flavour)
  int64_t nspecial = 0;
  for (int64_t o : L->offsets) nspecial += o < 0;
  if (nspecial > 0) {
    L->specials = static_cast<uint8_t*>(malloc((size_t)nspecial * BLOSC_EXTENDED_HEADER_LENGTH));
    if (!L->specials) rc = BLOSC2_ERROR_MEMORY_ALLOC;
  }
  std::vector<uint8_t*> index((size_t)H.nchunks, nullptr);
  for (int64_t i = 0, k = 0; i < H.nchunks && rc >= 0; i++) {
    const int64_t o = L->offsets[(size_t)i];
    if (o < 0) {
      uint8_t* c = L->specials + (k++) * BLOSC_EXTENDED_HEADER_LENGTH;
      rc = special_chunk(H, i, (uint64_t)o, c);
      index[(size_t)i] = c;
    } else if (L->cframe) {
      index[(size_t)i] = const_cast<uint8_t*>(L->cframe) + H.header_len + o;   // in place
    }
  }
  if (rc >= 0 && !copy) {
    // the attached handle: the index as it stands, the header's counters
    s->data = static_cast<uint8_t**>(calloc((size_t)std::max<int64_t>(H.nchunks, 1), sizeof(uint8_t*)));
    if (!s->data) rc = BLOSC2_ERROR_MEMORY_ALLOC;
    if (rc >= 0) {
      for (int64_t i = 0; i < H.nchunks; i++) s->data[i] = index[(size_t)i];
      s->data_len = (size_t)H.nchunks * sizeof(uint8_t*);
      s->nchunks = H.nchunks;
      s->nbytes = H.nbytes;
      s->cbytes = H.cbytes;
      s->chunksize = H.chunksize;
      s->blocksize = H.blocksize;
      s->storage->contiguous = true;
      if (urlpath) s->storage->urlpath = strdup(urlpath);
      s->frame = reinterpret_cast<blosc2_frame*>(L.release());
      if (s->nchunks > 0) {   // flags2 from the first chunk's header (frame.c:3000-3012)
        uint8_t* c0;
        bool nf;
        const int cb = b2h::link_get_chunk(s, 0, &c0, &nf);
        if (cb < 0) rc = cb;
        else s->flags2 = c0[BLOSC2_CHUNK_BLOSC2_FLAGS2];
        if (cb >= 0 && nf) free(c0);
      }
    }
  } else if (rc >= 0) {
    // the copy: every chunk read once (in place, or one read per run of adjacent chunks) and
    // appended as a malloc'd copy; a stack view of the link serves chunk_ptrs
    blosc2_schunk view{};
    view.frame = reinterpret_cast<blosc2_frame*>(L.get());
    view.data = index.data();
    int32_t common_bs = 0;
    b2h::ReadBuf hold;
    constexpr int32_t kGroup = 64;
    for (int64_t g0 = 0; g0 < H.nchunks && rc >= 0; g0 += kGroup) {
      const int32_t m = (int32_t)std::min<int64_t>(kGroup, H.nchunks - g0);
      std::vector<const uint8_t*> ptrs;
      rc = b2h::chunk_ptrs(&view, g0, m, &ptrs, &hold);
      for (int32_t k = 0; k < m && rc >= 0; k++) {
        const uint8_t* c = ptrs[(size_t)k];
        const int32_t bs = le32(c + 8);
        common_bs = g0 + k == 0 ? bs : (common_bs == bs ? bs : 0);
        const int64_t r = blosc2_schunk_append_chunk(s, const_cast<uint8_t*>(c), true);
        if (r < 0) rc = (int)r;
      }
    }
    if (rc >= 0 && s->nbytes != H.nbytes) rc = BLOSC2_ERROR_INVALID_HEADER;
    if (rc >= 0 && H.nchunks > 0) s->flags2 = s->data[0][BLOSC2_CHUNK_BLOSC2_FLAGS2];
    s->current_nchunk = 0;
    if (rc >= 0) {
      s->chunksize = H.chunksize;
      s->blocksize = common_bs;   // cbytes: the appended chunks' sum already
    }
  }
  if (rc < 0 && !s->frame) {
    // the stream closes before its params go (schunk.c:698-705 order); an attached handle's
    // free does both
    L.reset();
    if (io_destroy) io_destroy(io_params);
  }
  if (rc < 0) {
    blosc2_schunk_free(s);   // an attached handle's link goes with it
    return nullptr;
  }
  int nm = 0;
  rc = read_layers(head.data(), H.header_len, 89, BLOSC2_MAX_METALAYERS, s->metalayers, &nm);   // FRAME_IDX_SIZE
  s->nmetalayers = (uint16_t)nm;
  int nv = 0;
  if (rc >= 0) rc = read_layers(trailer.data(), (int64_t)trailer.size(), 4, BLOSC2_MAX_VLMETALAYERS, s->vlmetalayers, &nv);
  s->nvlmetalayers = (int16_t)nv;
  if (rc < 0) {
    blosc2_schunk_free(s);
    return nullptr;
  }
  return s;
}

}  // namespace

// ------------------------------------------------------------ super-chunk -> frame ----
namespace {

// new_header_frame (frame.c:591-889) for `s`, with the data section's length `cbytes`; the frame
// length (bytes 16-23) is patched in once known.
int frame_header(blosc2_schunk* s, int64_t cbytes, std::vector<uint8_t>* out) {
  std::vector<uint8_t>& h = *out;
  h.assign(kHeaderMin, 0);
  h[0] = 0x90 + 14;
  h[1] = 0xa0 + 8;
  memcpy(&h[kMagic], "b2frame", 8);   // with its NUL
  h[kHeaderLen - 1] = 0xd2;
  h[kFrameLen - 1] = 0xcf;
  h[kFlags - 1] = 0xa0 + 4;
  const bool vl = (s->flags2 & BLOSC2_VL_BLOCKS) != 0;
  uint8_t fl = (uint8_t)(((s->chunksize == 0 || vl) ? 3 : 2) + 0x10);   // format version, 64-bit offsets
  if (s->chunksize == 0) fl |= 0x40;                                    // FRAME_VARIABLE_CHUNKS
  if (vl) fl |= 0x80;                                                   // FRAME_VL_BLOCKS
  h[kFlags] = fl;
  h[kType] = 0;
  h[kCodecs] = (uint8_t)((s->compcode >= BLOSC_LAST_CODEC ? BLOSC_UDCODEC_FORMAT : s->compcode) + (s->clevel << 4));
  h[kFlags + 3] = (uint8_t)(s->splitmode - 1);
  h[kNbytes - 1] = 0xd3;
  put_be(&h[kNbytes], (uint64_t)s->nbytes, 8);
  h[kCbytes - 1] = 0xd3;
  put_be(&h[kCbytes], (uint64_t)cbytes, 8);
  h[kTypesize - 1] = 0xd2;
  put_be(&h[kTypesize], (uint32_t)s->typesize, 4);
  // The reference writes a frame-less super-chunk out through a copy into a new contiguous
  // super-chunk (blosc2_schunk_copy, schunk.c:246-366) whose cparams it zero-initialises and fills
  // from the source's compression context: the header's blocksize is that context's (the last
  // compressed chunk's, or the frame's it was opened from), its compression thread count 0, its
  // decompression thread count the default dparams' 1.
  blosc2_cparams cp;
  int32_t bs = s->blocksize;
  if (s->cctx && blosc2_ctx_get_cparams(s->cctx, &cp) >= 0) bs = cp.blocksize;
  h[kBlocksize - 1] = 0xd2;
  put_be(&h[kBlocksize], (uint32_t)bs, 4);
  h[kChunksize - 1] = 0xd2;
  put_be(&h[kChunksize], (uint32_t)s->chunksize, 4);
  h[62] = 0xd1;   // FRAME_NTHREADS_C
  put_be(&h[63], 0, 2);
  h[65] = 0xd1;   // FRAME_NTHREADS_D
  put_be(&h[66], (uint16_t)BLOSC2_DPARAMS_DEFAULTS.nthreads, 2);
  h[68] = s->nvlmetalayers > 0 ? 0xc3 : 0xc2;   // FRAME_HAS_VLMETALAYERS
  h[69] = 0xd8;                                 // fixext 16: the filter pipeline
  h[kFilters] = BLOSC2_MAX_FILTERS;
  for (int i = 0; i < BLOSC2_MAX_FILTERS; i++) {
    h[kFilters + 1 + i] = s->filters[i];
    h[kFilters + 1 + 8 + i] = s->filters_meta[i];
  }
  h[77] = s->compcode;                 // FRAME_UDCODEC
  h[78] = s->compcode_meta;            // FRAME_CODEC_META
  h[85] = s->use_dict ? 1 : 0;         // FRAME_OTHER_FLAGS2
  // metalayers: array(3) [idx size, map name -> offset, array of bin32 contents]
  const int nm = s->nmetalayers;
  if (nm > BLOSC2_MAX_METALAYERS) return BLOSC2_ERROR_DATA;
  h.push_back(0x90 + 3);
  h.push_back(0xcd);
  h.push_back(0);
  h.push_back(0);
  h.push_back(0xde);
  h.push_back((uint8_t)(nm >> 8));
  h.push_back((uint8_t)nm);
  std::vector<size_t> slot((size_t)nm);
  for (int k = 0; k < nm; k++) {
    const blosc2_metalayer* m = s->metalayers[k];
    const size_t nl = strlen(m->name);
    if (nl >= 32) return BLOSC2_ERROR_DATA;
    h.push_back((uint8_t)(0xa0 + nl));
    h.insert(h.end(), m->name, m->name + nl);
    h.push_back(0xd2);
    slot[(size_t)k] = h.size();
    h.insert(h.end(), 4, 0);
  }
  if (h.size() - kHeaderMin >= (1u << 16)) return BLOSC2_ERROR_DATA;
  put_be(&h[89], (uint16_t)(h.size() - kHeaderMin), 2);   // FRAME_IDX_SIZE
  h.push_back(0xdc);
  h.push_back((uint8_t)(nm >> 8));
  h.push_back((uint8_t)nm);
  for (int k = 0; k < nm; k++) {
    const blosc2_metalayer* m = s->metalayers[k];
    put_be(&h[slot[(size_t)k]], (uint32_t)h.size(), 4);
    h.push_back(0xc6);
    h.insert(h.end(), 4, 0);
    put_be(&h[h.size() - 4], (uint32_t)m->content_len, 4);
    h.insert(h.end(), m->content, m->content + m->content_len);
  }
  put_be(&h[kHeaderLen], (uint32_t)h.size(), 4);
  return 0;
}

// frame_update_trailer (frame.c:1422-1640): version, the vlmetalayers (as the header's
// metalayers), the trailer length and an empty 16-byte fingerprint.
int frame_trailer(const blosc2_schunk* s, std::vector<uint8_t>* out) {
  std::vector<uint8_t>& t = *out;
  const int nv = s->nvlmetalayers;
  if (nv < 0 || nv > BLOSC2_MAX_METALAYERS) return BLOSC2_ERROR_DATA;
  t = {0x90 + 4, 1, 0x90 + 3, 0xcd, 0, 0, 0xde, (uint8_t)(nv >> 8), (uint8_t)nv};
  std::vector<size_t> slot((size_t)nv);
  for (int k = 0; k < nv; k++) {
    const blosc2_metalayer* m = s->vlmetalayers[k];
    const size_t nl = strlen(m->name);
    if (nl >= 32) return BLOSC2_ERROR_DATA;
    t.push_back((uint8_t)(0xa0 + nl));
    t.insert(t.end(), m->name, m->name + nl);
    t.push_back(0xd2);
    slot[(size_t)k] = t.size();
    t.insert(t.end(), 4, 0);
  }
  if (t.size() - 3 >= (1u << 16)) return BLOSC2_ERROR_DATA;
  put_be(&t[4], (uint16_t)(t.size() - 3), 2);
  t.push_back(0xdc);
  t.push_back((uint8_t)(nv >> 8));
  t.push_back((uint8_t)nv);
  for (int k = 0; k < nv; k++) {
    const blosc2_metalayer* m = s->vlmetalayers[k];
    put_be(&t[slot[(size_t)k]], (uint32_t)t.size(), 4);
    t.push_back(0xc6);
    t.insert(t.end(), 4, 0);
    put_be(&t[t.size() - 4], (uint32_t)m->content_len, 4);
    t.insert(t.end(), m->content, m->content + m->content_len);
  }
  const uint32_t tlen = (uint32_t)t.size() + 23;
  t.push_back(0xce);
  t.insert(t.end(), 4, 0);
  put_be(&t[t.size() - 4], tlen, 4);
  t.push_back(0xd8);   // fixext 16: fingerprint type 0 (none), 16 zero bytes
  t.push_back(0);
  t.insert(t.end(), 16, 0);
  return 0;
}

// The pieces of the frame of `s` (frame_from_schunk, frame.c:1926-2100, with the offsets index
// compressed as frame_append_chunk compresses it, 4195-4215): header, offsets-index chunk,
// trailer, and per chunk its bytes' length in the data section (0 for a special chunk, which is
// an offset only, frame.c:4170-4195).  `sizes` drives the writer, which fetches the bytes.
struct FramePlan {
  std::vector<uint8_t> head, offchunk, trailer;
  std::vector<int32_t> stored;   // per chunk: its bytes in the data section
  int64_t cbytes = 0, len = 0;
};

int plan_frame(blosc2_schunk* s, FramePlan* P) {
  const int64_t n = s->nchunks;
  std::vector<int64_t> offs((size_t)n);
  P->stored.assign((size_t)n, 0);
  b2h::ReadBuf hold;
  constexpr int32_t kGroup = 256;
  int64_t at = 0;
  for (int64_t g0 = 0; g0 < n; g0 += kGroup) {   // the chunks' headers (a frame-attached handle reads them)
    const int32_t m = (int32_t)std::min<int64_t>(kGroup, n - g0);
    std::vector<const uint8_t*> ptrs;
    int rc = b2h::chunk_ptrs(s, g0, m, &ptrs, &hold);
    if (rc < 0) return rc;
    for (int32_t k = 0; k < m; k++) {
      const uint8_t* c = ptrs[(size_t)k];
      int32_t cb;
      if (!c || (rc = blosc2_cbuffer_sizes(c, nullptr, &cb, nullptr)) < 0) return c ? rc : BLOSC2_ERROR_DATA;
      const int special = cb >= BLOSC_EXTENDED_HEADER_LENGTH ? (c[BLOSC2_CHUNK_BLOSC2_FLAGS] >> 4) & BLOSC2_SPECIAL_MASK : 0;
      const int64_t i = g0 + k;
      if (special == BLOSC2_SPECIAL_ZERO || special == BLOSC2_SPECIAL_UNINIT || special == BLOSC2_SPECIAL_NAN) {
        offs[(size_t)i] = (int64_t)((uint64_t(1) << 63) | ((uint64_t)special << 56));
      } else {
        offs[(size_t)i] = at;
        P->stored[(size_t)i] = cb;
        at += cb;
      }
    }
  }
  P->cbytes = at;
  int rc = frame_header(s, at, &P->head);
  if (rc < 0) return rc;
  if ((rc = frame_trailer(s, &P->trailer)) < 0) return rc;
  P->offchunk.clear();
  if (n > 0) {
    if (n > (BLOSC2_MAX_BUFFERSIZE / 8)) return BLOSC2_ERROR_DATA;
    blosc2_cparams cp = BLOSC2_CPARAMS_DEFAULTS;
    cp.splitmode = BLOSC_NEVER_SPLIT;
    cp.typesize = 8;
    cp.blocksize = 16 * 1024;
    cp.nthreads = 4;
    cp.compcode = BLOSC_BLOSCLZ;
    b2h_codec_params exact = {B2H_CODEC_PARAMS_MAGIC, 0};   // the reference's bytes
    cp.codec_params = &exact;
    blosc2_context* cctx = blosc2_create_cctx(cp);
    if (!cctx) return BLOSC2_ERROR_NULL_POINTER;
    const int32_t nb = (int32_t)(n * 8);
    P->offchunk.resize((size_t)nb + BLOSC2_MAX_OVERHEAD);
    const int cb = blosc2_compress_ctx(cctx, offs.data(), nb, P->offchunk.data(), nb + BLOSC2_MAX_OVERHEAD);
    blosc2_free_ctx(cctx);
    if (cb < 0) return cb;
    P->offchunk.resize((size_t)cb);
  }
  P->len = (int64_t)P->head.size() + P->cbytes + (int64_t)P->offchunk.size() + (int64_t)P->trailer.size();
  put_be(&P->head[kFrameLen], (uint64_t)P->len, 8);
  return 0;
}

// Writes the frame of `s` through `emit(bytes, n)` in order: header, data chunks, offsets index,
// trailer.
template <class Emit>
int write_frame(blosc2_schunk* s, const FramePlan& P, Emit&& emit) {
  int rc = emit(P.head.data(), (int64_t)P.head.size());
  b2h::ReadBuf hold;
  constexpr int32_t kGroup = 64;
  for (int64_t g0 = 0; g0 < s->nchunks && rc >= 0; g0 += kGroup) {
    const int32_t m = (int32_t)std::min<int64_t>(kGroup, s->nchunks - g0);
    std::vector<const uint8_t*> ptrs;
    if ((rc = b2h::chunk_ptrs(s, g0, m, &ptrs, &hold)) < 0) break;
    for (int32_t k = 0; k < m && rc >= 0; k++)
      if (P.stored[(size_t)(g0 + k)] > 0) rc = emit(ptrs[(size_t)k], P.stored[(size_t)(g0 + k)]);
  }
  if (rc >= 0) rc = emit(P.offchunk.data(), (int64_t)P.offchunk.size());
  if (rc >= 0) rc = emit(P.trailer.data(), (int64_t)P.trailer.size());
  return rc;
}

}  // namespace

extern "C" {

// blosc2_schunk_from_buffer (blosc/schunk.c:731-750, frame_from_cframe frame.c:1873-1925): a
// contiguous frame in memory, read in place (copy = false) or copied chunk by chunk.
blosc2_schunk* blosc2_schunk_from_buffer(uint8_t* cframe, int64_t len, bool copy) {
  if (!cframe || len < kHeaderMin || memcmp(cframe + kMagic, "b2frame", 8) != 0) return nullptr;
  std::unique_ptr<FrameLink> L(new FrameLink());
  L->cframe = cframe;
  std::vector<uint8_t> head, trailer;
  if (link_open(L.get(), len, &head, &trailer) < 0) return nullptr;
  return schunk_from_link(std::move(L), copy, nullptr, nullptr, head, trailer);
}

// blosc2_schunk_open_offset_udio (blosc/schunk.c:405-470, frame_from_file_offset frame.c:1720-1870):
// the frame starting `offset` bytes into the file, attached, through the backend `udio` names.
blosc2_schunk* blosc2_schunk_open_offset_udio(const char* urlpath, int64_t offset, const blosc2_io* udio) {
  if (!urlpath) return nullptr;
  const blosc2_io* io = udio ? udio : &BLOSC2_IO_DEFAULTS;
  const blosc2_io_cb* cb = blosc2_get_io_cb(io->id);
  if (!cb) return nullptr;   // no such backend (the reference's BLOSC2_ERROR_PLUGIN_IO)
  auto fail = [&]() -> blosc2_schunk* {
    if (cb->destroy) (void)cb->destroy(io->params);   // schunk.c:414-424
    return nullptr;
  };
  struct stat st;
  if (offset < 0 || stat(urlpath, &st) != 0) return fail();
  if (S_ISDIR(st.st_mode)) return fail();   // sparse (directory) frames: not in the engine
  std::unique_ptr<FrameLink> L(new FrameLink());
  L->io = cb;
  L->params = io->params;
  L->file_offset = offset;
  L->serial = io->id >= BLOSC2_IO_REGISTERED;   // a user backend: one read at a time
  L->fp = cb->open(urlpath, "rb", io->params);
  if (!L->fp) return fail();
  if (offset > (int64_t)st.st_size) {
    L.reset();
    return fail();
  }
  std::vector<uint8_t> head, trailer;
  if (link_open(L.get(), (int64_t)st.st_size - offset, &head, &trailer) < 0) {
    L.reset();
    return fail();
  }
  blosc2_io local = *io;   // the handle keeps its own copy of the udio (get_new_storage, frame.c:2866-2874)
  return schunk_from_link(std::move(L), false, urlpath, &local, head, trailer);
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

// blosc2_schunk_to_buffer (blosc/schunk.c:481-513).
int64_t blosc2_schunk_to_buffer(blosc2_schunk* schunk, uint8_t** cframe, bool* needs_free) {
  if (!schunk || !cframe || !needs_free) return BLOSC2_ERROR_NULL_POINTER;
  *cframe = nullptr;
  *needs_free = false;
  const FrameLink* L0 = reinterpret_cast<const FrameLink*>(schunk->frame);
  if (L0 && L0->cframe) {   // attached to an in-memory frame: that frame
    *cframe = const_cast<uint8_t*>(L0->cframe);
    return L0->H.frame_len;
  }
  FramePlan P;
  int rc = plan_frame(schunk, &P);
  if (rc < 0) return rc;
  uint8_t* out = static_cast<uint8_t*>(malloc((size_t)std::max<int64_t>(P.len, 1)));
  if (!out) return BLOSC2_ERROR_MEMORY_ALLOC;
  int64_t at = 0;
  rc = write_frame(schunk, P, [&](const uint8_t* p, int64_t n) {
    memcpy(out + at, p, (size_t)n);
    at += n;
    return 0;
  });
  if (rc < 0 || at != P.len) {
    free(out);
    return rc < 0 ? rc : BLOSC2_ERROR_FAILURE;
  }
  *cframe = out;
  *needs_free = true;
  return P.len;
}

}  // extern "C"

namespace {
// The frame of `schunk` written at `pos` of an open filesystem-backend stream (frame_to_file /
// frame_from_schunk's file branch, schunk.c:517-540, frame.c:2039-2090).
int64_t write_to_stream(blosc2_schunk* schunk, const blosc2_io_cb* io, void* fp, int64_t pos) {
  const FrameLink* L0 = reinterpret_cast<const FrameLink*>(schunk->frame);
  if (L0 && L0->cframe)
    return io->write(L0->cframe, L0->H.frame_len, 1, pos, fp) == 1 ? L0->H.frame_len : BLOSC2_ERROR_FILE_WRITE;
  FramePlan P;
  int rc = plan_frame(schunk, &P);
  if (rc < 0) return rc;
  int64_t at = pos;
  rc = write_frame(schunk, P, [&](const uint8_t* p, int64_t n) {
    if (n > 0 && io->write(p, n, 1, at, fp) != 1) return (int)BLOSC2_ERROR_FILE_WRITE;
    at += n;
    return 0;
  });
  return rc < 0 ? rc : P.len;
}
}  // namespace

extern "C" {

// blosc2_schunk_to_file (blosc/schunk.c:591-618): the frame length.
int64_t blosc2_schunk_to_file(blosc2_schunk* schunk, const char* urlpath) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (!urlpath) return BLOSC2_ERROR_INVALID_PARAM;
  const blosc2_io_cb* io = blosc2_get_io_cb(BLOSC2_IO_FILESYSTEM);
  void* fp = io ? io->open(urlpath, "wb", nullptr) : nullptr;
  if (!fp) return BLOSC2_ERROR_FILE_OPEN;
  const int64_t len = write_to_stream(schunk, io, fp, 0);
  if (io->close(fp) != 0 && len >= 0) return BLOSC2_ERROR_FILE_WRITE;
  return len;
}

// blosc2_schunk_append_file (blosc/schunk.c:622-650, append_frame_to_file 540-589): the frame at
// the end of the file (created when missing); the offset it starts at.
int64_t blosc2_schunk_append_file(blosc2_schunk* schunk, const char* urlpath) {
  if (!schunk) return BLOSC2_ERROR_NULL_POINTER;
  if (!urlpath) return BLOSC2_ERROR_INVALID_PARAM;
  const blosc2_io_cb* io = blosc2_get_io_cb(BLOSC2_IO_FILESYSTEM);
  if (!io) return BLOSC2_ERROR_PLUGIN_IO;
  void* fp = io->open(urlpath, "rb+", nullptr);
  if (!fp) {
    fp = io->open(urlpath, "ab", nullptr);
    if (fp) {
      io->close(fp);
      fp = io->open(urlpath, "rb+", nullptr);
    }
  }
  if (!fp) return BLOSC2_ERROR_FILE_OPEN;
  const int64_t pos = io->size(fp);
  if (pos < 0) {
    io->close(fp);
    return BLOSC2_ERROR_FILE_READ;
  }
  const int64_t len = write_to_stream(schunk, io, fp, pos);
  if (io->close(fp) != 0 && len >= 0) return BLOSC2_ERROR_FILE_WRITE;
  return len < 0 ? len : pos;
}

}  // extern "C"
