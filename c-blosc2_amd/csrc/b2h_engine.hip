// b2h_engine.hip -- MI355X (gfx950) batch engine for the Blosc2 chunk pipeline.
//
// Compress (one uniform batch of chunks, all device-resident):
//   [k_copy_work]      only when >= 3 filters are active: the reference rewrites its input in
//                      place (blosc/blosc2.c:1048, 1173-1176), so we work on a private copy W
//   k_ffilter x K      forward filters, one launch per active filter, workgroup per block
//                      (block 0 of every chunk first when DELTA must see a rewritten block 0)
//   k_encode           one wave per stream: run test, entropy probe, exact BloscLZ parse
//   k_finalize         one lane per chunk: serial-layout bookkeeping of blosc_c/serial_blosc
//                      (csize words, bstarts, destsize checks via `peak`, memcpy fallback,
//                      SPECIAL_ZERO), header
//   k_scatter          payloads to their final offsets (workgroup per stream)
//   k_memcpy_chunks    memcpyed chunks
// Decompress (any chunks, device pointer arrays):
//   k_dplan_chunks -> k_dscan -> (one sync for totals) -> k_dplan_blocks -> k_decode ->
//   k_dfilter x K (block 0 first when DELTA is present) ; k_dspecial for memcpyed/special chunks
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <vector>
#include <unistd.h>

#include "b2h_engine.h"
#include "b2h_filters.h"
#include "b2h_lzseg.h"
#include "b2h_format.h"
#include "b2h_lz.h"
#include "b2h_lzfast.h"

namespace b2h {

// error codes (include/blosc2.h:453-492)
enum {
  E_FAILURE = -1, E_DATA = -3, E_MEMORY = -4, E_READ = -5, E_WRITE = -6, E_CODEC = -7, E_DICT = -9,
  E_VERSION = -10, E_HEADER = -11, E_PARAM = -12, E_RUNLEN = -17, E_FILTER = -18, E_MAXBUF = -35,
};
constexpr int32_t kMaxBlocksize = 536866816;   // BLOSC2_MAXBLOCKSIZE (include/blosc2.h:302)
constexpr uint8_t kFlag2VL = 0x1;              // BLOSC2_VL_BLOCKS in blosc2_flags2 (include/blosc2.h:293)
constexpr uint8_t kUseDict = 0x1;              // BLOSC2_USEDICT in blosc2_flags (include/blosc2.h:284)

static thread_local char g_err[256];
const char* last_error() { return g_err; }

#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      snprintf(g_err, sizeof g_err, "%s: %s (%s:%d)", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
      return E_FAILURE;                                                                        \
    }                                                                                          \
  } while (0)

// ------------------------------------------------------------------------------ workspace ----
// Grow-only scratch of one Workspace (see b2h_engine.h), freed with it; buffers carry 256 B of
// slack because the LZ kernels read a few bytes past a stream's end (ldu32).  A regrow frees the
// old buffer with hipFree, which waits for the device work still using it.
struct Scratch {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t n) {
    n += 256;
    if (n <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, n) != hipSuccess) { snprintf(g_err, sizeof g_err, "hipMalloc(%zu) failed", n); return E_MEMORY; }
    cap = n;
    static const bool poison = getenv("B2H_POISON") != nullptr;   // debug: expose unwritten bytes
    if (poison) (void)hipMemset(p, 0xA5, n);
    static const bool trace = getenv("B2H_TRACE_ALLOC") != nullptr;   // debug: where each buffer lives
    if (trace) fprintf(stderr, "b2h scratch %p + %zu\n", p, n);
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <typename T> T* as() const { return static_cast<T*>(p); }
};

struct Workspace {
  Scratch t1, t2, work, sbuf, res, place, mode, qctr, gtab, porder, fsync, fchain;    // compress
  bool porder_init = false;
  Scratch dchunks, dstreams, dblocks, dtotals, stage, stage2, ptrs, dqctr, ddbg, dorder, dbcnt;  // decompress
  std::mutex mu;
  hipEvent_t done = nullptr;       // recorded after the last kernel of the latest call
  hipStream_t last = nullptr;      // the stream that call ran on
  bool used = false;
  // Order this call after the previous user's kernels (same stream: already ordered).
  int acquire(hipStream_t st) {
    if (used && last != st && done) HIPCHK(hipStreamWaitEvent(st, done, 0));
    return 0;
  }
  void release(hipStream_t st) {
    if (!done && hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess) done = nullptr;
    if (done) (void)hipEventRecord(done, st);
    last = st;
    used = true;
  }
  void free_all() {
    if (used && done) (void)hipEventSynchronize(done);
    for (Scratch* s : {&t1, &t2, &work, &sbuf, &res, &place, &mode, &qctr, &gtab, &porder, &fsync, &fchain, &dchunks, &dstreams,
                       &dblocks, &dtotals, &stage, &stage2, &ptrs, &dqctr, &ddbg, &dorder, &dbcnt})
      s->release();
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
    used = false;
    porder_init = false;
  }
};

// The lock + stream ordering of one batch call; the event is recorded on every exit path.
struct WsUse {
  Workspace* ws;
  hipStream_t st;
  std::lock_guard<std::mutex> lock;
  int rc;
  WsUse(Workspace* w, hipStream_t s) : ws(w), st(s), lock(w->mu), rc(w->acquire(s)) {}
  ~WsUse() { ws->release(st); }
};

static std::mutex g_ws_mu;
static std::vector<Workspace*> g_ws_dev;   // process-wide default workspace per device

static Workspace* ws_for_current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> g(g_ws_mu);
  if ((int)g_ws_dev.size() <= dev) g_ws_dev.resize(dev + 1, nullptr);
  if (!g_ws_dev[dev]) g_ws_dev[dev] = new Workspace();
  return g_ws_dev[dev];
}

Workspace* workspace_create() { return new Workspace(); }

void workspace_destroy(Workspace* ws) {
  if (!ws) return;
  {
    std::lock_guard<std::mutex> g(ws->mu);
    ws->free_all();
  }
  delete ws;
}

void release_device_workspaces() {
  std::lock_guard<std::mutex> g(g_ws_mu);
  int cur = 0;
  if (hipGetDevice(&cur) != hipSuccess) cur = 0;
  for (size_t d = 0; d < g_ws_dev.size(); d++) {
    if (!g_ws_dev[d]) continue;
    (void)hipSetDevice((int)d);
    {
      std::lock_guard<std::mutex> l(g_ws_dev[d]->mu);
      g_ws_dev[d]->free_all();
    }
    delete g_ws_dev[d];
    g_ws_dev[d] = nullptr;
  }
  (void)hipSetDevice(cur);
}

int device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// ------------------------------------------------------------------------------- timing -----
static bool g_timing = false;

// Diagnostics: copy the per-stream encoder results of the last compression batch to the host.
int debug_stream_results(void* host, int32_t n) {
  Workspace* ws = ws_for_current_device();
  std::lock_guard<std::mutex> lock(ws->mu);
  if (!ws->res.p || (size_t)n * sizeof(StreamResult) > ws->res.cap) return E_PARAM;
  if (ws->used && ws->done) HIPCHK(hipEventSynchronize(ws->done));
  HIPCHK(hipMemcpy(host, ws->res.p, (size_t)n * sizeof(StreamResult), hipMemcpyDeviceToHost));
  return n;
}

// Diagnostics: BloscLZ mode 3's per-phase cycle sums (a -DB2H_SEG_PROF build; zeros otherwise), reset after
// the copy.  [0..7] probe pass, [8..15] emitting pass: candidates, counting walks, emitting walk,
// rounds, passes, max steps per lane; [16] run tests, [17] streams.
int debug_seg_prof(uint64_t* host) {
#ifdef B2H_SEG_PROF
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_seg_prof), 32 * sizeof(uint64_t)));
  static const uint64_t zero[32] = {};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_seg_prof), zero, sizeof zero));
#else
  memset(host, 0, 32 * sizeof(uint64_t));
#endif
  return 32;
}

// Diagnostics: whether the last fused encode launch on this device's default workspace hit a
// hand-off timeout (its sync word 4; the rescue launches then redid the batch).
int debug_fuse_timed_out() {
  Workspace* ws = ws_for_current_device();
  std::lock_guard<std::mutex> lock(ws->mu);
  if (!ws->fsync.p) return 0;
  if (ws->used && ws->done) HIPCHK(hipEventSynchronize(ws->done));
  int32_t v = 0;
  HIPCHK(hipMemcpy(&v, ws->fsync.as<int32_t>() + 4, sizeof v, hipMemcpyDeviceToHost));
  return v != 0;
}

// Diagnostics: per-stream decoder cycles of the last decompression batch (B2H_DECODE_DEBUG=1).
static const bool g_ddebug = getenv("B2H_DECODE_DEBUG") != nullptr;
int debug_decode_cycles(void* host, int32_t n) {
  Workspace* ws = ws_for_current_device();
  std::lock_guard<std::mutex> lock(ws->mu);
  if (!g_ddebug || !ws->ddbg.p || (size_t)n * 2 * sizeof(int64_t) > ws->ddbg.cap) return E_PARAM;
  if (ws->used && ws->done) HIPCHK(hipEventSynchronize(ws->done));
  HIPCHK(hipMemcpy(host, ws->ddbg.p, (size_t)n * 2 * sizeof(int64_t), hipMemcpyDeviceToHost));
  return n;
}

// Resident single-wave workgroups of `fn` with `lds` bytes of dynamic LDS (the grid size of the
// persistent work-pulling kernels), cached per (fn, lds).
static int resident_slots(const void* fn, size_t lds, int block = 64) {
  static std::mutex m;
  static std::vector<std::pair<std::pair<const void*, size_t>, int>> cache;
  std::lock_guard<std::mutex> g(m);
  for (auto& e : cache)
    if (e.first.first == fn && e.first.second == lds) return e.second;
  int dev = 0, per_cu = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds) != hipSuccess) per_cu = 1;
  const int slots = std::max(1, per_cu) * std::max(1, ncu);
  cache.push_back({{fn, lds}, slots});
  return slots;
}

// Per-phase HIP events of the batch calls since timing was enabled: a ring of at most kEvRing
// event pairs per phase (the oldest reused once full; mean over the ring), guarded by one mutex
// (contexts on several host threads time into the same rings).  Recording never waits on the
// host: the elapsed times are read only when asked for (last_times / mean_times).
static std::mutex g_ev_mu;
constexpr size_t kEvRing = 256;
struct EvPair {
  std::vector<std::pair<hipEvent_t, hipEvent_t>> rec;
  size_t n = 0;   // pairs recorded since the reset (slot = n % kEvRing)
  bool open = false;
  void start(hipStream_t s) {
    if (!g_timing) return;
    std::lock_guard<std::mutex> g(g_ev_mu);
    const size_t k = n % kEvRing;
    if (k == rec.size()) {
      hipEvent_t a = nullptr, b = nullptr;
      if (hipEventCreate(&a) != hipSuccess) return;
      if (hipEventCreate(&b) != hipSuccess) {
        (void)hipEventDestroy(a);
        return;
      }
      rec.push_back({a, b});
    }
    (void)hipEventRecord(rec[k].first, s);
    open = true;
  }
  void stop(hipStream_t s) {
    if (!g_timing) return;
    std::lock_guard<std::mutex> g(g_ev_mu);
    if (!open) return;
    (void)hipEventRecord(rec[n % kEvRing].second, s);
    n++;
    open = false;
  }
  float elapsed(size_t k) {
    float t = 0.f;
    (void)hipEventSynchronize(rec[k].second);
    (void)hipEventElapsedTime(&t, rec[k].first, rec[k].second);
    return t;
  }
  float last() {
    std::lock_guard<std::mutex> g(g_ev_mu);
    return n ? elapsed((n - 1) % kEvRing) : 0.f;
  }
  float mean() {
    std::lock_guard<std::mutex> g(g_ev_mu);
    const size_t m = std::min(n, kEvRing);
    double t = 0;
    for (size_t k = 0; k < m; k++) t += elapsed(k);
    return m ? (float)(t / (double)m) : 0.f;
  }
  void reset() {
    std::lock_guard<std::mutex> g(g_ev_mu);
    n = 0;
    open = false;
  }
};
static EvPair ev_filter, ev_encode, ev_final, ev_decode, ev_unfilter;
void enable_timing(bool on) {
  g_timing = on;
  if (on)
    for (EvPair* e : {&ev_filter, &ev_encode, &ev_final, &ev_decode, &ev_unfilter}) e->reset();
}
KernelTimes last_times() {
  return KernelTimes{ev_filter.last(), ev_encode.last(), ev_final.last(), ev_decode.last(), ev_unfilter.last()};
}
KernelTimes mean_times() {
  return KernelTimes{ev_filter.mean(), ev_encode.mean(), ev_final.mean(), ev_decode.mean(), ev_unfilter.mean()};
}

// ================================================================ compression: geometry ====
struct CGeom {
  int32_t nbytes, bs, nblocks, leftover, spb, nsc, neblock, ts, destsize, clevel, overhead, compcode;
  int32_t dict_size;   // LZ4 dictionary section [int32 size | bytes] after the bstarts (0: none)
  int32_t front;   // encoder pull schedule (pull_to_stream), 0 = stream order
  int32_t lzmode;  // BloscLZ encoder of this batch: 0 exact, 1 fast, 2 fast with deep candidates (the plan's, else the process default)
  int64_t src_stride, wstride, dst_stride;
  uint8_t* chain;  // mode 2: the fast encoder's prev[] arrays, one per workgroup of chain_len() positions
  const int32_t* gate;   // rescue launches (see compress_batch): run only if *gate != 0; null: always
};
// A launch of the rescue sequence queued behind a fused encode launch does its work only when that
// launch's hand-off wait timed out (the gate word is its timeout flag); otherwise every workgroup
// leaves at once.  Uniform: one scalar load per workgroup.
__device__ __forceinline__ bool gated_off(const CGeom& g) {
  return g.gate != nullptr &&
         __builtin_amdgcn_readfirstlane(__hip_atomic_load(g.gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0;
}
__host__ __device__ inline int64_t chain_len(const CGeom& g) { return g.neblock > g.leftover ? g.neblock : g.leftover; }

__device__ __forceinline__ void stream_locate(const CGeom& g, int32_t l, int32_t* off, int32_t* len, int32_t* blk) {
  const int32_t full = g.nblocks - (g.leftover ? 1 : 0);
  if (l < full * g.spb) {
    const int32_t b = l / g.spb, j = l - b * g.spb;
    *blk = b;
    *off = b * g.bs + j * g.neblock;
    *len = g.neblock;
  } else {
    *blk = g.nblocks - 1;
    *off = (g.nblocks - 1) * g.bs;
    *len = g.leftover;
  }
}

__global__ void k_copy_work(const uint8_t* __restrict__ src, int64_t src_stride, uint8_t* __restrict__ dst,
                            int64_t dst_stride, int32_t nbytes) {
  const int32_t c = blockIdx.y;
  const uint8_t* s = src + (int64_t)c * src_stride;
  uint8_t* d = dst + (int64_t)c * dst_stride;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x) d[i] = s[i];
}

// Forward filter stage: grid (blocks_per_launch, nchunks).  pass: 0 all blocks, 1 block 0, 2 blocks >= 1.
__global__ __launch_bounds__(kBlockThreads) void k_ffilter(CGeom g, int pass, uint8_t filter, uint8_t meta,
                                                           const uint8_t* __restrict__ in, int64_t in_stride,
                                                           uint8_t* __restrict__ out, int64_t out_stride,
                                                           const uint8_t* __restrict__ dref, int64_t dref_stride,
                                                           int zeroed) {
  if (gated_off(g)) return;
  const int32_t c = blockIdx.y;
  const int32_t b = pass == 2 ? (int32_t)blockIdx.x + 1 : (int32_t)blockIdx.x;
  if (b >= g.nblocks) return;
  const int32_t off = b * g.bs;
  const int32_t bsize = (b == g.nblocks - 1 && g.leftover) ? g.leftover : g.bs;
  const uint8_t* s = in + (int64_t)c * in_stride + off;
  uint8_t* d = out + (int64_t)c * out_stride + off;
  switch (filter) {
    case kShuffle: block_shuffle(s, d, bsize, meta ? meta : g.ts); break;
    case kBitshuffle: block_bitshuffle(s, d, bsize, g.ts); break;
    case kDelta: block_delta_encode(s, dref + (int64_t)c * dref_stride, d, bsize, g.ts, b == 0); break;
    case kTruncPrec: block_trunc(s, d, bsize, g.ts, zeroed); break;
    case kBytedelta: block_bytedelta_encode(s, d, bsize, meta); break;   // meta: channels (host-resolved)
    case kIntTrunc: block_int_trunc(s, d, bsize, g.ts, zeroed); break;
    default: break;
  }
}

// Fused forward (DELTA, SHUFFLE) pipeline (exactly these two filters, typesize 2/4/8): one pass
// over the input, delta in registers, planes stored once.  Blocks that are not whole quads or not
// 16-byte aligned run the two stages through `tmp` (the first stage's usual buffer) instead.
__global__ __launch_bounds__(kBlockThreads) void k_ffilter_ds(CGeom g, const uint8_t* __restrict__ raw, int64_t raw_stride,
                                                              uint8_t* __restrict__ tmp, uint8_t* __restrict__ out,
                                                              int64_t out_stride) {
  if (gated_off(g)) return;
  const int32_t c = blockIdx.y, b = blockIdx.x;
  if (b >= g.nblocks) return;
  const int32_t off = b * g.bs;
  const int32_t bsize = (b == g.nblocks - 1 && g.leftover) ? g.leftover : g.bs;
  const uint8_t* s = raw + (int64_t)c * raw_stride + off;
  const uint8_t* dref = raw + (int64_t)c * raw_stride;
  uint8_t* t = tmp + (int64_t)c * out_stride + off;
  uint8_t* d = out + (int64_t)c * out_stride + off;
  if (bsize % (4 * g.ts) == 0 && aligned16(s) && aligned16(d) && aligned16(dref)) {
    const int32_t n = bsize / g.ts;
    if (g.ts == 4) delta_shuffle_fast<4>(s, dref, d, n, b == 0);
    else if (g.ts == 8) delta_shuffle_fast<8>(s, dref, d, n, b == 0);
    else delta_shuffle_fast<2>(s, dref, d, n, b == 0);
  } else {
    block_delta_encode(s, dref, t, bsize, g.ts, b == 0);
    __syncthreads();
    block_shuffle(t, d, bsize, g.ts);
  }
}

// Persistent encoder: as many workgroups as fit on the chip, every wave pulling stream indices
// from a device counter until the batch is exhausted.  Stream cost varies ~100x (a float32
// mantissa plane vs an all-zero exponent plane) and the hardware deals workgroups to XCDs / shader
// engines by index, so one-workgroup-per-stream left most slots waiting behind the expensive
// planes; pulling keeps every resident wave busy.  Every wave exits once the counter passes
// `nstreams_total`.
//
// A workgroup holds NLDS waves whose hash table lives in LDS and NGLB waves whose table lives in
// global memory (`gtab`, one per wave slot, see GlbTab in b2h_lz.h).  LDS tables cost 32 KiB per
// wave (4 waves per CU); global tables cost L2/MALL traffic instead.  Dynamic LDS layout:
// [NLDS tables][per wave: bucket bitset + output ring].
// Pull index -> stream index.  With the plane costs learned from the previous batch of the same
// split (k_plane_cost: porder[0] = spb, porder[1] = costliest plane, porder[2..spb] = the others),
// the costliest plane's full-block streams are pulled `front` at a time per round of
// front + spb - 1 pulls (one of every other plane per round), so they are all started well before
// the end of the launch instead of uniformly up to it (T: the smooth plane's streams take ~3.5 ms,
// 10x the others; started last they left most slots idle for the final milliseconds), while every
// round still mixes the cheap planes in (grouping planes outright made the cheap, memory-bound
// probe streams contend with each other: measured slower).  After the costliest plane runs out,
// the other planes continue round-robin, then the leftover-block streams.  The mapping is a
// bijection on [0, ntot): scheduling only, outputs do not depend on it.
__device__ __forceinline__ int32_t pull_to_stream(const CGeom& g, const int32_t* __restrict__ porder, int32_t front,
                                                  int32_t i, int32_t ntot) {
  if (porder == nullptr || front <= 0 || g.spb < 2 || g.spb > 16 || porder[0] != g.spb) return i;
  const int32_t full = g.nblocks - (g.leftover ? 1 : 0);
  const int32_t P = (ntot / g.nsc) * full;   // streams per plane
  const int32_t F = P * g.spb;
  if (i >= F) return (i - F) * g.nsc + full * g.spb;
  const int32_t no = g.spb - 1, R = front + no;
  const int32_t Q = P / front;               // rounds of phase 1
  int32_t plane, item;
  if (i < Q * R) {
    const int32_t r = i / R, k = i - r * R;
    if (k < front) { plane = porder[1]; item = r * front + k; }
    else { plane = porder[2 + (k - front)]; item = r; }
  } else {
    const int32_t j = i - Q * R, left = P - Q * front;
    if (j < left) { plane = porder[1]; item = Q * front + j; }
    else { const int32_t jj = j - left; plane = porder[2 + jj % no]; item = Q + jj / no; }
  }
  const int32_t c = item / full, b = item - c * full;
  return c * g.nsc + b * g.spb + plane;
}

// Per-plane encode cost of a finished batch (sum of the streams' s_memtime cycles) -> the pull
// order of the next batch with the same split (see pull_to_stream).  Scheduling only: outputs
// do not depend on it.
__global__ __launch_bounds__(1024) void k_plane_cost(CGeom g, const StreamResult* __restrict__ res, int32_t ntot,
                                                     int32_t* __restrict__ porder) {
  __shared__ unsigned long long sum[16];
  if (gated_off(g)) return;
  if (g.spb < 2 || g.spb > 16) {
    if (threadIdx.x == 0) porder[0] = 0;
    return;
  }
  if (threadIdx.x < 16) sum[threadIdx.x] = 0ull;
  __syncthreads();
  const int32_t full = g.nblocks - (g.leftover ? 1 : 0);
  for (int32_t s = threadIdx.x; s < ntot; s += blockDim.x) {
    const int32_t l = s % g.nsc;
    if (l < full * g.spb) atomicAdd(&sum[l % g.spb], (unsigned long long)res[s].cycles);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int32_t ord[16];
    for (int j = 0; j < g.spb; j++) ord[j] = j;
    for (int a = 1; a < g.spb; a++) {   // insertion sort, costliest first, ties keep plane order
      const int32_t v = ord[a];
      int b = a;
      while (b > 0 && sum[ord[b - 1]] < sum[v]) { ord[b] = ord[b - 1]; b--; }
      ord[b] = v;
    }
    for (int j = 0; j < g.spb; j++) porder[1 + j] = ord[j];
    porder[0] = g.spb;
  }
}

// A wave-uniform copy of an LDS-resident value (word by word through readfirstlane).
template <typename T>
__device__ __forceinline__ T lds_uniform(const B2H_LDS T* p) {
  static_assert(sizeof(T) % 4 == 0, "word-sized fields only");
  union U {
    T v;
    uint32_t w[sizeof(T) / 4];
    __device__ U() {}
  } u;
  const volatile B2H_LDS uint32_t* q = (const volatile B2H_LDS uint32_t*)p;
#pragma unroll
  for (size_t k = 0; k < sizeof(T) / 4; k++) u.w[k] = __builtin_amdgcn_readfirstlane(q[k]);
  return u.v;
}
template <typename T>
__device__ __forceinline__ void lds_store(B2H_LDS T* p, const T& v) {
  static_assert(sizeof(T) % 4 == 0, "word-sized fields only");
  union U {
    T v;
    uint32_t w[sizeof(T) / 4];
    __device__ U() {}
  } u;
  u.v = v;
  B2H_LDS uint32_t* q = (B2H_LDS uint32_t*)p;
#pragma unroll
  for (size_t k = 0; k < sizeof(T) / 4; k++) q[k] = u.w[k];
}
// The exact encoder's arguments, staged in LDS at launch (see FusedArgs below: kept in kernel
// arguments they stayed live in SGPRs through the encode and ~100 SGPRs spilled into VGPR lanes).
struct EncArgs {
  CGeom g;
  const uint8_t* filt;
  uint8_t* sbuf;
  StreamResult* res;
  int32_t* next;
  const int32_t* porder;
  int32_t nstreams_total, pad;
};

// Where the 144 bytes would cost a workgroup per CU (u32 positions -- streams > 64 KiB -- fill
// exactly 80 KiB per workgroup at hashlog 14: 2 per CU) the loop reads the kernel argument.
template <typename T>
__device__ __forceinline__ T arg_uniform(const B2H_LDS T* p) { return lds_uniform(p); }
template <typename T>
__device__ __forceinline__ T arg_uniform(const T* p) { return *p; }
template <typename TAB, typename AP>
__device__ __forceinline__ void encode_loop(AP A, TAB htab, B2H_LDS uint32_t* dbits, B2H_LDS uint8_t* oring) {
  for (;;) {
    // branch-free grab: every lane takes part (lane 0 adds 1, the others 0), so no divergent
    // region sits between the atomic and the broadcast -- with a lane-0 branch the structurizer
    // let lanes 1..63 run ahead into the next iteration and re-read a stale index.
    // (a global-address-space atomic: the backend's atomic optimizer folds the 64 lanes into one;
    // through the generic pointer read back from LDS it issued 64 flat atomics per grab, and
    // ~4 M serialised RMWs on the one counter doubled the T encode)
    const int32_t i = __builtin_amdgcn_readfirstlane(__hip_atomic_fetch_add(
        (B2H_GLB int32_t*)arg_uniform(&A->next), lane_id() == 0 ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const int32_t ntot = arg_uniform(&A->nstreams_total);
    if (i >= ntot) return;
    int32_t s, len, clevel;
    gin_t in;
    gout_t out;
    bool runs;
    {
      const CGeom g = arg_uniform(&A->g);
      s = __builtin_amdgcn_readfirstlane(pull_to_stream(g, arg_uniform(&A->porder), g.front, i, ntot));
      const int32_t c = s / g.nsc, l = s - c * g.nsc;
      int32_t off, blk;
      stream_locate(g, l, &off, &len, &blk);
      in = (gin_t)(arg_uniform(&A->filt) + (int64_t)c * g.wstride + off);
      out = (gout_t)(arg_uniform(&A->sbuf) + (int64_t)c * g.wstride + off);
      clevel = g.clevel;
      runs = g.overhead == kHdrExt;
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide time base
    StreamResult r = encode_stream<TAB>(in, len, clevel, out, htab, dbits, oring, runs);
    r.cycles = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
    if (TAB::kGlobal) r.windows |= 1 << 30;   // diagnostics: the stream ran on a global-table wave
    r.t_start = (int64_t)((rt0 << 24) | ((__builtin_amdgcn_s_memrealtime() - rt0) & 0xffffff));
    if (lane_id() == 0) arg_uniform(&A->res)[s] = r;
  }
}

__host__ __device__ constexpr size_t enc_wave_lds(int hashlog) { return ((size_t(1) << hashlog) >> 3) + kOutRing; }
// EncArgs staged in LDS: u16 positions (see encode_loop)
template <typename POS>
__host__ __device__ constexpr bool enc_args_lds() { return sizeof(POS) == 2; }
template <typename POS>
__host__ __device__ constexpr size_t enc_wg_lds(int hashlog, int nlds, int nglb) {
  return (size_t)nlds * (sizeof(POS) << hashlog) + (size_t)(nlds + nglb) * enc_wave_lds(hashlog) +
         (enc_args_lds<POS>() ? ((sizeof(EncArgs) + 15) & ~size_t(15)) : 0);
}

template <typename POS, int NLDS, int NGLB>
__global__ __launch_bounds__(64 * (NLDS + NGLB)) __attribute__((amdgpu_waves_per_eu(3, 8)))   // <= 168 VGPRs (kExWords)
void k_encode(EncArgs args, POS* __restrict__ gtab) {
  if (gated_off(args.g)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int hashlog = args.g.clevel == 1 ? 12 : (args.g.clevel == 2 ? 13 : 14);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t tabsz = sizeof(POS) << hashlog;
  B2H_LDS EncArgs* A = (B2H_LDS EncArgs*)(smem + NLDS * tabsz + (NLDS + NGLB) * enc_wave_lds(hashlog));
  if (enc_args_lds<POS>()) {
    if (threadIdx.x == 0) lds_store(A, args);
    __syncthreads();
  }
  B2H_LDS uint8_t* mine = (B2H_LDS uint8_t*)(smem + NLDS * tabsz + w * enc_wave_lds(hashlog));
  B2H_LDS uint32_t* dbits = (B2H_LDS uint32_t*)mine;
  B2H_LDS uint8_t* oring = mine + ((size_t(1) << hashlog) >> 3);
  if (NLDS > 0 && w < NLDS) {
    LdsTab<POS> t;
    t.t = (volatile B2H_LDS POS*)(smem + w * tabsz);
    if (enc_args_lds<POS>()) encode_loop(static_cast<const B2H_LDS EncArgs*>(A), t, dbits, oring);
    else encode_loop(static_cast<const EncArgs*>(&args), t, dbits, oring);
  } else if (NGLB > 0) {
    GlbTab<POS> t;
    t.t = (B2H_GLB POS*)(gtab + (((size_t)blockIdx.x * NGLB + (w - NLDS)) << hashlog));
    if (enc_args_lds<POS>()) encode_loop(static_cast<const B2H_LDS EncArgs*>(A), t, dbits, oring);
    else encode_loop(static_cast<const EncArgs*>(&args), t, dbits, oring);
  }
}

// ------------------------------------------------------------------ BloscLZ fast mode ----
// One stream per workgroup of two waves: wave 0 matches, wave 1 parses (b2h_lzfast.h);
// persistent, pulling streams like k_encode.  LDS per workgroup: table + output ring + hand-over
// slots.
__host__ __device__ constexpr size_t fast_lds(size_t pos_bytes, int tablog) {
  return (pos_bytes << tablog) + kOutRing + ((sizeof(FastShared) + 15) & ~size_t(15));
}
template <typename POS, bool DEEP>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(4, 8)))   // <= 128 VGPRs: 16 waves per CU
void k_encode_fast(CGeom g, const uint8_t* __restrict__ filt, uint8_t* __restrict__ sbuf,
                   StreamResult* __restrict__ res, int32_t nstreams_total, int32_t* __restrict__ next, int tablog,
                   const int32_t* __restrict__ porder) {
  if (gated_off(g)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* tab = (B2H_LDS uint8_t*)smem;
  B2H_LDS uint8_t* oring = (B2H_LDS uint8_t*)(smem + (sizeof(POS) << tablog));
  B2H_LDS FastShared* sh = (B2H_LDS FastShared*)(smem + (sizeof(POS) << tablog) + kOutRing);
  const bool matcher = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  if (!matcher) __builtin_amdgcn_s_setprio(2);   // the parser issues first (see k_encode_fast_fused)
  // the pull is the loop's last statement and its broadcast result the loop's only exit test: a
  // loop that holds barriers with lane-0 code before a mid-body exit can be structurized into an
  // exec-masked nest whose waves meet different barriers (seen in round 4: a hang, or a stale
  // stream index and an illegal address)
  auto pull = [&]() {
    if (threadIdx.x == 0) sh->pull = atomicAdd(next, 1);
    __syncthreads();
    const int32_t v = __builtin_amdgcn_readfirstlane(sh->pull);
    __syncthreads();
    return v;
  };
  for (int32_t i = pull(); i < nstreams_total; i = pull()) {
    const int32_t s = __builtin_amdgcn_readfirstlane(pull_to_stream(g, porder, g.front, i, nstreams_total));
    const int32_t c = s / g.nsc, l = s - c * g.nsc;
    int32_t off, len, blk;
    stream_locate(g, l, &off, &len, &blk);
    gin_t in = (gin_t)(filt + (int64_t)c * g.wstride + off);
    gout_t out = (gout_t)(sbuf + (int64_t)c * g.wstride + off);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    StreamResult r = encode_stream_fast<POS, false, DEEP>(in, len, g.clevel, out, tab, tablog, oring, sh,
                                                          g.overhead == kHdrExt, matcher,
                                                          (B2H_GLB POS*)g.chain + (int64_t)blockIdx.x * chain_len(g));
    r.cycles = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
    r.t_start = (int64_t)((rt0 << 24) | ((__builtin_amdgcn_s_memrealtime() - rt0) & 0xffffff));
    if (!matcher && lane_id() == 0) res[s] = r;
  }
}

// BloscLZ encoder mode: exact (default, byte-identical to the reference) or fast (round-trip
// identical, same grammar and decisions, parse-independent candidates).  Process-wide; also
// B2H_LZ_MODE=fast|exact and B2H_FAST_TABLOG (12..14, default 13) in the environment.
static int g_lz_mode = -1;
static int lz_mode() {
  if (g_lz_mode < 0) {
    const char* e = getenv("B2H_LZ_MODE");
    g_lz_mode = (e && !strcmp(e, "fast")) ? 1 : (e && !strcmp(e, "deep")) ? 2 : (e && !strcmp(e, "seg")) ? 3 : 0;
  }
  return g_lz_mode;
}
int set_blosclz_mode(int mode) {
  const int old = lz_mode();
  if (mode >= 0 && mode <= 3) g_lz_mode = mode;
  return old;
}
static int fast_tablog() {
  static int v = 0;
  if (!v) {
    const char* e = getenv("B2H_FAST_TABLOG");
    v = e ? std::max(10, std::min(14, atoi(e))) : 13;
  }
  return v;
}

// Mode 2: one prev[] array of chain_len(g) positions per workgroup of the grid.
template <typename POS>
static int chain_prepare(Workspace* ws, CGeom& g, uint32_t grid) {
  g.chain = nullptr;
  if (g.lzmode != 2) return 0;
  if (ws->fchain.ensure((size_t)grid * (size_t)chain_len(g) * sizeof(POS) + 256)) return E_MEMORY;
  g.chain = ws->fchain.as<uint8_t>();
  return 0;
}

template <typename POS, bool DEEP>
static int launch_encode_fast_t(Workspace* ws, const CGeom& g0, const uint8_t* filt, StreamResult* res, int64_t ntot,
                                int32_t* next, const int32_t* porder, hipStream_t st) {
  CGeom g = g0;
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const int tablog = std::min(fast_tablog(), hashlog);
  const size_t lds = fast_lds(sizeof(POS), tablog);
  const void* fn = reinterpret_cast<const void*>(&k_encode_fast<POS, DEEP>);
  static bool attr_set = false;
  if (!attr_set) {   // > 64 KiB of dynamic LDS (u32, tablog 14): opt in once
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int slots = resident_slots(fn, lds, 128);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(ntot, slots));
  if (chain_prepare<POS>(ws, g, grid)) return E_MEMORY;
  k_encode_fast<POS, DEEP><<<grid, 128, lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot, next, tablog, porder);
  HIPCHK(hipGetLastError());
  return 0;
}

// u16 table entries (half the LDS: twice the waves per CU): BloscLZ mode 1 at any stream length
// (positions modulo 2^16, fast_exchange); mode 2 while every stream fits 64 KiB (its prev[] chains
// keep full positions).
static bool fast_u16(const CGeom& g) { return g.lzmode != 2 || std::max(g.neblock, g.leftover) <= 65536; }
static int launch_encode_fast(Workspace* ws, const CGeom& g, const uint8_t* filt, StreamResult* res, int64_t ntot,
                              int32_t* next, const int32_t* porder, hipStream_t st) {
  const bool small = fast_u16(g);
  if (g.lzmode == 2)
    return small ? launch_encode_fast_t<uint16_t, true>(ws, g, filt, res, ntot, next, porder, st)
                 : launch_encode_fast_t<uint32_t, true>(ws, g, filt, res, ntot, next, porder, st);
  return small ? launch_encode_fast_t<uint16_t, false>(ws, g, filt, res, ntot, next, porder, st)
               : launch_encode_fast_t<uint32_t, false>(ws, g, filt, res, ntot, next, porder, st);
}

// ----------------------------------------------------- BloscLZ mode 3: segmented parse ----
// One wave per workgroup and stream (b2h_lzseg.h): the LDS holds the stream's u16 table only while
// the candidates are exchanged; the distances and masks live in this workgroup's global scratch.
// W waves per workgroup, each encoding its own streams; they share the workgroup's one candidate
// table under an LDS lock (b2h_lzseg.h seg_lock).
template <bool CHK, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_encode_seg(CGeom g, const uint8_t* __restrict__ filt, uint8_t* __restrict__ sbuf,
                                                       StreamResult* __restrict__ res, int32_t nstreams_total,
                                                       int32_t* __restrict__ next, int tablog,
                                                       const int32_t* __restrict__ porder) {
  if (gated_off(g)) return;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* tab = (B2H_LDS uint8_t*)smem;
  const int64_t sb = seg_scratch_bytes(chain_len(g));
  int32_t* lock = reinterpret_cast<int32_t*>(g.chain + (int64_t)gridDim.x * W * sb) + 64 * blockIdx.x;
  if (threadIdx.x == 0) atomicExch(lock, 0);
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* mine = g.chain + ((int64_t)blockIdx.x * W + wave) * sb;
  B2H_GLB uint32_t* dist = (B2H_GLB uint32_t*)mine;
  B2H_GLB uint64_t* mask = (B2H_GLB uint64_t*)(mine + seg_dist_bytes(chain_len(g)));
  B2H_GLB uint32_t* snv = (B2H_GLB uint32_t*)(mine + seg_dist_bytes(chain_len(g)) + seg_mask_bytes(chain_len(g)));
  auto pull = [&]() {
    int32_t v = 0;
    if (lane_id() == 0) v = atomicAdd(next, 1);
    return __shfl(v, 0);
  };
  for (int32_t i = pull(); i < nstreams_total; i = pull()) {
    const int32_t s = __builtin_amdgcn_readfirstlane(pull_to_stream(g, porder, g.front, i, nstreams_total));
    const int32_t c = s / g.nsc, l = s - c * g.nsc;
    int32_t off, len, blk;
    stream_locate(g, l, &off, &len, &blk);
    gin_t in = (gin_t)(filt + (int64_t)c * g.wstride + off);
    gout_t out = (gout_t)(sbuf + (int64_t)c * g.wstride + off);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    StreamResult r = encode_stream_seg<false, CHK>(in, len, g.clevel, out, tab, tablog, dist, mask, snv,
                                                   g.overhead == kHdrExt, lock);
    r.cycles = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
    r.t_start = (int64_t)((rt0 << 24) | ((__builtin_amdgcn_s_memrealtime() - rt0) & 0xffffff));
    if (lane_id() == 0) res[s] = r;
  }
}

template <bool CHK, int W>
static int launch_encode_seg_t(Workspace* ws, const CGeom& g0, const uint8_t* filt, StreamResult* res, int64_t ntot,
                               int32_t* next, const int32_t* porder, hipStream_t st, int tablog) {
  CGeom g = g0;
  const size_t lds = CHK ? (size_t)4 << tablog : (size_t)2 << tablog;
  const void* fn = reinterpret_cast<const void*>(&k_encode_seg<CHK, W>);
  const int slots = resident_slots(fn, lds, 64 * W);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>((ntot + W - 1) / W, slots));
  const int64_t sb = seg_scratch_bytes(chain_len(g));
  if (ws->fchain.ensure((size_t)grid * W * (size_t)sb + (size_t)grid * 256 + 256)) return E_MEMORY;   // + lock words
  g.chain = ws->fchain.as<uint8_t>();
  k_encode_seg<CHK, W><<<grid, 64 * W, lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot, next, tablog, porder);
  HIPCHK(hipGetLastError());
  return 0;
}

// BloscLZ mode 3.  Streams of <= 2^16 positions: u32 table entries with a check of the hashed value
// (no candidate reads); longer streams: u16 entries (their aliasing rule reads the candidates).
// B2H_SEG_WAVES (1..4, default 4): waves per workgroup sharing one table (T: 2 / 3 / 4 waves
// 193.1 / 205.7 / 209.4 GiB/s unfused, profiles/r6_seg_bench_w*.log).
static int seg_waves() {
  static const int W = [] { const char* e = getenv("B2H_SEG_WAVES"); return e ? std::max(1, std::min(4, atoi(e))) : 4; }();
  return W;
}
static int launch_encode_seg(Workspace* ws, const CGeom& g, const uint8_t* filt, StreamResult* res, int64_t ntot,
                             int32_t* next, const int32_t* porder, hipStream_t st) {
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const int tablog = std::min(fast_tablog(), hashlog);
  const int W = seg_waves();
  const bool chk = chain_len(g) <= 65536;
#define B2H_SEG_LAUNCH(C, WW) return launch_encode_seg_t<C, WW>(ws, g, filt, res, ntot, next, porder, st, tablog)
  if (chk) {
    if (W == 1) B2H_SEG_LAUNCH(true, 1);
    if (W == 2) B2H_SEG_LAUNCH(true, 2);
    if (W == 3) B2H_SEG_LAUNCH(true, 3);
    B2H_SEG_LAUNCH(true, 4);
  }
  if (W == 1) B2H_SEG_LAUNCH(false, 1);
  if (W == 2) B2H_SEG_LAUNCH(false, 2);
  if (W == 3) B2H_SEG_LAUNCH(false, 3);
  B2H_SEG_LAUNCH(false, 4);
#undef B2H_SEG_LAUNCH
}

// ------------------------------------------------------------------------ LZ4 encoder ----
// LZ4_compress_fast (lz4 1.9.3, noDict, limited output; restated in oracle/blosc2_oracle.c
// or_lz4_compress) with acceleration 10 - clevel (blosc/blosc2.c:619-629), one wave per stream,
// hash table in LDS (byU16: 2^13 u16 positions; byU32: 2^12 u32 -- 16 KiB either way).
//
// LZ4's match search probes positions on a schedule fixed in advance: after probe k the walk
// steps by 1 (k = 0) or (accel*64 + k - 1) >> 6, whatever the data.  So a WINDOW of 64 consecutive
// probes is mapped onto the lanes (positions by a prefix sum of the steps): every lane hashes its
// position and reads its table entry at once.  Serially, probe k reads the table after the
// inserts of probes < k, so the window is cut before the first lane whose bucket already occurs
// at an earlier lane (one LDS atomic-or per lane on a bit-per-bucket table); below that cut every
// lane's entry is exact.  The first lane whose candidate matches ends the search; the inserts of
// the lanes up to it are committed (distinct buckets: one store each), the rest are dropped.  The
// sequence after a match (catch-up, literals, offset, match length, the insert at ip - 2 and the
// immediate re-probe) is wave-uniform scalar logic with 64-lane compares and copies.

__device__ __forceinline__ uint32_t lz4_hash_seq(uint32_t lo, uint32_t hi, bool u16tab) {
  if (u16tab) return (lo * 2654435761u) >> (32 - 13);                           // LZ4_hash4, log 12+1
  const uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
  return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));                // LZ4_hash5, log 12
}
__device__ __forceinline__ uint32_t lz4_hash_at(gin_t p, bool u16tab) {
  return lz4_hash_seq(ldu32(p), u16tab ? 0u : ldu32(p + 4), u16tab);
}

template <bool U16>
struct Lz4Lds {
  B2H_LDS uint8_t* base;
  __device__ __forceinline__ int32_t get(uint32_t h) const {
    if (U16) return ((B2H_LDS uint16_t*)base)[h];
    return (int32_t)((B2H_LDS uint32_t*)base)[h];
  }
  __device__ __forceinline__ void put(uint32_t h, int32_t pos) const {
    if (U16) ((B2H_LDS uint16_t*)base)[h] = (uint16_t)pos;
    else ((B2H_LDS uint32_t*)base)[h] = (uint32_t)pos;
  }
};
constexpr int32_t kLz4TabBytes = 16384, kLz4BitsBytes = 1024;

// first index i in [0, lim) with in[a + i] != in[b + i], or lim (64 lanes x 1 byte per step)
__device__ __forceinline__ int32_t wave_common_fwd(gin_t in, int32_t a, int32_t b, int32_t lim) {
  const int lane = lane_id();
  for (int32_t x = 0; x < lim; x += 64) {
    const int32_t i = x + lane;
    const bool diff = i < lim && in[a + i] != in[b + i];
    const uint64_t m = __ballot(diff);
    if (m) return x + __builtin_ctzll(m);
  }
  return lim;
}
// number of bytes k in [0, lim) with in[a - 1 - i] == in[b - 1 - i] for all i <= k (catch-up)
__device__ __forceinline__ int32_t wave_common_back(gin_t in, int32_t a, int32_t b, int32_t lim) {
  const int lane = lane_id();
  for (int32_t x = 0; x < lim; x += 64) {
    const int32_t i = x + lane;
    const bool diff = i < lim && in[a - 1 - i] != in[b - 1 - i];
    const uint64_t m = __ballot(diff);
    if (m) return x + __builtin_ctzll(m);
  }
  return lim;
}
// the same over two sequences a[..] and b[..] (an LZ4 match whose source is the dictionary)
__device__ __forceinline__ int32_t wave_common_fwd2(gin_t a, gin_t b, int32_t lim) {
  const int lane = lane_id();
  for (int32_t x = 0; x < lim; x += 64) {
    const int32_t i = x + lane;
    const bool diff = i < lim && a[i] != b[i];
    const uint64_t m = __ballot(diff);
    if (m) return x + __builtin_ctzll(m);
  }
  return lim;
}
__device__ __forceinline__ int32_t wave_common_back2(gin_t a, gin_t b, int32_t lim) {   // a[-1-i] vs b[-1-i]
  const int lane = lane_id();
  for (int32_t x = 0; x < lim; x += 64) {
    const int32_t i = x + lane;
    const bool diff = i < lim && a[-1 - i] != b[-1 - i];
    const uint64_t m = __ballot(diff);
    if (m) return x + __builtin_ctzll(m);
  }
  return lim;
}
__device__ __forceinline__ void wave_bytes(B2H_GLB uint8_t* o, gin_t s, int32_t n) {
  for (int32_t i = lane_id(); i < n; i += 64) o[i] = s[i];
}
__device__ __forceinline__ void wave_fill255(B2H_GLB uint8_t* o, int32_t n) {
  for (int32_t i = lane_id(); i < n; i += 64) o[i] = 255;
}

// Encode one stream with olimit = n (its own size).  Returns the encoded size, or 0 when an output
// check fails (the stream is then stored raw); *peak = the largest `op + need` tested.
template <bool U16>
__device__ int32_t lz4_encode_wave(gin_t in, int32_t n, int accel, B2H_GLB uint8_t* out, Lz4Lds<U16> tab,
                                   B2H_LDS uint32_t* bits, int32_t* peak_out) {
  constexpr int32_t kMfLimit = 12, kLastLit = 5, kRunMask = 15, kDMax = 65535;
  const int lane = lane_id();
  const int32_t mflimit1 = n - kMfLimit + 1, matchlimit = n - kLastLit;
  int32_t anchor = 0, op = 0, peak = 0;
  bool fail = false;
  auto need = [&](int32_t v) { peak = max(peak, v); return v <= n; };
  {  // LZ4_initStream: zeroed table
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    B2H_LDS u32x4* t = (B2H_LDS u32x4*)tab.base;
    for (int i = lane; i < kLz4TabBytes / 16; i += 64) t[i] = u32x4{0, 0, 0, 0};
    for (int i = lane; i < kLz4BitsBytes / 4; i += 64) bits[i] = 0u;
  }
  if (n >= kMfLimit + 1) {
    if (lane == 0) tab.put(lz4_hash_at(in, U16), 0);
    int32_t ip = 1;
    for (;;) {   // one match search (step schedule restarts) ... one match sequence
      // ---- search: windows of 64 probes ----
      int32_t pos = ip;          // position of the window's first probe
      int32_t k0 = 0;            // its probe index in this search
      int32_t match = 0;
      bool last = false;
      for (;;) {
        const int32_t k = k0 + lane;
        const int32_t stp = k == 0 ? 1 : ((accel << 6) + k - 1) >> 6;   // step after probe k
        const int32_t incl = wave_scan_add(stp);
        const int32_t p = pos + incl - stp;                              // this lane's probe
        const bool valid = p + stp <= mflimit1;                          // else: last literals
        const uint64_t vmask = __ballot(valid);
        const int32_t E = vmask == ~0ull ? 64 : __builtin_ctzll(~vmask);
        uint32_t seq = 0, h = 0;
        if (valid) {
          seq = ldu32(in + p);
          h = lz4_hash_seq(seq, U16 ? 0u : ldu32(in + p + 4), U16);
        }
        int32_t cand = valid ? tab.get(h) : 0;
        uint32_t old = 0;
        if (valid) {
          old = __hip_atomic_fetch_or(&bits[h >> 5], 1u << (h & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          bits[h >> 5] = 0u;
        }
        const uint64_t dup = __ballot(valid && ((old >> (h & 31)) & 1u));
        const int32_t W = min(E, dup ? __builtin_ctzll(dup) : 64);     // exact lanes: [0, W)
        bool ok = false;
        if (lane < W && (U16 || cand + kDMax >= p)) ok = ldu32(in + cand) == seq;
        const uint64_t om = __ballot(ok);
        const int32_t f = om ? __builtin_ctzll(om) : W;                  // lanes [0, f] insert
        if (lane < W && lane <= f) tab.put(h, p);
        if (om) {
          ip = __builtin_amdgcn_readlane(p, f);
          match = __builtin_amdgcn_readlane(cand, f);
          break;
        }
        if (W >= E && E < 64) { last = true; break; }
        pos = __builtin_amdgcn_readlane(p, W - 1) + __builtin_amdgcn_readlane(stp, W - 1);
        k0 += W;
      }
      if (last) break;
      // ---- catch up ----
      {
        const int32_t back = wave_common_back(in, ip, match, min(ip - anchor, match));
        ip -= back;
        match -= back;
      }
      int32_t token = op++;
      uint32_t tokv;
      {
        const int32_t lit = ip - anchor;
        if (!need(op + lit + (2 + 1 + kLastLit) + lit / 255)) { fail = true; break; }
        if (lit >= kRunMask) {
          const int32_t len = lit - kRunMask;
          tokv = kRunMask << 4;
          wave_fill255(out + op, len / 255);
          op += len / 255;
          if (lane == 0) out[op] = (uint8_t)(len % 255);
          op++;
        } else {
          tokv = (uint32_t)lit << 4;
        }
        if (lit > 64) wave_copy(out + op, in + anchor, lit);
        else wave_bytes(out + op, in + anchor, lit);
        op += lit;
      }
      bool done = false;
      for (;;) {   // _next_match
        const int32_t d = ip - match;
        if (lane == 0) { out[op] = (uint8_t)d; out[op + 1] = (uint8_t)(d >> 8); }
        op += 2;
        int32_t mc = wave_common_fwd(in, ip + 4, match + 4, max(0, matchlimit - (ip + 4)));
        ip += mc + 4;
        if (!need(op + (1 + kLastLit) + (mc + 240) / 255)) { fail = true; break; }
        if (mc >= 15) {
          tokv += 15;
          mc -= 15;
          wave_fill255(out + op, mc / 255);
          op += mc / 255;
          if (lane == 0) out[op] = (uint8_t)(mc % 255);
          op++;
        } else {
          tokv += (uint32_t)mc;
        }
        if (lane == 0) out[token] = (uint8_t)tokv;
        anchor = ip;
        if (ip >= mflimit1) { done = true; break; }
        if (lane == 0) tab.put(lz4_hash_at(in + ip - 2, U16), ip - 2);
        const uint32_t h = lz4_hash_at(in + ip, U16);
        const int32_t mi = tab.get(h);
        if (lane == 0) tab.put(h, ip);
        if ((U16 || mi + kDMax >= ip) && ldu32(in + mi) == ldu32(in + ip)) {
          match = mi;
          token = op++;
          tokv = 0;
          continue;
        }
        break;
      }
      if (fail || done) break;
      ip++;
    }
  }
  if (!fail) {
    const int32_t last = n - anchor;
    if (!need(op + last + 1 + (last + 255 - kRunMask) / 255)) {
      fail = true;
    } else {
      if (last >= kRunMask) {
        const int32_t acc = last - kRunMask;
        if (lane == 0) out[op] = kRunMask << 4;
        op++;
        wave_fill255(out + op, acc / 255);
        op += acc / 255;
        if (lane == 0) out[op] = (uint8_t)(acc % 255);
        op++;
      } else {
        if (lane == 0) out[op] = (uint8_t)(last << 4);
        op++;
      }
      if (last > 64) wave_copy(out + op, in + anchor, last);
      else wave_bytes(out + op, in + anchor, last);
      op += last;
    }
  }
  *peak_out = peak;
  return fail ? 0 : op;
}

// LZ4_loadDict(dict, dsz) + LZ4_compress_fast_continue, external-dictionary mode (lz4 1.9.3; the
// call sequence of lz4_wrap_compress with a dictionary, blosc/blosc2.c:455-465; restated in
// oracle/blosc2_oracle.c or_lz4_compress_dict and pinned to the reference there).  The same
// window search as lz4_encode_wave (byU32 table, hash5), on 32-bit indices: the dictionary's byte
// d is index 65536 - dsz + d, the stream's byte i is 65536 + i; the dictionary's positions 0, 3,
// 6, ... are inserted first (lanes of one store apply in lane order: the later position wins, as
// serially); candidates below 65536 - dsz (empty slots) or farther than 65535 are skipped; a
// match found in the dictionary extends to its end and then on from the stream's start.
__device__ int32_t lz4_encode_wave_dict(gin_t in, int32_t n, int accel, B2H_GLB uint8_t* out, Lz4Lds<false> tab,
                                        B2H_LDS uint32_t* bits, int32_t* peak_out, gin_t dict, int32_t dsz) {
  constexpr int32_t kMfLimit = 12, kLastLit = 5, kRunMask = 15, kDMax = 65535;
  constexpr uint32_t kStart = 65536;
  const int lane = lane_id();
  const uint32_t dict0 = kStart - (uint32_t)dsz;   // index of dict[0]; below it: empty slots
  const int32_t mflimit1 = n - kMfLimit + 1, matchlimit = n - kLastLit;
  int32_t anchor = 0, op = 0, peak = 0;
  bool fail = false;
  auto need = [&](int32_t v) { peak = max(peak, v); return v <= n; };
  auto at = [&](uint32_t idx) -> gin_t { return idx < kStart ? dict + (idx - dict0) : in + (idx - kStart); };
  {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    B2H_LDS u32x4* t = (B2H_LDS u32x4*)tab.base;
    for (int i = lane; i < kLz4TabBytes / 16; i += 64) t[i] = u32x4{0, 0, 0, 0};
    for (int i = lane; i < kLz4BitsBytes / 4; i += 64) bits[i] = 0u;
    for (int32_t base = 0; 3 * base <= dsz - 8; base += 64) {   // LZ4_loadDict
      // an atomic exchange per lane: the lanes of one LDS atomic apply in lane order, so of two
      // positions with one bucket the later (higher lane) stays, as in the serial insert loop
      const int32_t p = 3 * (base + lane);
      if (p <= dsz - 8)
        (void)__hip_atomic_exchange(&((B2H_LDS uint32_t*)tab.base)[lz4_hash_at(dict + p, false)], dict0 + (uint32_t)p,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  if (n >= kMfLimit + 1) {
    if (lane == 0) tab.put(lz4_hash_at(in, false), (int32_t)kStart);
    int32_t ip = 1;
    for (;;) {
      int32_t pos = ip, k0 = 0;
      uint32_t midx = 0;
      bool last = false;
      for (;;) {
        const int32_t k = k0 + lane;
        const int32_t stp = k == 0 ? 1 : ((accel << 6) + k - 1) >> 6;
        const int32_t incl = wave_scan_add(stp);
        const int32_t p = pos + incl - stp;
        const bool valid = p + stp <= mflimit1;
        const uint64_t vmask = __ballot(valid);
        const int32_t E = vmask == ~0ull ? 64 : __builtin_ctzll(~vmask);
        uint32_t seq = 0, h = 0;
        if (valid) {
          seq = ldu32(in + p);
          h = lz4_hash_seq(seq, ldu32(in + p + 4), false);
        }
        const uint32_t cand = valid ? (uint32_t)tab.get(h) : 0u;
        uint32_t old = 0;
        if (valid) {
          old = __hip_atomic_fetch_or(&bits[h >> 5], 1u << (h & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          bits[h >> 5] = 0u;
        }
        const uint64_t dup = __ballot(valid && ((old >> (h & 31)) & 1u));
        const int32_t W = min(E, dup ? __builtin_ctzll(dup) : 64);
        const uint32_t cur = kStart + (uint32_t)p;
        bool ok = false;
        if (lane < W && cand >= dict0 && cand + kDMax >= cur) ok = ldu32(at(cand)) == seq;
        const uint64_t om = __ballot(ok);
        const int32_t f = om ? __builtin_ctzll(om) : W;
        if (lane < W && lane <= f) tab.put(h, (int32_t)cur);
        if (om) {
          ip = __builtin_amdgcn_readlane(p, f);
          midx = (uint32_t)__builtin_amdgcn_readlane((int32_t)cand, f);
          break;
        }
        if (W >= E && E < 64) { last = true; break; }
        pos = __builtin_amdgcn_readlane(p, W - 1) + __builtin_amdgcn_readlane(stp, W - 1);
        k0 += W;
      }
      if (last) break;
      {   // catch up, not below the start of the match's segment
        const bool md = midx < kStart;
        const int32_t mpos = md ? (int32_t)(midx - dict0) : (int32_t)(midx - kStart);
        const int32_t back = wave_common_back2(in + ip, (md ? dict : in) + mpos, min(ip - anchor, mpos));
        ip -= back;
        midx -= (uint32_t)back;
      }
      int32_t token = op++;
      uint32_t tokv;
      {
        const int32_t lit = ip - anchor;
        if (!need(op + lit + (2 + 1 + kLastLit) + lit / 255)) { fail = true; break; }
        if (lit >= kRunMask) {
          const int32_t len = lit - kRunMask;
          tokv = kRunMask << 4;
          wave_fill255(out + op, len / 255);
          op += len / 255;
          if (lane == 0) out[op] = (uint8_t)(len % 255);
          op++;
        } else {
          tokv = (uint32_t)lit << 4;
        }
        if (lit > 64) wave_copy(out + op, in + anchor, lit);
        else wave_bytes(out + op, in + anchor, lit);
        op += lit;
      }
      bool done = false;
      for (;;) {   // _next_match
        const uint32_t d = kStart + (uint32_t)ip - midx;
        if (lane == 0) { out[op] = (uint8_t)d; out[op + 1] = (uint8_t)(d >> 8); }
        op += 2;
        int32_t mc;
        if (midx < kStart) {   // in the dictionary: up to its end, then on from the stream's start
          const int32_t mpos = (int32_t)(midx - dict0);
          const int32_t limit = min(ip + (dsz - mpos), matchlimit);
          mc = wave_common_fwd2(in + ip + 4, dict + mpos + 4, max(0, limit - (ip + 4)));
          ip += mc + 4;
          if (ip == limit) {
            const int32_t more = wave_common_fwd2(in + limit, in, max(0, matchlimit - limit));
            mc += more;
            ip += more;
          }
        } else {
          const int32_t mpos = (int32_t)(midx - kStart);
          mc = wave_common_fwd(in, ip + 4, mpos + 4, max(0, matchlimit - (ip + 4)));
          ip += mc + 4;
        }
        if (!need(op + (1 + kLastLit) + (mc + 240) / 255)) { fail = true; break; }
        if (mc >= 15) {
          tokv += 15;
          mc -= 15;
          wave_fill255(out + op, mc / 255);
          op += mc / 255;
          if (lane == 0) out[op] = (uint8_t)(mc % 255);
          op++;
        } else {
          tokv += (uint32_t)mc;
        }
        if (lane == 0) out[token] = (uint8_t)tokv;
        anchor = ip;
        if (ip >= mflimit1) { done = true; break; }
        if (lane == 0) tab.put(lz4_hash_at(in + ip - 2, false), (int32_t)(kStart + (uint32_t)(ip - 2)));
        const uint32_t h = lz4_hash_at(in + ip, false);
        const uint32_t mi = (uint32_t)tab.get(h);
        const uint32_t cur = kStart + (uint32_t)ip;
        if (lane == 0) tab.put(h, (int32_t)cur);
        if (mi >= dict0 && mi + kDMax >= cur && ldu32(at(mi)) == ldu32(in + ip)) {
          midx = mi;
          token = op++;
          tokv = 0;
          continue;
        }
        break;
      }
      if (fail || done) break;
      ip++;
    }
  }
  if (!fail) {
    const int32_t last = n - anchor;
    if (!need(op + last + 1 + (last + 255 - kRunMask) / 255)) {
      fail = true;
    } else {
      if (last >= kRunMask) {
        const int32_t acc = last - kRunMask;
        if (lane == 0) out[op] = kRunMask << 4;
        op++;
        wave_fill255(out + op, acc / 255);
        op += acc / 255;
        if (lane == 0) out[op] = (uint8_t)(acc % 255);
        op++;
      } else {
        if (lane == 0) out[op] = (uint8_t)(last << 4);
        op++;
      }
      if (last > 64) wave_copy(out + op, in + anchor, last);
      else wave_bytes(out + op, in + anchor, last);
      op += last;
    }
  }
  *peak_out = peak;
  return fail ? 0 : op;
}

// The dictionary section of a chunk's output ([int32 size | bytes] after the bstarts, blosc/blosc2.c:
// 3202-3221): the first dict_size bytes of the training pass's image -- the filtered blocks in
// order, which is the filtered image -- as they lie once the size word has been stored over four of
// them (the samples start at the bstarts and are moved behind the size word, 3205-3210).
__global__ void k_put_dict(CGeom g, const uint8_t* __restrict__ filt, uint8_t* __restrict__ dst) {
  const int32_t c = blockIdx.x;
  uint8_t* d = dst + (int64_t)c * g.dst_stride + g.overhead + 4 * g.nblocks;
  const uint8_t* f = filt + (int64_t)c * g.wstride;
  const int32_t dsz = g.dict_size, w = 4 * g.nblocks;
  for (int32_t i = threadIdx.x; i < dsz + 4; i += blockDim.x) {
    uint8_t v;
    if (i < 4) v = (uint8_t)((uint32_t)dsz >> (8 * i));
    else if (i - 4 >= w && i - 4 < w + 4) v = (uint8_t)((uint32_t)dsz >> (8 * (i - 4 - w)));
    else v = f[i - 4];
    d[i] = v;
  }
}

__global__ __launch_bounds__(64) void k_encode_lz4(CGeom g, const uint8_t* __restrict__ filt, uint8_t* __restrict__ sbuf,
                                                   StreamResult* __restrict__ res, int32_t nstreams_total,
                                                   int32_t* __restrict__ next, const uint8_t* __restrict__ dst) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* lds = (B2H_LDS uint8_t*)smem;
  B2H_LDS uint32_t* bits = (B2H_LDS uint32_t*)(lds + kLz4TabBytes);
  const int accel = 10 - g.clevel;
  for (;;) {
    const int32_t s = __builtin_amdgcn_readfirstlane(atomicAdd(next, lane_id() == 0 ? 1 : 0));
    if (s >= nstreams_total) return;
    const int32_t c = s / g.nsc, l = s - c * g.nsc;
    int32_t off, len, blk;
    stream_locate(g, l, &off, &len, &blk);
    gin_t in = (gin_t)(filt + (int64_t)c * g.wstride + off);
    B2H_GLB uint8_t* out = (B2H_GLB uint8_t*)(sbuf + (int64_t)c * g.wstride + off);
    StreamResult r;
    r.windows = 0;
    r.cycles = 0;
    r.t_start = 0;
    r.peak = 0;
    r.size = 0;
    if (g.overhead == kHdrExt && wave_is_run(in, len)) {
      r.size = in[0];
      r.kind = r.size ? kStreamByteRun : kStreamZeroRun;
    } else {
      int32_t peak = 0;
      int32_t cb;
      if (g.dict_size > 0) {   // LZ4_compress_fast_continue: byU32 whatever the length
        Lz4Lds<false> t{lds};
        gin_t dict = (gin_t)(dst + (int64_t)c * g.dst_stride + g.overhead + 4 * g.nblocks + 4);
        cb = lz4_encode_wave_dict(in, len, accel, out, t, bits, &peak, dict, g.dict_size);
      } else if (len < 65536 + 11) {
        Lz4Lds<true> t{lds};
        cb = lz4_encode_wave<true>(in, len, accel, out, t, bits, &peak);
      } else {
        Lz4Lds<false> t{lds};
        cb = lz4_encode_wave<false>(in, len, accel, out, t, bits, &peak);
      }
      r.kind = cb > 0 ? kStreamLz : kStreamRaw;
      r.size = cb;
      r.peak = peak;
    }
    if (lane_id() == 0) res[s] = r;
  }
}

static int launch_encode_lz4(Workspace* ws, const CGeom& g, const uint8_t* filt, StreamResult* res, int64_t ntot,
                             int32_t* next, hipStream_t st, uint8_t* d_dst) {
  (void)ws;
  const size_t lds = kLz4TabBytes + kLz4BitsBytes;
  int dev = 0, ncu = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(&k_encode_lz4), 64, lds) !=
      hipSuccess) per_cu = 1;
  const int64_t slots = (int64_t)std::max(1, per_cu) * std::max(1, ncu);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(ntot, slots));
  k_encode_lz4<<<grid, 64, lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot, next, d_dst);
  HIPCHK(hipGetLastError());
  return 0;
}

struct Place {
  int32_t off;    // payload offset inside the chunk output (csize word sits at off - 4)
  int32_t csize;  // csize word
};

// Serial reference bookkeeping per chunk (blosc/blosc2.c:1277-1466, 2161-2228, 3004-3107).
// mode: 0 compressed, 1 memcpy fallback, 2 special zero, 3 does not fit.
// One lane: `ld(l)` gives stream l's StreamResult (kind, size, peak), `put(l, off, csize)` takes its
// placement; writes the header and bstarts of chunk output `d`; returns the mode, *cb_out = cbytes.
template <typename LD, typename PUT>
__device__ __forceinline__ int32_t finalize_chunk(const CGeom& g, uint8_t* __restrict__ d,
                                                  const uint8_t* __restrict__ header_template, LD ld, PUT put,
                                                  int32_t* cb_out) {
  const int32_t ovh = g.overhead;
  int32_t ntbytes = ovh + 4 * g.nblocks + (g.dict_size ? 4 + g.dict_size : 0);
  const int32_t destsize = g.destsize;
  bool ok = true, all_zero = true;
  int32_t l = 0;
  for (int32_t b = 0; b < g.nblocks && ok; b++) {
    const bool lo = (b == g.nblocks - 1) && g.leftover;
    const int32_t ns = lo ? 1 : g.spb;
    const int32_t nl = lo ? g.leftover : g.neblock;
    int32_t bstart = ntbytes;
    uint8_t* bs = d + ovh + 4 * b;
    bs[0] = (uint8_t)bstart; bs[1] = (uint8_t)(bstart >> 8); bs[2] = (uint8_t)(bstart >> 16); bs[3] = (uint8_t)(bstart >> 24);
    for (int32_t j = 0; j < ns; j++, l++) {
      const StreamResult sr = ld(l);
      ntbytes += 4;
      if (sr.kind == kStreamZeroRun || sr.kind == kStreamByteRun) {
        if (ntbytes > destsize) { ok = false; break; }
        put(l, ntbytes, -sr.size);
        if (sr.size) {
          all_zero = false;
          ntbytes += 1;
          if (ntbytes > destsize) { ok = false; break; }
        }
        continue;
      }
      all_zero = false;
      int32_t maxout = nl;
      if (ntbytes + maxout > destsize) {
        maxout = destsize - ntbytes;
        if (maxout <= 0) { ok = false; break; }
      }
      // BloscLZ returns 0 below maxout 66 (blosc/blosclz.c:480-482); LZ4's limited-output checks
      // are all captured by `peak`
      int32_t cb = (sr.kind == kStreamLz && (g.compcode == 1 || maxout >= 66) && sr.peak <= maxout) ? sr.size : 0;
      if (cb == 0) cb = nl;
      if (cb == nl && ntbytes + nl > destsize) { ok = false; break; }
      put(l, ntbytes, cb);   // cb == nl means raw copy
      ntbytes += cb;
    }
  }
  // header (template already holds flags/typesize/nbytes/blocksize/filters)
  for (int i = 0; i < ovh; i++) d[i] = header_template[i];
  int32_t m, cb;
  if (ok) {
    const int32_t nstreams = g.nsc;
    if (all_zero && !g.dict_size && ntbytes == ovh + 4 * g.nblocks + 4 * nstreams) {
      m = 2;
      cb = ovh;
      d[31] |= (uint8_t)(kSpecialZero << 4);
    } else {
      m = 0;
      cb = ntbytes;
    }
  } else if (g.nbytes + ovh <= destsize) {
    m = 1;
    cb = g.nbytes + ovh;
    d[2] |= kFlagMemcpy;
  } else {
    m = 3;
    cb = 0;
  }
  d[12] = (uint8_t)cb; d[13] = (uint8_t)(cb >> 8); d[14] = (uint8_t)(cb >> 16); d[15] = (uint8_t)(cb >> 24);
  *cb_out = cb;
  return m;
}

__global__ void k_finalize(CGeom g, const StreamResult* __restrict__ res, Place* __restrict__ place,
                           int32_t* __restrict__ mode, uint8_t* __restrict__ dst, int32_t* __restrict__ cbytes,
                           int32_t nchunks, const uint8_t* __restrict__ header_template) {
  if (gated_off(g)) return;
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= nchunks) return;
  const StreamResult* r = res + (int64_t)c * g.nsc;
  Place* pl = place + (int64_t)c * g.nsc;
  int32_t cb = 0;
  mode[c] = finalize_chunk(
      g, dst + (int64_t)c * g.dst_stride, header_template, [&](int32_t l) { return r[l]; },
      [&](int32_t l, int32_t off, int32_t csize) { pl[l].off = off; pl[l].csize = csize; }, &cb);
  cbytes[c] = cb;
}

// Workgroup copy of n bytes to an arbitrarily aligned destination: aligned u32 stores, sources
// read with ldu32 (unaligned ok, slack guaranteed by the scratch layout).
__device__ void wg_copy(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, int32_t n) {
  const int32_t head = (int32_t)((4 - (reinterpret_cast<uintptr_t>(d) & 3)) & 3);
  const int32_t h = min(head, n);
  if ((int32_t)threadIdx.x < h) d[threadIdx.x] = s[threadIdx.x];
  const int32_t body = (n - h) / 4;
  uint32_t* d4 = reinterpret_cast<uint32_t*>(d + h);
  const uint8_t* s4 = s + h;
  if ((reinterpret_cast<uintptr_t>(s4) & 3) == 0) {
    const uint32_t* a = reinterpret_cast<const uint32_t*>(s4);
    for (int32_t i = threadIdx.x; i < body; i += blockDim.x) d4[i] = a[i];
  } else {
    for (int32_t i = threadIdx.x; i < body; i += blockDim.x) d4[i] = ldu32((gin_t)(s4 + 4 * i));
  }
  for (int32_t i = h + body * 4 + threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

__global__ __launch_bounds__(kBlockThreads) void k_scatter(CGeom g, const Place* __restrict__ place,
                                                           const int32_t* __restrict__ mode,
                                                           const StreamResult* __restrict__ res,
                                                           const uint8_t* __restrict__ filt,
                                                           const uint8_t* __restrict__ sbuf, uint8_t* __restrict__ dst,
                                                           int32_t nstreams_total) {
  if (gated_off(g)) return;
  for (int32_t s = blockIdx.x; s < nstreams_total; s += gridDim.x) {   // grid: min(streams, kScatterGrid)
    const int32_t c = s / g.nsc, l = s - c * g.nsc;
    if (mode[c] != 0) continue;
    int32_t off, len, blk;
    stream_locate(g, l, &off, &len, &blk);
    const Place pl = place[s];
    uint8_t* d = dst + (int64_t)c * g.dst_stride;
    if (threadIdx.x == 0) {
      const uint32_t w = (uint32_t)pl.csize;
      uint8_t* q = d + pl.off - 4;
      q[0] = (uint8_t)w; q[1] = (uint8_t)(w >> 8); q[2] = (uint8_t)(w >> 16); q[3] = (uint8_t)(w >> 24);
      if (pl.csize < 0) d[pl.off] = 0x1;   // run-length token
    }
    if (pl.csize <= 0) continue;
    const uint8_t* src = (pl.csize == len) ? filt + (int64_t)c * g.wstride + off : sbuf + (int64_t)c * g.wstride + off;
    // each wave moves a contiguous quarter with 16-byte aligned stores (wave_copy)
    const int32_t nw = kBlockThreads / 64, w = threadIdx.x >> 6;
    const int32_t q = ((pl.csize + nw - 1) / nw + 15) & ~15;
    const int32_t a = min(pl.csize, w * q), b = min(pl.csize, a + q);
    if (b > a) wave_copy((gout_t)(d + pl.off + a), (gin_t)(src + a), b - a);
  }
}
constexpr int32_t kScatterGrid = 16384;

// memcpyed chunks: header + raw bytes.  `only_mode1`: fallback chunks only (mode[] == 1).
__global__ void k_memcpy_chunks(const uint8_t* __restrict__ src, int64_t src_stride, uint8_t* __restrict__ dst,
                                int64_t dst_stride, int32_t nbytes, const int32_t* __restrict__ mode,
                                const uint8_t* __restrict__ header_template, int32_t* __restrict__ cbytes,
                                int32_t overhead, int32_t destsize, const int32_t* __restrict__ gate, int32_t nchunks) {
  if (gate && __builtin_amdgcn_readfirstlane(__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0)
    return;
  for (int32_t c = blockIdx.y; c < nchunks; c += gridDim.y) {   // grid.y: min(chunks, kMemcpyGridY)
    if (mode && mode[c] != 1) continue;
    const uint8_t* s = src + (int64_t)c * src_stride;
    uint8_t* d = dst + (int64_t)c * dst_stride;
    const bool fits = nbytes + overhead <= destsize;
    if (!mode && blockIdx.x == 0 && (int32_t)threadIdx.x < overhead) {
      // memcpyed from the start: header written here; cbytes 0 when it cannot fit
      // (blosc/blosc2.c:3038-3041)
      uint8_t v = header_template[threadIdx.x];
      const int32_t cb = fits ? nbytes + overhead : 0;
      if (threadIdx.x >= 12 && threadIdx.x < 16) v = (uint8_t)(cb >> (8 * (threadIdx.x - 12)));
      d[threadIdx.x] = v;
      if (threadIdx.x == 0) cbytes[c] = cb;
    }
    if (!fits) continue;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x)
      d[overhead + i] = s[i];
  }
}
constexpr int32_t kMemcpyGridY = 256;

// ------------------------------------- fast mode, one launch: shuffle -> encode -> finalize/scatter ----
// k_encode_fast with the passes on either side of it moved inside the launch, so that their HBM
// traffic runs in the shadow of the latency-bound encoder instead of as launches of their own:
//   * SHUFFLE jobs (f.raw != null; the lone filter is a typesize-4 byte shuffle, whole 64-byte
//     groups): before encoding a stream the workgroup makes sure every block up to the stream's own
//     + f.lead has been claimed (one atomic counter, blocks in chunk-major order), shuffles the
//     blocks it claimed, then waits for its stream's block;
//   * FINALIZE: the workgroup whose stream completes a chunk (per-chunk counter) runs the serial
//     layout bookkeeping of k_finalize for it and publishes the chunk in a ready list;
//   * SCATTER items (one per stream of a published chunk): claimed between streams while
//     available, and by every workgroup once the stream queue is empty (k_scatter's work).
// Hand-offs follow MI355X_MICROARCH.md § inter-workgroup visibility: every handed-off byte is stored
// write-through (sc1: the shuffled planes, the encoder's ring flushes, the placement words), each
// storing wave drains (vmcnt 0) before the workgroup barrier behind which one lane signals with an
// agent-scope atomic; consumers poll relaxed; the encoder reads its block with plain loads behind an
// agent acquire, the scatter reads its payload with sc1 loads.  Every wait is bounded (1 s; a
// timeout sets sync[4], reported as E_FAILURE by the host at its next synchronisation).
struct EncFuse {
  const uint8_t* raw;      // SHUFFLE source (null: `filt` is already filtered)
  int64_t raw_stride;
  uint8_t* filt;           // shuffle output = the encoder's input, stride g.wstride
  int32_t* sync;           // zeroed per launch: kFuseHdr words, blk_ready[nblk], chunk_cnt[nchunks], ready[nchunks]
  int32_t* fin;            // per stream: kind, size, peak (sc1)
  Place* place;
  int32_t* mode;
  uint8_t* dst;
  int32_t* cbytes;
  const uint8_t* htpl;
  int32_t nchunks, lead;
  int32_t* trace;          // debug (B2H_FUSE_TRACE): per workgroup, the phase it is in (host memory)
  int32_t mode_bits;       // fuse_bits()
  int32_t ds;              // raw's filter job: 0 the typesize-4 SHUFFLE, 2/4/8 (DELTA, SHUFFLE) at that typesize
};
// B2H_SEG_PROF (diagnostics build): the fused fast launch's per-phase clock, thread 0 of each
// workgroup into g_seg_prof[16..25] (b2h_debug_seg_prof): 16 filter-job cycles, 17 ready-word
// waits, 18 stream encodes, 19 job store drains, 20 jobs, 21 streams encoded, 22 / 23 the DS job's
// verdict / store pass, 24 scatter items
#ifdef B2H_SEG_PROF
#define FPROF_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define FPROF_ADD(i, a, b) do { if (threadIdx.x == 0) atomicAdd(&g_seg_prof[(i)], (unsigned long long)((b) - (a))); } while (0)
#define FPROF_CNT(i) do { if (threadIdx.x == 0) atomicAdd(&g_seg_prof[(i)], 1ull); } while (0)
#else
#define FPROF_T(v)
#define FPROF_ADD(i, a, b)
#define FPROF_CNT(i)
#endif
constexpr int32_t kFuseHdr = 16;   // [0] shuffle claims [1] scatter claims [2] ready slots [3] published items [4] timeouts
constexpr int32_t kFuseSpi = 8;    // streams per scatter item

typedef B2H_GLB int32_t* gi32_t;
__device__ __forceinline__ void st_agent(int32_t* p, int32_t v) {
  __hip_atomic_store((gi32_t)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t add_agent(int32_t* p, int32_t v) {
  return __hip_atomic_fetch_add((gi32_t)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// counters and flags are read with an atomic read-modify-write (performed where the atomics are),
// never with a load that a cache might serve
__device__ __forceinline__ int32_t rd_agent(int32_t* p) { return add_agent(p, 0); }
// one lane: poll *p until non-zero, bounded (~1 s or 2^21 polls); 0 on timeout (flagged in *tmo)
__device__ int32_t wait_nonzero(int32_t* p, int32_t* tmo) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int32_t it = 0; it < (1 << 21); it++) {
    const int32_t v = rd_agent(p);
    if (v) return v;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) break;   // 100 MHz clock
    __builtin_amdgcn_s_sleep(8);
  }
  st_agent(tmo, 1);
  return 0;
}
__device__ __forceinline__ void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
#define FUSE_TRACE(code, v)                                                                                  \
  do {                                                                                                     \
    int32_t* tr_ = FUSE_TRACE_PTR;                                                                         \
    if (tr_ && threadIdx.x == 0)                                                                            \
      __hip_atomic_store(tr_ + blockIdx.x, (int32_t)((code) | ((v) << 4)), __ATOMIC_RELAXED,                \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                                        \
  } while (0)
#define FUSE_TRACE_PTR f.trace

// Typesize-4 byte shuffle of one block by the workgroup (bsize % 64 == 0, s and d 16-aligned):
// 16 elements per lane step, 4 x 16 B loads, a 4x4 byte transpose per 4 elements (v_perm), one
// 16 B write-through store per plane.
__device__ __forceinline__ void tr4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t (&o)[4]) {
  const uint32_t t0 = __builtin_amdgcn_perm(b, a, 0x06020400u), t1 = __builtin_amdgcn_perm(b, a, 0x07030501u);
  const uint32_t t2 = __builtin_amdgcn_perm(d, c, 0x06020400u), t3 = __builtin_amdgcn_perm(d, c, 0x07030501u);
  o[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);
  o[2] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);
  o[1] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);
  o[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);
}
__device__ void shuffle4_block_wt(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int32_t bsize,
                                  int32_t tid = threadIdx.x, int32_t nth = blockDim.x) {
  const int32_t n = bsize / 4, groups = n / 16;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc((gout_t)d);
  const uint4* s4 = reinterpret_cast<const uint4*>(s);
  constexpr int U = 2;
  for (int32_t g0 = tid; g0 < groups; g0 += U * nth) {
    uint4 w[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t gi = g0 + u * nth;
#pragma unroll
      for (int k = 0; k < 4; k++) w[u][k] = gi < groups ? s4[4 * gi + k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t gi = g0 + u * nth;
      if (gi >= groups) break;
      uint32_t o[4][4];   // [element quad k][plane]
#pragma unroll
      for (int k = 0; k < 4; k++) tr4(w[u][k].x, w[u][k].y, w[u][k].z, w[u][k].w, o[k]);
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const u32x4 v = {o[0][p], o[1][p], o[2][p], o[3][p]};
        __builtin_amdgcn_raw_buffer_store_b128(v, r, p * n + 16 * gi, 0, 16);
      }
    }
  }
}

// shuffle4_block_wt deciding the run verdict on the way, as ds_block_runs does for (DELTA,
// SHUFFLE) -- but in one pass: every plane is stored and the mismatches against each plane's first
// byte (byte p of the block's first element) ORed in LDS word `red`.  Returns the run planes; the
// encoder then skips their streams and the run test of the others.  Whole 64-byte groups (the
// caller checks).  WG: the workgroup calls it together; else one wave (tid = lane, nth = 64, no
// LDS word).
template <bool WG>
__device__ __noinline__ uint32_t shuffle4_block_runs(const uint8_t* __restrict__ s, uint8_t* __restrict__ d, int32_t bsize,
                                                     B2H_LDS uint32_t* red, int32_t tid, int32_t nth) {
  const int32_t n = bsize / 4, groups = n / 16;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc((gout_t)d);
  const uint4* s4 = reinterpret_cast<const uint4*>(s);
  uint32_t rep[4];
#pragma unroll
  for (int p = 0; p < 4; p++) rep[p] = 0x01010101u * (uint32_t)s[p];
  if constexpr (WG) {
    if (tid == 0) *red = 0u;
    __syncthreads();
  }
  uint32_t mis = 0;
  constexpr int U = 2;
  for (int32_t g0 = tid; g0 < groups; g0 += U * nth) {
    uint4 w[U][4];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t gi = g0 + u * nth;
#pragma unroll
      for (int k = 0; k < 4; k++) w[u][k] = gi < groups ? s4[4 * gi + k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const int32_t gi = g0 + u * nth;
      if (gi >= groups) break;
      uint32_t o[4][4];
#pragma unroll
      for (int k = 0; k < 4; k++) tr4(w[u][k].x, w[u][k].y, w[u][k].z, w[u][k].w, o[k]);
#pragma unroll
      for (int p = 0; p < 4; p++) {
        const u32x4 v = {o[0][p], o[1][p], o[2][p], o[3][p]};
        mis |= (((v.x != rep[p]) | (v.y != rep[p]) | (v.z != rep[p]) | (v.w != rep[p])) ? 1u : 0u) << p;
        __builtin_amdgcn_raw_buffer_store_b128(v, r, p * n + 16 * gi, 0, 16);
      }
    }
  }
  uint32_t wm = 0;
#pragma unroll
  for (int p = 0; p < 4; p++) wm |= __ballot((mis >> p) & 1u) ? (1u << p) : 0u;
  if constexpr (!WG) return ~wm & 15u;
  if ((tid & 63) == 0 && wm) __hip_atomic_fetch_or(red, wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  const uint32_t M = __builtin_amdgcn_readfirstlane(*red);
  __syncthreads();
  return ~M & 15u;
}

// (DELTA, SHUFFLE) of one block by the workgroup (or one wave: tid / nth), the planes' dwords
// stored write-through: the fused launch's filter job for k_ffilter_ds's pipeline (the same
// arithmetic as delta_shuffle_fast: block 0 XORs each element with the previous one, the other
// blocks with the same element of the chunk's raw block 0, blosc/delta.c:18-92; then the byte
// shuffle, shuffle-generic.h:34-55).  Whole quads, 16-byte aligned (checked by the host).
template <int TS>
__device__ void ds_block_wt(const uint8_t* __restrict__ src, const uint8_t* __restrict__ dref, uint8_t* __restrict__ dst,
                            int32_t n, bool first_block, int32_t tid, int32_t nth) {
  const int32_t quads = n / 4;
  const __amdgpu_buffer_rsrc_t r = wt_rsrc((gout_t)dst);
  constexpr int EW = TS / 4 > 0 ? TS / 4 : 1;   // u32 words per element (TS 2: half a word)
  for (int32_t q = tid; q < quads; q += nth) {
    uint32_t w[TS], x[TS];
    load_words<TS>(src, q, w);
    if (first_block) {
      if constexpr (TS == 2) {
        const uint32_t pe = q ? (uint32_t)reinterpret_cast<const uint16_t*>(src)[4 * (int64_t)q - 1] : 0u;
        x[0] = (w[0] << 16) | pe;
        x[1] = (w[1] << 16) | (w[0] >> 16);
      } else {
        uint32_t prev[EW];
#pragma unroll
        for (int k = 0; k < EW; k++) prev[k] = q ? reinterpret_cast<const uint32_t*>(src)[(int64_t)q * TS - EW + k] : 0u;
#pragma unroll
        for (int k = 0; k < TS; k++) x[k] = k < EW ? prev[k] : w[k - EW];
      }
    } else {
      load_words<TS>(dref, q, x);
    }
#pragma unroll
    for (int k = 0; k < TS; k++) w[k] ^= x[k];
#pragma unroll
    for (int plane = 0; plane < TS; plane++) {
      uint32_t o = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int byte = e * TS + plane;
        o |= ((w[byte / 4] >> (8 * (byte % 4))) & 0xffu) << (8 * e);
      }
      __builtin_amdgcn_raw_buffer_store_b32(o, r, plane * n + 4 * q, 0, 16);
    }
  }
}

// The same job over a whole split block, deciding the run verdict on the way (VERDICT r4 item 3,
// blosc_c's per-stream run test, blosc/blosc2.c:1296-1340): a pass over the block computes every
// plane, compared with its first byte (byte j of the block's first element after DELTA); the
// workgroup ORs the mismatches (LDS word `red`), and a second pass writes only the planes that are
// not runs.  Returns the run planes (bit j: plane j's stream is a run of byte j of element 0) --
// the encoder never reads them.  A block of runs only (C4's blocks after the first) is read once
// and writes nothing.  The workgroup calls it together (tid / nth = its threads).
template <int TS>
__device__ uint32_t ds_block_runs(const uint8_t* __restrict__ src, const uint8_t* __restrict__ dref, uint8_t* __restrict__ dst,
                                  int32_t n, bool first_block, int32_t tid, int32_t nth, B2H_LDS uint32_t* red) {
  const int32_t quads = n / 4;
  uint32_t rep[TS];
#pragma unroll
  for (int p = 0; p < TS; p++) rep[p] = 0x01010101u * (uint32_t)(src[p] ^ (first_block ? 0 : dref[p]));
  constexpr int EW = TS / 4 > 0 ? TS / 4 : 1;
  auto planes = [&](int32_t q, uint32_t (&o)[TS]) {
    uint32_t w[TS], x[TS];
    load_words<TS>(src, q, w);
    if (first_block) {
      if constexpr (TS == 2) {
        const uint32_t pe = q ? (uint32_t)reinterpret_cast<const uint16_t*>(src)[4 * (int64_t)q - 1] : 0u;
        x[0] = (w[0] << 16) | pe;
        x[1] = (w[1] << 16) | (w[0] >> 16);
      } else {
        uint32_t prev[EW];
#pragma unroll
        for (int k = 0; k < EW; k++) prev[k] = q ? reinterpret_cast<const uint32_t*>(src)[(int64_t)q * TS - EW + k] : 0u;
#pragma unroll
        for (int k = 0; k < TS; k++) x[k] = k < EW ? prev[k] : w[k - EW];
      }
    } else {
      load_words<TS>(dref, q, x);
    }
#pragma unroll
    for (int k = 0; k < TS; k++) w[k] ^= x[k];
#pragma unroll
    for (int plane = 0; plane < TS; plane++) {
      uint32_t v = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int byte = e * TS + plane;
        v |= ((w[byte / 4] >> (8 * (byte % 4))) & 0xffu) << (8 * e);
      }
      o[plane] = v;
    }
  };
  if (tid == 0) *red = 0u;
  __syncthreads();
  FPROF_T(pv0);
  uint32_t mis = 0;
  for (int32_t q = tid; q < quads; q += nth) {
    uint32_t o[TS];
    planes(q, o);
#pragma unroll
    for (int p = 0; p < TS; p++) mis |= (o[p] != rep[p] ? 1u : 0u) << p;
  }
  uint32_t wm = 0;
#pragma unroll
  for (int p = 0; p < TS; p++) wm |= __ballot((mis >> p) & 1u) ? (1u << p) : 0u;
  if ((tid & 63) == 0 && wm) __hip_atomic_fetch_or(red, wm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __syncthreads();
  const uint32_t M = __builtin_amdgcn_readfirstlane(*red);
  __syncthreads();
  FPROF_T(pv1);
  FPROF_ADD(22, pv0, pv1);
  if (M) {
    const __amdgpu_buffer_rsrc_t r = wt_rsrc((gout_t)dst);
    for (int32_t q = tid; q < quads; q += nth) {
      uint32_t o[TS];
      planes(q, o);
#pragma unroll
      for (int plane = 0; plane < TS; plane++)
        if ((M >> plane) & 1u) __builtin_amdgcn_raw_buffer_store_b32(o[plane], r, plane * n + 4 * q, 0, 16);
    }
  }
  FPROF_T(pv2);
  FPROF_ADD(23, pv1, pv2);
  return ~M & ((1u << TS) - 1u);
}
__device__ __noinline__ uint32_t fuse_ds_block_runs(const uint8_t* chunk, uint8_t* d, int32_t ts, int32_t b, int32_t bsize,
                                                    int32_t bs, B2H_LDS uint32_t* red) {
  const uint8_t* s = chunk + (int64_t)b * bs;
  const int32_t tid = threadIdx.x, nth = blockDim.x;
  if (ts == 8) return ds_block_runs<8>(s, chunk, d, bsize / 8, b == 0, tid, nth, red);
  if (ts == 4) return ds_block_runs<4>(s, chunk, d, bsize / 4, b == 0, tid, nth, red);
  return ds_block_runs<2>(s, chunk, d, bsize / 2, b == 0, tid, nth, red);
}

// The fused launch's filter job for global block k = chunk cc, block b.  The (DELTA, SHUFFLE) job
// is an out-of-line call: inlined, it cost T's shuffle-only launch 0.1 ms (register allocation).
__device__ __noinline__ void fuse_ds_block(const uint8_t* chunk, uint8_t* d, int32_t ts, int32_t b, int32_t bsize,
                                           int32_t bs, int32_t tid, int32_t nth) {
  const uint8_t* s = chunk + (int64_t)b * bs;
  if (ts == 8) ds_block_wt<8>(s, chunk, d, bsize / 8, b == 0, tid, nth);
  else if (ts == 4) ds_block_wt<4>(s, chunk, d, bsize / 4, b == 0, tid, nth);
  else ds_block_wt<2>(s, chunk, d, bsize / 2, b == 0, tid, nth);
}
__device__ __forceinline__ void fuse_filter_block(const EncFuse& f, const CGeom& g, int32_t cc, int32_t b, int32_t bsize,
                                                  int32_t tid, int32_t nth) {
  const uint8_t* chunk = f.raw + (int64_t)cc * f.raw_stride;
  uint8_t* d = f.filt + (int64_t)cc * g.wstride + (int64_t)b * g.bs;
  if (f.ds == 0) shuffle4_block_wt(chunk + (int64_t)b * g.bs, d, bsize, tid, nth);
  else fuse_ds_block(chunk, d, f.ds, b, bsize, g.bs, tid, nth);
}

// The fused kernel's arguments, staged in LDS at launch and read back (as wave-uniform values) in
// each phase that needs them.  Kept in kernel arguments, the ~60 words of geometry, sync pointers
// and strides stayed live in SGPRs through the whole launch, the encoder's loops ran out of SGPRs
// and the compiler spilled ~170 of them into VGPR lanes (a v_readlane / v_writelane per reload in
// the tile loops).  A phase's copy is dead once it ends; the encode's barriers end every live range.
struct FusedArgs {
  CGeom g;
  EncFuse f;
  const uint8_t* filt;
  uint8_t* sbuf;
  StreamResult* res;
  int32_t* next;
  const int32_t* porder;
  int32_t nstreams_total, tablog;
};
__host__ __device__ constexpr size_t fused_lds(size_t pos_bytes, int tablog) {
  return fast_lds(pos_bytes, tablog) + ((sizeof(FusedArgs) + 15) & ~size_t(15));
}
// eight two-wave workgroups per CU (160 KiB of LDS) at the default u16 table
static_assert(fused_lds(2, 13) <= 160 * 1024 / 8, "fused fast encoder: more than 20 KiB of LDS per workgroup");

// Whether the fused filter job decides the run verdict of a block's streams: a split block (one
// stream per byte plane) of a chunk with run streams (extended header), the (DELTA, SHUFFLE) job or
// the 4-byte SHUFFLE one over whole 64-byte groups, not the leftover block, not opted out (bit 128)
__device__ __forceinline__ bool fuse_verdict(const EncFuse& f, const CGeom& g, bool lo) {
  if (lo || g.overhead != kHdrExt || (f.mode_bits & 128)) return false;
  return f.ds ? g.spb == f.ds : (g.spb == 4 && (g.bs & 255) == 0);
}

// The (DELTA, SHUFFLE) filter jobs of a fused fast launch, run ahead of it by a launch of their own
// (B2H_DS_PREPASS=1, off by default): one 256-thread workgroup per block, many per CU, instead of
// one wave pair each inside the encoder launch.  There a pair holds ~465 us per 512 KiB block and
// C4's encoder launch keeps only ~600 of its 2 048 pair slots on streams
// (profiles/r6_streams_C4_fast.log) -- but the separate pass costs about what exact mode's
// k_ffilter_ds does, and C4 compress went 7.2 -> 8.8 ms (profiles/r6_ab_ds_prepass.txt): the
// in-launch jobs overlap the encoding.  Each block's ready word is published exactly as the
// in-launch job does (1 | runs << 1, the verdict bit with it), and the claim counter is left at
// the block count, so the encoder launch claims no job and finds every block ready.
__global__ __launch_bounds__(256) void k_ds_prepass(EncFuse f, CGeom g, int32_t nblk) {
  __shared__ uint32_t red_s;
  B2H_LDS uint32_t* red = (B2H_LDS uint32_t*)&red_s;
  for (int32_t k = blockIdx.x; k < nblk; k += gridDim.x) {
    const int32_t cc = k / g.nblocks, b = k - cc * g.nblocks;
    const bool lo = b == g.nblocks - 1 && g.leftover;
    const int32_t bsize = lo ? g.leftover : g.bs;
    const uint8_t* chunk = f.raw + (int64_t)cc * f.raw_stride;
    uint8_t* fd = f.filt + (int64_t)cc * g.wstride + (int64_t)b * g.bs;
    uint32_t runs = 0;
    if (fuse_verdict(f, g, lo)) {
      const uint8_t* src = chunk + (int64_t)b * g.bs;
      if (f.ds == 8) runs = ds_block_runs<8>(src, chunk, fd, bsize / 8, b == 0, threadIdx.x, blockDim.x, red);
      else if (f.ds == 4) runs = ds_block_runs<4>(src, chunk, fd, bsize / 4, b == 0, threadIdx.x, blockDim.x, red);
      else runs = ds_block_runs<2>(src, chunk, fd, bsize / 2, b == 0, threadIdx.x, blockDim.x, red);
      runs |= 1u << 29;
    } else {
      fuse_ds_block(chunk, fd, f.ds, b, bsize, g.bs, threadIdx.x, blockDim.x);
    }
    __syncthreads();
    if (threadIdx.x == 0) f.sync[kFuseHdr + k] = (int32_t)(1u | (runs << 1));
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) f.sync[0] = nblk;   // every job claimed
}
static bool ds_prepass() {   // read per call (tests switch it)
  const char* e = getenv("B2H_DS_PREPASS");
  return e && atoi(e) != 0;
}

#undef FUSE_TRACE_PTR
#define FUSE_TRACE_PTR lds_uniform(&A->f.trace)
#ifndef B2H_FAST_WPE
#define B2H_FAST_WPE 4   // waves per SIMD the fused fast launch is compiled for (4: <= 128 VGPRs)
#endif
template <typename POS, bool DEEP>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(B2H_FAST_WPE, 8)))   // as k_encode_fast
void k_encode_fast_fused(CGeom g_arg, const uint8_t* __restrict__ filt_arg, uint8_t* __restrict__ sbuf_arg,
                         StreamResult* __restrict__ res_arg, int32_t nstreams_total_arg, int32_t* __restrict__ next_arg,
                         int tablog_arg, const int32_t* __restrict__ porder_arg, EncFuse f_arg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tablog0 = tablog_arg;
  B2H_LDS uint8_t* tab = (B2H_LDS uint8_t*)smem;
  B2H_LDS uint8_t* oring = (B2H_LDS uint8_t*)(smem + (sizeof(POS) << tablog0));
  B2H_LDS FastShared* sh = (B2H_LDS FastShared*)(smem + (sizeof(POS) << tablog0) + kOutRing);
  B2H_LDS FusedArgs* A = (B2H_LDS FusedArgs*)(smem + fast_lds(sizeof(POS), tablog0));
  if (threadIdx.x == 0) {
    lds_store(&A->g, g_arg);
    lds_store(&A->f, f_arg);
    A->filt = filt_arg;
    A->sbuf = sbuf_arg;
    A->res = res_arg;
    A->next = next_arg;
    A->porder = porder_arg;
    A->nstreams_total = nstreams_total_arg;
    A->tablog = tablog_arg;
  }
  __syncthreads();
  const bool matcher = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  // wave priority (B2H_FUSE bit 64, default): the parser -- the tile's latency chain -- issues
  // ahead of the matchers sharing its SIMD (T encode 18.0 -> 17.6 ms; the matcher first: 19.3)
  if ((lds_uniform(&A->f.mode_bits) & 64) && !matcher) __builtin_amdgcn_s_setprio(2);
  // lane 0 of the workgroup computes v, everyone gets it
  auto bcast = [&](int32_t v) -> int32_t {
    if (threadIdx.x == 0) sh->bcast = v;
    __syncthreads();
    const int32_t r = __builtin_amdgcn_readfirstlane(sh->bcast);
    __syncthreads();
    return r;
  };
  // scatter item k: streams [j0, j0 + kFuseSpi) of the chunk in ready slot k / ipc (the publish
  // poll, ONE agent acquire for the item, then plain loads of the placements and payloads)
  auto scatter_item = [&](int32_t k) {
    const CGeom g = lds_uniform(&A->g);
    const EncFuse f = lds_uniform(&A->f);
    const int32_t ipc = (g.nsc + kFuseSpi - 1) / kFuseSpi;   // items per chunk
    int32_t* ready = f.sync + kFuseHdr + f.nchunks * g.nblocks + f.nchunks;
    const int32_t slot = k / ipc, j0 = (k - slot * ipc) * kFuseSpi;
    int32_t v = 0;
    FUSE_TRACE(1, k);
    if (threadIdx.x == 0) {
      v = wait_nonzero(ready + slot, f.sync + 4);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_stores();
    }
    v = bcast(v);
    if (v <= 0) return;
    const CGeom g2 = lds_uniform(&A->g);   // re-read after the barriers of bcast
    const EncFuse f2 = lds_uniform(&A->f);
    const uint8_t* filt = lds_uniform(&A->filt);
    const uint8_t* sbuf = lds_uniform(&A->sbuf);
    const int32_t c = v - 1;
    if (__builtin_amdgcn_readfirstlane(f2.mode[c]) != 0) return;
    uint8_t* d = f2.dst + (int64_t)c * g2.dst_stride;
    const int32_t wv = threadIdx.x >> 6;
    for (int32_t l = j0; l < min(j0 + kFuseSpi, g2.nsc); l++) {
      const int32_t s = c * g2.nsc + l;
      Place pl;
      pl.off = __builtin_amdgcn_readfirstlane(f2.place[s].off);
      pl.csize = __builtin_amdgcn_readfirstlane(f2.place[s].csize);
      int32_t off, len, blk;
      stream_locate(g2, l, &off, &len, &blk);
      if (threadIdx.x == 0) {
        const uint32_t w = (uint32_t)pl.csize;
        uint8_t* q = d + pl.off - 4;
        q[0] = (uint8_t)w; q[1] = (uint8_t)(w >> 8); q[2] = (uint8_t)(w >> 16); q[3] = (uint8_t)(w >> 24);
        if (pl.csize < 0) d[pl.off] = 0x1;   // run-length token
      }
      if (pl.csize <= 0) continue;
      const uint8_t* src = (pl.csize == len ? filt : sbuf) + (int64_t)c * g2.wstride + off;
      const int32_t q = ((pl.csize + 1) / 2 + 15) & ~15;
      const int32_t a = min(pl.csize, wv * q), b = min(pl.csize, a + q);
      if (b > a) {
        if ((f2.mode_bits & 32) || !aligned16(src + a)) wave_copy((gout_t)(d + pl.off + a), (gin_t)(src + a), b - a);
        else wave_copy_a16((gout_t)(d + pl.off + a), (gin_t)(src + a), b - a);
      }
    }
  };
  // published scatter items, claimed with a CAS (never past the published count), a few tries.
  // Every loop below that holds a barrier is `while (uniform)` with its broadcast last in the body:
  // a `break` after lane-0-only code lets the compiler structurize the loop as divergent, and its
  // waves then meet different barriers (seen: a workgroup re-shuffling one block forever).
  auto try_claim_item = [&]() -> int32_t {   // lane 0
    int32_t* sync = lds_uniform(&A->f.sync);
    const int32_t pub = rd_agent(sync + 3);
    int32_t cur = rd_agent(sync + 1);
    for (int tries = 0; tries < 8 && cur < pub; tries++) {
      const int32_t want = cur;
      if (__hip_atomic_compare_exchange_strong((gi32_t)(sync + 1), &cur, want + 1, __ATOMIC_RELAXED,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return want;
    }
    return -1;
  };
  auto scatter_available = [&](int max_items) {   // the broadcast unconditional in every iteration
    int32_t k = 0;
    for (int it = 0; it < max_items && k >= 0; it++) {
      k = bcast(threadIdx.x == 0 ? try_claim_item() : -1);
      if (k >= 0) scatter_item(k);
    }
  };
  // lane 0: claim the next block to shuffle while the claims are behind `target`, else -1
  auto claim_block = [&](int32_t target) -> int32_t {
    int32_t* sync = lds_uniform(&A->f.sync);
    return rd_agent(sync) < target ? add_agent(sync, 1) : -1;
  };
  int32_t i = bcast(threadIdx.x == 0 ? atomicAdd(lds_uniform(&A->next), 1) : 0);
  while (i < lds_uniform(&A->nstreams_total)) {
    FUSE_TRACE(3, i);
    int32_t s, c;
    gin_t in;
    gout_t out;
    int32_t len, clevel, tablog;
    int32_t run_byte = -1;   // >= 0: the stream is a run of this byte (decided by the filter job)
    uint32_t verdict = 0;    // 1: the filter job decided the stream's run test
    bool runs;
    {
      const CGeom g = lds_uniform(&A->g);
      s = __builtin_amdgcn_readfirstlane(pull_to_stream(g, lds_uniform(&A->porder), g.front, i,
                                                         lds_uniform(&A->nstreams_total)));
      c = s / g.nsc;
      const int32_t l = s - c * g.nsc;
      int32_t off, blk;
      stream_locate(g, l, &off, &len, &blk);
      const EncFuse f = lds_uniform(&A->f);
      if (f.raw) {
        const int32_t nblk = f.nchunks * g.nblocks;
        const int32_t gb = c * g.nblocks + blk, target = min(gb + 1 + f.lead, nblk);
        int32_t k = bcast(threadIdx.x == 0 ? claim_block(target) : -1);
        while (k >= 0 && k < nblk) {   // keep the shuffle claims ahead of the streams
          FUSE_TRACE(4, k);
          const CGeom gk = lds_uniform(&A->g);
          const EncFuse fk = lds_uniform(&A->f);
          const int32_t cc = k / gk.nblocks, b = k - cc * gk.nblocks;
          const bool lo = b == gk.nblocks - 1 && gk.leftover;
          const int32_t bsize = lo ? gk.leftover : gk.bs;
          // a split (DELTA, SHUFFLE) block of a chunk with run streams (extended header): the run
          // verdict comes with the filter job, published with the block (ready word 1 | runs << 1)
          uint32_t runs = 0;
          FPROF_T(ja);
          if (fuse_verdict(fk, gk, lo)) {
            uint8_t* fd = fk.filt + (int64_t)cc * gk.wstride + (int64_t)b * gk.bs;
            runs = fk.ds ? fuse_ds_block_runs(fk.raw + (int64_t)cc * fk.raw_stride, fd, fk.ds, b, bsize, gk.bs, &sh->runred)
                         : shuffle4_block_runs<true>(fk.raw + (int64_t)cc * fk.raw_stride + (int64_t)b * gk.bs, fd, bsize, &sh->runred,
                                                   threadIdx.x, blockDim.x);
            runs |= 1u << 29;   // (bit 30 once published) the verdict is complete: no run test needed
          } else {
            fuse_filter_block(fk, gk, cc, b, bsize, threadIdx.x, blockDim.x);
          }
          FPROF_T(jd);
          drain_stores();
          __syncthreads();
          FPROF_T(jb);
          FPROF_ADD(16, ja, jb);
          FPROF_ADD(19, jd, jb);
          FPROF_CNT(20);
          int32_t nk = -1;
          if (threadIdx.x == 0) {
            st_agent(fk.sync + kFuseHdr + k, (int32_t)(1u | (runs << 1)));
            nk = claim_block(target);
          }
          k = bcast(nk);
        }
        FUSE_TRACE(5, gb);
        int32_t rv = 0;
        FPROF_T(wa);
        if (threadIdx.x == 0) {
          int32_t* sync = lds_uniform(&A->f.sync);
          rv = wait_nonzero(sync + kFuseHdr + gb, sync + 4);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          drain_stores();
        }
        rv = bcast(rv);
        FPROF_T(wb);
        FPROF_ADD(17, wa, wb);
        // the stream's plane was found a run by the filter job: its byte is plane j's of the
        // block's first element after DELTA, and nothing was stored for it
        const int32_t j = l - blk * g.spb;
        if (blk < g.nblocks - (g.leftover ? 1 : 0) && (((uint32_t)rv >> 1) >> j) & 1u) {
          const uint8_t* raw = f.raw + (int64_t)c * f.raw_stride;
          run_byte = (int32_t)(uint8_t)(raw[(int64_t)blk * g.bs + j] ^ (blk && f.ds ? raw[j] : 0));
        }
        verdict = ((uint32_t)rv >> 30) & 1u;
      }
      const CGeom g2 = lds_uniform(&A->g);
      in = (gin_t)(lds_uniform(&A->filt) + (int64_t)c * g2.wstride + off);
      out = (gout_t)(lds_uniform(&A->sbuf) + (int64_t)c * g2.wstride + off);
      clevel = g2.clevel;
      runs = g2.overhead == kHdrExt && __builtin_amdgcn_readfirstlane(verdict) == 0;
      tablog = lds_uniform(&A->tablog);
    }
    FUSE_TRACE(6, s);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    B2H_GLB POS* chain = nullptr;
    if constexpr (DEEP) {
      const CGeom g = lds_uniform(&A->g);
      chain = (B2H_GLB POS*)g.chain + (int64_t)blockIdx.x * chain_len(g);
    }
    StreamResult r;
    if (__builtin_amdgcn_readfirstlane(run_byte) >= 0) {   // what the run test would return
      r.windows = 0;
      r.cycles = 0;
      r.peak = 0;
      r.size = run_byte;
      r.kind = run_byte ? kStreamByteRun : kStreamZeroRun;
    } else {
      r = encode_stream_fast<POS, true, DEEP>(in, len, clevel, out, tab, tablog, oring, sh, runs, matcher, chain);
      FPROF_CNT(21);
    }
    r.cycles = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
    FPROF_ADD(18, t0, (uint64_t)__builtin_amdgcn_s_memtime());
    r.t_start = (int64_t)((rt0 << 24) | ((__builtin_amdgcn_s_memrealtime() - rt0) & 0xffffff));
    if (!matcher && lane_id() == 0) {
      int32_t* fin = lds_uniform(&A->f.fin);
      lds_uniform(&A->res)[s] = r;
      st_agent(fin + 3 * s, r.kind);
      st_agent(fin + 3 * s + 1, r.size);
      st_agent(fin + 3 * s + 2, r.peak);
    }
    FUSE_TRACE(7, s);
    drain_stores();
    __syncthreads();
    int32_t done;
    {
      const CGeom g = lds_uniform(&A->g);
      const EncFuse f = lds_uniform(&A->f);
      int32_t* chunk_cnt = f.sync + kFuseHdr + f.nchunks * g.nblocks;
      done = bcast(threadIdx.x == 0 ? add_agent(chunk_cnt + c, 1) : 0);
    }
    if (done == lds_uniform(&A->g.nsc) - 1) {   // last stream of chunk c: finalize it (its stream results -> LDS)
      B2H_LDS int32_t* fl = (B2H_LDS int32_t*)tab;
      FUSE_TRACE(8, c);
      if (threadIdx.x == 0) {   // the counter add returned: ONE acquire, then plain loads
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        drain_stores();
      }
      __syncthreads();
      {
        const int32_t nsc = lds_uniform(&A->g.nsc);
        const int32_t* fin = lds_uniform(&A->f.fin);
        for (int32_t j = threadIdx.x; j < 3 * nsc; j += blockDim.x) fl[j] = fin[3 * c * nsc + j];
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        const CGeom g = lds_uniform(&A->g);
        const EncFuse f = lds_uniform(&A->f);
        const int32_t ipc = (g.nsc + kFuseSpi - 1) / kFuseSpi;
        int32_t* ready = f.sync + kFuseHdr + f.nchunks * g.nblocks + f.nchunks;
        Place* pl = f.place + (int64_t)c * g.nsc;
        int32_t cb = 0;
        const int32_t m = finalize_chunk(
            g, f.dst + (int64_t)c * g.dst_stride, f.htpl,
            [&](int32_t j) {
              StreamResult x;
              x.kind = fl[3 * j];
              x.size = fl[3 * j + 1];
              x.peak = fl[3 * j + 2];
              return x;
            },
            [&](int32_t j, int32_t o, int32_t cs) { st_agent(&pl[j].off, o); st_agent(&pl[j].csize, cs); }, &cb);
        st_agent(f.mode + c, m);
        f.cbytes[c] = cb;
        drain_stores();
        const int32_t slot = add_agent(f.sync + 2, 1);
        st_agent(ready + slot, c + 1);
        drain_stores();
        add_agent(f.sync + 3, ipc);
      }
      __syncthreads();
    }
    FUSE_TRACE(2, 0);
    if (!(lds_uniform(&A->f.mode_bits) & 16)) scatter_available(2);
    i = bcast(threadIdx.x == 0 ? atomicAdd(lds_uniform(&A->next), 1) : 0);
  }
  // stream queue empty: every remaining scatter item
  FUSE_TRACE(9, 0);
  int32_t k = bcast(threadIdx.x == 0 ? add_agent(lds_uniform(&A->f.sync) + 1, 1) : 0);
  while (true) {
    const CGeom g = lds_uniform(&A->g);
    const int32_t nitems = lds_uniform(&A->f.nchunks) * ((g.nsc + kFuseSpi - 1) / kFuseSpi);
    if (k >= nitems) break;
    scatter_item(k);
    k = bcast(threadIdx.x == 0 ? add_agent(lds_uniform(&A->f.sync) + 1, 1) : 0);
  }
  FUSE_TRACE(15, 0);
}
#undef FUSE_TRACE_PTR
#define FUSE_TRACE_PTR f.trace

// A timed-out hand-off wait inside k_encode_fast_fused fails every chunk of the batch.
__global__ void k_fuse_check(const int32_t* __restrict__ sync, int32_t* __restrict__ cbytes, int32_t nchunks) {
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < nchunks && sync[4]) cbytes[c] = E_FAILURE;
}

// B2H_FUSE (A/B runs, tests): 0 separate launches; bit 1 finalize + scatter inside the encode launch,
// bit 2 + the byte shuffle, bit 4 exact mode too (k_encode_fused: per-wave shuffles and copies are
// latency-bound, T exact 26.98 -> 27.72 ms, so off by default), bit 16 scatter items only once the
// stream queue is empty, bit 8 BloscLZ mode 3 too (k_encode_seg_fused, same per-wave protocol:
// T seg 209.9 GiB/s unfused, 206.5 fused, 204.3 with only finalize + scatter fused -- lone waves'
// shuffles and copies contend with the segment walks -- so off by default), bit 32 plain
// dword-load scatter copies, bit 64 the parser wave at a
// higher issue priority.  Default 83 (1 + 2 + 16 + 64).  Measured on T (tools/fuse_prof.py, profiles/r2_v5_*):
// separate 1.54 + 16.55 + 1.10 ms; 19: 17.79 ms; scatter items claimed between streams (3) slow
// the concurrent encoders' short planes ~2x (22.5 ms), with non-temporal copies too (35).
static int fuse_bits() {
  const char* e = getenv("B2H_FUSE");
  return e ? atoi(e) : 83;
}
// Per host thread: the fused launches off (set around a retry after a hand-off timeout).
static thread_local bool t_fuse_off = false;
// The gated separate launches queued behind every fused launch (compress_batch); B2H_FUSE_RESCUE=0
// drops them (measurement only: a timed-out batch then fails with BLOSC2_ERROR_FAILURE).
static bool fuse_rescue() {
  const char* e = getenv("B2H_FUSE_RESCUE");
  return !e || atoi(e) != 0;
}
void set_fuse_disabled(bool off) { t_fuse_off = off; }
static bool fuse_enabled() { return !t_fuse_off && (fuse_bits() & 1) != 0; }
// B2H_FUSE_GRID (tests): cap the fused launch's persistent grid -- a few workgroups then do every
// shuffle, stream, finalisation and scatter item, the hand-off waits' worst case.
static int64_t fuse_grid_cap(int64_t slots) {
  const char* e = getenv("B2H_FUSE_GRID");
  return e && atoi(e) > 0 ? std::min<int64_t>(slots, atoi(e)) : slots;
}
// How far (in blocks) the fused launch's shuffle claims run ahead of the block a workgroup's stream
// needs.  T fast, same box (profiles/r5_ab_shuf_lead.txt): 512 214.9, 256 215.1, 128 215.8,
// 64 215.9, 32 215.7 GiB/s -- less shuffle traffic ahead of the encoders; C3 / C4 unchanged.
static int fuse_lead() {
  static const int v = [] { const char* e = getenv("B2H_SHUF_LEAD"); return e ? std::max(1, atoi(e)) : 64; }();
  return v;
}

// Sync words (zeroed) + per-stream results of a fused launch (f.raw / f.filt set by the caller).
static int fuse_prepare(Workspace* ws, const CGeom& g, int64_t ntot, EncFuse& f, hipStream_t st) {
  const size_t sync_words = kFuseHdr + (size_t)f.nchunks * g.nblocks + 2 * (size_t)f.nchunks;
  const size_t sync_bytes = (sync_words * 4 + 15) & ~size_t(15);
  if (ws->fsync.ensure(sync_bytes + 12 * (size_t)ntot)) return E_MEMORY;
  f.sync = ws->fsync.as<int32_t>();
  f.fin = reinterpret_cast<int32_t*>(ws->fsync.as<uint8_t>() + sync_bytes);
  f.lead = fuse_lead();
  f.mode_bits = fuse_bits();
  f.trace = nullptr;
  HIPCHK(hipMemsetAsync(f.sync, 0, sync_bytes, st));
  // B2H_FUSE_SIMULATE_TIMEOUT (tests): the launch starts with its timeout flag set, as if a
  // hand-off wait had run out -- the batch fails and the synchronous entry points retry unfused
  if (getenv("B2H_FUSE_SIMULATE_TIMEOUT")) HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(f.sync + 4), 1, 1, st));
  return 0;
}

// Sync words + per-stream results of the fused launch (f.raw / f.filt set by the caller).
template <typename POS, bool DEEP>
static int launch_encode_fast_fused_t(Workspace* ws, const CGeom& g0, const uint8_t* filt, StreamResult* res,
                                      int64_t ntot, int32_t* next, const int32_t* porder, EncFuse f, hipStream_t st) {
  CGeom g = g0;
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const int tablog = std::min(fast_tablog(), hashlog);
  const size_t lds = fused_lds(sizeof(POS), tablog);
  const void* fn = reinterpret_cast<const void*>(&k_encode_fast_fused<POS, DEEP>);
  static bool attr_set = false;
  if (!attr_set) {
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int slots = resident_slots(fn, lds, 128);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(ntot, fuse_grid_cap(slots)));
  if (fuse_prepare(ws, g, ntot, f, st)) return E_MEMORY;
  if (chain_prepare<POS>(ws, g, grid)) return E_MEMORY;
  if (f.raw && f.ds && ds_prepass()) {   // the (DELTA, SHUFFLE) jobs first, bandwidth-parallel
    const int32_t nblk = f.nchunks * g.nblocks;
    k_ds_prepass<<<(uint32_t)std::min<int32_t>(nblk, 8192), 256, 0, st>>>(f, g, nblk);
    HIPCHK(hipGetLastError());
  }
  static int32_t* trace = nullptr;
  static const bool tr = getenv("B2H_FUSE_TRACE") != nullptr;
  if (tr && !trace) HIPCHK(hipHostMalloc(&trace, 4 << 20, hipHostMallocCoherent));
  f.trace = tr ? trace : nullptr;
  if (tr) memset(trace, 0xff, 4 * (size_t)grid);
  k_encode_fast_fused<POS, DEEP><<<grid, 128, lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot, next, tablog,
                                                   porder, f);
  HIPCHK(hipGetLastError());
  if (tr) {   // debug watchdog: report where the workgroups are if the launch has not ended after 5 s
    for (int ms = 0; ms < 5000 && hipStreamQuery(st) == hipErrorNotReady; ms++) usleep(1000);
    if (hipStreamQuery(st) == hipErrorNotReady) {
      int hist[16][2] = {};
      for (uint32_t b = 0; b < grid; b++) {
        const int32_t v = __atomic_load_n(trace + b, __ATOMIC_RELAXED);
        if (v == -1) continue;
        hist[v & 15][0]++;
        hist[v & 15][1] = v >> 4;
      }
      fprintf(stderr, "k_encode_fast_fused stuck after 5 s (grid %u, ntot %lld):\n", grid, (long long)ntot);
      for (int k = 0; k < 16; k++)
        if (hist[k][0]) fprintf(stderr, "  phase %d: %d workgroups (e.g. value %d)\n", k, hist[k][0], hist[k][1]);
      fflush(stderr);
      abort();
    }
  }
  k_fuse_check<<<(f.nchunks + 255) / 256, 256, 0, st>>>(f.sync, f.cbytes, f.nchunks);
  HIPCHK(hipGetLastError());
  return 0;
}

// The fused launch applies to BloscLZ fast mode without a dictionary when the chunk's stream
// results fit the LDS table (the finalizing workgroup stages them there).
static void enc_mode(int* nlds, int* nglb);
static bool fused_encode_ok(const CGeom& g) {
  if (!fuse_enabled() || g.compcode != 0 || g.dict_size) return false;
  if (g.lzmode == 3) return (fuse_bits() & 8) != 0;   // mode 3: only with bit 8 (measured slower)
  if (g.lzmode == 0) {   // exact mode: only with bit 4 (measured slower), the default k_encode shape
    if (!(fuse_bits() & 4)) return false;
    int nl, ng;
    enc_mode(&nl, &ng);
    return (nl == 1 && ng == 3) || nl < 0;   // the fused exact kernel has the hyb3 shape
  }
  const bool small = fast_u16(g);
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const int tablog = std::min(fast_tablog(), hashlog);
  return (size_t)12 * g.nsc <= ((small ? 2u : 4u) << tablog);
}
static int launch_encode_fast_fused(Workspace* ws, const CGeom& g, const uint8_t* filt, StreamResult* res,
                                    int64_t ntot, int32_t* next, const int32_t* porder, const EncFuse& f,
                                    hipStream_t st) {
  const bool small = fast_u16(g);
  if (g.lzmode == 2)
    return small ? launch_encode_fast_fused_t<uint16_t, true>(ws, g, filt, res, ntot, next, porder, f, st)
                 : launch_encode_fast_fused_t<uint32_t, true>(ws, g, filt, res, ntot, next, porder, f, st);
  return small ? launch_encode_fast_fused_t<uint16_t, false>(ws, g, filt, res, ntot, next, porder, f, st)
               : launch_encode_fast_fused_t<uint32_t, false>(ws, g, filt, res, ntot, next, porder, f, st);
}


// ------------------------------------------- exact mode, one launch: shuffle -> encode -> scatter ----
// k_encode's waves pull streams independently, so the fused protocol of k_encode_fast_fused runs
// per wave here: shuffle claims ahead of the wave's stream, the wave that completes a chunk
// finalizes it, scatter items once the stream queue is empty.  Every wave-level decision comes
// from an atomic all 64 lanes take part in (lane 0 adds, the others add 0) and a readfirstlane,
// never from a value only lane 0 holds (see encode_loop).
// The arguments (FusedArgs) live in LDS and every phase re-reads the words it needs: kept in
// registers across the encode they cost ~300 SGPR spills (v_readlane / v_writelane reloads in the
// parse loops; T exact fused 25.94 ms against 23.03 for k_encode alone).
// `enc(in, len, clevel, out, runs_test)` encodes one stream (write-through output): the exact
// walker (k_encode_fused) or BloscLZ mode 3's segmented parse (k_encode_seg_fused).
template <typename ENC>
__device__ void encode_loop_fused(const B2H_LDS FusedArgs* A, ENC&& enc) {
  const int lane = lane_id();
  auto wadd = [&](int32_t* p, int32_t v) -> int32_t {
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_fetch_add((gi32_t)p, lane == 0 ? v : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  };
  auto wwait = [&](int32_t* p) -> int32_t {   // bounded poll, all lanes
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (int32_t it = 0; it < (1 << 21); it++) {
      const int32_t v = wadd(p, 0);
      if (v) return v;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) break;
      __builtin_amdgcn_s_sleep(8);
    }
    if (lane == 0) st_agent(lds_uniform(&A->f.sync) + 4, 1);
    return 0;
  };
  auto claim_block = [&](int32_t target) -> int32_t {
    int32_t* sync = lds_uniform(&A->f.sync);
    return wadd(sync, 0) < target ? wadd(sync, 1) : -1;
  };
  int32_t i = wadd(lds_uniform(&A->next), 1);
  while (i < lds_uniform(&A->nstreams_total)) {
    int32_t s, c, l, off, len, blk;
    int32_t rv = 0;   // the block's ready word: 1 | run planes << 1 | verdict << 30
    {
      const CGeom g = lds_uniform(&A->g);
      s = __builtin_amdgcn_readfirstlane(pull_to_stream(g, lds_uniform(&A->porder), g.front, i, lds_uniform(&A->nstreams_total)));
      c = s / g.nsc;
      l = s - c * g.nsc;
      stream_locate(g, l, &off, &len, &blk);
    }
    if (lds_uniform(&A->f.raw)) {
      int32_t gb, target, nblk;
      {
        const CGeom g = lds_uniform(&A->g);
        nblk = lds_uniform(&A->f.nchunks) * g.nblocks;
        gb = c * g.nblocks + blk;
        target = min(gb + 1 + lds_uniform(&A->f.lead), nblk);
      }
      int32_t k = claim_block(target);
      while (k >= 0 && k < nblk) {
        const CGeom g = lds_uniform(&A->g);
        const EncFuse f = lds_uniform(&A->f);
        const int32_t cc = k / g.nblocks, b = k - cc * g.nblocks;
        const int32_t bsize = (b == g.nblocks - 1 && g.leftover) ? g.leftover : g.bs;
        // the 4-byte SHUFFLE job decides its split block's run verdict (as in k_encode_fast_fused)
        uint32_t runs = 0;
        if (f.ds == 0 && fuse_verdict(f, g, b == g.nblocks - 1 && g.leftover)) {
          runs = shuffle4_block_runs<false>(f.raw + (int64_t)cc * f.raw_stride + (int64_t)b * g.bs,
                                            f.filt + (int64_t)cc * g.wstride + (int64_t)b * g.bs, bsize, nullptr, lane, 64);
          runs |= 1u << 29;
        } else {
          fuse_filter_block(f, g, cc, b, bsize, lane, 64);
        }
        drain_stores();
        if (lane == 0) st_agent(f.sync + kFuseHdr + k, (int32_t)(1u | (runs << 1)));
        k = claim_block(target);
      }
      rv = wwait(lds_uniform(&A->f.sync) + kFuseHdr + gb);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_stores();
    }
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t urv = (uint32_t)__builtin_amdgcn_readfirstlane(rv);
    const bool verdict = (urv >> 30) & 1u;
    StreamResult r;
    int32_t run_byte = -1;
    gin_t in;
    gout_t out;
    int clevel;
    bool runs_test;
    {
      const CGeom g = lds_uniform(&A->g);
      const int32_t j = l - blk * g.spb;
      if (verdict && ((urv >> 1) >> j) & 1u)   // what the run test would return
        run_byte = lds_uniform(&A->f.raw)[(int64_t)c * lds_uniform(&A->f.raw_stride) + (int64_t)blk * g.bs + j];
      in = (gin_t)(lds_uniform(&A->filt) + (int64_t)c * g.wstride + off);
      out = (gout_t)(lds_uniform(&A->sbuf) + (int64_t)c * g.wstride + off);
      clevel = g.clevel;
      runs_test = g.overhead == kHdrExt && !verdict;
    }
    if (__builtin_amdgcn_readfirstlane(run_byte) >= 0) {
      r.windows = 0;
      r.peak = 0;
      r.size = run_byte;
      r.kind = r.size ? kStreamByteRun : kStreamZeroRun;
    } else {
      r = enc(in, len, clevel, out, runs_test);
    }
    r.cycles = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
    r.t_start = (int64_t)((rt0 << 24) | ((__builtin_amdgcn_s_memrealtime() - rt0) & 0xffffff));
    {
      const CGeom g = lds_uniform(&A->g);
      const EncFuse f = lds_uniform(&A->f);
      if (lane == 0) {
        lds_uniform(&A->res)[s] = r;
        st_agent(f.fin + 3 * s, r.kind);
        st_agent(f.fin + 3 * s + 1, r.size);
        st_agent(f.fin + 3 * s + 2, r.peak);
      }
      drain_stores();
      int32_t* chunk_cnt = f.sync + kFuseHdr + f.nchunks * g.nblocks;
      int32_t* ready = chunk_cnt + f.nchunks;
      const int32_t ipc = (g.nsc + kFuseSpi - 1) / kFuseSpi;
      const int32_t done = wadd(chunk_cnt + c, 1);
      if (done == g.nsc - 1) {   // this wave completed chunk c: finalize it
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        drain_stores();
        const bool inreg = g.nsc <= 64;   // lane j holds stream j's results
        const int32_t* fc = f.fin + 3 * (int64_t)c * g.nsc;
        int32_t fk = 0, fs = 0, fp = 0;
        if (inreg && lane < g.nsc) {
          fk = fc[3 * lane];
          fs = fc[3 * lane + 1];
          fp = fc[3 * lane + 2];
        }
        if (lane == 0) {
          Place* pl = f.place + (int64_t)c * g.nsc;
          int32_t cb = 0;
          const int32_t m = finalize_chunk(
              g, f.dst + (int64_t)c * g.dst_stride, f.htpl,
              [&](int32_t jj) {
                StreamResult x;
                x.kind = inreg ? __builtin_amdgcn_readlane(fk, jj) : fc[3 * jj];
                x.size = inreg ? __builtin_amdgcn_readlane(fs, jj) : fc[3 * jj + 1];
                x.peak = inreg ? __builtin_amdgcn_readlane(fp, jj) : fc[3 * jj + 2];
                return x;
              },
              [&](int32_t jj, int32_t o, int32_t cs) { st_agent(&pl[jj].off, o); st_agent(&pl[jj].csize, cs); }, &cb);
          st_agent(f.mode + c, m);
          f.cbytes[c] = cb;
          drain_stores();
          const int32_t slot = add_agent(f.sync + 2, 1);
          st_agent(ready + slot, c + 1);
          drain_stores();
          add_agent(f.sync + 3, ipc);
        }
      }
    }
    i = wadd(lds_uniform(&A->next), 1);
  }
  // stream queue empty: scatter items
  const CGeom g = lds_uniform(&A->g);
  const EncFuse f = lds_uniform(&A->f);
  const uint8_t* filt = lds_uniform(&A->filt);
  const uint8_t* sbuf = lds_uniform(&A->sbuf);
  int32_t* ready = f.sync + kFuseHdr + f.nchunks * g.nblocks + f.nchunks;
  const int32_t ipc = (g.nsc + kFuseSpi - 1) / kFuseSpi, nitems = f.nchunks * ipc;
  int32_t k = wadd(f.sync + 1, 1);
  while (k < nitems) {
    const int32_t slot = k / ipc, j0 = (k - slot * ipc) * kFuseSpi;
    const int32_t v = wwait(ready + slot);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    drain_stores();
    const int32_t c = v - 1;
    if (v > 0 && __builtin_amdgcn_readfirstlane(f.mode[c]) == 0) {
      uint8_t* d = f.dst + (int64_t)c * g.dst_stride;
      for (int32_t l = j0; l < min(j0 + kFuseSpi, g.nsc); l++) {
        const int32_t s = c * g.nsc + l;
        const int32_t poff = __builtin_amdgcn_readfirstlane(f.place[s].off);
        const int32_t pcs = __builtin_amdgcn_readfirstlane(f.place[s].csize);
        int32_t off, len, blk;
        stream_locate(g, l, &off, &len, &blk);
        if (lane == 0) {
          const uint32_t w = (uint32_t)pcs;
          uint8_t* q = d + poff - 4;
          q[0] = (uint8_t)w; q[1] = (uint8_t)(w >> 8); q[2] = (uint8_t)(w >> 16); q[3] = (uint8_t)(w >> 24);
          if (pcs < 0) d[poff] = 0x1;   // run-length token
        }
        if (pcs <= 0) continue;
        const uint8_t* src = (pcs == len ? filt : sbuf) + (int64_t)c * g.wstride + off;
        if (aligned16(src)) wave_copy_a16((gout_t)(d + poff), (gin_t)src, pcs);
        else wave_copy((gout_t)(d + poff), (gin_t)src, pcs);
      }
    }
    k = wadd(f.sync + 1, 1);
  }
}

template <typename POS>
__host__ __device__ constexpr size_t enc_fused_lds(int hashlog, int nlds, int nglb) {
  return enc_wg_lds<POS>(hashlog, nlds, nglb) + ((sizeof(FusedArgs) + 15) & ~size_t(15));
}
// three 4-wave workgroups per CU (the VGPR limit) at hashlog 14 with u16 positions
static_assert(enc_fused_lds<uint16_t>(14, 1, 3) <= 160 * 1024 / 3, "exact fused encoder: LDS for fewer than 3 workgroups per CU");

template <typename POS, int NLDS, int NGLB>
__global__ __launch_bounds__(64 * (NLDS + NGLB)) __attribute__((amdgpu_waves_per_eu(3, 8)))
void k_encode_fused(CGeom g_arg, const uint8_t* __restrict__ filt_arg, uint8_t* __restrict__ sbuf_arg,
                    StreamResult* __restrict__ res_arg, int32_t nstreams_total_arg, int32_t* __restrict__ next_arg,
                    POS* __restrict__ gtab, const int32_t* __restrict__ porder_arg, EncFuse f_arg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int hashlog = g_arg.clevel == 1 ? 12 : (g_arg.clevel == 2 ? 13 : 14);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t tabsz = sizeof(POS) << hashlog;
  B2H_LDS FusedArgs* A = (B2H_LDS FusedArgs*)(smem + enc_wg_lds<POS>(hashlog, NLDS, NGLB));
  if (threadIdx.x == 0) {
    lds_store(&A->g, g_arg);
    lds_store(&A->f, f_arg);
    A->filt = filt_arg;
    A->sbuf = sbuf_arg;
    A->res = res_arg;
    A->next = next_arg;
    A->porder = porder_arg;
    A->nstreams_total = nstreams_total_arg;
    A->tablog = hashlog;
  }
  __syncthreads();
  B2H_LDS uint8_t* mine = (B2H_LDS uint8_t*)(smem + NLDS * tabsz + w * enc_wave_lds(hashlog));
  B2H_LDS uint32_t* dbits = (B2H_LDS uint32_t*)mine;
  B2H_LDS uint8_t* oring = mine + ((size_t(1) << hashlog) >> 3);
  if (NLDS > 0 && w < NLDS) {
    LdsTab<POS> t;
    t.t = (volatile B2H_LDS POS*)(smem + w * tabsz);
    encode_loop_fused(static_cast<const B2H_LDS FusedArgs*>(A), [&](gin_t in, int32_t len, int clevel, gout_t out, bool rt) {
      return encode_stream<LdsTab<POS>, true>(in, len, clevel, out, t, dbits, oring, rt);
    });
  } else if (NGLB > 0) {
    GlbTab<POS> t;
    t.t = (B2H_GLB POS*)(gtab + (((size_t)blockIdx.x * NGLB + (w - NLDS)) << hashlog));
    encode_loop_fused(static_cast<const B2H_LDS FusedArgs*>(A), [&](gin_t in, int32_t len, int clevel, gout_t out, bool rt) {
      StreamResult r = encode_stream<GlbTab<POS>, true>(in, len, clevel, out, t, dbits, oring, rt);
      r.windows |= 1 << 30;   // diagnostics: the stream ran on a global-table wave
      return r;
    });
  }
}

// BloscLZ mode 3 in one launch: k_encode_seg's W waves per workgroup (one shared candidate table
// under the LDS lock), each pulling its own streams through encode_loop_fused's per-wave protocol
// (typesize-4 SHUFFLE claims ahead of the wave's stream with the run verdict, finalisation by the
// wave completing a chunk, scatter items once the stream queue is empty).
template <bool CHK, int W>
__global__ __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(4, 8)))
void k_encode_seg_fused(CGeom g_arg, const uint8_t* __restrict__ filt_arg, uint8_t* __restrict__ sbuf_arg,
                        StreamResult* __restrict__ res_arg, int32_t nstreams_total_arg, int32_t* __restrict__ next_arg,
                        int tablog, const int32_t* __restrict__ porder_arg, EncFuse f_arg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* tab = (B2H_LDS uint8_t*)smem;
  B2H_LDS FusedArgs* A = (B2H_LDS FusedArgs*)(smem + (CHK ? (size_t)4 << tablog : (size_t)2 << tablog));
  const int64_t sb = seg_scratch_bytes(chain_len(g_arg));
  int32_t* lock = reinterpret_cast<int32_t*>(g_arg.chain + (int64_t)gridDim.x * W * sb) + 64 * blockIdx.x;
  if (threadIdx.x == 0) {
    atomicExch(lock, 0);
    lds_store(&A->g, g_arg);
    lds_store(&A->f, f_arg);
    A->filt = filt_arg;
    A->sbuf = sbuf_arg;
    A->res = res_arg;
    A->next = next_arg;
    A->porder = porder_arg;
    A->nstreams_total = nstreams_total_arg;
    A->tablog = tablog;
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* mine = g_arg.chain + ((int64_t)blockIdx.x * W + wave) * sb;
  B2H_GLB uint32_t* dist = (B2H_GLB uint32_t*)mine;
  B2H_GLB uint64_t* mask = (B2H_GLB uint64_t*)(mine + seg_dist_bytes(chain_len(g_arg)));
  B2H_GLB uint32_t* snv = (B2H_GLB uint32_t*)(mine + seg_dist_bytes(chain_len(g_arg)) + seg_mask_bytes(chain_len(g_arg)));
  encode_loop_fused(static_cast<const B2H_LDS FusedArgs*>(A), [&](gin_t in, int32_t len, int clevel, gout_t out, bool rt) {
    return encode_stream_seg<true, CHK>(in, len, clevel, out, tab, lds_uniform(&A->tablog), dist, mask, snv, rt, lock);
  });
}

// exact mode, default shape (1 LDS-table wave + 3 global-table waves, enc_mode hyb3) only
template <typename POS>
static int launch_encode_exact_fused(Workspace* ws, const CGeom& g, int hashlog, const uint8_t* filt,
                                     StreamResult* res, int64_t ntot, int32_t* next, const int32_t* porder, EncFuse f,
                                     hipStream_t st) {
  constexpr int NL = 1, NG = 3;
  const void* fn = reinterpret_cast<const void*>(&k_encode_fused<POS, NL, NG>);
  const size_t lds = enc_fused_lds<POS>(hashlog, NL, NG);
  static bool attr_set = false;
  if (!attr_set) {
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int slots = resident_slots(fn, lds, 64 * (NL + NG));
  const uint32_t grid =
      (uint32_t)std::max<int64_t>(1, std::min<int64_t>((ntot + NL + NG - 1) / (NL + NG), fuse_grid_cap(slots)));
  if (ws->gtab.ensure(((size_t)grid * NG << hashlog) * sizeof(POS))) return E_MEMORY;
  if (fuse_prepare(ws, g, ntot, f, st)) return E_MEMORY;
  k_encode_fused<POS, NL, NG><<<grid, 64 * (NL + NG), lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot,
                                                               next, ws->gtab.as<POS>(), porder, f);
  HIPCHK(hipGetLastError());
  k_fuse_check<<<(f.nchunks + 255) / 256, 256, 0, st>>>(f.sync, f.cbytes, f.nchunks);
  HIPCHK(hipGetLastError());
  return 0;
}
template <bool CHK, int W>
static int launch_encode_seg_fused_t(Workspace* ws, const CGeom& g0, const uint8_t* filt, StreamResult* res, int64_t ntot,
                                     int32_t* next, const int32_t* porder, EncFuse f, hipStream_t st, int tablog) {
  CGeom g = g0;
  const size_t lds = (CHK ? (size_t)4 << tablog : (size_t)2 << tablog) + ((sizeof(FusedArgs) + 15) & ~size_t(15));
  const void* fn = reinterpret_cast<const void*>(&k_encode_seg_fused<CHK, W>);
  static bool attr_set = false;
  if (!attr_set) {   // > 64 KiB of dynamic LDS at tablog 14: opt in once
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  const int slots = resident_slots(fn, lds, 64 * W);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>((ntot + W - 1) / W, fuse_grid_cap(slots)));
  const int64_t sb = seg_scratch_bytes(chain_len(g));
  if (ws->fchain.ensure((size_t)grid * W * (size_t)sb + (size_t)grid * 256 + 256)) return E_MEMORY;   // + lock words
  g.chain = ws->fchain.as<uint8_t>();
  if (fuse_prepare(ws, g, ntot, f, st)) return E_MEMORY;
  k_encode_seg_fused<CHK, W><<<grid, 64 * W, lds, st>>>(g, filt, ws->sbuf.as<uint8_t>(), res, (int32_t)ntot, next, tablog,
                                                        porder, f);
  HIPCHK(hipGetLastError());
  k_fuse_check<<<(f.nchunks + 255) / 256, 256, 0, st>>>(f.sync, f.cbytes, f.nchunks);
  HIPCHK(hipGetLastError());
  return 0;
}
static int launch_encode_seg_fused(Workspace* ws, const CGeom& g, const uint8_t* filt, StreamResult* res, int64_t ntot,
                                   int32_t* next, const int32_t* porder, const EncFuse& f, hipStream_t st) {
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const int tablog = std::min(fast_tablog(), hashlog);
  const int W = seg_waves();
#define B2H_SEG_LAUNCH(C, WW) return launch_encode_seg_fused_t<C, WW>(ws, g, filt, res, ntot, next, porder, f, st, tablog)
  if (chain_len(g) <= 65536) {
    if (W == 1) B2H_SEG_LAUNCH(true, 1);
    if (W == 2) B2H_SEG_LAUNCH(true, 2);
    if (W == 3) B2H_SEG_LAUNCH(true, 3);
    B2H_SEG_LAUNCH(true, 4);
  }
  if (W == 1) B2H_SEG_LAUNCH(false, 1);
  if (W == 2) B2H_SEG_LAUNCH(false, 2);
  if (W == 3) B2H_SEG_LAUNCH(false, 3);
  B2H_SEG_LAUNCH(false, 4);
#undef B2H_SEG_LAUNCH
}
// ============================================================ compression: host driver ====
static int32_t split_block(int32_t splitmode, int compcode, const uint8_t* filters, int32_t ts, int32_t bs) {
  // blosc/stune.c:186-215
  if (splitmode == 1) return 1;
  if (splitmode == 2) return 0;
  bool shuffle = false;
  for (int i = 0; i < kMaxFilters; i++) shuffle |= filters[i] == kShuffle;
  return (compcode == 0 || compcode == 1) && shuffle && ts <= kMaxStreams && (bs / ts) >= kMinBuffer;
}

int make_compress_plan(CompressPlan* p, int32_t nbytes, int32_t destsize, int clevel, int32_t typesize,
                       int32_t ctx_blocksize, int32_t splitmode, const uint8_t* filters,
                       const uint8_t* filters_meta, int32_t* computed_blocksize, bool extended, int compcode,
                       int compcode_meta, int user_version, int use_dict) {
  memset(p, 0, sizeof *p);
  // BloscLZ and LZ4 on the device; user codecs (> BLOSC2_DEFINED_CODECS_STOP) through host callbacks
  if (compcode != 0 && compcode != 1 && compcode <= 31) return -7;   // BLOSC2_ERROR_CODEC_SUPPORT
  p->compcode = compcode;
  p->overhead = extended ? kHdrExt : kHdrMin;
  if (nbytes > 0x7fffffff - kHdrExt) return E_MAXBUF;
  if (destsize < kHdrExt) return E_MAXBUF;
  if (clevel < 0 || clevel > 9) return -8;   // BLOSC2_ERROR_CODEC_PARAM
  // stune (blosc/stune.c:47-165) with the incoming typesize, before the >255 cap
  int32_t bs;
  if (nbytes < typesize) {
    bs = 1;
  } else {
    const int32_t splitmode_nb = split_block(splitmode, compcode, filters, typesize, nbytes);
    bs = nbytes;
    if (ctx_blocksize) {
      bs = ctx_blocksize;
    } else {
      if (nbytes >= 32 * 1024) {
        static const int32_t scale[10] = {8 << 10, 16 << 10, 32 << 10, 64 << 10, 128 << 10,
                                          128 << 10, 256 << 10, 256 << 10, 256 << 10, 256 << 10};
        bs = scale[clevel];
      }
      if (clevel > 0 && splitmode_nb) {
        static const int32_t per_ts[10] = {0, 32, 32, 32, 64, 64, 64, 128, 256, 512};
        bs = per_ts[clevel] * 1024 * typesize;
        if (bs > 4 * 1024 * 1024) bs = 4 * 1024 * 1024;
        if (bs < 32 * 1024) bs = 32 * 1024;
      }
    }
    if (bs > nbytes) bs = nbytes;
    if (bs > typesize) bs = bs / typesize * typesize;
  }
  *computed_blocksize = bs;
  const int32_t ts = typesize > 255 ? 1 : typesize;
  p->nbytes = nbytes;
  p->typesize = ts;
  p->clevel = clevel;
  p->blocksize = bs;
  p->destsize = destsize;
  memcpy(p->filters, filters, 6);
  memcpy(p->filters_meta, filters_meta, 6);
  const int32_t nblocks = bs ? nbytes / bs + (nbytes % bs ? 1 : 0) : 0;
  // write_compression_header (blosc/blosc2.c:2911-3001)
  uint8_t flags = extended ? (kFlagShuffle | kFlagBitshuffle) : 0;
  bool memcpyed = clevel == 0 || nbytes < kMinBuffer;
  // a dictionary's training pass writes no bstarts: only the header must fit (2940-2942, 2960)
  const bool dict_training = use_dict && compcode == 1 && extended;
  if (!memcpyed && p->overhead + (dict_training ? 0 : 4 * nblocks) > destsize) memcpyed = true;
  if (memcpyed) {
    flags |= kFlagMemcpy;
  } else {
    for (int i = 0; i < kMaxFilters; i++) {
      if (filters[i] == kShuffle) flags |= kFlagShuffle;
      if (filters[i] == kBitshuffle) flags |= kFlagBitshuffle;
      if (filters[i] == kDelta) flags |= kFlagDelta;
    }
    p->split = split_block(splitmode, compcode, filters, ts, bs) != 0;
    if (!p->split) flags |= kFlagDontSplit;
    // compformat (compcode_to_compformat, blosc/blosc2.c:396-414, 2990-2991): user codecs -> UDCODEC (6)
    flags |= (uint8_t)((compcode <= 1 ? compcode : 6) << 5);
  }
  p->memcpyed = memcpyed;
  int32_t hb = ctx_blocksize > 0 ? ctx_blocksize : bs;
  if (nbytes > 0 && hb > nbytes) hb = nbytes;
  p->header_blocksize = hb;
  uint8_t* h = p->header;
  memset(h, 0, 32);
  // versionlz: compcode_to_compversion (blosc/blosc2.c:418-446), a user codec's registered version
  h[0] = 5; h[1] = (uint8_t)(compcode <= 1 ? 1 : user_version); h[2] = flags; h[3] = (uint8_t)ts;
  for (int k = 0; k < 4; k++) { h[4 + k] = (uint8_t)(nbytes >> (8 * k)); h[8 + k] = (uint8_t)(hb >> (8 * k)); }
  for (int i = 0; i < 6; i++) { h[16 + i] = filters[i]; h[24 + i] = filters_meta[i]; }
  h[22] = (uint8_t)compcode;   // udcompcode = the codec (blosc/blosc2.c:1030)
  h[23] = (uint8_t)compcode_meta;
  // LZ4 dictionaries (blosc/blosc2.c:3151-3235): the size the reference derives from the chunk
  // geometry; below BLOSC2_MINUSEFULDICT (or a zero sample) it compresses without one
  p->use_dict = use_dict && compcode == 1 && !memcpyed;
  p->dict_size = 0;
  if (p->use_dict) {
    int32_t nbe = p->split ? nblocks * ts : nblocks;
    if (nbe < 8) nbe = 8;
    const int32_t sample = nbytes / nbe / 16;
    const int32_t dmax = std::min(32 * 1024, nbytes / 20);
    if (dmax >= 256 && sample > 0) {
      p->dict_size = (int32_t)std::min<int64_t>((int64_t)nbe * sample, dmax);
      h[31] |= 0x01;   // BLOSC2_USEDICT (blosc2_initialize_header_from_context, 1037-1039)
    }
  }
  return 0;
}

// int_trunc's precision check (plugins/filters/int_trunc/int_trunc.c:18-83): uint8 arithmetic on
// the zeroed bit count, element sizes 1/2/4/8 only.
static bool hostside_int_trunc_ok(int8_t prec, int32_t ts, int* zeroed) {
  if (ts != 1 && ts != 2 && ts != 4 && ts != 8) return false;
  const uint8_t bits = (uint8_t)(8 * ts);
  const uint8_t z = prec >= 0 ? (uint8_t)(bits - prec) : (uint8_t)(-prec);
  if (z >= bits) return false;
  *zeroed = z;
  return true;
}

static bool hostside_trunc_ok(int8_t prec, int32_t ts, int* zeroed) {
  const int mant = ts == 4 ? 23 : (ts == 8 ? 52 : -1);
  if (mant < 0) return false;
  const int pp = prec;
  if ((pp < 0 ? -pp : pp) > mant) return false;
  *zeroed = pp >= 0 ? mant - pp : -pp;
  return *zeroed < mant;
}

// Encoder workgroup shape: B2H_ENC_MODE = "lds" (one LDS-table wave per workgroup), "glb" (one
// global-table wave), or "hybN" (one LDS-table wave + N global-table waves).  Default: hyb3, i.e.
// 3 LDS-table + 9 global-table waves per CU (T bench: lds 54.2 ms, glb 30.3, hyb1 34.4, hyb2 33.1,
// hyb3 28.7, hyb4 32.3 ms per 4 GiB encode -- more global tables than that overflow L2 into MALL).
// Unset (and b2h_set_encode_shape(-1, -1)): "auto" -- hyb3, except that a batch whose streams all
// fit the LDS-only shape's resident waves at once (a per-call chunk: blosc1_compress and
// blosc2_compress_ctx encode one chunk, 8-64 streams) runs there: then every stream has its own
// LDS table and the call's latency is one stream's walk on it (C1 per call).
static int g_enc_ml = -2, g_enc_mg = -2;   // -2: not read yet; -1: auto
static void enc_mode(int* nlds, int* nglb) {
  if (g_enc_ml == -2) {
    const char* e = getenv("B2H_ENC_MODE");
    g_enc_ml = -1; g_enc_mg = -1;
    if (e && !strcmp(e, "lds")) { g_enc_ml = 1; g_enc_mg = 0; }
    else if (e && !strcmp(e, "glb")) { g_enc_ml = 0; g_enc_mg = 1; }
    else if (e && !strncmp(e, "hyb", 3)) { g_enc_ml = 1; g_enc_mg = std::max(1, std::min(4, atoi(e + 3))); }
  }
  *nlds = g_enc_ml;
  *nglb = g_enc_mg;
}
int set_encode_shape(int nlds, int nglb) {
  int ml, mg;
  enc_mode(&ml, &mg);
  const int prev = ml < 0 ? -1 : ml * 16 + mg;
  if (nlds == -1 && nglb == -1) { g_enc_ml = -1; g_enc_mg = -1; }
  else if (nlds == 1 && nglb >= 0 && nglb <= 4) { g_enc_ml = 1; g_enc_mg = nglb; }
  else if (nlds == 0 && nglb == 1) { g_enc_ml = 0; g_enc_mg = 1; }
  else if (nlds != -2) return -1;
  return prev;
}
// resident waves of the LDS-only shape (one LDS-table wave per workgroup) on this device
template <typename POS>
static int64_t lds_only_slots(int hashlog) {
  const void* fn = reinterpret_cast<const void*>(&k_encode<POS, 1, 0>);
  static bool attr_set = false;
  if (!attr_set) {
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  int dev = 0, per_cu = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64, enc_wg_lds<POS>(hashlog, 1, 0)) != hipSuccess) per_cu = 1;
  return (int64_t)std::max(1, per_cu) * std::max(1, ncu);
}

template <typename POS, int NL, int NG>
static int launch_encode_shape(Workspace* ws, const CGeom& g, int hashlog, const uint8_t* filt, StreamResult* res,
                               int64_t ntot, int32_t* next, const int32_t* porder, hipStream_t st) {
  const void* fn = reinterpret_cast<const void*>(&k_encode<POS, NL, NG>);
  const size_t lds = enc_wg_lds<POS>(hashlog, NL, NG);
  static bool attr_set = false;
  if (!attr_set) {   // > 64 KiB of dynamic LDS per workgroup: opt in once
    HIPCHK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = true;
  }
  int dev = 0, per_cu = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) ncu = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * (NL + NG), lds) != hipSuccess) per_cu = 1;
  const int64_t slots = (int64_t)std::max(1, per_cu) * std::max(1, ncu);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>((ntot + NL + NG - 1) / (NL + NG), slots));
  POS* gt = nullptr;
  if (NG > 0) {
    if (ws->gtab.ensure(((size_t)grid * NG << hashlog) * sizeof(POS))) return E_MEMORY;
    gt = ws->gtab.as<POS>();
  }
  EncArgs args;
  args.g = g;
  args.filt = filt;
  args.sbuf = ws->sbuf.as<uint8_t>();
  args.res = res;
  args.next = next;
  args.porder = porder;
  args.nstreams_total = (int32_t)ntot;
  args.pad = 0;
  k_encode<POS, NL, NG><<<grid, 64 * (NL + NG), lds, st>>>(args, gt);
  HIPCHK(hipGetLastError());
  return 0;
}

template <typename POS>
static int launch_encode(Workspace* ws, const CGeom& g, int hashlog, const uint8_t* filt, StreamResult* res,
                         int64_t ntot, int32_t* next, const int32_t* porder, hipStream_t st) {
  int nl, ng;
  enc_mode(&nl, &ng);
  if (nl < 0) {   // auto
    nl = 1;
    ng = ntot <= lds_only_slots<POS>(hashlog) ? 0 : 3;
  }
  if (nl == 1 && ng == 0) return launch_encode_shape<POS, 1, 0>(ws, g, hashlog, filt, res, ntot, next, porder, st);
  if (nl == 0) return launch_encode_shape<POS, 0, 1>(ws, g, hashlog, filt, res, ntot, next, porder, st);
  if (ng == 1) return launch_encode_shape<POS, 1, 1>(ws, g, hashlog, filt, res, ntot, next, porder, st);
  if (ng == 2) return launch_encode_shape<POS, 1, 2>(ws, g, hashlog, filt, res, ntot, next, porder, st);
  if (ng == 3) return launch_encode_shape<POS, 1, 3>(ws, g, hashlog, filt, res, ntot, next, porder, st);
  return launch_encode_shape<POS, 1, 4>(ws, g, hashlog, filt, res, ntot, next, porder, st);
}

static CGeom make_geom(const CompressPlan& P, int64_t src_stride, int64_t dst_stride) {
  CGeom g{};
  const int32_t n = P.nbytes;
  g.nbytes = n;
  g.bs = P.blocksize;
  g.ts = P.typesize;
  g.clevel = P.clevel;
  g.destsize = P.destsize;
  g.overhead = P.overhead;
  g.compcode = P.compcode;
  g.dict_size = P.use_dict ? P.dict_size : 0;
  g.lzmode = (P.lz_mode >= 0 && P.lz_mode <= 3) ? P.lz_mode : lz_mode();
  g.src_stride = src_stride;
  g.dst_stride = dst_stride;
  g.wstride = ((int64_t)n + 255) / 256 * 256 + 256;
  if (!P.memcpyed && g.bs > 0) {
    g.nblocks = n / g.bs + (n % g.bs ? 1 : 0);
    g.leftover = n % g.bs;
    g.spb = P.split ? g.ts : 1;
    g.neblock = g.bs / g.spb;
    const int32_t full = g.nblocks - (g.leftover ? 1 : 0);
    g.nsc = full * g.spb + (g.leftover ? 1 : 0);
  }
  return g;
}

static int encode_stage(Workspace* ws, const CompressPlan& P, CGeom& g, const uint8_t* filt, const uint8_t* raw,
                        int64_t raw_stride, uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes, int32_t nchunks,
                        const uint8_t* htpl, int64_t ntot, hipStream_t st, const uint8_t* fuse_raw = nullptr,
                        int fuse_ds_ts = 0, bool timed = true);

int compress_batch(const CompressPlan& P, const uint8_t* d_src, int64_t src_stride, int32_t nchunks, uint8_t* d_dst,
                   int64_t dst_stride, int32_t* d_cbytes, hipStream_t st, Workspace* wsx) {
  if (nchunks <= 0) return 0;
  Workspace* ws = wsx ? wsx : ws_for_current_device();
  WsUse use(ws, st);
  if (use.rc) return use.rc;
  const int32_t n = P.nbytes;
  CGeom g = make_geom(P, src_stride, dst_stride);
  if (P.memcpyed) {
    if (ws->mode.ensure(64) < 0) return E_MEMORY;
    uint8_t* htpl = ws->mode.as<uint8_t>();
    HIPCHK(hipMemcpyAsync(htpl, P.header, 32, hipMemcpyHostToDevice, st));
    dim3 grid(std::max(1, std::min(64, n / (256 * 16) + 1)), std::min(nchunks, kMemcpyGridY));
    k_memcpy_chunks<<<grid, 256, 0, st>>>(d_src, src_stride, d_dst, dst_stride, n, nullptr, htpl, d_cbytes,
                                          P.overhead, P.destsize, nullptr, nchunks);
    HIPCHK(hipGetLastError());
    return 0;
  }
  const int64_t ntot = (int64_t)nchunks * g.nsc;
  if (ntot > 0x7fffffff) { snprintf(g_err, sizeof g_err, "too many streams"); return E_PARAM; }

  // active forward filters and their buffers (ring tmp, tmp2, input -- see header comment)
  int act[6], nact = 0;
  for (int i = 0; i < 6; i++) if (P.filters[i] != kNoFilter) act[nact++] = i;
  for (int k = 0; k < nact; k++) {
    const uint8_t f = P.filters[act[k]];
    if (f > kTruncPrec && f != kBytedelta && f != kIntTrunc) {
      snprintf(g_err, sizeof g_err, "filter %d is neither built in nor a device plugin filter", f);
      return E_FILTER;
    }
  }
  const size_t wbytes = (size_t)g.wstride * nchunks;
  int rc = 0;
  if (nact >= 1) rc |= ws->t1.ensure(wbytes);
  if (nact >= 2) rc |= ws->t2.ensure(wbytes);
  const bool clobber = nact >= 3;
  if (clobber) rc |= ws->work.ensure(wbytes);
  rc |= ws->sbuf.ensure(wbytes);
  rc |= ws->res.ensure(sizeof(StreamResult) * (size_t)ntot);
  rc |= ws->place.ensure(sizeof(Place) * (size_t)ntot);
  rc |= ws->mode.ensure(sizeof(int32_t) * (size_t)nchunks + 64);
  if (rc) return E_MEMORY;
  uint8_t* htpl = ws->mode.as<uint8_t>() + sizeof(int32_t) * (size_t)nchunks;
  htpl = reinterpret_cast<uint8_t*>((reinterpret_cast<uintptr_t>(htpl) + 15) & ~uintptr_t(15));
  HIPCHK(hipMemcpyAsync(htpl, P.header, 32, hipMemcpyHostToDevice, st));
  if (P.use_dict && (int64_t)P.nbytes + P.overhead > P.destsize) {
    // The reference's training pass stores the filtered blocks uncompressed (blosc_c with
    // dict_training, blosc/blosc2.c:1343-1356), each after its filters ran: a filter error first;
    // then the first block that does not fit gives up the chunk when no room is left at all (the
    // memcpy bit stays set and both passes give up, 3036-3052: cbytes 0), and is an overrun
    // otherwise (cbytes > maxout, 1417-1420).
    for (int k = 0; k < nact; k++) {
      const uint8_t f = P.filters[act[k]], meta = P.filters_meta[act[k]];
      int zeroed = 0;
      if (f == kTruncPrec && !hostside_trunc_ok((int8_t)meta, g.ts, &zeroed)) return E_FILTER;
      if (f == kIntTrunc && !hostside_int_trunc_ok((int8_t)meta, P.typesize, &zeroed)) return E_FILTER;
    }
    const int64_t room = (int64_t)P.destsize - P.overhead;
    if (room > 0 && room % g.bs != 0) {
      snprintf(g_err, sizeof g_err, "dictionary training block overruns the destination");
      return E_WRITE;
    }
    k_memcpy_chunks<<<dim3(1, std::min(nchunks, kMemcpyGridY)), 256, 0, st>>>(d_src, src_stride, d_dst, dst_stride, n, nullptr,
                                                                            htpl, d_cbytes, P.overhead, P.destsize, nullptr,
                                                                            nchunks);
    HIPCHK(hipGetLastError());
    return 0;
  }
  if (g.dict_size > 0 && (int64_t)P.overhead + 4 * g.nblocks + 4 + g.dict_size > P.destsize) {
    // only with blocks of a few bytes: the reference then stores the dictionary past destsize
    snprintf(g_err, sizeof g_err, "bstarts + dictionary section exceed destsize");
    return E_PARAM;
  }

  const uint8_t* raw = d_src;
  int64_t raw_stride = src_stride;
  if (clobber) {
    dim3 grid(std::max(1, std::min(256, n / (256 * 16) + 1)), nchunks);
    k_copy_work<<<grid, 256, 0, st>>>(d_src, src_stride, ws->work.as<uint8_t>(), g.wstride, n);
    raw = ws->work.as<uint8_t>();
    raw_stride = g.wstride;
  }
  // forward filters
  ev_filter.start(st);
  const uint8_t* filt = raw;
  int64_t filt_stride = raw_stride;
  uint8_t* ring[3] = {ws->t1.as<uint8_t>(), ws->t2.as<uint8_t>(), ws->work.as<uint8_t>()};
  bool has_delta = false;
  for (int k = 0; k < nact; k++) has_delta |= P.filters[act[k]] == kDelta;
  const bool two_pass = clobber && has_delta && g.nblocks > 1;
  const bool fuse_ds = nact == 2 && P.filters[act[0]] == kDelta && P.filters[act[1]] == kShuffle &&
                       (P.filters_meta[act[1]] == 0 || P.filters_meta[act[1]] == g.ts) &&
                       (g.ts == 2 || g.ts == 4 || g.ts == 8);
  auto run_filters = [&]() -> int {
    if (fuse_ds) {   // output where the two-launch loop leaves it: ring[1], stride wstride
      dim3 grid(g.nblocks, nchunks);
      k_ffilter_ds<<<grid, kBlockThreads, 0, st>>>(g, raw, raw_stride, ring[0], ring[1], g.wstride);
      filt = ring[1];
      filt_stride = g.wstride;
    }
    for (int pass = two_pass ? 1 : 0; pass <= (two_pass ? 2 : 0) && !fuse_ds; pass++) {
      const uint8_t* cur = raw;
      int64_t cur_stride = raw_stride;
      for (int k = 0; k < nact; k++) {
        const uint8_t f = P.filters[act[k]], meta = P.filters_meta[act[k]];
        int zeroed = 0;
        if (f == kTruncPrec && !hostside_trunc_ok((int8_t)meta, g.ts, &zeroed)) return E_FILTER;
        if (f == kIntTrunc && !hostside_int_trunc_ok((int8_t)meta, P.typesize, &zeroed)) return E_FILTER;
        // bytedelta's channel count is its meta; 0 means the super-chunk's typesize (bytedelta.c:90-98),
        // which a caller without a super-chunk resolves before this point -- the chunk's own here
        const uint8_t kmeta = (f == kBytedelta && meta == 0) ? (uint8_t)g.ts : meta;
        uint8_t* outb = ring[k % 3];
        dim3 grid(pass == 1 ? 1 : (pass == 2 ? g.nblocks - 1 : g.nblocks), nchunks);
        k_ffilter<<<grid, kBlockThreads, 0, st>>>(g, pass, f, kmeta, cur, cur_stride, outb, g.wstride, raw, raw_stride, zeroed);
        cur = outb;
        cur_stride = g.wstride;
      }
      filt = cur;
      filt_stride = cur_stride;
    }
    return 0;
  };
  // the lone typesize-4 byte shuffle of a fast-mode batch runs inside the encode launch
  const uint8_t meta0 = nact == 1 ? P.filters_meta[act[0]] : 0;
  const bool fuse_shuffle = nact == 1 && P.filters[act[0]] == kShuffle && (meta0 == 0 || meta0 == 4) && g.ts == 4 &&
                            g.bs % 64 == 0 && g.leftover % 64 == 0 && !clobber && g.dict_size == 0 &&
                            (reinterpret_cast<uintptr_t>(raw) & 15) == 0 && raw_stride % 16 == 0 &&
                            (fuse_bits() & 2) && fused_encode_ok(g);
  // and (DELTA, SHUFFLE) at typesize 2/4/8 too (k_ffilter_ds's job, whole 64-byte groups)
  const bool fuse_dsjob = !fuse_shuffle && fuse_ds && g.bs % 64 == 0 && g.leftover % 64 == 0 && !clobber &&
                          g.dict_size == 0 && (reinterpret_cast<uintptr_t>(raw) & 15) == 0 && raw_stride % 16 == 0 &&
                          (fuse_bits() & 2) && fused_encode_ok(g);
  if (fuse_shuffle || fuse_dsjob) {
    filt = ring[0];
    filt_stride = g.wstride;
  } else if ((rc = run_filters())) {
    return rc;
  }
  if (nact > 0 && filt_stride != g.wstride) return E_FAILURE;
  // encoder reads the filtered streams at c*wstride: if no filter ran, stage the input there
  if (nact == 0) {
    rc = ws->t1.ensure(wbytes);
    if (rc) return rc;
    dim3 grid(std::max(1, std::min(256, n / (256 * 16) + 1)), nchunks);
    k_copy_work<<<grid, 256, 0, st>>>(raw, raw_stride, ws->t1.as<uint8_t>(), g.wstride, n);
    filt = ws->t1.as<uint8_t>();
  }
  if (g.dict_size > 0) {
    // the dictionary section comes from the training pass's image (blosc/blosc2.c:3146-3221)
    k_put_dict<<<nchunks, 256, 0, st>>>(g, filt, d_dst);
    // with >= 3 filters that pass rewrote the input (pipeline_forward's buffer cycle, 1048-1180): the real pass
    // filters the rewritten input again
    if (clobber && (rc = run_filters())) return rc;
  }
  ev_filter.stop(st);
  HIPCHK(hipGetLastError());
  const bool fused = g.compcode == 0 && fused_encode_ok(g);
  rc = encode_stage(ws, P, g, filt, raw, raw_stride, d_dst, dst_stride, d_cbytes, nchunks, htpl, ntot, st,
                    (fuse_shuffle || fuse_dsjob) ? raw : nullptr, fuse_dsjob ? g.ts : 0);
  if (rc || !fused || !fuse_rescue()) return rc;
  // Rescue: a fused launch whose hand-off wait timed out leaves every chunk of the batch
  // BLOSC2_ERROR_FAILURE (k_fuse_check).  The separate launches are queued behind it, gated on its
  // timeout word: they redo the batch (filters the fused launch ran, encode, finalize, scatter,
  // memcpy fallbacks) only when that word is set, and exit at once otherwise -- so the batch API
  // stays asynchronous and a timeout no longer fails it.
  g.gate = ws->fsync.as<int32_t>() + 4;
  if ((fuse_shuffle || fuse_dsjob) && (rc = run_filters())) return rc;
  const bool was_off = t_fuse_off;
  t_fuse_off = true;
  rc = encode_stage(ws, P, g, filt, raw, raw_stride, d_dst, dst_stride, d_cbytes, nchunks, htpl, ntot, st, nullptr, 0,
                    false);
  t_fuse_off = was_off;
  return rc;
}

// The codec stage of a batch whose filtered images sit at filt + c * g.wstride: encode every stream,
// then the serial-layout finalisation, the payload scatter and the memcpy fallbacks (from raw).
static int encode_stage(Workspace* ws, const CompressPlan& P, CGeom& g, const uint8_t* filt, const uint8_t* raw,
                        int64_t raw_stride, uint8_t* d_dst, int64_t dst_stride, int32_t* d_cbytes, int32_t nchunks,
                        const uint8_t* htpl, int64_t ntot, hipStream_t st, const uint8_t* fuse_raw, int fuse_ds_ts,
                        bool timed) {
  const int32_t n = P.nbytes;
  int rc = 0;
  // encode
  if (timed) ev_encode.start(st);
  const int hashlog = g.clevel == 1 ? 12 : (g.clevel == 2 ? 13 : 14);
  const bool small = std::max(g.neblock, g.leftover) <= 65536;
  StreamResult* res = ws->res.as<StreamResult>();
  const bool fused = fused_encode_ok(g);   // finalize + scatter (and fuse_raw's shuffle) inside the encode launch
  if (fuse_raw && !fused) return E_FAILURE;
  rc = ws->qctr.ensure(16);
  if (rc) return rc;
  int32_t* next = ws->qctr.as<int32_t>();
  HIPCHK(hipMemsetAsync(next, 0, sizeof(int32_t), st));
  if (g.compcode == 1) {
    rc = launch_encode_lz4(ws, g, filt, res, ntot, next, st, d_dst);
    if (rc) return rc;
  } else {
    static const int front = [] { const char* e = getenv("B2H_ENC_FRONT"); return e ? std::max(0, atoi(e)) : 2; }();
    g.front = front;
    if (ws->porder.ensure(32 * sizeof(int32_t))) return E_MEMORY;
    int32_t* porder = ws->porder.as<int32_t>();
    if (!ws->porder_init) {   // no learned order yet: stream order
      HIPCHK(hipMemsetAsync(porder, 0, 32 * sizeof(int32_t), st));
      ws->porder_init = true;
    }
    if (fused) {
      EncFuse f{};
      f.raw = fuse_raw;
      f.ds = fuse_ds_ts;
      f.raw_stride = raw_stride;
      f.filt = const_cast<uint8_t*>(filt);
      f.place = ws->place.as<Place>();
      f.mode = ws->mode.as<int32_t>();
      f.dst = d_dst;
      f.cbytes = d_cbytes;
      f.htpl = htpl;
      f.nchunks = nchunks;
      if (g.lzmode == 3) rc = launch_encode_seg_fused(ws, g, filt, res, ntot, next, porder, f, st);
      else if (g.lzmode != 0) rc = launch_encode_fast_fused(ws, g, filt, res, ntot, next, porder, f, st);
      else rc = small ? launch_encode_exact_fused<uint16_t>(ws, g, hashlog, filt, res, ntot, next, porder, f, st)
                      : launch_encode_exact_fused<uint32_t>(ws, g, hashlog, filt, res, ntot, next, porder, f, st);
    } else if (g.lzmode == 3) rc = launch_encode_seg(ws, g, filt, res, ntot, next, porder, st);
    else if (g.lzmode != 0) rc = launch_encode_fast(ws, g, filt, res, ntot, next, porder, st);
    else rc = small ? launch_encode<uint16_t>(ws, g, hashlog, filt, res, ntot, next, porder, st)
                    : launch_encode<uint32_t>(ws, g, hashlog, filt, res, ntot, next, porder, st);
    if (rc) return rc;
    k_plane_cost<<<1, 1024, 0, st>>>(g, res, (int32_t)ntot, porder);
  }
  if (timed) ev_encode.stop(st);
  HIPCHK(hipGetLastError());

  if (timed) ev_final.start(st);
  Place* place = ws->place.as<Place>();
  int32_t* mode = ws->mode.as<int32_t>();
  if (!fused) {
    k_finalize<<<(nchunks + 63) / 64, 64, 0, st>>>(g, res, place, mode, d_dst, d_cbytes, nchunks, htpl);
    k_scatter<<<(uint32_t)std::min<int64_t>(ntot, kScatterGrid), kBlockThreads, 0, st>>>(
        g, place, mode, res, filt, ws->sbuf.as<uint8_t>(), d_dst, (int32_t)ntot);
  }
  {
    dim3 grid(std::max(1, std::min(64, n / (256 * 16) + 1)), std::min(nchunks, kMemcpyGridY));
    k_memcpy_chunks<<<grid, 256, 0, st>>>(raw, raw_stride, d_dst, dst_stride, n, mode, htpl, d_cbytes,
                                          P.overhead, P.destsize, g.gate, nchunks);
  }
  if (timed) ev_final.stop(st);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------- single-chunk stages (host-driven pipelines) ----
// Chunks whose pipeline holds a user-registered filter or codec run the reference's per-block /
// per-stream host callbacks between device stages (blosc2_api.cpp).  These are the device stages,
// for ONE chunk in device buffers carrying >= 256 bytes of slack.

// One forward filter (slot `slot` of P) over the blocks of `pass` (0 all, 1 block 0, 2 the others).
int forward_filter_chunk(const CompressPlan& P, int slot, int pass, const uint8_t* d_in, uint8_t* d_out,
                         const uint8_t* d_raw, hipStream_t st) {
  CGeom g = make_geom(P, 0, 0);
  const uint8_t f = P.filters[slot], meta = P.filters_meta[slot];
  if (f == kNoFilter || g.nblocks == 0) return 0;
  int zeroed = 0;
  if (f == kTruncPrec && !hostside_trunc_ok((int8_t)meta, g.ts, &zeroed)) return E_FILTER;
  if (f == kIntTrunc && !hostside_int_trunc_ok((int8_t)meta, P.typesize, &zeroed)) return E_FILTER;
  if (f > kTruncPrec && f != kBytedelta && f != kIntTrunc) return E_FILTER;
  const uint8_t kmeta = (f == kBytedelta && meta == 0) ? (uint8_t)g.ts : meta;
  const int32_t nb = pass == 1 ? 1 : (pass == 2 ? g.nblocks - 1 : g.nblocks);
  if (nb <= 0) return 0;
  k_ffilter<<<dim3(nb, 1), kBlockThreads, 0, st>>>(g, pass, f, kmeta, d_in, 0, d_out, 0, d_raw, 0, zeroed);
  HIPCHK(hipGetLastError());
  return 0;
}

// The codec stage for one chunk whose filtered image is d_filt (BloscLZ / LZ4): chunk -> d_dst,
// cbytes -> *d_cbytes.  d_raw is what a memcpy fallback stores.
int encode_chunk_filtered(const CompressPlan& P, const uint8_t* d_filt, const uint8_t* d_raw, uint8_t* d_dst,
                          int32_t* d_cbytes, hipStream_t st, Workspace* wsx) {
  Workspace* ws = wsx ? wsx : ws_for_current_device();
  WsUse use(ws, st);
  if (use.rc) return use.rc;
  CGeom g = make_geom(P, 0, 0);
  const int64_t ntot = g.nsc;
  int rc = 0;
  rc |= ws->sbuf.ensure((size_t)g.wstride);
  rc |= ws->res.ensure(sizeof(StreamResult) * (size_t)std::max<int64_t>(1, ntot));
  rc |= ws->place.ensure(sizeof(Place) * (size_t)std::max<int64_t>(1, ntot));
  rc |= ws->mode.ensure(sizeof(int32_t) + 64);
  if (rc) return E_MEMORY;
  uint8_t* htpl = ws->mode.as<uint8_t>() + 16;
  HIPCHK(hipMemcpyAsync(htpl, P.header, 32, hipMemcpyHostToDevice, st));
  return encode_stage(ws, P, g, d_filt, d_raw, 0, d_dst, 0, d_cbytes, 1, htpl, ntot, st);
}

// One backward filter over the blocks of `pass` of one chunk: in -> out; delta's blocks >= 1 XOR
// with the final output's block 0 (d_final), as pipeline_backward does (blosc/blosc2.c:1505-1529).
__global__ __launch_bounds__(kBlockThreads) void k_dfilter_chunk(uint8_t filter, uint8_t meta, int32_t ts, int32_t nbytes,
                                                                 int32_t bs, uint8_t version, int pass,
                                                                 const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                                 const uint8_t* __restrict__ final_out) {
  const int32_t nblocks = nbytes / bs + (nbytes % bs ? 1 : 0);
  const int32_t b = pass == 2 ? (int32_t)blockIdx.x + 1 : (int32_t)blockIdx.x;
  if (b >= nblocks) return;
  const int32_t bsize = (b == nblocks - 1 && nbytes % bs) ? nbytes % bs : bs;
  const int64_t off = (int64_t)b * bs;
  switch (filter) {
    case kShuffle: block_unshuffle(in + off, out + off, bsize, meta ? meta : ts); break;
    case kBitshuffle: block_bitunshuffle(in + off, out + off, bsize, ts, version); break;
    case kBytedelta: block_bytedelta_decode(in + off, out + off, bsize, meta ? meta : ts); break;
    case kDelta:
      if (b == 0 || pass == 3) block_delta_decode_first(in + off, out + off, bsize, ts);   // 3: each block self
      else block_delta_decode_rest(in + off, final_out, out + off, bsize, ts);
      break;
    default: break;
  }
}

int backward_filter_chunk(uint8_t filter, uint8_t meta, int32_t typesize, int32_t nbytes, int32_t blocksize,
                          uint8_t version, int pass, const uint8_t* d_in, uint8_t* d_out, const uint8_t* d_final,
                          hipStream_t st) {
  if (nbytes <= 0 || blocksize <= 0) return 0;
  if (filter != kShuffle && filter != kBitshuffle && filter != kDelta && filter != kBytedelta) return E_FILTER;
  const int32_t nblocks = nbytes / blocksize + (nbytes % blocksize ? 1 : 0);
  const int32_t nb = pass == 1 ? 1 : (pass == 2 ? nblocks - 1 : nblocks);
  if (nb <= 0) return 0;
  k_dfilter_chunk<<<nb, kBlockThreads, 0, st>>>(filter, meta, typesize, nbytes, blocksize, version, pass, d_in, d_out,
                                                 d_final);
  HIPCHK(hipGetLastError());
  return 0;
}

// ============================================================== decompression: planning ====
__device__ __forceinline__ int32_t rd32(const uint8_t* p) {
  return (int32_t)((uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24));
}

// Filters with nothing to undo: TRUNC_PREC (blosc/blosc2.c:1531-1533) and int_trunc, whose
// backward is a plain copy (plugins/filters/int_trunc/int_trunc.c:116-125).
__host__ __device__ __forceinline__ bool bwd_noop(uint8_t f) { return f == kNoFilter || f == kTruncPrec || f == kIntTrunc; }

// The chunk-level checks of a decompression, in the reference's order and with its codes:
// read_chunk_header (blosc/blosc2.c:738-852), the destination check of
// blosc_run_decompression_with_context (3921-3924), blosc2_initialize_context_from_header
// (862-910) and initialize_context_decompression (2723-2906).  Block-level failures (bstarts,
// stream sizes, decoding, the filter pipeline) are keyed by position in DChunk::errkey, so the
// batch reports the error the reference's serial block walk meets first.
// mode bit 0: raw streams (host-driven pipelines apply the filters); bit 1: every block
// un-deltas against itself (blosc_d with dest_offset 0: getitem / decompress_block); bit 2: the
// dictionary flag is not read (those two entry points never parse the section).
__global__ void k_dplan_chunks(const uint8_t* const* __restrict__ srcs, const int32_t* __restrict__ srcsize,
                               const int32_t* __restrict__ dstsize, DChunk* __restrict__ ch, int32_t n,
                               int mode) {
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  DChunk d;
  memset(&d, 0, sizeof d);
  d.errkey = kNoErr;
  const uint8_t* s = srcs[c];
  const int32_t ss = srcsize[c];
  auto fail = [&](int32_t code) { d.status = code; d.nstreams = 0; d.nblocks = 0; ch[c] = d; };
  if (ss < kHdrMin) return fail(E_READ);
  d.version = s[0];
  d.flags = s[2];
  d.typesize = s[3];
  d.nbytes = rd32(s + 4);
  int32_t bs = rd32(s + 8);
  const int32_t cb = rd32(s + 12);
  if (cb < kHdrMin || bs <= 0 || bs > kMaxBlocksize || d.typesize == 0) return fail(E_HEADER);
  const bool ext = (d.flags & kFlagShuffle) && (d.flags & kFlagBitshuffle);
  uint8_t flags2 = 0, bflags = 0;
  if (ext) {
    if (cb < kHdrExt) return fail(E_HEADER);
    if (ss < kHdrExt) return fail(E_READ);
    for (int i = 0; i < 6; i++) { d.filters[i] = s[16 + i]; d.filters_meta[i] = s[24 + i]; }
    d.codec = s[22];
    flags2 = s[30];
    bflags = s[31];
    d.special = (bflags >> 4) & 7;
    if ((flags2 & kFlag2VL) && d.special != 0) return fail(E_HEADER);
    if (d.special == kSpecialValue) {
      const int32_t vts = cb - kHdrExt;
      if (vts <= 0 || vts > kMaxBlocksize || vts > d.nbytes || d.nbytes % vts != 0) return fail(E_HEADER);
    } else if (d.special != 0 && d.special != kSpecialZero && d.nbytes % d.typesize != 0) {
      return fail(E_HEADER);
    }
    if (d.version == 3) { d.filters[5] = 0; d.filters_meta[5] = 0; }
    d.overhead = kHdrExt;
  } else {
    // flags_to_filters (blosc/blosc2.c:704-735)
    if (d.flags & kFlagShuffle) d.filters[5] = kShuffle;
    if (d.flags & kFlagBitshuffle) d.filters[5] = kBitshuffle;
    if (d.flags & kFlagDelta) d.filters[4] = kDelta;
    d.overhead = kHdrMin;
  }
  if (d.version > 6 && (flags2 & ~kFlag2VL)) return fail(E_VERSION);
  const bool vl = flags2 & kFlag2VL;
  const bool memcpyed = d.flags & kFlagMemcpy;
  if (vl && memcpyed) return fail(E_HEADER);
  if (!vl && d.nbytes > 0 && bs > d.nbytes) bs = d.nbytes;
  if (d.nbytes > dstsize[c]) return fail(E_WRITE);
  // blosc2_calculate_blocks (854-860); VL chunks carry their block count in the blocksize field
  int32_t nblocks = vl ? bs : d.nbytes / bs;
  d.leftover = vl ? 0 : d.nbytes % bs;
  if (d.leftover > 0) nblocks++;
  d.blocksize = bs;
  const bool lazy = ext && (bflags & 0x08);
  if (!lazy && cb > ss) return fail(E_HEADER);
  if (d.special > kSpecialUninit) return fail(E_DATA);
  if (memcpyed && cb != d.nbytes + d.overhead) return fail(E_DATA);
  d.status = max(d.nbytes, 0);
  if (d.nbytes == 0 && cb == d.overhead && !d.special) return fail(0);
  int64_t bstarts_end = d.overhead;
  if (!d.special && !memcpyed) {
    bstarts_end += 4 * (int64_t)nblocks;
    if (nblocks < 0 || bstarts_end > 0x7fffffff) return fail(E_HEADER);
  }
  if (ss < bstarts_end) return fail(E_READ);
  if (vl && lazy && !d.special && !memcpyed && (int64_t)ss < bstarts_end + 12 + 4 * (int64_t)nblocks)
    return fail(E_READ);
  if ((bflags & kUseDict) && !lazy && !(mode & 4)) {
    // the dictionary section after the bstarts: [int32 size | bytes] (2790-2825); LZ4 streams
    // may match into it (LZ4_decompress_safe_usingDict, 504-508), BloscLZ ignores it
    const int64_t rem = ss - bstarts_end;
    if (rem < 4) return fail(E_READ);
    const int32_t dsz = rd32(s + bstarts_end);
    if (dsz <= 0 || dsz > 32 * 1024) return fail(E_DICT);
    if (rem - 4 < dsz) return fail(E_READ);
    d.dict_off = (int32_t)bstarts_end + 4;
    d.dict_size = dsz;
  }
  if (vl && !d.special && !memcpyed) return fail(E_VERSION);   // VL-block chunks: not on the device path
  d.dont_split = (d.flags >> 4) & 1;
  d.delta_self = (mode >> 1) & 1;
  if (nblocks <= 0) return fail(d.status = 0);   // the block walk has nothing to do
  if (lazy && !d.special) return fail(E_PARAM);   // lazy chunks need their frame (blosc_d 1757-1766)
  if (memcpyed || d.special) {
    // blosc_d's memcpyed path (1865-1935): set_nans / set_values need whole items in every block
    const int32_t ts = d.special == kSpecialValue ? cb - kHdrExt : d.typesize;
    const bool full_blocks = nblocks - (d.leftover ? 1 : 0) > 0;
    if ((d.special == kSpecialNan || d.special == kSpecialValue) &&
        ((full_blocks && bs % ts) || (d.leftover && d.leftover % ts)))
      return fail(E_DATA);
    if (d.special == kSpecialNan && ts != 4 && ts != 8) return fail(E_DATA);
    d.nblocks = 0;   // handled by k_dspecial, not by the block table
    d.nstreams = 0;
    ch[c] = d;
    return;
  }
  d.nblocks = nblocks;
  const int32_t spb = d.dont_split ? 1 : d.typesize;
  d.nstreams = (d.nblocks - (d.leftover ? 1 : 0)) * spb + (d.leftover ? 1 : 0);
  if (mode & 1) {   // the caller applies the filters itself (host-driven pipelines)
    d.nfilters_bwd = 0;
    ch[c] = d;
    return;
  }
  // backward pipeline (pipeline_backward, 1473-1609): active filters (not NOFILTER / TRUNC_PREC)
  // from slot 5 down; an unknown id <= 31 fails the block with -1 after the pass, a filter id > 31
  // other than the device plugins with FILTER_PIPELINE (user filters take the host path)
  int k = 0, K = 0;
  for (int i = 5; i >= 0; i--) if (!bwd_noop(d.filters[i])) K++;
  for (int i = 5; i >= 0; i--) {
    const uint8_t f = d.filters[i];
    if (bwd_noop(f)) continue;
    if (f > 31 && f != kBytedelta) d.ferr = (int8_t)E_FILTER;
    else if (f > kTruncPrec && f <= 31 && d.ferr == 0) d.ferr = (int8_t)E_FAILURE;
    d.has_delta |= f == kDelta;
    d.fsrc[i] = (k % 2 == 0) ? 0 : 1;
    d.fdst[i] = (k == K - 1) ? 2 : ((k % 2 == 0) ? 1 : 0);
    k++;
  }
  d.nfilters_bwd = (uint8_t)K;
  // a lone 4-byte SHUFFLE (the T pipeline) is undone inside the decode launch by the wave that
  // completes each block (k_decode finish_block); k_dfilter skips these chunks
  if (K == 1 && d.ferr == 0) {
    int i = 5;
    while (bwd_noop(d.filters[i])) i--;
    const int32_t ts = d.filters_meta[i] ? d.filters_meta[i] : d.typesize;
    d.fuse_unshuffle = d.filters[i] == kShuffle && ts == 4 && (mode & 8) == 0;
    // a block's streams are its four planes (or one stream holds the whole shuffled image): the
    // unshuffle reads raw streams where they lie in the chunk and synthesises run streams, so
    // only LZ planes are staged
    d.unshuf_direct = d.fuse_unshuffle && (d.dont_split || (d.typesize == 4 && bs % 4 == 0));
  }
  // (DELTA, SHUFFLE) at typesize 2 / 4 / 8 over whole quads (the C4 pipeline): undone inside the
  // decode launch as well -- block 0's completing wave un-shuffles and XOR-scans it, every other
  // block once block 0 is final (finish_block); not with block masks (a masked block 0 never
  // completes) nor for the self-referencing getitem semantics
  if (K == 2 && d.ferr == 0 && (mode & (8 | 16)) == 0 && !d.delta_self && d.filters[5] == kShuffle &&
      d.filters[4] == kDelta) {
    const int32_t ts = d.typesize;
    d.fuse_ds = (d.filters_meta[5] == 0 || d.filters_meta[5] == ts) && (ts == 2 || ts == 4 || ts == 8) &&
                d.blocksize % (4 * ts) == 0 && d.leftover % (4 * ts) == 0;
  }
  // (DELTA, SHUFFLE) undone by k_dfilter: a stream that is a run is never
  // staged -- k_dfilter reads its plane as the run byte straight from the csize word, so at C4's
  // ratio (~800, almost every stream a run) the decode writes the output once instead of staging
  // the whole image and reading it back
  if (K == 2 && d.ferr == 0 && !d.fuse_ds && d.filters[5] == kShuffle && d.filters[4] == kDelta) {
    const int32_t ts = d.typesize;
    d.ds_runs = (d.filters_meta[5] == 0 || d.filters_meta[5] == ts) && (ts == 2 || ts == 4 || ts == 8);
  }
  ch[c] = d;
}

struct DTotals {
  int64_t stage_bytes;
  int32_t nblocks, nstreams;
  int32_t any_delta, max_filters;
  int32_t slot_mask;   // filter slots with a backward filter in any chunk (bit i = slot i)
  int32_t any_special; // some chunk is memcpyed / special (k_dspecial has work)
  int32_t overflow;    // the batch exceeds the table capacities of the sync-free path
  int32_t any_ds;      // some chunk is ds_runs (k_dfilter_ds has work)
};

// Single-workgroup exclusive scans (block_base, stream_base, stage_off) + totals.  With
// capacities (cap_blocks >= 0, the sync-free path) a batch whose tables would not fit fails every
// chunk with E_MEMORY and leaves nothing for the later kernels to do.
__global__ __launch_bounds__(1024) void k_dscan(DChunk* __restrict__ ch, int32_t n, DTotals* __restrict__ tot,
                                                int64_t cap_blocks, int64_t cap_streams, int64_t cap_stage,
                                                uint8_t* const* __restrict__ dsts) {
  __shared__ int64_t sb[1024];
  __shared__ int32_t sbk[1024], sst[1024], sdl[1024], smf[1024];
  __shared__ int32_t s_over;
  const int32_t per = (n + blockDim.x - 1) / blockDim.x;
  const int32_t lo = min(n, (int32_t)threadIdx.x * per), hi = min(n, lo + per);
  int64_t a = 0;
  int32_t bk = 0, st = 0, dl = 0, mf = 0;
  for (int32_t i = lo; i < hi; i++) {
    if (ch[i].status < 0) continue;
    a += ch[i].nstreams ? ch[i].nbytes : 0;
    bk += ch[i].nblocks;
    st += ch[i].nstreams;
    dl |= (ch[i].has_delta && !ch[i].fuse_ds) ? 0x100 : 0;
    dl |= (ch[i].nstreams == 0 && ch[i].nbytes != 0) ? 0x200 : 0;   // k_dspecial's chunks
    dl |= ch[i].nstreams && (ch[i].nbytes & 15) ? 0x400 : 0;        // a stage offset not 16-aligned follows
    dl |= ch[i].ds_runs ? 0x800 : 0;
    // a ds_runs chunk whose every block takes the one-pass form leaves k_dfilter nothing to do
    // (decided for sure once every stage offset is 16-aligned: bit 0x400 clear batch-wide)
    const int32_t ts = ch[i].typesize;
    const bool all_fast = ch[i].ds_runs && ch[i].blocksize % (4 * ts) == 0 && ch[i].leftover % (4 * ts) == 0 &&
                          (reinterpret_cast<uintptr_t>(dsts[i]) & 15) == 0 && ch[i].blocksize % 16 == 0;
    for (int f = 0; f < 6; f++)
      if (!bwd_noop(ch[i].filters[f]) && !ch[i].fuse_unshuffle && !ch[i].fuse_ds)
        dl |= all_fast ? (1 << (12 + f)) : (1 << f);
    mf = max(mf, (int32_t)ch[i].nfilters_bwd);
  }
  sb[threadIdx.x] = a; sbk[threadIdx.x] = bk; sst[threadIdx.x] = st; sdl[threadIdx.x] = dl; smf[threadIdx.x] = mf;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t ra = 0, rb = 0, rs = 0;
    int32_t rd = 0, rm = 0;
    for (int t = 0; t < (int)blockDim.x; t++) {
      int64_t va = sb[t]; int32_t vb = sbk[t], vs = sst[t];
      sb[t] = ra; sbk[t] = (int32_t)rb; sst[t] = (int32_t)rs;
      ra += va; rb += vb; rs += vs; rd |= sdl[t]; rm = max(rm, smf[t]);
    }
    const bool over = cap_blocks >= 0 && (rb > cap_blocks || rs > cap_streams || ra > cap_stage);
    s_over = over;
    tot->overflow = over;
    tot->stage_bytes = over ? 0 : ra;
    tot->nblocks = over ? 0 : (int32_t)rb;
    tot->nstreams = over ? 0 : (int32_t)rs;
    const int32_t slots = (rd & 0x3f) | (((rd >> 10) & 1) ? (rd >> 12) & 0x3f : 0);
    tot->any_delta = (rd >> 8) & 1; tot->slot_mask = over ? 0 : slots; tot->max_filters = rm;
    tot->any_special = over ? 0 : (rd >> 9) & 1;
    tot->any_ds = over ? 0 : (rd >> 11) & 1;
  }
  __syncthreads();
  const bool over = s_over;
  int64_t ra = sb[threadIdx.x];
  int32_t rb = sbk[threadIdx.x], rs = sst[threadIdx.x];
  for (int32_t i = lo; i < hi; i++) {
    if (over) {
      if (ch[i].status >= 0) ch[i].status = E_MEMORY;
      ch[i].nblocks = 0;
      ch[i].nstreams = 0;
      continue;
    }
    ch[i].stage_off = ra;
    ch[i].block_base = rb;
    ch[i].stream_base = rs;
    if (ch[i].status < 0) continue;
    ra += ch[i].nstreams ? ch[i].nbytes : 0;
    rb += ch[i].nblocks;
    rs += ch[i].nstreams;
  }
}

struct DBlock {
  int32_t chunk, block;
};

__device__ int32_t find_chunk(const DChunk* ch, int32_t n, int32_t idx) {
  int32_t lo = 0, hi = n - 1;   // last chunk with block_base <= idx and nblocks > 0
  while (lo < hi) {
    const int32_t mid = (lo + hi + 1) >> 1;
    if (ch[mid].block_base <= idx) lo = mid; else hi = mid - 1;
  }
  while (lo > 0 && (ch[lo].nblocks == 0 || ch[lo].status < 0 || ch[lo].block_base > idx)) lo--;
  return lo;
}

__device__ __forceinline__ void rec_err(DChunk* ch, int32_t c, int32_t block, int32_t step, int32_t code) {
  atomicMin(reinterpret_cast<unsigned long long*>(&ch[c].errkey), (unsigned long long)err_key(block, step, code));
}

// Pull order of the decoder: LZ / LZ4 streams (thousands of tokens each; on T one per block, ~90 %
// of the decode wave-time) from the front, raw copies and runs (a 64 KiB memcpy / memset) from the
// back, so the long streams start first and the short ones fill the end of the launch.

// One block of the walk (blosc_d, blosc/blosc2.c:1734-2016): a masked block is skipped before any
// check; then the bstart (1937-1940), the stream count (1982-1986) and each stream's size words
// (2002-2015), every failure keyed by its position.
__device__ void dplan_block(const uint8_t* const* __restrict__ srcs, const int32_t* __restrict__ srcsize,
                            DChunk* __restrict__ ch, int32_t n, DBlock* __restrict__ blocks,
                            DStream* __restrict__ streams, int32_t idx, int32_t* __restrict__ order,
                            int32_t* __restrict__ octr, int32_t nstreams, const uint8_t* __restrict__ maskout,
                            int32_t mask_stride, int32_t* __restrict__ bcnt, int ord_mode) {
  const int32_t c = find_chunk(ch, n, idx);
  const DChunk d = ch[c];
  const int32_t b = idx - d.block_base;
  blocks[idx].chunk = c;
  blocks[idx].block = b;
  if (bcnt) bcnt[idx] = 0;
  const uint8_t* s = srcs[c];
  const int32_t ss = srcsize[c];
  const bool lo = (b == d.nblocks - 1) && d.leftover;
  const int32_t bsize = lo ? d.leftover : d.blocksize;
  const int32_t ns = (!d.dont_split && !lo) ? d.typesize : 1;
  const int32_t neblock = bsize / ns;
  const int32_t sbase = d.stream_base + b * (d.dont_split ? 1 : d.typesize);
  const bool masked = maskout && maskout[(int64_t)c * mask_stride + b];
  int32_t pos = rd32(s + d.overhead + 4 * b);
  int32_t err = 0;
  if (masked) err = 1;   // no stream is planned and nothing is recorded
  else if (pos <= 0 || pos >= ss) err = E_DATA;
  else if (neblock == 0) err = E_WRITE;
  if (err < 0) rec_err(ch, c, b, 0, err);
  else if (!masked && d.ferr) rec_err(ch, c, b, kStepFilters, d.ferr);
  for (int32_t j = 0; j < ns; j++) {
    DStream st;
    st.chunk = c;
    st.neblock = neblock;
    st.dst_off = b * d.blocksize + j * neblock;
    st.csize = 0;
    st.src = 0;
    if (!err) {
      if (ss - pos < 4) {
        err = E_READ;
      } else {
        const int32_t cs = rd32(s + pos);
        pos += 4;
        int32_t payload = cs > 0 ? cs : (cs < 0 ? 1 : 0);
        if (ss - pos < payload) err = E_READ;
        st.csize = cs;
        st.src = pos;
        pos += payload;
      }
      if (err) rec_err(ch, c, b, 1 + j, err);
    }
    if (err) st.neblock = -1;
    streams[sbase + j] = st;
    // Pull order.  Default (1): stream order, so every block's raw copies and LZ decodes are pulled
    // together and the bandwidth-bound copies overlap the latency-bound LZ streams all through the
    // launch (T fast decode 4.75 -> 4.14 ms, exact 6.72 -> 6.22; C1 175.7 -> 162.5 GB/s).
    // B2H_DEC_ORDER=0: by class -- LZ streams first, except in chunks whose blocks are unshuffled by
    // the wave that completes them, where raw / run streams go first.
    const bool heavy = st.neblock > 0 && st.csize > 0 && st.csize != st.neblock;
    const int32_t slot = ord_mode == 1 ? sbase + j
                         : (heavy != (bool)d.fuse_unshuffle) ? atomicAdd(&octr[0], 1) : nstreams - 1 - atomicAdd(&octr[1], 1);
    order[slot] = sbase + j;
  }
}

__global__ void k_dplan_blocks(const uint8_t* const* __restrict__ srcs, const int32_t* __restrict__ srcsize,
                               DChunk* __restrict__ ch, int32_t n, DBlock* __restrict__ blocks,
                               DStream* __restrict__ streams, const DTotals* __restrict__ tot,
                               int32_t* __restrict__ order, int32_t* __restrict__ octr,
                               const uint8_t* __restrict__ maskout, int32_t mask_stride, int32_t* __restrict__ bcnt,
                               int ord_mode) {
  const int32_t nb = tot->nblocks, ns = tot->nstreams;
  for (int32_t idx = blockIdx.x * blockDim.x + threadIdx.x; idx < nb; idx += gridDim.x * blockDim.x)
    dplan_block(srcs, srcsize, ch, n, blocks, streams, idx, order, octr, ns, maskout, mask_stride, bcnt, ord_mode);
}

// Decoder: one wave per stream, persistent (as many single-wave workgroups as the LDS ring
// allows), streams pulled from a device counter -- stream cost ranges from a 64 KiB memset to
// thousands of LZ tokens, and a blockIdx-based mapping parks the expensive byte planes on a
// fraction of the chip (workgroups are dealt to XCDs / shader engines by index).
// LDS output ring per wave: 2^RLOG bytes.  The ring is the decoder's only LDS, so it sets the
// waves per CU (32 KiB: 5, 16 KiB: 10, 8 KiB: 20 = the 96-VGPR limit).  B2H_DEC_RING = 12..15
// picks it; default 13 (T decode: 15 -> 10.2 ms, 14 -> 6.3 ms, 13 -> 5.6 ms: the token loop is
// latency-bound, and more resident waves beat keeping older match sources in LDS).

// Returns whether the stream was decoded (false: skipped -- failed chunk, unplanned or masked).
template <int RLOG>
__device__ __forceinline__ bool decode_stream(const uint8_t* const* __restrict__ srcs, uint8_t* const* __restrict__ dsts,
                                              DChunk* __restrict__ ch, const DStream& st, uint8_t* __restrict__ stage,
                                              const uint8_t* __restrict__ maskout, int32_t mask_stride,
                                              B2H_LDS uint8_t* ring, int32_t* kind_out) {
  const int lane = lane_id();
  const int32_t c = st.chunk;
  const DChunk d = ch[c];
  if (d.status < 0 || st.neblock < 0) return false;
  if (maskout && maskout[(int64_t)c * mask_stride + st.dst_off / d.blocksize]) return false;
  gin_t in = (gin_t)(srcs[c] + st.src);
  gout_t out = (gout_t)((d.nfilters_bwd ? stage + d.stage_off : dsts[c]) + st.dst_off);
  const int32_t nb = st.neblock;
  // the stream's place in the serial walk, for the error key
  const int32_t blk = st.dst_off / d.blocksize;
  const int32_t step = 1 + (st.dst_off - blk * d.blocksize) / nb;
  // ds_runs: k_dfilter synthesises run planes; unshuf_direct: finish_block reads raw planes in
  // place and synthesises run planes -- neither is staged
  const bool nostage = d.ds_runs || d.unshuf_direct;
  if (st.csize == 0) {
    if (!nostage) wave_fill<true>(out, 0, nb);
  } else if (st.csize < 0) {
    const uint8_t token = in[0];
    if (!(token & 1) || st.csize < -255) {
      if (lane == 0) rec_err(ch, c, blk, step, E_RUNLEN);
    } else {
      if (!nostage) wave_fill<true>(out, (uint8_t)(-st.csize), nb);
      *kind_out = 1;
    }
  } else if (st.csize == nb) {
    if (!d.unshuf_direct) wave_copy<true>(out, in, nb);
    *kind_out = 2;
  } else if ((d.flags >> 5) == 1) {   // LZ4 (blosc/blosc2.c:2062-2067)
    const int32_t got = wave_lz4_decode_ring<RLOG>(in, st.csize, out, nb, ring, (gin_t)(srcs[c] + d.dict_off), d.dict_size);
    if (got != nb && lane == 0) rec_err(ch, c, blk, step, E_DATA);
    *kind_out = 4;
  } else if ((d.flags >> 5) != 0) {
    if (lane == 0) rec_err(ch, c, blk, step, E_CODEC);
  } else {
    const int32_t got = wave_lz_decode_par<RLOG>(in, st.csize, out, nb, ring);
    if (got != nb && lane == 0) rec_err(ch, c, blk, step, E_DATA);
    *kind_out = 3;
  }
  return true;
}

// SHUFFLE-only chunks (DChunk::fuse_unshuffle): the wave that decodes the last of a block's streams
// unshuffles the block stage -> dst inside this launch, so the un-filter overlaps the latency-bound
// LZ streams instead of running as its own bandwidth pass (k_dfilter).  Hand-off, after
// MI355X_MICROARCH.md § inter-workgroup visibility R1: the decoders store their output write-
// through (sc1) and drain it (vmcnt(0)) before lane 0 adds to the block's counter (agent scope,
// relaxed); the wave whose add completes the count acquires (agent) before its plain loads.
// One wave unshuffles a typesize-4 block on its own, so it must keep many bytes in flight: rows
// of 1024 elements (1 KiB per plane) arrive by 16-byte lane-linear loads, the next row's loads
// issued before this row is transposed through the idle LDS ring (4 KiB) and leaves by 16-byte
// stores, each instruction 1 KiB contiguous.  The n % 256 remainder and the bsize % 4 tail
// take the per-quad and byte paths.
#ifndef B2H_UNSHUF_DEPTH
#define B2H_UNSHUF_DEPTH 2
#endif
constexpr int kUnshufDepth = B2H_UNSHUF_DEPTH;
// Where each of a block's four planes comes from (DChunk::unshuf_direct): the decoder's staged
// image (16-byte aligned), a raw stream in place in the chunk (any alignment: aligned dwords and a
// funnel shift, never a dword past the plane's last byte), or a run (bit j of runm, byte j of
// runb; never read).  `tail`: the bsize % 4 bytes after the planes (an unsplit image only).
struct PlaneSrc4 {
  const uint8_t* p[4];
  const uint8_t* tail;
  uint32_t runm, runb;
};
__device__ __forceinline__ uint32_t plane_splat(const PlaneSrc4& ps, int j) {
  return 0x01010101u * ((ps.runb >> (8 * j)) & 0xffu);
}
// 16 bytes of plane j at byte offset `off`
__device__ __forceinline__ u32x4 plane_ld16(const PlaneSrc4& ps, int j, int64_t off) {
  if ((ps.runm >> j) & 1u) {
    const uint32_t w = plane_splat(ps, j);
    return u32x4{w, w, w, w};
  }
  const uint8_t* s = ps.p[j] + off;
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(ps.p[j]) & 3);   // wave-uniform
  const uint32_t* q = reinterpret_cast<const uint32_t*>(s - sh);
  if (sh == 0) {
    typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
    const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(q);
    return u32x4{v.x, v.y, v.z, v.w};
  }
  const uint32_t a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  return u32x4{funnel(a, b, sh), funnel(b, c, sh), funnel(c, d, sh), funnel(d, e, sh)};
}
// the dword of plane j at element quad qd (bytes 4qd .. 4qd + 3)
__device__ __forceinline__ uint32_t plane_ld4(const PlaneSrc4& ps, int j, int32_t qd) {
  if ((ps.runm >> j) & 1u) return plane_splat(ps, j);
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(ps.p[j]) & 3);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(ps.p[j] - sh) + qd;
  return sh ? funnel(q[0], q[1], sh) : q[0];
}
__device__ __forceinline__ uint8_t plane_ld1(const PlaneSrc4& ps, int j, int32_t i) {
  return ((ps.runm >> j) & 1u) ? (uint8_t)(ps.runb >> (8 * j)) : ps.p[j][i];
}

// The block's typesize-4 unshuffle by one wave, planes -> dst.
__device__ __forceinline__ void unshuffle4_wave_lds(const PlaneSrc4& ps, uint8_t* __restrict__ dst, int32_t bsize,
                                                    B2H_LDS uint8_t* lds) {
  const int lane = lane_id();
  const int32_t n = bsize / 4;
  if (!aligned16(dst)) {
    for (int32_t i = lane; i < n * 4; i += 64) dst[i] = plane_ld1(ps, i & 3, i >> 2);
  } else {
    const int32_t rows = (n % 4 == 0) ? n / 1024 : 0;   // 1024 elements = 1 KiB per plane
    if (rows > 0) {
      // kUnshufDepth rows (4 KiB each) in flight: one wave is latency-bound on these loads
      u32x4 v[kUnshufDepth][4];
#pragma unroll
      for (int d = 0; d < kUnshufDepth; d++) {
        if (d < rows) {
#pragma unroll
          for (int p = 0; p < 4; p++) v[d][p] = plane_ld16(ps, p, d * 1024 + 16 * lane);
        }
      }
#pragma unroll 1
      for (int32_t r = 0; r < rows; r++) {
        // this row into LDS, then the loads kUnshufDepth rows ahead in flight while this one is transposed
#pragma unroll
        for (int p = 0; p < 4; p++) *reinterpret_cast<B2H_LDS u32x4*>(lds + p * 1024 + 16 * lane) = v[0][p];
#pragma unroll
        for (int d = 0; d + 1 < kUnshufDepth; d++) {
#pragma unroll
          for (int p = 0; p < 4; p++) v[d][p] = v[d + 1][p];
        }
        if (r + kUnshufDepth < rows) {
#pragma unroll
          for (int p = 0; p < 4; p++) v[kUnshufDepth - 1][p] = plane_ld16(ps, p, (int64_t)(r + kUnshufDepth) * 1024 + 16 * lane);
        }
        uint8_t* row = dst + (int64_t)r * 4096;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int32_t q = k * 64 + lane;
          uint32_t w[4];
#pragma unroll
          for (int p = 0; p < 4; p++) w[p] = *reinterpret_cast<const B2H_LDS uint32_t*>(lds + p * 1024 + 4 * q);
          store_quad<4>(row, q, w);
        }
      }
    }
    for (int32_t q = rows * 256 + lane; q < n / 4; q += 64) {   // quads after the whole rows
      uint32_t w[4];
#pragma unroll
      for (int p = 0; p < 4; p++) w[p] = plane_ld4(ps, p, q);
      store_quad<4>(dst, q, w);
    }
    for (int32_t i = (n / 4) * 16 + lane; i < n * 4; i += 64) dst[i] = plane_ld1(ps, i & 3, i >> 2);
  }
  for (int32_t i = n * 4 + lane; i < bsize; i += 64)
    dst[i] = ps.tail ? ps.tail[i - n * 4] : (uint8_t)ps.runb;
}

// One (DELTA, SHUFFLE) block by one wave, stage -> dst: block 0 un-shuffled and XOR-scanned over
// its elements, the others un-shuffled and XORed with the final block 0 (the bytes of k_dfilter's
// fused slot, b2h_filters.h unshuffle_scan_fast / unshuffle_xor_fast).  One wave moves a whole
// block, so it keeps rows in flight as unshuffle4_wave_lds does: a row is 1024 elements, every
// plane's 1 KiB of it loaded by one 16-byte lane-linear instruction, the next row's loads issued
// before this row is transposed through the decoder's idle LDS ring (TS KiB); each lane then
// owns 16 consecutive elements (16 * TS contiguous output bytes).  Block 0's row scan: lane
// totals scanned over the wave, then each lane's elements with its exclusive prefix.  The quads
// after the whole rows (and images whose planes are not 16-byte aligned) take the quad loop.
template <int TS>
__device__ __forceinline__ int32_t ds_wave_rows(const uint8_t* __restrict__ src, const uint8_t* __restrict__ ref,
                                                uint8_t* __restrict__ dst, int32_t n, B2H_LDS uint8_t* lds,
                                                uint64_t& carry) {
  const int lane = lane_id();
  const int32_t rows = n / 1024;
  if (rows == 0) return 0;
  u32x4 v[TS], nx[TS];
#pragma unroll
  for (int p = 0; p < TS; p++) v[p] = *reinterpret_cast<const u32x4*>(src + (int64_t)p * n + 16 * lane);
#pragma unroll 1
  for (int32_t r = 0; r < rows; r++) {
#pragma unroll
    for (int p = 0; p < TS; p++) *reinterpret_cast<B2H_LDS u32x4*>(lds + p * 1024 + 16 * lane) = v[p];
    if (r + 1 < rows) {
#pragma unroll
      for (int p = 0; p < TS; p++)
        nx[p] = *reinterpret_cast<const u32x4*>(src + (int64_t)p * n + (int64_t)(r + 1) * 1024 + 16 * lane);
    }
    asm volatile("" ::: "memory");   // the row's LDS writes before any lane reads it back
    const int64_t e0 = (int64_t)r * 1024 + 16 * lane;   // this lane's first element
    // element quad j of the lane: TS plane dwords -> TS element-order words
    auto quad = [&](int j, uint32_t (&w)[TS]) {
      uint32_t pl[TS];
#pragma unroll
      for (int p = 0; p < TS; p++) pl[p] = *reinterpret_cast<const B2H_LDS uint32_t*>(lds + p * 1024 + 16 * lane + 4 * j);
      planes_to_words<TS>(pl, w);
    };
    if (ref) {
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t w[TS], rw[TS];
        quad(j, w);
        load_words<TS>(ref, (int32_t)(e0 / 4) + j, rw);
#pragma unroll
        for (int k = 0; k < TS; k++) w[k] ^= rw[k];
        store_words<TS>(dst, (int32_t)(e0 / 4) + j, w);
      }
    } else {
      constexpr int K = TS / 2;   // u64 words per element quad
      uint64_t tot = 0;           // XOR of the lane's 16 elements (replicated per element width)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t w[TS];
        quad(j, w);
#pragma unroll
        for (int k = 0; k < K; k++) tot ^= (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
      }
      tot = xor_last_word64(xor_prefix64(tot, TS), TS);   // the XOR of every element, replicated
      uint64_t sc = tot;
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint64_t y = shfl_up64(sc, dd);
        if (lane >= dd) sc ^= y;
      }
      uint64_t run = carry ^ sc ^ tot;   // every element before this lane's first
#pragma unroll
      for (int j = 0; j < 4; j++) {
        uint32_t w[TS];
        quad(j, w);
        uint64_t x[K];
#pragma unroll
        for (int k = 0; k < K; k++) x[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
        x[0] = xor_prefix64(x[0], TS);
#pragma unroll
        for (int k = 1; k < K; k++) x[k] = xor_prefix64(x[k], TS) ^ xor_last_word64(x[k - 1], TS);
#pragma unroll
        for (int k = 0; k < K; k++) {
          const uint64_t o = x[k] ^ run;
          w[2 * k] = (uint32_t)o;
          w[2 * k + 1] = (uint32_t)(o >> 32);
        }
        run ^= xor_last_word64(x[K - 1], TS);
        store_words<TS>(dst, (int32_t)(e0 / 4) + j, w);
      }
      carry ^= (uint64_t)__shfl((long long)sc, 63);
    }
    asm volatile("" ::: "memory");   // every lane's LDS reads before the next row's writes
#pragma unroll
    for (int p = 0; p < TS; p++) v[p] = nx[p];
  }
  return rows * 256;   // quads done
}
template <int TS>
__device__ __forceinline__ void ds_wave_rest(const uint8_t* __restrict__ src, const uint8_t* __restrict__ ref,
                                             uint8_t* __restrict__ dst, int32_t n, int32_t q0) {
  const int32_t quads = n / 4;
  for (int32_t q = q0 + lane_id(); q < quads; q += 64) {
    uint32_t p[TS], r[TS], w[TS];
    load_planes<TS>(src, q, n, p);
    load_words<TS>(ref, q, r);
    planes_to_words<TS>(p, w);
#pragma unroll
    for (int k = 0; k < TS; k++) w[k] ^= r[k];
    store_words<TS>(dst, q, w);
  }
}
template <int TS>
__device__ __forceinline__ void ds_wave_first(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int32_t n,
                                              int32_t q0, uint64_t carry) {
  constexpr int K = TS / 2;   // u64 words per quad
  const int lane = lane_id();
  const int32_t quads = n / 4;
  for (int32_t base = q0; base < quads; base += 64) {
    const int32_t q = base + lane;
    uint32_t p[TS], w[TS];
    if (q < quads) {
      load_planes<TS>(src, q, n, p);
    } else {
#pragma unroll
      for (int k = 0; k < TS; k++) p[k] = 0u;
    }
    planes_to_words<TS>(p, w);
    uint64_t x[K];
#pragma unroll
    for (int k = 0; k < K; k++) x[k] = (uint64_t)w[2 * k] | ((uint64_t)w[2 * k + 1] << 32);
    // the quad's own inclusive scan, then the lanes' totals scanned over the wave
    x[0] = xor_prefix64(x[0], TS);
#pragma unroll
    for (int k = 1; k < K; k++) x[k] = xor_prefix64(x[k], TS) ^ xor_last_word64(x[k - 1], TS);
    const uint64_t t = xor_last_word64(x[K - 1], TS);
    uint64_t sc = t;
#pragma unroll
    for (int dd = 1; dd < 64; dd <<= 1) {
      const uint64_t y = shfl_up64(sc, dd);
      if (lane >= dd) sc ^= y;
    }
    const uint64_t ex = carry ^ sc ^ t;   // the elements before this quad
    if (q < quads) {
#pragma unroll
      for (int k = 0; k < K; k++) {
        const uint64_t o = x[k] ^ ex;
        w[2 * k] = (uint32_t)o;
        w[2 * k + 1] = (uint32_t)(o >> 32);
      }
      store_words<TS>(dst, q, w);
    }
    carry ^= (uint64_t)__shfl((long long)sc, 63);
  }
}
// The in-launch (DELTA, SHUFFLE) decode (park/claim protocol below) is a build option, off by
// default: measured slower than the separate k_dfilter pass, so default builds carry
// neither the protocol nor ds_finish_block in k_decode.  Build with -DB2H_DEC_FUSE_DS_BUILD=1 and
// run with B2H_DEC_FUSE_DS=1 to measure it.
#ifndef B2H_DEC_FUSE_DS_BUILD
#define B2H_DEC_FUSE_DS_BUILD 0
#endif
#if B2H_DEC_FUSE_DS_BUILD
// (templated on the decoder's ring size: one copy per k_decode instantiation, which then takes
// that kernel's register budget instead of its own)
template <int RLOG>
__device__ __noinline__ void ds_finish_block(const DChunk& d, int32_t c, int32_t blk, uint8_t* const* __restrict__ dsts,
                                             uint8_t* __restrict__ stage, B2H_LDS uint8_t* ring) {
  const bool lo = (blk == d.nblocks - 1) && d.leftover;
  const int32_t bsize = lo ? d.leftover : d.blocksize, ts = d.typesize, ne = bsize / ts;
  const int64_t off = (int64_t)blk * d.blocksize;
  const uint8_t* src = stage + d.stage_off + off;
  uint8_t* dst = dsts[c] + off;
  const uint8_t* ref = dsts[c];
  if (aligned16(src) && aligned16(dst) && aligned16(ref)) {
    // whole rows through the LDS ring when it holds TS KiB and every plane starts 16-byte aligned
    const bool rows = (1 << RLOG) >= ts * 1024 && ne % 16 == 0;
    const uint8_t* r = blk == 0 ? nullptr : ref;
    uint64_t carry = 0;
    int32_t q0 = 0;
    if (ts == 4) {
      if (rows) q0 = ds_wave_rows<4>(src, r, dst, ne, ring, carry);
      if (blk == 0) ds_wave_first<4>(src, dst, ne, q0, carry);
      else ds_wave_rest<4>(src, ref, dst, ne, q0);
    } else if (ts == 8) {
      if (rows) q0 = ds_wave_rows<8>(src, r, dst, ne, ring, carry);
      if (blk == 0) ds_wave_first<8>(src, dst, ne, q0, carry);
      else ds_wave_rest<8>(src, ref, dst, ne, q0);
    } else {
      if (rows) q0 = ds_wave_rows<2>(src, r, dst, ne, ring, carry);
      if (blk == 0) ds_wave_first<2>(src, dst, ne, q0, carry);
      else ds_wave_rest<2>(src, ref, dst, ne, q0);
    }
    return;
  }
  // unaligned images: the element loop (lane i gathers element base + i from the planes)
  const int lane = lane_id();
  uint64_t carry = 0;
  for (int32_t base = 0; base < ne; base += 64) {
    const int32_t i = base + lane;
    uint64_t v = 0;
    if (i < ne)
      for (int b = 0; b < ts; b++) v |= (uint64_t)src[(int64_t)b * ne + i] << (8 * b);
    if (blk == 0) {
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const uint64_t y = shfl_up64(v, dd);
        if (lane >= dd) v ^= y;
      }
      v ^= carry;
      carry = (uint64_t)__shfl((long long)v, 63);
    } else if (i < ne) {
      for (int b = 0; b < ts; b++) v ^= (uint64_t)ref[(int64_t)i * ts + b] << (8 * b);
    }
    if (i < ne)
      for (int b = 0; b < ts; b++) dst[(int64_t)i * ts + b] = (uint8_t)(v >> (8 * b));
  }
}
#endif

template <int RLOG>
__device__ __forceinline__ void finish_block(const DChunk* __restrict__ ch, const DStream* __restrict__ streams, int32_t s,
                                             const uint8_t* const* __restrict__ srcs,
                                             uint8_t* const* __restrict__ dsts, uint8_t* __restrict__ stage,
                                             int32_t* __restrict__ bcnt, B2H_LDS uint8_t* ring) {
  // re-read the plan words here: kept live across the decoder they cost it registers
  asm volatile("" ::: "memory");
  const DStream st = streams[s];
  const DChunk& d = ch[st.chunk];
#if B2H_DEC_FUSE_DS_BUILD
  const bool fuse_ds = __builtin_amdgcn_readfirstlane(d.fuse_ds) != 0;
#else
  constexpr bool fuse_ds = false;   // never planned: the host always sets mode bit 16
#endif
  if (!__builtin_amdgcn_readfirstlane(d.fuse_unshuffle) && !fuse_ds) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int32_t blk = st.dst_off / d.blocksize;
  const bool lo = (blk == d.nblocks - 1) && d.leftover;
  const int32_t ns = (!d.dont_split && !lo) ? d.typesize : 1;
  int32_t* cnt = bcnt + d.block_base;
  int32_t old = 0;
  if (lane_id() == 0) old = __hip_atomic_fetch_add(cnt + blk, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __builtin_amdgcn_readfirstlane(old);
  if (old != ns - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (!fuse_ds) {
    const int64_t off = (int64_t)blk * d.blocksize;
    const int32_t bsize = lo ? d.leftover : d.blocksize, n = bsize / 4;
    const uint8_t* img = stage + d.stage_off + off;
    PlaneSrc4 ps;
    ps.runm = 0;
    ps.runb = 0;
    for (int j = 0; j < 4; j++) ps.p[j] = img + (int64_t)j * n;
    ps.tail = img + 4 * (int64_t)n;
    if (__builtin_amdgcn_readfirstlane(d.unshuf_direct)) {
      // the block's streams: one per plane, or one holding the whole shuffled image
      const int32_t s0 = d.stream_base + blk * (d.dont_split ? 1 : d.typesize);
      const uint8_t* src = srcs[st.chunk];
      for (int j = 0; j < ns; j++) {
        const int32_t cs = __builtin_amdgcn_readfirstlane(streams[s0 + j].csize);
        const int32_t so = __builtin_amdgcn_readfirstlane(streams[s0 + j].src);
        const int32_t nb = __builtin_amdgcn_readfirstlane(streams[s0 + j].neblock);
        if (cs <= 0) {                          // a run (0: zeros; an invalid one failed the chunk)
          const uint32_t b = (uint8_t)(-cs);
          if (ns == 1) { ps.runm = 0xfu; ps.runb = b * 0x01010101u; ps.tail = nullptr; }
          else { ps.runm |= 1u << j; ps.runb |= b << (8 * j); }
        } else if (cs == nb) {                  // raw: in place
          if (ns == 1) {
            for (int k = 0; k < 4; k++) ps.p[k] = src + so + (int64_t)k * n;
            ps.tail = src + so + 4 * (int64_t)n;
          } else {
            ps.p[j] = src + so;
          }
        }
      }
    }
    unshuffle4_wave_lds(ps, dsts[st.chunk] + off, bsize, ring);
    return;
  }
#if B2H_DEC_FUSE_DS_BUILD
  // (DELTA, SHUFFLE): block 0 first; a block whose streams finish before block 0 is final parks,
  // and whichever of it and block 0's wave sees the other's mark takes it (exactly once: CLAIM)
  constexpr int32_t kDone = 1 << 30, kPark = 1 << 29, kClaim = 1 << 28;
  auto ld = [&](int32_t* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT));
  };
  auto orw = [&](int32_t* p, int32_t v) {
    int32_t o = 0;
    if (lane_id() == 0) o = __hip_atomic_fetch_or(p, v, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(o);
  };
  if (blk != 0) {
    if (!(ld(cnt) & kDone)) {
      orw(cnt + blk, kPark);
      if (!(ld(cnt) & kDone) || (orw(cnt + blk, kClaim) & kClaim)) return;   // block 0's wave takes it
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ds_finish_block<RLOG>(d, st.chunk, blk, dsts, stage, ring);
    return;
  }
  ds_finish_block<RLOG>(d, st.chunk, 0, dsts, stage, ring);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  orw(cnt, kDone);
  for (int32_t k = 1; k < d.nblocks; k++) {
    if (!(ld(cnt + k) & kPark) || (orw(cnt + k, kClaim) & kClaim)) continue;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    ds_finish_block<RLOG>(d, st.chunk, k, dsts, stage, ring);
  }
#endif
}

template <int RLOG>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(RLOG == 12 ? 8 : RLOG == 13 ? 5 : 1, 8))) void k_decode(const uint8_t* const* __restrict__ srcs, uint8_t* const* __restrict__ dsts,
                                               DChunk* __restrict__ ch, const DStream* __restrict__ streams,
                                               uint8_t* __restrict__ stage, const DTotals* __restrict__ tot,
                                               const uint8_t* __restrict__ maskout, int32_t mask_stride,
                                               int32_t* __restrict__ next, const int32_t* __restrict__ order,
                                               int32_t* __restrict__ bcnt, int64_t* __restrict__ dbg) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* ring = (B2H_LDS uint8_t*)smem;
  const int32_t nstreams_total = __builtin_amdgcn_readfirstlane(tot->nstreams);
  for (;;) {
    // branch-free grab (see k_encode), then the planner's pull order (LZ streams first)
    const int32_t i = __builtin_amdgcn_readfirstlane(atomicAdd(next, lane_id() == 0 ? 1 : 0));
    if (i >= nstreams_total) return;
    const int32_t s = __builtin_amdgcn_readfirstlane(order[i]);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    int32_t kind = 0;
    if (decode_stream<RLOG>(srcs, dsts, ch, streams[s], stage, maskout, mask_stride, ring, &kind))
      finish_block<RLOG>(ch, streams, s, srcs, dsts, stage, bcnt, ring);
    if (dbg && lane_id() == 0) {
      dbg[2 * s] = (int64_t)(__builtin_amdgcn_s_memtime() - t0);
      dbg[2 * s + 1] = kind;
    }
  }
}

// filters = (noop x4, DELTA, SHUFFLE) with the shuffle over the chunk's typesize in {2,4,8} and a
// block of whole quads: decoded by one fused pass (b2h_filters.h, unshuffle_scan/xor_fast).
__device__ __forceinline__ bool fused_delta_shuffle(const DChunk& d, int32_t bsize) {
  if (d.filters[5] != kShuffle || d.filters[4] != kDelta || d.fsrc[5] != 0 || d.fdst[4] != 2) return false;
  for (int i = 0; i < 4; i++) if (!bwd_noop(d.filters[i])) return false;
  const int32_t ts = d.typesize;
  if (d.filters_meta[5] != 0 && d.filters_meta[5] != ts) return false;
  if (ts != 2 && ts != 4 && ts != 8) return false;
  return bsize % (4 * ts) == 0;
}

// Backward filter for filter slot `slot` on one block; pass 0: all blocks, 1: block 0 only,
// 2: blocks >= 1.  Every early return is uniform over the workgroup.
// A (DELTA, SHUFFLE) block undone in one pass (unshuffle + un-delta, stage -> dst): whole quads,
// 16-byte aligned image and destination.  k_dfilter_ds and k_dfilter take the same decision.
__device__ __forceinline__ bool ds_fast_block(const DChunk& d, int32_t bsize, const uint8_t* img, const uint8_t* out,
                                              const uint8_t* dst0) {
  return fused_delta_shuffle(d, bsize) && aligned16(img) && aligned16(out) && aligned16(dst0);
}

// The run planes of block `bk` of a ds_runs chunk: bit j of the mask = plane j's stream is a run,
// byte j of *rb its byte (a block of one stream -- unsplit or the leftover -- that is a run has
// every plane of its byte).  Wave-uniform.
__device__ __forceinline__ uint32_t block_run_planes(const DChunk& d, const DStream* __restrict__ streams,
                                                     const DBlock& bk, uint64_t* rb) {
  const int32_t ts = d.typesize;
  const int32_t full = d.nblocks - (d.leftover ? 1 : 0);
  const bool split = !d.dont_split && bk.block < full;
  const int32_t spb = d.dont_split ? 1 : ts;
  const int32_t s0 = d.stream_base + (bk.block < full ? bk.block * spb : full * spb);
  uint32_t rm = 0;
  uint64_t b = 0;
  if (split) {
    for (int j = 0; j < ts; j++) {
      const int32_t cs = __builtin_amdgcn_readfirstlane(streams[s0 + j].csize);
      if (cs <= 0) {
        rm |= 1u << j;
        b |= (uint64_t)(uint8_t)(-cs) << (8 * j);
      }
    }
  } else {
    const int32_t cs = __builtin_amdgcn_readfirstlane(streams[s0].csize);
    if (cs <= 0) {
      rm = (1u << ts) - 1;
      b = 0x0101010101010101ull * (uint8_t)(-cs);
    }
  }
  *rb = b;
  return rm;
}

__device__ __forceinline__ void dfilter_block(DChunk* __restrict__ ch, const DBlock* __restrict__ blocks,
                                              const DStream* __restrict__ streams,
                                              uint8_t* const* __restrict__ dsts, uint8_t* __restrict__ stage,
                                              uint8_t* __restrict__ stage2, int slot, int pass, int32_t idx,
                                              const uint8_t* __restrict__ maskout, int32_t mask_stride) {
  const DBlock bk = blocks[idx];
  if (pass == 1 && bk.block != 0) return;
  if (pass == 2 && bk.block == 0) return;
  const DChunk d = ch[bk.chunk];
  if (d.status < 0 || d.fuse_unshuffle || d.fuse_ds) return;
  const uint8_t f = d.filters[slot];
  if (bwd_noop(f)) return;
  if (maskout && maskout[(int64_t)bk.chunk * mask_stride + bk.block]) return;
  const bool lo = (bk.block == d.nblocks - 1) && d.leftover;
  const int32_t bsize = lo ? d.leftover : d.blocksize;
  const int64_t off = (int64_t)bk.block * d.blocksize;
  uint8_t* bufs[3] = {stage + d.stage_off + off, stage2 + d.stage_off + off, dsts[bk.chunk] + off};
  // (DELTA, SHUFFLE) blocks in the one-pass form are k_dfilter_ds's (both slots)
  if (d.ds_runs && ds_fast_block(d, bsize, bufs[0], bufs[2], dsts[bk.chunk])) return;
  uint64_t rb = 0;
  const uint32_t rm = d.ds_runs ? block_run_planes(d, streams, bk, &rb) : 0u;
  if (rm && slot == 5) {   // any other form of the block: its run planes staged first, then as usual
    const int32_t ts = d.typesize;
    const int32_t pl = (d.dont_split || lo) ? bsize : bsize / ts;   // bytes per stream of the block
    const int32_t ns = (d.dont_split || lo) ? 1 : ts;
    for (int j = 0; j < ns; j++) {
      if (!((rm >> j) & 1)) continue;
      const uint8_t v = (uint8_t)(rb >> (8 * j));
      for (int32_t i = threadIdx.x; i < pl; i += blockDim.x) bufs[0][(int64_t)j * pl + i] = v;
    }
    __syncthreads();
  }
  const uint8_t* s = bufs[d.fsrc[slot]];
  uint8_t* o = bufs[d.fdst[slot]];
  const uint8_t meta = d.filters_meta[slot];
  switch (f) {
    case kShuffle: block_unshuffle(s, o, bsize, meta ? meta : d.typesize); break;
    case kBitshuffle: block_bitunshuffle(s, o, bsize, d.typesize, d.version); break;
    case kBytedelta: block_bytedelta_decode(s, o, bsize, meta ? meta : d.typesize); break;
    case kDelta:
      if (bk.block == 0 || d.delta_self) block_delta_decode_first(s, o, bsize, d.typesize);
      else block_delta_decode_rest(s, dsts[bk.chunk], o, bsize, d.typesize);
      break;
    default: break;
  }
}

// (DELTA, SHUFFLE) chunks' blocks in the one-pass form (DChunk::ds_runs + ds_fast_block): un-shuffle
// and un-delta stage -> dst, run planes synthesised from their csize words (never staged).  pass 1
// block 0 (an XOR scan), pass 2 the other blocks (XOR with the final block 0).  A kernel of its own:
// in the generic k_dfilter the bitunshuffle / bytedelta paths held it at 211 VGPRs (2 waves per
// SIMD), which left this bandwidth pass latency-bound.
// Block b >= 1 of a chunk of at most kDsFuseBlocks blocks whose output pass 1 writes together with
// block 0's (every plane a run: the block is a constant element XORed with block 0's output).
// Decided the same way by pass 1 (for block 0's workgroup) and pass 2 (which then skips it).
constexpr int32_t kDsFuseBlocks = 4;
__device__ __forceinline__ bool ds_later_fused(const DChunk& d, const DStream* __restrict__ streams, int32_t c, int32_t b,
                                               uint8_t* const* __restrict__ dsts, const uint8_t* __restrict__ stage,
                                               const uint8_t* __restrict__ maskout, int32_t mask_stride, uint64_t* rb) {
  if (d.delta_self || d.nblocks < 2 || d.nblocks > kDsFuseBlocks || b < 1 || b >= d.nblocks) return false;
  const int32_t ts = d.typesize;
  const bool lo0 = d.nblocks == 1 && d.leftover;
  const int32_t bs0 = lo0 ? d.leftover : d.blocksize;
  if (maskout && (maskout[(int64_t)c * mask_stride] || maskout[(int64_t)c * mask_stride + b])) return false;
  if (!ds_fast_block(d, bs0, stage + d.stage_off, dsts[c], dsts[c])) return false;
  const bool lo = b == d.nblocks - 1 && d.leftover;
  const int32_t bsize = lo ? d.leftover : d.blocksize;
  if (bsize != bs0) return false;   // the scan writes block 0's element count
  const int64_t off = (int64_t)b * d.blocksize;
  if (!ds_fast_block(d, bsize, stage + d.stage_off + off, dsts[c] + off, dsts[c])) return false;
  DBlock bk;
  bk.chunk = c;
  bk.block = b;
  return block_run_planes(d, streams, bk, rb) == (1u << ts) - 1u;
}

__global__ __launch_bounds__(kBlockThreads) void k_dfilter_ds(DChunk* __restrict__ ch, const DBlock* __restrict__ blocks,
                                                              const DStream* __restrict__ streams,
                                                              uint8_t* const* __restrict__ dsts, uint8_t* __restrict__ stage,
                                                              int pass, const DTotals* __restrict__ tot,
                                                              const uint8_t* __restrict__ maskout, int32_t mask_stride) {
  if (!tot->any_ds) return;
  const int32_t nb = tot->nblocks;
  for (int32_t idx = blockIdx.x; idx < nb; idx += gridDim.x) {
    const DBlock bk = blocks[idx];
    if (pass == 1 && bk.block != 0) continue;
    if (pass == 2 && bk.block == 0) continue;
    const DChunk d = ch[bk.chunk];
    if (d.status < 0 || !d.ds_runs) continue;
    if (maskout && maskout[(int64_t)bk.chunk * mask_stride + bk.block]) continue;
    const bool lo = (bk.block == d.nblocks - 1) && d.leftover;
    const int32_t bsize = lo ? d.leftover : d.blocksize;
    const int64_t off = (int64_t)bk.block * d.blocksize;
    const uint8_t* img = stage + d.stage_off + off;
    uint8_t* out = dsts[bk.chunk] + off;
    if (!ds_fast_block(d, bsize, img, out, dsts[bk.chunk])) continue;
    uint64_t rb = 0;
    const uint32_t rm = block_run_planes(d, streams, bk, &rb);
    const int32_t ne = bsize / d.typesize;
    if (bk.block == 0 || d.delta_self) {
      int nx = 0;
      uint8_t* xout[kDsFuseBlocks - 1];
      uint64_t xrb[kDsFuseBlocks - 1];
      if (bk.block == 0)
        for (int32_t b = 1; b < min(d.nblocks, kDsFuseBlocks); b++)
          if (ds_later_fused(d, streams, bk.chunk, b, dsts, stage, maskout, mask_stride, &xrb[nx]))
            xout[nx++] = dsts[bk.chunk] + (int64_t)b * d.blocksize;
      if (d.typesize == 4) unshuffle_scan_fast<4>(img, out, ne, rm, rb, nx, xout, xrb);
      else if (d.typesize == 8) unshuffle_scan_fast<8>(img, out, ne, rm, rb, nx, xout, xrb);
      else unshuffle_scan_fast<2>(img, out, ne, rm, rb, nx, xout, xrb);
    } else {
      uint64_t xr;
      if (ds_later_fused(d, streams, bk.chunk, bk.block, dsts, stage, maskout, mask_stride, &xr)) continue;   // pass 1 wrote it
      if (d.typesize == 4) unshuffle_xor_fast<4>(img, dsts[bk.chunk], out, ne, rm, rb);
      else if (d.typesize == 8) unshuffle_xor_fast<8>(img, dsts[bk.chunk], out, ne, rm, rb);
      else unshuffle_xor_fast<2>(img, dsts[bk.chunk], out, ne, rm, rb);
    }
  }
}

// Grid-stride over the batch's blocks (count and active slots from the device totals, so the
// sync-free path can launch every slot and pass: the ones with nothing to do exit at once).
// pass 1 / 2 are the block-0-first halves of a delta pipeline; without any delta chunk pass 1
// runs every block and pass 2 nothing.
__global__ __launch_bounds__(kBlockThreads) void k_dfilter(DChunk* __restrict__ ch, const DBlock* __restrict__ blocks,
                                                           const DStream* __restrict__ streams,
                                                           uint8_t* const* __restrict__ dsts, uint8_t* __restrict__ stage,
                                                           uint8_t* __restrict__ stage2, int slot, int pass,
                                                           const DTotals* __restrict__ tot,
                                                           const uint8_t* __restrict__ maskout, int32_t mask_stride) {
  if (!((tot->slot_mask >> slot) & 1)) return;
  if (!tot->any_delta) {
    if (pass == 2) return;
    pass = 0;
  }
  const int32_t nb = tot->nblocks;
  for (int32_t idx = blockIdx.x; idx < nb; idx += gridDim.x)
    dfilter_block(ch, blocks, streams, dsts, stage, stage2, slot, pass, idx, maskout, mask_stride);
}

// memcpyed / special chunks (blosc/blosc2.c:1865-1935): grid (pieces, chunks), chunks strided.
__device__ __forceinline__ void dspecial_chunk(const uint8_t* const* __restrict__ srcs, uint8_t* const* __restrict__ dsts,
                                               const DChunk* __restrict__ ch, int32_t c) {
  const DChunk d = ch[c];
  if (d.status < 0 || d.nstreams != 0 || d.nbytes == 0) return;
  const bool memcpyed = d.flags & kFlagMemcpy;
  const uint8_t* s = srcs[c];
  uint8_t* o = dsts[c];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t i0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (d.special == kSpecialZero) {
    for (int64_t i = i0; i < d.nbytes; i += stride) o[i] = 0;
  } else if (d.special == kSpecialNan) {
    if (d.typesize == 4) { for (int64_t i = i0; i < d.nbytes / 4; i += stride) reinterpret_cast<uint32_t*>(o)[i] = 0x7fc00000u; }
    else { for (int64_t i = i0; i < d.nbytes / 8; i += stride) reinterpret_cast<uint64_t*>(o)[i] = 0x7ff8000000000000ull; }
  } else if (d.special == kSpecialValue) {
    const int32_t ts = rd32(s + 12) - kHdrExt;
    for (int64_t i = i0; i < d.nbytes; i += stride) o[i] = s[kHdrExt + (i % ts)];
  } else if (d.special == kSpecialUninit) {
    // nothing to write
  } else if (memcpyed) {
    for (int64_t i = i0; i < d.nbytes; i += stride) o[i] = s[d.overhead + i];
  }
}

__global__ void k_dspecial(const uint8_t* const* __restrict__ srcs, uint8_t* const* __restrict__ dsts,
                           const DChunk* __restrict__ ch, int32_t n, const DTotals* __restrict__ tot) {
  if (!tot->any_special) return;
  for (int32_t c = blockIdx.y; c < n; c += gridDim.y) dspecial_chunk(srcs, dsts, ch, c);
}

__global__ void k_dstatus(const DChunk* __restrict__ ch, int32_t* __restrict__ status, int32_t n) {
  const int32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const DChunk& d = ch[c];
  status[c] = (d.status >= 0 && d.errkey != kNoErr) ? -(int32_t)(d.errkey & 0xff) : d.status;
}

// B2H_DEC_RING (read per call) forces the ring; unset: 8 KiB (20 waves per CU, T's best), or
// 32 KiB when every stream of the batch fits the 32 KiB shape's resident waves at once (a
// per-call chunk: then occupancy buys nothing, and the larger ring keeps far sources in LDS,
// allows 8 KiB batches and lifts the 96-VGPR cap).
static int dec_ring_log(int64_t nstreams) {
  const char* e = getenv("B2H_DEC_RING");
  if (e) return std::max(12, std::min(15, atoi(e)));
  static const int slots15 = resident_slots(reinterpret_cast<const void*>(&k_decode<15>), size_t(1) << 15);
  return nstreams <= slots15 ? 15 : 13;
}

template <int RLOG>
static void launch_decode(const uint8_t* const* d_src, uint8_t* const* d_dst, DChunk* ch, const DStream* streams,
                          uint8_t* stage, const DTotals* tot, int64_t nstreams_bound, const uint8_t* d_maskout,
                          int32_t mask_stride, int32_t* next, const int32_t* order, int32_t* bcnt, int64_t* dbg,
                          hipStream_t st) {
  const size_t lds = size_t(1) << RLOG;
  const int slots = resident_slots(reinterpret_cast<const void*>(&k_decode<RLOG>), lds);
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>(nstreams_bound, slots));
  k_decode<RLOG><<<grid, 64, lds, st>>>(d_src, d_dst, ch, streams, stage, tot, d_maskout, mask_stride, next, order,
                                        bcnt, dbg);
}

static int decompress_locked(Workspace* ws, const uint8_t* const* d_src, const int32_t* d_srcsize,
                             uint8_t* const* d_dst, const int32_t* d_dstsize, int32_t n, int64_t dst_bound,
                             int32_t* d_status, const uint8_t* d_maskout, hipStream_t st, int64_t src_bound,
                             int mode = 0, int32_t mask_stride = 0) {
  if (ws->dchunks.ensure(sizeof(DChunk) * (size_t)n) < 0 || ws->dtotals.ensure(sizeof(DTotals)) < 0) return E_MEMORY;
  DChunk* ch = ws->dchunks.as<DChunk>();
  DTotals* tot = ws->dtotals.as<DTotals>();
  const bool bounded = src_bound >= 0;
  // table capacities: exact (one host sync) or from the bounds (every block owns a 4-byte bstart
  // and every stream a 4-byte csize word inside its chunk)
  int64_t cap_blocks = -1, cap_streams = -1, cap_stage = -1;
  if (bounded) {
    cap_blocks = cap_streams = src_bound / 4 + 1;
    cap_stage = std::max<int64_t>(dst_bound, 0);
  }
  static const int no_fuse = getenv("B2H_FUSE_UNSHUFFLE") && atoi(getenv("B2H_FUSE_UNSHUFFLE")) == 0 ? 8 : 0;
  // mode bit 16: no in-launch DELTA + SHUFFLE -- always in default builds, and with block masks
  // (a masked block 0 never completes); a B2H_DEC_FUSE_DS_BUILD build plans it when
  // B2H_DEC_FUSE_DS=1.  Measured slower than the separate k_dfilter pass on C4 (decompress 20.2
  // vs 12.0 ms: one wave per 512 KiB block is latency-bound where k_dfilter's 256-thread
  // workgroups keep the bytes in flight)
#if B2H_DEC_FUSE_DS_BUILD
  const char* fds = getenv("B2H_DEC_FUSE_DS");
  const int ds_off = (d_maskout || !(fds && atoi(fds) == 1)) ? 16 : 0;
#else
  const int ds_off = 16;
#endif
  k_dplan_chunks<<<(n + 255) / 256, 256, 0, st>>>(d_src, d_srcsize, d_dstsize, ch, n, mode | no_fuse | ds_off);
  k_dscan<<<1, 1024, 0, st>>>(ch, n, tot, cap_blocks, cap_streams, cap_stage, d_dst);
  HIPCHK(hipGetLastError());
  DTotals h{};
  if (bounded) {
    h.nblocks = (int32_t)std::min<int64_t>(cap_blocks, 0x7fffffff);
    h.nstreams = (int32_t)std::min<int64_t>(cap_streams, 0x7fffffff);
    h.stage_bytes = cap_stage;
    h.max_filters = 2;      // unknown here: stage and stage2 both available
    h.slot_mask = 0x3f;     // every slot launched; the kernels read the real mask
    h.any_delta = 1;
    h.any_special = 1;
    h.any_ds = 1;
  } else {
    HIPCHK(hipMemcpyAsync(&h, tot, sizeof h, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  int rc = 0;
  if (h.nblocks > 0) {
    rc |= ws->dblocks.ensure(sizeof(DBlock) * (size_t)h.nblocks);
    rc |= ws->dstreams.ensure(sizeof(DStream) * (size_t)h.nstreams);
    rc |= ws->stage.ensure((size_t)h.stage_bytes);
    if (h.max_filters >= 2) rc |= ws->stage2.ensure((size_t)h.stage_bytes);
    if (rc) return E_MEMORY;
    if (ws->dorder.ensure(sizeof(int32_t) * (size_t)h.nstreams)) return E_MEMORY;
    if (ws->dbcnt.ensure(sizeof(int32_t) * (size_t)h.nblocks)) return E_MEMORY;
    int32_t* bcnt = ws->dbcnt.as<int32_t>();   // per-block finished-stream counts, zeroed by the planner
    DBlock* blocks = ws->dblocks.as<DBlock>();
    DStream* streams = ws->dstreams.as<DStream>();
    int32_t* order = ws->dorder.as<int32_t>();
    if (ws->dqctr.ensure(16)) return E_MEMORY;
    int32_t* next = ws->dqctr.as<int32_t>();   // [0]: the decoder's pull counter, [1..2]: the order's ends
    HIPCHK(hipMemsetAsync(next, 0, 4 * sizeof(int32_t), st));
    const int64_t pb_grid = std::max<int64_t>(1, std::min<int64_t>((h.nblocks + 255) / 256, 4096));
    static const int ord_mode = [] { const char* e = getenv("B2H_DEC_ORDER"); return e ? atoi(e) : 1; }();
    k_dplan_blocks<<<(uint32_t)pb_grid, 256, 0, st>>>(d_src, d_srcsize, ch, n, blocks, streams, tot, order, next + 1,
                                                       d_maskout, mask_stride, bcnt, ord_mode);
    ev_decode.start(st);
    {
      int64_t* dbg = nullptr;
      if (g_ddebug) {
        if (ws->ddbg.ensure(sizeof(int64_t) * 2 * (size_t)h.nstreams)) return E_MEMORY;
        dbg = ws->ddbg.as<int64_t>();
      }
      const int rlog = dec_ring_log(h.nstreams);
      uint8_t* stage = ws->stage.as<uint8_t>();
      if (rlog == 12) launch_decode<12>(d_src, d_dst, ch, streams, stage, tot, h.nstreams, d_maskout, mask_stride, next, order, bcnt, dbg, st);
      else if (rlog == 13) launch_decode<13>(d_src, d_dst, ch, streams, stage, tot, h.nstreams, d_maskout, mask_stride, next, order, bcnt, dbg, st);
      else if (rlog == 14) launch_decode<14>(d_src, d_dst, ch, streams, stage, tot, h.nstreams, d_maskout, mask_stride, next, order, bcnt, dbg, st);
      else launch_decode<15>(d_src, d_dst, ch, streams, stage, tot, h.nstreams, d_maskout, mask_stride, next, order, bcnt, dbg, st);
    }
    ev_decode.stop(st);
    ev_unfilter.start(st);
    if (h.max_filters > 0) {
      // exact path: one workgroup per block; bounded path: a resident grid striding the blocks.
      // The bounded grid is a prime count: with a power of two, every workgroup's blocks share
      // one index modulo the chunks' block count (4 in C4), so pass 1 (block 0 of each chunk)
      // ran on a quarter of the grid and pass 2 on three quarters (C4: 3.25 ms for block 0s).
      const uint32_t grid = (uint32_t)(bounded ? std::min<int64_t>(h.nblocks, 4093) : h.nblocks);
      const int passes = h.any_delta ? 2 : 1;
      for (int ps = 0; ps < passes; ps++) {
        const int pass = h.any_delta ? ps + 1 : 0;
        if (pass > 0 && h.any_ds)
          k_dfilter_ds<<<grid, kBlockThreads, 0, st>>>(ch, blocks, ws->dstreams.as<DStream>(), d_dst, ws->stage.as<uint8_t>(),
                                                       pass, tot, d_maskout, mask_stride);
        for (int slot = 5; slot >= 0; slot--)
          if ((h.slot_mask >> slot) & 1)
            k_dfilter<<<grid, kBlockThreads, 0, st>>>(ch, blocks, ws->dstreams.as<DStream>(), d_dst, ws->stage.as<uint8_t>(),
                                                     ws->stage2.as<uint8_t>(), slot, pass, tot, d_maskout, mask_stride);
      }
    }
    ev_unfilter.stop(st);
  }
  if (h.any_special) {
    dim3 grid(bounded ? 16 : 64, (uint32_t)std::min<int32_t>(n, 4096));
    k_dspecial<<<grid, 256, 0, st>>>(d_src, d_dst, ch, n, tot);
  }
  k_dstatus<<<(n + 255) / 256, 256, 0, st>>>(ch, d_status, n);
  HIPCHK(hipGetLastError());
  return 0;
}

int decompress_batch(const uint8_t* const* d_src, const int32_t* d_srcsize, uint8_t* const* d_dst,
                     const int32_t* d_dstsize, int32_t n, int64_t dst_bound, int32_t* d_status,
                     const uint8_t* d_maskout, hipStream_t st, Workspace* wsx, int64_t src_bound, int mode,
                     int32_t mask_stride) {
  if (n <= 0) return 0;
  Workspace* ws = wsx ? wsx : ws_for_current_device();
  WsUse use(ws, st);
  if (use.rc) return use.rc;
  return decompress_locked(ws, d_src, d_srcsize, d_dst, d_dstsize, n, dst_bound, d_status, d_maskout, st, src_bound,
                           mode, mask_stride);
}

__global__ void k_fill_ptrs(const uint8_t* src, int64_t src_stride, const int32_t* cbytes, uint8_t* dst, int64_t dst_stride,
                            int32_t dst_cap, const uint8_t** sp, int32_t* ss, uint8_t** dp, int32_t* ds, int32_t n) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  sp[i] = src + (int64_t)i * src_stride;
  // a chunk may not reach into the next one (the bound of the sync-free tables relies on it)
  ss[i] = src_stride > 0 ? (int32_t)min<int64_t>(cbytes[i], src_stride) : cbytes[i];
  dp[i] = dst + (int64_t)i * dst_stride;
  ds[i] = dst_cap;
}

int decompress_batch_strided(const uint8_t* d_src, int64_t src_stride, const int32_t* d_cbytes, int32_t n, uint8_t* d_dst,
                             int64_t dst_stride, int32_t dst_cap, int32_t* d_status, hipStream_t st, Workspace* wsx) {
  if (n <= 0) return 0;
  Workspace* ws = wsx ? wsx : ws_for_current_device();
  WsUse use(ws, st);
  if (use.rc) return use.rc;
  const size_t need = (size_t)n * (2 * sizeof(void*) + 2 * sizeof(int32_t)) + 64;
  if (ws->ptrs.ensure(need) < 0) return E_MEMORY;
  uint8_t* base = ws->ptrs.as<uint8_t>();
  const uint8_t** sp = reinterpret_cast<const uint8_t**>(base);
  uint8_t** dp = reinterpret_cast<uint8_t**>(base + sizeof(void*) * (size_t)n);
  int32_t* ss = reinterpret_cast<int32_t*>(base + 2 * sizeof(void*) * (size_t)n);
  int32_t* ds = ss + n;
  k_fill_ptrs<<<(n + 255) / 256, 256, 0, st>>>(d_src, src_stride, d_cbytes, d_dst, dst_stride, dst_cap, sp, ss, dp, ds, n);
  HIPCHK(hipGetLastError());
  // src_stride == 0 (every chunk the same source) gives no bound: exact tables
  const int64_t src_bound = src_stride > 0 ? (int64_t)n * src_stride : -1;
  return decompress_locked(ws, sp, ss, dp, ds, n, (int64_t)n * dst_cap, d_status, nullptr, st, src_bound);
}

// ================================================================ chunk packing (gatherv) ====
// Exclusive prefix sum of n int32 sizes into int64 offsets[0..n] (one workgroup, tiles of 1024).
__global__ __launch_bounds__(1024) void k_scan_sizes(const int32_t* __restrict__ sizes, int32_t n,
                                                     int64_t* __restrict__ off) {
  __shared__ int64_t part[1024 / 64];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int32_t base = 0; base < n; base += 1024) {
    const int32_t i = base + threadIdx.x;
    const int64_t v = i < n ? (int64_t)max(sizes[i], 0) : 0;
    int64_t incl = v;   // wave inclusive scan (64-bit, shuffles)
    for (int d = 1; d < 64; d <<= 1) {
      const int64_t o = __shfl_up(incl, d);
      if (lane >= d) incl += o;
    }
    if (lane == 63) part[w] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < w; k++) before += part[k];
    if (i < n) off[i] = before + incl - v;
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) off[n] = carry;
}

// grid (pieces, chunks): piece p of chunk c copies its 1/gridDim.x share, one wave per sub-share
__global__ __launch_bounds__(256) void k_pack(const uint8_t* __restrict__ src, int64_t src_stride,
                                              const int64_t* __restrict__ off, int32_t n, uint8_t* __restrict__ dst,
                                              int unpack) {
  for (int32_t c = blockIdx.y; c < n; c += gridDim.y) {
    const int64_t o = off[c];
    const int32_t len = (int32_t)(off[c + 1] - o);
    if (len <= 0) continue;
    const int32_t parts = gridDim.x * (blockDim.x / 64);
    const int32_t per = ((len + parts - 1) / parts + 15) & ~15;
    const int32_t k = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    const int32_t a = min(len, k * per), b = min(len, a + per);
    if (b <= a) continue;
    if (!unpack) wave_copy((gout_t)(dst + o + a), (gin_t)(src + (int64_t)c * src_stride + a), b - a);
    else wave_copy((gout_t)(dst + (int64_t)c * src_stride + a), (gin_t)(src + o + a), b - a);
  }
}

// Streaming device copy (the measured copy peak of bench.py): 16 B per lane, 4 loads in flight.
__global__ __launch_bounds__(256) void k_copy16(uint4* __restrict__ d, const uint4* __restrict__ s, int64_t n16) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = s[i], b = s[i + stride], c = s[i + 2 * stride], e = s[i + 3 * stride];
    d[i] = a; d[i + stride] = b; d[i + 2 * stride] = c; d[i + 3 * stride] = e;
  }
  for (; i < n16; i += stride) d[i] = s[i];
}

int device_copy(uint8_t* d_dst, const uint8_t* d_src, int64_t nbytes, hipStream_t st) {
  if (nbytes <= 0) return 0;
  if (((reinterpret_cast<uintptr_t>(d_dst) | reinterpret_cast<uintptr_t>(d_src)) & 15) != 0 || (nbytes & 15) != 0) {
    HIPCHK(hipMemcpyAsync(d_dst, d_src, (size_t)nbytes, hipMemcpyDeviceToDevice, st));
    return 0;
  }
  const int64_t n16 = nbytes / 16;
  const uint32_t grid = (uint32_t)std::max<int64_t>(1, std::min<int64_t>((n16 + 1023) / 1024, 256 * 16));
  k_copy16<<<grid, 256, 0, st>>>(reinterpret_cast<uint4*>(d_dst), reinterpret_cast<const uint4*>(d_src), n16);
  HIPCHK(hipGetLastError());
  return 0;
}

__global__ void k_sizes_from_offsets(const int64_t* __restrict__ off, int32_t n, int32_t* __restrict__ sizes) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) sizes[i] = (int32_t)(off[i + 1] - off[i]);
}

int pack_chunks(const uint8_t* d_src, int64_t src_stride, const int32_t* d_sizes, int32_t n, uint8_t* d_dst,
                int64_t* d_offsets, hipStream_t st) {
  if (n < 0) return E_PARAM;
  k_scan_sizes<<<1, 1024, 0, st>>>(d_sizes, n, d_offsets);
  if (n > 0) {
    dim3 grid(16, (uint32_t)std::min<int32_t>(n, 8192));
    k_pack<<<grid, 256, 0, st>>>(d_src, src_stride, d_offsets, n, d_dst, 0);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int unpack_chunks(const uint8_t* d_src, const int64_t* d_offsets, int32_t n, uint8_t* d_dst, int64_t dst_stride,
                  int32_t* d_sizes, hipStream_t st) {
  if (n <= 0) return n < 0 ? E_PARAM : 0;
  dim3 grid(16, (uint32_t)std::min<int32_t>(n, 8192));
  k_pack<<<grid, 256, 0, st>>>(d_src, dst_stride, d_offsets, n, d_dst, 1);
  if (d_sizes) k_sizes_from_offsets<<<(n + 255) / 256, 256, 0, st>>>(d_offsets, n, d_sizes);
  HIPCHK(hipGetLastError());
  return 0;
}

// ============================================================================ raw filters ====
__global__ __launch_bounds__(kBlockThreads) void k_raw_shuffle(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                               int32_t nbytes, int32_t ts, int inverse) {
  // blosc2_shuffle over a whole buffer (blosc/shuffle.c:416-449): every workgroup owns elements
  // [e0, e1) of all planes (plane stride n), 16-byte element-side loads / u32 plane-side stores
  const int32_t n = nbytes / ts;
  const int32_t per = ((n + gridDim.x - 1) / gridDim.x + 3) & ~3;
  const int32_t e0 = min(n, (int32_t)blockIdx.x * per), e1 = min(n, e0 + per);
  if (e0 < e1) {
    const int32_t cnt = e1 - e0;
    const bool fast = (cnt % 4 == 0) && (n % 4 == 0) && aligned16(s) && aligned16(d) &&
                      (ts == 2 || ts == 4 || ts == 8 || ts == 16);
    if (fast) {
      const uint8_t* es = (inverse ? d : s) + (int64_t)e0 * ts;   // element side
      const uint8_t* ps = (inverse ? s : d) + e0;                  // plane side
      if (!inverse) {
        uint8_t* pd = d + e0;
        if (ts == 4) shuffle_fast<4>(es, pd, cnt, n);
        else if (ts == 8) shuffle_fast<8>(es, pd, cnt, n);
        else if (ts == 2) shuffle_fast<2>(es, pd, cnt, n);
        else shuffle_fast<16>(es, pd, cnt, n);
      } else {
        uint8_t* ed = d + (int64_t)e0 * ts;
        if (ts == 4) unshuffle_fast<4>(ps, ed, cnt, n);
        else if (ts == 8) unshuffle_fast<8>(ps, ed, cnt, n);
        else if (ts == 2) unshuffle_fast<2>(ps, ed, cnt, n);
        else unshuffle_fast<16>(ps, ed, cnt, n);
      }
    } else {
      for (int64_t i = threadIdx.x; i < (int64_t)cnt * ts; i += blockDim.x) {
        const int32_t e = e0 + (int32_t)(i / ts), plane = (int32_t)(i % ts);
        if (!inverse) d[(int64_t)plane * n + e] = s[(int64_t)e * ts + plane];
        else d[(int64_t)e * ts + plane] = s[(int64_t)plane * n + e];
      }
    }
  }
  if (blockIdx.x == 0)
    for (int32_t i = n * ts + threadIdx.x; i < nbytes; i += blockDim.x) d[i] = s[i];
}

int shuffle_dev(int32_t ts, int32_t nbytes, const uint8_t* d_src, uint8_t* d_dst, bool inverse, hipStream_t st) {
  if (ts < 1 || ts > 256 || nbytes < 0) return E_PARAM;
  if (nbytes == 0) return 0;
  const int32_t n = nbytes / ts;
  const int grid = std::max(1, std::min(4096, n / 1024 + 1));
  k_raw_shuffle<<<grid, kBlockThreads, 0, st>>>(d_src, d_dst, nbytes, ts, inverse ? 1 : 0);
  HIPCHK(hipGetLastError());
  return nbytes;
}

__global__ __launch_bounds__(kBlockThreads) void k_raw_bitshuffle(const uint8_t* __restrict__ s, uint8_t* __restrict__ d,
                                                                  int32_t nbytes, int32_t ts, int inverse,
                                                                  uint8_t version) {
  const int32_t nel = nbytes / ts;
  if (inverse && version == 2 && (nel % 8) != 0) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nbytes; i += (int64_t)gridDim.x * blockDim.x) d[i] = s[i];
    return;
  }
  const int32_t m = nel & ~7;
  const int32_t rowlen = m / 8;
  for (int32_t gi = blockIdx.x * blockDim.x + threadIdx.x; gi < rowlen; gi += gridDim.x * blockDim.x) {
    if (!inverse) {
      const uint8_t* e8 = s + (int64_t)gi * 8 * ts;
      for (int32_t b = 0; b < ts; b++) {
        uint64_t x = 0;
        for (int r = 0; r < 8; r++) x |= (uint64_t)e8[r * ts + b] << (8 * r);
        x = bit_transpose8(x);
        for (int k = 0; k < 8; k++) d[(int64_t)(8 * b + k) * rowlen + gi] = (uint8_t)(x >> (8 * k));
      }
    } else {
      uint8_t* e8 = d + (int64_t)gi * 8 * ts;
      for (int32_t b = 0; b < ts; b++) {
        uint64_t y = 0;
        for (int k = 0; k < 8; k++) y |= (uint64_t)s[(int64_t)(8 * b + k) * rowlen + gi] << (8 * k);
        y = bit_transpose8(y);
        for (int r = 0; r < 8; r++) e8[r * ts + b] = (uint8_t)(y >> (8 * r));
      }
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = (int64_t)m * ts + threadIdx.x; i < nbytes; i += blockDim.x) d[i] = s[i];
}

int bitshuffle_dev(int32_t ts, int32_t nbytes, const uint8_t* d_src, uint8_t* d_dst, bool inverse, uint8_t version,
                   hipStream_t st) {
  if (ts < 1 || ts > 256 || nbytes < 0) return E_PARAM;
  if (nbytes == 0) return 0;
  const int32_t rows = (nbytes / ts) / 8;
  const int grid = std::max(1, std::min(4096, rows / 256 + 1));
  k_raw_bitshuffle<<<grid, kBlockThreads, 0, st>>>(d_src, d_dst, nbytes, ts, inverse ? 1 : 0, version);
  HIPCHK(hipGetLastError());
  return nbytes;
}

}  // namespace b2h
