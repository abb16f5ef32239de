// Encoder micro-benchmark (diagnostics only): encode one stream per wave with the product
// encode_stream, many waves, and report s_memtime cycles per stream plus per-phase sums.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../c-blosc2_amd/csrc enc_micro.hip -o enc_micro
//   ./enc_micro plane.bin expected_stream.bin [clevel]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#ifndef ENC_NOPROF
#define B2H_ENC_PROF 1
#endif
#include "b2h_lz.h"
using namespace b2h;

#ifdef ENC_WPE
#define ENC_ATTR __attribute__((amdgpu_waves_per_eu(ENC_WPE, ENC_WPE)))
#else
#define ENC_ATTR
#endif
__global__ __launch_bounds__(64) ENC_ATTR void k_enc(const uint8_t* in, int32_t n, int clevel, uint8_t* out, int64_t* cycles,
                                            StreamResult* res, uint16_t* gtab) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int hashlog = clevel == 1 ? 12 : (clevel == 2 ? 13 : 14);
#ifdef ENC_GTAB
#ifndef ENC_GPOS
#define ENC_GPOS uint16_t
#endif
  GlbTab<ENC_GPOS> htab;
  htab.t = (B2H_GLB ENC_GPOS*)((ENC_GPOS*)gtab + ((size_t)blockIdx.x << hashlog));
  B2H_LDS uint32_t* dbits = (B2H_LDS uint32_t*)smem;
  B2H_LDS uint8_t* oring = (B2H_LDS uint8_t*)(smem + ((1 << hashlog) >> 3));
#else
  LdsTab<uint16_t> htab;
  htab.t = (volatile B2H_LDS uint16_t*)smem;
  B2H_LDS uint32_t* dbits = (B2H_LDS uint32_t*)(smem + enc_bits_offset(2, hashlog));
  B2H_LDS uint8_t* oring = (B2H_LDS uint8_t*)(smem + enc_ring_offset(2, hashlog));
#endif
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  StreamResult r = encode_stream((gin_t)in, n, clevel, (gout_t)(out + (size_t)blockIdx.x * (n + 64)), htab, dbits,
                                 oring, true);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { cycles[blockIdx.x] = (int64_t)(t1 - t0); res[blockIdx.x] = r; }
}

static std::vector<uint8_t> slurp(const char* f) {
  FILE* fp = fopen(f, "rb");
  if (!fp) { perror(f); exit(1); }
  std::vector<uint8_t> v;
  uint8_t buf[65536];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, fp)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(fp);
  return v;
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s plane.bin expected.bin [clevel]\n", argv[0]); return 2; }
  auto in = slurp(argv[1]);
  auto want = slurp(argv[2]);
  const int clevel = argc > 3 ? atoi(argv[3]) : 5;
  const int32_t n = (int32_t)in.size();
  uint8_t *din, *dout;
  hipMalloc(&din, n + 64);
  hipMemset(din, 0, n + 64);
  hipMemcpy(din, in.data(), n, hipMemcpyHostToDevice);
  const int maxblk = 16384;
  hipMalloc(&dout, (size_t)maxblk * (n + 64));
  int64_t* dc; StreamResult* dr;
  hipMalloc(&dc, maxblk * 8); hipMalloc(&dr, maxblk * sizeof(StreamResult));
#ifdef ENC_GTAB
  const size_t lds = ((1 << 14) >> 3) + kOutRing;
#else
  const size_t lds = enc_lds_bytes(2, 14);
#endif
  uint16_t* gtab;
  hipMalloc(&gtab, (size_t)maxblk * (4 << 14));
  std::vector<int> sizes = {1, 256, 1024};
  if (argc > 4) sizes = {atoi(argv[4])};
  for (int nblk : sizes) {
#ifndef ENC_NOPROF
    uint64_t z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_enc_prof), z, sizeof z);
#endif
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k_enc<<<nblk, 64, lds>>>(din, n, clevel, dout, dc, dr, gtab);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    std::vector<int64_t> c(nblk);
    std::vector<StreamResult> r(nblk);
    hipMemcpy(c.data(), dc, nblk * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r.data(), dr, nblk * sizeof(StreamResult), hipMemcpyDeviceToHost);
    std::vector<uint8_t> o(r[0].size > 0 ? r[0].size : 1);
    hipMemcpy(o.data(), dout, o.size(), hipMemcpyDeviceToHost);
    // the kind blosc_c gives this stream (blosc/blosc2.c:1290-1340 run test before the codec;
    // an empty reference output = blosclz_compress returned 0 = stored raw), and for LZ streams
    // the reference's bytes
    bool same = true;
    for (uint8_t x : in) same &= x == in[0];
    const int want_kind = same ? (in[0] ? kStreamByteRun : kStreamZeroRun) : (want.empty() ? kStreamRaw : kStreamLz);
    const bool ok = r[0].kind == want_kind && (want_kind != kStreamLz || (o.size() == want.size() && o == want));
    if (!ok && r[0].kind == kStreamLz && argc > 5) {   // dump the stream for offline comparison
      FILE* fo = fopen(argv[5], "wb");
      if (fo) { fwrite(o.data(), 1, o.size(), fo); fclose(fo); }
    }
    double mean = 0; for (auto x : c) mean += x; mean /= nblk;
    printf("blocks %5d: %.3f ms, cycles/stream %.0f, kind %d size %d windows %d %s\n", nblk, ms, mean, r[0].kind,
           r[0].size, r[0].windows, ok ? "output OK (expected kind)" : "OUTPUT MISMATCH");
#ifndef ENC_NOPROF
    uint64_t pr[16];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_enc_prof), sizeof pr);
    const char* nm[8] = {"load", "hash+dups", "cand test", "chain walk", "emit", "(match ext)", "htab upd", "-"};
    for (int pass = 1; pass >= 0; pass--)
      for (int i = 0; i < 8; i++)
        printf("   %s %-12s %10.0f cycles/stream\n", pass ? "probe" : "main ", nm[i], pr[8 * pass + i] / (double)nblk);
#endif
  }
  return 0;
}
