// Fast-mode encoder micro-benchmark (diagnostics only): encode one stream per two-wave workgroup
// with the product encode_stream_fast (matcher + parser), many workgroups, and report cycles per
// stream and the parser's per-phase sums.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../c-blosc2_amd/csrc fast_micro.hip -o fast_micro
//   ./fast_micro plane.bin [clevel] [tablog]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define B2H_ENC_PROF 1
#ifndef FM_POS
#define FM_POS uint16_t
#define FM_POSB 2
#endif
#include "b2h_lzfast.h"
using namespace b2h;

__global__ __launch_bounds__(128) void k_enc(const uint8_t* in, int32_t n, int clevel, int tablog, uint8_t* out,
                                             int64_t* cycles, StreamResult* res) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  B2H_LDS uint8_t* tab = (B2H_LDS uint8_t*)smem;
  B2H_LDS uint8_t* oring = (B2H_LDS uint8_t*)(smem + ((size_t)FM_POSB << tablog));
  B2H_LDS FastShared* sh = (B2H_LDS FastShared*)(smem + ((size_t)FM_POSB << tablog) + kOutRing);
  const bool matcher = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  StreamResult r = encode_stream_fast<FM_POS>((gin_t)in, n, clevel, (gout_t)(out + (size_t)blockIdx.x * (n + 64)), tab,
                                              tablog, oring, sh, true, matcher);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 64) { cycles[blockIdx.x] = (int64_t)(t1 - t0); res[blockIdx.x] = r; }
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
  if (argc < 2) { fprintf(stderr, "usage: %s plane.bin [clevel] [tablog]\n", argv[0]); return 2; }
  auto in = slurp(argv[1]);
  const int clevel = argc > 2 ? atoi(argv[2]) : 5;
  const int tablog = argc > 3 ? atoi(argv[3]) : 13;
  const int32_t n = (int32_t)in.size();
  uint8_t *din, *dout;
  hipMalloc(&din, n + 256);
  hipMemset(din, 0, n + 256);
  hipMemcpy(din, in.data(), n, hipMemcpyHostToDevice);
  const int maxblk = 4096;
  hipMalloc(&dout, (size_t)maxblk * (n + 64));
  int64_t* dc; StreamResult* dr;
  hipMalloc(&dc, maxblk * 8); hipMalloc(&dr, maxblk * sizeof(StreamResult));
  const size_t lds = ((size_t)FM_POSB << tablog) + kOutRing + ((sizeof(FastShared) + 15) & ~size_t(15));
  hipFuncSetAttribute(reinterpret_cast<const void*>(&k_enc), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int nblk : {1, 256, 1024, 4096}) {
    uint64_t z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_enc_prof), z, sizeof z);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    k_enc<<<nblk, 128, lds>>>(din, n, clevel, tablog, dout, dc, dr);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0; hipEventElapsedTime(&ms, a, b);
    std::vector<int64_t> c(nblk);
    std::vector<StreamResult> r(nblk);
    hipMemcpy(c.data(), dc, nblk * 8, hipMemcpyDeviceToHost);
    hipMemcpy(r.data(), dr, nblk * sizeof(StreamResult), hipMemcpyDeviceToHost);
    double mean = 0; for (auto x : c) mean += x; mean /= nblk;
    printf("blocks %5d: %.3f ms, cycles/stream %.0f, kind %d size %d tiles %d (%.0f cycles/tile)\n", nblk, ms, mean,
           r[0].kind, r[0].size, r[0].windows, mean / (r[0].windows ? r[0].windows : 1));
    uint64_t pr[16];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_enc_prof), sizeof pr);
    const char* nm[8] = {"M: produce", "P: compare", "P: chain walk", "M: exchange", "M: barrier", "P: (match ext)", "P: barrier", "M: 1st words"};
    for (int pass = 1; pass >= 0; pass--)
      for (int i = 0; i < 8; i++)
        printf("   %s %-12s %10.0f cycles/stream\n", pass ? "probe" : "main ", nm[i], pr[8 * pass + i] / (double)nblk);
  }
  return 0;
}
