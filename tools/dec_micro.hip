// Decoder micro-benchmark (diagnostics only): decode one BloscLZ stream per wave, many waves,
// and report s_memtime cycles per stream for the product decoder and for stripped variants.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../c-blosc2_amd/csrc dec_micro.hip -o dec_micro
//   ./dec_micro stream.bin expected.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define B2H_DEC_PROF 1
#include "b2h_lz.h"
using namespace b2h;

// MODE 0: product decoder.  1: token parse only (no LDS traffic).  2: parse + LDS writes of
// literals/matches but no LDS reads (match bytes not copied).
template <int MODE>
__device__ int32_t variant(gin_t in, int32_t length, gout_t out, int32_t maxout, B2H_LDS uint8_t* ring) {
  if (MODE == 0) return wave_lz_decode_ring<15>(in, length, out, maxout, ring);
  if (MODE == 3) return wave_lz_decode_par<15>(in, length, out, maxout, ring);
  const int lane = lane_id();
  InWin W;
  inwin_reload(W, in, length, 0);
  int32_t ip = 0, op = 0;
  if (lane == 0) W.w0 &= ~(0xe0u << (8 * (-W.wpos)));
  asm volatile("" : "+s"(ip), "+s"(W.wpos));
  uint32_t acc = 0;
  for (;;) {
    const int32_t k = inwin_seek(W, in, length, ip);
    const uint32_t t = inwin_peek4(W, k);
    const uint32_t ctrl = t & 0xffu;
    int32_t p = ip + 1;
    if (ctrl >= 32) {
      int32_t len = (int32_t)(ctrl >> 5) + 2;
      const int32_t ofs = (int32_t)(ctrl & 31u) << 8;
      int32_t dist;
      if (len == 9) {
        uint32_t code;
        len = 6;
        do {
          code = inwin_byte(W, in, length, p++);
          len += (int32_t)code;
        } while (code == 255);
        code = inwin_byte(W, in, length, p++);
        len += 3;
        dist = ofs + (int32_t)code + 1;
        if (code == 255 && ofs == (31 << 8)) p += 2;
      } else {
        const uint32_t code = (t >> 8) & 0xffu;
        p += 1;
        dist = ofs + (int32_t)code + 1;
        if (code == 255 && ofs == (31 << 8)) p += 2;
      }
      if (p >= length) break;
      if (MODE == 2 && lane < len && len <= 64) ring[(op + lane) & 32767] = (uint8_t)dist;
      acc += dist;
      op += len;
    } else {
      const int32_t run = (int32_t)ctrl + 1;
      const int32_t idx = k + 1 + lane;
      uint32_t v = (uint32_t)__shfl((int)W.w0, idx >> 2);
      if (MODE == 2 && lane < run) ring[(op + lane) & 32767] = (uint8_t)(v >> (8 * (idx & 3)));
      acc += v;
      op += run;
      p += run;
      if (p >= length) break;
    }
    ip = p;
  }
  if (lane == 0 && acc == 0x12345) out[0] = 1;
  return op;
}

template <int MODE>
__global__ __launch_bounds__(64) void k_micro(const uint8_t* in, int32_t length, uint8_t* out, int32_t nb,
                                              int64_t* cycles, int32_t* got) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const int32_t g = variant<MODE>((gin_t)in, length, (gout_t)(out + (size_t)blockIdx.x * nb), nb,
                                  (B2H_LDS uint8_t*)smem);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { cycles[blockIdx.x] = (int64_t)(t1 - t0); got[blockIdx.x] = g; }
}

static std::vector<uint8_t> slurp(const char* f) {
  FILE* fp = fopen(f, "rb");
  if (!fp) { perror(f); exit(1); }
  std::vector<uint8_t> v;
  uint8_t buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, fp)) > 0) v.insert(v.end(), buf, buf + n);
  fclose(fp);
  return v;
}

template <int MODE>
static void run(const uint8_t* din, int32_t len, uint8_t* dout, int32_t nb, int nblk, const std::vector<uint8_t>& want) {
  int64_t* dc; int32_t* dg;
  hipMalloc(&dc, nblk * 8); hipMalloc(&dg, nblk * 4);
  hipMemset(dout, 0, (size_t)nblk * nb);
  k_micro<MODE><<<nblk, 64, 32768>>>(din, len, dout, nb, dc, dg);
  hipDeviceSynchronize();
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  k_micro<MODE><<<nblk, 64, 32768>>>(din, len, dout, nb, dc, dg);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0; hipEventElapsedTime(&ms, a, b);
  std::vector<int64_t> c(nblk); std::vector<int32_t> g(nblk);
  hipMemcpy(c.data(), dc, nblk * 8, hipMemcpyDeviceToHost);
  hipMemcpy(g.data(), dg, nblk * 4, hipMemcpyDeviceToHost);
  double mean = 0; for (auto x : c) mean += x; mean /= nblk;
  bool ok = true;
  if (MODE == 0 || MODE == 3) {
    std::vector<uint8_t> o(nb);
    hipMemcpy(o.data(), dout + (size_t)(nblk - 1) * nb, nb, hipMemcpyDeviceToHost);
    ok = g[0] == nb && o == want;
  }
  printf("mode %d blocks %5d: %.3f ms, cycles/stream mean %.0f (got %d%s)\n", MODE, nblk, ms, mean, g[0],
         (MODE == 0 || MODE == 3) ? (ok ? ", output OK" : ", OUTPUT MISMATCH") : "");
  if (MODE == 3) {
    uint64_t pr[8];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_dec_prof), sizeof pr);
    const char* nm[6] = {"parse", "walk", "scan+checks", "literals", "matches", "serial"};
    for (int i = 0; i < 6; i++) printf("   %-12s %10.0f cycles/stream\n", nm[i], pr[i] / (2.0 * nblk));
    uint64_t z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_dec_prof), z, sizeof z);
  }
  hipFree(dc); hipFree(dg);
}

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: %s stream.bin expected.bin\n", argv[0]); return 2; }
  auto s = slurp(argv[1]);
  auto want = slurp(argv[2]);
  const int32_t nb = (int32_t)want.size();
  uint8_t *din, *dout;
  hipMalloc(&din, s.size() + 64);
  hipMemcpy(din, s.data(), s.size(), hipMemcpyHostToDevice);
  const int maxblk = 2560;
  hipMalloc(&dout, (size_t)maxblk * nb);
  for (int nblk : {1, 256, 1280, 2560}) {
    run<0>(din, (int32_t)s.size(), dout, nb, nblk, want);
    run<1>(din, (int32_t)s.size(), dout, nb, nblk, want);
    run<2>(din, (int32_t)s.size(), dout, nb, nblk, want);
    run<3>(din, (int32_t)s.size(), dout, nb, nblk, want);
  }
  return 0;
}
