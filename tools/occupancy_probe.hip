// Calibration: how many 1-wave workgroups with L bytes of dynamic LDS are resident at once?
// Each workgroup spins ~200 us and records its realtime start/end.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
__global__ void spin(unsigned long long* rec, int lds_words) {
  extern __shared__ unsigned int sm[];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = threadIdx.x; i < lds_words; i += blockDim.x) sm[i] = i;
  while (__builtin_amdgcn_s_memrealtime() - t0 < 20000) __builtin_amdgcn_s_sleep(10);
  if (threadIdx.x == 0) { rec[2 * blockIdx.x] = t0; rec[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime(); }
  if (sm[threadIdx.x] == 12345678u) rec[0] = 0;
}
int main() {
  const int n = 8192;
  unsigned long long* d; hipMalloc(&d, 2 * n * 8);
  hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int threads : {64, 256}) for (int kb : {0, 16, 32, 36, 40, 48, 64}) {
    spin<<<n, threads, kb * 1024>>>(d, kb * 256);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * n);
    hipMemcpy(h.data(), d, 2 * n * 8, hipMemcpyDeviceToHost);
    std::vector<std::pair<long long, int>> ev;
    for (int i = 0; i < n; i++) { ev.push_back({(long long)h[2 * i], 1}); ev.push_back({(long long)h[2 * i + 1], -1}); }
    std::sort(ev.begin(), ev.end());
    int a = 0, mx = 0; for (auto& e : ev) { a += e.second; mx = std::max(mx, a); }
    long long span = ev.back().first - ev.front().first;
    printf("threads %d lds %2d KiB: max resident %d  span %.0f us (ideal %.0f us)\n", threads, kb, mx, span / 100.0,
           200.0 * n / std::max(1, mx));
  }
  return 0;
}
