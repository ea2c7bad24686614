// Occupancy probe (diagnostic): one-wave workgroups that hold their slot for
// ~200 us, with a given static LDS size and a register budget set by launch
// bounds; records each wave's start / end (wall clock) so the host can count
// the waves resident at once. Answers: how many 1-wave workgroups with
// 12.6 KB of LDS and 168 / 256 VGPRs are resident per CU on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int LDSB, int LB, int VG>
__global__ __launch_bounds__(64, LB) void k_hold(unsigned long long* st, double* sink, int spin) {
  __shared__ double lds[LDSB / 8];
  if constexpr (VG == 168) asm volatile("" ::: "v167");
  if constexpr (VG == 256) asm volatile("" ::: "v255");
  if constexpr (VG == 128) asm volatile("" ::: "v127");
  const unsigned long long t0 = wall_clock64();
  if (threadIdx.x == 0) st[2 * blockIdx.x] = t0;
  double acc = threadIdx.x;
  lds[threadIdx.x % (LDSB / 8)] = acc;
  __syncthreads();
  while (wall_clock64() - t0 < (unsigned long long)spin) acc = acc * 1.0000001 + lds[(threadIdx.x * 7) % (LDSB / 8)];
  if (acc == 12345.0) sink[blockIdx.x] = acc;
  if (threadIdx.x == 0) st[2 * blockIdx.x + 1] = wall_clock64();
}

template <int LDSB, int LB, int VG>
void run(const char* name, int n) {
  unsigned long long* st; double* sink;
  hipMalloc(&st, 16ull * n); hipMalloc(&sink, 8ull * n);
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL((k_hold<LDSB, LB, VG>), dim3(n), dim3(64), 0, 0, st, sink, 20000);  // 200 us at 100 MHz
    hipDeviceSynchronize();
  }
  std::vector<unsigned long long> h(2 * n);
  hipMemcpy(h.data(), st, 16ull * n, hipMemcpyDeviceToHost);
  std::vector<std::pair<unsigned long long, int>> ev;
  for (int i = 0; i < n; ++i) { ev.push_back({h[2 * i], 1}); ev.push_back({h[2 * i + 1], -1}); }
  std::sort(ev.begin(), ev.end());
  int cur = 0, mx = 0;
  for (auto& e : ev) { cur += e.second; mx = std::max(mx, cur); }
  printf("%-28s blocks %6d: max resident waves %5d (%.2f per CU)\n", name, n, mx, mx / 256.0);
  hipFree(st); hipFree(sink);
}

int main() {
  const int n = 8192;
  run<16, 8, 0>("no LDS, few VGPRs", n);
  run<16, 3, 168>("no LDS, 168 VGPRs", n);
  run<16, 2, 256>("no LDS, 256 VGPRs", n);
  run<12656, 8, 0>("12656 B LDS, few VGPRs", n);
  run<12656, 3, 168>("12656 B LDS, 168 VGPRs", n);
  run<12656, 2, 256>("12656 B LDS, 256 VGPRs", n);
  run<4704, 4, 128>("4704 B LDS, 128 VGPRs", n);
  run<8192, 8, 0>("8192 B LDS, few VGPRs", n);
  run<16384, 8, 0>("16384 B LDS, few VGPRs", n);
  return 0;
}
