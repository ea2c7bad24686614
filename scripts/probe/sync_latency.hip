// Host-side completion latency of a short kernel: hipStreamSynchronize vs a
// spin on hipStreamQuery vs a spin on a word the kernel writes to coherent
// mapped host memory (diagnostic for the one-candidate LCD calls).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ void k_short(unsigned* flag, unsigned v, int spin) {
  long long t0 = wall_clock64();
  while (wall_clock64() - t0 < spin) {}
  __threadfence_system();
  if (threadIdx.x == 0 && flag) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  unsigned* h = nullptr;
  unsigned* z = nullptr;
  hipHostMalloc((void**)&h, 64, hipHostMallocMapped | hipHostMallocCoherent);
  hipHostGetDevicePointer((void**)&z, h, 0);
  *h = 0;
  const int spin = 2500;  // ~25 us at 100 MHz wall clock
  for (int mode = 0; mode < 3; ++mode) {
    std::vector<double> us;
    for (int it = 0; it < 2000; ++it) {
      const unsigned v = it + 1 + mode * 100000;
      auto t0 = std::chrono::steady_clock::now();
      hipLaunchKernelGGL(k_short, dim3(1), dim3(64), 0, st, z, v, spin);
      if (mode == 0) hipStreamSynchronize(st);
      else if (mode == 1) { while (hipStreamQuery(st) == hipErrorNotReady) {} }
      else { while (__atomic_load_n(h, __ATOMIC_ACQUIRE) != v) {} }
      auto t1 = std::chrono::steady_clock::now();
      if (mode == 2) hipStreamSynchronize(st);
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::sort(us.begin(), us.end());
    printf("mode %d (%s): median %.1f us, p10 %.1f, p90 %.1f\n", mode,
           mode == 0 ? "hipStreamSynchronize" : mode == 1 ? "spin hipStreamQuery" : "spin on mapped flag",
           us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10]);
  }
  return 0;
}
