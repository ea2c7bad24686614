// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access patterns of
// k_hess (MI355X_MICROARCH.md, HBM: "FETCH_SIZE reports exactly 1/2 of the bytes
// of a wide coalesced streaming read ... other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern"). Each kernel
// reads (or writes) a known number of bytes in one of k_hess's patterns, once,
// from a buffer far larger than the L2s, after a flush kernel; run under
//   rocprofv3 --kernel-trace --pmc FETCH_SIZE -- ./traffic_probe
//   rocprofv3 --kernel-trace --pmc WRITE_SIZE -- ./traffic_probe
// and divide the counter by the bytes printed per kernel (scripts/probe/
// traffic_calib.py). Diagnostic only: not part of libkmx.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <numeric>
#include <random>
#include <vector>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

// 16 B per lane, contiguous: the guide's calibrated pattern (expect 1/2)
__global__ void k_stream16(const double2* a, size_t n, double* sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) sink[0] = s;
}
// k_hess records: lane per 80-B record, five 16-B loads
__global__ void k_rec80(const double2* a, size_t nrec, double* sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const double2 v = a[5 * i + k];
      s += v.x + v.y;
    }
  }
  if (s == 1.2345) sink[0] = s;
}
// k_hess own rows: lane (pose, row a) reads 32 B (two 16-B loads) at
// pose * 160 + 32 a; 12 poses (60 lanes) per wave
__global__ void k_rows32(const double2* a, size_t nposes, double* sink) {
  const int ln = threadIdx.x & 63, pw = ln / 5, r = ln - 5 * pw;
  double s = 0.0;
  if (pw < 12) {
    const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
    for (size_t w = blockIdx.x * (size_t)(blockDim.x / 64) + (threadIdx.x >> 6); w * 12 < nposes; w += waves) {
      const size_t p = w * 12 + pw;
      if (p >= nposes) break;
      const double2 v0 = a[p * 10 + 2 * r], v1 = a[p * 10 + 2 * r + 1];
      s += v0.x + v0.y + v1.x + v1.y;
    }
  }
  if (s == 1.2345) sink[0] = s;
}
// k_hess neighbour gathers: lane reads one whole 160-B row (ten 16-B loads)
// of a random pose (a permutation: every row once)
__global__ void k_gather160(const double2* a, const int* perm, size_t nposes, double* sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nposes; i += (size_t)gridDim.x * blockDim.x) {
    const size_t p = perm[i];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const double2 v = a[p * 10 + k];
      s += v.x + v.y;
    }
  }
  if (s == 1.2345) sink[0] = s;
}
// S / D / Pinv blocks: lane per pose reads W doubles at stride W (W/2 16-B loads)
template <int W>
__global__ void k_blockW(const double2* a, size_t nposes, double* sink) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nposes; i += (size_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int k = 0; k < W / 2; ++k) {
      const double2 v = a[(W / 2) * i + k];
      s += v.x + v.y;
    }
  }
  if (s == 1.2345) sink[0] = s;
}
// k_hess stores: lane (pose, row a) writes 32 B
__global__ void k_store32(double2* a, size_t nposes) {
  const int ln = threadIdx.x & 63, pw = ln / 5, r = ln - 5 * pw;
  if (pw >= 12) return;
  const size_t waves = (size_t)gridDim.x * (blockDim.x / 64);
  for (size_t w = blockIdx.x * (size_t)(blockDim.x / 64) + (threadIdx.x >> 6); w * 12 < nposes; w += waves) {
    const size_t p = w * 12 + pw;
    if (p >= nposes) break;
    a[p * 10 + 2 * r] = make_double2((double)p, 1.0);
    a[p * 10 + 2 * r + 1] = make_double2(2.0, (double)r);
  }
}
__global__ void k_store16(double2* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2((double)i, 1.0);
}
// evicts the L2s between the probes (streams 512 MB)
__global__ void k_flush(double2* a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i].x += 1.0;
}

int main() {
  const size_t bytes = 192ull << 20;  // per probe: past the 32 MB of L2s
  const size_t n16 = bytes / 16;
  double2 *a, *fl;
  double* sink;
  int* perm;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&fl, 512ull << 20));
  CK(hipMalloc(&sink, 8));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(fl, 0, 512ull << 20));
  const size_t nposes = bytes / 160;
  std::vector<int> hp(nposes);
  std::iota(hp.begin(), hp.end(), 0);
  std::shuffle(hp.begin(), hp.end(), std::mt19937(1));
  CK(hipMalloc(&perm, sizeof(int) * nposes));
  CK(hipMemcpy(perm, hp.data(), sizeof(int) * nposes, hipMemcpyHostToDevice));
  const dim3 G(4096), B(256);
  auto flush = [&] { hipLaunchKernelGGL(k_flush, G, B, 0, 0, fl, (512ull << 20) / 16); };
  struct P { const char* name; size_t bytes; };
  std::vector<P> probes;
  for (int rep = 0; rep < 2; ++rep) {
    flush();
    hipLaunchKernelGGL(k_stream16, G, B, 0, 0, a, n16, sink);
    probes.push_back({"k_stream16", n16 * 16});
    flush();
    hipLaunchKernelGGL(k_rec80, G, B, 0, 0, a, bytes / 80, sink);
    probes.push_back({"k_rec80", bytes / 80 * 80});
    flush();
    hipLaunchKernelGGL(k_rows32, G, B, 0, 0, a, nposes, sink);
    probes.push_back({"k_rows32", nposes * 160});
    flush();
    hipLaunchKernelGGL(k_gather160, G, B, 0, 0, a, perm, nposes, sink);
    probes.push_back({"k_gather160", nposes * 160});
    flush();
    hipLaunchKernelGGL(k_blockW<6>, G, B, 0, 0, a, bytes / 48, sink);
    probes.push_back({"k_blockW<6>", bytes / 48 * 48});
    flush();
    hipLaunchKernelGGL(k_blockW<10>, G, B, 0, 0, a, bytes / 80, sink);
    probes.push_back({"k_blockW<10>", bytes / 80 * 80});
    flush();
    hipLaunchKernelGGL(k_store32, G, B, 0, 0, a, nposes);
    probes.push_back({"k_store32", nposes * 160});
    flush();
    hipLaunchKernelGGL(k_store16, G, B, 0, 0, a, n16);
    probes.push_back({"k_store16", n16 * 16});
  }
  CK(hipDeviceSynchronize());
  for (const auto& p : probes) std::printf("%s %zu\n", p.name, p.bytes);
  return 0;
}
