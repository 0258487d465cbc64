// pmc_calib — known-byte-count kernels for calibrating rocprofv3 FETCH_SIZE /
// WRITE_SIZE on gfx950 per access width (MI355X_MICROARCH.md §HBM: FETCH_SIZE
// reads 1/2 of a 16 B/lane stream; other widths must be calibrated on a known
// byte count). Each kernel moves exactly `bytes` once, coalesced, far beyond
// the 256 MiB Infinity Cache; the sums are written to a sink so nothing is
// optimised away.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ void calib_read_dwordx4(const u32x4* __restrict__ a, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void calib_read_dword(const unsigned* __restrict__ a, size_t n, unsigned* sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= a[i];
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ void calib_write_dwordx4(u32x4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

__global__ void calib_write_dword(unsigned* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (unsigned)i;
}

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 1;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char** argv) {
  const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1ull << 30);
  void* buf = nullptr;
  unsigned* sink = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 4));
  CHECK(hipMemset(buf, 1, bytes));
  const dim3 grid(4096), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(calib_read_dwordx4, grid, block, 0, 0, (const u32x4*)buf, bytes / 16, sink);
    hipLaunchKernelGGL(calib_read_dword, grid, block, 0, 0, (const unsigned*)buf, bytes / 4, sink);
    hipLaunchKernelGGL(calib_write_dwordx4, grid, block, 0, 0, (u32x4*)buf, bytes / 16);
    hipLaunchKernelGGL(calib_write_dword, grid, block, 0, 0, (unsigned*)buf, bytes / 4);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("pmc_calib: each kernel moved %zu bytes\n", bytes);
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
