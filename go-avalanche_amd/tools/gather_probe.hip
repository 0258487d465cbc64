// Random-row gather floor on MI355X: how fast can one GPU read R uniformly
// random rows of W bytes from a table of N rows (the peer-preference gather
// of the round kernel: N = 1M nodes, R = N * k = 8M rows per round, W = 4 * BL
// = 128 B at 1 GPU ... 16 B at 8-way target sharding)? Diagnostics only.
//   gather_probe [rows_log2=20] [reads=8388608]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// LPR lanes per row (row = LPR dwords), 8 independent reads per lane in flight.
template <int LPR>
__global__ __launch_bounds__(256) void k_gather(const uint32_t* __restrict__ table, uint32_t rows, uint32_t reads,
                                                uint32_t salt, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const uint32_t row_slot = t / LPR, word = t % LPR;
  if (row_slot * 8u >= reads) return;
  uint32_t acc = 0;
  uint32_t v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t r = __umulhi(mix(row_slot * 8u + (uint32_t)j + salt), rows);
    v[j] = table[(size_t)r * LPR + word];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += v[j];
  if (acc == 0x12345678u) out[0] = acc;
}

// dwordx4 per lane: one lane reads a 16-byte row
__global__ __launch_bounds__(256) void k_gather16(const uint4* __restrict__ table, uint32_t rows, uint32_t reads,
                                                  uint32_t salt, uint32_t* out) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t * 8u >= reads) return;
  uint32_t acc = 0;
  uint4 v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t r = __umulhi(mix(t * 8u + (uint32_t)j + salt), rows);
    v[j] = table[r];
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) acc += v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float time_it(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int rows_log2 = argc > 1 ? std::atoi(argv[1]) : 20;
  const uint32_t reads = argc > 2 ? (uint32_t)std::atol(argv[2]) : 8u << 20;
  const uint32_t rows = 1u << rows_log2;
  uint32_t *table, *out;
  CK(hipMalloc(&table, (size_t)rows * 128));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(table, 1, (size_t)rows * 128));
  const int reps = 20;
  std::printf("{\"rows\": %u, \"reads\": %u, \"results\": [\n", rows, reads);
  auto line = [&](const char* name, int bytes, float ms, bool last) {
    std::printf("  {\"form\": \"%s\", \"row_bytes\": %d, \"ms\": %.4f, \"Grows_per_s\": %.2f, \"useful_GBs\": %.1f}%s\n",
                name, bytes, ms, reads / (ms * 1e-3) / 1e9, (double)reads * bytes / (ms * 1e-3) / 1e9,
                last ? "" : ",");
  };
  uint32_t salt = 1;
#define RUN_LPR(L)                                                                                   \
  {                                                                                                  \
    const uint32_t threads = (reads / 8u) * (L);                                                     \
    float ms = time_it(                                                                              \
        [&] {                                                                                        \
          hipLaunchKernelGGL(k_gather<L>, dim3((threads + 255) / 256), dim3(256), 0, 0, table, rows, \
                             reads, salt++, out);                                                    \
        },                                                                                           \
        reps);                                                                                       \
    line("dword_lanes_per_row_" #L, 4 * (L), ms, false);                                             \
  }
  RUN_LPR(1)
  RUN_LPR(4)
  RUN_LPR(8)
  RUN_LPR(32)
  {
    const uint32_t threads = reads / 8u;
    float ms = time_it(
        [&] {
          hipLaunchKernelGGL(k_gather16, dim3((threads + 255) / 256), dim3(256), 0, 0,
                             reinterpret_cast<const uint4*>(table), rows, reads, salt++, out);
        },
        reps);
    line("dwordx4_one_lane_per_row", 16, ms, true);
  }
  std::printf("]}\n");
  CK(hipFree(table));
  CK(hipFree(out));
  return 0;
}
