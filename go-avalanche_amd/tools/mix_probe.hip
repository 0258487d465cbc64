// Stream + gather mix of the 8-way target shard round (diagnostics only):
// 4M lanes, each reads 68 B of state (4 x dwordx4 + 1 dword) and writes them
// back, and gathers 8 peer words. Variants of the gather:
//   row16 : the node-major layout — a node's 4 lanes read one random 16-B row
//           of a 16 MB table (1M rows), coalesced into one request per row;
//   col4  : column-major layout with XCD-partitioned columns — every lane reads
//           a random 4-B word of a 4 MB column (the one its XCD owns);
//   none  : no gather (stream only);   gather : gathers only (row16 / col4).
//   mix_probe [lanes=4194304]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// MODE 0 none, 1 row16, 2 col4; STREAM: do the state stream
template <int MODE, bool STREAM>
__global__ __launch_bounds__(256) void k_mix(u32x4* state, uint32_t* table, uint32_t lanes, uint32_t salt,
                                             uint32_t* sink) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  if (g >= lanes) return;
  const uint32_t tile = g >> 6, l = g & 63u;
  u32x4* tp = state + (size_t)tile * (25u * 64u / 4u);  // the engine tile: 6400 B per 64 lanes
  u32x4 a, b, c, d;
  uint32_t e = 0;
  if (STREAM) {
    a = __builtin_nontemporal_load(tp + l);
    b = __builtin_nontemporal_load(tp + 64 + l);
    c = __builtin_nontemporal_load(tp + 128 + l);
    d = __builtin_nontemporal_load(tp + 192 + l);
    e = __builtin_nontemporal_load(reinterpret_cast<uint32_t*>(tp + 256) + l);
  }
  uint32_t acc = 0;
  if (MODE == 1) {  // node = g >> 2, word = g & 3
    const uint32_t node = g >> 2;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t peer = mix(node * 8u + j + salt) & ((1u << 20) - 1u);
      acc ^= table[peer * 4u + (g & 3u)];
    }
  } else if (MODE == 2) {  // column of 1M words, 4 MB
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t peer = mix(g * 8u + j + salt) & ((1u << 20) - 1u);
      acc ^= table[peer];
    }
  }
  if (STREAM) {
    a.x ^= acc ^ salt;
    __builtin_nontemporal_store(a, tp + l);
    __builtin_nontemporal_store(b, tp + 64 + l);
    __builtin_nontemporal_store(c, tp + 128 + l);
    __builtin_nontemporal_store(d, tp + 192 + l);
    __builtin_nontemporal_store(e, reinterpret_cast<uint32_t*>(tp + 256) + l);
  } else if (acc == 0x9e3779b9u) {
    sink[0] = acc;
  }
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
  const uint32_t lanes = argc > 1 ? (uint32_t)std::atol(argv[1]) : (4u << 20);
  u32x4* state;
  uint32_t *table, *sink;
  CK(hipMalloc(&state, (size_t)(lanes / 64 + 1) * 25 * 64 * 4));
  CK(hipMalloc(&table, (size_t)16 << 20));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(state, 1, (size_t)(lanes / 64 + 1) * 25 * 64 * 4));
  CK(hipMemset(table, 3, (size_t)16 << 20));
  const dim3 grid((lanes + 255) / 256);
  uint32_t salt = 7;
  std::printf("{\"lanes\": %u, \"results\": {\n", lanes);
#define RUN(NAME, MODE, STREAM, LAST)                                                                       \
  {                                                                                                         \
    float ms = time_it([&] { hipLaunchKernelGGL((k_mix<MODE, STREAM>), grid, dim3(256), 0, 0, state, table, \
                                                lanes, salt++, sink); },                                    \
                       20);                                                                                 \
    std::printf("  \"%s\": %.4f%s\n", NAME, ms, LAST ? "" : ",");                                          \
  }
  RUN("stream_only", 0, true, false)
  RUN("gather_row16_only", 1, false, false)
  RUN("gather_col4_only", 2, false, false)
  RUN("stream_row16", 1, true, false)
  RUN("stream_col4", 2, true, true)
  std::printf("}}\n");
  return 0;
}
