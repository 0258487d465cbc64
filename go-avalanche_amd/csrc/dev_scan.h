// Hand-written device-wide primitives for CDNA4 (64-lane waves, LDS), used by
// StatusUpdate delivery (log_ops.hip), the batched drop-in RegisterVotes
// grouping and the batched GetInvsForNextPoll (kernels.hip):
//  * launch_scan: exclusive prefix sum of n values into u64 out[0..n], out[n] =
//    the total. Reduce-then-scan over tiles of 4096 values (256 threads x 16
//    chunks, striped so every load is coalesced); the tile partials are scanned
//    by the same kernels recursively (in place), so any n runs in
//    2 * ceil(log_4096 n) + 1 launches with no host round trip.
//  * launch_radix_sort_pairs: stable LSD radix sort of (u32 key, u32 value)
//    pairs, 8 bits per pass: per-tile digit histograms (LDS atomics), one scan
//    of the digit-major histogram table, then a scatter that ranks each chunk of
//    256 items by wave ballots (the lanes holding the same digit: 8 ballots) and
//    per-wave digit counts in LDS, so that equal keys keep their input order.
// Nothing here is a compatibility layer: plain HIP kernels, no library calls.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace avk {
namespace dscan {
namespace {  // internal linkage: every translation unit that includes this gets its own kernels

constexpr uint32_t kThreads = 256;
constexpr uint32_t kChunks = 16;
constexpr uint32_t kTile = kThreads * kChunks;  // values per workgroup

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t t = __shfl_up((unsigned long long)v, (unsigned)d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// Exclusive scan of one value per thread over a 256-thread workgroup; total = the sum of all.
// lds: 4 u64. Every thread of the workgroup must call it (two barriers).
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* lds, uint64_t& total) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan64(v, lane);
  if (lane == 63u) lds[w] = incl;
  __syncthreads();
  uint64_t off = 0, tot = 0;
#pragma unroll
  for (uint32_t q = 0; q < kThreads / 64u; ++q) {
    const uint64_t s = lds[q];
    off += q < w ? s : 0ull;
    tot += s;
  }
  __syncthreads();  // lds is reused by the next call
  total = tot;
  return off + incl - v;
}

// Value sources.
struct In64 {
  const uint64_t* a;
  __device__ uint64_t operator()(uint64_t i) const { return a[i]; }
};
struct In32 {
  const uint32_t* a;
  __device__ uint64_t operator()(uint64_t i) const { return a[i]; }
};

template <class In>
__global__ __launch_bounds__(kThreads) void k_reduce_tiles(In in, uint64_t n, uint64_t* part) {
  __shared__ uint64_t lds[kThreads / 64u];
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint64_t s = 0;
#pragma unroll 4
  for (uint32_t c = 0; c < kChunks; ++c) {
    const uint64_t i = base + c * kThreads + threadIdx.x;
    if (i < n) s += in(i);
  }
  uint64_t tot;
  (void)block_excl_scan64(s, lds, tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// out[i] = (part ? part[tile] : 0) + the exclusive prefix of in within the tile; the last tile also
// writes out[n] = the grand total. In place (in reads the array out writes) is safe: every value is
// read and written by the same thread within one chunk, and a tile touches only its own values.
template <class In>
__global__ __launch_bounds__(kThreads) void k_scan_tiles(In in, uint64_t n, const uint64_t* part, uint64_t* out) {
  __shared__ uint64_t lds[kThreads / 64u];
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  uint64_t carry = part ? part[blockIdx.x] : 0ull;
  for (uint32_t c = 0; c < kChunks; ++c) {
    const uint64_t i = base + c * kThreads + threadIdx.x;
    const uint64_t v = i < n ? in(i) : 0ull;
    uint64_t tot;
    const uint64_t ex = block_excl_scan64(v, lds, tot);
    if (i < n) out[i] = carry + ex;
    carry += tot;
  }
  if (blockIdx.x == gridDim.x - 1u && threadIdx.x == 0) out[n] = carry;
}

// Scratch (u64 words) launch_scan needs for n values.
inline uint64_t scan_scratch_words(uint64_t n) {
  uint64_t w = 1;
  while (n > kTile) {
    n = (n + kTile - 1) / kTile;
    w += n + 1;
  }
  return w;
}

// Exclusive prefix sums of in(0..n) into out[0..n] (n + 1 slots; out[n] = total).
template <class In>
hipError_t launch_scan(In in, uint64_t n, uint64_t* out, uint64_t* scratch, hipStream_t s) {
  if (n <= kTile) {
    hipLaunchKernelGGL(k_scan_tiles<In>, dim3(1), dim3(kThreads), 0, s, in, n, (const uint64_t*)nullptr, out);
    return hipGetLastError();
  }
  const uint64_t nb = (n + kTile - 1) / kTile;
  if (nb > 0x7FFFFFFFull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_reduce_tiles<In>, dim3((uint32_t)nb), dim3(kThreads), 0, s, in, n, scratch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_scan(In64{scratch}, nb, scratch, scratch + nb + 1, s);  // the partials, in place
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_scan_tiles<In>, dim3((uint32_t)nb), dim3(kThreads), 0, s, in, n, (const uint64_t*)scratch,
                     out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Stable LSD radix sort of (u32 key, u32 value) pairs.
// ---------------------------------------------------------------------------
constexpr uint32_t kRadix = 256;

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// hist[d * n_tiles + t] = items of tile t whose digit is d
__global__ __launch_bounds__(kThreads) void k_radix_hist(const uint32_t* keys, uint32_t n, uint32_t shift,
                                                         uint32_t n_tiles, uint64_t* hist) {
  __shared__ uint32_t h[kRadix];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  for (uint32_t c = 0; c < kChunks; ++c) {
    const uint64_t i = base + c * kThreads + threadIdx.x;
    if (i < n) atomicAdd(&h[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * n_tiles + blockIdx.x] = h[threadIdx.x];
}

// Scatter tile t's items to off[d * n_tiles + t] + (their rank among the digit-d items of the tile,
// in input order). vin == nullptr: the values are the input positions.
__global__ __launch_bounds__(kThreads) void k_radix_scatter(const uint32_t* kin, const uint32_t* vin, uint32_t n,
                                                            uint32_t shift, uint32_t n_tiles, const uint64_t* off,
                                                            uint32_t* kout, uint32_t* vout) {
  __shared__ uint32_t base[kRadix];
  __shared__ uint32_t wcnt[kThreads / 64u][kRadix];
  const uint32_t tid = threadIdx.x, w = tid >> 6;
  base[tid] = (uint32_t)off[(uint64_t)tid * n_tiles + blockIdx.x];
#pragma unroll
  for (uint32_t q = 0; q < kThreads / 64u; ++q) wcnt[q][tid] = 0u;
  __syncthreads();
  const uint64_t tbase = (uint64_t)blockIdx.x * kTile;
  for (uint32_t c = 0; c < kChunks; ++c) {
    const uint64_t i = tbase + c * kThreads + tid;
    const bool ok = i < n;
    const uint32_t key = ok ? kin[i] : 0u;
    const uint32_t val = ok ? (vin ? vin[i] : (uint32_t)i) : 0u;
    const uint32_t d = (key >> shift) & 255u;
    // the lanes of this wave holding digit d
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (uint32_t b = 0; b < 8u; ++b) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint32_t wr = lanes_below(peers);
    if (ok && wr == 0u) wcnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (ok) {
      uint32_t pos = base[d] + wr;
      for (uint32_t q = 0; q < w; ++q) pos += wcnt[q][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    uint32_t add = 0;
#pragma unroll
    for (uint32_t q = 0; q < kThreads / 64u; ++q) {
      add += wcnt[q][tid];
      wcnt[q][tid] = 0u;
    }
    base[tid] += add;
    __syncthreads();
  }
}

inline uint32_t radix_tiles(uint32_t n) { return (n + kTile - 1) / kTile; }
// Scratch (u64 words) of launch_radix_sort_pairs.
inline uint64_t radix_scratch_words(uint32_t n) {
  const uint64_t h = (uint64_t)kRadix * radix_tiles(n);
  return h + 1 + scan_scratch_words(h);
}

// Sort n pairs on key bits [0, key_bits) into (k0, v0). The passes alternate between the buffer sets
// (k0, v0) and (k1, v1), starting with the one that makes the last pass write (k0, v0); the first pass
// reads (kin, vin) (vin == nullptr: the values are the input positions), which must not alias any of
// the four buffers.
inline hipError_t launch_radix_sort_pairs(const uint32_t* kin, const uint32_t* vin, uint32_t n, int key_bits,
                                          uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1,
                                          uint64_t* scratch, hipStream_t s) {
  const uint32_t tiles = radix_tiles(n);
  const uint64_t h = (uint64_t)kRadix * tiles;
  uint64_t* hist = scratch;
  uint64_t* sc = scratch + h + 1;
  const int passes = key_bits <= 0 ? 1 : (key_bits + 7) / 8;
  const uint32_t* ki = kin;
  const uint32_t* vi = vin;
  int set = (passes - 1) % 2;  // pass p writes set ^ (p % 2): the last one set 0
  hipError_t e = hipSuccess;
  for (int p = 0; p < passes; ++p) {
    if (n == 0) break;
    uint32_t* ko = set == 0 ? k0 : k1;
    uint32_t* vo = set == 0 ? v0 : v1;
    hipLaunchKernelGGL(k_radix_hist, dim3(tiles), dim3(kThreads), 0, s, ki, n, (uint32_t)(8 * p), tiles, hist);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = launch_scan(In64{hist}, h, hist, sc, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_radix_scatter, dim3(tiles), dim3(kThreads), 0, s, ki, vi, n, (uint32_t)(8 * p), tiles,
                       (const uint64_t*)hist, ko, vo);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    ki = ko;
    vi = vo;
    set ^= 1;
  }
  return hipSuccess;
}

}  // namespace
}  // namespace dscan
}  // namespace avk
