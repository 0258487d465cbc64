// StatusUpdate delivery on the device (processor.go:111's *[]StatusUpdate
// out-parameter): the round kernels leave their updates in a sharded log of
// single packed words and dense lane records (kernels.h); these kernels
//  * expand the dense records into packed words (A after slot j = the final
//    A plane ^ parity of the later slots' updates; vote.go:77-91 statuses),
//  * put the singles and the expanded words into the canonical (round, node,
//    slot, target) order with a device radix sort (rocPRIM via hipCUB) — the
//    packed word sorts exactly in that order (include/avhip.h),
//  * or reduce them to an order-independent digest (count, sum and xor of
//    splitmix64(word)) that the oracle computes the same way
//    (oracle/avalanche_oracle.c avo_mix64), for full-size parity checks that
//    do not copy billions of updates to the host.
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kernels.h"
#include "round_common.h"

namespace avk {
namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t wave_add64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
  return v;
}
__device__ __forceinline__ uint64_t wave_xor64(uint64_t v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v ^= (uint64_t)__shfl_xor((unsigned long long)v, d, 64);
  return v;
}

// Words of one dense record (kernels.h): w[0..1] key, w[2..1+K] E_j, w[2+K]
// final A plane, w[3+K] died. Calls f(word) for each of its updates.
template <typename F>
__device__ __forceinline__ void for_each_dense(const uint32_t* w, uint32_t K, F&& f) {
  const uint64_t key = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint32_t A = w[2 + K], died = w[3 + K];
  uint32_t par = 0u;
  for (int j = (int)K - 1; j >= 0; --j) {
    const uint32_t aj = A ^ par;
    const uint32_t e = w[2 + j];
    par ^= e;
    for (uint32_t em = e; em; em &= em - 1u) {
      const uint32_t bit = (uint32_t)__builtin_ctz(em);
      const uint64_t a = (aj >> bit) & 1u;
      const uint64_t st = ((died >> bit) & 1u) ? (a ? 3u : 0u) : (a ? 2u : 1u);  // vote.go:77-91
      f(key + ((uint64_t)j << 24) + ((uint64_t)bit << 2) + st);
    }
  }
}

// Medium record (kernels.h). Slot record (AVK_MED_S4): the dense expansion over the slots its mask
// names (A after slot j = A ^ parity of the later slots' updates); folded record: {key, payload}.
template <typename F>
__device__ __forceinline__ void for_each_med(const uint64_t* rec, F&& f) {
#if AVK_MED_S4
  const uint32_t* w = reinterpret_cast<const uint32_t*>(rec);
  const uint64_t key = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint32_t S = w[2], A = w[3];
  const uint32_t nw = (S & kMedS4Died) ? 3u : 4u;
  const uint32_t died = (S & kMedS4Died) ? w[7] : 0u;
  uint32_t slot[4], n = 0;
  for (uint32_t m = S & 0xFFu; m && n < nw; m &= m - 1u) slot[n++] = (uint32_t)__builtin_ctz(m);
  uint32_t par = 0u;
  for (int i = (int)n - 1; i >= 0; --i) {
    const uint32_t aj = A ^ par, e = w[4 + i];
    par ^= e;
    for (uint32_t em = e; em; em &= em - 1u) {
      const uint32_t bit = (uint32_t)__builtin_ctz(em);
      const uint64_t a = (aj >> bit) & 1u;
      const uint64_t st = ((died >> bit) & 1u) ? (a ? 3u : 0u) : (a ? 2u : 1u);  // vote.go:77-91
      f(key + ((uint64_t)slot[i] << 24) + ((uint64_t)bit << 2) + st);
    }
  }
#else
  const uint64_t key = rec[0], pl = rec[1];
  const uint32_t n = (uint32_t)(pl & 15u);
  for (uint32_t i = 0; i < n && i < kMedMax; ++i) f(med_word(key, (uint32_t)(pl >> (4u + 10u * i)) & 1023u));
#endif
}

// u64 words of one record: dense (k >= 1) or medium (kMedKind)
__host__ __device__ constexpr uint32_t rec_words(uint32_t K) { return K == kMedKind ? med_rec_words() : dense_words(K); }

template <typename F>
__device__ __forceinline__ void for_each_rec(const uint64_t* rec, uint32_t K, F&& f) {
  if (K == kMedKind)
    for_each_med(rec, f);
  else
    for_each_dense(reinterpret_cast<const uint32_t*>(rec), K, f);
}

__device__ __forceinline__ bool in_nodes(uint64_t w, uint32_t node0, uint32_t node1) {
  const uint32_t node = (uint32_t)(w >> 28) & 0xFFFFFFu;
  return node >= node0 && node < node1;
}

// Digest of every pending update of nodes [node0, node1): blockIdx.y = shard;
// the x-blocks stride over the shard's singles, then over its dense records.
__global__ __launch_bounds__(256) void k_log_digest(const uint64_t* log, const uint32_t* counts, uint32_t cap,
                                                    const uint64_t* dlog, const uint32_t* dcounts, uint32_t dcap,
                                                    const uint64_t* mlog, const uint32_t* mcounts, uint32_t mcap,
                                                    uint32_t K, uint32_t node0, uint32_t node1,
                                                    unsigned long long* out) {
  const uint32_t shard = blockIdx.y;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t s = 0, x = 0, c = 0;
  const uint32_t n = min(counts[shard * kCtrStride], cap);
  const uint64_t* src = log + (size_t)shard * cap;
  for (uint32_t i = t; i < n; i += stride) {
    const uint64_t w = src[i];
    if (!in_nodes(w, node0, node1)) continue;
    const uint64_t h = mix64(w);
    s += h;
    x ^= h;
    ++c;
  }
  const uint32_t DW = dense_words(K);
  const uint32_t nd = min(dcounts[shard * kCtrStride], dcap);
  const uint64_t* dsrc = dlog + (size_t)shard * dcap * DW;
  for (uint32_t i = t; i < nd; i += stride) {
    const uint32_t* rw = reinterpret_cast<const uint32_t*>(dsrc + (size_t)i * DW);
    if (!in_nodes((uint64_t)rw[0] | ((uint64_t)rw[1] << 32), node0, node1)) continue;
    for_each_dense(reinterpret_cast<const uint32_t*>(dsrc + (size_t)i * DW), K, [&](uint64_t wd) {
      const uint64_t h = mix64(wd);
      s += h;
      x ^= h;
      ++c;
    });
  }
  const uint32_t nm = mlog ? min(mcounts[shard * kCtrStride], mcap) : 0u;
  constexpr uint32_t MW = med_rec_words();
  const uint64_t* msrc = mlog + (size_t)shard * mcap * MW;
  for (uint32_t i = t; i < nm; i += stride) {
    if (!in_nodes(msrc[MW * i], node0, node1)) continue;
    for_each_med(msrc + MW * i, [&](uint64_t wd) {
      const uint64_t h = mix64(wd);
      s += h;
      x ^= h;
      ++c;
    });
  }
  c = wave_add64(c);
  s = wave_add64(s);
  x = wave_xor64(x);
  if ((threadIdx.x & 63u) == 0 && c) {
    atomicAdd(&out[0], (unsigned long long)c);
    atomicAdd(&out[1], (unsigned long long)s);
    atomicXor(&out[2], (unsigned long long)x);
  }
}

// Updates held by each dense record (popcount of its E_j) or medium record (its n).
__global__ __launch_bounds__(256) void k_dense_counts(const uint64_t* recs, uint64_t n, uint32_t K, uint64_t* cnt) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (K == kMedKind) {
#if AVK_MED_S4
    const uint32_t* w = reinterpret_cast<const uint32_t*>(recs + i * med_rec_words());
    const uint32_t nw = (w[2] & kMedS4Died) ? 3u : 4u;
    uint32_t c = 0;
    for (uint32_t j = 0; j < nw; ++j) c += (uint32_t)__popc(w[4 + j]);
    cnt[i] = c;
#else
    cnt[i] = min((uint32_t)(recs[2u * i + 1u] & 15u), kMedMax);
#endif
    return;
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(recs + i * dense_words(K));
  uint32_t c = 0;
  for (uint32_t j = 0; j < K; ++j) c += (uint32_t)__popc(w[2 + j]);
  cnt[i] = c;
}

// Expand record i at out[off[i] ...] (off: exclusive scan of k_dense_counts).
__global__ __launch_bounds__(256) void k_dense_expand(const uint64_t* recs, uint64_t n, uint32_t K,
                                                      const uint64_t* off, uint64_t* out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t* dst = out + off[i];
  for_each_rec(recs + i * rec_words(K), K, [&](uint64_t wd) { *dst++ = wd; });
}

}  // namespace

hipError_t launch_log_digest(const uint64_t* log, const uint32_t* counts, uint32_t cap, const uint64_t* dlog,
                             const uint32_t* dcounts, uint32_t dcap, const uint64_t* mlog, const uint32_t* mcounts,
                             uint32_t mcap, uint32_t shards, uint32_t k, uint32_t node0, uint32_t node1,
                             unsigned long long* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, 3 * sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_log_digest, dim3(16, shards), dim3(256), 0, s, log, counts, cap, dlog, dcounts, dcap, mlog,
                     mcounts, mcap, k, node0, node1, out);
  return hipGetLastError();
}

hipError_t launch_dense_expand(const uint64_t* recs, uint64_t n, uint32_t k, uint64_t* counts_scratch,
                               uint64_t* offsets, void* temp, size_t* temp_bytes, uint64_t* out, hipStream_t s) {
  if (!temp) {  // size query for the scan
    return hipcub::DeviceScan::ExclusiveSum(nullptr, *temp_bytes, counts_scratch, offsets, n, s);
  }
  if (!n) return hipSuccess;
  const uint64_t blocks = (n + 255) / 256;
  hipLaunchKernelGGL(k_dense_counts, dim3((uint32_t)blocks), dim3(256), 0, s, recs, n, k, counts_scratch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, counts_scratch, offsets, n, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_dense_expand, dim3((uint32_t)blocks), dim3(256), 0, s, recs, n, k, offsets, out);
  return hipGetLastError();
}

hipError_t launch_sort_updates(void* temp, size_t* temp_bytes, const uint64_t* in, uint64_t* out, uint64_t n,
                               int begin_bit, int end_bit, hipStream_t s) {
  return hipcub::DeviceRadixSort::SortKeys(temp, *temp_bytes, in, out, n, begin_bit, end_bit, s);
}

namespace {
__global__ __launch_bounds__(256) void k_iota(uint32_t* out, uint32_t n) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i < n) out[i] = i;
}
// entries[2i] = vote index, entries[2i+1] = packed vote (k_register_votes)
__global__ __launch_bounds__(256) void k_vote_entries(const uint32_t* perm, const uint32_t* vidx, const uint32_t* info,
                                                      uint32_t n, uint32_t* entries) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  const uint32_t j = perm[i];
  entries[2u * i] = vidx[j];
  entries[2u * i + 1u] = info[j];
}
}  // namespace

// Drop-in RegisterVotes batch (engine.cpp av_register_votes_batch): group the
// votes by lane (node, 32-target block) keeping their order inside a lane —
// a stable radix sort of (lane, position) pairs — then run-length encode the
// sorted lanes into the (lanes, offs) CSR k_register_votes walks. temp ==
// nullptr: *temp_bytes = the scratch the three hipcub passes need.
hipError_t launch_group_votes(void* temp, size_t* temp_bytes, const uint32_t* keys, const uint32_t* vidx,
                              const uint32_t* info, uint32_t n, int key_bits, uint32_t* keys_s, uint32_t* perm,
                              uint32_t* perm_s, uint32_t* lanes, uint32_t* counts, uint32_t* offs, uint32_t* n_runs,
                              uint32_t* entries, hipStream_t s) {
  size_t b_sort = 0, b_rle = 0, b_scan = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b_sort, keys, keys_s, perm, perm_s, n, 0, key_bits, s);
  if (e == hipSuccess) e = hipcub::DeviceRunLengthEncode::Encode(nullptr, b_rle, keys_s, lanes, counts, n_runs, n, s);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, b_scan, counts, offs, n + 1u, s);
  if (e != hipSuccess) return e;
  const size_t need = std::max(b_sort, std::max(b_rle, b_scan));
  if (!temp) {
    *temp_bytes = need;
    return hipSuccess;
  }
  if (*temp_bytes < need) return hipErrorInvalidValue;
  const uint32_t g = (n + 255u) / 256u;
  hipLaunchKernelGGL(k_iota, dim3(g), dim3(256), 0, s, perm, n);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  size_t t = need;
  if ((e = hipcub::DeviceRadixSort::SortPairs(temp, t, keys, keys_s, perm, perm_s, n, 0, key_bits, s)) != hipSuccess) return e;
  // counts has n + 1 slots: the runs' counts, then zeros, so that the scan's
  // entry n_runs is the total (offs[n_runs] = n)
  if ((e = hipMemsetAsync(counts, 0, (size_t)(n + 1u) * 4, s)) != hipSuccess) return e;
  t = need;
  if ((e = hipcub::DeviceRunLengthEncode::Encode(temp, t, keys_s, lanes, counts, n_runs, n, s)) != hipSuccess) return e;
  t = need;
  if ((e = hipcub::DeviceScan::ExclusiveSum(temp, t, counts, offs, n + 1u, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_vote_entries, dim3(g), dim3(256), 0, s, perm_s, vidx, info, n, entries);
  return hipGetLastError();
}

}  // namespace avk
