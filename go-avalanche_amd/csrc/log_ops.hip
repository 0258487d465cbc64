// StatusUpdate delivery on the device (processor.go:61,111's *[]StatusUpdate
// out-parameter, appended in vote order, processor.go:94). The round kernels
// leave a round's updates in a sharded log of single packed words, slot records
// and dense lane records (kernels.h); a lane's updates of one round are in one
// record kind. These kernels
//  * put every pending update into the canonical (round, node, slot, target)
//    order — the reference's append order under rule R1 —
//    with a counting sort keyed by (round, node): the key range is known from
//    the log layout (rounds since the last fetch x local nodes), so one pass
//    counts each bucket's entries and updates (wave-aggregated atomics), a
//    device scan (dev_scan.h) turns the counts into offsets, a scatter groups
//    the entries by bucket, and one wave per bucket lays its updates out in
//    (slot, target) order through a per-bucket table of (slot, 32-target
//    block) cells in LDS: the cells' prefix counts give every update's position
//    directly, so nothing is sorted by comparison and every output store is
//    coalesced;
//  * write them either as packed 8-byte words (av_fetch_updates) or as the
//    compact stream (av_fetch_compact*: per (round, node) group a node id and
//    a count, then 2 bytes per update when slot, local target and status fit);
//  * or reduce them to an order-independent digest (count, sum and xor of
//    splitmix64(word)) that the oracle computes the same way
//    (oracle/avalanche_oracle.c avo_mix64), for full-size parity checks that
//    do not copy billions of updates to the host.
// The drop-in RegisterVotes batch groups its votes by lane with the stable
// radix sort of dev_scan.h (launch_group_votes). No library sort or scan.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_scan.h"
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

// node field of an update word: bits [28, round_shift)
__device__ __forceinline__ uint32_t word_node(uint64_t w, uint32_t round_shift) {
  return (uint32_t)((w >> 28) & ((1ull << (round_shift - 28u)) - 1ull));
}
__device__ __forceinline__ bool in_nodes(uint64_t w, uint32_t node0, uint32_t node1, uint32_t round_shift) {
  const uint32_t node = word_node(w, round_shift);
  return node >= node0 && node < node1;
}

// Digest of every pending update of nodes [node0, node1): blockIdx.y = shard;
// the x-blocks stride over the shard's singles, then over its dense records.
__global__ __launch_bounds__(256) void k_log_digest(const uint64_t* log, const uint32_t* counts, uint32_t cap,
                                                    const uint64_t* dlog, const uint32_t* dcounts, uint32_t dcap,
                                                    const uint64_t* mlog, const uint32_t* mcounts, uint32_t mcap,
                                                    uint32_t K, uint32_t node0, uint32_t node1,
                                                    uint32_t rs, unsigned long long* out) {
  const uint32_t shard = blockIdx.y;
  const uint32_t stride = gridDim.x * blockDim.x;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t s = 0, x = 0, c = 0;
  const uint32_t n = min(counts[shard * kCtrStride], cap);
  const uint64_t* src = log + (size_t)shard * cap;
  for (uint32_t i = t; i < n; i += stride) {
    const uint64_t w = src[i];
    if (!in_nodes(w, node0, node1, rs)) continue;
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
    if (!in_nodes((uint64_t)rw[0] | ((uint64_t)rw[1] << 32), node0, node1, rs)) continue;
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
    if (!in_nodes(msrc[MW * i], node0, node1, rs)) continue;
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

// ---------------------------------------------------------------------------
// Canonical order by (round, node) buckets.
// ---------------------------------------------------------------------------
// Flat entry index f: the log's entries kind by kind (singles, slot records, dense records), shard by
// shard, each shard's first min(count, cap) entries. flat[kind * shards + shard] = the first f of that
// shard (dscan over the counters), flat[3 * shards] = the total.
struct FlatIn {
  const uint32_t* counts;  // [3][kLogShards][kCtrStride]
  uint32_t shards, cap0, cap1, cap2;
  __device__ uint64_t operator()(uint64_t i) const {
    const uint32_t kind = (uint32_t)(i / shards), shard = (uint32_t)(i - (uint64_t)kind * shards);
    const uint32_t cap = kind == 0 ? cap0 : kind == 1 ? cap1 : cap2;
    return min(counts[((size_t)kind * kLogShards + shard) * kCtrStride], cap);
  }
};

constexpr uint64_t kInvalid64 = ~0ull;
constexpr uint32_t kCntShift = 40;  // cnt64[b] = entries << 40 | updates
constexpr uint64_t kUpdMask = (1ull << kCntShift) - 1ull;

struct EncArgs {
  EncodeParams p;
  const uint64_t* flat;  // [3 * shards + 1]
  unsigned long long* cnt;  // [B]
  uint64_t* ekey;        // [entries]: bucket << 32 | rank, or kInvalid64
  uint32_t B;            // buckets of this pass = nr * NL
};

// Locate flat entry f: (kind, address of the entry in its kind's array, in entries).
__device__ __forceinline__ void locate(const uint64_t* flat_lds, uint32_t shards, uint64_t f, uint32_t& kind,
                                       uint64_t& addr, const EncodeParams& p) {
  uint32_t lo = 0, hi = 3u * shards - 1u;  // last slot s with flat[s] <= f
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1u) >> 1;
    if (flat_lds[mid] <= f) lo = mid; else hi = mid - 1u;
  }
  kind = lo / shards;
  const uint32_t shard = lo - kind * shards;
  const uint32_t cap = kind == 0 ? p.log_cap : kind == 1 ? p.mlog_cap : p.dlog_cap;
  addr = (uint64_t)shard * cap + (f - flat_lds[lo]);
}

// An entry's key word (pack_update of its first update or of its block) and number of updates.
__device__ __forceinline__ uint64_t entry_key(const EncodeParams& p, uint32_t kind, uint64_t addr, uint32_t& nu) {
  if (kind == 0) {
    nu = 1u;
    return p.log[addr];
  }
  if (kind == 1) {
    constexpr uint32_t MW = med_rec_words();
#if AVK_MED_S4
    const u32x4* q = reinterpret_cast<const u32x4*>(p.mlog + addr * MW);
    const u32x4 a = q[0], b = q[1];
    const uint32_t S = a[2];
    nu = (uint32_t)(__popc(b[0]) + __popc(b[1]) + __popc(b[2]) + ((S & kMedS4Died) ? 0 : __popc(b[3])));
    return (uint64_t)a[0] | ((uint64_t)a[1] << 32);
#else
    const uint64_t* r = p.mlog + addr * MW;
    nu = min((uint32_t)(r[1] & 15u), kMedMax);
    return r[0];
#endif
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p.dlog + addr * dense_words(p.K));
  uint32_t c = 0;
  for (uint32_t j = 0; j < p.K; ++j) c += (uint32_t)__popc(w[2 + j]);
  nu = c;
  return (uint64_t)w[0] | ((uint64_t)w[1] << 32);
}

constexpr uint32_t kEncThreads = 256;
constexpr uint32_t kFlatMax = 3u * kLogShards + 1u;

__device__ __forceinline__ void load_flat(uint64_t* lds, const uint64_t* flat, uint32_t shards) {
  for (uint32_t i = threadIdx.x; i <= 3u * shards; i += blockDim.x) lds[i] = flat[i];
  __syncthreads();
}

// Count pass: every entry of the pass's rounds adds (1 << 40 | its updates) to its bucket; runs of
// lanes with the same bucket (a wave's entries come from one writer wave's consecutive lanes, so a
// node's records sit together) add once, and every lane gets its rank among the bucket's entries.
__global__ __launch_bounds__(kEncThreads) void k_bucket_count(EncArgs a) {
  __shared__ uint64_t flat[kFlatMax];
  const EncodeParams& p = a.p;
  load_flat(flat, a.flat, p.shards);
  const uint64_t total = flat[3u * p.shards];
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t mask_le = lane == 63u ? ~0ull : ((2ull << lane) - 1ull);
  for (uint64_t base = (uint64_t)blockIdx.x * kEncThreads + (threadIdx.x & ~63u); base < total;
       base += (uint64_t)gridDim.x * kEncThreads) {
    const uint64_t f = base + lane;
    uint32_t b = 0xFFFFFFFFu, nu = 0u;
    if (f < total) {
      uint32_t kind;
      uint64_t addr;
      locate(flat, p.shards, f, kind, addr, p);
      const uint64_t key = entry_key(p, kind, addr, nu);
      const uint32_t rr = (uint32_t)(key >> p.round_shift), node = word_node(key, p.round_shift);
      const bool ok = node >= p.n0 && node - p.n0 < p.NL && rr < p.r_total;
      if (ok && rr >= p.r0 && rr < p.r0 + p.nr) b = (rr - p.r0) * p.NL + (node - p.n0);
      if (!ok) atomicOr(p.err, 1u);  // an entry outside the engine's nodes or the log's rounds
    }
    const uint32_t prev = (uint32_t)__shfl_up((int)b, 1u, 64);
    const bool head = lane == 0u || b != prev;
    const uint64_t H = __ballot(head);
    const uint32_t s0 = 63u - (uint32_t)__builtin_clzll(H & mask_le);
    const uint64_t above = H & ~mask_le;
    const uint32_t s1 = above ? (uint32_t)__builtin_ctzll(above) - 1u : 63u;
    const uint32_t incl = wave_incl_scan(nu, lane);
    const uint32_t excl0 = (uint32_t)__shfl((int)(incl - nu), (int)s0, 64);
    const uint32_t seg_upd = (uint32_t)__shfl((int)incl, (int)s1, 64) - excl0;
    unsigned long long old = 0ull;
    if (head && b != 0xFFFFFFFFu)
      old = atomicAdd(&a.cnt[b], ((unsigned long long)(s1 - s0 + 1u) << kCntShift) | seg_upd);
    old = __shfl(old, (int)s0, 64);
    if (f < total) a.ekey[f] = b == 0xFFFFFFFFu ? kInvalid64 : ((uint64_t)b << 32) | ((old >> kCntShift) + (lane - s0));
  }
}

// Scan sources over the buckets
struct EntriesIn {
  const unsigned long long* c;
  __device__ uint64_t operator()(uint64_t i) const { return c[i] >> kCntShift; }
};
struct UpdatesIn {
  const unsigned long long* c;
  __device__ uint64_t operator()(uint64_t i) const { return c[i] & kUpdMask; }
};
struct GroupBytesIn {  // compact stream: 8-B group header + the codes, padded to 4 B
  const unsigned long long* c;
  uint32_t cw;
  __device__ uint64_t operator()(uint64_t i) const {
    const uint64_t n = c[i] & kUpdMask;
    return n ? 8ull + ((n * cw + 3ull) & ~3ull) : 0ull;
  }
};

// Scatter pass: refs[eoff[bucket] + rank] = kind << 62 | address.
__global__ __launch_bounds__(kEncThreads) void k_bucket_scatter(EncArgs a, const uint64_t* eoff, uint64_t* refs) {
  __shared__ uint64_t flat[kFlatMax];
  const EncodeParams& p = a.p;
  load_flat(flat, a.flat, p.shards);
  const uint64_t total = flat[3u * p.shards];
  for (uint64_t f = (uint64_t)blockIdx.x * kEncThreads + threadIdx.x; f < total;
       f += (uint64_t)gridDim.x * kEncThreads) {
    const uint64_t k = a.ekey[f];
    if (k == kInvalid64) continue;
    uint32_t kind;
    uint64_t addr;
    locate(flat, p.shards, f, kind, addr, p);
    refs[eoff[k >> 32] + (k & 0xFFFFFFFFull)] = ((uint64_t)kind << 62) | addr;
  }
}

// Position of the r-th (0-based) set bit of m (r < popcount(m)).
__device__ __forceinline__ uint32_t nth_set(uint32_t m, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 16; w >= 1; w >>= 1) {
    const uint32_t low = m & ((1u << w) - 1u);
    const uint32_t c = (uint32_t)__popc(low);
    if (r >= c) {
      r -= c;
      m >>= w;
      pos += w;
    } else {
      m = low;
    }
  }
  return pos;
}

struct EmitArgs {
  EncodeParams p;
  const uint64_t* eoff;   // [B + 1]
  const uint64_t* uoff;   // [B + 1]
  const uint64_t* coff;   // [B + 1] (compact)
  const uint64_t* refs;
  uint32_t B;
  uint32_t C;             // cells = K * BL
  uint32_t* gtable;       // global tables (cells > kLdsCells): 3 * C u32 per wave, zeroed
  uint64_t* out;          // packed words (at ubase + uoff[b])
  uint8_t* cout;          // compact groups (at cbase + coff[b])
  uint64_t ubase, cbase;
};
constexpr uint32_t kLdsCells = 4096;  // 48 KiB of LDS per wave

template <bool G>
__device__ __forceinline__ uint32_t tld(const uint32_t* p) {
  if constexpr (G) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// Medium / dense record or single word -> cells (slot, block): the update masks, status bit 1 (A after
// the slot) and status bit 0 (~(A ^ died)) planes (vote.go:77-91: Rejected 1, Accepted 2, Invalid 0,
// Finalized 3; A after slot j = A_final ^ parity of the later slots' updates).
__device__ __forceinline__ void cell_or(uint32_t* msk, uint32_t* hi, uint32_t* lo, uint32_t cell, uint32_t e,
                                        uint32_t h, uint32_t l) {
  atomicOr(msk + cell, e);
  if (h) atomicOr(hi + cell, h);
  if (l) atomicOr(lo + cell, l);
}

// A log entry's updates as per-slot masks in registers: no array is indexed at run time, so nothing
// lives in scratch memory (a scratch access is a vector-memory operation, and the wave's one in-order
// vector-memory counter would make every such load wait behind the wave's output stores).
struct RecRegs {
  uint32_t kind;  // 0 single word, 1 slot (medium) record, 2 dense record
  uint32_t key;   // low half of the key word (a single: of the update word: slot, target, status)
  uint32_t E[8];  // updated records per slot (k <= 8); folded medium records (AVK_MED_S4 = 0): payload
  uint32_t A, died;
};

__device__ __forceinline__ uint32_t pick4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  return i == 0u ? a : i == 1u ? b : i == 2u ? c : d;
}

// k <= 8 only (E[8])
__device__ __forceinline__ void load_rec(const EncodeParams& p, uint64_t ref, RecRegs& r) {
  r.kind = (uint32_t)(ref >> 62);
  const uint64_t addr = ref & ((1ull << 62) - 1ull);
  r.A = r.died = 0u;
#pragma unroll
  for (int j = 0; j < 8; ++j) r.E[j] = 0u;
  if (r.kind == 0u) {
    r.key = (uint32_t)p.log[addr];
  } else if (r.kind == 1u) {
#if AVK_MED_S4
    const u32x4* q = reinterpret_cast<const u32x4*>(p.mlog + addr * med_rec_words());
    const u32x4 x = q[0], y = q[1];
    r.key = x[0];
    const uint32_t S = x[2];
    r.A = x[3];
    const bool hasd = (S & kMedS4Died) != 0u;
    r.died = hasd ? y[3] : 0u;
    const uint32_t nw = hasd ? 3u : 4u;  // E words stored, in slot order
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t i = (uint32_t)__popc(S & ((1u << j) - 1u));
      r.E[j] = ((S >> j) & 1u) && i < nw ? pick4(i, y[0], y[1], y[2], y[3]) : 0u;
    }
#else
    const uint64_t* q = p.mlog + addr * med_rec_words();
    const uint64_t k0 = q[0], pl = q[1];
    r.key = (uint32_t)k0;
    r.E[0] = (uint32_t)pl;
    r.E[1] = (uint32_t)(pl >> 32);
#endif
  } else {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p.dlog + addr * dense_words(p.K));
    r.key = w[0];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if ((uint32_t)j < p.K) r.E[j] = w[2 + j];
    r.A = w[2 + p.K];
    r.died = w[3 + p.K];
  }
}

__device__ __forceinline__ void fill_regs(const EncodeParams& p, const RecRegs& r, uint32_t* msk, uint32_t* hi,
                                          uint32_t* lo) {
  if (r.kind == 0u) {
    const uint32_t tl = ((r.key >> 2) & 0x3FFFFFu) - p.t0;
    const uint32_t slot = (r.key >> 24) & 15u, st = r.key & 3u, m = 1u << (tl & 31u);
    cell_or(msk, hi, lo, slot * p.BL + (tl >> 5), m, (st & 2u) ? m : 0u, (st & 1u) ? m : 0u);
    return;
  }
  const uint32_t blk = (((r.key >> 2) & 0x3FFFFFu) - p.t0) >> 5;  // the key's target field: the block's first
#if !AVK_MED_S4
  if (r.kind == 1u) {
    const uint64_t pl = (uint64_t)r.E[0] | ((uint64_t)r.E[1] << 32);
    const uint32_t n = min((uint32_t)(pl & 15u), kMedMax);
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t fld = (uint32_t)(pl >> (4u + 10u * i)) & 1023u;
      const uint32_t slot = fld >> 7, bit = (fld >> 2) & 31u, st = fld & 3u, m = 1u << bit;
      cell_or(msk, hi, lo, slot * p.BL + blk, m, (st & 2u) ? m : 0u, (st & 1u) ? m : 0u);
    }
    return;
  }
#endif
  uint32_t par = 0u;  // A after slot j = A_final ^ parity of the later slots' updates (vote.go:77-91)
#pragma unroll
  for (int j = 7; j >= 0; --j) {
    const uint32_t aj = r.A ^ par, e = r.E[j];
    par ^= e;
    if (e) cell_or(msk, hi, lo, (uint32_t)j * p.BL + blk, e, aj & e, ~(aj ^ r.died) & e);
  }
}

__device__ __forceinline__ void fill_entry(const EncodeParams& p, uint64_t ref, uint32_t* msk, uint32_t* hi,
                                           uint32_t* lo) {
  if (p.K <= 8u || (ref >> 62) != 2u) {  // (medium records exist at k <= 8 only)
    RecRegs r;
    load_rec(p, ref, r);
    fill_regs(p, r, msk, hi, lo);
    return;
  }
  // dense record at k > 8: the slot masks straight from memory
  const uint64_t addr = ref & ((1ull << 62) - 1ull);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p.dlog + addr * dense_words(p.K));
  const uint32_t blk = (((w[0] >> 2) & 0x3FFFFFu) - p.t0) >> 5;
  const uint32_t A = w[2 + p.K], died = w[3 + p.K];
  uint32_t par = 0u;
  for (int j = (int)p.K - 1; j >= 0; --j) {
    const uint32_t aj = A ^ par, e = w[2 + j];
    par ^= e;
    if (e) cell_or(msk, hi, lo, (uint32_t)j * p.BL + blk, e, aj & e, ~(aj ^ died) & e);
  }
}

// The waves of a workgroup work on different buckets: wave-level ordering only. LDS operations of one
// wave execute in issue order, so waiting for the wave's own LDS operations (lgkmcnt) and keeping the
// compiler from moving memory operations across is enough — no vmcnt wait: the output stores and the
// next bucket's loads stay in flight (a workgroup fence or barrier would wait for them every time).
// Global tables (rare: > 4096 cells) take a device fence.
template <bool G>
__device__ __forceinline__ void wave_sync() {
  if constexpr (G) {
    __threadfence();
    __builtin_amdgcn_wave_barrier();
  } else {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// One wave per bucket (grid-stride over buckets, several independent waves per workgroup): its
// entries OR their updates into the bucket's (slot, block) cells in LDS, then one pass over the cells
// in canonical order (slot-major, block-minor) writes them out. The next bucket's offsets, first 64
// entry refs and their record words (k <= 8) are loaded while this bucket is laid out.
template <bool COMPACT, bool G>
__global__ __launch_bounds__(256) void k_bucket_emit(EmitArgs a) {
  extern __shared__ uint32_t sm[];
  const EncodeParams& p = a.p;
  const uint32_t C = a.C, lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, W = blockDim.x >> 6;
  const uint32_t gw = blockIdx.x * W + wv, gstride = gridDim.x * W;
  uint32_t* tbl = G ? a.gtable + (size_t)gw * 3u * C : sm + (size_t)wv * 3u * C;
  uint32_t *msk = tbl, *hi = tbl + C, *lo = tbl + 2u * C;
  if (!G) {
    for (uint32_t c = lane; c < 3u * C; c += 64u) tbl[c] = 0u;
    wave_sync<G>();
  }
  const bool pref = p.K <= 8u;  // record words fit RecRegs
  uint32_t b = gw;
  uint64_t e0 = 0, e1 = 0, ref = 0;
  RecRegs rr_cur{};
  if (b < a.B) {
    e0 = a.eoff[b];
    e1 = a.eoff[b + 1];
    if (lane < e1 - e0) {
      ref = a.refs[e0 + lane];
      if (pref) load_rec(p, ref, rr_cur);
    }
  }
  while (b < a.B) {
    const uint32_t nb = b + gstride;
    uint64_t ne0 = 0, ne1 = 0;
    if (nb < a.B) {  // issued now, used after this bucket's fill
      ne0 = a.eoff[nb];
      ne1 = a.eoff[nb + 1];
    }
    uint64_t nref = 0;
    RecRegs rr_next{};
    if (e0 != e1) {
      const uint64_t u0 = a.uoff[b], u1 = a.uoff[b + 1];
      const uint64_t c0b = COMPACT ? a.coff[b] : 0ull;
      const uint32_t nl = b % p.NL, rnd = p.r0 + b / p.NL, node = p.n0 + nl;
      if (lane < e1 - e0) {
        if (pref) fill_regs(p, rr_cur, msk, hi, lo);
        else fill_entry(p, ref, msk, hi, lo);
      }
      for (uint64_t e = e0 + 64u + lane; e < e1; e += 64u) fill_entry(p, a.refs[e], msk, hi, lo);
      if (nb < a.B && lane < ne1 - ne0) {  // the next bucket's refs and records, in flight from here
        nref = a.refs[ne0 + lane];
        if (pref) load_rec(p, nref, rr_next);
      }
      wave_sync<G>();
      // one pass over the cells in canonical order (slot-major, block-minor): lane = cell within each
      // chunk of 64, its first output position from a wave scan of the counts, its updates written in
      // ascending target (stores of one instruction land within the bucket's few output lines); the
      // cell's one reader clears it for the next bucket
      const uint32_t want = (uint32_t)(u1 - u0);
      uint64_t* out = COMPACT ? nullptr : a.out + a.ubase + u0;
      uint8_t* grp = COMPACT ? a.cout + a.cbase + c0b : nullptr;
      const uint64_t hi_word = ((uint64_t)rnd << p.round_shift) | ((uint64_t)node << 28);
      uint32_t run = 0;
      for (uint32_t c0 = 0; c0 < C; c0 += 64u) {
        const uint32_t c = c0 + lane;
        uint32_t m = 0u, h = 0u, l = 0u;
        if (c < C) {
          m = tld<G>(msk + c);
          if (m) {
            h = tld<G>(hi + c);
            l = tld<G>(lo + c);
            msk[c] = 0u;
            hi[c] = 0u;
            lo[c] = 0u;
          }
        }
        const uint32_t cnt = (uint32_t)__popc(m);
        const uint32_t incl = wave_incl_scan(cnt, lane);
        if (m) {
          uint32_t pos = run + incl - cnt;
          const uint32_t slot = c / p.BL, tb = (c - slot * p.BL) * 32u;
          for (; m; m &= m - 1u, ++pos) {
            const uint32_t bit = (uint32_t)__builtin_ctz(m);
            const uint32_t st = (((h >> bit) & 1u) << 1) | ((l >> bit) & 1u);
            if (pos >= want) continue;  // a count mismatch (flagged below): no store leaves the span
            if constexpr (COMPACT) {
              const uint32_t code = (slot << (p.target_bits + 2u)) | ((tb + bit) << 2) | st;
              if (p.code_bytes == 2u) reinterpret_cast<uint16_t*>(grp + 8)[pos] = (uint16_t)code;
              else reinterpret_cast<uint32_t*>(grp + 8)[pos] = code;
            } else {
              out[pos] = hi_word | ((uint64_t)slot << 24) | ((uint64_t)(p.t0 + tb + bit) << 2) | st;
            }
          }
        }
        run += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
      }
      if (run != want && lane == 0) atomicOr(p.err, 2u);
      const uint32_t n = min(run, want);
      if constexpr (COMPACT) {
        if (lane == 0) {
          reinterpret_cast<uint32_t*>(grp)[0] = node;
          reinterpret_cast<uint32_t*>(grp)[1] = n;
          if (p.code_bytes == 2u && (n & 1u)) reinterpret_cast<uint16_t*>(grp + 8)[n] = 0u;  // pad to 4 B
        }
      }
      wave_sync<G>();
    } else if (nb < a.B && lane < ne1 - ne0) {
      nref = a.refs[ne0 + lane];
      if (pref) load_rec(p, nref, rr_next);
    }
    b = nb;
    e0 = ne0;
    e1 = ne1;
    ref = nref;
    rr_cur = rr_next;
  }
}

// Compact stream index: entry (round r0 + r, chunk c) = {byte offset of its first group from the groups'
// start, updates before it}; the last pass also writes the end entry.
__global__ void k_compact_index(const uint64_t* coff, const uint64_t* uoff, uint64_t* idx, uint32_t r0, uint32_t nr,
                                uint32_t chunks, uint32_t chunk_nodes, uint32_t NL, uint64_t cbase, uint64_t ubase,
                                uint32_t end_entry) {
  const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t n = nr * chunks;
  if (j < n) {
    const uint32_t r = j / chunks, c = j - r * chunks;
    const uint64_t b = (uint64_t)r * NL + (uint64_t)c * chunk_nodes;
    const uint64_t at = ((uint64_t)(r0 + r) * chunks + c) * 2u;
    idx[at] = cbase + coff[b];
    idx[at + 1] = ubase + uoff[b];
  } else if (j == n && end_entry) {
    const uint64_t B = (uint64_t)nr * NL;
    const uint64_t at = ((uint64_t)(r0 + nr) * chunks) * 2u;
    idx[at] = cbase + coff[B];
    idx[at + 1] = ubase + uoff[B];
  }
}

}  // namespace

hipError_t launch_log_digest(const uint64_t* log, const uint32_t* counts, uint32_t cap, const uint64_t* dlog,
                             const uint32_t* dcounts, uint32_t dcap, const uint64_t* mlog, const uint32_t* mcounts,
                             uint32_t mcap, uint32_t shards, uint32_t k, uint32_t node0, uint32_t node1,
                             uint32_t round_shift, unsigned long long* out, hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, 3 * sizeof(unsigned long long), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_log_digest, dim3(16, shards), dim3(256), 0, s, log, counts, cap, dlog, dcounts, dcap, mlog,
                     mcounts, mcap, k, node0, node1, round_shift, out);
  return hipGetLastError();
}

// ---- encoder scratch layout (u64 words) ----
namespace {
struct EncLayout {
  uint64_t flat, flat_sc, cnt, eoff, uoff, coff, bsc, ekey, refs, gtab, words;
};
EncLayout enc_layout(const EncodeParams& p, uint64_t entries, uint32_t B, uint32_t grid_g) {
  EncLayout L{};
  auto up = [](uint64_t w) { return (w + 31u) / 32u * 32u; };  // 256-B aligned regions
  uint64_t at = 0;
  L.flat = at;
  at += up(kFlatMax);
  L.flat_sc = at;
  at += up(dscan::scan_scratch_words(3u * p.shards));
  L.cnt = at;
  at += up(B);
  L.eoff = at;
  at += up((uint64_t)B + 1u);
  L.uoff = at;
  at += up((uint64_t)B + 1u);
  L.coff = at;
  at += up((uint64_t)B + 1u);
  L.bsc = at;
  at += up(dscan::scan_scratch_words((uint64_t)B + 1u));
  L.ekey = at;
  at += up(entries);
  L.refs = at;
  at += up(entries);
  L.gtab = at;
  const uint64_t C = (uint64_t)p.K * p.BL;
  at += C > kLdsCells ? up((uint64_t)grid_g * 3u * C / 2u + 1u) : 0u;
  L.words = at;
  return L;
}
uint32_t emit_global_grid(uint64_t cells) {
  // global tables: 12 B per cell per wave, at most ~1 GiB of them
  const uint64_t per = 12u * cells;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, (1ull << 30) / per));
}
}  // namespace

uint64_t encode_scratch_bytes(const EncodeParams& p, uint64_t entries, uint32_t B) {
  return enc_layout(p, entries, B, emit_global_grid((uint64_t)p.K * p.BL)).words * 8u;
}

hipError_t launch_encode_log(const EncodeParams& p, uint64_t entries, void* scratch, uint64_t* out, uint8_t* cout,
                             uint64_t* cidx, uint32_t chunks, uint32_t chunk_nodes, uint64_t ubase, uint64_t cbase,
                             bool last_pass, uint64_t* totals, hipStream_t s) {
  const uint32_t B = p.nr * p.NL;
  const uint64_t C = (uint64_t)p.K * p.BL;
  const bool G = C > kLdsCells;
  const uint32_t gg = emit_global_grid(C);
  const EncLayout L = enc_layout(p, entries, B, gg);
  uint64_t* w = static_cast<uint64_t*>(scratch);
  hipError_t e;
  // flat entry offsets of the shards (device counters: no host round trip)
  FlatIn fin{p.log_count, p.shards, p.log_cap, p.mlog_cap, p.dlog_cap};
  if ((e = dscan::launch_scan(fin, 3u * p.shards, w + L.flat, w + L.flat_sc, s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(w + L.cnt, 0, (size_t)B * 8u, s)) != hipSuccess) return e;
  EncArgs ea{p, w + L.flat, reinterpret_cast<unsigned long long*>(w + L.cnt), w + L.ekey, B};
  const uint32_t egrid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((entries + kEncThreads - 1) / kEncThreads, 2048));
  if (entries) {
    hipLaunchKernelGGL(k_bucket_count, dim3(egrid), dim3(kEncThreads), 0, s, ea);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  const unsigned long long* cnt = reinterpret_cast<const unsigned long long*>(w + L.cnt);
  if ((e = dscan::launch_scan(EntriesIn{cnt}, B, w + L.eoff, w + L.bsc, s)) != hipSuccess) return e;
  if ((e = dscan::launch_scan(UpdatesIn{cnt}, B, w + L.uoff, w + L.bsc, s)) != hipSuccess) return e;
  if (cout && (e = dscan::launch_scan(GroupBytesIn{cnt, p.code_bytes}, B, w + L.coff, w + L.bsc, s)) != hipSuccess)
    return e;
  if (entries) {
    hipLaunchKernelGGL(k_bucket_scatter, dim3(egrid), dim3(kEncThreads), 0, s, ea, (const uint64_t*)(w + L.eoff),
                       w + L.refs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  EmitArgs em{p, w + L.eoff, w + L.uoff, w + L.coff, w + L.refs, B, (uint32_t)C,
              reinterpret_cast<uint32_t*>(w + L.gtab), out, cout, ubase, cbase};
  if (entries && B) {
    if (G) {
      if ((e = hipMemsetAsync(w + L.gtab, 0, (size_t)gg * 12u * C, s)) != hipSuccess) return e;
      const uint32_t wpg = gg >= 4u ? 4u : 1u;  // waves per workgroup (each with its own table)
      const uint32_t grid = (uint32_t)std::min<uint64_t>((B + wpg - 1u) / wpg, gg / wpg);
      if (cout)
        hipLaunchKernelGGL((k_bucket_emit<true, true>), dim3(grid), dim3(64u * wpg), 0, s, em);
      else
        hipLaunchKernelGGL((k_bucket_emit<false, true>), dim3(grid), dim3(64u * wpg), 0, s, em);
    } else {
      // waves per workgroup: 4 while their tables fit 48 KiB (C <= 1024), fewer for larger tables
      const uint32_t wpg = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(4, kLdsCells / C));
      const uint32_t grid = (uint32_t)std::min<uint64_t>((B + wpg - 1u) / wpg, 256u * 32u / wpg);
      const size_t lds = (size_t)12u * C * wpg;
      if (cout)
        hipLaunchKernelGGL((k_bucket_emit<true, false>), dim3(grid), dim3(64u * wpg), lds, s, em);
      else
        hipLaunchKernelGGL((k_bucket_emit<false, false>), dim3(grid), dim3(64u * wpg), lds, s, em);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  if (cout && cidx) {
    const uint32_t n = p.nr * chunks + 1u;
    hipLaunchKernelGGL(k_compact_index, dim3((n + 255u) / 256u), dim3(256), 0, s, (const uint64_t*)(w + L.coff),
                       (const uint64_t*)(w + L.uoff), cidx, p.r0, p.nr, chunks, chunk_nodes, p.NL, cbase, ubase,
                       last_pass ? 1u : 0u);
    if ((e = hipGetLastError()) != hipSuccess) return e;
  }
  // this pass's totals: updates, compact bytes, entries grouped
  if (totals) {
    if ((e = hipMemcpyAsync(totals, w + L.uoff + B, 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    if (cout && (e = hipMemcpyAsync(totals + 1, w + L.coff + B, 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(totals + 2, w + L.eoff + B, 8, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
  }
  return hipSuccess;
}

// Device -> host-mapped pinned memory copy on a few workgroups (the compact stream's copy beside the
// next rounds): PCIe writes need only a few hundred KiB in flight, so a small grid saturates the link
// and leaves the CUs to the round kernel (the runtime's blit copy takes a full grid). Four 16-B loads
// in flight per thread, then their stores.
namespace {
__global__ __launch_bounds__(256) void k_stream_out(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x;
  for (; i + 3u * stride < n16; i += 4u * stride) {
    const u32x4 a = __builtin_nontemporal_load(src + i), b = __builtin_nontemporal_load(src + i + stride);
    const u32x4 c = __builtin_nontemporal_load(src + i + 2u * stride), d = __builtin_nontemporal_load(src + i + 3u * stride);
    dst[i] = a;
    dst[i + stride] = b;
    dst[i + 2u * stride] = c;
    dst[i + 3u * stride] = d;
  }
  for (; i < n16; i += stride) dst[i] = __builtin_nontemporal_load(src + i);
}
}  // namespace

hipError_t launch_stream_out(const void* src, void* dst, uint64_t bytes, uint32_t blocks, hipStream_t s) {
  const uint64_t n16 = (bytes + 15u) / 16u;
  if (!n16) return hipSuccess;
  const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(blocks, (n16 + 255u) / 256u));
  hipLaunchKernelGGL(k_stream_out, dim3(g), dim3(256), 0, s, static_cast<const u32x4*>(src), static_cast<u32x4*>(dst),
                     n16);
  return hipGetLastError();
}

// Diagnostics (engine option "warm_pref"): read a buffer once, so that the round kernel timed after
// it finds the lines where a GPU of its own would have them (tools/group_model.py --warm-pref). The
// sum is stored only if it equals a value no read can produce in practice, so the loads stay.
namespace {
__global__ __launch_bounds__(256) void k_touch(const u32x4* __restrict__ src, uint64_t n16, uint32_t* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  uint32_t acc = 0u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = src[i];
    acc += v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}
}  // namespace

hipError_t launch_touch(const void* src, uint64_t bytes, uint32_t* sink, hipStream_t s) {
  const uint64_t n16 = bytes / 16u;
  if (!n16) return hipSuccess;
  const uint32_t g = (uint32_t)std::min<uint64_t>(4096, (n16 + 255u) / 256u);
  hipLaunchKernelGGL(k_touch, dim3(g), dim3(256), 0, s, static_cast<const u32x4*>(src), n16, sink);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Drop-in RegisterVotes batch (engine.cpp av_register_votes_batch): group the votes by lane (node,
// 32-target block) keeping their order inside a lane — the stable radix sort of (lane, position) —
// then run-length encode the sorted lanes into the (lanes, offs) CSR k_register_votes walks.
// ---------------------------------------------------------------------------
namespace {
struct HeadsIn {
  const uint32_t* k;
  __device__ uint64_t operator()(uint64_t i) const { return (i == 0 || k[i] != k[i - 1]) ? 1u : 0u; }
};
// run r of the sorted keys: lanes[r] = its key, offs[r] = its first position; offs[n_runs] = n
__global__ __launch_bounds__(256) void k_rle_write(const uint32_t* ks, const uint64_t* run_of, uint32_t n,
                                                   uint32_t* lanes, uint32_t* offs, uint32_t* n_runs) {
  const uint32_t i = blockIdx.x * 256u + threadIdx.x;
  if (i >= n) return;
  if (i == 0 || ks[i] != ks[i - 1]) {
    const uint32_t r = (uint32_t)run_of[i];
    lanes[r] = ks[i];
    offs[r] = i;
  }
  if (i == n - 1u) {
    const uint32_t nr = (uint32_t)run_of[n];
    offs[nr] = n;
    *n_runs = nr;
  }
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

uint64_t group_votes_scratch_words(uint32_t n) {
  return std::max<uint64_t>(dscan::radix_scratch_words(n), (uint64_t)n + 1u + dscan::scan_scratch_words((uint64_t)n + 1u));
}

hipError_t launch_group_votes(uint64_t* scratch, const uint32_t* keys, const uint32_t* vidx, const uint32_t* info,
                              uint32_t n, int key_bits, uint32_t* keys_s, uint32_t* perm_s, uint32_t* keys_t,
                              uint32_t* perm_t, uint32_t* lanes, uint32_t* offs, uint32_t* n_runs, uint32_t* entries,
                              hipStream_t s) {
  if (n == 0) return hipMemsetAsync(n_runs, 0, 4, s);
  hipError_t e = dscan::launch_radix_sort_pairs(keys, nullptr, n, key_bits, keys_s, perm_s, keys_t, perm_t, scratch, s);
  if (e != hipSuccess) return e;
  // run index of every position: exclusive scan of the run heads (run_of[n] = runs)
  uint64_t* run_of = scratch;
  if ((e = dscan::launch_scan(HeadsIn{keys_s}, n, run_of, scratch + n + 1u, s)) != hipSuccess) return e;
  const uint32_t g = (n + 255u) / 256u;
  hipLaunchKernelGGL(k_rle_write, dim3(g), dim3(256), 0, s, (const uint32_t*)keys_s, (const uint64_t*)run_of, n,
                     lanes, offs, n_runs);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(k_vote_entries, dim3(g), dim3(256), 0, s, (const uint32_t*)perm_s, vidx, info, n, entries);
  return hipGetLastError();
}

}  // namespace avk
