// Device helpers shared by the round kernels (kernels.hip: per-lane round,
// capped round, drop-in; round_sweep.hip: the persistent streaming round).
// Philox4x32-10, the bit-sliced VoteRecord step (vote.go:54-75), peer
// sampling, wave scans, StatusUpdate emission (processor.go:111) and the
// per-wave counters. Header-only: every translation unit gets its own
// internal-linkage copy.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"

namespace avk {
namespace {

constexpr uint32_t kDomPeers = 1u, kDomByz = 2u, kDomInit = 3u, kDomPairs = 4u, kDomReplay = 5u;
// replay class thresholds: P(yes)=0.70, P(no)=0.25, P(neutral)=0.05
constexpr uint32_t kReplayYes = 3006477107u, kReplayNo = 4080218931u;

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11), same counter/key conventions as the
// oracle's restatement (oracle/avalanche_oracle.c) and Random123's KATs.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox(uint32_t x[4], uint64_t seed, uint32_t a, uint32_t b, uint32_t c,
                                       uint32_t dom) {
  uint32_t c0 = a, c1 = b, c2 = c, c3 = dom;
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  // opaque key: the 20-word key schedule is recomputed (SALU) per call instead
  // of being hoisted out of the tile loop into 20 live SGPRs (spills)
  k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);  // the seed is uniform: keep it scalar
  k1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
  asm volatile("" : "+s"(k0), "+s"(k1));
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)p1;
    c3 = (uint32_t)p0;
    c0 = n0;
    c2 = n2;
  }
  x[0] = c0; x[1] = c1; x[2] = c2; x[3] = c3;
}

__device__ __forceinline__ uint32_t bfi(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

// State-plane stream accessors. NT = non-temporal (global_load/store ... nt):
// the planes are touched once per round, so keeping them out of L2 / the
// Infinity Cache leaves room for the gathered preference table.
template <bool NT>
__device__ __forceinline__ uint32_t pld(const uint32_t* q) {
  if constexpr (NT) return __builtin_nontemporal_load(q);
  return *q;
}
template <bool NT>
__device__ __forceinline__ void pst(uint32_t* q, uint32_t v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, q);
  else
    *q = v;
}
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ u32x4 pld4(const u32x4* q) {
  if constexpr (NT) return __builtin_nontemporal_load(q);
  return *q;
}
template <bool NT>
__device__ __forceinline__ void pst4(u32x4* q, u32x4 v) {
  if constexpr (NT)
    __builtin_nontemporal_store(v, q);
  else
    *q = v;
}

// The k replayed (yes, consider) word pairs of lane g (kernels.h replay_idx):
// ceil(K/2) dwordx4 loads; the stream is read once per round (non-temporal).
template <int K>
__device__ __forceinline__ void replay_load(const uint32_t* rp, uint32_t g, uint32_t* w, uint32_t* cw) {
  constexpr int G = (K + 1) / 2;
  const u32x4* q = reinterpret_cast<const u32x4*>(rp) + (size_t)(g >> 6) * (G * 64) + (g & 63u);
#pragma unroll
  for (int i = 0; i < G; ++i) {
    const u32x4 v = pld4<true>(q + i * 64);
    w[2 * i] = v[0];
    cw[2 * i] = v[1];
    if (2 * i + 1 < K) {
      w[2 * i + 1] = v[2];
      cw[2 * i + 1] = v[3];
    }
  }
}

// Byzantine flip-flop answer: err = ((r ^ t) & 1) ? 1 : 0, so
// "yes" on even targets in even rounds. Blocks start at multiples of 32.
__device__ __forceinline__ uint32_t byz_pattern(uint32_t round) { return (round & 1u) ? 0xAAAAAAAAu : 0x55555555u; }

__device__ __forceinline__ bool is_byz(const uint32_t* byz, uint32_t node) { return (byz[node >> 5] >> (node & 31u)) & 1u; }

// The word a node publishes for 32 targets (what its responder answers,
// main.go:168-192): live records their accepted bit; records it does not hold
// (K7): mode 0 the finalized decision kept in A (harness rule R2), mode 1
// false (IsAccepted literally, processor.go:125-130), mode 2 true (the
// example's responder re-adds &tx{isAccepted: true} first, main.go:175-182).
__device__ __forceinline__ uint32_t publish_word(uint32_t A, uint32_t K7, uint32_t mode) {
  return mode == 0u ? A : mode == 1u ? (A & ~K7) : (A | K7);
}

struct St {
  uint32_t V[8], C[8], A, K[8];
};

// Tile layout (1600 words = 6400 B per 64 lanes), see kernels.h:
//   [0,1024)    V0-3 | V4-7 | K0-3 | K4-7 as 16-byte groups, lane-interleaved:
//               group q, lane l, plane i -> q*256 + l*4 + i  (one dwordx4 per
//               lane, 1 KiB contiguous per wave-instruction)
//   [1024,1536) C0..C7 dword planes: 1024 + c*64 + l
//   [1536,1600) A dword plane:       1536 + l
__host__ __device__ constexpr uint32_t plane_off(int p, uint32_t lane) {
  return p < kPC ? (uint32_t)(p >> 2) * 256u + lane * 4u + (uint32_t)(p & 3)
       : p < kPA ? 1024u + (uint32_t)(p - kPC) * 64u + lane
       : p == kPA ? 1536u + lane
       : (uint32_t)(2 + ((p - kPK) >> 2)) * 256u + lane * 4u + (uint32_t)((p - kPK) & 3);
}

__device__ __forceinline__ uint32_t* tile_of(const uint32_t* planes, uint32_t g) {
  return const_cast<uint32_t*>(planes) + (size_t)(g >> 6) * (kPlanes * 64);
}

// pointer to the word of plane p for lane g
__device__ __forceinline__ uint32_t* pw(const uint32_t* planes, uint32_t g, int p) {
  return tile_of(planes, g) + plane_off(p, g & 63u);
}

__device__ __forceinline__ void load_state(const uint32_t* planes, uint32_t g, St& s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) s.V[i] = *pw(planes, g, kPV + i);
#pragma unroll
  for (int i = 0; i < 8; ++i) s.C[i] = *pw(planes, g, kPC + i);
  s.A = *pw(planes, g, kPA);
#pragma unroll
  for (int i = 0; i < 8; ++i) s.K[i] = *pw(planes, g, kPK + i);
}

__device__ __forceinline__ void store_state(uint32_t* planes, uint32_t g, const St& s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) *pw(planes, g, kPV + i) = s.V[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) *pw(planes, g, kPC + i) = s.C[i];
  *pw(planes, g, kPA) = s.A;
#pragma unroll
  for (int i = 0; i < 8; ++i) *pw(planes, g, kPK + i) = s.K[i];
}

// No live record in any of the 32 slots (canonical dead form).
__device__ __forceinline__ void dead_state(St& s) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s.V[i] = 0u;
    s.C[i] = ~0u;
    s.K[i] = 0u;
  }
  s.K[7] = ~0u;
  s.A = 0u;
}

// Bit-sliced "popcount of 8 > 6" (vote.go:58,61): at most one zero among x[].
__device__ __forceinline__ uint32_t atleast7(const uint32_t (&x)[8]) {
  uint32_t t = x[0], u = ~0u;
#pragma unroll
  for (int i = 1; i < 8; ++i) {
    u = (u & x[i]) | t;
    t &= x[i];
  }
  return u;
}

// One regsiterVote (vote.go:54-75) applied to the records of `part`.
//   yw : err == 0            (vote.go:55)
//   cw : int32(err) >= 0     (vote.go:56)
// MASKED=false shifts every bit (caller restores non-participants at the end
// of the round); MASKED=true leaves non-participating records untouched.
// Outputs E = records whose regsiterVote returned true, fin = finalized now.
template <bool MASKED>
__device__ __forceinline__ void vote_step(St& s, uint32_t yw, uint32_t cw, uint32_t part, uint32_t& E,
                                          uint32_t& fin) {
  yw &= cw;
  if (MASKED) {
#pragma unroll
    for (int i = 7; i > 0; --i) {
      s.V[i] = bfi(part, s.V[i - 1], s.V[i]);
      s.C[i] = bfi(part, s.C[i - 1], s.C[i]);
    }
    s.V[0] = bfi(part, yw, s.V[0]);
    s.C[0] = bfi(part, cw, s.C[0]);
  } else {
#pragma unroll
    for (int i = 7; i > 0; --i) {
      s.V[i] = s.V[i - 1];
      s.C[i] = s.C[i - 1];
    }
    s.V[0] = yw;
    s.C[0] = cw;
  }
  uint32_t y[8], n[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    y[i] = s.V[i] & s.C[i];   // votes & consider            (vote.go:58)
    n[i] = ~s.V[i] & s.C[i];  // (-votes-1) & consider        (vote.go:61)
  }
  const uint32_t yes = atleast7(y);
  const uint32_t no = atleast7(n);
  const uint32_t concl = (yes | no) & part;  // conclusive     (vote.go:61-63)
  const uint32_t flip = concl & (s.A ^ yes);  // disagrees      (vote.go:72-74)
  uint32_t carry = concl ^ flip;              // agrees: conf+=2 (vote.go:66-69)
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const uint32_t c2 = s.K[i] & carry;
    s.K[i] = (s.K[i] ^ carry) & ~flip;  // flip resets the count
    carry = c2;
  }
  s.K[7] |= carry;  // count reached exactly 128 (vote.go:68), record deleted
  s.A = bfi(flip, yes, s.A);
  E = flip | carry;
  fin = carry;
}

// General form of the peer draw: walk the Philox candidate stream of (node,
// round) and keep the first K distinct values (avo_sample_peers in the
// oracle). Taken only when the first ceil(K/4) blocks hold a repeat.
template <int K>
__device__ __forceinline__ void sample_peers_slow(uint64_t seed, uint32_t node, uint32_t round, uint32_t others,
                                               uint32_t (&out)[K]) {
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) out[j] = 0u;
  for (uint32_t blk = 0; cnt < (uint32_t)K; ++blk) {
    uint32_t x[4];
    philox(x, seed, node, round, blk, kDomPeers);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = (uint32_t)(((uint64_t)x[i] * others) >> 32);
      const uint32_t pp = u + (u >= node ? 1u : 0u);
      bool dup = false;
#pragma unroll
      for (int j = 0; j < K; ++j) dup |= ((uint32_t)j < cnt) && (out[j] == pp);
      if (!dup && cnt < (uint32_t)K) {
#pragma unroll
        for (int j = 0; j < K; ++j) out[j] = ((uint32_t)j == cnt) ? pp : out[j];
        ++cnt;
      }
    }
  }
}

// k distinct peers != node, uniform over the other N-1 nodes (first K
// distinct values of the Philox candidate stream; same definition as
// avo_sample_peers in the oracle). Fast path = the first ceil(K/4) Philox
// blocks give K distinct candidates; otherwise a rarely taken general loop.
template <int K>
__device__ __forceinline__ void sample_peers(uint64_t seed, uint32_t node, uint32_t round, uint32_t n_nodes,
                                             int mode, uint32_t (&out)[K]) {
  const uint32_t others = n_nodes - 1u;
  if (mode == 1 || (uint32_t)K >= others) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint64_t q = (mode == 1) ? (uint64_t)round * (uint64_t)K + (uint64_t)j : (uint64_t)j;
      const uint32_t idx = (uint32_t)(q % others);
      out[j] = idx + (idx >= node ? 1u : 0u);
    }
    return;
  }
  constexpr int NB = (K + 3) / 4;
  uint32_t cand[NB * 4];
#pragma unroll
  for (int blk = 0; blk < NB; ++blk) {
    uint32_t x[4];
    philox(x, seed, node, round, (uint32_t)blk, kDomPeers);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = (uint32_t)(((uint64_t)x[i] * others) >> 32);
      cand[blk * 4 + i] = u + (u >= node ? 1u : 0u);
    }
  }
  bool distinct = true;
#pragma unroll
  for (int i = 1; i < K; ++i)
#pragma unroll
    for (int j = 0; j < i; ++j) distinct &= cand[i] != cand[j];
  if (distinct) {
#pragma unroll
    for (int j = 0; j < K; ++j) out[j] = cand[j];
    return;
  }
  sample_peers_slow<K>(seed, node, round, others, out);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = (uint32_t)__shfl_up((int)v, (unsigned)d, 64);
    if (lane >= (uint32_t)d) v += t;
  }
  return v;
}

// Sum over the wave's lanes (every lane active): the device library's DPP
// reduction (6 DPP adds + 2 readlanes) instead of 6 ds_bpermute rounds.
extern "C" __device__ uint32_t __ockl_wfred_add_u32(uint32_t);
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) { return __ockl_wfred_add_u32(v); }

// Raise the log-overflow flag: a relaxed check first and a plain store (the
// flag only ever goes 0 -> 1 inside a round), so that a full log does not
// put every wave of the grid behind one atomic on one word.
__device__ __forceinline__ void note_overflow(const RoundParams& p, uint32_t lane) {
  if (lane == 0 && __hip_atomic_load(p.log_overflow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
    __hip_atomic_store(p.log_overflow, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// End-of-round StatusUpdate emission (processor.go:111) for one wave. Status
// comes from the final A plane: after slot j, A_j = A_final ^ parity(E at
// later slots) (only flips change A); a record finalized this round has a
// single E bit (count 127 -> 128 cannot follow a flip within 16 votes).
//  * a lane with >= dense_min(K) updates (6 at k=8) writes one dense record
//    (kernels.h: key, E_0..E_{K-1}, A, died; 48 B at k=8) — a finalization
//    storm costs ~3 B per update instead of 8;
//  * the other lanes' updates are single packed words: one atomic per wave on
//    a sharded counter reserves the wave's total, then each iteration lets
//    every lane with updates left write one entry into consecutive slots
//    (mbcnt over the active lanes), one contiguous run per store instruction.
// The log order is irrelevant: the packed key sorts to the canonical (round,
// node, slot, target) order on fetch. Returns the bytes written (wave-uniform)
// and adds the wave's update count to *updates.
template <int K>
__device__ __forceinline__ uint32_t emit_updates(const RoundParams& p, uint32_t wave_id, uint32_t lane,
                                                 uint32_t node, uint32_t tbase, const uint32_t (&E)[K],
                                                 uint32_t A_final, uint32_t died, uint32_t& updates) {
  uint32_t any = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) any |= E[j];
  if (__ballot(any != 0u) == 0ull) return 0u;
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) cnt += (uint32_t)__popc(E[j]);
  constexpr uint32_t DW = dense_words(K);
  const bool dense = cnt >= p.dense_min;
  const uint64_t dl = __ballot(dense);
  const uint32_t tot_u = wave_sum(cnt), tot_s = wave_sum(dense ? 0u : cnt);
  const uint32_t tot_d = (uint32_t)__popcll(dl);
  updates += tot_u;
  if (p.ablate_emit == 1u) return 0u;  // diagnostics: the cost of the round without its log stores
  const uint32_t shard = wave_id % p.log_shards;
  uint32_t base = 0, dbase = 0;
  if (p.ablate_emit == 2u) {  // diagnostics: stores at made-up positions, no reserving atomic (log invalid)
    base = p.log_cap > 8192u ? (wave_id * 509u) % (p.log_cap - 4096u) : 0u;
    dbase = p.dlog_cap > 128u ? (wave_id * 131u) % (p.dlog_cap - 64u) : 0u;
  } else if (lane == 0) {
    if (tot_s) base = atomicAdd(&p.log_count[shard * kCtrStride], tot_s);
    if (tot_d) dbase = atomicAdd(&p.dlog_count[shard * kCtrStride], tot_d);
  }
  base = (uint32_t)__shfl((int)base, 0, 64);
  dbase = (uint32_t)__shfl((int)dbase, 0, 64);
  bool ovf = false;
  if (dense) {
    const uint32_t pos = dbase + __builtin_amdgcn_mbcnt_hi((uint32_t)(dl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dl, 0u));
    if (pos < p.dlog_cap) {
      uint32_t* rec = reinterpret_cast<uint32_t*>(p.dlog + ((size_t)shard * p.dlog_cap + pos) * DW);
      const uint64_t key = pack_update(p.round_rel, node, 0u, tbase, 0u, p.round_shift);
      rec[0] = (uint32_t)key;
      rec[1] = (uint32_t)(key >> 32);
#pragma unroll
      for (int j = 0; j < K; ++j) rec[2 + j] = E[j];
      rec[2 + K] = A_final;
      rec[3 + K] = died;
    } else {
      ovf = true;
    }
  }
  if (tot_s) {
    uint32_t Aj[K];
    uint32_t par = 0;
#pragma unroll
    for (int j = K - 1; j >= 0; --j) {
      Aj[j] = A_final ^ par;
      par ^= E[j];
    }
    uint64_t* dst = p.log + (size_t)shard * p.log_cap;
    uint32_t run = base;  // wave-uniform
    if (base >= p.log_cap) {  // shard already full: nothing can be stored
      ovf = true;
    } else {
      for (int j = 0; j < K; ++j) {  // not unrolled (data-dependent inner loop); E/Aj stay in VGPRs
        uint32_t e = dense ? 0u : E[j];
        for (;;) {
          const uint64_t act = __ballot(e != 0u);
          if (act == 0ull) break;
          if (e) {
            const uint32_t bit = (uint32_t)__ffs(e) - 1u;
            e &= e - 1u;
            const uint32_t a = (Aj[j] >> bit) & 1u;
            const uint32_t st = ((died >> bit) & 1u) ? (a ? 3u : 0u) : (a ? 2u : 1u);  // vote.go:77-91
            const uint32_t pos = run + __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
            if (pos < p.log_cap)
              dst[pos] = pack_update(p.round_rel, node, (uint32_t)j, tbase + bit, st, p.round_shift);
            else
              ovf = true;
          }
          run += (uint32_t)__popcll(act);
        }
      }
    }
  }
  if (__ballot(ovf) != 0ull) note_overflow(p, lane);
  // bytes actually stored (wave-uniform): entries past a full shard were dropped
  const uint32_t st_s = base >= p.log_cap ? 0u : min(tot_s, p.log_cap - base);
  const uint32_t st_d = dbase >= p.dlog_cap ? 0u : min(tot_d, p.dlog_cap - dbase);
  return 8u * st_s + 8u * DW * st_d;
}

// Per-wave counters: regsiterVote applications (the metric numerator) and the
// algorithmic bytes this wave moved (state planes actually read/written,
// gathered vote words, the published word, the StatusUpdate log bytes written).
// StatusUpdate emission without LDS staging (k_round_sweep's warm modes,
// where staging registers spill, and k_round_node): the same log as
// emit_updates, but a sparse lane walks its own updates (fewer than dense_min) one per iteration
// at its exclusive prefix, so the wave runs max(updates per sparse lane)
// iterations instead of one ballot loop per slot. A record emits at most two
// updates per round at k <= 8 (two flips are >= 6 votes apart; a record that
// finalizes does not flip in the same round), so its status
// after an update is A_final, flipped back once for the first of two (T: the
// records with two updates, S: those whose first was already written).
template <int K>
__device__ __forceinline__ uint32_t emit_updates_flat(const RoundParams& p, uint32_t wave_id, uint32_t lane,
                                                      uint32_t node, uint32_t tbase, const uint32_t (&E)[K],
                                                      uint32_t A_final, uint32_t died, uint32_t& updates,
                                                      uint32_t round_rel) {
  static_assert(K <= 8, "two updates per record per round at most: k <= 8 (and no finalization, died = 0, unless k = 8)");
  uint32_t any = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) any |= E[j];
  if (__ballot(any != 0u) == 0ull) return 0u;
  uint32_t cnt = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) cnt += (uint32_t)__popc(E[j]);
  constexpr uint32_t DW = dense_words(K);
  const bool dense = cnt >= p.dense_min;
  const uint64_t dl = __ballot(dense);
  const uint32_t scnt = dense ? 0u : cnt;
  const uint32_t incl = wave_incl_scan(scnt, lane);
  const uint32_t tot_s = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  const uint32_t tot_d = (uint32_t)__popcll(dl);
  updates += wave_sum(cnt);
  if (p.ablate_emit == 1u) return 0u;  // diagnostics: the cost of the round without its log stores
  const uint32_t shard = wave_id % p.log_shards;
  uint32_t base = 0, dbase = 0;
  if (p.ablate_emit == 2u) {  // diagnostics: stores at made-up positions, no reserving atomic (log invalid)
    base = p.log_cap > 8192u ? (wave_id * 509u) % (p.log_cap - 4096u) : 0u;
    dbase = p.dlog_cap > 128u ? (wave_id * 131u) % (p.dlog_cap - 64u) : 0u;
  } else if (lane == 0) {
    if (tot_s) base = atomicAdd(&p.log_count[shard * kCtrStride], tot_s);
    if (tot_d) dbase = atomicAdd(&p.dlog_count[shard * kCtrStride], tot_d);
  }
  base = (uint32_t)__builtin_amdgcn_readfirstlane((int)base);
  dbase = (uint32_t)__builtin_amdgcn_readfirstlane((int)dbase);
  const uint32_t st_d = dbase >= p.dlog_cap ? 0u : min(tot_d, p.dlog_cap - dbase);
  const uint32_t st_s = base >= p.log_cap ? 0u : min(tot_s, p.log_cap - base);
  const bool ovf = st_d < tot_d || st_s < tot_s;
  if (dense) {
    const uint32_t pos = dbase + __builtin_amdgcn_mbcnt_hi((uint32_t)(dl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)dl, 0u));
    if (pos < p.dlog_cap) {
      uint32_t* rec = reinterpret_cast<uint32_t*>(p.dlog + ((size_t)shard * p.dlog_cap + pos) * DW);
      const uint64_t key = pack_update(round_rel, node, 0u, tbase, 0u, p.round_shift);
      rec[0] = (uint32_t)key;
      rec[1] = (uint32_t)(key >> 32);
#pragma unroll
      for (int j = 0; j < K; ++j) rec[2 + j] = E[j];
      rec[2 + K] = A_final;
      rec[3 + K] = died;
    }
  }
  if (tot_s) {
    // T: records with two updates this round; nz: slots with updates left
    uint32_t seen = 0u, T = 0u, nz = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      T |= seen & E[j];
      seen |= E[j];
      nz |= (E[j] != 0u ? 1u : 0u) << j;
    }
    if (dense) nz = 0u;
    uint64_t* const dst = p.log + (size_t)shard * p.log_cap;
    uint32_t pos = base + incl - scnt;  // this lane's first entry
    const uint32_t end = base + st_s;   // entries at or past it were dropped (overflow)
    uint32_t S = 0u, j = 0u, cur = 0u;
    const uint64_t hi = ((uint64_t)round_rel << p.round_shift) | ((uint64_t)node << 28);
    for (uint32_t r = 0; r < 64u; ++r) {
      const bool more = r < scnt;
      if (__ballot(more) == 0ull) break;
      if (more) {
        if (cur == 0u) {  // next slot with updates
          j = (uint32_t)__ffs(nz) - 1u;
          nz &= nz - 1u;
          cur = E[0];
#pragma unroll
          for (int q = 1; q < K; ++q) cur = j == (uint32_t)q ? E[q] : cur;
        }
        const uint32_t bit = (uint32_t)__ffs(cur) - 1u;
        cur &= cur - 1u;
        const uint32_t m = 1u << bit;
        const uint32_t a = ((A_final ^ (T & ~S)) >> bit) & 1u;  // A after slot j (vote.go:77-91)
        S |= m;
        const uint32_t st = (died & m) ? (a ? 3u : 0u) : (a ? 2u : 1u);
        if (pos < end) dst[pos] = hi | ((uint64_t)j << 24) | ((uint64_t)(tbase + bit) << 2) | st;
        ++pos;
      }
    }
  }
  if (__ballot(ovf) != 0ull) note_overflow(p, lane);
  // bytes actually stored (wave-uniform): entries past a full shard were dropped
  return 8u * st_s + 8u * DW * st_d;
}

// StatusUpdate emission with medium records (p.med, k <= 8): every lane with
// updates stores exactly one entry — a single packed word (1 update), a
// medium record (2..kMedMax: key + 10 bits per update, kernels.h) or a dense
// record (more) — at its rank among the wave's lanes of that kind, so each
// kind is one contiguous run per wave written by one store instruction (the
// dense record: three dwordx4). No per-update store loop: a medium lane folds
// its updates into the payload in registers. Statuses as emit_updates_flat (A
// after slot j = A_final, flipped back for the first of a record's two
// updates; vote.go:77-91). Returns the bytes stored (wave-uniform).
// E[j] for a per-lane slot j: a 3-level mux at K = 8 (7 selects on 3 masks instead of a 7-step
// compare-and-select chain), the chain otherwise.
template <int K>
__device__ __forceinline__ uint32_t select_slot(const uint32_t (&E)[K], uint32_t j) {
  if constexpr (K == 8) {
    const bool b0 = (j & 1u) != 0u, b1 = (j & 2u) != 0u, b2 = (j & 4u) != 0u;
    const uint32_t a0 = b0 ? E[1] : E[0], a1 = b0 ? E[3] : E[2], a2 = b0 ? E[5] : E[4], a3 = b0 ? E[7] : E[6];
    const uint32_t c0 = b1 ? a1 : a0, c1 = b1 ? a3 : a2;
    return b2 ? c1 : c0;
  } else {
    uint32_t cur = E[0];
#pragma unroll
    for (int t = 1; t < K; ++t) cur = j == (uint32_t)t ? E[t] : cur;
    return cur;
  }
}

// Lowest set bit's index, 0xFFFFFFFF for 0 (v_ffbl_b32 as is: no zero test and select around it)
__device__ __forceinline__ uint32_t ffbl_u32(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// bit (b & 31) of x
__device__ __forceinline__ uint32_t bfe1(uint32_t x, uint32_t b) { return __builtin_amdgcn_ubfe(x, b & 31u, 1u); }
// E[j & 7] as a bit-select tree: 7 v_bfi_b32 on the sign-extended bits of j (no compare writing a lane
// mask, so no VALU-wrote-SGPR wait states before the selects)
template <int K>
__device__ __forceinline__ uint32_t select_slot_bfi(const uint32_t (&E)[K], uint32_t j) {
  if constexpr (K != 8) return select_slot<K>(E, j);
  else {
  const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)j, 0u, 1u);
  const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)j, 1u, 1u);
  const uint32_t m2 = (uint32_t)__builtin_amdgcn_sbfe((int)j, 2u, 1u);
  const uint32_t a0 = (m0 & E[1]) | (~m0 & E[0]), a1 = (m0 & E[3]) | (~m0 & E[2]);
  const uint32_t a2 = (m0 & E[5]) | (~m0 & E[4]), a3 = (m0 & E[7]) | (~m0 & E[6]);
  const uint32_t c0 = (m1 & a1) | (~m1 & a0), c1 = (m1 & a3) | (~m1 & a2);
  return (m2 & c1) | (~m2 & c0);
  }
}

#ifndef AVK_MED_WALK
#define AVK_MED_WALK 1
#endif
// StatusUpdate log stores (k = 8 slot-record path) non-temporal: the log is read only after the
// round, so its lines need not displace the gathered preference rows in L2 / MALL (A/B,
// profiles/r04/session11/ablognt.log: C4p -3.1 / -3.7 %, C4 -3.6 %, C4pb -1.7 % per epoch)
#ifndef AVK_LOG_NT
#define AVK_LOG_NT 1
#endif

// A/B build knob: lanes with at least this many updates log a dense record (0: the default, above
// kMedMax; 2: no medium records, the walk that folds a lane's updates into one is never run)
#ifndef AVK_MED_DENSE_MIN
#define AVK_MED_DENSE_MIN 0
#endif

// The reservation half of emit_updates_med: per-lane update count, the wave's
// per-kind totals and the three reserving atomics, issued but not waited for
// (their results are read in emit_store_med). A caller that issues it before
// its plane stores waits for the atomics' return only, not for those stores
// (vmcnt counts in issue order: an atomic issued after the stores would make
// the wave wait for every store of the tile first).
struct EmitRes {
  uint32_t tot_s, tot_m, tot_d;  // wave-uniform: lanes of each kind
  uint32_t raw;                  // lanes 0, 1, 2: the singles / medium / dense atomics' results (one VGPR)
  uint32_t lk;                   // per lane (AVK_MED_S4): slots with updates (bits 0-7), kind (bits 8-9)
  bool any;                      // wave-uniform: some lane has an update
};

__device__ __forceinline__ uint32_t lane_updates8(const uint32_t* E, int K) {
  uint32_t c = 0;
  for (int j = 0; j < K; ++j) c += (uint32_t)__popc(E[j]);
  return c;
}

// Medium records, two formats (kernels.h kMedS4 selects; the log readers in log_ops.hip follow it):
//  * AVK_MED_S4 = 1 (default): a lane whose updates lie in at most 4 slots (3 if a record of it was
//    deleted this round) stores a 32-byte slot record {key, slot mask | died flag, A_final, up to 4
//    E_j words in slot order (the 4th: the died plane when flagged)}: the slot words are compacted
//    by a shift-in network, no per-update work at all;
//  * AVK_MED_S4 = 0: a 16-byte record folding up to kMedMax updates into 10-bit fields, walked one
//    update per step (the round-3 form, kept for A/B).
constexpr uint32_t kLkSingle = 1u << 8, kLkMed = 2u << 8, kLkDense = 3u << 8;
constexpr uint32_t kLkTwo = 1u << 10;  // a single-word lane with two updates (SMAX = 2)

// SMAX (AVK_MED_S4, k = 8): a lane with at most SMAX updates logs them as single packed words (8 B
// each) instead of a 32-B slot record. At 2 (round 6, build knob AVK_SINGLE_MAX for k_round_sweep)
// two words take 16 B where the record took 32, and in conflicting rounds a third of the lanes have
// exactly two updates (the pair's two targets flip together): C4p's log shrinks from 25.6 to 20.3 B
// per lane. The store needs no per-update loop (the second update is the first's slot's next bit, or
// the next slot's only bit). Measured level (C4p epoch 6.43-6.50 ms at 1 and 2, C4 3.58-3.65, C4pb
// 6.49-6.52; profiles/r06/delivery/ab_smax.log): the storm rounds are not paced by the log's bytes,
// and two words are two entries for the delivery encoder, so 1 stays the default.
#ifndef AVK_SINGLE_MAX
#define AVK_SINGLE_MAX 1
#endif

template <int K, int SMAX = 1>
__device__ __forceinline__ EmitRes emit_reserve_med(const RoundParams& p, uint32_t shard, uint32_t lane,
                                                    const uint32_t (&E)[K], uint32_t died, uint32_t& updates) {
  static_assert(SMAX == 1 || SMAX == 2, "one or two single words per lane");
  EmitRes r;
  uint32_t any = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) any |= E[j];
  r.any = __ballot(any != 0u) != 0ull;
  r.tot_s = r.tot_m = r.tot_d = 0u;
  r.raw = 0u;
  r.lk = 0u;
  if (!r.any) return r;
  const uint32_t cnt = lane_updates8(E, K);
#if AVK_MED_S4
  uint32_t nz = 0u;
#pragma unroll
  for (int j = 0; j < K; ++j) nz |= (E[j] != 0u ? 1u : 0u) << j;
  const uint32_t ns = (uint32_t)__popc(nz);
  // (A/B option wave_dense: a wave with many lanes holding updates logs them all dense)
  const bool wd = p.wave_dense != 0u && (uint32_t)__popcll(__ballot(cnt != 0u)) >= p.wave_dense;
  const bool two = !wd && SMAX >= 2 && cnt == 2u;
  const bool single = !wd && (cnt == 1u || two);
  const bool med = !wd && cnt > (uint32_t)SMAX && (ns <= 3u || (ns == 4u && died == 0u));
  const bool dense = wd ? cnt != 0u : cnt > (uint32_t)SMAX && !med;
  r.lk = nz | (single ? kLkSingle : med ? kLkMed : dense ? kLkDense : 0u) | (two ? kLkTwo : 0u);
#else
  (void)died;
  const uint32_t dmin = AVK_MED_DENSE_MIN ? AVK_MED_DENSE_MIN : max(p.dense_min, kMedMax + 1u);
  const bool dense = cnt >= dmin, med = !dense && cnt >= 2u, single = cnt == 1u;
#endif
  r.tot_d = (uint32_t)__popcll(__ballot(dense));
  r.tot_m = (uint32_t)__popcll(__ballot(med));
  r.tot_s = (uint32_t)__popcll(__ballot(single));
#if AVK_MED_S4
  if constexpr (SMAX >= 2) r.tot_s += (uint32_t)__popcll(__ballot(two));  // words, not lanes
#endif
  updates += wave_sum(cnt);
  if (p.ablate_emit == 1u) return r;  // diagnostics: the cost of the round without its log stores
  // one atomic instruction, lanes 0 / 1 / 2 reserving the singles / medium / dense runs
  // The three counter arrays are one allocation, [singles | medium | dense] x kLogShards x kCtrStride (engine.cpp),
  // so lane q's counter is an offset from one kernel argument: a per-lane choice among three pointer
  // arguments compiles to a load of the chosen argument from the kernarg segment, and the wait for
  // that load (vmcnt(0)) also waited for every store and load the wave had in flight.
  const uint32_t want = lane == 0 ? r.tot_s : lane == 1 ? r.tot_m : lane == 2 ? r.tot_d : 0u;
  // (opaque: the per-lane offset is formed here, not hoisted out of the caller's tile loop as a
  // 64-bit address that spills to scratch and is reloaded, with a vmcnt(0) wait, before each atomic)
  uint32_t cofs = (min(lane, 2u) * kLogShards + shard) * kCtrStride;
  asm volatile("" : "+v"(cofs));
  uint32_t* const ctr = p.log_count + cofs;
  if (p.ablate_emit >= 2u) {  // diagnostics (log invalid): stores at made-up per-wave positions; 3: the
    // reserving atomic still issued, its result unused (no wait for it)
    const uint32_t wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.log_cap);
    const uint32_t c1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.mlog_cap);
    const uint32_t c2 = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.dlog_cap);
    const uint32_t cap = lane == 0 ? c0 : lane == 1 ? c1 : c2;
    r.raw = cap > 8192u ? (wv * 509u) % (cap - 4096u) : 0u;
    if (p.ablate_emit == 3u && want) atomicAdd(ctr, want);
    return r;
  }
  if (want) r.raw = atomicAdd(ctr, want);
  return r;
}

// The store half: every lane with updates stores its one entry at its rank among the wave's lanes
// of its kind (see emit_updates_med). Returns the bytes stored (wave-uniform).
template <int K, int SMAX = 1>
__device__ __forceinline__ uint32_t emit_store_med(const RoundParams& p, uint32_t shard, uint32_t lane,
                                                   uint32_t node, uint32_t tbase, const uint32_t (&E)[K],
                                                   uint32_t A_final, uint32_t died, const EmitRes& r,
                                                   uint32_t round_rel) {
  static_assert(K <= 8, "slot fits 3 bits of a medium field; two updates per record per round at most");
  if (!r.any || p.ablate_emit == 1u) return 0u;
#if AVK_MED_S4
  if constexpr (K == 8) {
    const uint32_t kind = r.lk & (3u << 8), nz = r.lk & 0xFFu;
    const bool dense = kind == kLkDense, med = kind == kLkMed, single = kind == kLkSingle;
    const bool two = SMAX >= 2 && (r.lk & kLkTwo) != 0u;
    const uint64_t dl = __ballot(dense), ml = __ballot(med), sl = __ballot(single);
    const uint64_t tl = SMAX >= 2 ? __ballot(two) : 0ull;
    const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 0);
    const uint32_t mbase = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 1);
    const uint32_t dbase = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 2);
    const uint32_t st_d = dbase >= p.dlog_cap ? 0u : min(r.tot_d, p.dlog_cap - dbase);
    const uint32_t st_m = mbase >= p.mlog_cap ? 0u : min(r.tot_m, p.mlog_cap - mbase);
    const uint32_t st_s = base >= p.log_cap ? 0u : min(r.tot_s, p.log_cap - base);
    const bool ovf = st_d < r.tot_d || st_m < r.tot_m || st_s < r.tot_s;
    const uint64_t key = pack_update(round_rel, node, 0u, tbase, 0u, p.round_shift);
    const uint64_t mine = dense ? dl : med ? ml : sl;
    uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
    if (SMAX >= 2 && single)  // the lower lanes' second words come first
      rank += __builtin_amdgcn_mbcnt_hi((uint32_t)(tl >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)tl, 0u));
    if (dense) {
      if (rank < st_d) {
        constexpr uint32_t DW = dense_words(K);
        uint64_t* const rec = p.dlog + ((size_t)shard * p.dlog_cap + dbase + rank) * DW;
        u32x4* const q = reinterpret_cast<u32x4*>(rec);
        pst4<AVK_LOG_NT>(q, u32x4{(uint32_t)key, (uint32_t)(key >> 32), E[0], E[1]});
        pst4<AVK_LOG_NT>(q + 1, u32x4{E[2], E[3], E[4], E[5]});
        pst4<AVK_LOG_NT>(q + 2, u32x4{E[6], E[7], A_final, died});
      }
    } else if (med || single) {  // (lanes without updates skip the network: a wave of dense lanes skips it)
      // the first 4 slots with updates, in slot order: shift in from the last slot down
      uint32_t o0 = 0u, o1 = 0u, o2 = 0u, o3 = 0u;
#pragma unroll
      for (int j = K - 1; j >= 0; --j) {
        const bool h = E[j] != 0u;
        o3 = h ? o2 : o3;
        o2 = h ? o1 : o2;
        o1 = h ? o0 : o1;
        o0 = h ? E[j] : o0;
      }
      if (med) {
        if (rank < st_m) {
          const bool hasd = died != 0u;  // then at most 3 slots: the died plane takes the 4th word
          u32x4* const q = reinterpret_cast<u32x4*>(p.mlog + ((size_t)shard * p.mlog_cap + mbase + rank) * 4u);
          pst4<AVK_LOG_NT>(q, u32x4{(uint32_t)key, (uint32_t)(key >> 32), nz | (hasd ? kMedS4Died : 0u), A_final});
          pst4<AVK_LOG_NT>(q + 1, u32x4{o0, o1, o2, hasd ? died : o3});
        }
      } else if (single && rank < st_s) {
        // the first update: slot ffbl(nz), record ffbl(o0); status from A_final and died (vote.go:77-91)
        const uint32_t j = ffbl_u32(nz), bit = ffbl_u32(o0);
        uint32_t a = bfe1(A_final, bit);
        uint64_t* const w = p.log + (size_t)shard * p.log_cap + base + rank;
        if (SMAX >= 2 && two) {
          // the second: o0's next bit (same slot), else the next slot's only bit. A record with both
          // (the same bit in two slots: a flip and its flip back) had A_final ^ 1 after the first
          const uint32_t rest = o0 & (o0 - 1u);
          const uint32_t j2 = rest ? j : ffbl_u32(nz & (nz - 1u)), bit2 = ffbl_u32(rest ? rest : o1);
          a ^= (j2 != j && bit2 == bit) ? 1u : 0u;
          const uint32_t a2 = bfe1(A_final, bit2), d2 = bfe1(died, bit2);
          const uint64_t word2 = key + ((uint64_t)j2 << 24) + ((uint64_t)bit2 << 2) + ((a2 << 1) | (~(a2 ^ d2) & 1u));
          if (rank + 1u < st_s) {
            if constexpr (AVK_LOG_NT) __builtin_nontemporal_store(word2, w + 1); else w[1] = word2;
          }
        }
        const uint32_t d = bfe1(died, bit);
        const uint32_t st = (a << 1) | (~(a ^ d) & 1u);
        const uint64_t word = key + ((uint64_t)j << 24) + ((uint64_t)bit << 2) + st;
        if constexpr (AVK_LOG_NT) __builtin_nontemporal_store(word, w); else *w = word;
      }
    }
    if (__ballot(ovf) != 0ull) note_overflow(p, lane);
    return 8u * st_s + 32u * st_m + 8u * dense_words(K) * st_d;
  }
#endif
  const uint32_t cnt = lane_updates8(E, K);
  const uint32_t dmin = AVK_MED_DENSE_MIN ? AVK_MED_DENSE_MIN : max(p.dense_min, kMedMax + 1u);
  const bool dense = cnt >= dmin, med = !dense && cnt >= 2u, single = cnt == 1u;
  const uint64_t dl = __ballot(dense), ml = __ballot(med), sl = __ballot(single);
  const uint32_t tot_d = r.tot_d, tot_m = r.tot_m, tot_s = r.tot_s;
  const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 0);
  const uint32_t mbase = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 1);
  const uint32_t dbase = (uint32_t)__builtin_amdgcn_readlane((int)r.raw, 2);
  const uint32_t st_d = dbase >= p.dlog_cap ? 0u : min(tot_d, p.dlog_cap - dbase);
  const uint32_t st_m = mbase >= p.mlog_cap ? 0u : min(tot_m, p.mlog_cap - mbase);
  const uint32_t st_s = base >= p.log_cap ? 0u : min(tot_s, p.log_cap - base);
  const bool ovf = st_d < tot_d || st_m < tot_m || st_s < tot_s;
  const uint64_t key = pack_update(round_rel, node, 0u, tbase, 0u, p.round_shift);
  const uint64_t mine = dense ? dl : med ? ml : sl;
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
  if (dense) {
    if (rank < st_d) {
      constexpr uint32_t DW = dense_words(K);
      uint32_t w[2 * DW];
      w[0] = (uint32_t)key;
      w[1] = (uint32_t)(key >> 32);
#pragma unroll
      for (int j = 0; j < K; ++j) w[2 + j] = E[j];
      w[2 + K] = A_final;
      w[3 + K] = died;
#pragma unroll
      for (uint32_t i = 4 + K; i < 2 * DW; ++i) w[i] = 0u;
      uint64_t* const rec = p.dlog + ((size_t)shard * p.dlog_cap + dbase + rank) * DW;
      if constexpr (DW % 2u == 0u) {  // 16-B aligned records (k = 8: 48 B, three dwordx4)
#pragma unroll
        for (uint32_t i = 0; i < DW / 2u; ++i)
          reinterpret_cast<u32x4*>(rec)[i] = u32x4{w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]};
      } else {
#pragma unroll
        for (uint32_t i = 0; i < DW; ++i) rec[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
      }
    }
  } else if (AVK_MED_WALK && K == 8) {
    // T: records with two updates this round. The walk runs for the wave's largest count (one
    // wave-uniform test per step, no exec-mask branches); lanes past their own count (and dense or
    // update-less lanes) compute a field that is masked out. Per step: the next slot with updates
    // when the current one is used up (a bit-select mux on the slot index, select_slot_bfi), its
    // lowest update, the status from two planes fixed per walk (a = A after slot j, vote.go:77-91:
    // A_final flipped back for the first of a record's two updates; status bit 0 = ~(a ^ died)).
    uint32_t seen = 0u, T = 0u, nz = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      T |= seen & E[j];
      seen |= E[j];
      nz |= (E[j] != 0u ? 1u : 0u) << j;
    }
    const uint32_t cm = dense ? 0u : cnt;  // updates this lane folds into its payload
    const uint32_t Ad = A_final ^ died;
    uint32_t S = 0u, j = 0u, cur = 0u;
    uint64_t pl = cnt;
#pragma unroll
    for (uint32_t q = 0; q < kMedMax; ++q) {
      if (__ballot(q < cm) == 0ull) break;  // wave-uniform
      const bool adv = cur == 0u;
      const uint32_t jn = ffbl_u32(nz);
      j = adv ? jn : j;
      nz = adv ? nz & (nz - 1u) : nz;
      cur = adv ? select_slot_bfi<K>(E, jn) : cur;
      const uint32_t bit = ffbl_u32(cur);
      cur &= cur - 1u;
      const uint32_t first = T & ~S;  // records whose first of two updates is still ahead
      S |= 1u << bit;
      const uint32_t st = (bfe1(A_final ^ first, bit) << 1) | bfe1(~(Ad ^ first), bit);
      const uint32_t f = (j << 7) | (bit << 2) | st;
      pl |= (uint64_t)(q < cm ? f : 0u) << (4u + 10u * q);
    }
    if (med) {
      if (rank < st_m) {
        u32x4* rec = reinterpret_cast<u32x4*>(p.mlog + ((size_t)shard * p.mlog_cap + mbase + rank) * 2u);
        *rec = u32x4{(uint32_t)key, (uint32_t)(key >> 32), (uint32_t)pl, (uint32_t)(pl >> 32)};
      }
    } else if (single && rank < st_s) {
      p.log[(size_t)shard * p.log_cap + base + rank] = med_word(key, (uint32_t)(pl >> 4) & 1023u);
    }
  } else if (cnt) {
    // T: records with two updates this round; walk the updates in slot order
    uint32_t seen = 0u, T = 0u, nz = 0u;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      T |= seen & E[j];
      seen |= E[j];
      nz |= (E[j] != 0u ? 1u : 0u) << j;
    }
    uint32_t S = 0u, j = 0u, cur = 0u;
    uint64_t pl = cnt;  // payload: n, then one field per update
#pragma unroll
    for (uint32_t q = 0; q < kMedMax; ++q) {
      if (q < cnt) {
        if (cur == 0u) {  // next slot with updates
          j = (uint32_t)__ffs(nz) - 1u;
          nz &= nz - 1u;
          cur = select_slot<K>(E, j);
        }
        const uint32_t bit = (uint32_t)__ffs(cur) - 1u;
        cur &= cur - 1u;
        const uint32_t m = 1u << bit;
        const uint32_t a = ((A_final ^ (T & ~S)) >> bit) & 1u;  // A after slot j (vote.go:77-91)
        S |= m;
        const uint32_t st = (died & m) ? (a ? 3u : 0u) : (a ? 2u : 1u);
        pl |= (uint64_t)med_field(j, bit, st) << (4u + 10u * q);
      }
    }
    if (med) {
      if (rank < st_m) {
        u32x4* rec = reinterpret_cast<u32x4*>(p.mlog + ((size_t)shard * p.mlog_cap + mbase + rank) * 2u);
        *rec = u32x4{(uint32_t)key, (uint32_t)(key >> 32), (uint32_t)pl, (uint32_t)(pl >> 32)};
      }
    } else if (rank < st_s) {
      p.log[(size_t)shard * p.log_cap + base + rank] = med_word(key, (uint32_t)(pl >> 4) & 1023u);
    }
  }
  if (__ballot(ovf) != 0ull) note_overflow(p, lane);
  return 8u * st_s + 16u * st_m + 8u * dense_words(K) * st_d;
}

// StatusUpdate emission with medium records (p.med, k <= 8): every lane with
// updates stores exactly one entry — a single packed word (1 update), a
// medium record (2..kMedMax: key + 10 bits per update, kernels.h) or a dense
// record (more) — at its rank among the wave's lanes of that kind, so each
// kind is one contiguous run per wave written by one store instruction (the
// dense record: three dwordx4). No per-update store loop: a medium lane folds
// its updates into the payload in registers. Statuses as emit_updates_flat (A
// after slot j = A_final, flipped back for the first of a record's two
// updates; vote.go:77-91). Returns the bytes stored (wave-uniform).
template <int K>
__device__ __forceinline__ uint32_t emit_updates_med(const RoundParams& p, uint32_t shard, uint32_t lane,
                                                     uint32_t node, uint32_t tbase, const uint32_t (&E)[K],
                                                     uint32_t A_final, uint32_t died, uint32_t& updates,
                                                     uint32_t round_rel) {
  const EmitRes r = emit_reserve_med<K>(p, shard, lane, E, died, updates);
  return emit_store_med<K>(p, shard, lane, node, tbase, E, A_final, died, r, round_rel);
}

__device__ __forceinline__ void count_stats(const RoundParams& p, uint32_t wave_id, uint32_t lane, uint32_t applied,
                                            bool active, uint32_t bytes_per_lane, uint32_t emitted_bytes,
                                            uint32_t updates, uint32_t died) {
  const uint32_t s = wave_sum(applied);
  const uint32_t f = wave_sum(__popc(died));
  const uint32_t nact = (uint32_t)__popcll(__ballot(active));
  if (lane == 0) {
    const uint32_t shard = wave_id % p.log_shards;
    if (s) atomicAdd(&p.applied[shard], (unsigned long long)s);
    if (f) atomicAdd(&p.finalized[shard], (unsigned long long)f);
    atomicAdd(&p.bytes[shard], (unsigned long long)nact * bytes_per_lane + emitted_bytes);
    if (updates) atomicAdd(&p.upd_count[shard], updates);
  }
}

}  // namespace
}  // namespace avk
