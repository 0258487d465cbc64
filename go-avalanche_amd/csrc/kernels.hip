// CDNA4 (gfx950) kernels of the batched Avalanche voting engine.
//
// The hot path is one round of go-avalanche's poll loop for every simulated
// node at once: peer sampling (processor.go:173-182 / main.go:110-116 replaced
// by a counter-RNG k-peer draw), the peer-preference gather (main.go:168-192
// responder), the VoteRecord shift-register / confidence update
// (vote.go:54-91) inside RegisterVotes (processor.go:92-117) and StatusUpdate
// emission (processor.go:111) with deletion on finalization (:114-116).
//
// Records are bit-sliced: one lane owns 32 records (a block of 32 targets of
// one node) as 25 u32 planes, so every VALU instruction advances 32
// VoteRecords. Nothing here is a dense contraction; there is no MFMA. The
// kernels are HBM-bound streaming kernels (DESIGN.md "Roofline").
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dev_scan.h"
#include "kernels.h"
#include "round_common.h"

namespace avk {
namespace {
// ---------------------------------------------------------------------------
// Body of the uncapped round kernel for one lane (one 32-record block).
// WARM (sim mode only): every consider plane of the wave's blocks is all-ones
// (each record has seen >= 8 votes and, with no replay / neutral vote ever
// applied in this engine, every consider bit shifted in was 1). Then the 7
// younger consider planes are neither loaded nor stored: 176 B per lane
// instead of 236 B at k=8. NT: non-temporal plane stream.
// ---------------------------------------------------------------------------
template <int K, bool REPLAY, bool WARM, bool NT>
__device__ __forceinline__ void round_fast_body(const RoundParams& p, uint32_t g, uint32_t lane, bool active,
                                                uint32_t b, uint32_t node) {
  St s;
  uint32_t* const tile = tile_of(p.planes, g);
  u32x4* const grp = reinterpret_cast<u32x4*>(tile) + lane;  // V0-3, V4-7, K0-3, K4-7 at +0, +64, +128, +192
  if (!active) {
    dead_state(s);
  } else {
    const u32x4 v0 = pld4<NT>(grp), v1 = pld4<NT>(grp + 64), k0 = pld4<NT>(grp + 128), k1 = pld4<NT>(grp + 192);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s.V[i] = v0[i];
      s.V[4 + i] = v1[i];
      s.K[i] = k0[i];
      s.K[4 + i] = k1[i];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) s.C[i] = WARM ? ~0u : pld<NT>(tile + plane_off(kPC + i, lane));
    s.A = pld<NT>(tile + plane_off(kPA, lane));
  }

  uint32_t w[K], cw[K], peer_of[K];
  if (REPLAY) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      w[j] = active ? p.replay[replay_idx(g, K, j, 0)] : 0u;
      cw[j] = active ? p.replay[replay_idx(g, K, j, 1)] : 0u;
    }
  } else {
    uint32_t peers[K];
    sample_peers<K>(p.seed, node, p.round, p.n_nodes, p.peer_mode, peers);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      // peer's published preference; the ablation (timing diagnostics only,
      // results invalid) reads the node's own row instead: coalesced, same count
      const uint32_t src = p.ablate_gather ? (node ^ (uint32_t)j) % p.n_nodes : peers[j];
      w[j] = active ? p.pref_in[(size_t)src * p.PS + b] : 0u;
      cw[j] = ~0u;  // honest/Byzantine votes are 0 or 1
      peer_of[j] = src - p.n0;  // local row of the peer (responder re-adds: single-engine networks only)
    }
  }
  const uint32_t vmask = active ? p.valid[b] : 0u;
  const uint32_t live0 = ~s.K[7];
  // a node whose run loop has returned (main.go:160-162) polls nothing
  const uint32_t nl = g / p.BL;
  const bool polls = !p.nopoll || !((p.nopoll[nl >> 5] >> (nl & 31u)) & 1u);
  const uint32_t P0 = polls ? live0 & vmask : 0u;

  uint32_t alive = P0, applied = 0, E[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    applied += __popc(alive);
    // the example's responder re-adds what it is queried for (main.go:175-177)
    if (!REPLAY && p.readd && alive) atomicOr(&p.readd[peer_of[j] * p.BL + b], alive);
    uint32_t fin;
    vote_step<false>(s, w[j], cw[j], alive, E[j], fin);
    alive &= ~fin;
  }
  const uint32_t died = P0 & ~alive;
  const uint32_t keep = live0 & ~P0;  // live but !IsValid() (processor.go:101-103) or not polling: untouched
  if (p.died_out && active) p.died_out[g] = died;

  if (active) {
    uint32_t Vo[8], Co[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) Vo[i] = Co[i] = 0u;
    if (keep) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        Vo[i] = tile[plane_off(kPV + i, lane)];
        if (!WARM) Co[i] = tile[plane_off(kPC + i, lane)];
      }
    }
    const uint32_t dead = ~(alive | keep);
    u32x4 v0, v1, k0, k1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v0[i] = (s.V[i] & alive) | (Vo[i] & keep);
      v1[i] = (s.V[4 + i] & alive) | (Vo[4 + i] & keep);
      k0[i] = s.K[i];
      k1[i] = s.K[4 + i];
    }
    pst4<NT>(grp, v0);
    pst4<NT>(grp + 64, v1);
    pst4<NT>(grp + 128, k0);
    pst4<NT>(grp + 192, k1);
    if (!WARM) {  // WARM: consider planes stay all-ones (dead records are canonical all-ones too)
#pragma unroll
      for (int i = 0; i < 8; ++i) pst<NT>(tile + plane_off(kPC + i, lane), (s.C[i] & alive) | (Co[i] & keep) | dead);
    }
    pst<NT>(tile + plane_off(kPA, lane), s.A);
    p.pref_out[(size_t)node * p.PS + b] =
        is_byz(p.byz, node) ? byz_pattern(p.round + 1u) : publish_word(s.A, s.K[7], p.pub_mode);
  }
  const uint32_t wave_id = g >> 6;
  uint32_t upd = 0;
  const uint32_t emitted = emit_updates<K>(p, wave_id, lane, node, p.t0 + b * 32u, E, s.A, died, upd);
  constexpr uint32_t plane_bytes = WARM ? (18u + 17u) * 4u : 2u * kPlanes * 4u;
  constexpr uint32_t bytes = plane_bytes + (REPLAY ? 8u : 4u) * K + 4u;
  count_stats(p, wave_id, lane, applied, active, bytes, emitted, upd, died);
}

// ---------------------------------------------------------------------------
// Round kernel, uncapped path (every node has <= 4096 live valid targets, so
// GetInvsForNextPoll never truncates: processor.go:165-167). One lane = one
// 32-record block; no cross-lane dependence except the emission scan.
// ---------------------------------------------------------------------------
template <int K, bool REPLAY>
__global__ __launch_bounds__(256) void k_round_fast(const RoundParams p) {
  const uint32_t g = blockIdx.x * 256u + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  if ((g & ~63u) >= p.L) return;  // whole wave beyond the last tile
  const bool active = g < p.L;
  const uint32_t nl = active ? g / p.BL : 0u;
  const uint32_t b = active ? g - nl * p.BL : 0u;
  const uint32_t node = p.n0 + nl;
  if (!REPLAY && p.warm_skip) {
    const uint32_t c7 = active ? *pw(p.planes, g, kPC + 7) : ~0u;
    if (__all(c7 == ~0u)) {  // wave-uniform
      if (p.plane_nt)
        round_fast_body<K, false, true, true>(p, g, lane, active, b, node);
      else
        round_fast_body<K, false, true, false>(p, g, lane, active, b, node);
      return;
    }
  }
  if (p.plane_nt)
    round_fast_body<K, REPLAY, false, true>(p, g, lane, active, b, node);
  else
    round_fast_body<K, REPLAY, false, false>(p, g, lane, active, b, node);
}

// ---------------------------------------------------------------------------
// Round kernel, capped path: one workgroup per node; per slot a workgroup
// prefix count of live valid records selects the first 4096 in ascending
// target order (GetInvsForNextPoll truncation, processor.go:165-167).
// ---------------------------------------------------------------------------
template <int K, bool REPLAY>
__device__ __forceinline__ void capped_node(const RoundParams& p, uint32_t nl, uint32_t (&wsum)[2][16]);

template <int K, bool REPLAY>
__global__ __launch_bounds__(1024) void k_round_capped(const RoundParams p) {
  __shared__ uint32_t wsum[2][16];
  if (!p.node_flags) {
    capped_node<K, REPLAY>(p, blockIdx.x, wsum);
    return;
  }
  // exact pass behind k_round_node: a small grid walks the nodes and takes
  // only the ones it flagged (an almost empty pass costs ~1-2 us, not the
  // dispatch of one workgroup per node)
  for (uint32_t nl = blockIdx.x; nl < p.NL; nl += gridDim.x) {
    const uint32_t f = p.node_flags[nl];  // workgroup-uniform
    if (f == 0u || f - 1u > p.exact_rel) continue;
    __syncthreads();
    if (threadIdx.x == 0 && !p.exact_keep) p.node_flags[nl] = 0u;
    capped_node<K, REPLAY>(p, nl, wsum);
    __syncthreads();  // wsum reuse by the next node
  }
}

template <int K, bool REPLAY>
__device__ __forceinline__ void capped_node(const RoundParams& p, uint32_t nl, uint32_t (&wsum)[2][16]) {
  const uint32_t b = threadIdx.x;
  const uint32_t lane = b & 63u, wave = b >> 6;
  const bool active = b < p.BL;
  const uint32_t g = nl * p.BL + b;
  const uint32_t node = p.n0 + nl;

  St s;
  if (active)
    load_state(p.planes, g, s);
  else
    dead_state(s);
  uint32_t w[K], cw[K];
  if (REPLAY) {
#pragma unroll
    for (int j = 0; j < K; ++j) {
      w[j] = active ? p.replay[replay_idx(g, K, j, 0)] : 0u;
      cw[j] = active ? p.replay[replay_idx(g, K, j, 1)] : 0u;
    }
  } else {
    uint32_t peers[K];
    sample_peers<K>(p.seed, node, p.round, p.n_nodes, p.peer_mode, peers);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      w[j] = active ? p.pref_in[(size_t)peers[j] * p.PS + b] : 0u;
      cw[j] = ~0u;
    }
  }
  const uint32_t vmask = active ? p.valid[b] : 0u;
  const uint32_t P0 = ~s.K[7] & vmask;

  uint32_t alive = P0, applied = 0, E[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t c = __popc(alive);
    const uint32_t incl = wave_incl_scan(c, lane);
    if (lane == 63u) wsum[j & 1][wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < wave; ++q) before += wsum[j & 1][q];
    const uint32_t excl = before + incl - c;
    uint32_t polled;
    if (excl >= kMaxPoll) {
      polled = 0u;
    } else if (excl + c <= kMaxPoll) {
      polled = alive;
    } else {  // keep the lowest (4096 - excl) set bits
      uint32_t x = alive;
      polled = 0u;
      for (uint32_t q = 0; q < kMaxPoll - excl; ++q) {
        const uint32_t low = x & (0u - x);
        polled |= low;
        x ^= low;
      }
    }
    applied += __popc(polled);
    uint32_t fin;
    vote_step<true>(s, w[j], cw[j], polled, E[j], fin);
    alive &= ~fin;
  }
  const uint32_t died = P0 & ~alive;
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      s.V[i] &= ~died;
      s.C[i] |= died;
    }
    store_state(p.planes, g, s);
    p.pref_out[(size_t)node * p.PS + b] =
        is_byz(p.byz, node) ? byz_pattern(p.round + 1u) : publish_word(s.A, s.K[7], p.pub_mode);
  }
  const uint32_t wave_id = nl * (blockDim.x >> 6) + wave;  // dense: matches log_shards sizing
  uint32_t upd = 0;
  const uint32_t emitted = emit_updates<K>(p, wave_id, lane, node, p.t0 + b * 32u, E, s.A, died, upd);
  count_stats(p, wave_id, lane, applied, active, 2u * kPlanes * 4u + (REPLAY ? 8u : 4u) * K + 4u, emitted, upd,
              died);
}

// ---------------------------------------------------------------------------
// Drop-in RegisterVotes for one node (processor.go:61-122): one thread per
// touched block applies that block's votes in Response order, so duplicate
// hashes in one Response apply sequentially. Status per vote position. One
// thread per touched lane (node, 32-target block) of any number of nodes
// (av_register_votes_batch): a node's Responses apply one after the other.
// ---------------------------------------------------------------------------
__global__ void k_register_votes(const DropInParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n_blocks) return;
  const uint32_t g = p.blocks[i];  // lane: local node * BL + block
  if (g >= p.L) return;            // the run of votes for unknown targets: no update (status -1)
  const uint32_t nl = g / p.BL, b = g - nl * p.BL;
  const uint32_t node = p.n0 + nl;
  St s;
  load_state(p.planes, g, s);
  const uint32_t vmask = p.valid[b];
  uint32_t died = 0;
  for (uint32_t e = p.offs[i]; e < p.offs[i + 1]; ++e) {
    const uint32_t pos = p.entries[2 * e];
    const uint32_t meta = p.entries[2 * e + 1];
    const uint32_t m = 1u << (meta & 31u);
    const uint32_t part = ~s.K[7] & vmask & m;  // skip unknown/deleted (:95-99) and invalid (:101-103)
    uint32_t E, fin;
    vote_step<true>(s, (meta >> 5) & 1u ? m : 0u, (meta >> 6) & 1u ? m : 0u, part, E, fin);
    died |= fin;
    int32_t st = -1;
    if (E & m) st = (fin & m) ? ((s.A & m) ? 3 : 0) : ((s.A & m) ? 2 : 1);
    p.status_out[pos] = (int8_t)st;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    s.V[q] &= ~died;
    s.C[q] |= died;
  }
  store_state(p.planes, g, s);
  p.pref[(size_t)node * p.PS + b] =
      is_byz(p.byz, node) ? byz_pattern(p.round) : publish_word(s.A, s.K[7], p.pub_mode);
}

// av_register_votes_batch, fast path: every Response's targets strictly
// ascending. A Response's votes for one (node, 32-target block) lane are then
// consecutive and in order, and the run's first vote is the one whose
// predecessor is in another block: one thread per run applies it (<= 32
// votes) exactly as k_register_votes does, with no sort. One workgroup per
// node (grid-stride over nodes): its Responses apply one after the other
// (processor.go:61-122 per Response, in call order). A Response is walked in
// chunks of kDropChunk votes: the chunk's run heads are collected in LDS, then
// the workgroup's threads take one run each (a run may reach into the next
// chunk; its head is in this one).
constexpr uint32_t kDropChunk = 4096;

__device__ __forceinline__ void dropin_run(const DropInParams& p, uint32_t v, uint32_t o1, uint32_t nl, uint32_t node) {
  const uint32_t blk = (p.packed[v] & kDropTl) >> 5;
  const uint32_t g = nl * p.BL + blk;
  St s;
  load_state(p.planes, g, s);
  const uint32_t vmask = p.valid[blk];
  uint32_t died = 0;
  for (uint32_t u = v; u < o1; ++u) {
    const uint32_t x = p.packed[u];
    if ((x & kDropUnknown) || ((x & kDropTl) >> 5) != blk) break;
    const uint32_t m = 1u << (x & 31u);
    const uint32_t part = ~s.K[7] & vmask & m;  // skip deleted (:95-99) and invalid (:101-103)
    uint32_t E, fin;
    vote_step<true>(s, (x & kDropYes) ? m : 0u, (x & kDropCons) ? m : 0u, part, E, fin);
    died |= fin;
    int32_t st = -1;
    if (E & m) st = (fin & m) ? ((s.A & m) ? 3 : 0) : ((s.A & m) ? 2 : 1);
    p.status_out[u] = (int8_t)st;
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    s.V[q] &= ~died;
    s.C[q] |= died;
  }
  store_state(p.planes, g, s);
  p.pref[(size_t)node * p.PS + blk] = is_byz(p.byz, node) ? byz_pattern(p.round) : publish_word(s.A, s.K[7], p.pub_mode);
}

__global__ __launch_bounds__(256) void k_dropin_resp(const DropInParams p) {
  __shared__ uint32_t heads[kDropChunk];
  __shared__ uint32_t nheads;
  for (uint32_t gi = blockIdx.x; gi < p.n_groups; gi += gridDim.x) {
    for (uint32_t k = p.grp_off[gi]; k < p.grp_off[gi + 1]; ++k) {
      const uint32_t r = p.order[k];
      const uint32_t o0 = p.resp_off[r], o1 = p.resp_off[r + 1];
      const uint32_t nl = p.resp_node[r], node = p.n0 + nl;
      for (uint32_t c0 = o0; c0 < o1; c0 += kDropChunk) {
        const uint32_t c1 = min(o1, c0 + kDropChunk);
        if (threadIdx.x == 0) nheads = 0u;
        __syncthreads();
        for (uint32_t v = c0 + threadIdx.x; v < c1; v += blockDim.x) {
          const uint32_t w = p.packed[v];
          if (w & kDropUnknown) continue;
          if (v > o0) {
            const uint32_t q = p.packed[v - 1u];
            if (!(q & kDropUnknown) && ((q ^ w) & kDropTl) >> 5 == 0u) continue;  // inside a run
          }
          heads[atomicAdd(&nheads, 1u)] = v;
        }
        __syncthreads();
        const uint32_t nh = nheads;
        for (uint32_t h = threadIdx.x; h < nh; h += blockDim.x) dropin_run(p, heads[h], o1, nl, node);
        __syncthreads();  // heads reused; the node's next Response sees this one's records
      }
    }
  }
}

// General path: one workgroup per Response writes each vote's lane key (L for
// an unknown target), its index and its packed (bit | yes << 5 | considered << 6)
// for the stable radix grouping (log_ops.hip launch_group_votes).
__global__ __launch_bounds__(256) void k_dropin_keys(const DropInParams p, uint32_t* keys, uint32_t* vidx,
                                                     uint32_t* info) {
  for (uint32_t r = blockIdx.x; r < p.n_resp; r += gridDim.x) {
    const uint32_t o0 = p.resp_off[r], o1 = p.resp_off[r + 1];
    const uint32_t nl = p.resp_node[r];
    for (uint32_t v = o0 + threadIdx.x; v < o1; v += blockDim.x) {
      const uint32_t w = p.packed[v];
      const uint32_t tl = w & kDropTl;
      keys[v] = (w & kDropUnknown) ? p.L : nl * p.BL + (tl >> 5);
      vidx[v] = v;
      info[v] = (tl & 31u) | ((w & kDropYes) ? 1u << 5 : 0u) | ((w & kDropCons) ? 1u << 6 : 0u);
    }
  }
}

// AddTargetToReconcile (processor.go:45-58) for a list of targets of one
// node, applied sequentially by one thread (duplicates return false).
__global__ void k_add_targets(const AddParams p) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  for (uint32_t i = 0; i < p.n; ++i) {
    const uint32_t t = p.targets[i];
    const uint32_t b = t >> 5, m = 1u << (t & 31u);
    const uint32_t g = p.node_local * p.BL + b;
    const bool valid = (p.valid[b] & m) != 0u;               // isWorthyPolling (:46-48)
    const bool exists = (*pw(p.planes, g, kPK + 7) & m) == 0u;  // record present (:50-53)
    if (!valid || exists) {
      p.added[i] = 0;
      continue;
    }
    for (int q = 0; q < 8; ++q) {  // NewVoteRecord(t.IsAccepted()) (vote.go:33-35)
      *pw(p.planes, g, kPV + q) &= ~m;
      *pw(p.planes, g, kPC + q) &= ~m;
      *pw(p.planes, g, kPK + q) &= ~m;
    }
    uint32_t* a = pw(p.planes, g, kPA);
    *a = p.accepted[i] ? (*a | m) : (*a & ~m);
    p.added[i] = 1;
    p.pref[(size_t)p.node * p.PS + b] = is_byz(p.byz, p.node) ? byz_pattern(p.round)
                                                               : publish_word(*a, *pw(p.planes, g, kPK + 7), p.pub_mode);
  }
}

__device__ __forceinline__ uint32_t init_accept_block(uint64_t seed, int mode, uint32_t param, uint32_t node,
                                                      uint32_t tb /* first target, multiple of 32 */) {
  uint32_t a = 0;
  if (mode == 2) return ~0u;
  if (mode == 3) {  // Bernoulli: philox(node, t>>2, 0, INIT)[t&3] < param
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      uint32_t x[4];
      philox(x, seed, node, (tb >> 2) + q, 0u, kDomInit);
#pragma unroll
      for (int i = 0; i < 4; ++i) a |= (x[i] < param ? 1u : 0u) << (q * 4 + i);
    }
  } else if (mode == 4) {  // pairs (2p, 2p+1): coin = philox(node, p>>2, 0, PAIRS)[p&3] >> 31
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      uint32_t x[4];
      philox(x, seed, node, (tb >> 3) + q, 0u, kDomPairs);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t coin = x[i] >> 31;
        const int pr = q * 4 + i;  // pair index inside the block (0..15)
        a |= (coin << (2 * pr)) | ((coin ^ 1u) << (2 * pr + 1));
      }
    }
  }
  return a;
}

__device__ __forceinline__ uint32_t target_mask(uint32_t tb, uint32_t n_targets) {
  if (tb >= n_targets) return 0u;
  const uint32_t r = n_targets - tb;
  return r >= 32u ? ~0u : ((1u << r) - 1u);
}

__global__ void k_init_planes(const InitParams p) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.L) return;
  const uint32_t nl = g / p.BL, b = g - nl * p.BL;
  const uint32_t tb = p.t0 + 32u * b;
  const uint32_t live = p.mode == 0 ? 0u : target_mask(tb, p.n_targets);
  const uint32_t acc = init_accept_block(p.seed, p.mode, p.param, p.n0 + nl, tb) & live;
  St s;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s.V[i] = 0u;
    s.C[i] = ~live;
    s.K[i] = 0u;
  }
  s.K[7] = ~live;
  s.A = acc;
  store_state(p.planes, g, s);
}

__global__ void k_init_pref(const InitParams p) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)p.n_nodes * p.BL) return;
  const uint32_t node = (uint32_t)(i / p.BL), b = (uint32_t)(i - (size_t)node * p.BL);
  const size_t o = (size_t)node * p.PS + b;
  const uint32_t tb = p.t0 + 32u * b;
  uint32_t v;
  if (is_byz(p.byz, node))
    v = byz_pattern(p.round);
  else
    v = p.mode == 0 ? (p.pub_mode == 2u ? target_mask(tb, p.n_targets) : 0u)  // no records (K7 set)
                    : (init_accept_block(p.seed, p.mode, p.param, node, tb) & target_mask(tb, p.n_targets));
  p.pref[o] = v;
}

__global__ void k_byz(uint32_t* byz, uint32_t n_nodes, uint64_t seed, uint32_t threshold) {
  const uint32_t wi = blockIdx.x * blockDim.x + threadIdx.x;
  if (wi >= (n_nodes + 31u) / 32u) return;
  uint32_t bits = 0;
  for (uint32_t i = 0; i < 32u; ++i) {
    const uint32_t node = wi * 32u + i;
    if (node >= n_nodes) break;
    uint32_t x[4];
    philox(x, seed, node, 0u, 0u, kDomByz);
    bits |= (x[0] < threshold ? 1u : 0u) << i;
  }
  byz[wi] = bits;
}

__global__ void k_read_records(const uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1, uint32_t tl0,
                               uint32_t tl1, uint32_t* out) {
  const uint32_t W = tl1 - tl0;
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)(nl1 - nl0) * W) return;
  const uint32_t nl = nl0 + (uint32_t)(i / W), tl = tl0 + (uint32_t)(i % W);
  const uint32_t g = nl * BL + (tl >> 5), bit = tl & 31u;
  const uint32_t a = (*pw(planes, g, kPA) >> bit) & 1u;
  if ((*pw(planes, g, kPK + 7) >> bit) & 1u) {
    out[i] = 0xFFFE0000u | (a << 16);
    return;
  }
  uint32_t v = 0, c = 0, k = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    v |= ((*pw(planes, g, kPV + q) >> bit) & 1u) << q;
    c |= ((*pw(planes, g, kPC + q) >> bit) & 1u) << q;
  }
#pragma unroll
  for (int q = 0; q < 7; ++q) k |= ((*pw(planes, g, kPK + q) >> bit) & 1u) << q;
  out[i] = v | (c << 8) | (((k << 1) | a) << 16);
}

// The same canonical words, one thread per 32-record lane, WITHOUT writing
// back the deferred forms the warm rounds leave behind (kernels.h vv / klazy):
// a stale tile's vote register is regathered from the previous snapshot
// (p.pref_prev) with round p.round - 1's peers, and a tile's pending +8 count
// steps are added to its polled (live, valid) records. Reads (IsAccepted,
// GetConfidence, GetInvsForNextPoll, dumps) then leave the next round's fast
// paths in place. p.vv / p.klazy: some tile may be stale / hold pending steps.
__global__ __launch_bounds__(256) void k_read_records_v(const RoundParams p, uint32_t nl0, uint32_t nl1, uint32_t tl0,
                                                        uint32_t tl1, uint32_t* out) {
  const uint32_t b0 = tl0 >> 5, NB = ((tl1 + 31u) >> 5) - b0, W = tl1 - tl0;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (nl1 - nl0) * NB) return;
  const uint32_t nl = nl0 + i / NB, b = b0 + i % NB;
  const uint32_t g = nl * p.BL + b, tile = g >> 6;
  St s;
  load_state(p.planes, g, s);
  const uint32_t raw = p.vv ? p.vstale[tile] : 0u, st = raw & kVMask;
  if (raw & kCAll) {  // consider planes left unstored by the fresh round: all-ones
#pragma unroll
    for (int q = 0; q < 8; ++q) s.C[q] = ~0u;
  }
  if (st == kVStale) {  // V_i = the vote of round - 1's slot 7 - i (k = 8)
    uint32_t pp[8];
    sample_peers<8>(p.seed, p.n0 + nl, p.round - 1u, p.n_nodes, p.peer_mode, pp);
#pragma unroll
    for (int q = 0; q < 8; ++q) s.V[q] = p.pref_prev[pp[7 - q] * p.PS + b];
  } else if (st == kVUniform) {  // every polled record's vote register = its accepted bit
#pragma unroll
    for (int q = 0; q < 8; ++q) s.V[q] = s.A;
  }
  if (p.klazy) {
    const uint32_t kw = p.kpend[tile];
    if (kw & kHiVirt) {  // the K4..K7 group is virtual (kernels.h)
      s.K[4] = s.K[5] = s.K[6] = 0u;
      s.K[7] = ~real_mask(p.tn, b);
    }
    const uint32_t pend = kw & 0xFFu;
    if (pend) {  // + 8 * pend on the polled records: pend added to count bits 3..6
      const uint32_t P0 = ~s.K[7] & p.valid[b];
      uint32_t cy = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t bi = ((pend >> q) & 1u) ? P0 : 0u;
        const uint32_t t = s.K[3 + q] ^ bi;
        const uint32_t si = t ^ cy;
        cy = (t & cy) | (s.K[3 + q] & bi);
        s.K[3 + q] = si;
      }
    }
  }
  const uint32_t lo = max(tl0, b * 32u), hi = min(tl1, b * 32u + 32u);
  uint32_t* dst = out + (size_t)(nl - nl0) * W;
  for (uint32_t tl = lo; tl < hi; ++tl) {
    const uint32_t bit = tl & 31u;
    const uint32_t a = (s.A >> bit) & 1u;
    uint32_t word;
    if ((s.K[7] >> bit) & 1u) {
      word = 0xFFFE0000u | (a << 16);
    } else {
      uint32_t v = 0, c = 0, k = 0;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        v |= ((s.V[q] >> bit) & 1u) << q;
        c |= ((s.C[q] >> bit) & 1u) << q;
      }
#pragma unroll
      for (int q = 0; q < 7; ++q) k |= ((s.K[q] >> bit) & 1u) << q;
      word = v | (c << 8) | (((k << 1) | a) << 16);
    }
    dst[tl - tl0] = word;
  }
}

__global__ void k_write_records(uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1, uint32_t tl0,
                                uint32_t tl1, const uint32_t* in) {
  const uint32_t b0 = tl0 >> 5, b1 = (tl1 + 31u) >> 5, NB = b1 - b0, W = tl1 - tl0;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (nl1 - nl0) * NB) return;
  const uint32_t nl = nl0 + i / NB, b = b0 + i % NB;
  const uint32_t g = nl * BL + b;
  St s;
  load_state(planes, g, s);
  for (uint32_t bit = 0; bit < 32u; ++bit) {
    const uint32_t tl = b * 32u + bit;
    if (tl < tl0 || tl >= tl1) continue;
    const uint32_t w = in[(size_t)(nl - nl0) * W + (tl - tl0)];
    const uint32_t m = 1u << bit;
    const uint32_t conf = w >> 16;
    const bool live = (conf >> 1) < 128u;
    for (int q = 0; q < 8; ++q) {
      const uint32_t vb = live ? (w >> q) & 1u : 0u;
      const uint32_t cb = live ? (w >> (8 + q)) & 1u : 1u;
      const uint32_t kb = live ? ((conf >> 1) >> q) & 1u : (q == 7 ? 1u : 0u);
      s.V[q] = (s.V[q] & ~m) | (vb << bit);
      s.C[q] = (s.C[q] & ~m) | (cb << bit);
      s.K[q] = (s.K[q] & ~m) | (kb << bit);
    }
    s.A = (s.A & ~m) | ((conf & 1u) << bit);
  }
  store_state(planes, g, s);
}

__global__ void k_refresh_pref(uint32_t pub_mode, const uint32_t* planes, uint32_t* pref, const uint32_t* byz,
                               uint32_t n0, uint32_t NL, uint32_t BL, uint32_t PS, uint32_t round) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= NL * BL) return;
  const uint32_t nl = g / BL, b = g - nl * BL, node = n0 + nl;
  pref[(size_t)node * PS + b] =
      is_byz(byz, node) ? byz_pattern(round) : publish_word(*pw(planes, g, kPA), *pw(planes, g, kPK + 7), pub_mode);
}

// The example's responder (main.go:175-177), after a round: every record a
// node was queried for (readd, OR of the querying lanes' polled masks) and
// did not hold at the round start (no record now, not deleted this round) is
// re-created as AddTargetToReconcile(&tx{isAccepted: true}) (processor.go:
// 45-58, valid targets only): votes, consider and count zero, accepted.
__global__ __launch_bounds__(256) void k_readd(const RoundParams p) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= p.L) return;
  const uint32_t q = p.readd[g];
  if (!q) return;
  p.readd[g] = 0u;
  const uint32_t b = g % p.BL;
  const uint32_t m = q & *pw(p.planes, g, kPK + 7) & ~p.died_out[g] & p.valid[b];
  if (!m) return;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    *pw(p.planes, g, kPV + i) &= ~m;
    *pw(p.planes, g, kPC + i) &= ~m;
    *pw(p.planes, g, kPK + i) &= ~m;
  }
  *pw(p.planes, g, kPA) |= m;
}

template <int K>
__global__ void k_sample_peers(uint64_t seed, uint32_t n_nodes, uint32_t a, uint32_t b, uint32_t round, int mode,
                               uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (a + i >= b) return;
  uint32_t peers[K];
  sample_peers<K>(seed, a + i, round, n_nodes, mode, peers);
#pragma unroll
  for (int j = 0; j < K; ++j) out[(size_t)i * K + j] = peers[j];
}

// Synthetic replayed vote stream (C2): class per (node, round, slot, target)
// from philox(node, round, t>>1, REPLAY | slot<<8); same definition as
// avo_replay_err in the oracle. Output: the tiled replay layout (kernels.h replay_idx).
__global__ void k_gen_replay(uint64_t seed, uint32_t n0, uint32_t BL, uint32_t L, uint32_t Lpad, uint32_t t0,
                             uint32_t n_targets, uint32_t round, int k, uint32_t* out) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= Lpad) return;
  if (g >= L) {
    for (int s = 0; s < k; ++s) {
      out[replay_idx(g, k, s, 0)] = 0u;
      out[replay_idx(g, k, s, 1)] = 0u;
    }
    return;
  }
  const uint32_t nl = g / BL, b = g - nl * BL, node = n0 + nl;
  const uint32_t tb = t0 + 32u * b;
  const uint32_t tm = target_mask(tb, n_targets);
  for (int s = 0; s < k; ++s) {
    uint32_t y = 0, c = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      uint32_t x[4];
      philox(x, seed, node, round, (tb >> 1) + q, kDomReplay | ((uint32_t)s << 8));
      const uint32_t v0 = x[0], v1 = x[2];
      y |= (v0 < kReplayYes ? 1u : 0u) << (2 * q);
      c |= (v0 < kReplayNo ? 1u : 0u) << (2 * q);
      y |= (v1 < kReplayYes ? 1u : 0u) << (2 * q + 1);
      c |= (v1 < kReplayNo ? 1u : 0u) << (2 * q + 1);
    }
    out[replay_idx(g, k, s, 0)] = y & tm;
    out[replay_idx(g, k, s, 1)] = c & tm;
  }
}

// Live valid records (optionally of honest nodes only): the convergence
// measure for rounds-to-finalization. Grid-stride, one atomic per block.
__global__ void k_count_live(const uint32_t* planes, const uint32_t* valid, const uint32_t* byz, uint32_t n0,
                             uint32_t BL, uint32_t L, int honest_only, unsigned long long* out) {
  __shared__ unsigned long long part[4];
  unsigned long long c = 0;
  for (uint32_t g = blockIdx.x * blockDim.x + threadIdx.x; g < L; g += gridDim.x * blockDim.x) {
    const uint32_t nl = g / BL, b = g - nl * BL;
    if (honest_only && is_byz(byz, n0 + nl)) continue;
    c += __popc(~*pw(planes, g, kPK + 7) & valid[b]);
  }
  const uint32_t w = wave_sum((uint32_t)c);  // <= 32 * 64 per wave per pass: fits u32
  if ((threadIdx.x & 63u) == 0) part[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}

// Batched GetInvsForNextPoll (processor.go:144-170) for local nodes
// [nl0, nl0 + gridDim.x): one 64-lane workgroup per node walks the node's
// blocks in order with a running wave prefix count of live, valid records
// (rule R1: ascending target order, at most kMaxPoll). counts != nullptr: only
// count them. Else write the poll set at out + offsets[node] (entries at or past
// cap skipped): per 64-block chunk, lane i writes the chunk's records i, i + 64,
// ... (its block by binary search over the chunk's prefix counts in LDS, its
// target by the rank-th set bit), so every store is coalesced — the output may
// be host-mapped memory written over PCIe. lane 0 of each node also writes
// offs_out[node] (and the last node offs_out[n]) as int64.
__global__ __launch_bounds__(64) void k_poll_sets(const uint32_t* planes, const uint32_t* valid, uint32_t BL,
                                                  uint32_t nl0, uint32_t t0, uint32_t* counts,
                                                  const uint64_t* offsets, uint64_t cap, int64_t* offs_out,
                                                  int32_t* out) {
  __shared__ uint32_t pre[64];
  __shared__ uint32_t bits_s[64];
  const uint32_t i = blockIdx.x, nl = nl0 + i, lane = threadIdx.x;
  const uint64_t o0 = counts ? 0ull : offsets[i];
  if (!counts && lane == 0) {
    offs_out[i] = (int64_t)o0;
    if (i == gridDim.x - 1u) offs_out[i + 1u] = (int64_t)offsets[i + 1u];
  }
  uint32_t run = 0;  // records selected so far (wave-uniform)
  for (uint32_t b0 = 0; b0 < BL && run < kMaxPoll; b0 += 64u) {
    const uint32_t b = b0 + lane;
    const uint32_t bits = b < BL ? ~*pw(planes, nl * BL + b, kPK + 7) & valid[b] : 0u;
    const uint32_t c = (uint32_t)__popc(bits);
    const uint32_t incl = wave_incl_scan(c, lane);
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
    if (!counts) {
      pre[lane] = incl - c;
      bits_s[lane] = bits;
      __syncthreads();
      const uint32_t take = min(tot, kMaxPoll - run);
      for (uint32_t q = lane; q < take; q += 64u) {
        uint32_t l0 = 0, l1 = 63;  // the last block lane whose prefix is <= q
        while (l0 < l1) {
          const uint32_t mid = (l0 + l1 + 1u) >> 1;
          if (pre[mid] <= q) l0 = mid; else l1 = mid - 1u;
        }
        uint32_t m = bits_s[l0], r = q - pre[l0], pos = 0;
#pragma unroll
        for (uint32_t w = 16; w >= 1; w >>= 1) {
          const uint32_t low = m & ((1u << w) - 1u);
          const uint32_t cl = (uint32_t)__popc(low);
          if (r >= cl) {
            r -= cl;
            m >>= w;
            pos += w;
          } else {
            m = low;
          }
        }
        const uint64_t at = o0 + run + q;
        if (at < cap) out[at] = (int32_t)(t0 + 32u * (b0 + l0) + pos);
      }
      __syncthreads();
    }
    run += tot;
  }
  if (counts && lane == 0) counts[i] = min(run, kMaxPoll);
}

template <int K>
hipError_t launch_round_k(const RoundParams& p, bool replay, bool capped, hipStream_t s) {
  if (capped) {
    const uint32_t bt = ((p.BL + 63u) / 64u) * 64u;
    const uint32_t grid = p.node_flags ? std::min(p.NL, 128u) : p.NL;
    if (replay)
      hipLaunchKernelGGL((k_round_capped<K, true>), dim3(grid), dim3(bt), 0, s, p);
    else
      hipLaunchKernelGGL((k_round_capped<K, false>), dim3(grid), dim3(bt), 0, s, p);
  } else {
    const uint32_t blocks = (p.Lpad + 255u) / 256u;
    if (replay)
      hipLaunchKernelGGL((k_round_fast<K, true>), dim3(blocks), dim3(256), 0, s, p);
    else
      hipLaunchKernelGGL((k_round_fast<K, false>), dim3(blocks), dim3(256), 0, s, p);
  }
  return hipGetLastError();
}

template <int K>
hipError_t launch_sample_k(uint64_t seed, uint32_t n_nodes, uint32_t a, uint32_t b, uint32_t round, int mode,
                           uint32_t* out, hipStream_t s) {
  const uint32_t n = b - a;
  hipLaunchKernelGGL((k_sample_peers<K>), dim3((n + 255) / 256), dim3(256), 0, s, seed, n_nodes, a, b, round, mode,
                     out);
  return hipGetLastError();
}

}  // namespace

#define AVK_K_SWITCH(k, CALL) \
  switch (k) {                \
    case 1: return CALL(1);   \
    case 2: return CALL(2);   \
    case 3: return CALL(3);   \
    case 4: return CALL(4);   \
    case 5: return CALL(5);   \
    case 6: return CALL(6);   \
    case 7: return CALL(7);   \
    case 8: return CALL(8);   \
    case 9: return CALL(9);   \
    case 10: return CALL(10); \
    case 11: return CALL(11); \
    case 12: return CALL(12); \
    case 13: return CALL(13); \
    case 14: return CALL(14); \
    case 15: return CALL(15); \
    case 16: return CALL(16); \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_round(const RoundParams& p, int k, bool replay, bool capped, hipStream_t s) {
#define AVK_ROUND(K) launch_round_k<K>(p, replay, capped, s)
  AVK_K_SWITCH(k, AVK_ROUND)
#undef AVK_ROUND
}

hipError_t launch_sample_peers(uint64_t seed, uint32_t n_nodes, uint32_t a, uint32_t b, uint32_t round, int k,
                               int mode, uint32_t* out, hipStream_t s) {
  if (b <= a) return hipSuccess;
#define AVK_SAMPLE(K) launch_sample_k<K>(seed, n_nodes, a, b, round, mode, out, s)
  AVK_K_SWITCH(k, AVK_SAMPLE)
#undef AVK_SAMPLE
}

hipError_t launch_init(const InitParams& p, hipStream_t s) {
  if (p.L) hipLaunchKernelGGL(k_init_planes, dim3((p.L + 255) / 256), dim3(256), 0, s, p);
  const size_t rows = (size_t)p.n_nodes * p.BL;
  if (rows) hipLaunchKernelGGL(k_init_pref, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_byz(uint32_t* byz, uint32_t n_nodes, uint64_t seed, uint32_t threshold, hipStream_t s) {
  const uint32_t words = (n_nodes + 31u) / 32u;
  hipLaunchKernelGGL(k_byz, dim3((words + 255) / 256), dim3(256), 0, s, byz, n_nodes, seed, threshold);
  return hipGetLastError();
}

hipError_t launch_register_votes(const DropInParams& p, hipStream_t s) {
  if (!p.n_blocks) return hipSuccess;
  hipLaunchKernelGGL(k_register_votes, dim3((p.n_blocks + 63) / 64), dim3(64), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_dropin_resp(const DropInParams& p, hipStream_t s) {
  if (!p.n_resp) return hipSuccess;
  hipLaunchKernelGGL(k_dropin_resp, dim3(std::min<uint32_t>(p.n_groups, 65535u)), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_dropin_keys(const DropInParams& p, uint32_t* keys, uint32_t* vidx, uint32_t* info, hipStream_t s) {
  if (!p.n_resp) return hipSuccess;
  hipLaunchKernelGGL(k_dropin_keys, dim3(std::min<uint32_t>(p.n_resp, 65535u)), dim3(256), 0, s, p, keys, vidx, info);
  return hipGetLastError();
}

hipError_t launch_add_targets(const AddParams& p, hipStream_t s) {
  if (!p.n) return hipSuccess;
  hipLaunchKernelGGL(k_add_targets, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_read_records(const uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1, uint32_t tl0,
                               uint32_t tl1, uint32_t* out, hipStream_t s) {
  const size_t n = (size_t)(nl1 - nl0) * (tl1 - tl0);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_read_records, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, planes, BL, nl0, nl1, tl0,
                     tl1, out);
  return hipGetLastError();
}

hipError_t launch_read_records_virtual(const RoundParams& p, uint32_t nl0, uint32_t nl1, uint32_t tl0, uint32_t tl1,
                                       uint32_t* out, hipStream_t s) {
  const uint32_t nb = ((tl1 + 31u) >> 5) - (tl0 >> 5);
  const uint32_t n = (nl1 - nl0) * nb;
  if (!n || tl1 <= tl0) return hipSuccess;
  hipLaunchKernelGGL(k_read_records_v, dim3((n + 255) / 256), dim3(256), 0, s, p, nl0, nl1, tl0, tl1, out);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Peer-push exchange of node-sharded engines. Replaces the
// per-round all-gather of published-preference rows (main.go:168-192: every
// responder answers from its current IsAccepted) when the ranks' snapshot
// buffers are mapped into each other's address space (av_peer_init).
// ---------------------------------------------------------------------------
// Copy words [w0, w1) of a local snapshot buffer into every peer replica:
// a full resynchronisation, used after rounds whose kernel does not push.
__global__ __launch_bounds__(256) void k_push_rows(const uint32_t* src, PeerPtrs dst, uint32_t n_dst, uint64_t w0,
                                                   uint64_t w1) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = w0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w1; i += stride) {
    const uint32_t v = src[i];
#pragma unroll
    for (int r = 0; r < kMaxPeers; ++r)  // static indices: the pointers stay in SGPRs
      if ((uint32_t)r < n_dst) __hip_atomic_store(dst.p[r] + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Need-masked exchange, step 1: the rows this rank's nodes draw (R1's peer sampling, the same
// sample_peers the oracle restates) in the W rounds of a window, as bytes mine[w][N] (plain stores of
// the same value: concurrent writers of one byte agree; the caller clears mine first).
template <int K>
__global__ __launch_bounds__(256) void k_need_draw(uint64_t seed, uint32_t n_nodes, uint32_t n0, uint32_t NL,
                                                   uint32_t round0, uint32_t W, int mode, uint8_t* mine) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)W * NL) return;
  const uint32_t w = (uint32_t)(i / NL), nl = (uint32_t)(i - (uint64_t)w * NL);
  uint32_t peers[K];
  sample_peers<K>(seed, n0 + nl, round0 + w, n_nodes, mode, peers);
  uint8_t* row = mine + (size_t)w * n_nodes;
#pragma unroll
  for (int j = 0; j < K; ++j) row[peers[j]] = 1u;
}

// Step 2: rank d's slice of mine, 32 rows per word, stored into d's needin[par][rank][w][NLw]
// (system scope: over xGMI, ordered before d reads it by the round barrier).
__global__ __launch_bounds__(256) void k_need_push(const uint8_t* mine, uint32_t n_nodes, uint32_t NL, uint32_t W,
                                                   uint32_t world, uint32_t rank, uint32_t par, PeerPtrs needin) {
  const uint32_t NLw = (NL + 31u) / 32u;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)world * W * NLw) return;
  const uint32_t d = (uint32_t)(i / ((uint64_t)W * NLw));
  const uint32_t rem = (uint32_t)(i - (uint64_t)d * W * NLw);
  const uint32_t w = rem / NLw, q = rem - w * NLw;
  if (d == rank) return;
  const uint8_t* src = mine + (size_t)w * n_nodes + (size_t)d * NL + (size_t)q * 32u;
  const uint32_t nb = min(32u, NL - q * 32u);
  uint32_t bits = 0u;
  for (uint32_t j = 0; j < nb; ++j) bits |= (uint32_t)(src[j] != 0u) << j;
  uint32_t* dst = needin.p[0];  // rank d's table, selected with static indices (SGPRs)
#pragma unroll
  for (int r = 1; r <= kMaxPeers; ++r)
    if ((uint32_t)r == d) dst = needin.p[r];
  __hip_atomic_store(dst + (((size_t)par * world + rank) * W + w) * NLw + q, bits, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

// Step 3 (after the barrier): per local row and round of the window, the peers (push order: ranks
// ascending, this rank skipped) whose nodes draw it.
__global__ __launch_bounds__(256) void k_need_combine(const uint32_t* needin, uint32_t world, uint32_t rank,
                                                      uint32_t par, uint32_t W, uint32_t NL, uint32_t ref_local,
                                                      uint8_t* needmask) {
  const uint32_t NLw = (NL + 31u) / 32u;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (uint64_t)W * NL) return;
  const uint32_t w = (uint32_t)(i / NL), nl = (uint32_t)(i - (uint64_t)w * NL);
  uint32_t m = 0u, pi = 0u;
  for (uint32_t d = 0; d < world; ++d) {
    if (d == rank) continue;
    const uint32_t word = needin[(((size_t)par * world + d) * W + w) * NLw + (nl >> 5)];
    m |= ((word >> (nl & 31u)) & 1u) << pi;
    ++pi;
  }
  if (nl == ref_local) m = (1u << (world - 1u)) - 1u;  // every rank reads the reference row (uniform rows)
  needmask[(size_t)w * NL + nl] = (uint8_t)m;
}

// One wave. Lane i (< world) stores seq into rank i's arrival slot `rank`
// (release, system scope: this rank's earlier kernels and pushes are visible
// first), then waits for its own slot i to reach seq (acquire, system scope).
// Every lane leaves after at most `ticks` wall-clock ticks; a timeout sets *err
// (pinned host memory) and every later barrier of the engine returns without
// waiting; the host refuses further rounds and results (engine.cpp
// peer_failed, AV_ERR_PEER).
__global__ __launch_bounds__(64) void k_peer_barrier(PeerPtrs arrive, const uint32_t* own, uint32_t world,
                                                     uint32_t rank, uint32_t seq, uint32_t* err, uint64_t ticks,
                                                     const uint32_t* uslot, PeerPtrs slot_dst, uint32_t wait) {
  const uint32_t i = threadIdx.x;
  if (uslot && i < world && i != rank) {  // this rank's uniform-rows slot into rank i's replica (before arriving)
    uint32_t* d = slot_dst.p[0];
#pragma unroll
    for (int r = 1; r <= kMaxPeers; ++r)
      if ((uint32_t)r == i) d = slot_dst.p[r];
    __hip_atomic_store(d, *uslot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (!wait) return;
  uint32_t* mine = arrive.p[0];  // lane i's rank-i array, selected with static indices
#pragma unroll
  for (int r = 1; r <= kMaxPeers; ++r)
    if ((uint32_t)r == i) mine = arrive.p[r];
  if (i < world) __hip_atomic_store(mine + rank, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  const bool failed = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
  if (i >= world || failed) return;
  const uint32_t* slot = own + i;  // own == arrive.p[rank]
  const uint64_t t0 = (uint64_t)wall_clock64();
  while ((int32_t)(__hip_atomic_load(slot, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - seq) < 0) {
    if ((uint64_t)wall_clock64() - t0 > ticks) {
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // host-visible (pinned)
      return;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

hipError_t launch_write_records(uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1, uint32_t tl0, uint32_t tl1,
                                const uint32_t* in, hipStream_t s) {
  const uint32_t nb = ((tl1 + 31u) >> 5) - (tl0 >> 5);
  const uint32_t n = (nl1 - nl0) * nb;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_write_records, dim3((n + 255) / 256), dim3(256), 0, s, planes, BL, nl0, nl1, tl0, tl1, in);
  return hipGetLastError();
}

hipError_t launch_refresh_pref(uint32_t pub_mode, const uint32_t* planes, uint32_t* pref, const uint32_t* byz,
                               uint32_t n0, uint32_t NL, uint32_t BL, uint32_t PS, uint32_t round, hipStream_t s) {
  const uint32_t n = NL * BL;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_refresh_pref, dim3((n + 255) / 256), dim3(256), 0, s, pub_mode, planes, pref, byz, n0, NL, BL,
                     PS, round);
  return hipGetLastError();
}

hipError_t launch_readd(const RoundParams& p, hipStream_t s) {
  if (!p.readd || !p.died_out || !p.L) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_readd, dim3((p.L + 255) / 256), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_gen_replay(uint64_t seed, uint32_t n0, uint32_t NL, uint32_t BL, uint32_t L, uint32_t Lpad,
                             uint32_t t0, uint32_t n_targets, uint32_t round, int k, uint32_t* out, hipStream_t s) {
  (void)NL;
  if (!Lpad) return hipSuccess;
  hipLaunchKernelGGL(k_gen_replay, dim3((Lpad + 255) / 256), dim3(256), 0, s, seed, n0, BL, L, Lpad, t0, n_targets,
                     round, k, out);
  return hipGetLastError();
}

hipError_t launch_count_live(const uint32_t* planes, const uint32_t* valid, const uint32_t* byz, uint32_t n0,
                             uint32_t BL, uint32_t L, int honest_only, unsigned long long* out, hipStream_t s) {
  if (!L) return hipSuccess;
  const uint32_t blocks = std::min<uint32_t>(2048u, (L + 255u) / 256u);
  hipLaunchKernelGGL(k_count_live, dim3(blocks), dim3(256), 0, s, planes, valid, byz, n0, BL, L, honest_only, out);
  return hipGetLastError();
}


hipError_t launch_push_rows(const uint32_t* src, PeerPtrs dst, uint32_t n_dst, uint64_t w0, uint64_t w1,
                            hipStream_t s) {
  if (w1 <= w0 || !n_dst) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>(4096u, (w1 - w0 + 255u) / 256u);
  hipLaunchKernelGGL(k_push_rows, dim3((uint32_t)blocks), dim3(256), 0, s, src, dst, n_dst, w0, w1);
  return hipGetLastError();
}

template <int K>
hipError_t launch_need_draw_k(uint64_t seed, uint32_t n_nodes, uint32_t n0, uint32_t NL, uint32_t round0, uint32_t W,
                              int mode, uint8_t* mine, hipStream_t s) {
  const uint64_t n = (uint64_t)W * NL;
  hipLaunchKernelGGL(k_need_draw<K>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, seed, n_nodes, n0, NL,
                     round0, W, mode, mine);
  return hipGetLastError();
}

hipError_t launch_need_draw(uint64_t seed, uint32_t n_nodes, uint32_t n0, uint32_t NL, uint32_t round0, uint32_t W,
                            int k, int mode, uint8_t* mine, hipStream_t s) {
  if (!NL || !W) return hipSuccess;
#define AVK_NEED(K) launch_need_draw_k<K>(seed, n_nodes, n0, NL, round0, W, mode, mine, s)
  AVK_K_SWITCH(k, AVK_NEED)
#undef AVK_NEED
}

hipError_t launch_need_push(const uint8_t* mine, uint32_t n_nodes, uint32_t NL, uint32_t W, uint32_t world,
                            uint32_t rank, uint32_t par, PeerPtrs needin, hipStream_t s) {
  if (world > (uint32_t)kMaxPeers + 1u || rank >= world) return hipErrorInvalidValue;
  const uint64_t n = (uint64_t)world * W * ((NL + 31u) / 32u);
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_need_push, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, mine, n_nodes, NL, W, world,
                     rank, par, needin);
  return hipGetLastError();
}

hipError_t launch_need_combine(const uint32_t* needin, uint32_t world, uint32_t rank, uint32_t par, uint32_t W,
                               uint32_t NL, uint32_t ref_local, uint8_t* needmask, hipStream_t s) {
  if (world < 2 || world > 9u || rank >= world) return hipErrorInvalidValue;  // <= 8 peers: a byte mask
  const uint64_t n = (uint64_t)W * NL;
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_need_combine, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, needin, world, rank, par, W,
                     NL, ref_local, needmask);
  return hipGetLastError();
}

hipError_t peer_timeout_ticks(int device, uint32_t timeout_ms, uint64_t* ticks) {
  int khz = 0;
  const hipError_t e = hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device);
  if (e != hipSuccess) return e;
  *ticks = (uint64_t)timeout_ms * (uint64_t)(khz > 0 ? khz : 100000);
  return hipSuccess;
}

hipError_t launch_peer_barrier(PeerPtrs arrive, uint32_t world, uint32_t rank, uint32_t seq, uint32_t* err,
                               uint64_t timeout_ticks, hipStream_t s, const uint32_t* slot, PeerPtrs slot_dst,
                               uint32_t wait) {
  if (world > (uint32_t)kMaxPeers + 1u || rank >= world) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_peer_barrier, dim3(1), dim3(64), 0, s, arrive, arrive.p[rank], world, rank, seq, err,
                     timeout_ticks, slot, slot_dst, wait);
  return hipGetLastError();
}

uint64_t poll_sets_scratch_words(uint32_t n) {
  return ((uint64_t)n + 1u) / 2u + 1u + ((uint64_t)n + 1u) + dscan::scan_scratch_words(n);
}

hipError_t launch_poll_sets_batch(const uint32_t* planes, const uint32_t* valid, uint32_t BL, uint32_t nl0,
                                  uint32_t n, uint32_t t0, uint64_t cap, uint64_t* scratch, int64_t* offs_out,
                                  int32_t* targets_out, hipStream_t s) {
  if (!n) return hipSuccess;
  uint32_t* counts = reinterpret_cast<uint32_t*>(scratch);
  uint64_t* offs = scratch + ((uint64_t)n + 1u) / 2u + 1u;
  uint64_t* sc = offs + (uint64_t)n + 1u;
  hipLaunchKernelGGL(k_poll_sets, dim3(n), dim3(64), 0, s, planes, valid, BL, nl0, t0, counts,
                     (const uint64_t*)nullptr, (uint64_t)0, (int64_t*)nullptr, (int32_t*)nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if ((e = dscan::launch_scan(dscan::In32{counts}, n, offs, sc, s)) != hipSuccess) return e;
  hipLaunchKernelGGL(k_poll_sets, dim3(n), dim3(64), 0, s, planes, valid, BL, nl0, t0, (uint32_t*)nullptr,
                     (const uint64_t*)offs, cap, offs_out, targets_out);
  return hipGetLastError();
}

}  // namespace avk
