// Round kernel under the 4096 poll cap (M > 4096, k <= 8): one workgroup per
// node, one lane per 32-record block. GetInvsForNextPoll (processor.go:144-170)
// hands the node's first 4096 live, valid targets in ascending target order
// (rule R1); a workgroup prefix count of the live-valid bits selects them.
//
// The cap set changes inside a round only when a polled record finalizes
// (it is deleted and the next record moves up). So:
//  * no polled record of the node has count >= 120 (the usual case): the poll
//    set is selected once, and the round runs like k_round_sweep — per-slot
//    threshold networks, deferred confidence update, the shift registers of
//    the polled records advanced by k votes at once (round_slots.h);
//  * otherwise the node is flagged and left untouched; a second launch of the
//    first version's exact kernel (kernels.hip k_round_capped: per-vote
//    poll-set re-selection, deletion at 128) processes the flagged nodes only.
//    Keeping the exact path out of this kernel keeps it at ~66 VGPRs.
// Same layout, outputs and counters as k_round_capped; V/K move as dwordx4.
#include <hip/hip_runtime.h>

#include "kernels.h"
#include "round_common.h"
#include "round_slots.h"

namespace avk {
namespace {

// The first (4096 - already) set bits of `bits`, in bit order.
__device__ __forceinline__ uint32_t lowest_bits(uint32_t bits, uint32_t n) {
  uint32_t out = 0u;
  for (uint32_t q = 0; q < n; ++q) {
    const uint32_t low = bits & (0u - bits);
    out |= low;
    bits ^= low;
  }
  return out;
}

// Poll-set selection (processor.go:165-167): the first kMaxPoll set bits of
// `live` over the workgroup's lanes in lane order. Two barriers; wsum is
// double-buffered by `phase`.
__device__ __forceinline__ uint32_t cap_select(uint32_t live, uint32_t lane, uint32_t wave, uint32_t (&wsum)[2][16],
                                               uint32_t phase) {
  const uint32_t c = (uint32_t)__popc(live);
  const uint32_t incl = wave_incl_scan(c, lane);
  if (lane == 63u) wsum[phase][wave] = incl;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t q = 0; q < wave; ++q) before += wsum[phase][q];
  const uint32_t excl = before + incl - c;
  if (excl >= kMaxPoll) return 0u;
  if (excl + c <= kMaxPoll) return live;
  return lowest_bits(live, kMaxPoll - excl);
}

// The state loads of one lane beyond its K4-7 group and A plane (V, K0-3,
// C, the replayed vote planes, or the peer gather).
template <int K, bool REPLAY, bool NT>
struct NodeLane {
  u32x4 v0, v1, k0;
  uint32_t C[8];
  uint32_t w[K], cw[REPLAY ? K : 1];
};

template <int K, bool REPLAY, bool NT>
__device__ __forceinline__ void node_lane_load(const RoundParams& p, uint32_t* tp, u32x4* grp, uint32_t tl, uint32_t g,
                                               uint32_t bc, uint32_t node, uint32_t nl, uint32_t lane,
                                               NodeLane<K, REPLAY, NT>& in) {
  in.v0 = pld4<NT>(grp);
  in.v1 = pld4<NT>(grp + 64);
  in.k0 = pld4<NT>(grp + 128);
#pragma unroll
  for (int i = 0; i < 8; ++i) in.C[i] = pld<NT>(tp + 1024u + (uint32_t)i * 64u + tl);
  if constexpr (REPLAY) {
    if (p.ablate_node & 2u) {  // diagnostics: no replay loads
#pragma unroll
      for (int j = 0; j < K; ++j) {
        in.cw[j] = ~(g * 0x9E3779B9u + (uint32_t)j);
        in.w[j] = g * 0x85EBCA6Bu ^ (uint32_t)j;
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      in.cw[j] = p.replay[(size_t)(2 * j + 1) * p.Lpad + g];
      in.w[j] = p.replay[(size_t)(2 * j) * p.Lpad + g];
    }
  } else {
    uint32_t peers[K];
    draw_peers<K>(p, p.round, node, nl, nl, 1u, lane, peers);  // every lane of the workgroup is the same node
#pragma unroll
    for (int j = 0; j < K; ++j) in.w[j] = p.pref_in[peers[j] * p.BL + bc];  // < N * BL < 2^31 (engine check)
  }
}

// One workgroup per node, one lane per 32-record block. Only the first
// kMaxPoll live valid records of the node are polled (processor.go:165-167),
// so the lanes of blocks b >= kMaxPoll / 32 (C2: 185 of 313) are polled only
// when dead or invalid records come before them. Those lanes load their K4-7
// group and A plane only; after the workgroup prefix count, a wave with a
// polled record loads the rest (rare), a wave without one just republishes A
// (24 B per lane instead of ~270). Lanes of blocks b < kMaxPoll / 32 can
// always be polled and issue every load at once.
template <int K, bool REPLAY, bool NT, int MAXT>
__global__ __launch_bounds__(MAXT) void k_round_node(const RoundParams p) {
  __shared__ uint32_t wsum[2][16];
  const uint32_t nl = blockIdx.x;
  const uint32_t b = threadIdx.x;
  const uint32_t lane = b & 63u, wave = b >> 6;
  const bool active = b < p.BL;
  const uint32_t bc = active ? b : p.BL - 1u;  // inactive lanes read a valid lane, never store
  const uint32_t g = nl * p.BL + bc;
  const uint32_t node = p.n0 + nl;
  const bool early = b < kMaxPoll / 32u;  // wave-uniform (128 lanes = 2 waves)

  // ---- state (tile layout of kernels.h: per-lane dwordx4 V/K groups, dword C/A planes)
  uint32_t* const tp = p.planes + (size_t)(g >> 6) * (kPlanes * 64u);
  const uint32_t tl = g & 63u;
  u32x4* const grp = reinterpret_cast<u32x4*>(tp) + tl;
  const u32x4 k1 = pld4<NT>(grp + 192);
  uint32_t A = pld<NT>(tp + 1536u + tl);
  const uint32_t vmask = active ? p.valid[bc] : 0u;
  NodeLane<K, REPLAY, NT> in;
  if (early) node_lane_load<K, REPLAY, NT>(p, tp, grp, tl, g, bc, node, nl, lane, in);

  const uint32_t live0 = ~k1[3];
  const uint32_t P0 = live0 & vmask;  // live and IsValid (processor.go:95-103)
  const uint32_t polled = cap_select(P0, lane, wave, wsum, 0u);
  const bool heavy = early || __ballot(polled != 0u) != 0ull;  // wave-uniform
  if (!early && heavy) node_lane_load<K, REPLAY, NT>(p, tp, grp, tl, g, bc, node, nl, lane, in);
  const uint32_t nearfin = heavy ? polled & k1[2] & k1[1] & k1[0] & in.k0[3] : 0u;  // count >= 120
  const bool exact = __syncthreads_or(nearfin != 0u) != 0;  // workgroup-uniform

  if (exact) {  // some polled record may reach 128: the exact pass (k_round_capped) takes this node
    if (b == 0) p.node_flags[nl] = 1u;
    return;
  }
  const uint32_t wave_id = blockIdx.x * (blockDim.x >> 6) + wave;  // dense: matches log_shards sizing
  const uint32_t prow = node * p.BL + b;
  const uint32_t pub_byz = is_byz(p.byz, node) ? 1u : 0u;
  if (!heavy) {  // nothing polled in this wave: records unchanged, A republished
    if (active) p.pref_out[prow] = pub_byz ? byz_pattern(p.round + 1u) : A;
    count_stats(p, wave_id, lane, 0u, active, 16u + 4u + 4u, 0u, 0u, 0u);
    return;
  }

  // ---- votes of this round: ys/ns hold y/n of [V_6..V_0, w_0..w_{K-1}]
  uint32_t ys[7 + K], ns[7 + K], cwv[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t cw = REPLAY ? in.cw[REPLAY ? j : 0] : ~0u;
    const uint32_t yw = in.w[j] & cw;  // err == 0 implies considered
    ys[7 + j] = yw;
    ns[7 + j] = ~yw & cw;
    cwv[j] = cw;
  }
  const u32x4 v0 = in.v0, v1 = in.v1, k0 = in.k0;
  const uint32_t* const C = in.C;
#pragma unroll
  for (int i = 0; i < 7; ++i) {  // old planes V_6..V_0
    const uint32_t vi = (6 - i) < 4 ? v0[6 - i] : v1[2 - i];
    ys[i] = vi & C[6 - i];
    ns[i] = ~vi & C[6 - i];
  }
  uint32_t Kp[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Kp[i] = k0[i];
    Kp[4 + i] = k1[i];
  }
  uint32_t E[K], applied = 0u;
  const uint32_t died = 0u;
  // the poll set is fixed for the round: every polled record shifts by K
  // votes; its V/C planes are final now (stored before the slot loop so
  // their registers are free during it). A lane with no polled record keeps
  // its planes: no stores.
  const bool any = polled != 0u;
  const bool st = !(p.ablate_node & 4u);  // diagnostics: no plane stores
  if (active && any && st) {
    u32x4 o0, o1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t vi = i < 4 ? v0[i] : v1[i - 4];
      const uint32_t vs = i < K ? ys[6 + K - i] : (i - K < 4 ? v0[i - K] : v1[i - K - 4]);
      const uint32_t vn = (vs & polled) | (vi & ~polled);
      if (i < 4)
        o0[i] = vn;
      else
        o1[i - 4] = vn;
      const uint32_t cs = i < K ? cwv[K - 1 - i] : C[i - K];
      pst<NT>(tp + 1024u + (uint32_t)i * 64u + tl, (cs & polled) | (C[i] & ~polled));
    }
    pst4<NT>(grp, o0);
    pst4<NT>(grp + 64, o1);
  }
  {
    uint32_t alive = polled, c[4] = {0u, 0u, 0u, 0u}, F = 0u;
    const uint32_t low3[3] = {Kp[0], Kp[1], Kp[2]};
    round_slots<K, false>(ys, ns, low3, 0u, false, alive, A, E, c, F, applied);
    applied = (uint32_t)K * (uint32_t)__popc(polled);
    uint32_t cy = 0u;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const uint32_t ci = i < 4 ? c[i] : 0u;
      const uint32_t t = Kp[i] ^ ci;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[i] & ci);
      Kp[i] = (F & ci) | (~F & si);
    }
  }

  if (active) {
    if (any && st) {
      u32x4 o2, o3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o2[i] = Kp[i];
        o3[i] = Kp[4 + i];
      }
      pst4<NT>(grp + 128, o2);
      pst4<NT>(grp + 192, o3);
      pst<NT>(tp + 1536u + tl, A);
    }
    p.pref_out[prow] = pub_byz ? byz_pattern(p.round + 1u) : A;
  }
  uint32_t upd = 0;
  const uint32_t emitted = emit_updates<K>(p, wave_id, lane, node, p.t0 + b * 32u, E, A, died, upd);
  // bytes: a lane of a polling wave reads all 25 planes and its k vote words,
  // writes its published word, and writes its planes back if it polled a record
  const uint32_t lane_bytes = kPlanes * 4u + (REPLAY ? 8u : 4u) * K + 4u + (any ? kPlanes * 4u : 0u);
  count_stats(p, wave_id, lane, applied, active, lane_bytes, emitted, upd, died);
}

template <int K, int MAXT>
hipError_t launch_node_t(const RoundParams& p, bool replay, uint32_t bt, hipStream_t s) {
  if (replay) {
    if (p.plane_nt)
      hipLaunchKernelGGL((k_round_node<K, true, true, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
    else
      hipLaunchKernelGGL((k_round_node<K, true, false, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
  } else {
    if (p.plane_nt)
      hipLaunchKernelGGL((k_round_node<K, false, true, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
    else
      hipLaunchKernelGGL((k_round_node<K, false, false, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
  }
  return hipGetLastError();
}

// workgroup = the node's blocks rounded up to whole waves; a 512-thread bound
// (M <= 16384) leaves the register allocator room (no scratch)
template <int K>
hipError_t launch_node_k(const RoundParams& p, bool replay, hipStream_t s) {
  uint32_t bt = ((p.BL + 63u) / 64u) * 64u;
  if ((p.ablate_node & 1u) && bt > kMaxPoll / 32u) bt = kMaxPoll / 32u;  // diagnostics: lanes past the cap never run
  return bt <= 512u ? launch_node_t<K, 512>(p, replay, bt, s) : launch_node_t<K, 1024>(p, replay, bt, s);
}

}  // namespace

hipError_t launch_round_node(const RoundParams& p, int k, bool replay, bool exact_pass, hipStream_t s) {
  if (!p.node_flags) return hipErrorInvalidValue;
  hipError_t e;
  switch (k) {
    case 1: e = launch_node_k<1>(p, replay, s); break;
    case 2: e = launch_node_k<2>(p, replay, s); break;
    case 3: e = launch_node_k<3>(p, replay, s); break;
    case 4: e = launch_node_k<4>(p, replay, s); break;
    case 5: e = launch_node_k<5>(p, replay, s); break;
    case 6: e = launch_node_k<6>(p, replay, s); break;
    case 7: e = launch_node_k<7>(p, replay, s); break;
    case 8: e = launch_node_k<8>(p, replay, s); break;
    default: return hipErrorInvalidValue;
  }
  if (e != hipSuccess || !exact_pass) return e;
  return launch_round(p, k, replay, /*capped=*/true, s);  // the exact pass over the flagged nodes
}

}  // namespace avk
