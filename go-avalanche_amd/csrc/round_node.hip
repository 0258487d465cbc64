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
    replay_load<K>(p.replay, g, in.w, in.cw);
  } else {
    uint32_t peers[K];
    draw_peers<K>(p, p.round, node, nl, nl, 1u, lane, peers);  // every lane of the workgroup is the same node
#pragma unroll
    for (int j = 0; j < K; ++j) in.w[j] = p.pref_in[peers[j] * p.PS + bc];  // < N * BL < 2^31 (engine check)
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
  const uint32_t prow = node * p.PS + b;
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
  const uint32_t emitted = emit_updates_flat<K>(p, wave_id, lane, node, p.t0 + b * 32u, E, A, died, upd, p.round_rel);
  // bytes: a lane of a polling wave reads all 25 planes and its k vote words,
  // writes its published word, and writes its planes back if it polled a record
  const uint32_t lane_bytes = kPlanes * 4u + (REPLAY ? 8u : 4u) * K + 4u + (any ? kPlanes * 4u : 0u);
  count_stats(p, wave_id, lane, applied, active, lane_bytes, emitted, upd, died);
}

// Fused replay rounds: p.fuse_rounds consecutive replay rounds of one node
// in one workgroup. In replay mode a node's votes come from its own stream,
// never from another node's published preference (processor.go:92-117 on
// recorded Responses), so its records evolve independently of every other
// node and a workgroup can carry them through R rounds in registers: the 25
// planes are read once and written once per launch instead of once per
// round. The poll set (processor.go:165-167) can change inside a round only
// when a polled record finalizes, so it is selected once; before each round
// the workgroup checks whether a polled record has count >= 120 and, if so,
// stores the state reached so far and leaves the node to the exact pass from
// that round on (node_flags[nl] = 1 + round; k_round_capped runs it per
// round). Every round's votes are applied and its StatusUpdates emitted with
// its own round key; the published word is written for the last three rounds
// of the launch (the three snapshot buffers; replay rounds do not read them).
template <int K, bool NT, int MAXT>
__global__ __launch_bounds__(MAXT) void k_replay_node(const RoundParams p) {
  __shared__ uint32_t wsum[2][16];
  const uint32_t nl = blockIdx.x;
  const uint32_t b = threadIdx.x;
  const uint32_t lane = b & 63u, wave = b >> 6;
  const bool active = b < p.BL;
  const uint32_t bc = active ? b : p.BL - 1u;  // inactive lanes read a valid lane, never store
  const uint32_t g = nl * p.BL + bc;
  const uint32_t node = p.n0 + nl;
  // wave-uniform; waves 0-1 always (kMaxPoll / 32 = 128 lanes): wave 0 is always heavy, which the
  // round loop's barriers rely on
  const bool early = b < kMaxPoll / 32u;
  static_assert(kMaxPoll / 32u >= 64u, "wave 0 must be early (heavy)");

  uint32_t* const tp = p.planes + (size_t)(g >> 6) * (kPlanes * 64u);
  const uint32_t tl = g & 63u;
  u32x4* const grp = reinterpret_cast<u32x4*>(tp) + tl;
  const u32x4 k1 = pld4<NT>(grp + 192);
  const uint32_t vmask = active ? p.valid[bc] : 0u;
  // k_replay_fast ran this launch's rounds for nodes whose first 128 lanes hold 4096 live, valid
  // records (the poll set is exactly those) and published their other lanes' words: such a node's
  // workgroup leaves before any other load (workgroup-uniform)
  if (p.replay_fast && p.BL >= kMaxPoll / 32u && __syncthreads_and(!early || (~k1[3] & vmask) == ~0u)) return;
  uint32_t A = pld<NT>(tp + 1536u + tl);
  u32x4 v0 = u32x4{0u, 0u, 0u, 0u}, v1 = v0, k0 = v0;
  uint32_t C[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) C[i] = 0u;
  if (early) {
    v0 = pld4<NT>(grp);
    v1 = pld4<NT>(grp + 64);
    k0 = pld4<NT>(grp + 128);
#pragma unroll
    for (int i = 0; i < 8; ++i) C[i] = pld<NT>(tp + 1024u + (uint32_t)i * 64u + tl);
  }
  const uint32_t P0 = ~k1[3] & vmask;  // live and IsValid (processor.go:95-103)
  const uint32_t polled = cap_select(P0, lane, wave, wsum, 0u);
  // k_replay_fast ran this launch's rounds for nodes whose first 128 lanes hold 4096 live, valid
  // records (the poll set is exactly those): only their other lanes' published words are left here
  const bool fast_node = p.replay_fast && p.BL >= kMaxPoll / 32u && wsum[0][0] + wsum[0][1] == kMaxPoll;
  if (fast_node) {  // workgroup-uniform; no barrier follows for this workgroup
    if (!early) {   // records unchanged through the launch: publish the last three rounds
      const uint32_t R = p.fuse_rounds, r0 = R > 3u ? R - 3u : 0u;
      const bool byz = is_byz(p.byz, node);
      for (uint32_t r = r0; r < R; ++r)
        if (active) p.pref_ring[(p.ring_next + r) % 3u][node * p.PS + b] = byz ? byz_pattern(p.round + r + 1u) : A;
      count_stats(p, blockIdx.x * (blockDim.x >> 6) + wave, lane, 0u, active, 20u + 4u + 4u * (R - r0), 0u, 0u, 0u);
    }
    return;
  }
  const bool heavy = early || __ballot(polled != 0u) != 0ull;  // wave-uniform
  if (!early && heavy) {
    v0 = pld4<NT>(grp);
    v1 = pld4<NT>(grp + 64);
    k0 = pld4<NT>(grp + 128);
#pragma unroll
    for (int i = 0; i < 8; ++i) C[i] = pld<NT>(tp + 1024u + (uint32_t)i * 64u + tl);
  }
  uint32_t V[8], Kp[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    V[i] = v0[i];
    V[4 + i] = v1[i];
    Kp[i] = k0[i];
    Kp[4 + i] = k1[i];
  }
  const uint32_t wave_id = blockIdx.x * (blockDim.x >> 6) + wave;  // dense: matches log_shards sizing
  const uint32_t prow = node * p.PS + b;
  const bool byz = is_byz(p.byz, node);
  const uint32_t R = p.fuse_rounds;
  // A count grows by at most K per round, so no polled record can reach 120
  // before round J = ceil((120 - max count) / K): those rounds need no
  // workgroup check (the waves run them without a barrier).
  uint32_t hi = 0u;  // bit q: some polled record of the lane has count bit q set, ignoring lower bits
  {
    uint32_t m = polled;  // records whose count matches the maximum so far, bit by bit from the top
#pragma unroll
    for (int q = 6; q >= 0; --q) {
      const uint32_t t = m & Kp[q];
      if (t) {
        m = t;
        hi |= 1u << q;
      }
    }
    if (!heavy || !polled) hi = 0u;
  }
  uint32_t wm = hi;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) wm = max(wm, (uint32_t)__shfl_xor((int)wm, o, 64));
  if (lane == 0) wsum[1][wave] = wm;  // (cap_select used wsum[0])
  __syncthreads();
  uint32_t maxc = 0u;  // largest polled count of the node
  for (uint32_t q = 0; q < (blockDim.x >> 6); ++q) maxc = max(maxc, wsum[1][q]);
  const uint32_t J = maxc >= 120u ? 0u : (120u - maxc + (uint32_t)K - 1u) / (uint32_t)K;
  if (!heavy) {
    // no polled record in this wave: its records and published words stay
    // as they are through the launch (a record leaves or joins the poll set
    // only in the exact pass, which rewrites the node's rows of its rounds
    // afterwards). Publish the last three rounds now and end the wave: its
    // registers go to other workgroups, and the barriers below count only the
    // waves still running.
    const uint32_t r0 = R > 3u ? R - 3u : 0u;
    for (uint32_t r = r0; r < R; ++r)
      if (active) p.pref_ring[(p.ring_next + r) % 3u][prow] = byz ? byz_pattern(p.round + r + 1u) : A;
    count_stats(p, wave_id, lane, 0u, active, 20u + 4u + 4u * (R - r0), 0u, 0u, 0u);
    return;
  }
  uint32_t done = R, applied = 0u, upd = 0u, emitted = 0u, pubs = 0u;
  for (uint32_t r = 0; r < R; ++r) {
    // a polled record with count >= 120 may finalize (and leave the poll set) this round.
    // Only the heavy waves reach this barrier: the light ones ended above. CDNA's s_barrier counts
    // the waves of the workgroup that have not ended, and wave 0 (lanes 0-63, early) is always
    // heavy, so the workgroup's barrier is never empty (see the comment on `early`).
    if (r >= J) {
      const uint32_t nearfin = heavy ? polled & Kp[6] & Kp[5] & Kp[4] & Kp[3] : 0u;
      if (__syncthreads_or(nearfin != 0u)) {  // workgroup-uniform
        done = r;
        break;
      }
    }
    uint32_t E[K];
    if (heavy) {
      uint32_t w[K], cw[K];
      replay_load<K>(p.replay + (size_t)r * p.replay_stride, g, w, cw);
      // ys/ns: y/n of [V_6..V_0, w_0..w_{K-1}] (vote.go:55-56)
      uint32_t ys[7 + K], ns[7 + K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t yw = w[j] & cw[j];  // err == 0 implies considered
        ys[7 + j] = yw;
        ns[7 + j] = ~yw & cw[j];
      }
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        ys[i] = V[6 - i] & C[6 - i];
        ns[i] = ~V[6 - i] & C[6 - i];
      }
      // every polled record shifts in the K votes (vote.go:55-56)
#pragma unroll
      for (int i = 7; i >= 0; --i) {
        const uint32_t vs = i < K ? ys[6 + K - i] : V[i - K];
        const uint32_t cs = i < K ? cw[K - 1 - i] : C[i - K];
        V[i] = (vs & polled) | (V[i] & ~polled);
        C[i] = (cs & polled) | (C[i] & ~polled);
      }
      uint32_t alive = polled, c[4] = {0u, 0u, 0u, 0u}, F = 0u, ap = 0u;
      const uint32_t low3[3] = {Kp[0], Kp[1], Kp[2]};
      round_slots<K, false>(ys, ns, low3, 0u, false, alive, A, E, c, F, ap);
      applied += (uint32_t)K * (uint32_t)__popc(polled);
      uint32_t cy = 0u;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint32_t ci = i < 4 ? c[i] : 0u;
        const uint32_t t = Kp[i] ^ ci;
        const uint32_t si = t ^ cy;
        cy = (t & cy) | (Kp[i] & ci);
        Kp[i] = (F & ci) | (~F & si);
      }
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) E[j] = 0u;
    }
    if (r + 3u >= R) {  // the last three rounds fill the three snapshot buffers
      if (active) p.pref_ring[(p.ring_next + r) % 3u][prow] = byz ? byz_pattern(p.round + r + 1u) : A;
      ++pubs;
    }
    if (heavy) emitted += emit_updates_flat<K>(p, wave_id, lane, node, p.t0 + b * 32u, E, A, 0u, upd, p.round_rel + r);
  }
  if (done < R && b == 0) p.node_flags[nl] = done + 1u;  // the exact pass takes rounds done..R-1
  const bool any = heavy && polled != 0u && done > 0u;
  if (active && any) {
    pst4<NT>(grp, u32x4{V[0], V[1], V[2], V[3]});
    pst4<NT>(grp + 64, u32x4{V[4], V[5], V[6], V[7]});
#pragma unroll
    for (int i = 0; i < 8; ++i) pst<NT>(tp + 1024u + (uint32_t)i * 64u + tl, C[i]);
    pst4<NT>(grp + 128, u32x4{Kp[0], Kp[1], Kp[2], Kp[3]});
    pst4<NT>(grp + 192, u32x4{Kp[4], Kp[5], Kp[6], Kp[7]});
    pst<NT>(tp + 1536u + tl, A);
  }
  // bytes: state read once (heavy: 25 planes, light: K4-7 and A) and written
  // once if a record was polled; 8 B per replayed vote word pair per round;
  // the published words written
  const uint32_t lane_bytes = (heavy ? kPlanes * 4u + 8u * K * done : 20u) + 4u + 4u * pubs +
                              (any ? kPlanes * 4u : 0u);
  count_stats(p, wave_id, lane, applied, active, lane_bytes, emitted, upd, 0u);
}

// Fused replay rounds for a node whose first 128 lanes (4096 targets) hold
// 4096 live, valid records: the poll set (processor.go:165-167) is exactly
// those records until one of them is deleted, which only the exact pass does,
// so the node's other lanes take no vote in the launch (k_replay_node
// publishes their words). One 128-thread workgroup per node, lane b = block
// b: every record of every lane is polled, so the vote and consider registers
// shift without masks. Few waves (2 per node) and a large register budget:
// the next round's replayed votes are loaded while this round is computed.
// Same round loop, hand-off to the exact pass (count >= 120), StatusUpdates,
// published words and counters as k_replay_node.
#ifndef AVK_REPLAY_LATE_REFILL
#define AVK_REPLAY_LATE_REFILL 0
#endif
// A/B knob: the StatusUpdate pipeline's depth (k = 8): 1 = round r's entries stored in round r + 1
// (two pending sets), 2 = in round r + 2 (four sets, loop unrolled four times), so that the wait for
// the reserving atomic's result (vmcnt counts in issue order: also every load and store issued before
// it) is for operations two rounds old
// A/B knob: the near-finalization check (a workgroup barrier) every round instead of from round J on
#ifndef AVK_REPLAY_ALWAYS_CHECK
#define AVK_REPLAY_ALWAYS_CHECK 0
#endif
#ifndef AVK_REPLAY_VMWAIT
#define AVK_REPLAY_VMWAIT 0
#endif
#ifndef AVK_REPLAY_BUF3
#define AVK_REPLAY_BUF3 0
#endif
#ifndef AVK_REPLAY_PIPE3
#define AVK_REPLAY_PIPE3 0
#endif
#ifndef AVK_REPLAY_PIPE3_LATE
#define AVK_REPLAY_PIPE3_LATE 0
#endif
// (round 5, tools/fuse_probe.py --repeat 15, three alternations on one box: depth 2 3.52-3.53 us per
// round against 3.69-3.73 at depth 1; profiles/r05/s11/ab_c2e.log)
#ifndef AVK_REPLAY_EMIT_DEPTH
#define AVK_REPLAY_EMIT_DEPTH 2
#endif
template <int K, bool NT>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void k_replay_fast(const RoundParams p) {
  __shared__ uint32_t wmax[2];
  const uint32_t nl = blockIdx.x;
  const uint32_t b = threadIdx.x;  // < 128 <= BL
  const uint32_t lane = b & 63u, wave = b >> 6;
  const uint32_t g = nl * p.BL + b;
  const uint32_t node = p.n0 + nl;
  uint32_t* const tp = p.planes + (size_t)(g >> 6) * (kPlanes * 64u);
  const uint32_t tl = g & 63u;
  u32x4* const grp = reinterpret_cast<u32x4*>(tp) + tl;
  // every load of the launch's start issued at once (planes, the first two rounds' replayed votes),
  // before the eligibility barrier: one memory latency instead of three in a row (an ineligible node,
  // rare, has loaded for nothing and runs in k_replay_node)
  const u32x4 k1 = pld4<NT>(grp + 192);
  const uint32_t vmask = p.valid[b];
  uint32_t A = pld<NT>(tp + 1536u + tl);
  const u32x4 v0 = pld4<NT>(grp), v1 = pld4<NT>(grp + 64), k0 = pld4<NT>(grp + 128);
  uint32_t V[8], C[8], Kp[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    V[i] = v0[i];
    V[4 + i] = v1[i];
    Kp[i] = k0[i];
    Kp[4 + i] = k1[i];
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) C[i] = pld<NT>(tp + 1024u + (uint32_t)i * 64u + tl);
  const uint32_t R = p.fuse_rounds;
  // replayed (yes, consider) word pairs as loaded: {w_2i, cw_2i, w_2i+1, cw_2i+1} per dwordx4 (kept as
  // vectors, so the refilled buffer is the loads' own registers across the loop)
  constexpr int RQ = (K + 1) / 2;
  const u32x4* const rq = reinterpret_cast<const u32x4*>(p.replay) + (size_t)(g >> 6) * (RQ * 64) + (g & 63u);
  const size_t rstride = p.replay_stride / 4u;  // u32x4 per round
  u32x4 wb0[RQ], wb1[RQ];
#pragma unroll
  for (int i = 0; i < RQ; ++i) wb0[i] = pld4<true>(rq + i * 64);
#pragma unroll
  for (int i = 0; i < RQ; ++i) wb1[i] = pld4<true>(rq + (R > 1u ? rstride : 0u) + i * 64);  // (R = 1: unused)
  // eligibility: every record of lanes 0..127 live and valid
  const bool all = __syncthreads_and((~k1[3] & vmask) == ~0u) != 0;
  if (!all) return;  // workgroup-uniform: k_replay_node runs the node
  const uint32_t wave_id = blockIdx.x * 2u + wave;
  const uint32_t prow = node * p.PS + b;
  const bool byz = is_byz(p.byz, node);
  // the node's other lanes take no vote in the launch (the poll set is lanes 0..127): their records
  // are unchanged, so their published words for the launch's last three rounds are their A planes
  // (loaded here, stored after the round loop: no load latency before the loop)
  constexpr uint32_t kOther = 2u;  // other lanes per thread: BL <= 3 * 128 (M <= 12288; more take k_replay_node's
                                   // per-lane loop below)
  uint32_t Aother[kOther];
#pragma unroll
  for (uint32_t q = 0; q < kOther; ++q) {
    const uint32_t lb = b + (q + 1u) * (kMaxPoll / 32u);
    const uint32_t go = nl * p.BL + lb;
    Aother[q] = lb < p.BL ? pld<NT>(p.planes + (size_t)(go >> 6) * (kPlanes * 64u) + 1536u + (go & 63u)) : 0u;
  }
  // largest count of the node (bit by bit from the top, as k_replay_node): no record can reach 120
  // before round J, so those rounds need no workgroup check
  uint32_t hi = 0u;
  {
    uint32_t m = ~0u;
#pragma unroll
    for (int q = 6; q >= 0; --q) {
      const uint32_t t = m & Kp[q];
      if (t) {
        m = t;
        hi |= 1u << q;
      }
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) hi = max(hi, (uint32_t)__shfl_xor((int)hi, o, 64));
  if (lane == 0) wmax[wave] = hi;
  __syncthreads();
  const uint32_t maxc = max(wmax[0], wmax[1]);
  const uint32_t J = maxc >= 120u ? 0u : (120u - maxc + (uint32_t)K - 1u) / (uint32_t)K;
  uint32_t done = R, applied = 0u, upd = 0u, emitted = 0u, pubs = 0u;
  // The replayed votes are prefetched two rounds ahead into two register buffers, (wb0) for even
  // rounds and (wb1) for odd ones (the loop is unrolled twice): a round refills its own buffer with
  // round r + 2's votes as soon as it has read them, and no register is copied while a load into it
  // is in flight (a rotating copy made every round wait for the load issued at its start).
  // StatusUpdates (k = 8: one entry per lane): round r's log space is reserved at the end of round r
  // and its entries stored after round r + 1's slot network, so the reserving atomics' round trip
  // overlaps a round of compute; the pending reservations alternate between two sets of registers too.
  EmitRes pendA{}, pendB{};
  uint32_t EpA[K], EpB[K], ApA = 0u, ApB = 0u;
  const uint32_t shard = wave_id % p.log_shards;  // once (a runtime modulo is a long sequence)
  // wb: this round's replayed votes; nb: the buffer refilled with round r + 2's (wb itself with two
  // buffers; with three (AVK_REPLAY_BUF3) the one read last round, whose registers are free)
  auto step = [&](uint32_t r, u32x4 (&wb)[RQ], u32x4 (&nb)[RQ], EmitRes& pc, uint32_t (&Ec)[K], uint32_t& Ac,
                  const EmitRes& pp, const uint32_t (&Ep)[K], uint32_t Ap) -> bool {
    if (AVK_REPLAY_ALWAYS_CHECK || r >= J) {  // a record with count >= 120 may finalize (and leave the poll set) this round
      const uint32_t nearfin = Kp[6] & Kp[5] & Kp[4] & Kp[3];
      if (__syncthreads_or(nearfin != 0u)) {  // workgroup-uniform
        done = r;
        return false;
      }
    }
    uint32_t ys[7 + K], ns[7 + K], cv[K];
#if AVK_REPLAY_VMWAIT
    // this round's votes were loaded two rounds ago, and at least the RQ loads of last round's refill
    // were issued after them: vmcnt(RQ) retires them (vmcnt counts in issue order). The compiler's own
    // wait, which merges the loop's paths (stores and atomics in lane-conditional blocks), asked for
    // vmcnt(0) here, i.e. for the refill just issued too: one memory latency per round
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt((RQ & 15) | (7 << 4) | (15 << 8) | ((RQ >> 4) << 14));
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const uint32_t wj = wb[j >> 1][(j & 1) * 2];
      cv[j] = wb[j >> 1][(j & 1) * 2 + 1];
      const uint32_t yw = wj & cv[j];  // err == 0 implies considered (vote.go:55-56)
      ys[7 + j] = yw;
      ns[7 + j] = ~yw & cv[j];
    }
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      ys[i] = V[6 - i] & C[6 - i];
      ns[i] = ~V[6 - i] & C[6 - i];
    }
#pragma unroll
    for (int i = 7; i >= 0; --i) {  // every record shifts in the K votes
      V[i] = i < K ? ys[6 + K - i] : V[i - K];
      if (i < K) {  // a real copy: C must not stay in the buffer's registers, which the refill reuses
        uint32_t cc;
        asm volatile("v_mov_b32 %0, %1" : "=v"(cc) : "v"(cv[K - 1 - i]));
        C[i] = cc;
      } else {
        C[i] = C[i - K];
      }
    }
    // the buffer is read: refill it with round r + 2's votes (unconditionally — the last two rounds
    // reload round R - 1's, unused — so that the loaded registers need no merge copy, which would wait)
    // (no instruction crosses this point: the loads below are not hoisted above the buffer's last
    // reads, so the buffer and the loads' destinations can be the same registers across the loop)
    auto refill = [&]() {
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RQ; ++i) nb[i] = pld4<true>(rq + (size_t)min(r + 2u, R - 1u) * rstride + i * 64);
    };
    if (!(K == 8 && AVK_REPLAY_LATE_REFILL)) refill();
    // the round's update masks go straight into this round's pending set (no copy)
    uint32_t alive = ~0u, c[4] = {0u, 0u, 0u, 0u}, F = 0u, ap = 0u;
    const uint32_t low3[3] = {Kp[0], Kp[1], Kp[2]};
    round_slots<K, false>(ys, ns, low3, 0u, false, alive, A, Ec, c, F, ap);
    applied += (uint32_t)K * 32u;
    uint32_t cy = 0u;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const uint32_t ci = i < 4 ? c[i] : 0u;
      const uint32_t t = Kp[i] ^ ci;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[i] & ci);
      Kp[i] = (F & ci) | (~F & si);
    }
    if (r + 3u >= R) {  // the last three rounds fill the three snapshot buffers
      p.pref_ring[(p.ring_next + r) % 3u][prow] = byz ? byz_pattern(p.round + r + 1u) : A;
      ++pubs;
    }
    if constexpr (K == 8) {
      pc = emit_reserve_med<K>(p, shard, lane, Ec, 0u, upd);
      // AVK_REPLAY_LATE_REFILL: the refill issued after this round's reserving atomic, so that the
      // store of round r - 1's entries below (which waits for round r - 1's atomic: vmcnt counts in
      // issue order) does not also wait for the votes of round r + 1, loaded after that atomic
      if (AVK_REPLAY_LATE_REFILL) refill();
      if (r >= (uint32_t)AVK_REPLAY_EMIT_DEPTH)
        emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, Ep, Ap, 0u, pp,
                                     p.round_rel + r - (uint32_t)AVK_REPLAY_EMIT_DEPTH);
      Ac = A;
    } else {
      (void)pc;
      (void)Ac;
      (void)pp;
      (void)Ep;
      (void)Ap;
      emitted += emit_updates_flat<K>(p, wave_id, lane, node, p.t0 + b * 32u, Ec, A, 0u, upd, p.round_rel + r);
    }
    return true;
  };
#if AVK_REPLAY_PIPE3
  if constexpr (K == 8) {
    // The emission one step later still: round q's update masks are made in step q, its log space
    // reserved at the start of step q + 1 and its entries stored at the start of step q + 2, beside
    // the refill. Every memory operation of a step is then issued before its slot network, so that
    // when the next step's head waits for everything outstanding (the compiler's vmcnt(0) there:
    // stores and atomics sit in lane-conditional blocks), those operations are a whole step old.
    // Three vote buffers and three (E, A, reservation) sets, the loop unrolled three times.
    EmitRes RX{}, RY{}, RZ{};
    uint32_t EX[K], EY[K], EZ[K], AX = 0u, AY = 0u, AZ = 0u;
    u32x4 wb2[RQ];
    auto stepP = [&](uint32_t r, u32x4 (&wb)[RQ], u32x4 (&nb)[RQ], uint32_t (&Ec)[K], uint32_t& Ac,
                     const uint32_t (&Er)[K], EmitRes& Rr, const uint32_t (&Es)[K], uint32_t As,
                     const EmitRes& Rs) -> bool {
      if (r >= J) {
        const uint32_t nearfin = Kp[6] & Kp[5] & Kp[4] & Kp[3];
        if (__syncthreads_or(nearfin != 0u)) {
          done = r;
          return false;
        }
      }
      uint32_t ys[7 + K], ns[7 + K], cv[K];
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint32_t wj = wb[j >> 1][(j & 1) * 2];
        cv[j] = wb[j >> 1][(j & 1) * 2 + 1];
        const uint32_t yw = wj & cv[j];  // err == 0 implies considered (vote.go:55-56)
        ys[7 + j] = yw;
        ns[7 + j] = ~yw & cv[j];
      }
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        ys[i] = V[6 - i] & C[6 - i];
        ns[i] = ~V[6 - i] & C[6 - i];
      }
#pragma unroll
      for (int i = 7; i >= 0; --i) {
        V[i] = i < K ? ys[6 + K - i] : V[i - K];
        if (i < K) {
          uint32_t cc;
          asm volatile("v_mov_b32 %0, %1" : "=v"(cc) : "v"(cv[K - 1 - i]));
          C[i] = cc;
        } else {
          C[i] = C[i - K];
        }
      }
      // round r - 2's entries first: their wait for its reservation (made a step ago; vmcnt counts in
      // issue order) then covers nothing issued in this step; then round r - 1's reservation and the
      // refill, which the next step's head waits for a whole step later
      if (r >= 2u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, Es, As, 0u, Rs, p.round_rel + r - 2u);
      if (r >= 1u) Rr = emit_reserve_med<K>(p, shard, lane, Er, 0u, upd);  // round r - 1
#if !AVK_REPLAY_PIPE3_LATE
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RQ; ++i) nb[i] = pld4<true>(rq + (size_t)min(r + 2u, R - 1u) * rstride + i * 64);
      __builtin_amdgcn_sched_barrier(0);
#endif
      uint32_t alive = ~0u, c[4] = {0u, 0u, 0u, 0u}, F = 0u, ap = 0u;
      const uint32_t low3[3] = {Kp[0], Kp[1], Kp[2]};
      round_slots<K, false>(ys, ns, low3, 0u, false, alive, A, Ec, c, F, ap);
      applied += (uint32_t)K * 32u;
      uint32_t cy = 0u;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint32_t ci = i < 4 ? c[i] : 0u;
        const uint32_t t = Kp[i] ^ ci;
        const uint32_t si = t ^ cy;
        cy = (t & cy) | (Kp[i] & ci);
        Kp[i] = (F & ci) | (~F & si);
      }
      if (r + 3u >= R) {  // the last three rounds fill the three snapshot buffers
        p.pref_ring[(p.ring_next + r) % 3u][prow] = byz ? byz_pattern(p.round + r + 1u) : A;
        ++pubs;
      }
#if AVK_REPLAY_PIPE3_LATE
      // the refill as the step's last memory operations: whatever else the step issued (stores and
      // atomics in lane-conditional blocks), at least these RQ loads follow the buffer the next step
      // reads, on every path
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < RQ; ++i) nb[i] = pld4<true>(rq + (size_t)min(r + 2u, R - 1u) * rstride + i * 64);
#endif
      Ac = A;
      return true;
    };
    for (uint32_t r = 0; r < R; r += 3u) {
      if (!stepP(r, wb0, wb2, EX, AX, EZ, RZ, EY, AY, RY)) break;
      if (r + 1u >= R || !stepP(r + 1u, wb1, wb0, EY, AY, EX, RX, EZ, AZ, RZ)) break;
      if (r + 2u >= R || !stepP(r + 2u, wb2, wb1, EZ, AZ, EY, RY, EX, AX, RX)) break;
    }
    // rounds done - 2 (reserved, not stored) and done - 1 (neither)
    const uint32_t tb = p.t0 + b * 32u;
    if (done >= 2u) {
      const uint32_t q = done - 2u, rk = p.round_rel + q;
      if (q % 3u == 0u) emitted += emit_store_med<K>(p, shard, lane, node, tb, EX, AX, 0u, RX, rk);
      else if (q % 3u == 1u) emitted += emit_store_med<K>(p, shard, lane, node, tb, EY, AY, 0u, RY, rk);
      else emitted += emit_store_med<K>(p, shard, lane, node, tb, EZ, AZ, 0u, RZ, rk);
    }
    if (done >= 1u) {
      const uint32_t q = done - 1u, rk = p.round_rel + q;
      if (q % 3u == 0u) {
        RX = emit_reserve_med<K>(p, shard, lane, EX, 0u, upd);
        emitted += emit_store_med<K>(p, shard, lane, node, tb, EX, AX, 0u, RX, rk);
      } else if (q % 3u == 1u) {
        RY = emit_reserve_med<K>(p, shard, lane, EY, 0u, upd);
        emitted += emit_store_med<K>(p, shard, lane, node, tb, EY, AY, 0u, RY, rk);
      } else {
        RZ = emit_reserve_med<K>(p, shard, lane, EZ, 0u, upd);
        emitted += emit_store_med<K>(p, shard, lane, node, tb, EZ, AZ, 0u, RZ, rk);
      }
    }
  } else {
#endif
#if AVK_REPLAY_BUF3
  // three replayed-vote buffers and three pending sets, the loop unrolled three times: round r reads
  // buffer r % 3 and refills buffer (r + 2) % 3 (read in round r - 1: its registers are dead, so the
  // loads need no copy into the loop header's registers, which waited for them); it reserves into set
  // r % 3 and stores set (r - depth) % 3
  u32x4 wb2[RQ];
  EmitRes pendC{};
  uint32_t EpC[K], ApC = 0u;
  constexpr bool D2 = AVK_REPLAY_EMIT_DEPTH == 2;
  for (uint32_t r = 0; r < R; r += 3u) {
    if (!(D2 ? step(r, wb0, wb2, pendA, EpA, ApA, pendB, EpB, ApB) : step(r, wb0, wb2, pendA, EpA, ApA, pendC, EpC, ApC))) break;
    if (r + 1u >= R ||
        !(D2 ? step(r + 1u, wb1, wb0, pendB, EpB, ApB, pendC, EpC, ApC) : step(r + 1u, wb1, wb0, pendB, EpB, ApB, pendA, EpA, ApA)))
      break;
    if (r + 2u >= R ||
        !(D2 ? step(r + 2u, wb2, wb1, pendC, EpC, ApC, pendA, EpA, ApA) : step(r + 2u, wb2, wb1, pendC, EpC, ApC, pendB, EpB, ApB)))
      break;
  }
  if constexpr (K == 8) {  // the last rounds run's entries (rounds done - depth .. done - 1)
    for (uint32_t q = done >= (uint32_t)AVK_REPLAY_EMIT_DEPTH ? done - (uint32_t)AVK_REPLAY_EMIT_DEPTH : 0u; q < done; ++q) {
      const uint32_t sset = q % 3u;
      const uint32_t rk = p.round_rel + q;
      if (sset == 0u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpA, ApA, 0u, pendA, rk);
      else if (sset == 1u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpB, ApB, 0u, pendB, rk);
      else emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpC, ApC, 0u, pendC, rk);
    }
  }
#elif AVK_REPLAY_EMIT_DEPTH == 2
  // four pending sets: round r reserves into set r % 4 and stores set (r - 2) % 4; the replayed-vote
  // buffers keep alternating (r % 2)
  EmitRes pendC{}, pendD{};
  uint32_t EpC[K], EpD[K], ApC = 0u, ApD = 0u;
  for (uint32_t r = 0; r < R; r += 4u) {
    if (!step(r, wb0, wb0, pendA, EpA, ApA, pendC, EpC, ApC)) break;
    if (r + 1u >= R || !step(r + 1u, wb1, wb1, pendB, EpB, ApB, pendD, EpD, ApD)) break;
    if (r + 2u >= R || !step(r + 2u, wb0, wb0, pendC, EpC, ApC, pendA, EpA, ApA)) break;
    if (r + 3u >= R || !step(r + 3u, wb1, wb1, pendD, EpD, ApD, pendB, EpB, ApB)) break;
  }
  if constexpr (K == 8) {  // the last two rounds run's entries (rounds done - 2, done - 1)
    for (uint32_t q = done >= 2u ? done - 2u : 0u; q < done; ++q) {
      const uint32_t sset = q & 3u;
      const uint32_t rk = p.round_rel + q;
      if (sset == 0u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpA, ApA, 0u, pendA, rk);
      else if (sset == 1u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpB, ApB, 0u, pendB, rk);
      else if (sset == 2u) emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpC, ApC, 0u, pendC, rk);
      else emitted += emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpD, ApD, 0u, pendD, rk);
    }
  }
#else
  for (uint32_t r = 0; r < R; r += 2u) {
    if (!step(r, wb0, wb0, pendA, EpA, ApA, pendB, EpB, ApB)) break;
    if (r + 1u >= R || !step(r + 1u, wb1, wb1, pendB, EpB, ApB, pendA, EpA, ApA)) break;
  }
  if constexpr (K == 8) {  // the last round run's entries (round done - 1)
    if (done > 0u) {
      const bool odd = ((done - 1u) & 1u) != 0u;
      emitted += odd ? emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpB, ApB, 0u, pendB, p.round_rel + done - 1u)
                     : emit_store_med<K>(p, shard, lane, node, p.t0 + b * 32u, EpA, ApA, 0u, pendA, p.round_rel + done - 1u);
    }
  }
#endif
#if AVK_REPLAY_PIPE3
  }
#endif
  if (done < R && b == 0) p.node_flags[nl] = done + 1u;  // the exact pass takes rounds done..R-1
  if (done > 0u) {
    pst4<NT>(grp, u32x4{V[0], V[1], V[2], V[3]});
    pst4<NT>(grp + 64, u32x4{V[4], V[5], V[6], V[7]});
#pragma unroll
    for (int i = 0; i < 8; ++i) pst<NT>(tp + 1024u + (uint32_t)i * 64u + tl, C[i]);
    pst4<NT>(grp + 128, u32x4{Kp[0], Kp[1], Kp[2], Kp[3]});
    pst4<NT>(grp + 192, u32x4{Kp[4], Kp[5], Kp[6], Kp[7]});
    pst<NT>(tp + 1536u + tl, A);
  }
  // the other lanes' published words (see above); lanes past 3 * 128 (BL > 384) one by one
  uint32_t pub_bytes = 0u;
  {
    const uint32_t r0 = R > 3u ? R - 3u : 0u;
    for (uint32_t lb = b + kMaxPoll / 32u, q = 0; lb < p.BL; lb += kMaxPoll / 32u, ++q) {
      uint32_t Ao = q == 0u ? Aother[0] : Aother[1];
      if (q >= kOther) {
        const uint32_t go = nl * p.BL + lb;
        Ao = pld<NT>(p.planes + (size_t)(go >> 6) * (kPlanes * 64u) + 1536u + (go & 63u));
      }
      for (uint32_t r = r0; r < R; ++r)
        p.pref_ring[(p.ring_next + r) % 3u][node * p.PS + lb] = byz ? byz_pattern(p.round + r + 1u) : Ao;
      pub_bytes += 4u + 4u * (R - r0);
    }
  }
  // bytes: 25 planes read once and written once (if a round ran), 8 B per replayed vote word pair
  // per round, the published words
  const uint32_t lane_bytes = kPlanes * 4u + 8u * K * done + 4u * pubs + (done > 0u ? kPlanes * 4u : 0u);
  count_stats(p, wave_id, lane, applied, true, lane_bytes, emitted + wave_sum(pub_bytes), upd, 0u);
}

template <int K, int MAXT>
hipError_t launch_replay_t(const RoundParams& p, uint32_t bt, hipStream_t s) {
  if (p.plane_nt)
    hipLaunchKernelGGL((k_replay_node<K, true, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
  else
    hipLaunchKernelGGL((k_replay_node<K, false, MAXT>), dim3(p.NL), dim3(bt), 0, s, p);
  return hipGetLastError();
}

template <int K>
hipError_t launch_replay_k(const RoundParams& p, hipStream_t s) {
  if (p.replay_fast) {  // nodes with 4096 live valid records in their first 128 lanes first
    if (p.plane_nt)
      hipLaunchKernelGGL((k_replay_fast<K, true>), dim3(p.NL), dim3(128), 0, s, p);
    else
      hipLaunchKernelGGL((k_replay_fast<K, false>), dim3(p.NL), dim3(128), 0, s, p);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  const uint32_t bt = ((p.BL + 63u) / 64u) * 64u;
  return bt <= 512u ? launch_replay_t<K, 512>(p, bt, s) : launch_replay_t<K, 1024>(p, bt, s);
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

hipError_t launch_replay_node(const RoundParams& p, int k, hipStream_t s) {
  if (!p.node_flags || p.fuse_rounds == 0u || !p.replay) return hipErrorInvalidValue;
  switch (k) {
    case 1: return launch_replay_k<1>(p, s);
    case 2: return launch_replay_k<2>(p, s);
    case 3: return launch_replay_k<3>(p, s);
    case 4: return launch_replay_k<4>(p, s);
    case 5: return launch_replay_k<5>(p, s);
    case 6: return launch_replay_k<6>(p, s);
    case 7: return launch_replay_k<7>(p, s);
    case 8: return launch_replay_k<8>(p, s);
    default: return hipErrorInvalidValue;
  }
}

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
