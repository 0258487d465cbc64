// Device pieces shared by the streaming round kernels (round_sweep.hip: the
// uncapped sweep; round_node.hip: one workgroup per node under the 4096 poll
// cap): BL division, the peer draw, the per-slot thresholds of vote.go:58,61
// and the deferred confidence update, plane-stream cache policies.
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.h"
#include "round_common.h"

namespace avk {
namespace {

__device__ __forceinline__ uint32_t div_bl(const RoundParams& p, uint32_t n) {
  const uint32_t t = __umulhi(n, p.bl_magic);
  return (t + ((n - t) >> p.bl_sh1)) >> p.bl_sh2;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

// Thresholds of vote.go:58,61 at slot j. The 8-vote window after slot j is
// seq[j .. j+7] of the sequence seq = [V_6 .. V_0, w_0 .. w_{K-1}] (old
// shift-register planes, oldest first, then this round's votes). y = votes &
// consider, n = ^votes & consider (vote.go:58, :61); "popcount > 6" of 8
// planes = "at most one zero". Over a set of planes, Agg2 keeps z0 = "no
// zero" and z1 = "at most one zero" (2 VALU ops per plane pushed, one
// v_and_or + one and). Window j = new votes w_0..w_j (a prefix carried from
// slot to slot, one push per slot) + old planes V_0..V_{6-j} (recomputed per
// slot: 6-j pushes), combined in 2 ops: 144 VALU ops for all 8 slots of both
// sides instead of 8 x 2 x 14 for the plain per-window network, and only 4
// registers of carried state.
struct Agg2 {
  uint32_t z0, z1;
};
__device__ __forceinline__ void agg_push(Agg2& a, uint32_t x) {
  a.z1 = a.z0 | (a.z1 & x);
  a.z0 &= x;
}
__device__ __forceinline__ uint32_t agg_le1(const Agg2& p, const Agg2& q) { return (p.z0 & q.z1) | (p.z1 & q.z0); }

// yes / no thresholds of slot J; Py / Pn carry the new-vote prefix of the two
// sides. SYM: n == ~y on the whole window (sim votes on warm planes), so the
// no side runs on the complement of ys in place (the NOT folds into bitop3).
template <int J, int K, bool SYM>
__device__ __forceinline__ void thresholds(const uint32_t (&ys)[7 + K], const uint32_t (&ns)[7 + K], Agg2& Py,
                                           Agg2& Pn, uint32_t& yes, uint32_t& no) {
  const uint32_t y = ys[7 + J], n = SYM ? ~ys[7 + J] : ns[7 + J];
  if constexpr (J == 0) {
    Py = Agg2{y, ~0u};
    Pn = Agg2{n, ~0u};
  } else {
    agg_push(Py, y);
    agg_push(Pn, n);
  }
  if constexpr (J <= 6) {
    Agg2 Sy{ys[6], ~0u}, Sn{SYM ? ~ys[6] : ns[6], ~0u};  // V_0
#pragma unroll
    for (int i = 5; i >= J; --i) {  // V_1 .. V_{6-J}
      agg_push(Sy, ys[i]);
      agg_push(Sn, SYM ? ~ys[i] : ns[i]);
    }
    yes = agg_le1(Py, Sy);
    no = agg_le1(Pn, Sn);
  } else {
    yes = Py.z1;
    no = Pn.z1;
  }
}

// The rarely taken peer draws (round-robin mode, N - 1 <= k, one block per
// node, or a repeated candidate) out of line, so their registers do not
// weigh on the hot path.
template <int K>
struct PeerList {
  uint32_t v[K];
};
template <int K>
__device__ __forceinline__ PeerList<K> sample_peers_general(uint64_t seed, uint32_t node, uint32_t round,
                                                         uint32_t n_nodes, int mode) {
  PeerList<K> r;
  sample_peers<K>(seed, node, round, n_nodes, mode, r.v);
  return r;
}

// Per-slot step of the round. The count update is deferred: c (4 planes)
// counts the agreeing conclusive votes since the last flip (vote.go:66-69),
// F marks records that flipped (vote.go:72-74; count reset to 0), and at the
// end count_new = F ? c : count + c. det (some polled record of the wave has
// count >= 120, wave-uniform): also detect the vote that takes a record from 127 to 128 —
// an agreement with no flip before it in the round and low3 + c == 8, where
// low3 = count & 7 (count >= 120 means bits 3..6 are set) — which finalizes
// and deletes it (vote.go:68, processor.go:114-116); later slots skip it.
template <int K, bool SYM, int J = 0>
__device__ __forceinline__ void round_slots(const uint32_t (&ys)[7 + K], const uint32_t (&ns)[7 + K],
                                            const uint32_t (&low3)[3], uint32_t nearfin, bool det, uint32_t& alive,
                                            uint32_t& A, uint32_t (&E)[K], uint32_t (&c)[4], uint32_t& F,
                                            uint32_t& applied, Agg2 Py = Agg2{}, Agg2 Pn = Agg2{}) {
  if constexpr (J < K) {
    uint32_t yes, no;
    thresholds<J, K, SYM>(ys, ns, Py, Pn, yes, no);
    applied += (uint32_t)__popc(alive);
    const uint32_t concl = (yes | no) & alive;  // conclusive (vote.go:61-63)
    const uint32_t flip = concl & (A ^ yes);    // disagrees: reset to yes?1:0 (vote.go:72-74)
    const uint32_t agree = concl ^ flip;        // agrees: confidence += 2 (vote.go:66-69)
    uint32_t carry = agree;
    A ^= flip;
    constexpr int planes = J < 1 ? 1 : J < 3 ? 2 : J < 7 ? 3 : 4;  // c <= J + 1
#pragma unroll
    for (int i = 0; i < planes; ++i) {
      const uint32_t ci = J == 0 ? 0u : c[i] & ~flip;
      c[i] = ci ^ carry;
      carry &= ci;
    }
    uint32_t e = flip;
    if (det) {  // wave-uniform
      // low3 + c == 8 (c <= 8, low3 <= 7): sum bits 0..2 clear, bit 3 set
      const uint32_t c3 = planes > 3 ? c[3] : 0u;
      const uint32_t c2 = planes > 2 ? c[2] : 0u;
      const uint32_t s0 = low3[0] ^ c[0], k0 = low3[0] & c[0];
      const uint32_t t1 = low3[1] ^ c[1], s1 = t1 ^ k0, k1 = bfi(t1, k0, low3[1]);
      const uint32_t t2 = low3[2] ^ c2, s2 = t2 ^ k1, k2 = bfi(t2, k1, low3[2]);
      const uint32_t s3 = c3 ^ k2;
      const uint32_t fin = agree & ~F & nearfin & ~(s0 | s1 | s2) & s3;
      e |= fin;
      alive &= ~fin;
    }
    F |= flip;
    E[J] = e;
    round_slots<K, SYM, J + 1>(ys, ns, low3, nearfin, det, alive, A, E, c, F, applied, Py, Pn);
  }
}

// Plane-stream cache policy POL: 0 = default loads/stores, 1 = non-temporal
// loads and stores, 2 = non-temporal loads + sc1 stores (write-through, the
// line leaves the XCD's L2), 3 = non-temporal loads + nt sc1 stores. 2/3 keep
// the streamed state out of L2 so that more of the gathered preference table
// stays there (MI355X_MICROARCH.md: plain/nt stores keep the line in L2, sc1
// stores drop it).
constexpr int32_t kRsrcWord3 = 0x00020000;  // raw 32-bit buffer (gfx9 family)
template <int POL>
__device__ __forceinline__ u32x4 ld4(const u32x4* q) {
  return pld4<(POL > 0)>(q);
}
template <int POL>
__device__ __forceinline__ uint32_t ld1(const uint32_t* q) {
  return pld<(POL > 0)>(q);
}
template <int POL>
__device__ __forceinline__ void st4(__amdgpu_buffer_rsrc_t r, u32x4* q, uint32_t off, u32x4 v) {
  if constexpr (POL < 2)
    pst4<(POL > 0)>(q, v);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, POL == 2 ? 16 : 18);
}
template <int POL>
__device__ __forceinline__ void st1(__amdgpu_buffer_rsrc_t r, uint32_t* q, uint32_t off, uint32_t v) {
  if constexpr (POL < 2)
    pst<(POL > 0)>(q, v);
  else
    __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, POL == 2 ? 16 : 18);
}

// The k peers of this lane's node for this round (R1: Philox4x32-10 keyed by
// (node, round), the first k distinct candidates; oracle avo_sample_peers).
// The wave's lanes cover nn consecutive nodes starting at local node nlA;
// lane q draws Philox block q % NB of node nlA + q / NB and every lane takes
// its node's candidates with ds_bpermute. The rare cases (round-robin peers,
// N - 1 <= k, more than 64 / NB nodes in the wave, a repeated candidate) take
// the general draw.
template <int K>
__device__ __forceinline__ void draw_peers(const RoundParams& p, uint32_t round, uint32_t node, uint32_t nl,
                                           uint32_t nlA, uint32_t nn, uint32_t lane, uint32_t (&peers)[K]) {
  const uint32_t others = p.n_nodes - 1u;
  constexpr uint32_t NB = (K + 3) / 4;
  bool general = p.peer_mode == 1 || (uint32_t)K >= others || nn * NB > 64u;
  if (!general) {
    // producer lane q draws Philox block q % NB of the tile's node q / NB ...
    uint32_t q = lane;
    asm volatile("" : "+v"(q));  // opaque: keep the lane-derived counters inside the tile loop
    const uint32_t pnode = p.n0 + nlA + min(q / NB, nn - 1u);
    uint32_t x[4];
    philox(x, p.seed, pnode, round, q % NB, kDomPeers);
    uint32_t prod[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = __umulhi(x[i], others);
      prod[i] = u + (u >= pnode ? 1u : 0u);
    }
    // ... and every lane of that node takes its candidates with ds_bpermute
    const uint32_t base = (nl - nlA) * NB;
    if constexpr (K == 8) {
      // distinctness on the two producer lanes (own 4 + partner's 4), one ballot
      bool ok = true;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t part = (uint32_t)__shfl((int)prod[i], (int)(q ^ 1u), 64);
#pragma unroll
        for (int j = 0; j < 4; ++j) ok &= prod[j] != part;
#pragma unroll
        for (int j = 0; j < i; ++j) ok &= prod[i] != prod[j];
      }
      const unsigned long long bad = __ballot(!ok);
#pragma unroll
      for (int c = 0; c < K; ++c) peers[c] = (uint32_t)__shfl((int)prod[c & 3], (int)(base + (uint32_t)c / 4u), 64);
      general = ((bad >> base) & 3ull) != 0ull;
    } else {
      bool distinct = true;
#pragma unroll
      for (int c = 0; c < K; ++c) {
        peers[c] = (uint32_t)__shfl((int)prod[c & 3], (int)(base + (uint32_t)c / 4u), 64);
#pragma unroll
        for (int d = 0; d < c; ++d) distinct &= peers[c] != peers[d];
      }
      general = !distinct;
    }
  }
  if (general) {
    const PeerList<K> r = sample_peers_general<K>(p.seed, node, round, p.n_nodes, p.peer_mode);
#pragma unroll
    for (int j = 0; j < K; ++j) peers[j] = r.v[j];
  }
}

// Both draws a stale vv tile needs (kernels.h vv, k = 8): round - 1's peers
// (to regather the vote register) and this round's, from ONE Philox pass over
// the wave: lanes 0-31 produce round - 1's blocks, lanes 32-63 this round's (a
// tile needs nn * 2 <= 32 producer lanes per draw). The distinctness of a
// node's 8 candidates is decided on its two producer lanes (own 4 + partner's
// 4: 6 + 16 compares) and handed out by ballot, instead of 28 compares per
// draw on every lane. pick_peers then hands one draw to the node's lanes.
// Same peers as draw_peers.
struct PairDraw {
  uint32_t prod[4];
  unsigned long long bad;  // bit l: producer lane l saw a repeated candidate
  bool fallback;           // wave-uniform: per-draw draw_peers instead
};

__device__ __forceinline__ PairDraw pair_draw(const RoundParams& p, uint32_t round, uint32_t nlA, uint32_t nn,
                                              uint32_t lane) {
  PairDraw d;
  const uint32_t others = p.n_nodes - 1u;
  d.fallback = p.peer_mode == 1 || 8u >= others || nn * 2u > 32u;
  d.bad = 0ull;
  if (d.fallback) return d;
  // opaque copy of the lane index: keeps the compiler from hoisting the
  // lane-derived Philox counters out of the tile loop and spilling them
  uint32_t ln = lane;
  asm volatile("" : "+v"(ln));
  const uint32_t half = ln >> 5, q = ln & 31u;
  const uint32_t pnode = p.n0 + nlA + min(q >> 1, nn - 1u);
  uint32_t x[4];
  philox(x, p.seed, pnode, round - 1u + half, q & 1u, kDomPeers);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u = __umulhi(x[i], others);
    d.prod[i] = u + (u >= pnode ? 1u : 0u);
  }
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t part = (uint32_t)__shfl((int)d.prod[i], (int)(lane ^ 1u), 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) ok &= d.prod[j] != part;
#pragma unroll
    for (int j = 0; j < i; ++j) ok &= d.prod[i] != d.prod[j];
  }
  d.bad = __ballot(!ok);
  return d;
}

// One draw of `round` for the nn nodes starting at local node nlA (nn * 2
// <= 64 producer lanes at k = 8): producer lane q holds Philox block q % 2 of
// node nlA + q / 2; distinctness of a node's 8 candidates is decided on its
// two producer lanes. The layout of pair_draw's second half, for all 64 lanes.
__device__ __forceinline__ PairDraw single_draw(const RoundParams& p, uint32_t round, uint32_t nlA, uint32_t nn,
                                                uint32_t lane) {
  PairDraw d;
  const uint32_t others = p.n_nodes - 1u;
  d.fallback = p.peer_mode == 1 || 8u >= others || nn * 2u > 64u;
  d.bad = 0ull;
  if (d.fallback) return d;
  uint32_t q = lane;
  asm volatile("" : "+v"(q));  // opaque: keep the lane-derived counters where they are used
  const uint32_t pnode = p.n0 + nlA + min(q >> 1, nn - 1u);
  uint32_t x[4];
  philox(x, p.seed, pnode, round, q & 1u, kDomPeers);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t u = __umulhi(x[i], others);
    d.prod[i] = u + (u >= pnode ? 1u : 0u);
  }
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t part = (uint32_t)__shfl((int)d.prod[i], (int)(lane ^ 1u), 64);
#pragma unroll
    for (int j = 0; j < 4; ++j) ok &= d.prod[j] != part;
#pragma unroll
    for (int j = 0; j < i; ++j) ok &= d.prod[i] != d.prod[j];
  }
  d.bad = __ballot(!ok);
  return d;
}

// A draw parked in LDS as preference-row byte offsets (sd[q * 4 + i] =
// producer lane q's prod[i] * row_bytes): the node whose producers are lanes
// base, base + 1 reads its 8 candidates' rows as two 16-byte broadcasts.
// `bad` = the draw's ballot.
__device__ __forceinline__ void park_draw(const PairDraw& d, uint32_t* sd, uint32_t lane, uint32_t row_bytes) {
  *reinterpret_cast<u32x4*>(sd + lane * 4u) =
      u32x4{d.prod[0] * row_bytes, d.prod[1] * row_bytes, d.prod[2] * row_bytes, d.prod[3] * row_bytes};
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// rows[j] = byte offset of peer j's preference row (peer * row_bytes)
__device__ __forceinline__ void pick_parked(const RoundParams& p, const uint32_t* sd, unsigned long long bad,
                                            uint32_t base, uint32_t node, uint32_t round, uint32_t row_bytes,
                                            uint32_t (&rows)[8]) {
  const u32x4 lo = *reinterpret_cast<const u32x4*>(sd + base * 4u);
  const u32x4 hi = *reinterpret_cast<const u32x4*>(sd + base * 4u + 4u);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    rows[c] = lo[c];
    rows[c + 4] = hi[c];
  }
  if ((bad >> base) & 3ull) {
    const PeerList<8> g = sample_peers_general<8>(p.seed, node, round, p.n_nodes, p.peer_mode);
#pragma unroll
    for (int j = 0; j < 8; ++j) rows[j] = g.v[j] * row_bytes;
  }
}

// which = 0: round - 1's peers, 1: round's (pair_draw's round)
__device__ __forceinline__ void pick_peers(const RoundParams& p, const PairDraw& d, uint32_t which, uint32_t round,
                                           uint32_t node, uint32_t nl, uint32_t nlA, uint32_t nn, uint32_t lane,
                                           uint32_t (&peers)[8]) {
  const uint32_t r = round - 1u + which;
  if (d.fallback) {
    draw_peers<8>(p, r, node, nl, nlA, nn, lane, peers);
    return;
  }
  const uint32_t base = which * 32u + (nl - nlA) * 2u;
#pragma unroll
  for (int c = 0; c < 8; ++c) peers[c] = (uint32_t)__shfl((int)d.prod[c & 3], (int)(base + (uint32_t)c / 4u), 64);
  if ((d.bad >> base) & 3ull) {
    const PeerList<8> g = sample_peers_general<8>(p.seed, node, r, p.n_nodes, p.peer_mode);
#pragma unroll
    for (int j = 0; j < 8; ++j) peers[j] = g.v[j];
  }
}

}  // namespace
}  // namespace avk
