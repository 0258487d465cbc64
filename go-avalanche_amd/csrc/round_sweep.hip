// Persistent streaming round kernel (uncapped path, k <= 8): the hot path of
// the engine. One round of go-avalanche's poll loop for every simulated node
// (processor.go:92-117 driven by main.go:110-136, rules R1-R4 of SURVEY.md
// §8): peer draw (processor.go:173-182 replaced by a Philox k-peer draw),
// gather of each peer's published IsAccepted word (main.go:168-192 responder),
// k regsiterVote steps (vote.go:54-75) on 32 bit-sliced VoteRecords per lane,
// StatusUpdate emission (processor.go:111) and deletion on finalization
// (:114-116).
//
// Same HBM layout, outputs and counters as k_round_fast (kernels.hip); what
// differs is how the work maps onto CDNA4:
//  * the Philox peer draw runs once per (node, Philox block) across the
//    wave's lanes and is handed to the node's lanes with ds_bpermute, instead
//    of every lane of a node redrawing the same peers (round_slots.h);
//  * per slot, the ">6 of 8" thresholds of vote.go:58,61 are "at most one
//    zero" over the 8-vote window of [old planes | new votes]: a prefix of the
//    new votes carried from slot to slot plus the shrinking old part,
//    combined in 2 ops (round_slots.h); on warm planes with sim votes the no
//    side runs on the complement of the same registers;
//  * the confidence update is deferred: a 4-plane counter of agreements since
//    the last flip, added once at the end (count = flipped ? c : count + c);
//    a wave holding a record with count >= 120 also detects, per slot, the
//    vote that takes a record from 127 to 128 (finalization and deletion);
//  * once every consider plane is known to be all-ones (sim votes only, the
//    engine tracks it), the consider planes are neither read nor written and
//    the per-tile warmth probe disappears;
//  * 72 VGPRs at k = 8 (7 waves per SIMD); one wave per tile, or a resident
//    grid walking the tiles when tiles are few (the per-wave counters are
//    then flushed once per wave, and each wave issues its next tile's loads
//    before computing the current one).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"
#include "round_common.h"
#include "round_slots.h"

// A/B build knob: the StatusUpdate log reservation issued before the tile's stores (1) or after
// them, inside the emission (0)
#ifndef AVK_EMIT_HOIST
#define AVK_EMIT_HOIST 1
#endif
// A/B build knob: compile the per-phase ablation diagnostics (option "ablate_phase") into the warm
// path (1: the Makefile's "ablate" variant library only; the product kernel is built without them)
#ifndef AVK_ABLATE_PHASE
#define AVK_ABLATE_PHASE 0
#endif
// A/B build knob: in rounds that count changed words (peer pushes), the overwritten published words
// are loaded ahead of time with the tile (1) or by each publish (0)
// (0: the prefetched words' registers spilled in the counting build: C4 epoch 7.40 ms against 5.95,
// C4p 24.0 against 15.4 with count_changed on, profiles/r04/ab_count_changed.log)
#ifndef AVK_CC_PREFETCH
#define AVK_CC_PREFETCH 0
#endif
// A/B build knob: the storm path's publish loads (overwritten word, stale and need bytes) issued
// before the tile's plane stores (1) or by publish itself, after them (0, default: measured 3 % faster
// on masked C4p node shards at 8 ranks, profiles/r06/ab_pub_preload.log)
#ifndef AVK_PUB_PRELOAD
#define AVK_PUB_PRELOAD 0
#endif

namespace avk {
namespace {

constexpr bool kAblatePhase = AVK_ABLATE_PHASE != 0;

struct SweepAcc {
  uint32_t applied = 0, died = 0, lane_bytes = 0;
  uint32_t reread = 0;  // per lane: gathered preference bytes beyond the one compulsory read of each word
  uint32_t emitted_bytes = 0, updates = 0;  // wave-uniform: StatusUpdate log bytes written, updates emitted
  uint32_t umis = 0;  // per lane: some published word differed from ref_node's word of pref_in (p.uni_out)
  // wave-uniform (p.count_changed): published words that differ from the word they overwrite, and the
  // 16-lane groups holding one (64-B row segments when PS == BL, a multiple of 16); two scalars, so
  // that a wave walking many tiles (a small grid) cannot carry one count into the other
  uint32_t changed = 0, changed_segs = 0;
  uint32_t pushed = 0;  // wave-uniform: words stored into peer replicas (all peers)
  // deferred pushes (p.push_q): the wave's queue in LDS, slot = the tile's place in the wave's tiles
  uint32_t* qpub = nullptr;
  uint8_t* qpm = nullptr;
  uint32_t qslot = 0;
  uint32_t shard = 0;  // wave-uniform: this wave's log / counter shard (wave index % log_shards)
};

// Peer r's replica pointer from the engine's device table: a scalar load through the constant address
// space (the table is written once at av_peer_init), so a pushing lane issues no vector load and its
// wave no vmcnt drain.
__device__ __forceinline__ uint32_t* peer_ptr(uint32_t* const* tbl, uint32_t r) {
  using cptr = __attribute__((address_space(4))) const uint64_t*;
  const cptr t = (cptr)(tbl);
  return reinterpret_cast<uint32_t*>(t[__builtin_amdgcn_readfirstlane((int)r)]);
}

// One word into a peer's replica (p.push_store): 1 = a plain store (default: the round kernel's
// completion releases it at system scope before the barrier kernel that follows it on the stream runs,
// which orders it for the peer; measured far cheaper to issue than the scoped form), 0 = a system-scope
// store (the first form), 2 = none (diagnostics: the exchange's stores ablated, results invalid).
__device__ __forceinline__ void push_word(const RoundParams& p, uint32_t* dst, uint32_t v) {
  if (p.push_store == 1u)
    *dst = v;
  else if (p.push_store == 0u)
    __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The published word of one lane into pref_out. In a peer-push round the word being overwritten is
// what every peer replica holds (kernels.h), so only a changed word is stored into each replica
// (system-scope write-through stores over xGMI; the barrier after the round orders them before any
// peer reads them). Changed words are counted when p.count_changed (the push volume),
// per wave by ballot (a scalar: a per-lane counter live across the tile loop spilled).
// `old`: the overwritten word when the caller knows it (`known`: loaded ahead of time, or implied by
// the tile's history, below); else it is loaded here (its latency then sits on the tile's chain).
// A tile whose count steps were deferred in the two rounds before this one (kpend >= 2) kept its
// accepted plane through them, so an honest row it publishes unchanged this round equals the
// snapshot being overwritten (written three rounds ago): no load, no push; a Byzantine row's word
// there is the pattern of that snapshot.
// Need-masked exchange (p.stale, kernels.h): peer i gets this lane's word if one of its nodes draws
// the row next round (need bit i) and either the word changed or peer i's copy of the segment may
// differ (stale bit i: a change it did not need was withheld earlier); a withheld change marks the
// segment stale for that peer, a push to it clears the mark. The segment's bits are decided per wave
// (any changed word of the wave: a superset, so a mark is never lost; a segment never straddles a
// wave), so every lane of a segment stores the same byte.
// Deferred pushes (p.push_q): the peers a lane's word goes to (bit i: peer i) and the word are queued
// in LDS and stored after the wave's last tile (flush_pushes), so that no load of a later tile waits
// for them (vmcnt counts loads and stores in issue order, and a system-scope store to a peer completes
// only at the peer: pushed from inside the tile loop, every tile waited for the last one's pushes).
// The loads publish() needs (the overwritten word, the segment's stale byte, the node's need byte),
// issued by the caller before the tile's plane stores: vmcnt counts loads and stores in issue order,
// so loads issued after the stores would make the tile wait for the stores' completion too (a round
// trip per tile in every peer-push round; the stale and need bytes exist on need-masked engines only).
struct PubPre {
  uint32_t old, st, nm;
  bool have;
};
__device__ __forceinline__ PubPre publish_loads(const RoundParams& p, uint32_t prow, uint32_t nl) {
  PubPre q{0u, 0u, p.peer_all, true};
  q.old = p.pref_out[prow];
  if (p.stale) {
    q.st = p.stale[nl * p.segs + ((prow - (p.n0 + nl) * p.PS) >> 5)];
    if (p.need) q.nm = (uint32_t)p.need[nl];
  }
  return q;
}

template <int POL, bool CC>
__device__ __forceinline__ void publish(const RoundParams& p, uint32_t prow, uint32_t pub, uint32_t old,
                                        SweepAcc& acc, bool known, uint32_t nl, uint32_t slot,
                                        const PubPre* pre = nullptr) {
  if (CC && p.count_changed) {
    const bool pl = pre && pre->have;  // loaded ahead (an unknown word only)
    if (!known && !AVK_CC_PREFETCH) old = pl ? pre->old : p.pref_out[prow];
    uint32_t nm = p.peer_all, st = 0u, si = 0u;
    if (p.stale) {
      si = nl * p.segs + ((prow - (p.n0 + nl) * p.PS) >> 5);
      st = pl ? pre->st : p.stale[si];
      // a word known unchanged (a settled tile) goes out only where a change was withheld: the need
      // mask is read only then (settled rounds after the catch-up read one byte per lane, not two)
      if (p.need && (!known || __ballot(st != 0u) != 0ull)) nm = pl ? pre->nm : (uint32_t)p.need[nl];
    }
    const unsigned long long m = __ballot(pub != old);
    const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
    const uint32_t groups = ((lo & 0xFFFFu) ? 1u : 0u) + ((lo >> 16) ? 1u : 0u) + ((hi & 0xFFFFu) ? 1u : 0u) + ((hi >> 16) ? 1u : 0u);
    acc.changed += (uint32_t)__popcll(m);
    acc.changed_segs += groups;
    if (p.push_q) {
      const uint32_t push = p.stale ? nm & (pub != old ? p.peer_all : st) : (pub != old ? p.peer_all : 0u);
      const uint32_t lane = __lane_id();
      acc.qpm[slot * 64u + lane] = (uint8_t)push;
      if (push) acc.qpub[slot * 64u + lane] = pub;  // (read only where pm != 0; counted by flush_pushes)
      if (p.stale) {
        const uint32_t nst = (st | (m ? p.peer_all : 0u)) & ~nm;
        if (nst != st) p.stale[si] = (uint8_t)nst;
      }
    } else if (p.stale) {
      const uint32_t push = nm & (pub != old ? p.peer_all : st);
      for (uint32_t r = 0; r < p.push_n; ++r) {
        const bool go = (push >> r) & 1u;
        if (go) push_word(p, peer_ptr(p.push_dst, r) + prow, pub);
        acc.pushed += (uint32_t)__popcll(__ballot(go));
      }
      const uint32_t nst = (st | (m ? p.peer_all : 0u)) & ~nm;
      if (nst != st) p.stale[si] = (uint8_t)nst;
    } else {
      if (pub != old)
        for (uint32_t r = 0; r < p.push_n; ++r)
          push_word(p, peer_ptr(p.push_dst, r) + prow, pub);
      acc.pushed += (uint32_t)__popcll(m) * p.push_n;
    }
  }
  const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(p.pref_out, 0, (int)0xFFFFFFFFu, kRsrcWord3);
  st1<POL>(pr, p.pref_out + prow, prow * 4u, pub);
}

// The queued pushes of a wave's tiles (p.push_q): tile first + s * step for queue slot s < n. The peer
// pointers are read once; the stores are the wave's last memory instructions, back to back.
__device__ __forceinline__ uint32_t flush_pushes(const RoundParams& p, uint32_t lane, uint32_t first, uint32_t step,
                                                 uint32_t n, const uint32_t* qpub, const uint8_t* qpm) {
  uint32_t* dst[8];
#pragma unroll
  for (uint32_t r = 0; r < 8u; ++r) dst[r] = r < p.push_n ? peer_ptr(p.push_dst, r) : nullptr;
  uint32_t words = 0u;  // this lane's pushed words (returned: the caller sums the wave once)
  for (uint32_t s = 0; s < n; ++s) {
    const uint32_t g = (first + s * step) * 64u + lane;
    const uint32_t pm = g < p.L ? (uint32_t)qpm[s * 64u + lane] : 0u;
    words += (uint32_t)__popc(pm);
    if (pm == 0u) continue;
    const uint32_t pub = qpub[s * 64u + lane];
    const uint32_t nl = div_bl(p, g);
    const uint32_t prow = (p.n0 + nl) * p.PS + (g - nl * p.BL);
#pragma unroll
    for (uint32_t r = 0; r < 8u; ++r)
      if ((pm >> r) & 1u) push_word(p, dst[r] + prow, pub);
  }
  return words;
}

enum : int { kModeWarm = 0, kModeCheck = 1, kModeReplay = 2, kModeAblate = 3, kModeWarmPipe = 4, kModeFresh = 5 };

// Everything one 64-lane tile loads before its round step: the state planes
// (vote.go:25-29; V0-7 and K0-7 as dwordx4 groups, A, C0-7 unless warm), the
// validity word, the node's Byzantine word, and the k vote words (replayed
// planes, or the peers' published preference words). Split from the step so
// that a wave can issue tile t + stride's loads before it computes tile t.
template <int K, bool REPLAY, bool WARM>
struct TileIn {
  u32x4 v0, v1, k0, k1;
  uint32_t A, vmask, byzw;
  uint32_t stale;                // wave-uniform: V planes stale, v0/v1 regathered (kernels.h vstale & kVMask)
  uint32_t cflag;                // wave-uniform: vstale & kCAll (consider planes virtual, all-ones)
  uint32_t kw;                   // wave-uniform: kpend[tile] (kernels.h klazy); K planes not loaded if all-live
  uint32_t C[WARM ? 1 : 8];
  uint32_t uref;                 // uniform rows (p.uni_out): ref_node's word of pref_in for the lane's block
  uint32_t old;                  // p.count_changed: the word of pref_out this lane's published word overwrites
  uint32_t w[K];                 // yes bits: err == 0 (vote.go:55)
  uint32_t cw[REPLAY ? K : 1];   // consider bits: int32(err) >= 0 (vote.go:56); sim votes: all-ones
};

// The peer draws of a wave's run of consecutive tiles, made once for the
// whole run (kModeWarm with p.tpw, k = 8): `pair` = round - 1's and round's
// draws (some tile of the run is kVStale), else round's only; `ok` = the
// run's nodes fit the producer lanes (otherwise every tile draws its own).
struct WaveDraw {
  // the draws parked in LDS (round_slots.h park_draw): node rel of the run has its 8 candidates at
  // sdc + rel * 8 (this round) and sdp + rel * 8 (round - 1, if pair); badc / badp: the draws'
  // repeated-candidate ballots, bit rel * 2 (and rel * 2 + 1) for node rel
  const uint32_t* sdc;
  const uint32_t* sdp;
  unsigned long long badc, badp;
  uint32_t fofs;  // REF: bit offset of this round's producer lanes in flagok (32 in the paired layout)
  uint32_t nlA, t0, nn;
  // REF: producer lane q's 4 candidates all carry pref_in's reference-row tag (bit q): a node's 8
  // peers are flagged iff both of its producer lanes' bits are set
  unsigned long long flagok;
  uint32_t meta;  // lane i: tile t0 + i's vstale << 8 | kpend & (kPendAllLive | 0xFF)
  bool pair, ok;
};

__device__ __forceinline__ uint32_t meta_of(const WaveDraw& wd, uint32_t tile) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wd.meta, (int)(tile - wd.t0));
}

// word at a 32-bit byte offset from a wave-uniform base (SGPR base + VGPR
// offset addressing: one VALU add per gather instead of a 64-bit multiply-add)
__device__ __forceinline__ uint32_t at_byte(const uint32_t* base, uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(base) + off);
}

struct LaneIdx {
  uint32_t g, gc, nl, b, node;
  bool active;
};

__device__ __forceinline__ LaneIdx lane_idx(const RoundParams& p, uint32_t tile, uint32_t lane) {
  LaneIdx x;
  x.g = tile * 64u + lane;
  x.active = x.g < p.L;
  x.gc = x.active ? x.g : p.L - 1u;  // inactive lanes read a valid lane, never store
  x.nl = div_bl(p, x.gc);
  x.b = x.gc - x.nl * p.BL;
  x.node = p.n0 + x.nl;
  return x;
}

constexpr uint32_t kUniVotes = 1u, kUniPrev = 2u;
// uflags (p.uni_votes; the warm k = 8 sweep only), kernel-uniform:
//  * kUniVotes: the input snapshot is uniform (kernels.h uni_in): every row of pref_in is the
//    reference row of pref_prev, so each of the 8 votes a lane would gather is that row's word for
//    its block: one load of it instead of 8 gathers (a klazy round whose tiles are not yet settled
//    candidates, e.g. C5's round 4 after the network converged);
//  * kUniPrev: pref_prev is uniform too (kernels.h uni_prev): a stale tile's vote register (last
//    round's 8 votes, gathered from pref_prev) is its reference row's word: no regather (the round
//    after, e.g. C4's and C5's round 5).
template <int K, bool REPLAY, bool WARM, int POL, bool ABLATE, bool VVM = false, bool FRESH = false, bool CC = true>
__device__ __forceinline__ void load_tile(const RoundParams& p, uint32_t tile, uint32_t lane,
                                          TileIn<K, REPLAY, WARM>& in, const WaveDraw* wd = nullptr,
                                          uint32_t uflags = 0u) {
  const LaneIdx x = lane_idx(p, tile, lane);
  const uint32_t* const tp = p.planes + (size_t)tile * (kPlanes * 64u);
  const u32x4* const grp = reinterpret_cast<const u32x4*>(tp) + lane;
  constexpr bool VV = VVM && WARM && !REPLAY && K == 8;  // VVM: the warm sim modes only
  const bool meta = VV && wd && wd->t0 <= tile && tile - wd->t0 < 64u && p.tpw;
  const uint32_t raw = VV && p.vv ? (meta ? (meta_of(*wd, tile) >> 8) & 0xFFu : uni(p.vstale[tile])) : 0u;
  in.stale = raw & kVMask;
  in.cflag = raw & kCAll;
  in.kw = 0u;
  if constexpr (FRESH) {
    // NewVoteRecords (vote.go:33-35): votes, consider and count all zero; K7
    // marks the slots past the engine's last target (never added)
    const uint32_t rem = p.tn - x.b * 32u;
    const uint32_t real = rem >= 32u ? ~0u : ((1u << rem) - 1u);
    in.v0 = in.v1 = in.k0 = u32x4{0u, 0u, 0u, 0u};
    in.k1 = u32x4{0u, 0u, 0u, ~real};
#pragma unroll
    for (int i = 0; i < (WARM ? 1 : 8); ++i) in.C[i] = 0u;
  } else {
    if (!in.stale) {
      in.v0 = ld4<POL>(grp);
      in.v1 = ld4<POL>(grp + 64);
    }
    if constexpr (VV) {
      if (p.klazy || p.kconsume) in.kw = meta ? meta_of(*wd, tile) & (kPendAllLive | kHiVirt | 0xFFu) : uni(p.kpend[tile]);
    }
    if (kAblatePhase && VV && (p.ablate_phase & 2u)) {  // diagnostics: no K / A loads
      in.k0 = u32x4{lane, 0u, 0u, 0u};
      in.k1 = u32x4{0u, 0u, 0u, ~real_mask(p.tn, x.b)};
    } else if (!(in.kw & kPendAllLive) || !p.klazy) {
      in.k0 = ld4<POL>(grp + 128);
      if (in.kw & kHiVirt)  // the K4..K7 group is virtual (kernels.h kHiVirt)
        in.k1 = u32x4{0u, 0u, 0u, ~real_mask(p.tn, x.b)};
      else
        in.k1 = ld4<POL>(grp + 192);
    } else {
      in.k0 = u32x4{0u, 0u, 0u, 0u};
      in.k1 = u32x4{0u, 0u, 0u, 0u};
    }
    if constexpr (!WARM) {
#pragma unroll
      for (int i = 0; i < 8; ++i) in.C[i] = ld1<POL>(tp + 1024u + (uint32_t)i * 64u + lane);
    }
  }
  in.A = kAblatePhase && VV && (p.ablate_phase & 2u) ? (lane * 0x9E3779B9u) : ld1<POL>(tp + 1536u + lane);
  if (in.stale == kVUniform) {  // the vote register of every polled record = its accepted bit (kernels.h)
    in.v0 = u32x4{in.A, in.A, in.A, in.A};
    in.v1 = u32x4{in.A, in.A, in.A, in.A};
  }
  in.vmask = x.active ? p.valid[x.b] : 0u;
  in.byzw = p.byz[x.node >> 5];
  // loaded with the tile (an in-order vmcnt wait for it late in the step would also wait for the
  // step's plane stores)
  in.uref = p.uni_out ? p.pref_in[p.ref_node * p.PS + x.b] : 0u;
  in.old = AVK_CC_PREFETCH && CC && p.count_changed ? p.pref_out[x.node * p.PS + x.b] : 0u;  // (publish)
  if constexpr (REPLAY) {
    replay_load<K>(p.replay, x.gc, in.w, in.cw);
  } else {
    const uint32_t nlA = uni(x.nl), nn = (uint32_t)__builtin_amdgcn_readlane((int)x.nl, 63) - nlA + 1u;
    uint32_t peers[K];
    // the gathers address the preference table by 32-bit byte offsets (SGPR
    // base + VGPR offset: one add per gather): the engine runs the sweep only
    // for tables below 4 GiB (N * BL < 2^30)
    const uint32_t rb = p.PS * 4u, bo = x.b * 4u;
    uint32_t rows[K];  // byte offsets of the peers' rows
    bool drawn = false, have_rows = false;
    if constexpr (VV) {
      if (wd && wd->ok) {  // the wave's draws, made once for its run of tiles (implies off32)
        const uint32_t base = (x.nl - wd->nlA) * 2u;
        const bool nog = kAblatePhase && (p.ablate_phase & 1u);  // diagnostics: no gathers (votes from the row offsets)
        if (in.stale == kVStale && (uflags & kUniPrev)) {  // every regathered word is the reference word
          const uint32_t rp = at_byte(p.pref_prev, p.ref_node * rb + bo);
          in.v0 = u32x4{rp, rp, rp, rp};
          in.v1 = u32x4{rp, rp, rp, 0u};
        } else if (in.stale == kVStale) {
          uint32_t pp[K];
          pick_parked(p, wd->sdp, wd->badp, base, x.node, p.round - 1u, rb, pp);
#pragma unroll
          for (int i = 0; i < 4; ++i) in.v0[i] = nog ? pp[7 - i] * 0x9E3779B9u : at_byte(p.pref_prev, pp[7 - i] + bo);
#pragma unroll
          for (int i = 0; i < 3; ++i) in.v1[i] = nog ? pp[3 - i] * 0x9E3779B9u : at_byte(p.pref_prev, pp[3 - i] + bo);
          in.v1[3] = 0u;
        }
        pick_parked(p, wd->sdc, wd->badc, base, x.node, p.round, rb, rows);
        drawn = have_rows = true;
        if (nog) {
#pragma unroll
          for (int j = 0; j < K; ++j) in.w[j] = (rows[j] + bo) * 0x9E3779B9u;
          return;
        }
      } else if (in.stale == kVStale) {
        // the vote register after last round's 8 sim votes is those votes:
        // V_i = (previous round's slot 7 - i vote); V_7 is never read at k = 8
        const PairDraw pd = pair_draw(p, p.round, nlA, nn, lane);
        {
          uint32_t pp[K];
          pick_peers(p, pd, 0u, p.round, x.node, x.nl, nlA, nn, lane, pp);
#pragma unroll
          for (int i = 0; i < 4; ++i) in.v0[i] = p.pref_prev[pp[7 - i] * p.PS + x.b];
#pragma unroll
          for (int i = 0; i < 3; ++i) in.v1[i] = p.pref_prev[pp[3 - i] * p.PS + x.b];
          in.v1[3] = 0u;
        }
        pick_peers(p, pd, 1u, p.round, x.node, x.nl, nlA, nn, lane, peers);
        drawn = true;
      }
    }
    if (uflags & kUniVotes) {  // kernel-uniform: no draw of this round's peers, no gathers
      const uint32_t rw = at_byte(p.pref_prev, p.ref_node * rb + bo);
#pragma unroll
      for (int j = 0; j < K; ++j) in.w[j] = rw;
      return;
    }
    if (!drawn) draw_peers<K>(p, p.round, x.node, x.nl, nlA, nn, lane, peers);
    if (!have_rows) {
#pragma unroll
      for (int j = 0; j < K; ++j) rows[j] = (ABLATE ? x.node : peers[j]) * rb;
    }
    // ABLATE (timing diagnostics only, results invalid): the node's own row, coalesced
#pragma unroll
    for (int j = 0; j < K; ++j) in.w[j] = at_byte(p.pref_in, rows[j] + bo);
  }
}

// The round step of one loaded tile. WARM: consider planes all-ones (neither
// loaded nor stored; sim votes only). POL: plane-stream cache policy.
// Reference-row flag of the node whose lanes include this one (kernels.h
// rflag_out): every lane of the node published REF's word. BL divides 64, so
// the node's lanes are the aligned BL-lane segment of this wave that holds
// the lane; the node's block-0 lane stores the byte (and pushes it to the
// peers' replicas when it changed, as the published words). The byte is the
// snapshot's tag (ref_tag) when the row equals the reference row, else 0; a
// reader trusts only its own snapshot's tag, so flags are written by settled
// tiles only and every other byte (older snapshots' tags, 0) reads as "gather".
__device__ __forceinline__ uint8_t ref_tag(uint32_t snapshot_round) { return (uint8_t)(0x80u | (snapshot_round & 0x7Fu)); }

__device__ __forceinline__ void ref_flag_store(const RoundParams& p, uint32_t lane, bool active, uint32_t b,
                                               uint32_t node, uint32_t pub, uint32_t ref) {
  const uint64_t eq = __ballot(!active || pub == ref);
  const uint32_t s0 = lane - b;  // the node's first lane (active lanes only)
  const uint64_t seg = (p.BL >= 64u ? ~0ull : ((1ull << p.BL) - 1ull)) << (s0 & 63u);
  if (active && b == 0u) {
    const uint8_t f = (eq & seg) == seg ? ref_tag(p.round + 1u) : 0u;  // pref_out = snapshot round + 1
    if (p.push_n && p.rflag_out[node] != f) {
      for (uint32_t r = 0; r < p.push_n; ++r)
        __hip_atomic_store(reinterpret_cast<uint8_t*>(peer_ptr(p.push_dst, r)) + p.rflag_off + node, f, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    p.rflag_out[node] = f;
  }
}

template <int K, bool REPLAY, bool WARM, int POL, bool VVM = false, bool REF = false, bool CC = true>
__device__ __forceinline__ void process_tile(const RoundParams& p, uint32_t tile, uint32_t lane,
                                             const TileIn<K, REPLAY, WARM>& in, uint32_t extra_bytes, SweepAcc& acc,
                                             uint32_t uflags = 0u) {
  const LaneIdx x = lane_idx(p, tile, lane);
  const bool active = x.active;
  const uint32_t b = x.b, node = x.node;
  // the node's Byzantine bit from the word loaded with the tile (a load of it here, after the plane
  // stores, made the wave wait for those stores: vmcnt counts in issue order)
  const bool nbyz = ((in.byzw >> (node & 31u)) & 1u) != 0u;
  uint32_t* const tp = p.planes + (size_t)tile * (kPlanes * 64u);
  u32x4* const grp = reinterpret_cast<u32x4*>(tp) + lane;
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(tp, 0, kPlanes * 64 * 4, kRsrcWord3);
  const u32x4 v0 = in.v0, v1 = in.v1;
  u32x4 k0 = in.k0, k1 = in.k1;
  uint32_t A = in.A;
  uint32_t C[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) C[i] = WARM ? ~0u : in.C[WARM ? 0 : i];
  const uint32_t vmask = in.vmask;

  // ---- ys/ns hold y/n of [V_6..V_0, w_0..w_{K-1}]
  constexpr bool SYM = WARM && !REPLAY;  // n == ~y everywhere: ns is never read
  uint32_t ys[7 + K], ns[7 + K], cwv[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t cw = REPLAY ? in.cw[REPLAY ? j : 0] : ~0u;
    const uint32_t yw = in.w[j] & cw;  // err == 0 implies considered
    ys[7 + j] = yw;
    ns[7 + j] = SYM ? 0u : ~yw & cw;
    cwv[j] = cw;
  }
#pragma unroll
  for (int i = 0; i < 7; ++i) {  // old planes V_6..V_0
    const uint32_t vi = (6 - i) < 4 ? v0[6 - i] : v1[2 - i];
    ys[i] = WARM ? vi : (vi & C[6 - i]);
    ns[i] = SYM ? 0u : WARM ? ~vi : (~vi & C[6 - i]);
  }

  constexpr bool KL = VVM && WARM && !REPLAY && K == 8;  // deferred count planes possible (kernels.h klazy)
  const bool klazy = KL && p.klazy;                      // wave-uniform: no record can finalize this round
  const bool kcons = KL && p.kconsume;                   // wave-uniform: apply pending steps, defer nothing
  const bool kunread = klazy && (in.kw & kPendAllLive);  // K planes not loaded: live == valid
  const uint32_t live0 = kunread ? in.vmask : ~k1[3];    // K7 = no live record
  const uint32_t P0 = live0 & vmask;                     // polled: live and IsValid (processor.go:95-103)
  const uint32_t keep = active ? (live0 & ~vmask) : 0u;  // live but !IsValid: untouched (processor.go:101-103)

  // ---- the shift-register planes after K votes are final for every record
  // that survives the round: store them now (a record deleted this round is
  // rewritten below)
  // a warm sim wave with no live-but-invalid record leaves its V planes
  // unstored: next round (or av materialize) regathers them (kernels.h vv)
  bool virt = false;
  if constexpr (VVM && !REPLAY && K == 8) {
    virt = p.vv && __ballot(keep != 0u) == 0ull;
    if (virt && p.vv_uniform) {
      // uniform form only (narrow rows, BL < vv_min_bl): a tile leaves V unstored only if it is
      // settled this round (V = A next round, nothing to regather); the test is the settled test
      // below, made early (klazy rounds: no record is near 128)
      bool st = false;
      if constexpr (SYM) {
        if (klazy) {
          uint32_t agree = P0;
#pragma unroll
          for (int i = 0; i < 7 + K; ++i) agree &= ~(ys[i] ^ in.A);
          st = __ballot(agree != P0) == 0ull;
        }
      }
      virt = st;
    }
  }
  if (active && !virt) {
    u32x4 o0, o1;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t vi = i < 4 ? v0[i] : v1[i - 4];
      const uint32_t vs = i < K ? ys[6 + K - i] : (i - K < 4 ? v0[i - K] : v1[i - K - 4]);
      const uint32_t vn = (vs & P0) | (vi & keep);
      if (i < 4)
        o0[i] = vn;
      else
        o1[i - 4] = vn;
    }
    st4<POL>(tr, grp, lane * 16u, o0);
    st4<POL>(tr, grp + 64, 1024u + lane * 16u, o1);
  }
  // fresh round with virtual vote planes: every consider bit of the tile is 1
  // after the 8 sim votes (C_i = P0 | dead0 with keep = 0): leave them unstored
  const bool cvirt = virt && !WARM && !REPLAY && p.fresh;
  if (!WARM && active && !cvirt) {  // consider planes
    const uint32_t dead0 = ~(P0 | keep);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t cs = i < K ? cwv[K - 1 - i] : C[i - K];
      st1<POL>(tr, tp + 1024u + (uint32_t)i * 64u + lane, (1024u + (uint32_t)i * 64u + lane) * 4u,
               (cs & P0) | (C[i] & keep) | dead0);
    }
  }

  uint32_t Kp[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Kp[i] = k0[i];
    Kp[4 + i] = k1[i];
  }
  if (kcons && (in.kw & 0xFFu)) {  // pending +8 steps on the polled records: pend added to count bits 3..6
    const uint32_t pend = in.kw & 0xFFu;
    uint32_t cy = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t bi = ((pend >> i) & 1u) ? P0 : 0u;
      const uint32_t t = Kp[3 + i] ^ bi;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[3 + i] & bi);
      Kp[3 + i] = si;
    }
  }
  uint32_t E[K], alive = P0, applied = 0u, c[4] = {0u, 0u, 0u, 0u}, F = 0u;
  const uint32_t low3[3] = {Kp[0], Kp[1], Kp[2]};
  constexpr bool KLZ_ABLATE = VVM && WARM && !REPLAY && K == 8;  // the warm general tiles (ablate_phase)
  // count >= 120: may reach 128 (K <= 8); never in a klazy round (engine bound)
  const uint32_t nearfin = klazy ? 0u : P0 & Kp[6] & Kp[5] & Kp[4] & Kp[3];
  const bool det = __ballot(nearfin != 0u) != 0ull;
  const uint32_t A_in = A;
  // Settled tiles (warm sim votes, K == 8, no record near 128): when every
  // polled record's 7 old votes and 8 new votes all agree with its accepted
  // bit, every 8-vote window of the round is unanimous, so each slot is a
  // conclusive agreeing vote (vote.go:58-69: confidence += 2, no flip, no
  // StatusUpdate) and the slot network can be skipped: c = 8, F = 0.
  bool settled = false;
  if constexpr (SYM && K == 8) {
    if (!det) {
      uint32_t agree = P0;
#pragma unroll
      for (int i = 0; i < 7 + K; ++i) agree &= ~(ys[i] ^ A);
      settled = __ballot(agree != P0) == 0ull;
    }
  }
  if (settled) {
#pragma unroll
    for (int j = 0; j < K; ++j) E[j] = 0u;
    c[3] = P0;
    applied = 8u * (uint32_t)__popc(P0);
  } else if (kAblatePhase && KLZ_ABLATE && (p.ablate_phase & 16u)) {  // diagnostics: no slot network
#pragma unroll
    for (int j = 0; j < K; ++j) E[j] = 0u;
    c[3] = P0;
    applied = 8u * (uint32_t)__popc(P0);
  } else {
    round_slots<K, SYM>(ys, ns, low3, nearfin, det, alive, A, E, c, F, applied);
  }
  // deferred count planes: every polled record agreed on all 8 votes (no flip,
  // c == 8) -> K stays as stored and the tile's pending +8 steps grow by one
  bool kdefer = false;
  uint32_t pend = 0u;
  if constexpr (KL) {
    if (klazy) {
      const uint32_t c8 = c[3] & ~(c[0] | c[1] | c[2]);
      const bool lane_uniform = !active || (((F & P0) | (~c8 & P0)) == 0u);
      kdefer = __ballot(!lane_uniform) == 0ull;
      pend = in.kw & 0xFFu;
      if (!kdefer) {
        if (kunread) {  // late load: the tile leaves the deferred state
          k0 = ld4<POL>(reinterpret_cast<const u32x4*>(tp) + lane + 128);
          k1 = in.kw & kHiVirt ? u32x4{0u, 0u, 0u, ~real_mask(p.tn, b)}
                               : ld4<POL>(reinterpret_cast<const u32x4*>(tp) + lane + 192);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            Kp[i] = k0[i];
            Kp[4 + i] = k1[i];
          }
        }
        // true count = K + 8 * pend on the polled records: add pend to planes 3..6
        uint32_t cy = 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t bi = ((pend >> i) & 1u) ? P0 : 0u;
          const uint32_t t = Kp[3 + i] ^ bi;
          const uint32_t si = t ^ cy;
          cy = (t & cy) | (Kp[3 + i] & bi);
          Kp[3 + i] = si;
        }
      }
    }
  }
  // count_new = F ? c : count + c on planes 0..6 (survivors stay <= 127); deleted: count 128 (K7 set)
  const uint32_t died = P0 & ~alive;
#if AVK_EMIT_HOIST
  // StatusUpdate log reservation (k = 8) before this tile's plane and published-word stores, so that
  // reading the atomics' results waits for them alone, not for those stores (round_common.h)
  EmitRes er{};
  if constexpr (K == 8) er = emit_reserve_med<K, AVK_SINGLE_MAX>(p, acc.shard, lane, E, died, acc.updates);
#endif
  {
    uint32_t cy = 0u;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const uint32_t ci = i < 4 ? c[i] : 0u;
      const uint32_t t = Kp[i] ^ ci;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[i] & ci);
      Kp[i] = ((F & ci) | (~F & si)) & ~died;
    }
    Kp[7] |= died;
  }

  // klazy rounds: a tile whose A plane did not change does not rewrite it
  const bool astore = !klazy || __ballot(active && A != A_in) != 0ull;
  // the K4..K7 group stays virtual (kernels.h kHiVirt) while every count is < 16 and nothing was
  // deleted: set by the fresh round, kept by klazy rounds (deferred tiles leave K as it is)
  bool hv = false;
  if (K == 8 && p.hivirt && ((!WARM && p.fresh) || (klazy && (in.kw & kHiVirt))))
    hv = kdefer || __ballot(active && ((Kp[4] | Kp[5] | Kp[6] | died) != 0u)) == 0ull;
  if (active && !(kAblatePhase && KLZ_ABLATE && (p.ablate_phase & 4u))) {
    const bool known = AVK_CC_PREFETCH || (kdefer && pend >= 2u);  // (publish)
    PubPre pre{0u, 0u, 0u, false};
    if (AVK_PUB_PRELOAD && CC && p.count_changed && !known) pre = publish_loads(p, node * p.PS + b, node - p.n0);
    if (!kdefer) {
      u32x4 o2, o3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o2[i] = Kp[i];
        o3[i] = Kp[4 + i];
      }
      st4<POL>(tr, grp + 128, 2048u + lane * 16u, o2);
      if (!hv) st4<POL>(tr, grp + 192, 3072u + lane * 16u, o3);
    }
    if (astore) st1<POL>(tr, tp + 1536u + lane, (1536u + lane) * 4u, A);
    const uint32_t prow = node * p.PS + b;  // < N * PS < 2^31
    const uint32_t pub = nbyz ? byz_pattern(p.round + 1u) : A;
    if (p.uni_out) acc.umis |= pub != in.uref ? 1u : 0u;  // uniform rows (kernels.h)
    publish<POL, CC>(p, prow, pub, AVK_CC_PREFETCH ? in.old : (nbyz ? byz_pattern(p.round - 2u) : pub), acc,
                     known, node - p.n0, acc.qslot, &pre);
    // a record deleted this round keeps the vote/consider planes stored
    // above: K7 marks it dead, every reader masks by K7 (k_read_records,
    // k_add_targets resets all planes) and the next round's store zeroes them
  }
  if (REF && p.rflag_out && settled) {  // reference-row flag of the row a settled tile just published
    ref_flag_store(p, lane, active, b, node, nbyz ? byz_pattern(p.round + 1u) : A,
                   p.pref_in[p.ref_node * p.PS + (active ? b : 0u)]);
    if (active) acc.lane_bytes += 4u + (b == 0u ? 1u : 0u);
  }
  if constexpr (VVM && !REPLAY && K == 8) {
    // a settled tile's 8 new votes all equal its accepted plane on the polled
    // records: its vote register is A next round (no regather)
    const uint32_t nv = (virt ? (settled ? kVUniform : kVStale) : 0u) | in.cflag | (cvirt ? kCAll : 0u);
    if (p.vv && lane == 0 && nv != (in.stale | in.cflag)) p.vstale[tile] = nv;
  }
  if constexpr (KL) {
    if (klazy) {
      // live records == valid targets in every lane (no live-but-invalid record):
      // the next round need not read K to find the polled set
      const bool all_live = __ballot(active && live0 != vmask) == 0ull;
      const uint32_t kw = (kdefer ? pend + 1u : 0u) | (all_live ? kPendAllLive : 0u) | (hv ? kHiVirt : 0u);
      if (lane == 0 && kw != in.kw) p.kpend[tile] = kw;
      if (lane == 0) acc.lane_bytes += kw != in.kw ? 8u : 4u;  // kpend word read (+ written)
    } else if (kcons) {
      if (lane == 0 && in.kw) p.kpend[tile] = 0u;
      if (lane == 0) acc.lane_bytes += in.kw ? 8u : 4u;
    }
  }
  if constexpr (!WARM && !REPLAY && K == 8) {  // the fresh round starts the tile's virtual K4..K7 group
    if (hv && lane == 0) {
      p.kpend[tile] = kHiVirt;
      acc.lane_bytes += 4u;
    }
  }
  // k = 8: single words, medium and dense records, one contiguous entry per lane (round_common.h)
  uint32_t emitted;
  if constexpr (K == 8)
#if AVK_EMIT_HOIST
    emitted = emit_store_med<K, AVK_SINGLE_MAX>(p, acc.shard, lane, node, p.t0 + b * 32u, E, A, died, er, p.round_rel);
#else
    emitted = emit_updates_med<K>(p, acc.shard, lane, node, p.t0 + b * 32u, E, A, died, acc.updates, p.round_rel);
#endif
  else
    emitted = emit_updates<K>(p, tile, lane, node, p.t0 + b * 32u, E, A, died, acc.updates);

  // fresh (p.fresh, cold template): no plane is read but A (96 B fewer)
  constexpr uint32_t plane_bytes = WARM ? 2u * 17u * 4u : 2u * kPlanes * 4u;
  const uint32_t lane_bytes = plane_bytes + (REPLAY ? 8u : 4u) * K + 4u - (!WARM && p.fresh ? 96u : 0u);
  acc.applied += applied;
  acc.died += (uint32_t)__popc(died);
  // stale: 7 regathered words instead of the 8 V planes read; virt: V planes not written
  // push: + the 4-B read of the word being overwritten
  // kl: K planes neither read (kunread and deferred) nor written (deferred); A not rewritten
  const uint32_t kbytes = (kunread && kdefer ? 32u : 0u) + (kdefer ? 32u : 0u) +
                          // virtual K4..K7 group (kHiVirt): not read (if K was read), not written
                          (WARM && (in.kw & kHiVirt) && !(kunread && kdefer) ? 16u : 0u) + (hv && !kdefer ? 16u : 0u);
  // V read: 32 B stored, 28 B regathered (stale), 0 B uniform
  // uflags: one 4-B reference word read instead of the K gathered votes / the 7 regathered ones
  acc.lane_bytes += active ? lane_bytes + extra_bytes - (in.stale == kVStale ? 4u : in.stale == kVUniform ? 32u : 0u) -
                                 (virt ? 32u : 0u) - (cvirt ? 32u : 0u) + (p.count_changed ? 4u : 0u) -
                                 kbytes - (astore ? 0u : 4u) - ((uflags & kUniVotes) ? 4u * K - 4u : 0u) -
                                 (in.stale == kVStale && (uflags & kUniPrev) ? 24u : 0u)
                           : 0u;
  acc.emitted_bytes += emitted;
  // sim rounds gather 8 peer words per lane (each word of the round-start snapshot is gathered by
  // ~k lanes: 28 of the 32 B re-read), stale tiles 7 more from the previous snapshot (24 B re-read)
  if constexpr (!REPLAY)
    acc.reread += active ? ((uflags & kUniVotes) ? 4u : 4u * K - 4u) +
                               (in.stale == kVStale ? ((uflags & kUniPrev) ? 4u : 24u) : 0u)
                         : 0u;
}

// Settled-tile fast path (kModeWarm, k = 8, klazy round, the wave's parked
// draw): a tile whose vote register is uniform (kVUniform: V = A on every
// polled record) and whose count planes are deferred with every live record
// valid (kPendAllLive) is settled this round iff every polled record's 8
// gathered votes equal its accepted bit. process_tile would then store only
// the published words and the tile's pending count (+8 steps deferred once
// more): no flip, no StatusUpdate, no deletion, V stays uniform, A and K
// unchanged. This reads A, the validity word and the 8 votes and does exactly
// that; any other tile returns false and takes the general load + step.
template <int POL, bool REF, bool CC>
__device__ __forceinline__ bool settled_tile(const RoundParams& p, uint32_t tile, uint32_t lane, uint32_t kw,
                                             const WaveDraw& wd, SweepAcc& acc) {
  const uint32_t g = tile * 64u + lane;
  const bool active = g < p.L;
  const uint32_t gc = active ? g : p.L - 1u;
  const uint32_t nl = div_bl(p, gc);
  const uint32_t b = gc - nl * p.BL;
  // A plane: a buffer resource on the tile (SGPRs) + the lane's constant byte
  // offset, so no 64-bit per-lane address is kept live across the tile loop
  // (the flat form was hoisted into a VGPR pair that spilled and was reloaded
  // from scratch, with a full vmcnt wait, at every settled tile)
  const __amdgpu_buffer_rsrc_t ta =
      __builtin_amdgcn_make_buffer_rsrc(p.planes + (size_t)tile * (kPlanes * 64u), 0, kPlanes * 64 * 4, kRsrcWord3);
  const uint32_t A = __builtin_amdgcn_raw_buffer_load_b32(ta, (1536u + lane) * 4u, 0, POL > 0 ? 2 : 0);
  const uint32_t old = AVK_CC_PREFETCH && CC && p.count_changed ? p.pref_out[(p.n0 + nl) * p.PS + b] : 0u;  // (publish)
  const uint32_t P0 = active ? at_byte(p.valid, b * 4u) : 0u;  // polled = live (kPendAllLive) and valid
  const uint32_t uref = p.uni_out ? p.pref_in[p.ref_node * p.PS + b] : 0u;  // uniform rows (kernels.h)
  uint32_t rows[8];
  pick_parked(p, wd.sdc, wd.badc, (nl - wd.nlA) * 2u, p.n0 + nl, p.round, p.PS * 4u, rows);
  const uint32_t bo = b * 4u;
  uint32_t dis = 0u, all = ~0u;
  bool gather = true;
  uint32_t rbytes = 0u;  // reference-row reads
  if (REF && p.rflag_in) {
    // peers whose published row is the reference row (kernels.h rflag_in):
    // when all 8 are, each of the 8 votes is that row's word (the reference
    // word is loaded beside the flags, not after them)
    const uint32_t rw = p.pref_prev[p.ref_node * p.PS + b];
    uint32_t fl = 1u;
#pragma unroll
    for (int j = 0; j < 8; ++j) fl &= p.rflag_in[rows[j] >> p.ps_shift] == ref_tag(p.round) ? 1u : 0u;
    rbytes = 4u + (b == 0u ? 8u : 0u);
    if (fl) {
      dis = all = rw;
      gather = false;
    }
  }
  if (gather) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dis |= at_byte(p.pref_in, rows[j] + bo);
#pragma unroll
    for (int j = 0; j < 8; ++j) all &= at_byte(p.pref_in, rows[j] + bo);
  }
  // every vote equals A  <=>  (OR of votes) == A == (AND of votes) on P0
  if (__ballot(((dis ^ A) | (all ^ A)) & P0) != 0ull) return false;
  const uint32_t node = p.n0 + nl;
  const uint32_t pub = is_byz(p.byz, node) ? byz_pattern(p.round + 1u) : A;
  if (active) {
    if (p.uni_out) acc.umis |= pub != uref ? 1u : 0u;
    const uint32_t prow = node * p.PS + b;  // < N * PS < 2^30 (sweep gate)
    const bool known = AVK_CC_PREFETCH || (kw & 0xFFu) >= 2u;  // (publish)
    publish<POL, CC>(p, prow, pub, AVK_CC_PREFETCH ? old : (is_byz(p.byz, node) ? byz_pattern(p.round - 2u) : pub),
                     acc, known, nl, acc.qslot);
  }
  if (REF && p.rflag_out) ref_flag_store(p, lane, active, b, node, pub, p.pref_in[p.ref_node * p.PS + (active ? b : 0u)]);
  if (lane == 0) p.kpend[tile] = ((kw & 0xFFu) + 1u) | kPendAllLive | (kw & kHiVirt);
  acc.applied += 8u * (uint32_t)__popc(P0);
  // process_tile's accounting for this case: 17 plane words + 8 vote words +
  // valid read, minus V (uniform), V store (virtual), K read + store (deferred),
  // A store (unchanged) = 40 B per lane (+ 4 B push read); kpend read + write
  // reference rows: 8 flag bytes per node read, the reference word instead of
  // the 32 B of gathered votes, the next reference word + the flag written
  acc.reread += active && gather ? 28u : 0u;
  acc.lane_bytes += (active ? 40u + (p.count_changed ? 4u : 0u) + rbytes - (gather ? 0u : 32u) +
                                  (REF && p.rflag_out ? 4u + (b == 0u ? 1u : 0u) : 0u)
                            : 0u) +
                    (lane == 0 ? 8u : 0u);
  return true;
}

// The settled candidates of a wave's run in one lean loop (p.lean: kModeWarm,
// k = 8, klazy round, BL dividing 64, the run's draw parked with no repeated
// candidate). Same test and outputs as settled_tile, with everything that does
// not depend on the tile hoisted out of the loop: a lane's block b = lane % BL
// and its validity word, the run's Byzantine bits (one ballot), the A-plane
// buffer resource (the tile moves the scalar offset only), the node index
// (shift, no division); the kpend words of the settled tiles are written by one
// store per run (lane i: tile t0 + i) and the counters accumulated per tile
// without a branch. Per settled tile: the A load, 8 gathers, 2 LDS reads, one
// ballot, the published-word store. Returns the run's settled tiles (bit i =
// tile t0 + i); the others take the general load + step afterwards.
//
// REF (reference rows, kernels.h rflag_*): a tile whose 8 peers' rows are all
// flagged equal to the reference row takes the reference word (one hoisted
// load per run) for all 8 votes instead of gathering them. The run's flags are
// read in the prologue next to the draw (4 byte loads per producer lane, from
// 1 MB at C4: L2-resident where the 128 MB of rows are not) and kept as one
// ballot. Every settled tile writes its nodes' flags for the row it published.
template <int POL, bool REF, bool CC>
__device__ __forceinline__ uint32_t settled_run(const RoundParams& p, uint32_t lane, uint32_t tile_end,
                                                const WaveDraw& wd, SweepAcc& acc) {
  const uint32_t t0 = wd.t0, ntiles = tile_end - t0;
  const uint32_t b = lane & (p.BL - 1u), bo = b * 4u;
  const uint32_t vw = at_byte(p.valid, bo);
  // Byzantine bits of the run's nodes (local nodes nlA .. nlA + nn - 1, nn <= 64)
  const unsigned long long byzm = __ballot(lane < wd.nn && is_byz(p.byz, p.n0 + wd.nlA + lane));
  const uint32_t bpat = byz_pattern(p.round + 1u);
  const __amdgpu_buffer_rsrc_t ta =
      __builtin_amdgcn_make_buffer_rsrc(p.planes + (size_t)t0 * (kPlanes * 64u), 0, (int)(ntiles * kPlanes * 64u * 4u),
                                        kRsrcWord3);
  const uint32_t aoff = (1536u + lane) * 4u;
  // reference words of this lane's block: the snapshot being written is flagged against rin, the
  // flags of the snapshot being read (prefetched for the run's nodes: wd.flagok) against rprev
  const bool rd = REF && p.rflag_in && wd.flagok != 0ull;
  const uint32_t rprev = rd ? at_byte(p.pref_prev, p.ref_node * p.PS * 4u + bo) : 0u;
  const uint32_t rin = (REF && p.rflag_out) || p.uni_out ? at_byte(p.pref_in, p.ref_node * p.PS * 4u + bo) : 0u;
  uint32_t done = 0u, umis = 0u;
  uint32_t applied = 0u, bytes = 0u, reread = 0u;  // per lane
  for (uint32_t i = 0; i < ntiles; ++i) {
    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)wd.meta, (int)i);
    if ((m & (kPendAllLive | (kVMask << 8))) != (kPendAllLive | (kVUniform << 8))) continue;
    const uint32_t tile = t0 + i;
    const uint32_t A = __builtin_amdgcn_raw_buffer_load_b32(ta, aoff + i * (kPlanes * 64u * 4u), 0, POL > 0 ? 2 : 0);
    const uint32_t g = tile * 64u + lane;
    const bool active = g < p.L;
    const uint32_t nl = (active ? g : p.L - 1u) >> p.bl_log2;
    const uint32_t old = AVK_CC_PREFETCH && CC && p.count_changed ? p.pref_out[(p.n0 + nl) * p.PS + b] : 0u;  // (publish)
    const uint32_t P0 = active ? vw : 0u;  // polled = live (kPendAllLive) and valid
    const uint32_t rel = nl - wd.nlA;
    uint32_t rows[8];
    {
      const uint32_t* q = wd.sdc + rel * 8u;
      const u32x4 lo = *reinterpret_cast<const u32x4*>(q);
      const u32x4 hi = *reinterpret_cast<const u32x4*>(q + 4);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        rows[c] = lo[c];
        rows[c + 4] = hi[c];
      }
    }
    uint32_t dis = 0u, all = ~0u;
    bool gather = true;
    if (rd) {
      const uint32_t base = rel * 2u + wd.fofs;  // the node's producer lanes
      const bool fl = ((wd.flagok >> base) & 3ull) == 3ull;
      if (__ballot(active && !fl) == 0ull) {
        dis = all = rprev;
        gather = false;
      }
    }
    if (gather) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t w = at_byte(p.pref_in, rows[j] + bo);
        dis |= w;
        all &= w;
      }
    }
    // every vote equals A  <=>  (OR of votes) == A == (AND of votes) on P0
    if (__ballot(((dis ^ A) | (all ^ A)) & P0) != 0ull) continue;
    const uint32_t node = p.n0 + nl;
    const uint32_t pub = ((byzm >> rel) & 1ull) ? bpat : A;
    if (active) {
      umis |= pub != rin ? 1u : 0u;
      const uint32_t prow = node * p.PS + b;  // < N * PS < 2^30 (sweep gate)
      const bool known = AVK_CC_PREFETCH || (m & 0xFFu) >= 2u;  // (publish)
      publish<POL, CC>(p, prow, pub, AVK_CC_PREFETCH ? old : (((byzm >> rel) & 1ull) ? byz_pattern(p.round - 2u) : pub),
                       acc, known, nl, i);
    }
    if (REF && p.rflag_out) ref_flag_store(p, lane, active, b, node, pub, rin);
    done |= 1u << i;
    applied += 8u * (uint32_t)__popc(P0);
    // settled_tile's accounting: 40 B per active lane (+ 4 B push read), 28 of the 32 gathered re-read;
    // reference rows: the 8 flag bytes per node instead of the 32 B of votes, the flag byte written
    bytes += active ? 40u + (p.count_changed ? 4u : 0u) - (gather ? 0u : 32u) +
                          (REF && p.rflag_out ? (b == 0u ? 1u : 0u) : 0u)
                    : 0u;
    reread += active && gather ? 28u : 0u;
  }
  // the settled tiles' pending count steps: +1 deferred +8 step each (lane i: tile t0 + i)
  if (lane < ntiles && ((done >> lane) & 1u)) {
    p.kpend[t0 + lane] = ((wd.meta & 0xFFu) + 1u) | kPendAllLive | (wd.meta & kHiVirt);
    bytes += 8u;  // kpend read (prologue) + written
  }
  acc.applied += applied;
  acc.lane_bytes += bytes;
  acc.reread += reread;
  if (p.uni_out) acc.umis |= umis;
  return done;
}

// The settled candidates of a wave's run when every row of pref_in is ref_node's row of pref_prev
// (uniform rows, kernels.h uni_in): each of a lane's 8 gathered votes would be that row's word
// `refp`, whoever the peers are, so the settled test of settled_run needs no peer draw and no
// gather: every polled record's accepted bit equals refp. Same outputs and accounting as
// settled_run otherwise (the published word, the deferred +8 step); the votes' 32 B per lane are
// not read. Bit i of the result = tile t0 + i settled; the other tiles take the draw and the
// general path.
constexpr uint32_t kUniRun = 16;  // longest run settled_run_uni takes (p.tpw <= 16)

// Everything settled_run_uni reads that depends on no other load (the run's A planes, the validity
// word, the reference row's words, the Byzantine bits), requested at the start of the wave's run,
// before the uniform test's slot words and the run's tile words are waited for: the settled wave
// then waits for one memory latency instead of three in a row (slot words -> tile words -> A).
// (A/B: requested at run start, before the uniform test, 4.24 vs 4.19-4.22 ms per C4 epoch after it,
// profiles/r05/s14/ab_pre.log: the settled waves are not waiting on that chain; left off)
#ifndef AVK_UNI_PREFETCH
#define AVK_UNI_PREFETCH 0
#endif
struct UniPre {
  uint32_t Av[kUniRun];
  uint32_t vw, refp, rin;
  unsigned long long byzm[4];
};

template <int POL>
__device__ __forceinline__ void uni_prefetch(const RoundParams& p, uint32_t lane, uint32_t t0, uint32_t tile_end,
                                             uint32_t nlA, uint32_t nn, UniPre& u) {
  const uint32_t ntiles = tile_end - t0;
  const uint32_t bo = (lane & (p.BL - 1u)) * 4u;
  const __amdgpu_buffer_rsrc_t ta =
      __builtin_amdgcn_make_buffer_rsrc(p.planes + (size_t)t0 * (kPlanes * 64u), 0, (int)(ntiles * kPlanes * 64u * 4u),
                                        kRsrcWord3);
  const uint32_t aoff = (1536u + lane) * 4u;
#pragma unroll
  for (uint32_t i = 0; i < kUniRun; ++i)  // tiles past the run: offset past the resource (reads 0, no access)
    u.Av[i] = __builtin_amdgcn_raw_buffer_load_b32(ta, i < ntiles ? aoff + i * (kPlanes * 64u * 4u) : 0x80000000u, 0,
                                                   POL > 0 ? 2 : 0);
  u.vw = at_byte(p.valid, bo);
  u.refp = at_byte(p.pref_prev, p.ref_node * p.PS * 4u + bo);  // every vote word this round
  u.rin = p.uni_out ? at_byte(p.pref_in, p.ref_node * p.PS * 4u + bo) : 0u;
  // the run's Byzantine bits, node nlA + rel at bit rel & 63 of byzm[rel >> 6]: up to 256 nodes (runs of
  // 16 tiles at BL >= 4, the merged runs of uni_merge on target shards)
#pragma unroll
  for (uint32_t j = 0; j < 4u; ++j)
    u.byzm[j] = __ballot(lane + 64u * j < nn && is_byz(p.byz, p.n0 + nlA + lane + 64u * j));
}

template <int POL, bool CC>
__device__ __forceinline__ uint32_t settled_run_uni(const RoundParams& p, uint32_t lane, uint32_t t0,
                                                    uint32_t tile_end, uint32_t meta, uint32_t nlA, uint32_t nn,
                                                    const UniPre& u, SweepAcc& acc) {
  const uint32_t ntiles = tile_end - t0;
  const uint32_t b = lane & (p.BL - 1u);
  const uint32_t vw = u.vw, refp = u.refp, rin = u.rin;
  // a run holding a Byzantine node is left to the general path (a uniform input with Byzantine voters
  // needs every honest row equal to their flip-flop pattern: rare), so that every settled word here
  // is the tile's A plane, with no per-lane Byzantine-bit lookup per tile
  if ((u.byzm[0] | u.byzm[1] | u.byzm[2] | u.byzm[3]) != 0ull) return 0u;
  uint32_t cand = 0u;
  for (uint32_t i = 0; i < ntiles; ++i) {
    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)meta, (int)i);
    if ((m & (kPendAllLive | (kVMask << 8))) == (kPendAllLive | (kVUniform << 8))) cand |= 1u << i;
  }
  uint32_t Av[kUniRun], Ov[kUniRun];
#pragma unroll
  for (uint32_t i = 0; i < kUniRun; ++i) Av[i] = u.Av[i];
  // the overwritten published words (p.count_changed: publish) with them, not one dependent load per tile
#pragma unroll
  for (uint32_t i = 0; i < kUniRun; ++i) {
    const uint32_t g = (t0 + i) * 64u + lane;
    const uint32_t nl = (g < p.L ? g : p.L - 1u) >> p.bl_log2;
    Ov[i] = AVK_CC_PREFETCH && CC && p.count_changed && ((cand >> i) & 1u) ? p.pref_out[(p.n0 + nl) * p.PS + b] : 0u;
  }
  if constexpr (!CC) {
    // The single-GPU (non-counting) build walks the run with no per-tile branch: a tile is settled iff
    // it is a candidate and no polled record's A differs from the reference word (one ballot, a
    // scalar bit); its published words are stored through a resource bounded to the snapshot, with
    // an out-of-range offset for the lanes that must not store (the store is dropped), and the
    // counters take the settled bit as a factor. Per tile: ~half the scalar instructions of the
    // branching walk (the settled rounds are bound by the CU's scalar issue).
    const __amdgpu_buffer_rsrc_t prb =
        __builtin_amdgcn_make_buffer_rsrc(p.pref_out, 0, (int)(p.n_nodes * p.PS * 4u), kRsrcWord3);
    uint32_t done = 0u, applied = 0u, bytes = 0u, umis = 0u;
    // a tile holds 64 / BL nodes: the lane's node and row advance by constants from tile to tile
    // (lanes past the last lane compute a row they never store)
    const uint32_t npt = 64u >> p.bl_log2;
    const uint32_t rel0 = ((t0 * 64u + lane) >> p.bl_log2) - nlA;
    uint32_t prow = (p.n0 + nlA + rel0) * p.PS + b;  // < N * PS < 2^30 (sweep gate)
#pragma unroll
    for (uint32_t i = 0; i < kUniRun; ++i) {
      const uint32_t g = (t0 + i) * 64u + lane;
      const bool active = g < p.L;
      const uint32_t P0 = active ? vw : 0u;  // polled = live (kPendAllLive) and valid
      const uint32_t A = Av[i];
      const uint32_t mis = __ballot((refp ^ A) & P0) != 0ull ? 1u : 0u;  // always evaluated: no branch
      const bool ok = (((cand >> i) & 1u) & (mis ^ 1u)) != 0u;             // wave-uniform
      const uint32_t pub = A;
      const bool st = ok && active;
      __builtin_amdgcn_raw_buffer_store_b32(pub, prb, st ? prow * 4u : 0xFFFFFFFCu, 0, POL == 1 ? 2 : 0);  // (table < 4 GiB: 0xFFFFFFFC is past it)
      umis |= (st & (pub != rin)) ? 1u : 0u;
      done |= ok ? 1u << i : 0u;
      applied += st ? 8u * (uint32_t)__popc(P0) : 0u;
      bytes += st ? 8u : 0u;  // settled_run's accounting without the 32 B of gathered votes
      prow += npt * p.PS;
    }
    if (lane < ntiles && ((done >> lane) & 1u)) {
      p.kpend[t0 + lane] = ((meta & 0xFFu) + 1u) | kPendAllLive | (meta & kHiVirt);
      bytes += 8u;  // kpend read (prologue) + written
    }
    acc.applied += applied;
    acc.lane_bytes += bytes;
    if (p.uni_out) acc.umis |= umis;
    return done;
  }
  uint32_t done = 0u, applied = 0u, bytes = 0u, umis = 0u;
#pragma unroll
  for (uint32_t i = 0; i < kUniRun; ++i) {
    if (!((cand >> i) & 1u)) continue;
    const uint32_t tile = t0 + i;
    const uint32_t A = Av[i];
    const uint32_t g = tile * 64u + lane;
    const bool active = g < p.L;
    const uint32_t nl = (active ? g : p.L - 1u) >> p.bl_log2;
    const uint32_t P0 = active ? vw : 0u;  // polled = live (kPendAllLive) and valid
    if (__ballot((refp ^ A) & P0) != 0ull) continue;
    const uint32_t node = p.n0 + nl;
    const uint32_t pub = A;
    if (active) {
      umis |= pub != rin ? 1u : 0u;
      const uint32_t prow = node * p.PS + b;  // < N * PS < 2^30 (sweep gate)
      // kpend >= 2: this settled tile's accepted plane is unchanged since the snapshot being
      // overwritten (publish): honest rows publish that word again, Byzantine rows its pattern's
      const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)meta, (int)i);
      const bool known = AVK_CC_PREFETCH || (m & 0xFFu) >= 2u;
      const uint32_t old = AVK_CC_PREFETCH ? Ov[i] : pub;
      publish<POL, CC>(p, prow, pub, old, acc, known, nl, i);
    }
    done |= 1u << i;
    applied += 8u * (uint32_t)__popc(P0);
    // settled_run's accounting without the 32 B of gathered votes: A read, valid, published word
    bytes += active ? 8u + (p.count_changed ? 4u : 0u) : 0u;
  }
  if (lane < ntiles && ((done >> lane) & 1u)) {
    p.kpend[t0 + lane] = ((meta & 0xFFu) + 1u) | kPendAllLive | (meta & kHiVirt);
    bytes += 8u;  // kpend read (prologue) + written
  }
  acc.applied += applied;
  acc.lane_bytes += bytes;
  if (p.uni_out) acc.umis |= umis;
  return done;
}

// MODE: kModeWarm (sim, every consider plane all-ones), kModeCheck (sim, per
// tile: the oldest consider plane decides), kModeReplay (replayed votes),
// kModeAblate (kModeCheck with the peer gather replaced by a coalesced read of
// the node's own row: timing diagnostics only, results invalid), kModeWarmPipe
// (kModeWarm for a resident grid: the next tile's loads are issued before the
// current tile is computed; 93 VGPRs, 5 waves per SIMD).
// A/B build knob (Makefile variant libraries): the warm modes' waves per SIMD. Round 3: 6 (80 VGPRs,
// 7 spilled to scratch in cold paths) beat 5 (87 VGPRs) by 4 % (profiles/r03/ab_waves_per_simd.log).
// Round 4 (slot records, non-temporal log): 5 (92 VGPRs, none spilled) beats 6 (80, 8-9 spilled):
// C4p epoch -2.8 / -2.9 %, C4 -0.9 / -1.4 %, C4pb -1.1 %; 7 is 1.3x slower
// (profiles/r04/session13/abwpe.log; 4 compiles to the same code as 5)
#ifndef AVK_WARM_WPE
#define AVK_WARM_WPE 5
#endif
// (the fresh mode at 5 instead: round 0 -1 %, epochs within noise, profiles/r04/session15/abf5.log)
#ifndef AVK_FRESH_WPE
#define AVK_FRESH_WPE 6
#endif
template <int K, int MODE, int POL, bool REF = false, bool CC = true>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MODE == kModeWarmPipe ? 5 : MODE == kModeWarm ? AVK_WARM_WPE : MODE == kModeFresh ? AVK_FRESH_WPE : MODE == kModeReplay ? 6 : 7))) void k_round_sweep(const RoundParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave0 = uni(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t nwaves = gridDim.x * 4u;
  const uint32_t tiles = p.Lpad >> 6;
  SweepAcc acc;
  acc.shard = wave0 & (p.log_shards - 1u);  // a power of two (engine.cpp set_log_layout)
  if constexpr (CC) {  // deferred pushes: the wave's queue (dynamic LDS, launched only with p.push_q)
    extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
    const uint32_t w = threadIdx.x >> 6;
    acc.qpub = reinterpret_cast<uint32_t*>(s_dyn) + w * (kPushQ * 64u);
    acc.qpm = s_dyn + 4u * 4u * kPushQ * 64u + w * (kPushQ * 64u);
  }
  // uniform rows (kernels.h): no rank's slot of pref_in carries this round's tag
  bool uniform = p.uni_in != nullptr;
  if (uniform)
    for (uint32_t r = 0; r < p.uni_world; ++r) uniform = uniform && p.uni_in[r] != p.round;
  // (and of pref_prev: its slots carry round - 1's tag if a row of it differed)
  bool uniform_prev = uniform && p.uni_prev != nullptr && K == 8 && p.uni_votes && p.vv;
  if (uniform_prev)
    for (uint32_t r = 0; r < p.uni_world; ++r) uniform_prev = uniform_prev && p.uni_prev[r] != p.round - 1u;
  const uint32_t uflags = (K == 8 && uniform && p.uni_votes && p.vv ? kUniVotes : 0u) | (uniform_prev ? kUniPrev : 0u);
  if constexpr (MODE == kModeWarmPipe) {
    // software-pipelined: tile t + nwaves's loads (state, peer draw, gathers)
    // are in flight while tile t is computed
    TileIn<K, false, true> cur, nxt;
    uint32_t tile = wave0;
    if (tile < tiles) load_tile<K, false, true, POL, false, true>(p, tile, lane, cur);
    for (; tile < tiles; tile += nwaves) {
      const uint32_t next = tile + nwaves;
      if (next < tiles) load_tile<K, false, true, POL, false, true>(p, next, lane, nxt);
      process_tile<K, false, true, POL, true>(p, tile, lane, cur, 0u, acc);
      cur = nxt;
    }
  } else {
    uint32_t tile = wave0, tile_end = tiles, stride = nwaves;
    WaveDraw wd;
    wd.ok = false;
    wd.pair = false;
    wd.nlA = 0u;
    wd.nn = 0u;
    wd.flagok = 0ull;
    wd.t0 = 0u;
    wd.meta = 0u;
    wd.badc = wd.badp = 0ull;
    wd.sdc = wd.sdp = nullptr;
    wd.fofs = 0u;
    uint32_t uni_done = 0u;  // uniform rows: run tiles settled with no draw (settled_run_uni)
    bool uni_ran = false;
    __shared__ __attribute__((aligned(16))) uint32_t s_draw[4][512];
    uint32_t* const sd = s_draw[threadIdx.x >> 6];
    if constexpr (MODE == kModeWarm && K == 8) {
      if (p.tpw) {
        // a run of p.tpw consecutive tiles per wave; one Philox pass draws the
        // peers of all its nodes (round - 1's too if a tile is kVStale)
        tile = wave0 * p.tpw;
        tile_end = min(tile + p.tpw, tiles);
        stride = 1u;
        if (p.uni_merge > 1u && p.lean && p.settled_fast && p.klazy && p.vv && p.tpw * p.uni_merge <= kUniRun &&
            uniform) {
          // uniform input: most tiles settle with no draw, and what is left per wave is its set-up,
          // so every uni_merge-th wave takes its neighbours' runs too and the others end here
          if (wave0 % p.uni_merge) tile = tile_end = tiles;
          else tile_end = min(tile + p.tpw * p.uni_merge, tiles);
        }
        if (tile < tiles) {
          const uint32_t nlA = uni(div_bl(p, tile * 64u));
          const uint32_t nlB = uni(div_bl(p, min(tile_end * 64u, p.L) - 1u));
          const uint32_t nn = nlB - nlA + 1u;
          // uniform rows: settled_run_uni's loads requested first (UniPre); wasted only in a klazy round
          // whose input is not uniform (the converging rounds), where the general path re-reads A
          UniPre upre;
          const bool uni_ok = p.uni_in && p.lean && p.settled_fast && p.klazy && p.vv && nn <= 256u &&
                              tile_end - tile <= kUniRun;
#if AVK_UNI_PREFETCH
          if (uni_ok) uni_prefetch<POL>(p, lane, tile, tile_end, nlA, nn, upre);
#endif
          // the run's per-tile words, one lane per tile (tpw <= 16)
          const uint32_t ti = tile + lane;
          const uint32_t st = p.vv && ti < tile_end ? p.vstale[ti] : 0u;
          const uint32_t kw = (p.klazy || p.kconsume) && ti < tile_end ? p.kpend[ti] : 0u;
          wd.meta = (st << 8) | (kw & (kPendAllLive | kHiVirt | 0xFFu));
          wd.t0 = tile;
          wd.nlA = nlA;
          wd.nn = nn;
          // uniform rows: the run's settled candidates first, with no draw; the draw only if a tile is left
          const uint32_t all_tiles = (uint32_t)((1ull << (tile_end - tile)) - 1ull);
          if (uni_ok && uniform) {
#if !AVK_UNI_PREFETCH
            uni_prefetch<POL>(p, lane, tile, tile_end, nlA, nn, upre);
#endif
            uni_done = settled_run_uni<POL, CC>(p, lane, tile, tile_end, wd.meta, nlA, nn, upre, acc);
            uni_ran = true;
          }
          const bool any_stale = __ballot((st & kVMask) == kVStale) != 0ull;
          if (uni_done != all_tiles) {
            wd.pair = any_stale;
            wd.flagok = 0ull;
            if (any_stale && nn * 2u > 32u) {
              // both rounds' draws for up to 32 nodes: two passes over all 64 lanes, parked side by side
              const PairDraw dp = single_draw(p, p.round - 1u, nlA, nn, lane);
              const PairDraw dc = single_draw(p, p.round, nlA, nn, lane);
              wd.ok = !dp.fallback && !dc.fallback;
              if (wd.ok) {
                park_draw(dp, sd, lane, p.PS * 4u);
                park_draw(dc, sd + 256, lane, p.PS * 4u);
              }
              wd.sdp = sd;
              wd.sdc = sd + 256;
              wd.badp = dp.bad;
              wd.badc = dc.bad;
            } else {
              // one pass: lanes 0-31 round - 1 and 32-63 this round (pair), or all 64 this round
              const PairDraw d = any_stale ? pair_draw(p, p.round, nlA, nn, lane) : single_draw(p, p.round, nlA, nn, lane);
              wd.ok = !d.fallback;
              if (wd.ok) park_draw(d, sd, lane, p.PS * 4u);
              wd.sdp = sd;
              wd.sdc = any_stale ? sd + 128 : sd;
              wd.badp = d.bad & 0xFFFFFFFFull;
              wd.badc = any_stale ? d.bad >> 32 : d.bad;
              wd.fofs = any_stale ? 32u : 0u;
              if constexpr (REF) {
                if (wd.ok && p.rflag_in && p.klazy) {  // the run's peer flags in 4 loads (settled_run)
                  const uint8_t tag = ref_tag(p.round);
                  uint32_t ok = 1u;
#pragma unroll
                  for (int i = 0; i < 4; ++i) ok &= p.rflag_in[d.prod[i]] == tag ? 1u : 0u;
                  wd.flagok = __ballot(ok != 0u);
                }
              }
            }
          }
        }
      }
    }
    uint32_t lean_done = uni_done;  // run tiles the lean settled loop completed (bit i: tile wd.t0 + i)
    bool lean_ran = uni_ran;        // the run's settled candidates were all tested by it
    if constexpr (MODE == kModeWarm && K == 8) {
      if (!uni_ran && wd.ok && wd.badc == 0ull && p.lean && p.settled_fast && p.klazy && p.vv && tile < tile_end) {
        lean_done = settled_run<POL, REF, CC>(p, lane, tile_end, wd, acc);
        lean_ran = true;
      }
    }
    const uint32_t qfirst = tile, qstep = stride;  // deferred pushes: slot s = tile qfirst + s * qstep
    uint32_t qn = 0;
    if constexpr (MODE == kModeWarm && K == 8) {
      // every tile of the run settled in the lean loops (the settled rounds): no tile loop at all, whose
      // per-tile skip test cost a settled wave ~8 scalar instructions per tile (the settled rounds are
      // bound by the CU's scalar issue); the queued pushes of those tiles are still flushed below
      if (lean_ran && stride == 1u && tile < tile_end &&
          lean_done == (uint32_t)((1ull << (tile_end - tile)) - 1ull)) {
        qn = tile_end - tile;
        tile = tile_end;
      }
    }
    // tile draws (p.tile_draw): a run whose nodes overflow the run's draw (narrow rows: at BL <= 16 a
    // 16-tile run holds 64-256 nodes) still shares one Philox pass per tile, 2 producer lanes per
    // node (a tile's 64 / BL nodes fit: BL >= 2, or >= 4 with a stale tile's paired draw), instead of
    // every lane drawing its node's 8 peers alone (4-16 lanes per node repeating the same draw)
    const bool tdraw = MODE == kModeWarm && K == 8 && p.tile_draw && p.tpw && !wd.ok && tile < tile_end;
    for (; tile < tile_end; tile += stride) {
      constexpr bool AB = MODE == kModeAblate;
      if constexpr (CC) acc.qslot = qn++;
      if constexpr (MODE == kModeWarm) {
        if constexpr (K == 8) {
          if (lean_done && ((lean_done >> (tile - wd.t0)) & 1u)) continue;
          if (tdraw) {
            const uint32_t tnlA = uni(div_bl(p, tile * 64u));
            const uint32_t tnn = uni(div_bl(p, min(tile * 64u + 64u, p.L) - 1u)) - tnlA + 1u;
            const bool tst = ((meta_of(wd, tile) >> 8) & kVMask) == kVStale;  // wave-uniform
            const PairDraw d = tst ? pair_draw(p, p.round, tnlA, tnn, lane) : single_draw(p, p.round, tnlA, tnn, lane);
            wd.ok = !d.fallback;
            if (wd.ok) {
              park_draw(d, sd, lane, p.PS * 4u);
              wd.nlA = tnlA;
              wd.nn = tnn;
              wd.pair = tst;
              wd.sdp = sd;
              wd.sdc = tst ? sd + 128 : sd;
              wd.badp = d.bad & 0xFFFFFFFFull;
              wd.badc = tst ? d.bad >> 32 : d.bad;
              wd.fofs = tst ? 32u : 0u;
              wd.flagok = 0ull;
            }
          }
          if (wd.ok && p.settled_fast && p.klazy && p.vv && !lean_ran) {
            const uint32_t m = meta_of(wd, tile);
            if (((m >> 8) & kVMask) == kVUniform && (m & kPendAllLive) &&
                settled_tile<POL, REF, CC>(p, tile, lane, m & (kPendAllLive | kHiVirt | 0xFFu), wd, acc))
              continue;
          }
        }
        TileIn<K, false, true> in;
        load_tile<K, false, true, POL, false, true, false, CC>(p, tile, lane, in, &wd, uflags);
        process_tile<K, false, true, POL, true, REF, CC>(p, tile, lane, in, 0u, acc, uflags);
      } else if constexpr (MODE == kModeFresh) {
        TileIn<K, false, false> in;
        load_tile<K, false, false, POL, false, true, true>(p, tile, lane, in);
        process_tile<K, false, false, POL, true>(p, tile, lane, in, 0u, acc);
      } else if constexpr (MODE == kModeReplay) {
        TileIn<K, true, false> in;
        load_tile<K, true, false, POL, false>(p, tile, lane, in);
        process_tile<K, true, false, POL>(p, tile, lane, in, 0u, acc);
      } else {
        bool warm = false;
        if (p.warm_skip) {
          // all-ones oldest consider plane <=> all consider planes all-ones (monotone sim votes)
          const uint32_t g = tile * 64u + lane;
          const uint32_t c7 = g < p.L ? p.planes[(size_t)tile * (kPlanes * 64u) + 1024u + 7u * 64u + lane] : ~0u;
          warm = __all(c7 == ~0u);
        }
        if (warm) {
          TileIn<K, false, true> in;
          load_tile<K, false, true, POL, AB>(p, tile, lane, in);
          process_tile<K, false, true, POL>(p, tile, lane, in, 4u, acc);
        } else {
          TileIn<K, false, false> in;
          load_tile<K, false, false, POL, AB>(p, tile, lane, in);
          process_tile<K, false, false, POL>(p, tile, lane, in, 0u, acc);
        }
      }
    }
    if constexpr (CC) {
      if (p.push_q && qn) acc.pushed += (uint32_t)wave_sum(flush_pushes(p, lane, qfirst, qstep, qn, acc.qpub, acc.qpm));
    }
  }
  // one flush per wave (shard = wave index); 32-bit sums: a wave's lanes
  // accumulate < 2^32 over the tiles a grid gives it (the engine's grids
  // walk <= 16 tiles per wave by default, 2^32 / (64 * 32 * 8) = 262k at most)
  const unsigned long long s = wave_sum(acc.applied);
  const unsigned long long f = __ballot(acc.died != 0u) ? wave_sum(acc.died) : 0ull;
  const unsigned long long by = (unsigned long long)wave_sum(acc.lane_bytes) + acc.emitted_bytes;
  const unsigned long long rr = wave_sum(acc.reread);
  if (lane == 0) {
    const uint32_t shard = acc.shard;
    if (s) atomicAdd(&p.applied[shard], s);
    if (f) atomicAdd(&p.finalized[shard], f);
    if (by) atomicAdd(&p.bytes[shard], by);
    if (rr) atomicAdd(&p.bytes[kLogShards + shard], rr);
    if (acc.updates) atomicAdd(&p.upd_count[shard], acc.updates);
  }
  if (p.count_changed && lane == 0 && acc.changed) {
    atomicAdd(&p.changed[acc.shard], (unsigned long long)acc.changed);
    atomicAdd(&p.changed[kLogShards + acc.shard], (unsigned long long)acc.changed_segs);
  }
  if (p.count_changed && lane == 0 && acc.pushed) atomicAdd(&p.changed[2 * kLogShards + acc.shard], (unsigned long long)acc.pushed);
  if (p.uni_out && __ballot(acc.umis != 0u) != 0ull && lane == 0) {
    // some word this wave published differs from the reference row: tag the output snapshot's slot
    // of this rank in every replica (read by the next round, after the barrier in a peer exchange)
    // (p.uni_post: the engine copies the slot to the peers once after the round, in the barrier
    // kernel: every wave of a storm round tags, and 7 system-scope stores per wave into the same 7
    // words serialised the whole round, 0.13 -> 0.6 ms per rank at 8 ranks)
    const uint32_t tag = p.round + 1u;
    p.uni_out[p.uni_rank] = tag;
    if (!p.uni_post)
      for (uint32_t r = 0; r < p.push_n; ++r)
        __hip_atomic_store(peer_ptr(p.push_dst, r) + p.uni_off + p.uni_rank, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// dynamic LDS of a sweep launch: the deferred-push queue of its 4 waves (p.push_q)
constexpr uint32_t kPushQBytes = 4u * kPushQ * 64u * 5u;

template <int K, int MODE, bool CC>
hipError_t launch_mode_cc(const RoundParams& p, uint32_t grid, hipStream_t s) {
  const uint32_t shm = CC && p.push_q ? kPushQBytes : 0u;
  // write-through store policies are built for k = 8 only (the measured workloads)
  const uint32_t pol = (K == 8 && p.store_policy >= 2) ? p.store_policy : (p.plane_nt ? 1u : 0u);
  if constexpr (K == 8 && MODE == kModeWarm) {
    // reference rows (kernels.h): the walking warm mode writes the flags and settled tiles read them
    if (p.rflag_out) {
      if (pol == 1)
        hipLaunchKernelGGL((k_round_sweep<K, MODE, 1, true, CC>), dim3(grid), dim3(256), shm, s, p);
      else
        hipLaunchKernelGGL((k_round_sweep<K, MODE, 0, true, CC>), dim3(grid), dim3(256), shm, s, p);
      return hipGetLastError();
    }
  }
  switch (pol) {
    case 0: hipLaunchKernelGGL((k_round_sweep<K, MODE, 0, false, CC>), dim3(grid), dim3(256), shm, s, p); break;
    case 1: hipLaunchKernelGGL((k_round_sweep<K, MODE, 1, false, CC>), dim3(grid), dim3(256), shm, s, p); break;
    default:
      if constexpr (K == 8) {
        if (pol == 2)
          hipLaunchKernelGGL((k_round_sweep<K, MODE, 2, false, CC>), dim3(grid), dim3(256), shm, s, p);
        else
          hipLaunchKernelGGL((k_round_sweep<K, MODE, 3, false, CC>), dim3(grid), dim3(256), shm, s, p);
      }
  }
  return hipGetLastError();
}

// CC (changed-word counting and peer pushes, p.count_changed): the walking warm mode at k = 8 (the
// hot path) has a separate build without it, so that its single-GPU rounds carry none of the
// prefetched overwritten words' registers; every other mode keeps the runtime switch
template <int K, int MODE>
hipError_t launch_mode(const RoundParams& p, uint32_t grid, hipStream_t s) {
  if constexpr (K == 8 && MODE == kModeWarm) {
    if (!p.count_changed) return launch_mode_cc<K, MODE, false>(p, grid, s);
  }
  return launch_mode_cc<K, MODE, true>(p, grid, s);
}

template <int K>
hipError_t launch_sweep_k(const RoundParams& p_in, bool replay, uint32_t blocks, hipStream_t s, bool* ref_written) {
  if (ref_written) *ref_written = false;
  const uint32_t need = (p_in.Lpad / 64u + 3u) / 4u;
  const uint32_t grid = std::max(1u, blocks ? std::min(blocks, need) : need);
  RoundParams p = p_in;
  p.tpw = 0u;
  // deferred pushes: every wave of the grid takes at most kPushQ tiles (a run, or a grid stride over
  // <= kPushQ tiles) and at most 8 peers (the queue's byte per lane); the resident pipelined grid and
  // larger worlds push from the tile loop
  {
    const uint32_t waves = grid * 4u, tiles = p.Lpad / 64u;
    p.push_q = p.push_defer && p.push_n && p.push_n <= 8u && (tiles + waves - 1u) / waves <= kPushQ ? 1u : 0u;
  }
  if (p_in.tpw && K == 8 && !replay && !p.ablate_gather && !p.fresh && p.warm_skip && p.warm_all) {
    // p_in.tpw = enabled: each wave takes a run of consecutive tiles
    const uint32_t tiles = p.Lpad / 64u, waves = grid * 4u;
    p.tpw = (tiles + waves - 1u) / waves;
    if (p.tpw > 16u) p.tpw = 0u;  // long runs: grid stride (their nodes overflow the shared draw anyway)
    if (p.tpw) {
      if (ref_written) *ref_written = p.rflag_out != nullptr;
      return launch_mode<K, kModeWarm>(p, grid, s);
    }
  }
  p.rflag_out = nullptr;  // only the walking warm mode writes reference-row flags
  p.rflag_in = nullptr;
  if (replay) return launch_mode<K, kModeReplay>(p, grid, s);
  if (p.ablate_gather) return launch_mode<K, kModeAblate>(p, grid, s);
  if (p.fresh) return launch_mode<K, kModeFresh>(p, grid, s);
  if (p.warm_skip && p.warm_all) {  // a resident grid walks several tiles per wave: pipeline them
    if (blocks && grid < need && !p.nopipe) {
      p.push_q = 0u;
      return launch_mode<K, kModeWarmPipe>(p, grid, s);
    }
    return launch_mode<K, kModeWarm>(p, grid, s);
  }
  return launch_mode<K, kModeCheck>(p, grid, s);
}

// Materialize stale V planes (kernels.h vv) before anything other than a warm
// k = 8 sim round reads or writes the records: the vote register of a stale
// tile is the last round's 8 gathered votes, V_i = slot 7 - i.
__global__ __launch_bounds__(256) void k_vv_materialize(const RoundParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t tile = uni(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t raw = tile < (p.Lpad >> 6) ? uni(p.vstale[tile]) : 0u;
  if (raw == 0u) return;
  const uint32_t st = raw & kVMask;
  const LaneIdx x = lane_idx(p, tile, lane);
  if (raw & kCAll) {  // consider planes: all-ones
    if (x.active) {
      uint32_t* const tp = p.planes + (size_t)tile * (kPlanes * 64u);
#pragma unroll
      for (int i = 0; i < 8; ++i) tp[1024u + (uint32_t)i * 64u + lane] = ~0u;
    }
    if (st == 0u) {
      if (lane == 0) p.vstale[tile] = 0u;
      return;
    }
  }
  u32x4 o0, o1;
  if (st == kVUniform) {  // V_i = A on every polled record
    const uint32_t A = p.planes[(size_t)tile * (kPlanes * 64u) + 1536u + lane];
    o0 = o1 = u32x4{A, A, A, A};
  } else {
    const uint32_t nlA = uni(x.nl), nn = (uint32_t)__builtin_amdgcn_readlane((int)x.nl, 63) - nlA + 1u;
    uint32_t pp[8];
    draw_peers<8>(p, p.round - 1u, x.node, x.nl, nlA, nn, lane, pp);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o0[i] = p.pref_prev[pp[7 - i] * p.PS + x.b];
      o1[i] = p.pref_prev[pp[3 - i] * p.PS + x.b];
    }
  }
  if (x.active) {
    u32x4* const grp = reinterpret_cast<u32x4*>(p.planes + (size_t)tile * (kPlanes * 64u)) + lane;
    grp[0] = o0;
    grp[64] = o1;
  }
  if (lane == 0) p.vstale[tile] = 0u;
}

// Apply deferred count planes (kernels.h klazy): + 8 * pending on the polled
// (live, valid) records of each tile with pending steps, then clear them.
__global__ __launch_bounds__(256) void k_kl_materialize(const RoundParams p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t tile = uni(blockIdx.x * 4u + (threadIdx.x >> 6));
  if (tile >= (p.Lpad >> 6)) return;
  const uint32_t kw = uni(p.kpend[tile]);
  const uint32_t pend = kw & 0xFFu;
  if (kw == 0u) return;
  const LaneIdx x = lane_idx(p, tile, lane);
  if ((pend || (kw & kHiVirt)) && x.active) {
    u32x4* const grp = reinterpret_cast<u32x4*>(p.planes + (size_t)tile * (kPlanes * 64u)) + lane;
    const u32x4 k0 = grp[128];
    const u32x4 k1 = kw & kHiVirt ? u32x4{0u, 0u, 0u, ~real_mask(p.tn, x.b)} : grp[192];  // kernels.h kHiVirt
    uint32_t Kp[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      Kp[i] = k0[i];
      Kp[4 + i] = k1[i];
    }
    const uint32_t P0 = ~Kp[7] & p.valid[x.b];
    uint32_t cy = 0u;
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // + pend on count bits 3..6
      const uint32_t bi = ((pend >> i) & 1u) ? P0 : 0u;
      const uint32_t t = Kp[3 + i] ^ bi;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[3 + i] & bi);
      Kp[3 + i] = si;
    }
    u32x4 o0, o1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o0[i] = Kp[i];
      o1[i] = Kp[4 + i];
    }
    grp[128] = o0;
    grp[192] = o1;
  }
  if (lane == 0) p.kpend[tile] = 0u;
}

// The write-back's stores non-temporal (a write-only stream; the next round streams the planes back
// with non-temporal loads of its own), which also leaves L2 / MALL to the stale tiles' regathered
// rows. A/B (tools/wb_probe.py, three alternations on one box, profiles/r05/s18/ab_matnt.log):
// C4 0.80 -> 0.74 ms, C4p 0.65 -> 0.455, C5 1.56 -> 1.42 per segment end.
#ifndef AVK_MAT_NT
#define AVK_MAT_NT 1
#endif
// Both deferred forms written back in one pass (do_v: stale vote planes and unstored consider planes,
// as k_vv_materialize; do_k: pending count steps and virtual K4..K7 groups, as k_kl_materialize).
// Per tile every load (A for a uniform vote register, the K groups, a stale tile's peer rows) is issued
// before any store: vmcnt counts loads and stores in issue order, so a load issued after the tile's
// consider-plane stores waited for their write acknowledgements too (round 5's walking version paid
// that per tile, 16 tiles in a row per wave: ~5 TB/s at C4's segment end). A wave takes `run`
// consecutive tiles (default 1: the memory system hides each tile's round trip behind other waves').
__device__ __forceinline__ void materialize_tile(const RoundParams& p, uint32_t tile, uint32_t lane, uint32_t raw,
                                                 uint32_t kw) {
  const LaneIdx x = lane_idx(p, tile, lane);
  uint32_t* const tp = p.planes + (size_t)tile * (kPlanes * 64u);
  u32x4* const grp = reinterpret_cast<u32x4*>(tp) + lane;
  const uint32_t st = raw & kVMask;
  const uint32_t pend = kw & 0xFFu;
  const bool dok = (pend || (kw & kHiVirt)) && x.active;
  // ---- loads
  u32x4 o0, o1, k0, k1;
  if (st == kVUniform) {  // V_i = A on every polled record
    const uint32_t A = tp[1536u + lane];
    o0 = o1 = u32x4{A, A, A, A};
  } else if (st) {  // the last round's 8 gathered votes, V_i = slot 7 - i
    const uint32_t nlA = uni(x.nl), nn = (uint32_t)__builtin_amdgcn_readlane((int)x.nl, 63) - nlA + 1u;
    uint32_t pp[8];
    draw_peers<8>(p, p.round - 1u, x.node, x.nl, nlA, nn, lane, pp);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      o0[c] = p.pref_prev[pp[7 - c] * p.PS + x.b];
      o1[c] = p.pref_prev[pp[3 - c] * p.PS + x.b];
    }
  }
  uint32_t vb = 0u;
  if (dok) {
    k0 = grp[128];
    k1 = kw & kHiVirt ? u32x4{0u, 0u, 0u, ~real_mask(p.tn, x.b)} : grp[192];  // kernels.h kHiVirt
    vb = p.valid[x.b];
  }
  // ---- stores
  if ((raw & kCAll) && x.active) {  // consider planes: all-ones
#pragma unroll
    for (int c = 0; c < 8; ++c) pst<AVK_MAT_NT>(tp + 1024u + (uint32_t)c * 64u + lane, ~0u);
  }
  if (st && x.active) {
    pst4<AVK_MAT_NT>(grp, o0);
    pst4<AVK_MAT_NT>(grp + 64, o1);
  }
  if (dok) {  // + 8 * pend on the polled records' counts
    uint32_t Kp[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      Kp[c] = k0[c];
      Kp[4 + c] = k1[c];
    }
    const uint32_t P0 = ~Kp[7] & vb;
    uint32_t cy = 0u;
#pragma unroll
    for (int c = 0; c < 4; ++c) {  // + pend on count bits 3..6
      const uint32_t bi = ((pend >> c) & 1u) ? P0 : 0u;
      const uint32_t t = Kp[3 + c] ^ bi;
      const uint32_t si = t ^ cy;
      cy = (t & cy) | (Kp[3 + c] & bi);
      Kp[3 + c] = si;
    }
    u32x4 o2, o3;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      o2[c] = Kp[c];
      o3[c] = Kp[4 + c];
    }
    pst4<AVK_MAT_NT>(grp + 128, o2);
    pst4<AVK_MAT_NT>(grp + 192, o3);
  }
}

__global__ __launch_bounds__(256) void k_materialize(const RoundParams p, uint32_t run, uint32_t do_v, uint32_t do_k) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = uni(blockIdx.x * 4u + (threadIdx.x >> 6));
  const uint32_t tiles = p.Lpad >> 6;
  if (run == 1u) {  // the tile words as scalar loads (the tile index is wave-uniform)
    if (wave >= tiles) return;
    const uint32_t raw = do_v ? uni(p.vstale[wave]) : 0u;
    const uint32_t kw = do_k ? uni(p.kpend[wave]) : 0u;
    if (raw == 0u && kw == 0u) return;
    materialize_tile(p, wave, lane, raw, kw);
    if (lane == 0) {
      if (raw) p.vstale[wave] = 0u;
      if (kw) p.kpend[wave] = 0u;
    }
    return;
  }
  const uint32_t t0 = wave * run;
  if (t0 >= tiles) return;
  const uint32_t n = min(run, tiles - t0);
  const uint32_t ti = t0 + lane;
  const uint32_t stw = do_v && lane < n ? p.vstale[ti] : 0u;
  const uint32_t kww = do_k && lane < n ? p.kpend[ti] : 0u;
  if (__ballot(stw != 0u || kww != 0u) == 0ull) return;
  for (uint32_t i = 0; i < n; ++i) {
    const uint32_t raw = (uint32_t)__builtin_amdgcn_readlane((int)stw, (int)i);
    const uint32_t kw = (uint32_t)__builtin_amdgcn_readlane((int)kww, (int)i);
    if (raw == 0u && kw == 0u) continue;
    materialize_tile(p, t0 + i, lane, raw, kw);
  }
  if (lane < n) {
    if (stw) p.vstale[ti] = 0u;
    if (kww) p.kpend[ti] = 0u;
  }
}

template <int K>
hipError_t occupancy_k(bool replay, int* bpc) {
  return replay ? hipOccupancyMaxActiveBlocksPerMultiprocessor(bpc, k_round_sweep<K, kModeReplay, 1>, 256, 0)
                : hipOccupancyMaxActiveBlocksPerMultiprocessor(bpc, k_round_sweep<K, kModeWarmPipe, 1>, 256, 0);
}

}  // namespace

#define AVK_SWEEP_SWITCH(k, CALL) \
  switch (k) {                    \
    case 1: return CALL(1);       \
    case 2: return CALL(2);       \
    case 3: return CALL(3);       \
    case 4: return CALL(4);       \
    case 5: return CALL(5);       \
    case 6: return CALL(6);       \
    case 7: return CALL(7);       \
    case 8: return CALL(8);       \
    default: return hipErrorInvalidValue; \
  }

hipError_t launch_round_sweep(const RoundParams& p, int k, bool replay, uint32_t blocks, hipStream_t s,
                              bool* ref_written) {
#define AVK_SW(K) launch_sweep_k<K>(p, replay, blocks, s, ref_written)
  AVK_SWEEP_SWITCH(k, AVK_SW)
#undef AVK_SW
}

hipError_t launch_vv_materialize(const RoundParams& p, hipStream_t s) {
  if (!p.vstale || !p.pref_prev) return hipErrorInvalidValue;
  const uint32_t tiles = p.Lpad / 64u;
  hipLaunchKernelGGL(k_vv_materialize, dim3((tiles + 3u) / 4u), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t launch_materialize(const RoundParams& p, bool do_v, bool do_k, hipStream_t s) {
  if ((do_v && (!p.vstale || !p.pref_prev)) || (do_k && !p.kpend)) return hipErrorInvalidValue;
  if (!do_v && !do_k) return hipSuccess;
  const uint32_t run = p.mat_run ? p.mat_run : 1u;
  const uint32_t tiles = p.Lpad / 64u;
  const uint32_t waves = (tiles + run - 1u) / run;
  hipLaunchKernelGGL(k_materialize, dim3((waves + 3u) / 4u), dim3(256), 0, s, p, run, do_v ? 1u : 0u, do_k ? 1u : 0u);
  return hipGetLastError();
}

hipError_t launch_kl_materialize(const RoundParams& p, hipStream_t s) {
  if (!p.kpend) return hipErrorInvalidValue;
  const uint32_t tiles = p.Lpad / 64u;
  hipLaunchKernelGGL(k_kl_materialize, dim3((tiles + 3u) / 4u), dim3(256), 0, s, p);
  return hipGetLastError();
}

hipError_t round_sweep_occupancy(int k, bool replay, int* blocks_per_cu, int* cus) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  e = hipDeviceGetAttribute(cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
#define AVK_OCC(K) occupancy_k<K>(replay, blocks_per_cu)
  AVK_SWEEP_SWITCH(k, AVK_OCC)
#undef AVK_OCC
}

}  // namespace avk
