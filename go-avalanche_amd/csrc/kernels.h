// Internal interface between the C-ABI engine (engine.cpp) and the CDNA4
// kernels (kernels.hip). Not part of the public ABI (include/avhip.h).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace avk {

// ---------------------------------------------------------------------------
// State layout in HBM (see DESIGN.md "Data layout").
//
// One *block* = 32 consecutive targets of one node. Its 32 VoteRecords
// (vote.go:25-29) are stored bit-sliced as 25 u32 planes:
//   V0..V7  votes shift register, V0 = most recent vote   (vote.go:26)
//   C0..C7  consider shift register                         (vote.go:27)
//   A       accepted bit = confidence & 1                   (vote.go:38-40)
//   K0..K7  count = confidence >> 1 (0..127 live); K7 = 1 marks "no live
//           record" (deleted after finalization, processor.go:114-116, or
//           never added). A dead record keeps A = published decision.
// A *lane* is one (local node, local block) pair, g = node_local * BL + b.
// Lanes are grouped in tiles of 64 (one wavefront); a tile stores its 25
// planes in one contiguous 6400-byte span (plane_off() in kernels.hip):
// V0-3, V4-7, K0-3, K4-7 as lane-interleaved 16-byte groups (one dwordx4 per
// lane = 1 KiB contiguous per wave-instruction), then C0..C7 and A as dword
// planes (256 B per wave-instruction).
// ---------------------------------------------------------------------------
constexpr int kPlanes = 25;
constexpr int kPV = 0, kPC = 8, kPA = 16, kPK = 17;
constexpr uint32_t kLogShards = 1024;   // update-log / counter shards
// u32 elements between two shards' log counters: one counter per 128-B line, so that the reserving
// atomics of different shards (3 per wave-tile in a storm round) do not serialize on shared lines
constexpr uint32_t kCtrStride = 32;
constexpr uint32_t kMaxPoll = 4096;     // AvalancheMaxElementPoll, avalanche.go:17
constexpr int kMaxK = 16;
constexpr int kMaxPeers = 15;           // peer-push exchange: other ranks of a node-sharded network

// Replay stream layout (one round): per tile of 64 lanes, ceil(k/2) groups of
// 64 lane-interleaved 16-byte records; group q of lane g holds (yes, consider)
// of slot 2q and of slot 2q+1. A wave reads two slots with one dwordx4 per
// lane (1 KiB contiguous per wave-instruction), like the V/K plane groups.
__host__ __device__ constexpr size_t replay_groups(int k) { return (size_t)((k + 1) / 2); }
__host__ __device__ inline size_t replay_words(uint32_t Lpad, int k) { return replay_groups(k) * 4u * Lpad; }
// word index of slot j's yes (c = 0) or consider (c = 1) word of lane g
__host__ __device__ inline size_t replay_idx(uint32_t g, int k, int j, int c) {
  return (((size_t)(g >> 6) * replay_groups(k) + (size_t)(j >> 1)) * 64u + (g & 63u)) * 4u + (size_t)((j & 1) * 2 + c);
}

// Words per node row of the published-preference tables: BL rounded up to a
// power of two (BL <= 32) or to a multiple of 32 (BL > 32), so that the k
// rows a node gathers each round start on 128-B line boundaries (an
// unaligned 63-word row touches 3 lines instead of 2). Padding words are
// never read.
__host__ __device__ constexpr uint32_t pref_stride(uint32_t BL) {
  return BL > 32u ? (BL + 31u) / 32u * 32u : (BL <= 1u ? 1u : 1u << (32 - __builtin_clz(BL - 1u)));
}

// Device pointers of every rank's copy of a buffer, passed by value (kernel arguments: static
// indices keep them in SGPRs, no table load per use).
struct PeerPtrs {
  uint32_t* p[kMaxPeers + 1];
};

struct RoundParams {
  uint32_t* planes;
  const uint32_t* pref_in;   // [N_pad][PS] published preference (round start)
  uint32_t* pref_out;        // [N_pad][PS] published preference (round end)
  const uint32_t* valid;     // [BL] Target.IsValid() bits
  const uint32_t* byz;       // [ceil(N/32)] Byzantine node bits
  const uint32_t* replay;    // replay mode: yes/consider words of each lane and slot (replay_idx)
  uint64_t* log;             // [kLogShards][log_cap] single StatusUpdates
  uint32_t* log_count;       // [3][kLogShards][kCtrStride]: singles, medium, dense records reserved per shard (element 0)
  uint64_t* dlog;            // [kLogShards][dlog_cap][dense_words(k)] dense lane records
  uint32_t* dlog_count;      // = log_count + 2 * kLogShards * kCtrStride
  uint32_t* upd_count;       // [kLogShards] StatusUpdates emitted (singles + medium + dense)
  uint64_t* mlog;            // [kLogShards][mlog_cap][med_rec_words()] medium lane records
  uint32_t* mlog_count;      // = log_count + kLogShards * kCtrStride
  uint32_t* log_overflow;    // [1]
  uint32_t* node_flags;      // [NL] capped path: nodes left to the exact pass (nullptr: none)
  // exact pass (k_round_capped behind k_round_node / k_replay_node): node_flags[nl] = 1 + the first
  // round, relative to the fused launch, that the exact pass takes the node (k_round_node: 1); the
  // launch for relative round exact_rel takes the nodes with 0 < flag <= exact_rel + 1 and clears
  // their flags unless exact_keep
  uint32_t exact_rel;
  uint32_t exact_keep;
  // fused replay rounds (k_replay_node): rounds in the launch, replay words per round, the three
  // preference snapshots and the index of the one the launch's first round writes
  uint32_t fuse_rounds;
  uint32_t ring_next;
  uint32_t replay_fast;  // k_replay_fast takes the nodes whose first 128 lanes are all live and valid
  uint64_t replay_stride;
  uint32_t* pref_ring[3];
  unsigned long long* applied;  // [kLogShards] regsiterVote applications
  unsigned long long* bytes;    // [2 kLogShards] model bytes moved by the round kernel; [kLogShards + i]: the part
                                // that re-reads preference words already gathered this round (not compulsory)
  unsigned long long* finalized;  // [kLogShards] records finalized (deleted, processor.go:114-116)
  uint64_t seed;
  uint32_t log_cap;          // entries per shard
  uint32_t dlog_cap;         // dense records per shard
  uint32_t mlog_cap;         // medium records per shard
  uint32_t log_shards;       // shards in use (<= kLogShards; min(waves, kLogShards))
  uint32_t n_nodes;          // N (global)
  uint32_t n0;               // first local node (global id)
  uint32_t NL;               // local nodes
  uint32_t BL;               // local blocks per node
  uint32_t PS;               // words per node row of the preference tables (pref_stride(BL))
  uint32_t L;                // lanes = NL * BL
  uint32_t Lpad;             // tiles * 64
  uint32_t t0;               // first local target (global id, multiple of 32)
  uint32_t round;            // global round index (RNG counter, byz pattern)
  uint32_t round_rel;        // round - log base (update key field)
  uint32_t round_shift;      // bit of the update word's round field (pack_update)
  int32_t peer_mode;
  uint32_t warm_skip;        // consider planes are monotone (sim votes only): skip all-ones planes
  uint32_t plane_nt;         // stream state planes with non-temporal loads/stores
  uint32_t ablate_gather;    // diagnostics only: gather the node's own row (wrong results)
  uint32_t ablate_emit;      // diagnostics only: count StatusUpdates, store none (log left empty)
  // diagnostics only (k_round_sweep's warm k = 8 general tiles; results invalid), per-phase ablation:
  // 1 = no peer-row gathers (the votes are made from the row offsets), 2 = no K / A plane loads,
  // 4 = no K / A / published-word stores, 16 = no slot network (no vote changes anything)
  uint32_t ablate_phase;
  uint32_t ablate_node;      // diagnostics only (k_round_node, wrong results): 1 = only the lanes below the
                             // cap run, 4 = no plane stores
  // k_round_sweep only
  uint32_t warm_all;         // every consider plane of every lane is all-ones (no per-tile check)
  uint32_t store_policy;     // 0/1: per plane_nt; 2: sc1 plane/pref stores; 3: nt sc1 (k = 8)
  uint32_t bl_magic, bl_sh1, bl_sh2;  // n / BL = (t + ((n - t) >> sh1)) >> sh2, t = mulhi(n, magic)
  // Recomputed vote registers (k = 8, warm sim rounds): after a
  // round of 8 sim votes a record's vote register is exactly that round's 8
  // gathered words, so a tile may skip storing its V planes and the next
  // round regathers them from the previous snapshot instead of reading them.
  uint32_t vv;               // this round may leave V planes unstored (vstale)
  uint32_t vv_uniform;       // ... only in the uniform form (kVUniform: settled tiles; never kVStale)
  // [tiles] kVStale: the tile's V planes are stale, V = votes of round - 1
  // (regathered with round - 1's peers); kVUniform: the tile was settled (all
  // 8 votes of round - 1 equal the accepted bit of every polled record), so V
  // = A on the polled records and nothing needs gathering; 0: V stored.
  // | kCAll: the tile's consider planes were left unstored by the fresh round
  // (after 8 sim votes every consider bit of the tile is 1; no record of the
  // tile is live-but-invalid) and read as all-ones until written back.
  uint32_t* vstale;
  const uint32_t* pref_prev; // [N_pad][PS] snapshot of round - 1 (read by stale tiles)
  // Peer-push exchange (node-sharded engines, k_round_sweep only):
  // every replica of a snapshot buffer is identical between rounds, so the
  // word a lane is about to overwrite in its own row of pref_out is also what
  // every peer's replica holds; a lane whose published word changed stores the
  // new word into each peer's replica (push_dst[i] = peer i's pref_out; a
  // device table, read with scalar loads through the constant address space: no vector load and no
  // vmcnt drain per push).
  uint32_t push_n;
  uint32_t* const* push_dst;
  // Changed published words (engine option "count_changed"; always counted in a peer-push round): a
  // lane whose published word differs from the word it overwrites in pref_out (= what every peer
  // replica holds) counts one in changed[shard] — the words a peer-push round sends to each peer
  // 
  // (and [kLogShards + shard]: the 16-lane groups of a wave holding a changed word = 64-B row segments
  // when a wave's lanes are contiguous row words, PS == BL a multiple of 16; per-wave 16-bit sums)
  uint32_t count_changed;
  unsigned long long* changed;  // [3 kLogShards]: changed words, changed segments, words pushed (all peers)
  // Need-masked exchange (engine option "peer_mask"): a peer replica's copy of a row is
  // read only by the rounds that draw that row, so a rank pushes a row segment to peer i only if one of
  // peer i's nodes draws the row in the next round (need[nl] bit i, peer i in push_dst order; nullptr:
  // every peer), and keeps per (row, 32-word segment) and snapshot buffer the peers whose copy may
  // differ from its own (stale[nl * segs + seg] bit i, for pref_out's buffer): such a segment is
  // pushed whole the next time that peer needs it. Segments never straddle a wave (BL a power of two
  // <= 32 or a multiple of 32), so a wave's ballot decides a segment's bits alone.
  const uint8_t* need;
  uint8_t* stale;       // nullptr: unmasked pushes (every changed word to every peer)
  uint32_t segs;        // 32-word segments per row: ceil(BL / 32)
  uint32_t peer_all;    // (1 << push_n) - 1
  // the pushes queued in LDS and stored after a wave's last tile (round_sweep.hip flush_pushes): the
  // sweep's waves each take at most kPushQ tiles and push_n <= 8 (a byte per lane and tile)
  uint32_t push_q;
  uint32_t push_defer;  // engine option "push_defer" (default 1): the sweep may queue its pushes (push_q)
  uint32_t tile_draw;   // engine option "tile_draw": per-tile shared draws in runs that overflow the run's draw
  uint32_t mat_run;     // engine option "materialize_run": tiles per wave of k_materialize (0 = 1)
  uint32_t push_store;  // engine option "push_store": 1 = plain stores (default), 0 = system scope, 2 = none (diagnostics)
  // Deferred count planes (`kl`, k = 8, warm sim rounds in which no record can
  // finalize): a tile all of whose polled records agreed with
  // their accepted bit on all 8 votes gains exactly +8 on every polled count
  // (vote.go:66-69) and nothing else changes in its K planes; it leaves them
  // unstored and counts the pending +8 steps in kpend[tile] instead. The true
  // count of a live, valid record is K + 8 * pending; dead or invalid records
  // are untouched. kpend[tile]: bits 0..7 pending steps, bit 31 the tile's
  // live records are exactly its valid targets' records (its K planes need not
  // be read to find the polled set).
  uint32_t klazy;            // this round may defer count planes
  uint32_t* kpend;           // [tiles]
  // kconsume: a warm k = 8 sim round that may finalize records (no deferral)
  // applies the tiles' pending steps itself before it tests for count 120
  // (instead of a separate write-back pass) and clears kpend.
  uint32_t kconsume;
  // Reference rows (converged networks; k_round_sweep with BL dividing 64, so a node's lanes sit in
  // one wave): rflag_out[node] = 1 iff the row the node publishes into pref_out equals node
  // ref_node's row in pref_in (written for every node by every such round); rflag_in = the same
  // flags of pref_in, against ref_node's row in pref_prev. A settled-tile candidate whose 8 peers
  // are all flagged reads that reference row once instead of gathering 8 peer rows: each of them
  // IS the reference row, bit for bit. nullptr: not used / not written.
  uint32_t ref_node;
  uint32_t ps_shift;         // log2(PS * 4): peer index of a row byte offset
  const uint8_t* rflag_in;
  uint8_t* rflag_out;
  uint32_t rflag_off;        // byte offset of the flag bytes in every snapshot buffer (peer pushes)

  // Uniform rows (k_round_sweep, k = 8). Every snapshot buffer holds, uni_off words
  // in, one mismatch slot per rank. A wave that publishes into pref_out a word differing from
  // ref_node's word in pref_in stores the tag p.round + 1 into its rank's slot of pref_out (and of
  // every peer replica): uni_out = pref_out + uni_off. uni_in = pref_in + uni_off (nullptr: pref_in
  // was not written by such a round): if none of its uni_world slots holds p.round, every row of
  // pref_in equals ref_node's row of pref_prev, so every gathered vote word is that row's word and a
  // settled-candidate tile is tested with no peer draw and no gather (settled_run_uni). A stale slot
  // can only read as a mismatch (tags are unique per round), never hide one.
  uint32_t* uni_out;
  const uint32_t* uni_in;
  const uint32_t* uni_prev;  // pref_prev + uni_off (nullptr: its slots not maintained); round_sweep.hip kUniPrev
  uint32_t uni_world, uni_rank, uni_off;
  uint32_t uni_merge;  // a round with a uniform input: every uni_merge-th wave takes uni_merge runs (1: off)
  uint32_t uni_post;   // peer-push rounds: the rank's slot reaches the peers after the round (launch_peer_barrier)

  // fresh: the round right after av_init_records: every record is a
  // NewVoteRecord (votes = consider = 0, count 0, vote.go:33-35), so the
  // kernel reads only the A plane; the live mask of a block is its existing
  // targets (tn = targets in this engine's range).
  uint32_t fresh;
  uint32_t tn;
  uint32_t hivirt;  // k = 8 sweep rounds may leave the K4..K7 group unstored (kHiVirt)
  uint32_t tpw;     // kModeWarm, k = 8: run length of consecutive tiles per wave with one shared peer draw (0 = grid stride)
  uint32_t settled_fast;  // kModeWarm, k = 8: settled tiles skip process_tile (round_sweep.hip settled_fast)
  // kModeWarm, k = 8, BL dividing 64 (a lane's block is lane % BL): the settled candidates of a wave's
  // run are tested first in one lean loop (round_sweep.hip settled_run); bl_log2 = log2(BL)
  uint32_t lean;
  uint32_t bl_log2;
  uint32_t nopipe;  // tuning: a grid smaller than the tile count runs kModeWarm (no next-tile prefetch)
  // Responder variants (engine option "responder", first-generation kernel
  // only; see publish_word): pub_mode 0 = R2 decision, 1 = IsAccepted
  // literally, 2 = the example's responder, whose re-adds of queried targets
  // are marked in readd[g] (OR of the polled masks per peer lane) and applied
  // by k_readd after the round (died_out[g]: records deleted this round).
  // nopoll: [ceil(NL/32)] local nodes that do not poll (their loop returned).
  uint32_t pub_mode;
  uint32_t* readd;
  uint32_t* died_out;
  const uint32_t* nopoll;
  uint32_t dense_min;  // a lane with >= dense_min updates logs one dense record (default dense_min(k))
  uint32_t uni_votes;  // k = 8 warm sweep, uniform input (uni_in): general-path tiles take the reference word
                       // as their 8 votes instead of gathering them (option "uni_votes"; round_sweep.hip load_tile)
  uint32_t wave_dense; // k = 8 sweep (A/B option "wave_dense"): a wave with >= wave_dense lanes holding updates
                       // logs every such lane as a dense record (one store branch, no slot-word network); 0 off
};
constexpr uint32_t kPendAllLive = 0x80000000u;
// kpend bit 30 (kHiVirt, k = 8 sweep rounds while every count is < 16; option "k_hi_virtual"): the
// tile's K4..K7 group is not stored: K4 = K5 = K6 = 0 on every record and K7 = the records past the
// engine's last target (k_init_planes: every existing target's record live, none deleted since).
// Set by the fresh round; kept by a warm round whose counts all stay < 16 with no deletion (or
// that defers the tile's count planes); written back by the round that breaks it, kconsume and
// k_kl_materialize (k_read_records_v reads it virtually).
constexpr uint32_t kHiVirt = 0x40000000u;
__host__ __device__ inline uint32_t real_mask(uint32_t tn, uint32_t b) {  // existing targets of local block b
  const uint32_t rem = tn > b * 32u ? tn - b * 32u : 0u;
  return rem >= 32u ? ~0u : ((1u << rem) - 1u);
}
constexpr uint32_t kVStale = 1u, kVUniform = 2u, kVMask = 3u, kCAll = 4u;

// Division by the (runtime) block count BL without a hardware divide:
// Granlund-Montgomery round-up magic, exact for every 32-bit n.
inline void bl_divider(uint32_t d, uint32_t& magic, uint32_t& sh1, uint32_t& sh2) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  magic = (uint32_t)((((1ull << l) - d) << 32) / d + 1);
  sh1 = l < 1 ? l : 1;
  sh2 = l > 1 ? l - 1 : 0;
}

// A lane (32-record block) with many StatusUpdates in one round logs one dense
// record instead of single entries: u32 words [key lo, key hi (pack_update
// with the block's first target, slot 0, status 0), E_0 .. E_{k-1} (updated
// records per slot), A (final accepted plane), died (records deleted this
// round)], padded to whole u64 words; fetch expands it. Dense when its size
// is at most that of the singles: 8 * count >= 8 * dense_words(k).
__host__ __device__ constexpr uint32_t dense_words(uint32_t k) { return (k + 5u) / 2u; }  // u64 words
__host__ __device__ constexpr uint32_t dense_min(uint32_t k) { return dense_words(k); }   // updates

// Medium lane records (k = 8 round kernels, round_common.h emit_store_med), two formats:
//  * AVK_MED_S4 = 1 (default): a slot record of four u64 = u32 words [key lo, key hi (pack_update
//    with the block's first target, slot 0, status 0), S (bits 0-7: slots with updates; bit 8
//    kMedS4Died: the last word is the died plane), A (final accepted plane), E of the first, second,
//    third and fourth slot with updates (zero past the last; the fourth is the died plane when
//    flagged)]. Logged by a lane with >= 2 updates in at most 4 slots (at most 3 when a record of it
//    was deleted this round); other lanes with >= 2 updates log a dense record. Expanded as a dense
//    record over the slots S names.
//  * AVK_MED_S4 = 0: a lane with 2..kMedMax StatusUpdates in one round (k <= 8) logs one medium
// record of two u64: the key (pack_update with the block's first target, slot
// 0, status 0) and a payload: bits [3:0] = n updates, then n 10-bit fields at
// bit 4 + 10 i, each (slot << 7 | bit << 2 | status) = the update's offset
// from the key (expanded word = key + (slot << 24) + (bit << 2) + status).
#ifndef AVK_MED_S4
#define AVK_MED_S4 1
#endif
constexpr uint32_t kMedS4Died = 1u << 8;
__host__ __device__ constexpr uint32_t med_rec_words() { return AVK_MED_S4 ? 4u : 2u; }  // u64 per medium record
constexpr uint32_t kMedMax = 6;
__host__ __device__ constexpr uint32_t med_field(uint32_t slot, uint32_t bit, uint32_t status) {
  return (slot << 7) | (bit << 2) | status;
}
__host__ __device__ inline uint64_t med_word(uint64_t key, uint32_t f) {
  return key + ((uint64_t)(f >> 7) << 24) + ((uint64_t)((f >> 2) & 31u) << 2) + (f & 3u);
}

// Update-log entry (one StatusUpdate, avalanche.go:59-62):
//   [63:S] round - log_base | [S-1:28] node | [27:24] slot | [23:2] target | [1:0] status
// S = the engine's round shift: 28 + max(24, bits of N) (52 below 2^24 nodes, include/avhip.h).
// Ascending order of the packed word == canonical (round, node, slot, target).
__host__ __device__ inline uint64_t pack_update(uint32_t round_rel, uint32_t node, uint32_t slot,
                                                uint32_t target, uint32_t status, uint32_t round_shift) {
  return ((uint64_t)round_rel << round_shift) | ((uint64_t)node << 28) | ((uint64_t)slot << 24) |
         ((uint64_t)target << 2) | (uint64_t)status;
}

hipError_t launch_round(const RoundParams& p, int k, bool replay, bool capped, hipStream_t s);
// k_replay_node: p.fuse_rounds replay rounds of every node in one launch (capped engines, k <= 8);
// nodes that reach count 120 are left to the exact pass from that round on (node_flags)
hipError_t launch_replay_node(const RoundParams& p, int k, hipStream_t s);
// Persistent streaming round kernel (round_sweep.hip), uncapped path, k <= 8:
// `blocks` workgroups of 256 threads sweep the tiles; 0 = one wave per tile.
// ref_written (may be null): whether the launch wrote p.rflag_out (only the walking warm mode does)
hipError_t launch_round_sweep(const RoundParams& p, int k, bool replay, uint32_t blocks, hipStream_t s,
                              bool* ref_written = nullptr);
// Capped round (M > 4096, k <= 8; round_node.hip): one workgroup per node;
// nodes that may finalize a record this round are flagged in p.node_flags and
// left to the exact pass (k_round_capped over the flagged nodes only), which
// the caller may skip when no count can have reached 120 (exact_pass false).
hipError_t launch_round_node(const RoundParams& p, int k, bool replay, bool exact_pass, hipStream_t s);
// Resident 256-thread workgroups per CU for the sweep kernel and the CU count.
hipError_t round_sweep_occupancy(int k, bool replay, int* blocks_per_cu, int* cus);
// Write back the V planes of stale tiles (p.vstale, p.pref_prev, p.round = the
// round after the one that left them stale); k = 8 only.
hipError_t launch_vv_materialize(const RoundParams& p, hipStream_t s);
// Apply the pending +8 steps of deferred count planes (p.kpend) and clear them.
hipError_t launch_kl_materialize(const RoundParams& p, hipStream_t s);
// Both write-backs in one pass over runs of 16 tiles per wave (do_v: launch_vv_materialize's part,
// do_k: launch_kl_materialize's); tiles with nothing deferred are skipped with no memory access.
hipError_t launch_materialize(const RoundParams& p, bool do_v, bool do_k, hipStream_t s);

// Need-masked exchange: the rows each rank's nodes draw in the rounds of one window.
// need_draw: mine[w][N] = 1 for every row drawn by a local node in round round0 + w (w < W).
// need_push: the bits of mine for peer d's rows into peer d's needin[par][rank][w][NLw] (words).
// need_combine: needmask[w][nl] = the peers (push order) whose nodes draw local row nl in round
// round0 + w (ref_local: the reference row, read by every rank, is needed by all).
constexpr uint32_t kNeedWin = 16;  // rounds per need window
constexpr uint32_t kPushQ = 16;    // tiles per wave whose pushes the sweep queues in LDS
hipError_t launch_need_draw(uint64_t seed, uint32_t n_nodes, uint32_t n0, uint32_t NL, uint32_t round0, uint32_t W,
                            int k, int mode, uint8_t* mine, hipStream_t s);
hipError_t launch_need_push(const uint8_t* mine, uint32_t n_nodes, uint32_t NL, uint32_t W, uint32_t world,
                            uint32_t rank, uint32_t par, PeerPtrs needin, hipStream_t s);
hipError_t launch_need_combine(const uint32_t* needin, uint32_t world, uint32_t rank, uint32_t par, uint32_t W,
                               uint32_t NL, uint32_t ref_local, uint8_t* needmask, hipStream_t s);

// Peer-push exchange helpers (kernels.hip). push_rows: copy words [w0, w1) of
// a local snapshot buffer into the same range of every peer replica.
hipError_t launch_push_rows(const uint32_t* src, PeerPtrs dst, uint32_t n_dst, uint64_t w0, uint64_t w1,
                            hipStream_t s);
// Barrier across the ranks of a node-sharded network: lane i writes `seq`
// into slot `rank` of rank i's arrival array (arrive[i], system scope), then
// waits until every slot of its own array (arrive[rank]) has reached `seq`.
// Gives up after timeout_ticks of the wall clock and sets *err (later barriers then return at once).
hipError_t launch_peer_barrier(PeerPtrs arrive, uint32_t world, uint32_t rank, uint32_t seq, uint32_t* err,
                               uint64_t timeout_ticks, hipStream_t s, const uint32_t* slot = nullptr,
                               PeerPtrs slot_dst = PeerPtrs{}, uint32_t wait = 1u);
// (slot: this rank's uniform-rows mismatch slot of the snapshot the round wrote, copied into every
// peer's replica (slot_dst.p[i]: rank i's copy) before the arrival; wait = 0: no arrival and no wait
// (the serial peer group, whose stream order is the barrier))
// Wall-clock ticks of a timeout (the device's wall clock rate; queried once per engine).
hipError_t peer_timeout_ticks(int device, uint32_t timeout_ms, uint64_t* ticks);

struct InitParams {
  uint32_t* planes;
  uint32_t* pref;       // [N_pad][PS]
  const uint32_t* byz;
  uint64_t seed;
  uint32_t n_nodes, n0, NL, BL, PS, L, Lpad, t0, n_targets, round;
  int32_t mode;
  uint32_t param;
  uint32_t pub_mode;    // RoundParams::pub_mode
};
hipError_t launch_init(const InitParams& p, hipStream_t s);
hipError_t launch_byz(uint32_t* byz, uint32_t n_nodes, uint64_t seed, uint32_t threshold, hipStream_t s);

struct DropInParams {
  uint32_t* planes;
  uint32_t* pref;          // current published snapshot row for the node
  const uint32_t* valid;
  const uint32_t* byz;
  const uint32_t* blocks;  // touched lanes (local node * BL + block), each once; >= L: votes for unknown targets
  const uint32_t* offs;    // [n_blocks + 1] into entries
  const uint32_t* entries; // pairs (pos, meta = bit | yes<<5 | considered<<6)
  int8_t* status_out;      // per vote position, -1 = no update
  uint32_t n_blocks, n0, BL, PS, round, L;
  uint32_t pub_mode;
  // av_register_votes_batch's Responses (k_dropin_resp / k_dropin_keys): packed votes (dropin_word),
  // Response r = votes [resp_off[r], resp_off[r + 1]) of local node resp_node[r]
  const uint32_t* packed;
  const uint32_t* resp_off;
  const uint32_t* resp_node;
  uint32_t n_resp;
  // fast path: the Responses grouped by node (order = Response indices, stable by node; group i =
  // order[grp_off[i] .. grp_off[i + 1]))
  const uint32_t* order;
  const uint32_t* grp_off;
  uint32_t n_groups;
};
// A drop-in vote as the host packs it: the target's local index, "unknown hash" (outside this
// engine's targets: skipped, processor.go:95-99), err == 0 (yes) and int32(err) >= 0 (considered),
// vote.go:55-56.
constexpr uint32_t kDropUnknown = 1u << 29, kDropYes = 1u << 30, kDropCons = 1u << 31, kDropTl = (1u << 22) - 1u;
__host__ __device__ inline uint32_t dropin_word(int64_t tl, bool local, uint32_t err) {
  return (local ? (uint32_t)tl & kDropTl : kDropUnknown) | (err == 0u ? kDropYes : 0u) |
         ((int32_t)err >= 0 ? kDropCons : 0u);
}
hipError_t launch_register_votes(const DropInParams& p, hipStream_t s);
// Fast path of a batch whose Responses each have strictly ascending targets: one workgroup per node
// (its Responses in order), the first vote of each (node, block) run applies the run.
hipError_t launch_dropin_resp(const DropInParams& p, hipStream_t s);
// General path: per vote, the lane key (L for unknown targets), its index and the packed vote for
// launch_group_votes.
hipError_t launch_dropin_keys(const DropInParams& p, uint32_t* keys, uint32_t* vidx, uint32_t* info, hipStream_t s);

struct AddParams {
  uint32_t* planes;
  uint32_t* pref;
  const uint32_t* valid;
  const uint32_t* byz;
  const uint32_t* targets;  // local target index
  const uint8_t* accepted;
  uint8_t* added;
  uint32_t n, node_local, node, BL, PS, round;
  uint32_t pub_mode;
};
hipError_t launch_add_targets(const AddParams& p, hipStream_t s);

hipError_t launch_read_records(const uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1,
                               uint32_t tl0, uint32_t tl1, uint32_t* out, hipStream_t s);
// Canonical words without writing back deferred state (kernels.hip
// k_read_records_v): p = the engine's round parameters with p.vv = "some tile
// may be stale" and p.klazy = "some tile may hold pending count steps".
hipError_t launch_read_records_virtual(const RoundParams& p, uint32_t nl0, uint32_t nl1, uint32_t tl0, uint32_t tl1,
                                       uint32_t* out, hipStream_t s);

// Device-side StatusUpdate delivery (log_ops.hip).
// Digest {count, sum, xor} of splitmix64(packed word) over every pending update
// of nodes [node0, node1).
hipError_t launch_log_digest(const uint64_t* log, const uint32_t* counts, uint32_t cap, const uint64_t* dlog,
                             const uint32_t* dcounts, uint32_t dcap, const uint64_t* mlog, const uint32_t* mcounts,
                             uint32_t mcap, uint32_t shards, uint32_t k, uint32_t node0, uint32_t node1,
                             uint32_t round_shift, unsigned long long* out, hipStream_t s);
// Canonical order of the pending StatusUpdates (log_ops.hip): a counting sort by (round, node) bucket
// for rounds [r0, r0 + nr) of the log (round_rel < r_total), then one wave per bucket writing its
// updates in (slot, target) order, as packed words (out + ubase + the bucket's update offset) or as
// compact groups (cout + cbase + its byte offset; index entries into cidx). Reads the log counters on
// the device. totals (device, may be null): this pass's updates, compact bytes, entries.
struct EncodeParams {
  const uint64_t* log;
  const uint64_t* mlog;
  const uint64_t* dlog;
  const uint32_t* log_count;  // [3][kLogShards][kCtrStride]: singles, slot records, dense records
  uint32_t log_cap, mlog_cap, dlog_cap, shards;
  uint32_t K, n0, NL, BL, t0;
  uint32_t r0, nr, r_total;
  uint32_t round_shift;  // the update words' round field (pack_update); node = bits [28, round_shift)
  uint32_t code_bytes, target_bits;  // compact codes: slot << (target_bits + 2) | local target << 2 | status
  uint32_t* err;  // bit 0: an entry outside the engine's nodes / rounds; bit 1: a bucket's count mismatch
};
uint64_t encode_scratch_bytes(const EncodeParams& p, uint64_t entries, uint32_t buckets);
hipError_t launch_encode_log(const EncodeParams& p, uint64_t entries, void* scratch, uint64_t* out, uint8_t* cout,
                             uint64_t* cidx, uint32_t chunks, uint32_t chunk_nodes, uint64_t ubase, uint64_t cbase,
                             bool last_pass, uint64_t* totals, hipStream_t s);
// Copy bytes (rounded up to 16; both buffers 16-B aligned and that large) from device memory into
// host-mapped pinned memory with `blocks` workgroups (k_stream_out).
hipError_t launch_stream_out(const void* src, void* dst, uint64_t bytes, uint32_t blocks, hipStream_t s);
// diagnostics: read `bytes` of src once (log_ops.hip k_touch)
hipError_t launch_touch(const void* src, uint64_t bytes, uint32_t* sink, hipStream_t s);
// Drop-in batch grouping: stable radix sort of (lane key, position) into (keys_s, perm_s) (keys_t,
// perm_t: the other buffer set), run-length encoding into lanes / offs (n_runs + 1) / *n_runs, and the
// (vote index, packed vote) entries in grouped order. scratch: group_votes_scratch_words(n) u64.
uint64_t group_votes_scratch_words(uint32_t n);
hipError_t launch_group_votes(uint64_t* scratch, const uint32_t* keys, const uint32_t* vidx, const uint32_t* info,
                              uint32_t n, int key_bits, uint32_t* keys_s, uint32_t* perm_s, uint32_t* keys_t,
                              uint32_t* perm_t, uint32_t* lanes, uint32_t* offs, uint32_t* n_runs, uint32_t* entries,
                              hipStream_t s);

hipError_t launch_write_records(uint32_t* planes, uint32_t BL, uint32_t nl0, uint32_t nl1, uint32_t tl0,
                                uint32_t tl1, const uint32_t* in, hipStream_t s);
// After a round with the example's responder (pub_mode 2): re-create the
// records queried this round that their responder did not hold.
hipError_t launch_readd(const RoundParams& p, hipStream_t s);
hipError_t launch_refresh_pref(uint32_t pub_mode, const uint32_t* planes, uint32_t* pref, const uint32_t* byz,
                               uint32_t n0, uint32_t NL, uint32_t BL, uint32_t PS, uint32_t round, hipStream_t s);
hipError_t launch_sample_peers(uint64_t seed, uint32_t n_nodes, uint32_t a, uint32_t b, uint32_t round,
                               int k, int mode, uint32_t* out, hipStream_t s);
hipError_t launch_gen_replay(uint64_t seed, uint32_t n0, uint32_t NL, uint32_t BL, uint32_t L, uint32_t Lpad,
                             uint32_t t0, uint32_t n_targets, uint32_t round, int k, uint32_t* out,
                             hipStream_t s);
hipError_t launch_count_live(const uint32_t* planes, const uint32_t* valid, const uint32_t* byz, uint32_t n0,
                             uint32_t BL, uint32_t L, int honest_only, unsigned long long* out, hipStream_t s);
// Batched poll sets (GetInvsForNextPoll of nodes [nl0, nl0 + n)): the per-node counts, their device
// scan into offsets (n + 1, u64) and the CSR targets in one stream-ordered sequence; entries at or past
// cap are not written. offs_out / targets_out may be host-mapped pinned memory (hipHostGetDevicePointer):
// the fill kernel's stores are coalesced. scratch: poll_sets_scratch_words(n) u64.
uint64_t poll_sets_scratch_words(uint32_t n);
hipError_t launch_poll_sets_batch(const uint32_t* planes, const uint32_t* valid, uint32_t BL, uint32_t nl0,
                                  uint32_t n, uint32_t t0, uint64_t cap, uint64_t* scratch, int64_t* offs_out,
                                  int32_t* targets_out, hipStream_t s);

}  // namespace avk
