/*
 * avhip.h — C ABI of libavhip.so, the MI355X-native batched Avalanche voting
 * engine (drop-in for go-avalanche's Processor/VoteRecord hot path).
 *
 * One engine = the VoteRecord state of a network of N simulated nodes x M
 * targets (or one shard of it) held in HBM. Every function is plain C: opaque
 * handle, plain pointers and sizes, int status codes, caller-owned host
 * buffers that are not retained after the call returns (the cgo rule).
 * Calls on one handle must be serialized by the caller (the reference
 * Processor is not thread-safe either: processor.go:12-25, main.go:101,122,135).
 *
 * Reference interfaces replaced (itsdevbear/go-avalanche):
 *   av_add_targets      <- (*Processor).AddTargetToReconcile   processor.go:45-58
 *   av_register_votes   <- (*Processor).RegisterVotes           processor.go:61-122
 *   av_register_votes_batch <- RegisterVotes of many Responses /  processor.go:61-122, main.go:136
 *                          Processors in one call
 *   av_is_accepted      <- (*Processor).IsAccepted              processor.go:125-130
 *   av_get_confidence   <- (*Processor).GetConfidence           processor.go:133-140
 *   av_get_invs         <- (*Processor).GetInvsForNextPoll      processor.go:144-170
 *   av_get_invs_batch   <- GetInvsForNextPoll of many Processors processor.go:144-170
 *   av_get_round        <- (*Processor).GetRound                processor.go:40-42
 *   av_set_round        <- the caller's `p.round = ...`          avalanche_test.go:302 (Processor.round is a
 *                          field nothing in the Processor advances: processor.go:15,40-42)
 *   av_set_valid        <- Target.IsValid / isWorthyPolling     avalanche.go:89-90, processor.go:185-187
 *   av_run_rounds       <- the example's poll loop for every node at once
 *                          (main.go:110-137 + responder main.go:168-192,
 *                          peers from getSuitableNodeToQuery processor.go:173-182
 *                          / Connman.NodesIDs net.go:25-31 replaced by
 *                          counter-RNG k-peer sampling)
 *   av_fetch_updates    <- the *[]StatusUpdate out-parameter     processor.go:61,111
 *                          (device-side canonical ordering: counting sort by
 *                          (round, node) + per-node (slot, target) layout)
 *   av_fetch_compact[_async/_wait], av_compact_expand <- the same out-parameter
 *                          as a compact stream (~2 B per update), pipelined
 *                          with the next rounds
 */
#ifndef AVHIP_H
#define AVHIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AVHIP_ABI_VERSION 1

/* return codes */
#define AV_OK 0
#define AV_ERR_INVALID_ARG (-1)
#define AV_ERR_HIP (-2)
#define AV_ERR_OOM (-3)
#define AV_ERR_NOT_FOUND (-4)   /* GetConfidence's panic("VoteRecord not found") */
#define AV_ERR_OVERFLOW (-5)    /* update log or caller buffer too small */
#define AV_ERR_UNSUPPORTED (-6)
#define AV_ERR_RCCL (-7)
#define AV_ERR_PEER (-8)        /* peer-push exchange broken (a rank missed a barrier); sticky */

/* Status (avalanche.go:42-56, iota order) */
#define AV_STATUS_INVALID 0
#define AV_STATUS_REJECTED 1
#define AV_STATUS_ACCEPTED 2
#define AV_STATUS_FINALIZED 3

#define AV_FINALIZATION_SCORE 128  /* avalanche.go:10 */
#define AV_MAX_ELEMENT_POLL 4096   /* avalanche.go:17 */

/* peer selection for av_run_rounds */
#define AV_PEERS_RANDOM 0      /* k distinct uniform peers != self, Philox4x32-10 */
#define AV_PEERS_ROUND_ROBIN 1 /* the example's i % N skipping self (main.go:110-116) */

/* bulk population for av_init_records */
#define AV_INIT_NONE 0      /* no records; add them with av_add_targets */
#define AV_INIT_REJECTED 1  /* every node adds every target, IsAccepted() = false */
#define AV_INIT_ACCEPTED 2  /* ... IsAccepted() = true */
#define AV_INIT_BERNOULLI 3 /* IsAccepted() = philox(node, t) < init_param */
#define AV_INIT_PAIRS 4     /* double-spend pairs (2p, 2p+1), complementary per node */

/* Canonical record word used by av_read_records / av_write_records:
 *   live record : votes | consider << 8 | confidence << 16  (vote.go:25-29,
 *                 confidence >> 1 < 128)
 *   no record   : 0xFFFE0000 | decision << 16  (deleted after finalization,
 *                 processor.go:114-116, or never added; decision = 1 iff the
 *                 record finalized accepted) */
#define AV_ABSENT_WORD 0xFFFE0000u

typedef struct av_engine av_engine;

typedef struct {
  int64_t n_nodes;       /* N, whole network (< 2^30) */
  int64_t n_targets;     /* M, whole network (target slots 0..M-1) */
  int32_t k;             /* polls (Responses) per node per round, 1..16 */
  int32_t peer_mode;     /* AV_PEERS_* */
  uint64_t seed;         /* Philox key for peers / Byzantine set / init */
  uint32_t byz_threshold;/* node j Byzantine iff philox(j) < threshold (0 = none) */
  int32_t device;        /* HIP device ordinal */
  int64_t node_begin;    /* this engine's node shard [node_begin, node_end) */
  int64_t node_end;      /*   (0,0 = all nodes) */
  int64_t target_begin;  /* this engine's target shard [target_begin, target_end), */
  int64_t target_end;    /*   begin a multiple of 32 (0,0 = all targets) */
  int64_t update_log_capacity; /* device StatusUpdate log entries (0 = default) */
} av_config;

/* Packed StatusUpdate as returned by av_fetch_updates (uint64):
 *   [63:S] round - round of the previous fetch | [S-1:28] node |
 *   [27:24] slot (poll index within the round)  | [23:2] target | [1:0] status
 * S = the engine's round shift (av_update_round_shift): 52 for networks of
 * fewer than 2^24 nodes, 28 + ceil(log2 N) above (the node field widens, the
 * round field narrows: a log then spans at most 2^(64 - S) rounds).
 * Sorted ascending == (round, node, slot, target) == reference append order.
 * The first helpers take S; the short forms assume S = 52. */
static inline int64_t av_update_round_rel_s(uint64_t u, int32_t s) { return (int64_t)(u >> s); }
static inline int64_t av_update_node_s(uint64_t u, int32_t s) {
  return (int64_t)((u >> 28) & ((1ull << (s - 28)) - 1ull));
}
static inline int64_t av_update_round_rel(uint64_t u) { return av_update_round_rel_s(u, 52); }
static inline int64_t av_update_node(uint64_t u) { return av_update_node_s(u, 52); }
static inline int32_t av_update_slot(uint64_t u) { return (int32_t)((u >> 24) & 0xFu); }
static inline int64_t av_update_target(uint64_t u) { return (int64_t)((u >> 2) & 0x3FFFFFu); }
static inline int32_t av_update_status(uint64_t u) { return (int32_t)(u & 3u); }

/* ---- lifecycle ---- */
int av_abi_version(void);
void av_config_init(av_config* cfg);
int av_create(const av_config* cfg, av_engine** out);
int av_destroy(av_engine* e);
const char* av_strerror(int code);
const char* av_last_error(void); /* thread-local detail of the last failure */

/* ---- population (processor.go:45-58) ---- */
/* AddTargetToReconcile of every target for every local node (a fresh network:
 * NewVoteRecord, vote.go:33-35) with the initial acceptance of init_mode. On a
 * peer-push engine (av_peer_init) this is collective: every rank calls it, and
 * the new rows reach every peer replica before the next round. */
int av_init_records(av_engine* e, int32_t init_mode, uint32_t init_param);
/* AddTargetToReconcile for targets[0..n) of one node, in order;
 * added[i] = 1 iff a record was created (false if !IsValid or live record). */
int av_add_targets(av_engine* e, int64_t node, const int64_t* targets, const uint8_t* accepted, int64_t n,
                   uint8_t* added);
/* Target.IsValid() of a target for every node (isWorthyPolling, processor.go:101).
 * Validity is per target (per Hash), shared by every node of the engine: the
 * reference keeps, per Processor, the Target object it was given
 * (processor.go:55) and asks it IsValid() at vote time (:101), so two
 * Processors holding different Target objects under one Hash could disagree.
 * This engine cannot represent that case ("Validity"). */
int av_set_valid(av_engine* e, int64_t target, int32_t valid);

/* ---- one-node Processor methods (drop-in path) ---- */
/* RegisterVotes: votes (targets[i], errs[i]) applied in order. status_out[i] =
 * Status of the StatusUpdate that vote appended, or -1 if none. Unknown
 * targets (< 0 or >= M) and targets outside this shard are skipped as the
 * reference skips unknown hashes. Always returns AV_OK on valid input
 * (RegisterVotes returns true: processor.go:121). */
int av_register_votes(av_engine* e, int64_t node, const int64_t* targets, const uint32_t* errs, int64_t n,
                      int32_t* status_out);
/* RegisterVotes for many Responses in one call (processor.go:61-122 once per
 * Response, as main.go:136 calls it): Response i is registered by node
 * nodes[i] with the votes offsets[i] .. offsets[i+1]-1 of targets/errs, in
 * order; a node may appear several times (its Responses apply one after the
 * other). status_out[v] as for av_register_votes.
 * Limits of both drop-in calls: AV_ERR_UNSUPPORTED on an engine (shard) with
 * more than 4M (2^22) local targets (a packed vote carries a 22-bit local
 * target index), AV_ERR_INVALID_ARG for >= 2^31 votes or Responses in one call. */
int av_register_votes_batch(av_engine* e, int64_t n_resp, const int64_t* nodes, const int64_t* offsets,
                            const int64_t* targets, const uint32_t* errs, int32_t* status_out);
int av_is_accepted(av_engine* e, int64_t node, int64_t target, int32_t* out);
/* AV_ERR_NOT_FOUND where the reference panics "VoteRecord not found". */
int av_get_confidence(av_engine* e, int64_t node, int64_t target, uint16_t* out);
/* Live valid targets in ascending index, truncated to 4096. */
int av_get_invs(av_engine* e, int64_t node, int64_t* out_targets, int64_t cap, int64_t* n_out);
/* GetInvsForNextPoll for every local node in [n0, n1) at once (device
 * compaction): node n's poll set is targets[offsets[n-n0] .. offsets[n-n0+1])
 * (offsets: n1-n0+1 entries). AV_ERR_OVERFLOW with *total = the required size
 * if cap is too small. */
int av_get_invs_batch(av_engine* e, int64_t n0, int64_t n1, int64_t* offsets, int32_t* targets, int64_t cap,
                      int64_t* total);

/* ---- batched rounds: the hot path ---- */
/* Enqueue `rounds` synchronous rounds: each node polls
 * k peers; votes = peers' round-start published preference. Asynchronous. */
int av_run_rounds(av_engine* e, int32_t rounds);
/* One replayed round: errs is a HOST array [local nodes][k][local targets]
 * of err words (vote.go:55-56 classes), consumed for the polled targets. */
int av_replay_round_errs(av_engine* e, const uint32_t* errs);
/* Synthetic replayed stream (C2 workload): generate the vote classes of the
 * next `rounds` rounds on the device (avo_replay_err definition) ... */
int av_replay_prepare(av_engine* e, int32_t rounds);
/* ... and consume them (asynchronous). On engines where the 4096 poll cap
 * binds (M > 4096) consecutive replay rounds run fused, up to option
 * "replay_fuse" (16) per launch: every node's records depend only on its own
 * stream, so a workgroup carries them through the rounds in registers; nodes
 * that reach count 120 continue in the per-round exact pass. Results are
 * identical to one launch per round (tests/test_gpu_replay_fused.py). */
int av_replay_rounds(av_engine* e, int32_t rounds);
int av_synchronize(av_engine* e);
/* Batched rounds run so far (the engine's round counter: the RNG counter of
 * the peer draw, R1). Not the reference's GetRound: see av_get_round. */
int av_round_index(av_engine* e, int64_t* out);
/* Processor.GetRound of one node (processor.go:40-42): a per-Processor field
 * that only its owner changes (the reference test sets it, avalanche_test.go:
 * 302); 0 until av_set_round. Not advanced by rounds. */
int av_get_round(av_engine* e, int64_t node, int64_t* out);
/* Whether `node` polls in the batched rounds (default 1). The example's run
 * loop returns once the node counted every tx finalized (main.go:143-162);
 * such a node still answers queries. Rounds with non-polling nodes run the
 * first-generation kernel; not on peer-push engines. */
int av_set_polling(av_engine* e, int64_t node, int32_t polls);
int av_set_round(av_engine* e, int64_t node, int64_t round);

/* ---- outputs ---- */
int av_updates_count(av_engine* e, int64_t* n);
/* Whether the device StatusUpdate log overflowed since the last fetch/discard
 * (the next av_fetch_updates will then fail with AV_ERR_OVERFLOW). */
int av_update_log_overflowed(av_engine* e, int32_t* out);
/* All StatusUpdates since the previous fetch, sorted canonical; clears the
 * log. AV_ERR_OVERFLOW if the device log or `cap` overflowed (*n_out holds the
 * required count when cap is too small). */
int av_fetch_updates(av_engine* e, uint64_t* out, int64_t cap, int64_t* n_out);
/* The round the pending log's round fields count from (the engine round at
 * the last fetch/discard): round of a fetched word = this + av_update_round_rel. */
int av_log_base_round(av_engine* e, int64_t* out);
/* The engine's update-word round shift S (see the packed StatusUpdate above). */
int av_update_round_shift(av_engine* e, int32_t* out);

/* ---- compact StatusUpdate stream (the same updates as av_fetch_updates, in the
 * same canonical order, ~2 B per update instead of 8; processor.go:61,111) ----
 * Layout (little-endian):
 *   av_compact_header (80 B)
 *   index: n_rounds * chunks + 1 entries of {uint64 byte offset of the entry's
 *          first group from the start of the groups, uint64 updates before it};
 *          entry r * chunks + c covers the groups of round log_base + r and
 *          nodes [node_base + c * chunk_nodes, node_base + (c + 1) * chunk_nodes)
 *   groups: one per (round, node) with >= 1 update, ascending (round, node):
 *          uint32 node (global id), uint32 count, then count codes of
 *          code_bytes each in (slot, target) order, zero-padded to 4 B;
 *          code = slot << (target_bits + 2) | (target - target_base) << 2 | status
 * av_compact_expand turns a stream back into av_fetch_updates' packed words. */
#define AV_COMPACT_MAGIC 0x31435641u /* "AVC1" */
#define AV_COMPACT_VERSION 1
typedef struct {
  uint32_t magic;
  uint32_t version;
  int64_t log_base;     /* round of the stream's round 0 */
  int64_t n_updates;
  int64_t bytes;        /* whole stream, header included */
  int64_t node_base;
  int64_t target_base;
  int32_t n_rounds;
  int32_t chunks;       /* index entries per round */
  int32_t chunk_nodes;
  int32_t code_bytes;   /* 2 or 4 */
  int32_t target_bits;
  int32_t slot_bits;
  int32_t round_shift;  /* of the expanded words (av_update_round_shift) */
  int32_t reserved;
} av_compact_header;
/* Every pending update as a compact stream into out (cap bytes), clearing the
 * log; AV_ERR_OVERFLOW with *bytes = the size needed (log kept) if cap is too
 * small. */
int av_fetch_compact(av_engine* e, void* out, int64_t cap, int64_t* bytes);
/* Pipelined delivery: encode every pending update on the device (waiting for
 * the rounds enqueued before), start its copy into engine-owned pinned host
 * memory on a copy stream, clear the log and return at once with a ticket; the
 * caller enqueues the next rounds while the copy runs. av_fetch_compact_wait
 * blocks until that copy landed and returns the stream (engine memory, valid
 * until the av_fetch_compact_async call three tickets later or av_destroy), so a
 * consumer may read one stream while the next two are encoded and copied. At
 * most three tickets are outstanding: the fourth call waits for the oldest copy. */
int av_fetch_compact_async(av_engine* e, int64_t* ticket);
int av_fetch_compact_wait(av_engine* e, int64_t ticket, const void** stream, int64_t* bytes);
/* Host-side expansion of a compact stream into packed update words (the
 * av_fetch_updates form; round fields relative to the header's log_base),
 * multi-threaded. AV_ERR_OVERFLOW with *n_out = the count if cap is too small;
 * AV_ERR_INVALID_ARG for a malformed stream. */
int av_compact_expand(const void* stream, int64_t bytes, uint64_t* out, int64_t cap, int64_t* n_out);
/* Order-independent digest of every pending StatusUpdate without fetching
 * (or clearing) them: out = {count, sum, xor} of splitmix64(packed word).
 * AV_ERR_OVERFLOW if the log overflowed. Full-size parity checks compare it
 * with the oracle's digest of the same round. */
int av_updates_digest(av_engine* e, uint64_t out[3]);
/* The same over the updates of nodes [n0, n1) only. */
int av_updates_digest_range(av_engine* e, int64_t n0, int64_t n1, uint64_t out[3]);
/* Number of regsiterVote applications (vote.go:54) since creation. */
int av_applied_votes(av_engine* e, int64_t* out);
/* Records deleted after finalization by round kernels since creation. */
int av_finalized_count(av_engine* e, int64_t* out);
/* Live valid records now (honest_only: skip Byzantine nodes). */
int av_live_records(av_engine* e, int32_t honest_only, int64_t* out);
/* Drop pending StatusUpdates without copying them (long convergence runs). */
int av_discard_updates(av_engine* e);
/* Log entries pending, per kind: out = {single updates, slot records (2-4
 * slots of one 32-record lane), dense records (a lane's whole round)}; a
 * lane's updates of one round are one slot or dense record, or (k = 8 sweep
 * rounds: at most two updates) one or two single words. Sizing input for
 * av_resize_log. */
int av_log_entries(av_engine* e, int64_t out[3]);
/* Re-allocate the (empty: AV_ERR_UNSUPPORTED otherwise) device log for about
 * entries[k] entries of each kind (8, 32 and 48 B each at k = 8), instead of
 * av_config.update_log_capacity's worst case per update (36 B per update).
 * The log is sharded by the round kernel's writer waves: each writer wave gets
 * ceil(entries[k] / writers) + 1 entries, i.e. the sizing assumes the entries
 * are spread evenly over the writers. That holds for entries = {2, 1, 1} x the
 * lane count (one round never needs more than two single words or one record
 * per lane); a
 * measured count with skewed emission can overflow one shard while the total
 * stays below entries[k] — the overflow is detected (av_update_log_overflowed,
 * AV_ERR_OVERFLOW on fetch), never silent. */
int av_resize_log(av_engine* e, const int64_t entries[3]);
/* Algorithmic bytes moved by the round kernels since creation: state planes
 * read/written, gathered vote words, published words, 8 B per StatusUpdate
 * (DESIGN.md §3). */
int av_alg_bytes(av_engine* e, int64_t* out);
/* The part of av_alg_bytes that re-reads a published preference word another
 * lane already gathered in the same round (k_round_sweep: 28 B of the 8 peer
 * words per lane, 24 B of a stale tile's 7 regathered words). av_alg_bytes
 * minus this = the compulsory bytes (every word read or written once), a lower
 * bound on HBM traffic. Diagnostics; no reference counterpart. */
int av_alg_bytes_reread(av_engine* e, int64_t* out);
/* Published preference words that changed in sweep rounds since creation: a
 * word differs from the word of the snapshot buffer it overwrites (the snapshot
 * of two rounds before, which every peer replica holds). Counted in every round
 * of a peer-push engine (= the words pushed to each peer) and,
 * with option "count_changed" = 1, in every sweep round of any engine.
 * segments (may be null): the 64-B row segments holding a changed word (16
 * consecutive words of a row; exact when the rows are 16 or 32 words wide).
 * Diagnostics; no reference counterpart. */
int av_changed_words(av_engine* e, int64_t* words, int64_t* segments);
/* Write back the engine's deferred state (stale vote planes, pending count
 * steps: DESIGN.md §3) now instead of at the next access that needs it. Every
 * result is the same either way; timed as one launch when timing is on.
 * Engine maintenance; no reference counterpart. */
int av_materialize(av_engine* e);
/* Canonical words for local nodes [n0,n1) x targets [t0,t1) (global ids). */
int av_read_records(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, uint32_t* out);
int av_write_records(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, const uint32_t* in);
/* Round-start published preference (0/1) for nodes [n0,n1) x targets [t0,t1). */
int av_read_pref(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, uint8_t* out);
/* Round-start published preference rows of nodes [n0,n1) as stored: [n][BL]
 * u32 bitsets of this engine's target range (bit t % 32 of word t / 32). */
int av_read_pref_words(av_engine* e, int64_t n0, int64_t n1, uint32_t* out);
/* Device peer sampling dump: peers of nodes [n0,n1) in round `round`, [n][k]. */
int av_sample_peers(av_engine* e, int64_t round, int64_t n0, int64_t n1, int32_t* out);

/* ---- tuning ----
 * "plane_nt"  (0/1): stream the state planes with non-temporal loads/stores.
 * "warm_skip" (0)  : disable skipping all-ones consider planes (A/B only).
 * "kernel"    (1/2): round kernel for the uncapped path: 2 = persistent sweep
 *                    (default, k <= 8), 1 = one wave per tile (A/B only).
 * "sweep_blocks"   : workgroups of the sweep grid (0 = one wave per tile,
 *                    -1 = the engine's choice (default), -2 = every resident
 *                    workgroup once, walking the tiles).
 * "store_policy"   : 2 = write-through (sc1) plane stores, 3 = nt sc1 (A/B).
 * "peer_fine" (0/1): snapshot buffers fine-grained once exported (default 1;
 *                    set before av_peer_handles).
 * "barrier_timeout_ms": peer barrier timeout (default 30000).
 * "responder" (0/1/2): what a node publishes for a target it no longer holds
 *                    (what its responder answers, main.go:168-192): 0 = the
 *                    finalized decision (harness rule R2, default); 1 =
 *                    IsAccepted literally, false after deletion
 *                    (processor.go:125-130); 2 = the example's responder,
 *                    which re-adds a queried target it does not hold as
 *                    accepted and answers yes (main.go:175-182; unsharded
 *                    engines, M <= 4096). 1 and 2 run the first-generation
 *                    kernel.
 * Sweep-kernel tuning and A/B switches (defaults are the measured best;
 * DESIGN.md §3-4): "tiles_per_wave" (0 = by size: 16 at BL <= 8; else the
 * longest of 16 / 8 / 4 with at most BL tiles that keeps >= 15000 waves;
 * node shards of an exchange of >= 4 ranks at BL >= 16: 16), "wave_runs" (1: a wave takes a run
 * of consecutive tiles and draws their peers once), "settled_fast" (1),
 * "sweep_nopipe" (1), "virtual_votes" (1), "vv_min_bl" (16), "count_lazy"
 * (1), "fresh" (1), "dense_min" (6 at k = 8: updates per lane that make a
 * dense log record), "ref_rows" (0; 1: in converged sweep rounds a settled
 * tile whose 8 peers published the reference node's row reads that row once
 * instead of gathering 8 copies of it; exact, measured slower), "replay_fuse" (16: replay
 * rounds per k_replay_node launch on capped engines, <= 1 = one launch per
 * round), "uni_merge" (1: runs per wave in a round with a uniform input),
 * "tile_draw" (0; 1: runs whose nodes overflow the run's peer draw share one
 * draw per tile; exact, measured level), "materialize_run" (1: tiles per wave
 * of the deferred state's write-back), "pref_uncached" (0; 1: snapshot
 * buffers in uncached memory; exact, measured slower), "peer_mask" (1:
 * need-masked peer pushes; set before the exchange), "push_defer" (1: a
 * wave's pushes queued in LDS and issued after its tiles), "peer_fine" (1),
 * "uni_votes" (1: in a round whose input snapshot is uniform, every tile takes
 * the reference word as its votes instead of gathering them; exact),
 * "wave_dense" (0; n: a wave with >= n lanes holding updates logs them all as
 * dense records; exact, measured slower).
 * StatusUpdate delivery: "enc_buckets" (2^26: (round, node) buckets per
 * encoder pass; a log spanning more takes several passes), "copy_blocks" (0:
 * the compact stream's copy to host memory by the runtime's copy; n: by an
 * n-workgroup copy kernel; measured slower).
 * Diagnostics that make results invalid: "ablate_gather",
 * "ablate_emit" (StatusUpdates counted, not stored), "ablate_node"
 * (k_round_node: 1 = lanes past the cap skipped, 4 = no plane stores),
 * "unsynced_shard". Diagnostics that leave results valid: "count_changed"
 * (1: count changed published words in every sweep round, av_changed_words),
 * "solo_barrier" (1: a one-rank peer barrier after every round of an engine
 * without an exchange: the barrier's fixed cost alone), "warm_pref" (1: the
 * snapshots a sweep round gathers from are read once, untimed, before its
 * timed kernel: the cache state of a GPU of its own, tools/group_model.py). */
int av_set_option(av_engine* e, const char* name, int64_t value);

/* ---- measurement ---- */
/* HIP-event timing of every round kernel launch on the engine stream. */
int av_set_timing(av_engine* e, int32_t enable);
int av_kernel_stats(av_engine* e, double* total_ms, int64_t* launches);
/* Bytes per round of the round kernel's algorithmic traffic. */
int av_layout_info(av_engine* e, int64_t* lanes, int64_t* local_nodes, int64_t* local_blocks, int32_t* capped);

/* ---- multi-GPU (node-sharded engines exchange preferences over RCCL) ---- */
int av_comm_unique_id(uint8_t out[128]);
int av_comm_init(av_engine* e, int32_t world, int32_t rank, const uint8_t id[128]);

/* ---- multi-GPU, peer-push exchange (node-sharded engines; replaces the
 * per-round all-gather above). Same network split as av_comm_init. Each rank
 * exports IPC handles of its preference snapshots (av_peer_handles), the
 * caller exchanges the blobs (any host collective), and av_peer_init maps every
 * peer's buffers. A round then stores only the published words that changed
 * straight into every peer's replica (the responder of main.go:168-192 answers
 * from IsAccepted, processor.go:125-130, of the round-start snapshot), followed
 * by a device-side barrier across the ranks. Collective: every rank must make
 * the same calls. Record writes outside a round (av_add_targets,
 * av_register_votes, av_write_records) return AV_ERR_UNSUPPORTED on such an
 * engine. */
#define AV_PEER_HANDLE_BYTES 320  /* 4 IPC handles + the device's PCI bus id */
int av_peer_handles(av_engine* e, uint8_t out[AV_PEER_HANDLE_BYTES]);
/* handles: world * AV_PEER_HANDLE_BYTES bytes, rank-ordered (this rank's own blob is ignored) */
int av_peer_init(av_engine* e, int32_t world, int32_t rank, const uint8_t* handles);
/* One-device rehearsal and measurement harness of the peer-push exchange: the
 * `world` node-shard engines of one network (engines[r] = rank r, created in
 * this process on one device, same configuration, same round) become one peer
 * group sharing one stream. Each rank's round kernel pushes into the others'
 * buffers exactly as over IPC; the stream's order (round r of every rank in
 * rank order, then round r + 1) replaces the device barrier, so per-rank
 * kernel times are those of a rank alone on the device. A rank may run a round
 * only when every lower rank has run it and no higher rank has
 * (AV_ERR_UNSUPPORTED otherwise). The snapshot buffers are made fine-grained
 * as av_peer_handles makes them (option "peer_fine", default 1). Destroy the
 * group's engines together: once one is destroyed, the others' rounds, pushes
 * and syncs return AV_ERR_UNSUPPORTED. */
int av_peer_group_serial(av_engine** engines, int32_t world);
/* Need-masked exchange (option "peer_mask", default on for 2..9 ranks when a
 * row's 32-word segments never straddle a wave: BL a power of two <= 32 or a
 * multiple of 32): a round sends a changed row segment only to
 * the ranks whose nodes draw that row in the next round (R1's sampling is a
 * function of (seed, node, round), so every rank draws its own nodes' rows of
 * a 16-round window ahead and tells their owners), and later sends whatever it
 * withheld once that rank needs the row. Every result is the same as with full
 * pushes; a rank's replica of another rank's rows can then hold rows no local
 * node reads: av_read_pref / av_read_pref_words of another rank's rows are
 * current only after av_peer_sync. Collective: every rank's own rows of the
 * current snapshot pushed whole to every replica, then a barrier. */
int av_peer_sync(av_engine* e);
/* Words stored into peer replicas by sweep rounds since creation, summed over
 * the peers (the exchange's volume; diagnostics, no reference counterpart). */
int av_pushed_words(av_engine* e, int64_t* out);

#ifdef __cplusplus
}
#endif
#endif
