// libavhip.so — C ABI (include/avhip.h) over the CDNA4 kernels in kernels.hip.
//
// The engine owns all device memory: the bit-sliced VoteRecord planes, the two
// published-preference snapshots, validity / Byzantine bitsets, the sharded
// StatusUpdate log and the applied-vote counters. Host buffers passed in are
// only read or written for the duration of the call.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "../../include/avhip.h"
#include "kernels.h"

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

#define AV_HIP(call)                                                                                    \
  do {                                                                                                  \
    hipError_t _e = (call);                                                                             \
    if (_e != hipSuccess) return fail(AV_ERR_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(_e), \
                                      __FILE__, __LINE__);                                              \
  } while (0)

#define AV_CHECK(cond, code, ...) \
  do {                            \
    if (!(cond)) return fail(code, __VA_ARGS__); \
  } while (0)

template <typename T>
hipError_t dev_alloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
}

}  // namespace

struct av_engine;
// An in-process peer group (av_peer_group_serial): the ranks of a node-sharded network as engines of
// one process on one device, sharing one stream; its order replaces the device barrier.
struct PeerGroup {
  std::vector<av_engine*> members;  // by rank; nullptr once destroyed
  hipStream_t stream = nullptr;
  int alive = 0;
};

struct av_engine {
  av_config cfg{};
  int64_t N = 0, M = 0, n0 = 0, n1 = 0, t0 = 0, t1 = 0;
  uint32_t NL = 0, BL = 0, L = 0, Lpad = 0;
  int k = 0;
  bool capped = false;
  hipStream_t stream = nullptr;
  uint32_t* planes = nullptr;
  // published-preference snapshots, rotated by 3: round r reads pref[cur]
  // (S_r) and writes pref[nxt(cur)] (S_r+1); pref[prv(cur)] (S_r-1) is kept
  // for tiles whose vote planes are recomputed (vstale)
  uint32_t* pref[3] = {nullptr, nullptr, nullptr};
  // words per node row of the preference tables: BL rounded up to a power of two (BL <= 32) or to a
  // multiple of 32 (BL > 32), so that a gathered row covers whole 128-B lines (avk::pref_stride)
  uint32_t PS = 0;
  // reference rows (kernels.h ref_node / rflag_*): one flag byte per node after the preference words
  // of every snapshot buffer (so rotation, IPC export and peer pushes carry them); rflag_ok[b]: the
  // flags of buffer b were written by the round that wrote its rows, against ref_node's row of the
  // buffer that round read, and nothing has written either buffer since
  // option "ref_rows" (default off: measured slower): the flag loads, the reference
  // word and the writer's ballot + byte store cost more issue/latency than the 8 gathers they replace
  bool ref_rows = false;
  int64_t ref_node = -1;  // first honest node (chosen at the first round that can use it); -2: none
  size_t rflag_off = 0;   // byte offset of the flags in a snapshot buffer
  bool rflag_ok[3] = {false, false, false};
  // option "uniform_rows" (default on; kernels.h uni_*): every snapshot buffer carries one mismatch
  // slot per rank at word uni_off; uni_ok[b]: buffer b was written by a sweep round that tagged them
  bool uni_rows = true;
  uint32_t uni_merge = 1;  // option "uni_merge": runs per wave in a round with a uniform input (kernels.h)
  bool k_hi_virtual = true;  // option "k_hi_virtual": the K4..K7 group left unstored while counts are < 16 (kernels.h kHiVirt)
  size_t uni_off = 0;
  bool uni_ok[3] = {false, false, false};

  int cur = 0;
  static int nxt(int c) { return c == 2 ? 0 : c + 1; }
  static int prv(int c) { return c == 0 ? 2 : c - 1; }
  // recomputed vote registers (kernels.h vv): option "virtual_votes" and the
  // smallest BL it is used at (option "vv_min_bl": below it the 7 extra
  // gathered rows cost more requests than the 64 B per lane of V planes save)
  uint32_t* vstale = nullptr;  // [tiles]
  // deferred count planes (kernels.h klazy): option "count_lazy"
  uint32_t* kpend = nullptr;   // [tiles]
  bool k_pend = false;         // some tile may hold pending steps or flags
  bool count_lazy = true;
  bool v_stale = false;        // some tile may be stale
  bool virtual_votes = true;
  uint32_t vv_min_bl = 16;
  uint32_t* valid = nullptr;
  uint32_t* byz = nullptr;
  uint64_t* log = nullptr;
  uint32_t* log_count = nullptr;
  uint64_t* dlog = nullptr;          // dense lane records (kernels.h dense_words(k) u64 each)
  uint32_t* dlog_count = nullptr;
  uint64_t* mlog = nullptr;          // medium lane records (kernels.h kMedMax: 2 u64 each)
  uint32_t* mlog_count = nullptr;
  uint32_t mlog_cap = 0;
  uint32_t* upd_count = nullptr;     // StatusUpdates emitted per shard (singles + dense bits)
  uint32_t dlog_cap = 0;
  uint32_t* log_overflow = nullptr;
  uint32_t* node_flags = nullptr;  // capped engines: nodes k_round_node leaves to the exact pass
  uint32_t log_cap = 0;
  uint32_t log_shards = 1;
  // allocated entries of the three log kinds (all shards together); log_cap / mlog_cap / dlog_cap are
  // these divided by log_shards, which follows the round kernels' wave count (set_log_layout)
  size_t log_alloc = 0, mlog_alloc = 0, dlog_alloc = 0;
  unsigned long long* applied = nullptr;
  unsigned long long* bytes = nullptr;
  unsigned long long* finalized = nullptr;
  unsigned long long* scratch_count = nullptr;
  int64_t round = 0, log_base = 0;
  // update words (kernels.h pack_update): the round field starts at bit round_shift = 28 + the node
  // field's width, max(24, bits of N); the log spans at most 2^(64 - round_shift) rounds
  uint32_t round_shift = 52;
  int64_t max_log_rounds() const { return (int64_t)1 << (64 - round_shift); }
  // every consider bit ever shifted in was 1 (no replay, no neutral drop-in
  // vote, no write_records): an all-ones oldest consider plane implies all
  // consider planes are all-ones (lets k_round_fast skip them)
  bool c_monotone = true;
  bool plane_nt = true;  // tuning option "plane_nt" (A/B on MI355X: -8 % kernel time warm, -16 % cold)
  bool ablate_gather = false;  // diagnostics option "ablate_gather" (invalid results)
  uint32_t ablate_node = 0;  // diagnostics option "ablate_node" (k_round_node, invalid results)
  int ablate_emit = 0;  // diagnostics option "ablate_emit": 1 = StatusUpdates counted, not stored; 2 = no reserving atomic; 3 = atomic issued, result unused
  uint32_t ablate_phase = 0;  // diagnostics option "ablate_phase" (kernels.h; results invalid)
  // diagnostics option "unsynced_shard": a node-sharded engine runs rounds with no exchange (other
  // shards' preference rows keep their initial values; per-rank kernel timing only, invalid results)
  bool unsynced_shard = false;
  // diagnostics option "warm_pref": before each timed round, read the snapshots the round gathers
  // from (untimed), as a GPU of the rank's own would hold them in its caches (tools/group_model.py:
  // the serial group runs every rank's kernel on one GPU, each after the others' traffic)
  bool warm_pref = false;
  uint32_t* touch_sink = nullptr;
  // round kernels (option "kernel"): 2 = k_round_sweep (uncapped) / k_round_node (capped), k <= 8;
  // 1 = k_round_fast / k_round_capped (the first versions; any k, A/B baseline)
  int kernel = 2;
  uint32_t sweep_blocks = 0;  // resident workgroups of the sweep grid (option "sweep_blocks"; 0 = one wave per tile)
  bool sweep_blocks_explicit = false;  // "sweep_blocks" set to a value >= 0: "tiles_per_wave" leaves it alone
  // option "sweep_nopipe": a walking grid runs without next-tile prefetch
  // (kModeWarm; default); 0 = the prefetching kModeWarmPipe (A/B)
  bool sweep_nopipe = true;
  // option "wave_runs": a walking grid gives each wave a run of consecutive
  // tiles whose peers one Philox pass draws (round_sweep.hip WaveDraw)
  bool wave_runs = true;
  // option "settled_fast": settled warm tiles skip the round step's bookkeeping
  bool settled_fast = true;
  // option "settled_lean": with BL dividing 64, a wave tests its run's settled candidates in one
  // lean loop first (round_sweep.hip settled_run)
  bool settled_lean = true;
  // option "tiles_per_wave" (default grid, default_sweep_blocks); 0 = by size: up to 16, at most BL, with
  // >= 15000 waves (C4: 500k tiles, 16 per wave; C3's 98k tiles: 4 — 8 per wave leaves two generations
  // of waves and was 6 % slower)
  uint32_t tiles_per_wave = 0;
  // every consider plane of every lane is all-ones: set after a sim round with k >= 8 in which every
  // live record was polled (all targets valid, uncapped); cleared by anything that can write a 0
  // consider bit (init, add, write_records, drop-in votes, replay)
  bool warm_all = false;
  // every record is a NewVoteRecord from av_init_records (votes = consider =
  // count = 0): the next sweep round reads only the A plane (kernels.h fresh)
  bool fresh = false;
  uint32_t bl_magic = 1, bl_sh1 = 0, bl_sh2 = 0;
  uint32_t store_policy = 0;  // option "store_policy": 2 = sc1 (write-through) plane stores, 3 = nt sc1
  // upper bound on any live record's count (confidence >> 1) at the start of the next round: a
  // round adds at most k, init/add start at 0, anything else sets it to 127. While it is < 120 no
  // record can finalize in the next round (k <= 8), so the capped path skips its exact pass.
  int count_bound = 127;
  std::vector<uint32_t> valid_host;
  // replay stream
  uint32_t* replay = nullptr;
  int64_t replay_cap_rounds = 0, replay_first = 0, replay_ready = 0;
  int replay_fuse = 16;  // option "replay_fuse": replay rounds per k_replay_node launch (capped engines; <= 1: off)
  bool replay_fast = true;  // option "replay_fast": k_replay_fast for nodes whose poll set is their first 128 lanes
  // timing
  bool timing = false;
  bool round_marker = false;  // option "round_marker" (diagnostics)
  hipEvent_t marker = nullptr;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  double timed_ms = 0.0;
  int64_t timed_launches = 0;
  // RCCL
  ncclComm_t comm = nullptr;
  int world = 1, rank = 0;
  // peer-push exchange (av_peer_init): every rank's three
  // snapshot buffers and arrival slots mapped into this process over IPC
  int peer_world = 0, peer_rank = 0;
  uint32_t* peer_pref[3][avk::kMaxPeers + 1] = {};  // [buffer][rank]; own rank = the local buffer
  uint32_t* arrive = nullptr;                        // [kMaxPeers + 1] arrival slots (local)
  // barrier timeout flag in pinned host memory (the barrier kernel stores it
  // with system scope): the host reads it without synchronizing the stream
  uint32_t* barrier_err = nullptr;                   // device view of barrier_err_host
  volatile uint32_t* barrier_err_host = nullptr;
  bool failed = false;                               // sticky: a peer barrier timed out
  bool pref_uncached = false;  // option "pref_uncached": snapshot buffers in uncached device memory (A/B)
  bool peer_fine = true;  // option "peer_fine": snapshot buffers fine-grained once exported (xGMI coherence)
  size_t pref_alloc_words = 0;
  uint32_t barrier_seq = 0;
  uint32_t barrier_timeout_ms = 30000;
  std::vector<void*> peer_opened;                    // IPC mappings to close
  avk::PeerPtrs peer_arrive{};
  uint32_t** push_tbl = nullptr;                     // device [3][kMaxPeers]: peers' replicas of each buffer
  uint64_t barrier_ticks = 0;                        // barrier_timeout_ms in wall-clock ticks (peer_timeout_ticks)
  // diagnostics option "solo_barrier": a one-rank barrier (the same 1-wave kernel, world 1) after every
  // round of an engine without a peer exchange — the exchange's fixed cost per round without the
  // pushes and without other ranks (tools/exchange_cost.py)
  bool solo_barrier = false;
  // sticky: solo_barrier was enabled at some point (its arrival slots were allocated and its barrier
  // sequence advanced outside an exchange): this engine can no longer join a peer exchange
  bool solo_used = false;
  // in-process peer group (av_peer_group_serial): e->stream is the group's stream, own_stream this
  // engine's (destroyed with it)
  PeerGroup* group = nullptr;
  hipStream_t own_stream = nullptr;
  // need-masked exchange (option "peer_mask", default on; kernels.h RoundParams::need / stale,
  // DESIGN.md §5): a sweep round pushes a row segment only to the peers whose nodes draw that row in
  // the next round, and remembers per segment, buffer and peer the changes it withheld
  bool peer_mask = true;
  bool push_defer = true;          // option "push_defer": sweep pushes queued per wave (RoundParams::push_q)
  uint32_t push_store = 1;         // option "push_store" (RoundParams::push_store)
  uint32_t tile_draw = 0;          // option "tile_draw" (RoundParams::tile_draw, A/B)
  uint32_t mat_run = 1;            // option "materialize_run" (RoundParams::mat_run, A/B)
  bool masked = false;             // set up by the exchange's initialisation (mask_setup)
  uint32_t segs = 1;               // 32-word segments per row
  uint8_t* need_mine = nullptr;    // [kNeedWin][N]: rows this rank's nodes draw in a window's rounds
  uint8_t* needmask = nullptr;     // [kNeedWin][NL]: peers (push order) that draw each local row
  uint8_t* stale = nullptr;        // [3][NL * segs]: per snapshot buffer, peers whose copy may differ
  uint32_t* needin = nullptr;      // [2][world][kNeedWin][ceil(NL/32)]: the peers' drawn-row bits (IPC:
                                   // inside the exported arrival allocation, at kNeedinOff)
  avk::PeerPtrs peer_needin{};     // every rank's needin
  int64_t need_ready = -1;         // window whose needmask is combined
  int64_t need_pushed = -1;        // window whose drawn rows were pushed to the peers
  // the next window's rows are drawn on a side stream while the current window's rounds run
  // (need_draw_ahead): need_free = the last push that read need_mine, need_drawn = the draw done
  hipStream_t need_stream = nullptr;
  hipEvent_t need_free = nullptr, need_drawn = nullptr;
  int64_t need_drawn_w = -1;       // window whose rows the side stream drew (or is drawing)
  // changed published words (kernels.h RoundParams::changed): counted in every peer-push round and,
  // with option "count_changed", in every sweep round
  unsigned long long* changed = nullptr;
  bool count_changed = false;
  // the reference-row flag bytes of every buffer were cleared (or the engine created) at this round;
  // a flag byte carries a 7-bit round tag, so they are cleared again before 128 rounds have passed
  int64_t rflag_clear_round = 0;

  // responder variant (option "responder", kernels.h pub_mode) and the nodes
  // that no longer poll (av_set_polling); both run the first-generation kernel
  uint32_t dense_min = 0;  // option "dense_min" (kernels.h dense records; default dense_min(k))
  uint32_t wave_dense = 0;  // option "wave_dense" (kernels.h RoundParams::wave_dense; A/B)
  uint32_t uni_votes = 1;   // option "uni_votes" (kernels.h RoundParams::uni_votes)
  int32_t pub_mode = 0;
  uint32_t* readd = nullptr;     // [L] pub_mode 2: re-add marks
  uint32_t* died_out = nullptr;  // [L] pub_mode 2: records deleted this round
  std::vector<uint32_t> nopoll_host;
  uint32_t* nopoll = nullptr;    // [ceil(NL/32)]
  bool any_nopoll = false;
  // per-local-node Processor.round (processor.go:15,40-42): a field only the
  // caller changes (avalanche_test.go:302); allocated on the first set
  std::vector<int64_t> proc_round;
  // device scratch kept across calls (StatusUpdate delivery, digests)
  void* fetch_scratch = nullptr;
  size_t fetch_scratch_bytes = 0;
  unsigned long long* digest = nullptr;  // [3]
  // drop-in batches (av_register_votes_batch): pinned host staging; option "dropin_fast" (0: always the
  // sort-grouped general path, A/B and tests)
  void* dropin_host = nullptr;
  size_t dropin_host_bytes = 0;
  // StatusUpdate delivery into pageable caller memory: two pinned staging chunks (copy_out)
  void* stage[2] = {nullptr, nullptr};
  hipEvent_t stage_ev[2] = {nullptr, nullptr};
  bool dropin_fast = true;
  // StatusUpdate encoder (log_ops.hip launch_encode_log): error flags and per-pass totals (device)
  uint32_t* enc_err = nullptr;
  uint64_t* enc_tot = nullptr;  // [4]
  uint32_t enc_buckets = 1u << 26;  // option "enc_buckets": (round, node) buckets per encoder pass
  // option "copy_blocks": workgroups of the compact stream's device-to-host copy kernel (k_stream_out);
  // 0 = hipMemcpyAsync (the runtime's copy)
  uint32_t copy_blocks = 0;
  // compact stream delivery (av_fetch_compact_async / _wait): kSlots slots, each a device buffer
  // the encoder writes and a pinned host buffer its copy lands in, the copy on copy_stream (overlaps
  // the next rounds on the engine stream); ticket t uses slot t % kSlots
  static constexpr int kSlots = 3;
  hipStream_t copy_stream = nullptr;
  void* cdev[kSlots] = {};
  size_t cdev_bytes[kSlots] = {};
  void* chost[kSlots] = {};
  size_t chost_bytes[kSlots] = {};
  hipEvent_t cev[kSlots] = {};
  av_compact_header chdr[kSlots] = {};
  int64_t cticket = 0;           // next ticket
  bool cpend[kSlots] = {};       // a copy was issued into the slot
  // high-water marks: a slot that grows grows to the largest stream seen, so a caller's warm-up pass
  // sizes every slot and later rounds never allocate (pinned allocations take tens of ms)
  size_t cdev_hwm = 0, chost_hwm = 0;
  // batched poll sets (av_get_invs_batch): host-mapped pinned output the fill kernel writes
  void* invs_host = nullptr;
  size_t invs_host_bytes = 0;

  size_t round_replay_words() const { return avk::replay_words(Lpad, k); }
};

namespace {

int set_device(av_engine* e) {
  AV_CHECK(e, AV_ERR_INVALID_ARG, "null engine");
  AV_HIP(hipSetDevice(e->cfg.device));
  return AV_OK;
}

#define AV_ENTER(e)              \
  do {                           \
    int _rc = set_device(e);     \
    if (_rc != AV_OK) return _rc; \
  } while (0)

bool local_node(const av_engine* e, int64_t node) { return node >= e->n0 && node < e->n1; }
bool local_target(const av_engine* e, int64_t t) { return t >= e->t0 && t < e->t1; }

// Growable device scratch (drop-in / readback paths only; never inside a round).
struct Scratch {
  void* p = nullptr;
  size_t bytes = 0;
  ~Scratch() {
    if (p) (void)hipFree(p);
  }
  hipError_t ensure(size_t n) {
    if (n <= bytes) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
    hipError_t e = hipMalloc(&p, n);
    if (e == hipSuccess) bytes = n;
    return e;
  }
};

// Anything but a reference-row sweep round that writes a snapshot buffer
// (drop-in votes, adds, writes, init, validity/publish-rule refreshes, peer
// and RCCL set-up, other round kernels) leaves its flags stale.
void ref_invalidate(av_engine* e) {
  e->rflag_ok[0] = e->rflag_ok[1] = e->rflag_ok[2] = false;
  e->uni_ok[0] = e->uni_ok[1] = e->uni_ok[2] = false;
}

avk::RoundParams round_params(const av_engine* e, const uint32_t* replay) {
  avk::RoundParams p{};
  p.planes = e->planes;
  p.pref_in = e->pref[e->cur];
  p.pref_out = e->pref[av_engine::nxt(e->cur)];
  p.pref_prev = e->pref[av_engine::prv(e->cur)];
  p.vstale = e->vstale;
  p.valid = e->valid;
  p.byz = e->byz;
  p.replay = replay;
  p.log = e->log;
  p.log_count = e->log_count;
  p.dlog = e->dlog;
  p.dlog_count = e->dlog_count;
  p.upd_count = e->upd_count;
  p.dlog_cap = e->dlog_cap;
  p.mlog = e->mlog;
  p.mlog_count = e->mlog_count;
  p.mlog_cap = e->mlog_cap;
  p.log_overflow = e->log_overflow;
  p.applied = e->applied;
  p.bytes = e->bytes;
  p.finalized = e->finalized;
  p.warm_skip = e->c_monotone ? 1u : 0u;
  p.plane_nt = e->plane_nt ? 1u : 0u;
  p.ablate_gather = e->ablate_gather ? 1u : 0u;
  p.ablate_emit = (uint32_t)e->ablate_emit;
  p.ablate_phase = e->ablate_phase;
  p.ablate_node = e->ablate_node;
  p.mat_run = e->mat_run;
  p.tile_draw = e->tile_draw;
  p.seed = e->cfg.seed;
  p.log_cap = e->log_cap;
  p.log_shards = e->log_shards;  // a power of two (set_log_layout): the sweep kernel masks by it
  p.n_nodes = (uint32_t)e->N;
  p.n0 = (uint32_t)e->n0;
  p.NL = e->NL;
  p.BL = e->BL;
  p.PS = e->PS;
  p.L = e->L;
  p.Lpad = e->Lpad;
  p.t0 = (uint32_t)e->t0;
  p.round = (uint32_t)e->round;
  p.round_rel = (uint32_t)(e->round - e->log_base);
  p.round_shift = e->round_shift;
  p.peer_mode = e->cfg.peer_mode;
  p.warm_all = e->warm_all ? 1u : 0u;
  p.store_policy = e->store_policy;
  p.node_flags = nullptr;
  p.bl_magic = e->bl_magic;
  p.bl_sh1 = e->bl_sh1;
  p.bl_sh2 = e->bl_sh2;
  p.kpend = e->kpend;
  p.klazy = 0u;
  p.kconsume = 0u;
  p.fresh = 0u;
  p.tn = (uint32_t)(e->t1 - e->t0);
  p.nopipe = e->sweep_nopipe ? 1u : 0u;
  p.tpw = e->wave_runs && e->sweep_blocks ? 1u : 0u;
  p.settled_fast = e->settled_fast ? 1u : 0u;
  p.lean = e->settled_lean && 64 % e->BL == 0 ? 1u : 0u;
  p.bl_log2 = (uint32_t)__builtin_ctz(e->BL);
  p.pub_mode = (uint32_t)e->pub_mode;
  p.readd = e->pub_mode == 2 ? e->readd : nullptr;
  p.died_out = e->pub_mode == 2 ? e->died_out : nullptr;
  p.nopoll = e->any_nopoll ? e->nopoll : nullptr;
  p.dense_min = e->dense_min;
  p.wave_dense = e->wave_dense;
  p.uni_votes = e->uni_votes;
  return p;
}

// Write back the vote planes of tiles the last warm k = 8 sim round left
// stale (kernels.h vv); every path that reads or writes records other than
// such a round calls this first.
int materialize_votes_only(av_engine* e) {
  if (!e->v_stale) return AV_OK;
  AV_HIP(avk::launch_materialize(round_params(e, nullptr), true, false, e->stream));
  e->v_stale = false;
  return AV_OK;
}

// Apply the pending +8 steps of deferred count planes (kernels.h klazy);
// every path that reads or writes counts other than a klazy round calls this
// first.
int materialize_counts(av_engine* e) {
  if (!e->k_pend) return AV_OK;
  AV_HIP(avk::launch_materialize(round_params(e, nullptr), false, true, e->stream));
  e->k_pend = false;
  return AV_OK;
}

// Both deferred forms (vote planes, count planes) written back, in one pass.
int materialize_votes(av_engine* e) {
  if (!e->v_stale && !e->k_pend) return AV_OK;
  AV_HIP(avk::launch_materialize(round_params(e, nullptr), e->v_stale, e->k_pend, e->stream));
  e->v_stale = false;
  e->k_pend = false;
  return AV_OK;
}

// A serial peer group's members store into each other's buffers: once any member was destroyed (its
// buffers freed), no member may push or exchange need masks any more.
int group_alive(const av_engine* e) {
  if (e->group)
    for (const av_engine* m : e->group->members) AV_CHECK(m, AV_ERR_UNSUPPORTED, "peer group: a rank was destroyed");
  return AV_OK;
}

// Peer-push exchange: copy this rank's rows of snapshot buffer `b` into every
// peer replica (a full resynchronisation of those rows).
int push_own_rows(av_engine* e, int b) {
  {
    int rc = group_alive(e);
    if (rc != AV_OK) return rc;
  }
  avk::PeerPtrs dst{};
  uint32_t n = 0;
  for (int r = 0; r < e->peer_world; ++r)
    if (r != e->peer_rank) dst.p[n++] = e->peer_pref[b][r];
  const uint64_t w0 = (uint64_t)e->n0 * e->PS, w1 = w0 + (uint64_t)e->NL * e->PS;
  AV_HIP(avk::launch_push_rows(e->pref[b], dst, n, w0, w1, e->stream));
  return AV_OK;
}

// Barrier across the peer ranks, on the engine stream (kernels.h).
// slot_buf >= 0: the barrier kernel first copies this rank's uniform-rows mismatch slot of snapshot
// buffer slot_buf into every peer's replica (the round kernel writes only its own copy, RoundParams::
// uni_post). A serial group has no barrier: the copy alone runs.
int peer_barrier(av_engine* e, int slot_buf = -1) {
  const uint32_t* slot = nullptr;
  avk::PeerPtrs sd{};
  if (slot_buf >= 0 && e->peer_world > 1) {
    slot = e->pref[slot_buf] + e->uni_off + e->peer_rank;
    for (int r = 0; r < e->peer_world; ++r) sd.p[r] = e->peer_pref[slot_buf][r] + e->uni_off + e->peer_rank;
  }
  if (e->group) {  // serial group: every rank's kernels run in one stream's order
    if (slot)
      AV_HIP(avk::launch_peer_barrier(e->peer_arrive, (uint32_t)e->peer_world, (uint32_t)e->peer_rank, 0u, nullptr,
                                      0u, e->stream, slot, sd, 0u));
    return AV_OK;
  }
  if (!e->barrier_ticks) AV_HIP(avk::peer_timeout_ticks(e->cfg.device, e->barrier_timeout_ms, &e->barrier_ticks));
  AV_HIP(avk::launch_peer_barrier(e->peer_arrive, (uint32_t)std::max(1, e->peer_world), (uint32_t)e->peer_rank,
                                  ++e->barrier_seq, e->barrier_err, e->barrier_ticks, e->stream, slot, sd, 1u));
  return AV_OK;
}

// ---- need-masked exchange (kernels.h RoundParams::need / stale) ----
constexpr size_t kNeedinOff = 4096;  // byte offset of needin in the exported arrival allocation

size_t needin_words(const av_engine* e, int world) {
  return (size_t)2 * (size_t)world * avk::kNeedWin * ((e->NL + 31) / 32);
}

// a row's 32-word segments never straddle a wave: BL a power of two <= 32 (a node's lanes inside one
// tile) or a multiple of 32 (32-aligned segments inside 64-aligned tiles)
bool mask_layout_ok(const av_engine* e) {
  return (e->BL <= 32 && (e->BL & (e->BL - 1)) == 0) || e->BL % 32 == 0;
}

// After the exchange's pointers are set (own needin allocated, peer_needin filled): buffers of the
// masked form, every replica identical (nothing withheld).
uint32_t default_sweep_blocks(const av_engine* e, bool force);
extern "C" int relayout_log_if_empty(av_engine* e);

int mask_setup(av_engine* e) {
  // node shards of an exchange: runs of up to 16 tiles per wave (the longest the shared draw holds,
  // BL >= 16) unless set: the single-GPU rule (>= 15000 waves) gave 4 at 8 ranks of C4, whose settled
  // rounds then paid 4x the per-wave set-up (tools/group_model.py)
  if (!e->tiles_per_wave && !e->sweep_blocks_explicit && e->BL >= 16 && e->peer_world >= 4) {
    e->tiles_per_wave = 16;
    e->sweep_blocks = default_sweep_blocks(e, false);
    int rc = relayout_log_if_empty(e);  // fewer writer waves
    if (rc != AV_OK) return rc;
  }
  e->masked = e->peer_mask && e->peer_world >= 2 && e->peer_world <= 9 && mask_layout_ok(e) && e->needin;
  if (!e->masked) return AV_OK;
  e->segs = (e->BL + 31) / 32;
  AV_HIP(dev_alloc(&e->need_mine, (size_t)avk::kNeedWin * e->N));
  AV_HIP(dev_alloc(&e->needmask, (size_t)avk::kNeedWin * e->NL));
  AV_HIP(dev_alloc(&e->stale, (size_t)3 * e->NL * e->segs));
  AV_HIP(hipMemsetAsync(e->stale, 0, (size_t)3 * e->NL * e->segs, e->stream));
  AV_HIP(hipStreamCreateWithFlags(&e->need_stream, hipStreamNonBlocking));
  AV_HIP(hipEventCreateWithFlags(&e->need_free, hipEventDisableTiming));
  AV_HIP(hipEventCreateWithFlags(&e->need_drawn, hipEventDisableTiming));
  e->need_ready = e->need_pushed = e->need_drawn_w = -1;
  return AV_OK;
}

// Every replica of snapshot buffer b was just given this rank's rows whole: nothing withheld.
int stale_clear(av_engine* e, int b) {
  if (!e->masked) return AV_OK;
  const size_t n = (size_t)e->NL * e->segs;
  AV_HIP(hipMemsetAsync(e->stale + (size_t)b * n, 0, n, e->stream));
  return AV_OK;
}

// Window w = push rounds [w W, w W + W): the rows this rank's nodes draw in rounds w W + 1 .. w W + W
// (R1's sampling), pushed to their owners; enqueued before a barrier, combined after it.
int need_draw(av_engine* e, int64_t w, hipStream_t s) {
  const uint32_t W = avk::kNeedWin;
  AV_HIP(hipMemsetAsync(e->need_mine, 0, (size_t)W * e->N, s));
  AV_HIP(avk::launch_need_draw(e->cfg.seed, (uint32_t)e->N, (uint32_t)e->n0, e->NL, (uint32_t)(w * W + 1), W, e->k,
                               e->cfg.peer_mode, e->need_mine, s));
  return AV_OK;
}

int need_gen(av_engine* e, int64_t w) {
  if (!e->masked || e->need_pushed == w) return AV_OK;
  {
    int rc = group_alive(e);
    if (rc != AV_OK) return rc;
  }
  if (e->need_drawn_w == w) {
    AV_HIP(hipStreamWaitEvent(e->stream, e->need_drawn, 0));  // drawn ahead on the side stream
  } else {
    int rc = need_draw(e, w, e->stream);
    if (rc != AV_OK) return rc;
  }
  AV_HIP(avk::launch_need_push(e->need_mine, (uint32_t)e->N, e->NL, avk::kNeedWin, (uint32_t)e->peer_world,
                               (uint32_t)e->peer_rank, (uint32_t)(w & 1), e->peer_needin, e->stream));
  AV_HIP(hipEventRecord(e->need_free, e->stream));
  e->need_pushed = w;
  e->need_drawn_w = -1;
  return AV_OK;
}

// Window w + 1's rows drawn on the side stream while window w's rounds run (after window w's push
// released need_mine); need_gen at the end of window w waits for it.
// (not in a serial peer group: there every rank's side stream would run beside the other ranks'
// rounds on the one device, which a rank of a real run never sees; the group draws inline)
int need_draw_ahead(av_engine* e, int64_t w) {
  if (!e->masked || e->group || e->need_drawn_w == w || e->need_pushed >= w) return AV_OK;
  AV_HIP(hipStreamWaitEvent(e->need_stream, e->need_free, 0));
  int rc = need_draw(e, w, e->need_stream);
  if (rc != AV_OK) return rc;
  AV_HIP(hipEventRecord(e->need_drawn, e->need_stream));
  e->need_drawn_w = w;
  return AV_OK;
}

int ref_pick(av_engine* e);

// After the barrier that ordered every rank's need_gen of window w: the per-row peer masks.
int need_combine(av_engine* e, int64_t w) {
  if (!e->masked || e->need_ready == w || e->need_pushed != w) return AV_OK;
  int rc = ref_pick(e);  // the reference row (uniform rows) is read by every rank
  if (rc != AV_OK) return rc;
  const uint32_t ref_local =
      e->ref_node >= e->n0 && e->ref_node < e->n1 ? (uint32_t)(e->ref_node - e->n0) : 0xFFFFFFFFu;
  AV_HIP(avk::launch_need_combine(e->needin, (uint32_t)e->peer_world, (uint32_t)e->peer_rank, (uint32_t)(w & 1),
                                  avk::kNeedWin, e->NL, ref_local, e->needmask, e->stream));
  e->need_ready = w;
  return AV_OK;
}

// Peer-push engines keep every replica of a snapshot buffer identical; a
// write to this rank's rows outside a round would break that.
int peer_local_write_check(const av_engine* e) {
  AV_CHECK(e->peer_world <= 1, AV_ERR_UNSUPPORTED,
           "record writes outside a round are not supported on a peer-push node-sharded engine");
  return AV_OK;
}

// A peer barrier that timed out (a rank stopped taking part) leaves the
// ranks' snapshot replicas unordered: every later round and every result of
// this engine is refused (sticky), AV_ERR_PEER.
int peer_failed(av_engine* e) {
  if (e->peer_world > 1 && !e->failed && e->barrier_err_host && *e->barrier_err_host) e->failed = true;
  if (e->failed)
    return fail(AV_ERR_PEER, "peer barrier timed out (a rank stopped taking part in the rounds): the exchange is "
                             "broken, results of this engine are invalid");
  return AV_OK;
}

#define AV_PEER_CHECK(e)          \
  do {                            \
    int _rc = peer_failed(e);     \
    if (_rc != AV_OK) return _rc; \
  } while (0)

// For calls that return results: every round enqueued so far (and its
// barrier) completes first, then the flag decides.
#define AV_PEER_SYNC_CHECK(e)                                      \
  do {                                                             \
    if ((e)->peer_world > 1) AV_HIP(hipStreamSynchronize((e)->stream)); \
    int _rc = peer_failed(e);                                      \
    if (_rc != AV_OK) return _rc;                                  \
  } while (0)

// Growable device scratch owned by the engine.
int engine_scratch(av_engine* e, size_t bytes, void** out) {
  if (bytes > e->fetch_scratch_bytes) {
    if (e->fetch_scratch) AV_HIP(hipFree(e->fetch_scratch));
    e->fetch_scratch = nullptr;
    e->fetch_scratch_bytes = 0;
    hipError_t he = hipMalloc(&e->fetch_scratch, bytes);
    AV_CHECK(he == hipSuccess, he == hipErrorOutOfMemory ? AV_ERR_OOM : AV_ERR_HIP, "scratch (%zu B): %s", bytes,
             hipGetErrorString(he));
    e->fetch_scratch_bytes = bytes;
  }
  *out = e->fetch_scratch;
  return AV_OK;
}

// The reference node: the first honest node (a Byzantine row changes every
// round and would never match).
int ref_pick(av_engine* e) {
  if (e->ref_node != -1) return AV_OK;
  e->ref_node = -2;
  const size_t words = std::min<size_t>((e->N + 31) / 32, 1024);
  std::vector<uint32_t> w(words);
  AV_HIP(hipMemcpyAsync(w.data(), e->byz, words * 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  for (size_t i = 0; i < words && e->ref_node < 0; ++i)
    if (~w[i]) {
      const int64_t n = (int64_t)i * 32 + __builtin_ctz(~w[i]);
      if (n < e->N) e->ref_node = n;
    }
  return AV_OK;
}

int launch_one_round(av_engine* e, const uint32_t* replay) {
  AV_CHECK(e->round - e->log_base < e->max_log_rounds(), AV_ERR_OVERFLOW,
           "StatusUpdate log spans %lld rounds: call av_fetch_updates more often", (long long)e->max_log_rounds());
  if (e->group) {
    // serial group: round r of rank i is enqueued after round r of every lower rank and before
    // round r of every higher one (the stream order is the exchange's barrier)
    for (const av_engine* m : e->group->members) AV_CHECK(m, AV_ERR_UNSUPPORTED, "peer group: a rank was destroyed");
    for (const av_engine* m : e->group->members)
      if (m != e)
        AV_CHECK(m->round == e->round + (m->peer_rank < e->peer_rank ? 1 : 0), AV_ERR_UNSUPPORTED,
                 "peer group: rank %d at round %lld, rank %d at round %lld: run one round of every rank in rank "
                 "order", e->peer_rank, (long long)e->round, m->peer_rank, (long long)m->round);
  }
  AV_CHECK(e->NL == (uint32_t)e->N || e->comm != nullptr || e->peer_world > 1 || e->N == e->n1 - e->n0 ||
               e->unsynced_shard,
           AV_ERR_UNSUPPORTED,
           "node-sharded engine needs av_comm_init before running rounds");
  avk::RoundParams p = round_params(e, replay);
  // responder variants and non-polling nodes run the first-generation kernels
  const bool compat = e->pub_mode != 0 || e->any_nopoll;
  AV_CHECK(!(compat && e->capped && (e->pub_mode == 2 || e->any_nopoll)), AV_ERR_UNSUPPORTED,
           "the example responder and av_set_polling need M <= 4096 (uncapped)");
  // the sweep addresses the preference table by 32-bit byte offsets
  const bool sweep = e->kernel == 2 && e->k <= 8 && !e->capped && !compat && (uint64_t)e->N * e->PS < (1ull << 30);
  // the round after av_init_records: planes known to be zero are not read
  const bool fresh = e->fresh && sweep && !replay && !e->ablate_gather;
  // the sweep's warm sim modes (launch_sweep_k): every consider plane all-ones
  const bool warm = sweep && !replay && e->c_monotone && e->warm_all && !e->ablate_gather && !fresh;
  // vote planes may be left unstored: warm (or fresh) k = 8 sim rounds
  // below vv_min_bl only the uniform form (a settled tile's V = A: nothing to regather)
  const bool vv = e->virtual_votes && e->k == 8 && (warm || fresh);
  const bool vv_uniform = vv && e->BL < e->vv_min_bl;
  if (!vv) {
    int rc = materialize_votes_only(e);
    if (rc != AV_OK) return rc;
  }
  p.vv = vv ? 1u : 0u;
  p.vv_uniform = vv_uniform ? 1u : 0u;
  if (vv) e->v_stale = true;
  p.fresh = fresh ? 1u : 0u;
  // count planes may be deferred: warm k = 8 sim rounds while no record can
  // finalize (every true count < 120 at round start); the first warm round
  // that can finalize applies the pending steps itself (kconsume)
  const bool klazy = e->count_lazy && warm && e->k == 8 && e->count_bound < 120;
  const bool kconsume = !klazy && e->k_pend && warm && e->k == 8;
  if (!klazy && !kconsume) {
    int rc = materialize_counts(e);
    if (rc != AV_OK) return rc;
  }
  p.klazy = klazy ? 1u : 0u;
  p.kconsume = kconsume ? 1u : 0u;
  p.hivirt = e->k_hi_virtual && e->k == 8 ? 1u : 0u;
  if (klazy) e->k_pend = true;
  if (kconsume) e->k_pend = false;
  bool all_valid = true;
  for (uint32_t b = 0; b < e->BL; ++b) {
    const int64_t tb = e->t0 + 32ll * b;
    const int64_t r = std::min<int64_t>(e->t1 - tb, 32);
    all_valid &= e->valid_host[b] == (r >= 32 ? ~0u : ((1u << r) - 1u));
  }
  // peer-push exchange: the sweep kernel's sim rounds push changed words; any
  // other round is followed by a full push of this rank's rows (uniform across
  // ranks: it depends only on the engine configuration and the call)
  const bool peer = e->peer_world > 1;
  const int nb = av_engine::nxt(e->cur);
  if (peer && sweep && !replay) {
    p.push_n = (uint32_t)e->peer_world - 1u;
    p.push_dst = e->push_tbl + (size_t)nb * avk::kMaxPeers;
    if (e->masked) {  // need-masked pushes: this round's row masks (window of push round e->round)
      const int64_t w = e->round / avk::kNeedWin;  // combined below (need_combine) if not yet
      const bool have = e->need_ready == w || e->need_pushed == w;
      p.need = have ? e->needmask + (size_t)(e->round % avk::kNeedWin) * e->NL : nullptr;
      p.stale = e->stale + (size_t)nb * e->NL * e->segs;
      p.segs = e->segs;
    }
    p.peer_all = (1u << std::min<uint32_t>(p.push_n, 31u)) - 1u;
    p.push_defer = e->push_defer ? 1u : 0u;
    p.push_store = e->push_store;
  }
  p.count_changed = (p.push_n || e->count_changed) && sweep && !replay ? 1u : 0u;
  p.changed = e->changed;
  // reference rows: sweep rounds at k = 8 with a node's lanes inside one wave
  bool refr = e->ref_rows && sweep && e->k == 8 && !replay && 64 % e->BL == 0 && !e->comm && !e->ablate_gather;
  if (refr) {
    int rc = ref_pick(e);
    if (rc != AV_OK) return rc;
    refr = e->ref_node >= 0;
  }
  if (refr && e->round - e->rflag_clear_round >= 120) {
    // flag bytes carry a 7-bit snapshot tag (round_sweep.hip ref_tag): every buffer's flags are
    // cleared before 128 rounds have passed since the last clear, whatever kind of round ran in
    // between (replay, capped, non-refr), so no byte outlives its tag's period
    for (int b = 0; b < 3; ++b)
      AV_HIP(hipMemsetAsync(reinterpret_cast<uint8_t*>(e->pref[b]) + e->rflag_off, 0, (size_t)e->N, e->stream));
    e->rflag_clear_round = e->round;
    ref_invalidate(e);
  }
  if (refr) {
    p.ref_node = (uint32_t)e->ref_node;
    p.ps_shift = (uint32_t)__builtin_ctz(e->PS * 4u);
    p.rflag_off = (uint32_t)e->rflag_off;

    p.rflag_out = reinterpret_cast<uint8_t*>(e->pref[nb]) + e->rflag_off;
    p.rflag_in = e->rflag_ok[e->cur] ? reinterpret_cast<const uint8_t*>(e->pref[e->cur]) + e->rflag_off : nullptr;
  }
  // uniform rows: sweep rounds at k = 8 tag the snapshot they write; a round whose input snapshot
  // is known uniform tests settled tiles with no peer draw and no gather (kernels.h uni_*)
  // (a node-sharded engine sees every row only through the peer exchange, whose pushes carry the slots)
  // (unsynced_shard, diagnostics: a rank's share alone, on its own slot: timing as in a peer-push run)
  bool uni = e->uni_rows && sweep && e->k == 8 && !replay && !e->comm && !e->ablate_gather &&
             (e->NL == (uint32_t)e->N || e->peer_world > 1 || e->unsynced_shard);
  if (uni) {
    int rc = ref_pick(e);
    if (rc != AV_OK) return rc;
    uni = e->ref_node >= 0;
  }
  if (uni) {
    p.ref_node = (uint32_t)e->ref_node;
    p.uni_off = (uint32_t)e->uni_off;
    p.uni_world = (uint32_t)std::max(1, e->peer_world);
    p.uni_rank = (uint32_t)std::max(0, e->peer_rank);
    p.uni_out = e->pref[nb] + e->uni_off;
    p.uni_in = e->uni_ok[e->cur] ? e->pref[e->cur] + e->uni_off : nullptr;
    const int pv = av_engine::prv(e->cur);
    p.uni_prev = e->uni_ok[pv] ? e->pref[pv] + e->uni_off : nullptr;
    p.uni_merge = e->uni_merge;
    p.uni_post = peer && sweep && !replay ? 1u : 0u;  // the slot reaches the peers in the barrier kernel
  }
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (e->warm_pref && sweep) {  // diagnostics (untimed): the round's gather sources, read once
    if (!e->touch_sink) AV_HIP(hipMalloc(&e->touch_sink, 64));
    AV_HIP(avk::launch_touch(p.pref_prev, (size_t)e->N * e->PS * 4u, e->touch_sink, e->stream));
    AV_HIP(avk::launch_touch(p.pref_in, (size_t)e->N * e->PS * 4u, e->touch_sink, e->stream));
  }
  if (e->timing) {
    AV_HIP(hipEventCreate(&ev0));
    AV_HIP(hipEventCreate(&ev1));
    AV_HIP(hipEventRecord(ev0, e->stream));
  }
  if (p.push_n && e->masked) {  // (inside the round's timing: the exchange's own work)
    int rc = need_combine(e, e->round / avk::kNeedWin);
    if (rc == AV_OK) rc = need_draw_ahead(e, e->round / avk::kNeedWin + 1);
    if (rc != AV_OK) return rc;
  }
  bool refw = false;  // the round wrote reference-row flags for the snapshot it published
  if (sweep)
    AV_HIP(avk::launch_round_sweep(p, e->k, replay != nullptr, e->sweep_blocks, e->stream, &refw));
  else if (e->kernel == 2 && e->k <= 8 && e->capped && !compat) {
    p.node_flags = e->node_flags;
    AV_HIP(avk::launch_round_node(p, e->k, replay != nullptr, /*exact_pass=*/e->count_bound >= 120, e->stream));
  }
  else
    AV_HIP(avk::launch_round(p, e->k, replay != nullptr, e->capped, e->stream));
  if (e->pub_mode == 2) {  // the responders' re-adds (main.go:175-177)
    AV_HIP(avk::launch_readd(p, e->stream));
    e->warm_all = false;
    e->count_bound = 127;
  }
  e->count_bound = std::min(127, e->count_bound + e->k);
  if (fresh && p.hivirt) e->k_pend = true;  // the fresh round flags its tiles kHiVirt
  e->fresh = false;
  e->rflag_ok[nb] = refr && refw;
  e->uni_ok[nb] = uni;
  if (replay)
    e->warm_all = false;
  else if (e->c_monotone && e->k >= 8 && !e->capped && all_valid)
    e->warm_all = true;  // every live record was polled and shifted in 8 considered votes
  if (peer) {
    // the next push round's window drawn and pushed before the barrier (combined after it)
    int rc = need_gen(e, (e->round + 1) / avk::kNeedWin);
    if (rc != AV_OK) return rc;
  }
  if (e->timing) {
    AV_HIP(hipEventRecord(ev1, e->stream));
    e->events.emplace_back(ev0, ev1);
  } else if (e->round_marker) {  // diagnostics: a timing-free event after every round
    if (!e->marker) AV_HIP(hipEventCreateWithFlags(&e->marker, hipEventDisableTiming));
    AV_HIP(hipEventRecord(e->marker, e->stream));
  }
  if (peer) {
    if (!p.push_n) {
      int rc = push_own_rows(e, nb);
      if (rc == AV_OK) rc = stale_clear(e, nb);
      if (rc != AV_OK) return rc;
    }
    int rc = peer_barrier(e, p.uni_post ? nb : -1);
    if (rc != AV_OK) return rc;
  } else if (e->solo_barrier) {
    int rc = peer_barrier(e);
    if (rc != AV_OK) return rc;
  }
  if (e->comm) {
    const size_t count = (size_t)e->NL * e->PS;
    uint32_t* out = e->pref[av_engine::nxt(e->cur)];
    ncclResult_t r = ncclAllGather(out + (size_t)e->n0 * e->PS, out, count, ncclUint32, e->comm, e->stream);
    AV_CHECK(r == ncclSuccess, AV_ERR_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
  }
  e->cur = av_engine::nxt(e->cur);
  e->round++;
  return AV_OK;
}

// Replay rounds [round, round + R) of a capped engine in one k_replay_node
// launch, followed per round by the exact pass over the nodes it left at that
// round (count >= 120). Host-side round bookkeeping as launch_one_round.
int launch_replay_fused(av_engine* e, const uint32_t* replay0, int32_t R) {
  if (e) ref_invalidate(e);
  AV_CHECK(e->round + R - 1 - e->log_base < e->max_log_rounds(), AV_ERR_OVERFLOW,
           "StatusUpdate log spans %lld rounds: call av_fetch_updates more often", (long long)e->max_log_rounds());
  int rc = materialize_votes_only(e);
  if (rc != AV_OK) return rc;
  rc = materialize_counts(e);
  if (rc != AV_OK) return rc;
  const size_t per = e->round_replay_words();
  avk::RoundParams p = round_params(e, replay0);
  p.node_flags = e->node_flags;
  p.fuse_rounds = (uint32_t)R;
  p.replay_fast = e->replay_fast && e->BL >= avk::kMaxPoll / 32 ? 1u : 0u;
  p.replay_stride = per;
  p.ring_next = (uint32_t)av_engine::nxt(e->cur);
  for (int i = 0; i < 3; ++i) p.pref_ring[i] = e->pref[i];
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (e->timing) {
    AV_HIP(hipEventCreate(&ev0));
    AV_HIP(hipEventCreate(&ev1));
    AV_HIP(hipEventRecord(ev0, e->stream));
  }
  AV_HIP(avk::launch_replay_node(p, e->k, e->stream));
  for (int32_t r = 0; r < R; ++r) {
    if (e->count_bound >= 120) {  // a node may have reached count 120 by this round
      avk::RoundParams q = round_params(e, replay0 + per * (size_t)r);
      q.node_flags = e->node_flags;
      q.exact_rel = (uint32_t)r;
      q.exact_keep = r + 1 < R ? 1u : 0u;
      AV_HIP(avk::launch_round(q, e->k, /*replay=*/true, /*capped=*/true, e->stream));
    }
    e->count_bound = std::min(127, e->count_bound + e->k);
    e->fresh = false;
    e->warm_all = false;
    e->cur = av_engine::nxt(e->cur);
    e->round++;
  }
  if (e->timing) {
    AV_HIP(hipEventRecord(ev1, e->stream));
    e->events.emplace_back(ev0, ev1);
  }
  return AV_OK;
}

// Sweep grid (0 = one wave per tile). Each wave walks `tiles_per_wave`
// tiles (grid stride, no next-tile prefetch): the wave's prologue — kernel
// parameters, the loop-invariant Philox key schedule and the SGPR spills the
// compiler parks in VGPR lanes, ~150 SALU and ~100 VALU instructions — is then
// paid once per 4 tiles instead of per tile. Measured on MI355X
// (tools/round_probe.py, C4 epoch): one wave per tile 9.37 ms, 4 tiles per
// wave 8.37 ms, 17 per wave 8.39 ms; the prefetching resident grid
// (kModeWarmPipe, 5 waves per SIMD) 9.5-10.2 ms. force: the resident grid (A/B).
uint32_t default_sweep_blocks(const av_engine* e, bool force = false) {
  if (e->k > 8 || e->capped) return 0;
  const uint64_t tiles = e->Lpad / 64;
  if (force) {
    int bpc = 0, cus = 0;
    if (avk::round_sweep_occupancy(e->k, false, &bpc, &cus) != hipSuccess || bpc <= 0 || cus <= 0) return 0;
    return (uint32_t)(bpc * cus);
  }
  // (by size: a run's nodes must fit the shared draw, 2 producer lanes each: 8 tiles need BL >= 16)
  // (a run's nodes must fit the run's peer draw: 2 producer lanes per node and round, 64 lanes; runs
  // of 16 tiles at BL >= 32 draw both rounds in two passes: C4 epoch 5.14 -> 4.95 ms, the settled
  // rounds 0.112 -> 0.088 ms, storm rounds +2 %, profiles/r03/ab_tiles_per_wave.log)
  // Default: the longest run (16, 8 or 4 tiles) whose nodes fit one 64-lane draw (tiles_per_wave <= BL:
  // 64 * tpw / BL nodes per run) while the grid keeps >= 15000 waves. Target shards of C4
  // (tools/shard_model.py, profiles/r04/tshard_c4_*.json, rank 0's settled rounds): BL 16 (G = 2)
  // 0.083 ms at 4 tiles per wave, 0.038 at 16; BL 8 (G = 4) 0.046 at 4, 0.031 at 8, 0.166 at 16 (the
  // run's nodes overflow the draw); BL 4 (G = 8) 0.027 at 4, 0.124 at 8.
  // Narrow rows (BL <= 8: C5, the target shards of C4 at 4 and 8 ranks): a run's nodes overflow the
  // draw at any length >= BL / 2, so every tile draws its own peers whatever the run, and the longest
  // run pays the per-wave set-up least; the uniform settled runs take up to 256 nodes (settled_run_uni).
  // Round 5 (tools/group_model.py, profiles/r05/s11/gm_td16_*.log; tools/round_probe.py, ab_c5td.log):
  // C4 rank 0 at G = 8 window 1.545 -> 1.309 ms, G = 4 2.078 -> 1.955, C5 epoch 17.2 -> 16.2 ms, C4p /
  // C4pb within 1 %.
  uint64_t tpw = e->tiles_per_wave;
  if (!tpw && e->BL <= 8) tpw = 16;
  if (!tpw) {
    tpw = 16;
    while (tpw > 4 && (tpw > (uint64_t)e->BL || tiles / tpw < 15000)) tpw /= 2;
  }
  const uint64_t waves = (tiles + tpw - 1) / tpw;
  return (uint32_t)std::max<uint64_t>(1, (waves + 3) / 4);
}

// Waves that write the StatusUpdate log in the fewest-wave round kernel the engine may launch: every
// writer picks shard wave % log_shards, so with more shards than writers the rest would sit empty and
// the usable capacity shrink by that factor. Capped engines: k_round_node (one wave per node per 64
// blocks); uncapped: the sweep grid's waves that own a run of tiles (launch_sweep_k: runs of
// ceil(tiles / waves) tiles), never more than the tiles (the first-generation kernels: one per tile).
uint64_t log_writer_waves(const av_engine* e) {
  if (e->capped) return (uint64_t)e->NL * ((e->BL + 63) / 64);
  const uint64_t tiles = e->Lpad / 64;
  if (!e->sweep_blocks) return tiles;
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(e->sweep_blocks, (tiles + 3) / 4));
  const uint64_t run = (tiles + grid * 4 - 1) / (grid * 4);
  return std::max<uint64_t>(1, (tiles + run - 1) / run);
}

// Shard count and per-shard capacities of the (empty) log from the allocation and the writers: a
// power of two with >= 4 writers per shard in every kernel, so that the modulo's uneven wrap (W
// writers over S shards: some get ceil(W / S)) loads no shard more than 1.25x the mean.
uint64_t log_shards_for(uint64_t w) {
  uint64_t sh = 1;
  while (sh * 2 <= avk::kLogShards && sh * 2 * 4 <= w) sh *= 2;
  return sh;
}

void set_log_layout(av_engine* e) {
  e->log_shards = (uint32_t)log_shards_for(log_writer_waves(e));
  e->log_cap = (uint32_t)std::min<size_t>(e->log_alloc / e->log_shards, 0xFFFFFFFFu);
  e->mlog_cap = (uint32_t)std::min<size_t>(e->mlog_alloc / e->log_shards, 0xFFFFFFFFu);
  e->dlog_cap = (uint32_t)std::min<size_t>(e->dlog_alloc / e->log_shards, 0xFFFFFFFFu);
}


// The arrival slots of the peer barrier (one per rank, fine-grained when peers store into them over
// xGMI) and the barrier's timeout flag in pinned host memory (the barrier kernel stores it with
// system scope, so the host sees it without synchronizing the stream; av_run_rounds refuses to
// enqueue once it is set). Zeroed before any peer can see them: the exchange of handles orders the two.
// The same allocation carries, at kNeedinOff, the table the peers' need_push stores into (sized for
// the world of equal node shards this engine's shard implies, N / NL).
int alloc_arrival(av_engine* e) {
  const int world = e->N % e->NL == 0 && e->N / e->NL <= avk::kMaxPeers + 1 ? (int)(e->N / e->NL) : 1;
  const size_t bytes = (kNeedinOff + needin_words(e, world) * 4 + (2u << 20) - 1) / (2u << 20) * (2u << 20);
  if (e->peer_fine)
    AV_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&e->arrive), bytes, hipDeviceMallocFinegrained));
  else
    AV_HIP(dev_alloc(&e->arrive, bytes / 4));
  void* hp = nullptr;
  AV_HIP(hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent));
  e->barrier_err_host = static_cast<volatile uint32_t*>(hp);
  *e->barrier_err_host = 0u;
  void* dp = nullptr;
  AV_HIP(hipHostGetDevicePointer(&dp, hp, 0));
  e->barrier_err = static_cast<uint32_t*>(dp);
  AV_HIP(hipMemset(e->arrive, 0, (size_t)(avk::kMaxPeers + 1) * 4));
  AV_HIP(hipDeviceSynchronize());
  return AV_OK;
}

int refresh_pref(av_engine* e) {
  ref_invalidate(e);
  AV_HIP(avk::launch_refresh_pref((uint32_t)e->pub_mode, e->planes, e->pref[e->cur], e->byz, (uint32_t)e->n0, e->NL,
                                  e->BL, e->PS, (uint32_t)e->round, e->stream));
  return AV_OK;
}

}  // namespace

extern "C" {

int av_abi_version(void) { return AVHIP_ABI_VERSION; }

void av_config_init(av_config* c) {
  if (!c) return;
  std::memset(c, 0, sizeof(*c));
  c->k = 8;
  c->seed = 0xA7A1A9C4ull;
}

const char* av_strerror(int code) {
  switch (code) {
    case AV_OK: return "ok";
    case AV_ERR_INVALID_ARG: return "invalid argument";
    case AV_ERR_HIP: return "HIP runtime error";
    case AV_ERR_OOM: return "out of device memory";
    case AV_ERR_NOT_FOUND: return "VoteRecord not found";
    case AV_ERR_OVERFLOW: return "buffer overflow";
    case AV_ERR_UNSUPPORTED: return "unsupported configuration";
    case AV_ERR_RCCL: return "RCCL error";
    case AV_ERR_PEER: return "peer exchange failed";
    default: return "unknown error";
  }
}

const char* av_last_error(void) { return g_last_error.c_str(); }

int av_destroy(av_engine* e) {
  if (!e) return AV_OK;
  (void)hipSetDevice(e->cfg.device);
  if (e->stream) (void)hipStreamSynchronize(e->stream);
  for (auto& ev : e->events) {
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  if (e->comm) (void)ncclCommDestroy(e->comm);
  for (void* m : e->peer_opened) (void)hipIpcCloseMemHandle(m);
  if (e->arrive) (void)hipFree(e->arrive);
  if (e->barrier_err_host) (void)hipHostFree(const_cast<uint32_t*>(e->barrier_err_host));
  if (e->fetch_scratch) (void)hipFree(e->fetch_scratch);
  if (e->dropin_host) (void)hipHostFree(e->dropin_host);
  for (int i = 0; i < 2; ++i) {
    if (e->stage[i]) (void)hipHostFree(e->stage[i]);
    if (e->stage_ev[i]) (void)hipEventDestroy(e->stage_ev[i]);
  }
  if (e->digest) (void)hipFree(e->digest);
  if (e->copy_stream) {
    (void)hipStreamSynchronize(e->copy_stream);
    (void)hipStreamDestroy(e->copy_stream);
  }
  for (int i = 0; i < av_engine::kSlots; ++i) {
    if (e->cdev[i]) (void)hipFree(e->cdev[i]);
    if (e->chost[i]) (void)hipHostFree(e->chost[i]);
    if (e->cev[i]) (void)hipEventDestroy(e->cev[i]);
  }
  if (e->invs_host) (void)hipHostFree(e->invs_host);
  if (e->enc_err) (void)hipFree(e->enc_err);
  if (e->touch_sink) (void)hipFree(e->touch_sink);
  if (e->enc_tot) (void)hipFree(e->enc_tot);
  if (e->changed) (void)hipFree(e->changed);
  if (e->push_tbl) (void)hipFree(e->push_tbl);
  if (e->marker) (void)hipEventDestroy(e->marker);
  if (e->need_stream) {
    (void)hipStreamSynchronize(e->need_stream);
    (void)hipStreamDestroy(e->need_stream);
  }
  if (e->need_free) (void)hipEventDestroy(e->need_free);
  if (e->need_drawn) (void)hipEventDestroy(e->need_drawn);
  if (e->group) {
    PeerGroup* g = e->group;
    g->members[(size_t)e->peer_rank] = nullptr;
    e->stream = e->own_stream;  // destroyed below; the group's stream with its last member
    if (--g->alive == 0) {
      (void)hipStreamDestroy(g->stream);
      delete g;
    }
  }
  void* bufs[] = {e->planes, e->pref[0], e->pref[1], e->pref[2], e->vstale, e->kpend, e->valid, e->byz, e->log, e->log_count, e->log_overflow, e->node_flags,
                  e->readd, e->died_out, e->nopoll,
                  e->dlog, e->upd_count, e->mlog,
                  e->applied, e->bytes, e->finalized, e->scratch_count, e->replay,
                  e->need_mine, e->needmask, e->stale, e->group ? e->needin : nullptr};
  for (void* b : bufs)
    if (b) (void)hipFree(b);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  delete e;
  return AV_OK;
}

int av_create(const av_config* cfg, av_engine** out) {
  AV_CHECK(cfg && out, AV_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  const av_config& c = *cfg;
  // node ids are 32-bit in the kernels; the update word's node field widens past 24 bits by taking
  // bits from its round field (pack_update), which keeps >= 2^6 rounds between fetches below 2^30
  AV_CHECK(c.n_nodes >= 2 && c.n_nodes < (1ll << 30), AV_ERR_INVALID_ARG, "n_nodes must be in [2, 2^30)");
  AV_CHECK(c.n_targets >= 1 && c.n_targets < (1ll << 22), AV_ERR_INVALID_ARG, "n_targets must be in [1, 2^22)");
  AV_CHECK(c.k >= 1 && c.k <= avk::kMaxK, AV_ERR_INVALID_ARG, "k must be in [1, 16]");
  AV_CHECK(c.peer_mode == AV_PEERS_RANDOM || c.peer_mode == AV_PEERS_ROUND_ROBIN, AV_ERR_INVALID_ARG,
           "bad peer_mode");
  auto* e = new av_engine();
  e->cfg = c;
  e->N = c.n_nodes;
  e->M = c.n_targets;
  e->n0 = c.node_begin;
  e->n1 = c.node_end;
  if (e->n0 == 0 && e->n1 == 0) e->n1 = e->N;
  e->t0 = c.target_begin;
  e->t1 = c.target_end;
  if (e->t0 == 0 && e->t1 == 0) e->t1 = e->M;
  e->k = c.k;
  {
    uint32_t nb = 24;
    while (nb < 32 && (1ll << nb) < e->N) ++nb;
    e->round_shift = 28 + nb;
  }
  auto bad = [&](const char* msg) {
    delete e;
    return fail(AV_ERR_INVALID_ARG, "%s", msg);
  };
  if (!(e->n0 >= 0 && e->n0 < e->n1 && e->n1 <= e->N)) return bad("bad node shard");
  if (!(e->t0 >= 0 && e->t0 < e->t1 && e->t1 <= e->M && e->t0 % 32 == 0)) return bad("bad target shard");
  e->capped = e->M > (int64_t)avk::kMaxPoll;
  if (e->capped && (e->t0 != 0 || e->t1 != e->M)) {
    delete e;
    return fail(AV_ERR_UNSUPPORTED,
                "target sharding needs M <= 4096: the 4096 poll cap couples targets (processor.go:165-167)");
  }
  e->NL = (uint32_t)(e->n1 - e->n0);
  e->BL = (uint32_t)((e->t1 - e->t0 + 31) / 32);
  e->PS = avk::pref_stride(e->BL);
  if (e->capped && e->BL > 1024) return bad("capped path supports M <= 32768");
  const uint64_t L = (uint64_t)e->NL * e->BL;
  if (L >= (1ull << 31)) return bad("too many lanes for one engine: shard further");
  // the round kernels index the published-preference table (all N nodes x PS words) in 32 bits
  if ((uint64_t)e->N * e->PS >= (1ull << 31)) return bad("preference table over 2^31 words: shard targets further");
  e->L = (uint32_t)L;
  e->Lpad = (uint32_t)((L + 63) / 64 * 64);
  avk::bl_divider(e->BL, e->bl_magic, e->bl_sh1, e->bl_sh2);

  int rc = AV_OK;
  auto hip_fail = [&](hipError_t he, const char* what) {
    av_destroy(e);
    return fail(he == hipErrorOutOfMemory ? AV_ERR_OOM : AV_ERR_HIP, "%s: %s", what, hipGetErrorString(he));
  };
  hipError_t he = hipSetDevice(c.device);
  if (he != hipSuccess) return hip_fail(he, "hipSetDevice");
  if ((he = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking)) != hipSuccess)
    return hip_fail(he, "hipStreamCreate");
  const size_t plane_words = (size_t)(e->Lpad / 64) * avk::kPlanes * 64;
  const size_t pref_words = (size_t)e->N * e->PS;
  int64_t cap = c.update_log_capacity;
  if (cap <= 0) cap = std::min<int64_t>(std::max<int64_t>((int64_t)L * 8, 1 << 20), 1ll << 28);
  // one shard per wave up to kLogShards: waves of the round kernel that runs
  const uint64_t waves = e->capped ? (uint64_t)e->NL * ((e->BL + 63) / 64) : (uint64_t)(e->Lpad / 64);
  e->log_shards = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(waves, avk::kLogShards));
  e->log_cap = (uint32_t)std::max<int64_t>((cap + e->log_shards - 1) / e->log_shards, 64);
  if ((he = dev_alloc(&e->planes, plane_words)) != hipSuccess) return hip_fail(he, "alloc planes");
  // whole 2-MiB units: each snapshot buffer is an allocation of its own (IPC export, av_peer_handles)
  e->rflag_off = (pref_words * 4 + 255) / 256 * 256;
  e->uni_off = (e->rflag_off + (size_t)e->N + 255) / 256 * 256 / 4;  // uniform-rows slots (kernels.h)
  const size_t pref_alloc =
      ((e->uni_off * 4 + (avk::kMaxPeers + 1) * 4 + (2u << 20) - 1) / (2u << 20)) * (2u << 20) / 4;
  e->pref_alloc_words = pref_alloc;
  if ((he = dev_alloc(&e->pref[0], pref_alloc)) != hipSuccess) return hip_fail(he, "alloc pref");
  if ((he = dev_alloc(&e->pref[1], pref_alloc)) != hipSuccess) return hip_fail(he, "alloc pref");
  if ((he = dev_alloc(&e->pref[2], pref_alloc)) != hipSuccess) return hip_fail(he, "alloc pref");
  if ((he = dev_alloc(&e->vstale, e->Lpad / 64)) != hipSuccess) return hip_fail(he, "alloc planes");
  if ((he = dev_alloc(&e->kpend, e->Lpad / 64)) != hipSuccess) return hip_fail(he, "alloc planes");
  (void)hipMemsetAsync(e->vstale, 0, (size_t)(e->Lpad / 64) * 4, e->stream);
  (void)hipMemsetAsync(e->kpend, 0, (size_t)(e->Lpad / 64) * 4, e->stream);
  if ((he = dev_alloc(&e->valid, e->BL)) != hipSuccess) return hip_fail(he, "alloc valid");
  if ((he = dev_alloc(&e->byz, (e->N + 31) / 32)) != hipSuccess) return hip_fail(he, "alloc byz");
  if ((he = dev_alloc(&e->log, (size_t)e->log_cap * e->log_shards)) != hipSuccess) return hip_fail(he, "alloc log");
  // the singles', medium and dense records' per-shard counters: one array (round_common.h
  // emit_reserve_med indexes it by kind)
  if ((he = dev_alloc(&e->log_count, 3 * avk::kLogShards * avk::kCtrStride)) != hipSuccess) return hip_fail(he, "alloc log");
  e->mlog_count = e->log_count + avk::kLogShards * avk::kCtrStride;
  e->dlog_count = e->log_count + 2 * avk::kLogShards * avk::kCtrStride;
  // a dense record holds >= dense_min(k) updates: log_cap / dense_min records
  // take any log_cap updates that go dense (8 B of capacity per update)
  const uint32_t dw = avk::dense_words((uint32_t)e->k);
  e->dense_min = avk::dense_min((uint32_t)e->k);
  // k = 8 with slot records (kernels.h AVK_MED_S4): a lane goes dense from 4 slots with updates on
  const uint32_t dense_least = e->k == 8 && AVK_MED_S4 ? 4u : e->dense_min;
  e->dlog_cap = std::max<uint32_t>(e->log_cap / dense_least, 16);
  if ((he = dev_alloc(&e->dlog, (size_t)e->dlog_cap * e->log_shards * dw)) != hipSuccess) return hip_fail(he, "alloc log");
  if ((he = dev_alloc(&e->upd_count, avk::kLogShards)) != hipSuccess) return hip_fail(he, "alloc log");
  // a medium record holds >= 2 updates: log_cap / 2 records per shard (kernels.h med_rec_words: 32 B
  // slot records, 16 B per update of capacity). Only k = 8 kernels emit them (round_common.h
  // emit_updates_med: the sweep, k_replay_fast): other engines keep a token 16 records per shard.
  e->mlog_cap = e->k == 8 ? std::max<uint32_t>(e->log_cap / 2, 16) : 16u;
  if ((he = dev_alloc(&e->mlog, (size_t)e->mlog_cap * e->log_shards * avk::med_rec_words())) != hipSuccess)
    return hip_fail(he, "alloc log");
  e->log_alloc = (size_t)e->log_cap * e->log_shards;
  e->mlog_alloc = (size_t)e->mlog_cap * e->log_shards;
  e->dlog_alloc = (size_t)e->dlog_cap * e->log_shards;
  (void)hipMemsetAsync(e->log_count, 0, (size_t)3 * avk::kLogShards * avk::kCtrStride * 4, e->stream);
  (void)hipMemsetAsync(e->upd_count, 0, avk::kLogShards * 4, e->stream);
  if ((he = dev_alloc(&e->log_overflow, 1)) != hipSuccess) return hip_fail(he, "alloc log");
  if (e->capped) {
    if ((he = dev_alloc(&e->node_flags, e->NL)) != hipSuccess) return hip_fail(he, "alloc node flags");
    (void)hipMemsetAsync(e->node_flags, 0, (size_t)e->NL * 4, e->stream);
  }
  if ((he = dev_alloc(&e->applied, avk::kLogShards)) != hipSuccess) return hip_fail(he, "alloc counters");
  // [0, kLogShards): model bytes moved; [kLogShards, 2 kLogShards): the part of them that re-reads a
  // preference word another lane of the same round already gathered (av_alg_bytes_reread)
  if ((he = dev_alloc(&e->bytes, 2 * avk::kLogShards)) != hipSuccess) return hip_fail(he, "alloc counters");
  (void)hipMemsetAsync(e->bytes, 0, 2 * avk::kLogShards * 8, e->stream);
  if ((he = dev_alloc(&e->finalized, avk::kLogShards)) != hipSuccess) return hip_fail(he, "alloc counters");
  (void)hipMemsetAsync(e->finalized, 0, avk::kLogShards * 8, e->stream);
  if ((he = dev_alloc(&e->scratch_count, 1)) != hipSuccess) return hip_fail(he, "alloc counters");
  if ((he = dev_alloc(&e->changed, 3 * avk::kLogShards)) != hipSuccess) return hip_fail(he, "alloc counters");
  (void)hipMemsetAsync(e->changed, 0, 3 * avk::kLogShards * 8, e->stream);

  (void)hipMemsetAsync(e->log_overflow, 0, 4, e->stream);
  (void)hipMemsetAsync(e->applied, 0, avk::kLogShards * 8, e->stream);
  (void)hipMemsetAsync(e->pref[0], 0, e->pref_alloc_words * 4, e->stream);
  (void)hipMemsetAsync(e->pref[1], 0, e->pref_alloc_words * 4, e->stream);
  (void)hipMemsetAsync(e->pref[2], 0, e->pref_alloc_words * 4, e->stream);
  // every real target starts valid
  e->valid_host.assign(e->BL, 0u);
  for (uint32_t b = 0; b < e->BL; ++b) {
    const int64_t tb = e->t0 + 32ll * b;
    const int64_t r = std::min<int64_t>(e->t1 - tb, 32);
    e->valid_host[b] = r >= 32 ? ~0u : ((1u << r) - 1u);
  }
  if ((he = hipMemcpyAsync(e->valid, e->valid_host.data(), e->BL * 4, hipMemcpyHostToDevice, e->stream)) !=
      hipSuccess)
    return hip_fail(he, "upload valid");
  if ((he = avk::launch_byz(e->byz, (uint32_t)e->N, c.seed, c.byz_threshold, e->stream)) != hipSuccess)
    return hip_fail(he, "byz kernel");
  e->sweep_blocks = default_sweep_blocks(e);
  set_log_layout(e);  // shards = the sweep grid's writers (a wave takes a run of tiles), not the tiles
  *out = e;
  rc = av_init_records(e, AV_INIT_NONE, 0);
  if (rc != AV_OK) {
    av_destroy(e);
    *out = nullptr;
    return rc;
  }
  return AV_OK;
}

int av_init_records(av_engine* e, int32_t init_mode, uint32_t init_param) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  e->warm_all = false;
  // every record starts at count 0 with no considered vote (NewVoteRecord, vote.go:33-35), and a
  // count step needs > 6 considered votes in the 8-vote window (vote.go:58-61): the first 6 votes
  // of a fresh record cannot step it, so after v votes every count is <= v - 6
  e->count_bound = -6;
  if (e->v_stale) {  // every plane is rewritten
    AV_HIP(hipMemsetAsync(e->vstale, 0, (size_t)(e->Lpad / 64) * 4, e->stream));
    e->v_stale = false;
  }
  if (e->k_pend) {
    AV_HIP(hipMemsetAsync(e->kpend, 0, (size_t)(e->Lpad / 64) * 4, e->stream));
    e->k_pend = false;
  }
  AV_CHECK(init_mode >= AV_INIT_NONE && init_mode <= AV_INIT_PAIRS, AV_ERR_INVALID_ARG, "bad init_mode");
  avk::InitParams p{};
  p.planes = e->planes;
  p.pref = e->pref[e->cur];
  p.byz = e->byz;
  p.seed = e->cfg.seed;
  p.n_nodes = (uint32_t)e->N;
  p.n0 = (uint32_t)e->n0;
  p.NL = e->NL;
  p.BL = e->BL;
  p.PS = e->PS;
  p.L = e->L;
  p.Lpad = e->Lpad;
  p.t0 = (uint32_t)e->t0;
  p.n_targets = (uint32_t)e->t1;  // targets >= t1 belong to another shard (or do not exist)
  p.round = (uint32_t)e->round;
  p.mode = init_mode;
  p.pub_mode = (uint32_t)e->pub_mode;
  p.param = init_param;
  AV_HIP(avk::launch_init(p, e->stream));
  if (e->peer_world > 1) {
    // peer-push engine: this rank's new rows of the current snapshot go to every peer replica, and
    // no rank's next round may read them before all ranks have pushed (collective: every rank
    // re-initialises). The other two buffers are untouched, so their replicas stay identical.
    int rc = push_own_rows(e, e->cur);
    if (rc == AV_OK) rc = stale_clear(e, e->cur);
    if (rc == AV_OK) rc = need_gen(e, e->round / avk::kNeedWin);
    if (rc != AV_OK) return rc;
    rc = peer_barrier(e);
    if (rc != AV_OK) return rc;
  }
  e->fresh = init_mode != AV_INIT_NONE;
  // lanes of the padded tail of the last tile hold no records
  if (e->Lpad > e->L) {
    // padded lanes are never loaded (active = g < L), nothing to do
  }
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_set_valid(av_engine* e, int64_t target, int32_t valid) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  AV_CHECK(target >= 0 && target < e->M, AV_ERR_INVALID_ARG, "target out of range");
  if (!local_target(e, target)) return AV_OK;
  int rc = materialize_votes(e);  // stale tiles must not gain live-but-invalid records
  if (rc != AV_OK) return rc;
  const int64_t tl = target - e->t0;
  const uint32_t b = (uint32_t)(tl >> 5), m = 1u << (tl & 31);
  e->valid_host[b] = valid ? (e->valid_host[b] | m) : (e->valid_host[b] & ~m);
  AV_HIP(hipMemcpyAsync(e->valid + b, &e->valid_host[b], 4, hipMemcpyHostToDevice, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_add_targets(av_engine* e, int64_t node, const int64_t* targets, const uint8_t* accepted, int64_t n,
                   uint8_t* added) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  {
    int rc = peer_local_write_check(e);
    if (rc != AV_OK) return rc;
  }
  AV_CHECK(n >= 0 && (n == 0 || (targets && accepted && added)), AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(local_node(e, node), AV_ERR_INVALID_ARG, "node %lld not in this shard", (long long)node);
  {
    int rc = materialize_votes(e);
    if (rc != AV_OK) return rc;
  }
  e->warm_all = false;
  e->fresh = false;
  std::vector<uint32_t> tl;
  std::vector<uint8_t> acc;
  std::vector<int64_t> pos;
  for (int64_t i = 0; i < n; ++i) {
    added[i] = 0;
    if (!local_target(e, targets[i])) continue;
    tl.push_back((uint32_t)(targets[i] - e->t0));
    acc.push_back(accepted[i] ? 1 : 0);
    pos.push_back(i);
  }
  if (tl.empty()) return AV_OK;
  const size_t m = tl.size();
  Scratch s;
  AV_HIP(s.ensure(m * 6 + 64));
  auto* dt = static_cast<uint32_t*>(s.p);
  auto* da = reinterpret_cast<uint8_t*>(dt + m);
  auto* dadd = da + m;
  AV_HIP(hipMemcpyAsync(dt, tl.data(), m * 4, hipMemcpyHostToDevice, e->stream));
  AV_HIP(hipMemcpyAsync(da, acc.data(), m, hipMemcpyHostToDevice, e->stream));
  avk::AddParams p{};
  p.planes = e->planes;
  p.pref = e->pref[e->cur];
  p.valid = e->valid;
  p.byz = e->byz;
  p.targets = dt;
  p.accepted = da;
  p.added = dadd;
  p.n = (uint32_t)m;
  p.node_local = (uint32_t)(node - e->n0);
  p.node = (uint32_t)node;
  p.BL = e->BL;
  p.PS = e->PS;
  p.round = (uint32_t)e->round;
  p.pub_mode = (uint32_t)e->pub_mode;
  AV_HIP(avk::launch_add_targets(p, e->stream));
  std::vector<uint8_t> res(m);
  AV_HIP(hipMemcpyAsync(res.data(), dadd, m, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  for (size_t i = 0; i < m; ++i) added[pos[i]] = res[i];
  return AV_OK;
}

extern "C++" {
namespace {
// Host work of the drop-in path (packing the caller's votes, expanding the
// statuses) split over threads for large batches: the box's CPU share
// (OMP_NUM_THREADS, else up to 16 hardware threads).
int host_threads() {
  static const int n = [] {
    int t = 0;
    if (const char* s = std::getenv("OMP_NUM_THREADS")) t = std::atoi(s);
    if (t <= 0) t = (int)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
    return std::max(1, std::min(t, 64));
  }();
  return n;
}

template <class F>
void parallel_chunks(int64_t n, int64_t min_chunk, F f) {
  const int t = (int)std::max<int64_t>(1, std::min<int64_t>(host_threads(), n / std::max<int64_t>(1, min_chunk)));
  if (t <= 1) {
    f(0, (int64_t)0, n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(t);
  for (int i = 0; i < t; ++i) th.emplace_back([&, i] { f(i, n * i / t, n * (i + 1) / t); });
  for (auto& x : th) x.join();
}

// Pinned host staging of the drop-in path, grown on demand and kept by the engine.
int dropin_staging(av_engine* e, size_t bytes) {
  if (bytes <= e->dropin_host_bytes) return AV_OK;
  if (e->dropin_host) AV_HIP(hipHostFree(e->dropin_host));
  e->dropin_host = nullptr;
  e->dropin_host_bytes = 0;
  const size_t want = std::max(bytes, (size_t)1 << 20);
  AV_HIP(hipHostMalloc(&e->dropin_host, want, hipHostMallocDefault));
  e->dropin_host_bytes = want;
  return AV_OK;
}
}  // namespace
}  // extern "C++"

int av_register_votes(av_engine* e, int64_t node, const int64_t* targets, const uint32_t* errs, int64_t n,
                      int32_t* status_out) {
  const int64_t offs[2] = {0, n};
  return av_register_votes_batch(e, 1, &node, offs, targets, errs, status_out);
}

// Many Responses in one call (processor.go:61-122 for each, in order). The
// host packs each vote into one u32 (target's local index, unknown-hash, yes
// and considered bits: dropin_word) in pinned memory, in parallel, and checks
// on the way whether every Response has strictly ascending targets (a poll
// set's order, rule R1). Then:
//  * fast path (it holds): one workgroup per node applies the node's
//    Responses in call order, each lane's run of votes where it lies
//    (k_dropin_resp), no grouping step;
//  * otherwise: lane keys on the device, the hand-written stable radix sort
//    of (lane, vote position) and run-length encoding (log_ops.hip
//    launch_group_votes, dev_scan.h), then
//    k_register_votes over the runs.
// Statuses come back as one byte per vote and are widened on the host.
// Copies: 4 B per vote each way plus 1 B back (the caller's int64 hashes and
// u32 errs are never copied as such).
int av_register_votes_batch(av_engine* e, int64_t n_resp, const int64_t* nodes, const int64_t* offsets,
                            const int64_t* targets, const uint32_t* errs, int32_t* status_out) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  {
    int rc = peer_local_write_check(e);
    if (rc != AV_OK) return rc;
  }
  AV_CHECK(n_resp >= 0 && (n_resp == 0 || (nodes && offsets)), AV_ERR_INVALID_ARG, "null argument");
  if (n_resp == 0) return AV_OK;
  AV_CHECK(n_resp < (1ll << 31), AV_ERR_INVALID_ARG, "too many Responses in one call");
  AV_CHECK(offsets[0] == 0, AV_ERR_INVALID_ARG, "offsets[0] must be 0");
  for (int64_t i = 0; i < n_resp; ++i) {
    AV_CHECK(offsets[i + 1] >= offsets[i], AV_ERR_INVALID_ARG, "offsets must not decrease");
    AV_CHECK(local_node(e, nodes[i]), AV_ERR_INVALID_ARG, "node %lld not in this shard", (long long)nodes[i]);
  }
  const int64_t n = offsets[n_resp];
  AV_CHECK(n == 0 || (targets && errs && status_out), AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(n < (1ll << 31), AV_ERR_INVALID_ARG, "too many votes in one call");
  AV_CHECK(e->t1 - e->t0 <= (int64_t)avk::kDropTl + 1, AV_ERR_UNSUPPORTED, "drop-in votes need <= 4M local targets");
  {
    int rc = materialize_votes(e);
    if (rc != AV_OK) return rc;
  }
  e->fresh = false;
  // at most one confidence step per vote: bound by the most votes one node gets; the Responses
  // grouped by node, in call order inside a group (fast path)
  int64_t max_node_votes = 0;
  std::vector<uint32_t> order((size_t)n_resp), grp_off;
  {
    std::vector<std::pair<int64_t, uint32_t>> nn((size_t)n_resp);
    for (int64_t i = 0; i < n_resp; ++i) nn[(size_t)i] = {nodes[i], (uint32_t)i};
    std::sort(nn.begin(), nn.end());  // (node, Response index): call order inside a node
    for (size_t i = 0; i < nn.size();) {
      int64_t c = 0;
      size_t j = i;
      grp_off.push_back((uint32_t)i);
      for (; j < nn.size() && nn[j].first == nn[i].first; ++j) {
        c += offsets[nn[j].second + 1] - offsets[nn[j].second];
        order[j] = nn[j].second;
      }
      max_node_votes = std::max(max_node_votes, c);
      i = j;
    }
    grp_off.push_back((uint32_t)n_resp);
  }
  const uint32_t n_groups = (uint32_t)grp_off.size() - 1u;
  e->count_bound = (int)std::min<int64_t>(127, e->count_bound + max_node_votes);
  if (n == 0) return AV_OK;
  // ---- pack (pinned): votes, then the Response table
  const size_t tab_words = 2 * (size_t)n_resp + 1 + (size_t)n_resp + n_groups + 1;  // off, node, order, grp_off
  const size_t hb = (size_t)n * 5 + tab_words * 4 + 64;
  {
    int rc = dropin_staging(e, hb);
    if (rc != AV_OK) return rc;
  }
  auto* hpack = static_cast<uint32_t*>(e->dropin_host);
  auto* hoff = hpack + n;
  auto* hnode = hoff + n_resp + 1;
  auto* horder = hnode + n_resp;
  auto* hgrp = horder + n_resp;
  auto* hstat = reinterpret_cast<int8_t*>(hgrp + n_groups + 1);
  for (int64_t i = 0; i <= n_resp; ++i) hoff[i] = (uint32_t)offsets[i];
  for (int64_t i = 0; i < n_resp; ++i) hnode[i] = (uint32_t)(nodes[i] - e->n0);
  std::memcpy(horder, order.data(), (size_t)n_resp * 4);
  std::memcpy(hgrp, grp_off.data(), ((size_t)n_groups + 1) * 4);
  std::vector<uint8_t> asc_t(64, 1), neutral_t(64, 0);
  const int64_t T0 = e->t0, T1 = e->t1;
  parallel_chunks(n_resp, std::max<int64_t>(1, n_resp * (1 << 18) / std::max<int64_t>(1, n)),
                  [&](int t, int64_t r0, int64_t r1) {
    bool asc = true, neutral = false;
    for (int64_t r = r0; r < r1; ++r) {
      for (int64_t v = offsets[r]; v < offsets[r + 1]; ++v) {
        const int64_t tg = targets[v];
        const uint32_t err = errs[v];
        hpack[v] = avk::dropin_word(tg - T0, tg >= T0 && tg < T1, err);
        neutral |= (int32_t)err < 0;
        if (v > offsets[r]) asc &= tg > targets[v - 1];
      }
    }
    asc_t[t] = asc;
    neutral_t[t] = neutral;
  });
  bool ascending = true;
  for (int t = 0; t < 64; ++t) {
    ascending &= asc_t[t] != 0;
    if (neutral_t[t]) e->c_monotone = false;  // a neutral vote shifts in consider = 0
  }
  const bool fast = ascending && e->dropin_fast;
  // ---- device: packed votes + Response table + byte statuses (+ grouping scratch)
  size_t tb = 0;
  int key_bits = 1;
  const uint32_t m = (uint32_t)n;
  if (!fast) {
    const uint64_t keys_total = (uint64_t)e->L + 1;  // L = unknown targets
    while (key_bits < 32 && (1ull << key_bits) < keys_total) ++key_bits;
    tb = (size_t)avk::group_votes_scratch_words(m) * 8;
  }
  // packed | off | node | status bytes || keys vidx info keys_s perm_s keys_t perm_t lanes offs(m+1) nruns
  // entries(2m) | u64 scratch (radix sort, run scan)
  const size_t head_words = (size_t)m + tab_words + ((size_t)m + 3) / 4;
  const size_t grp_words = fast ? 0 : 8 * (size_t)m + ((size_t)m + 1) + 1 + 2 * (size_t)m;
  void* buf = nullptr;
  int rc = engine_scratch(e, (head_words + grp_words) * 4 + tb + 512, &buf);
  if (rc != AV_OK) return rc;
  auto* w = static_cast<uint32_t*>(buf);
  uint32_t *dpack = w, *doff = dpack + m, *dnode = doff + n_resp + 1, *dorder = dnode + n_resp,
           *dgrp = dorder + n_resp;
  auto* dstat = reinterpret_cast<int8_t*>(dgrp + n_groups + 1);
  AV_HIP(hipMemcpyAsync(dpack, hpack, ((size_t)m + tab_words) * 4, hipMemcpyHostToDevice, e->stream));
  AV_HIP(hipMemsetAsync(dstat, 0xFF, (size_t)m, e->stream));
  avk::DropInParams p{};
  p.planes = e->planes;
  p.pref = e->pref[e->cur];
  p.valid = e->valid;
  p.byz = e->byz;
  p.status_out = dstat;
  p.n0 = (uint32_t)e->n0;
  p.BL = e->BL;
  p.PS = e->PS;
  p.L = e->L;
  p.round = (uint32_t)e->round;
  p.pub_mode = (uint32_t)e->pub_mode;
  p.packed = dpack;
  p.resp_off = doff;
  p.resp_node = dnode;
  p.n_resp = (uint32_t)n_resp;
  p.order = dorder;
  p.grp_off = dgrp;
  p.n_groups = n_groups;
  if (fast) {
    AV_HIP(avk::launch_dropin_resp(p, e->stream));
  } else {
    uint32_t* g0 = w + head_words;
    uint32_t *keys = g0, *vidx = keys + m, *info = vidx + m, *keys_s = info + m, *perm_s = keys_s + m,
             *keys_t = perm_s + m, *perm_t = keys_t + m, *lanes = perm_t + m, *offs = lanes + m,
             *nruns = offs + m + 1, *ent = nruns + 1;
    auto* temp = reinterpret_cast<uint64_t*>(((uintptr_t)(ent + 2 * (size_t)m) + 255) & ~(uintptr_t)255);
    AV_HIP(avk::launch_dropin_keys(p, keys, vidx, info, e->stream));
    AV_HIP(avk::launch_group_votes(temp, keys, vidx, info, m, key_bits, keys_s, perm_s, keys_t, perm_t, lanes, offs,
                                   nruns, ent, e->stream));
    uint32_t nb = 0;
    AV_HIP(hipMemcpyAsync(&nb, nruns, 4, hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipStreamSynchronize(e->stream));
    p.blocks = lanes;
    p.offs = offs;
    p.entries = ent;
    p.n_blocks = nb;
    AV_HIP(avk::launch_register_votes(p, e->stream));
  }
  AV_HIP(hipMemcpyAsync(hstat, dstat, (size_t)m, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  parallel_chunks(n, 1 << 20, [&](int, int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) status_out[i] = hstat[i];
  });
  return AV_OK;
}

int av_read_records(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, uint32_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out && n0 >= e->n0 && n0 <= n1 && n1 <= e->n1 && t0 >= e->t0 && t0 <= t1 && t1 <= e->t1,
           AV_ERR_INVALID_ARG, "range outside this engine's shard");
  const size_t n = (size_t)(n1 - n0) * (size_t)(t1 - t0);
  if (!n) return AV_OK;
  // the deferred forms (stale vote planes, pending count steps) are read
  // through, not written back: a read leaves the next round's fast paths on
  avk::RoundParams p = round_params(e, nullptr);
  p.vv = e->v_stale ? 1u : 0u;
  p.klazy = e->k_pend ? 1u : 0u;
  void* buf = nullptr;
  int rc = engine_scratch(e, n * 4, &buf);
  if (rc != AV_OK) return rc;
  AV_HIP(avk::launch_read_records_virtual(p, (uint32_t)(n0 - e->n0), (uint32_t)(n1 - e->n0), (uint32_t)(t0 - e->t0),
                                          (uint32_t)(t1 - e->t0), static_cast<uint32_t*>(buf), e->stream));
  AV_HIP(hipMemcpyAsync(out, buf, n * 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  AV_PEER_CHECK(e);
  return AV_OK;
}

int av_write_records(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, const uint32_t* in) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  {
    int rc = peer_local_write_check(e);
    if (rc != AV_OK) return rc;
  }
  AV_CHECK(in && n0 >= e->n0 && n0 <= n1 && n1 <= e->n1 && t0 >= e->t0 && t0 <= t1 && t1 <= e->t1,
           AV_ERR_INVALID_ARG, "range outside this engine's shard");
  {
    int rc = materialize_votes(e);
    if (rc != AV_OK) return rc;
  }
  const size_t n = (size_t)(n1 - n0) * (size_t)(t1 - t0);
  if (!n) return AV_OK;
  e->c_monotone = false;
  e->fresh = false;
  e->count_bound = 127;  // arbitrary counts written
  Scratch s;
  AV_HIP(s.ensure(n * 4));
  AV_HIP(hipMemcpyAsync(s.p, in, n * 4, hipMemcpyHostToDevice, e->stream));
  AV_HIP(avk::launch_write_records(e->planes, e->BL, (uint32_t)(n0 - e->n0), (uint32_t)(n1 - e->n0),
                                   (uint32_t)(t0 - e->t0), (uint32_t)(t1 - e->t0), static_cast<uint32_t*>(s.p),
                                   e->stream));
  int rc = refresh_pref(e);
  if (rc != AV_OK) return rc;
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_is_accepted(av_engine* e, int64_t node, int64_t target, int32_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  *out = 0;
  if (!local_node(e, node) || !local_target(e, target)) return AV_OK;  // no record -> false
  uint32_t w = 0;
  int rc = av_read_records(e, node, node + 1, target, target + 1, &w);
  if (rc != AV_OK) return rc;
  if (((w >> 17) < (uint32_t)AV_FINALIZATION_SCORE)) *out = (int32_t)((w >> 16) & 1u);
  return AV_OK;
}

int av_get_confidence(av_engine* e, int64_t node, int64_t target, uint16_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  if (!local_node(e, node) || !local_target(e, target)) return fail(AV_ERR_NOT_FOUND, "VoteRecord not found");
  uint32_t w = 0;
  int rc = av_read_records(e, node, node + 1, target, target + 1, &w);
  if (rc != AV_OK) return rc;
  if ((w >> 17) >= (uint32_t)AV_FINALIZATION_SCORE) return fail(AV_ERR_NOT_FOUND, "VoteRecord not found");
  *out = (uint16_t)(w >> 17);
  return AV_OK;
}

int av_get_invs(av_engine* e, int64_t node, int64_t* out_targets, int64_t cap, int64_t* n_out) {
  AV_CHECK(e && n_out && (cap == 0 || out_targets), AV_ERR_INVALID_ARG, "null argument");
  *n_out = 0;
  AV_CHECK(local_node(e, node), AV_ERR_INVALID_ARG, "node not in this shard");
  std::vector<uint32_t> w((size_t)(e->t1 - e->t0));
  int rc = av_read_records(e, node, node + 1, e->t0, e->t1, w.data());
  if (rc != AV_OK) return rc;
  int64_t cnt = 0;
  for (int64_t tl = 0; tl < (int64_t)w.size() && cnt < AV_MAX_ELEMENT_POLL; ++tl) {
    const bool live = (w[tl] >> 17) < (uint32_t)AV_FINALIZATION_SCORE;
    const bool valid = (e->valid_host[tl >> 5] >> (tl & 31)) & 1u;
    if (!live || !valid) continue;
    if (cnt < cap) out_targets[cnt] = e->t0 + tl;
    cnt++;
  }
  *n_out = cnt;
  AV_CHECK(cnt <= cap, AV_ERR_OVERFLOW, "cap too small (%lld needed)", (long long)cnt);
  return AV_OK;
}

// GetInvsForNextPoll for a node range (processor.go:144-170): counts, their device scan and the CSR
// fill enqueued back to back, the fill writing offsets and targets straight into host-mapped pinned
// staging (coalesced stores): one synchronization per call, then a host copy into the caller's arrays.
int av_get_invs_batch(av_engine* e, int64_t n0, int64_t n1, int64_t* offsets, int32_t* targets, int64_t cap,
                      int64_t* total) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(offsets && total && (cap == 0 || targets), AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(n0 >= e->n0 && n0 <= n1 && n1 <= e->n1, AV_ERR_INVALID_ARG, "node range outside this engine's shard");
  const uint32_t n = (uint32_t)(n1 - n0);
  *total = 0;
  offsets[0] = 0;
  if (!n) return AV_OK;
  // staging: offsets (n + 1 int64) then up to min(cap, the largest possible poll sets) int32 targets
  const uint64_t most = (uint64_t)n * (uint64_t)std::min<int64_t>(AV_MAX_ELEMENT_POLL, e->t1 - e->t0);
  const uint64_t keep = std::min<uint64_t>((uint64_t)std::max<int64_t>(cap, 0), most);
  const size_t hb = ((size_t)n + 1) * 8 + (size_t)keep * 4;
  if (hb > e->invs_host_bytes) {
    if (e->invs_host) AV_HIP(hipHostFree(e->invs_host));
    e->invs_host = nullptr;
    e->invs_host_bytes = 0;
    AV_HIP(hipHostMalloc(&e->invs_host, hb, hipHostMallocMapped));
    e->invs_host_bytes = hb;
  }
  void* dev_view = nullptr;
  AV_HIP(hipHostGetDevicePointer(&dev_view, e->invs_host, 0));
  auto* hoffs = static_cast<int64_t*>(e->invs_host);
  auto* doffs = static_cast<int64_t*>(dev_view);
  void* scratch = nullptr;
  int rc = engine_scratch(e, (size_t)avk::poll_sets_scratch_words(n) * 8, &scratch);
  if (rc != AV_OK) return rc;
  AV_HIP(avk::launch_poll_sets_batch(e->planes, e->valid, e->BL, (uint32_t)(n0 - e->n0), n, (uint32_t)e->t0, keep,
                                     static_cast<uint64_t*>(scratch), doffs, reinterpret_cast<int32_t*>(doffs + n + 1),
                                     e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  *total = hoffs[n];
  std::memcpy(offsets, hoffs, ((size_t)n + 1) * 8);
  AV_CHECK(*total <= cap, AV_ERR_OVERFLOW, "cap too small (%lld needed)", (long long)*total);
  if (*total) std::memcpy(targets, reinterpret_cast<const int32_t*>(hoffs + n + 1), (size_t)*total * 4);
  return AV_OK;
}

int av_run_rounds(av_engine* e, int32_t rounds) {
  AV_ENTER(e);
  AV_PEER_CHECK(e);
  AV_CHECK(rounds >= 0, AV_ERR_INVALID_ARG, "rounds < 0");
  for (int32_t r = 0; r < rounds; ++r) {
    int rc = launch_one_round(e, nullptr);
    if (rc != AV_OK) return rc;
  }
  return AV_OK;
}

int av_replay_round_errs(av_engine* e, const uint32_t* errs) {
  AV_ENTER(e);
  AV_PEER_CHECK(e);
  AV_CHECK(errs, AV_ERR_INVALID_ARG, "null argument");
  e->c_monotone = false;
  const int64_t TL = e->t1 - e->t0;
  std::vector<uint32_t> planes(e->round_replay_words(), 0u);
  for (uint32_t nl = 0; nl < e->NL; ++nl)
    for (int s = 0; s < e->k; ++s) {
      const uint32_t* row = errs + ((size_t)nl * e->k + s) * TL;
      for (uint32_t b = 0; b < e->BL; ++b) {
        uint32_t y = 0, c = 0;
        for (uint32_t i = 0; i < 32; ++i) {
          const int64_t tl = 32ll * b + i;
          if (tl >= TL) break;
          const uint32_t err = row[tl];
          y |= (err == 0u ? 1u : 0u) << i;             // vote.go:55
          c |= ((int32_t)err >= 0 ? 1u : 0u) << i;     // vote.go:56
        }
        const size_t g = (size_t)nl * e->BL + b;
        planes[avk::replay_idx((uint32_t)g, e->k, s, 0)] = y;
        planes[avk::replay_idx((uint32_t)g, e->k, s, 1)] = c;
      }
    }
  Scratch s;
  AV_HIP(s.ensure(planes.size() * 4));
  AV_HIP(hipMemcpyAsync(s.p, planes.data(), planes.size() * 4, hipMemcpyHostToDevice, e->stream));
  int rc = launch_one_round(e, static_cast<uint32_t*>(s.p));
  if (rc != AV_OK) return rc;
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_replay_prepare(av_engine* e, int32_t rounds) {
  AV_ENTER(e);
  AV_CHECK(rounds >= 1, AV_ERR_INVALID_ARG, "rounds < 1");
  const size_t per = e->round_replay_words();
  if (rounds > e->replay_cap_rounds) {
    if (e->replay) AV_HIP(hipFree(e->replay));
    e->replay = nullptr;
    e->replay_cap_rounds = 0;
    hipError_t he = dev_alloc(&e->replay, per * rounds);
    AV_CHECK(he == hipSuccess, he == hipErrorOutOfMemory ? AV_ERR_OOM : AV_ERR_HIP, "alloc replay: %s",
             hipGetErrorString(he));
    e->replay_cap_rounds = rounds;
  }
  for (int32_t r = 0; r < rounds; ++r)
    AV_HIP(avk::launch_gen_replay(e->cfg.seed, (uint32_t)e->n0, e->NL, e->BL, e->L, e->Lpad, (uint32_t)e->t0,
                                  (uint32_t)e->t1, (uint32_t)(e->round + r), e->k, e->replay + per * r, e->stream));
  e->replay_first = e->round;
  e->replay_ready = rounds;
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_replay_rounds(av_engine* e, int32_t rounds) {
  AV_ENTER(e);
  AV_PEER_CHECK(e);
  AV_CHECK(rounds >= 0, AV_ERR_INVALID_ARG, "rounds < 0");
  AV_CHECK(e->round >= e->replay_first && e->round + rounds <= e->replay_first + e->replay_ready,
           AV_ERR_INVALID_ARG, "replay stream not prepared for these rounds");
  if (rounds > 0) e->c_monotone = false;
  const size_t per = e->round_replay_words();
  // capped engines (poll cap binds) fuse consecutive replay rounds: every node's
  // records depend only on its own stream (k_replay_node)
  const bool fuse = e->replay_fuse > 1 && e->kernel == 2 && e->k <= 8 && e->capped && e->pub_mode == 0 &&
                    !e->any_nopoll && e->peer_world <= 1 && !e->comm && e->NL == (uint32_t)e->N;
  for (int32_t r = 0; r < rounds;) {
    const uint32_t* rp = e->replay + per * (size_t)(e->round - e->replay_first);
    const int32_t n = fuse ? std::min<int32_t>(rounds - r, e->replay_fuse) : 1;
    int rc = n > 1 ? launch_replay_fused(e, rp, n) : launch_one_round(e, rp);
    if (rc != AV_OK) return rc;
    r += n;
  }
  return AV_OK;
}

int av_synchronize(av_engine* e) {
  AV_ENTER(e);
  AV_HIP(hipStreamSynchronize(e->stream));
  AV_PEER_CHECK(e);
  return AV_OK;
}

int av_round_index(av_engine* e, int64_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  *out = e->round;
  return AV_OK;
}

int av_get_round(av_engine* e, int64_t node, int64_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(local_node(e, node), AV_ERR_INVALID_ARG, "node %lld not in this shard", (long long)node);
  *out = e->proc_round.empty() ? 0 : e->proc_round[(size_t)(node - e->n0)];
  return AV_OK;
}

int av_set_round(av_engine* e, int64_t node, int64_t round) {
  AV_CHECK(e, AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(local_node(e, node), AV_ERR_INVALID_ARG, "node %lld not in this shard", (long long)node);
  if (e->proc_round.empty()) e->proc_round.assign(e->NL, 0);
  e->proc_round[(size_t)(node - e->n0)] = round;
  return AV_OK;
}

int av_set_polling(av_engine* e, int64_t node, int32_t polls) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  AV_CHECK(local_node(e, node), AV_ERR_INVALID_ARG, "node %lld not in this shard", (long long)node);
  AV_CHECK(e->peer_world <= 1, AV_ERR_UNSUPPORTED, "av_set_polling on a peer-push engine");
  if (e->nopoll_host.empty()) {
    e->nopoll_host.assign((e->NL + 31) / 32, 0u);
    AV_HIP(dev_alloc(&e->nopoll, e->nopoll_host.size()));
  }
  const uint32_t nl = (uint32_t)(node - e->n0);
  uint32_t& w = e->nopoll_host[nl >> 5];
  w = polls ? (w & ~(1u << (nl & 31))) : (w | (1u << (nl & 31)));
  int rc = materialize_votes(e);  // rounds of non-polling networks run the first-generation kernel
  if (rc != AV_OK) return rc;
  AV_HIP(hipMemcpyAsync(e->nopoll, e->nopoll_host.data(), e->nopoll_host.size() * 4, hipMemcpyHostToDevice,
                        e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  e->any_nopoll = false;
  for (uint32_t v : e->nopoll_host) e->any_nopoll |= v != 0;
  return AV_OK;
}

int av_update_round_shift(av_engine* e, int32_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  *out = (int32_t)e->round_shift;
  return AV_OK;
}

int av_log_base_round(av_engine* e, int64_t* out) {
  AV_CHECK(e && out, AV_ERR_INVALID_ARG, "null argument");
  *out = e->log_base;
  return AV_OK;
}

// Reset the three log counters (and the overflow flag) on the engine stream.
int clear_log(av_engine* e) {
  AV_HIP(hipMemsetAsync(e->log_count, 0, (size_t)3 * avk::kLogShards * avk::kCtrStride * 4, e->stream));
  AV_HIP(hipMemsetAsync(e->upd_count, 0, avk::kLogShards * 4, e->stream));
  AV_HIP(hipMemsetAsync(e->log_overflow, 0, 4, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  e->log_base = e->round;
  set_log_layout(e);  // empty now: the shards follow the current sweep grid
  return AV_OK;
}

int av_updates_count(av_engine* e, int64_t* n) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(n, AV_ERR_INVALID_ARG, "null argument");
  std::vector<uint32_t> counts(avk::kLogShards);
  AV_HIP(hipMemcpyAsync(counts.data(), e->upd_count, avk::kLogShards * 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  int64_t total = 0;
  for (uint32_t c : counts) total += c;
  *n = total;
  return AV_OK;
}

int av_update_log_overflowed(av_engine* e, int32_t* out) {
  AV_ENTER(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  uint32_t ovf = 0;
  AV_HIP(hipMemcpyAsync(&ovf, e->log_overflow, 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  *out = ovf ? 1 : 0;
  return AV_OK;
}

// Pending log state: per-shard counters copied to the host.
struct LogCounts {
  std::vector<uint32_t> singles, dense, med, upd;
  uint32_t ovf = 0;
  int64_t total = 0, n_singles = 0, n_records = 0, n_med = 0;
  std::vector<uint64_t> soff, doff, moff;
};

int read_log_counts(av_engine* e, LogCounts& c) {
  c.singles.assign(avk::kLogShards, 0);
  c.dense.assign(avk::kLogShards, 0);
  c.upd.assign(avk::kLogShards, 0);
  c.med.assign(avk::kLogShards, 0);
  // the three kinds' counters, one per 128-B line (kernels.h kCtrStride): copied 2-D, element 0 of each
  AV_HIP(hipMemcpy2DAsync(c.singles.data(), 4, e->log_count, avk::kCtrStride * 4, 4, avk::kLogShards,
                          hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipMemcpy2DAsync(c.dense.data(), 4, e->dlog_count, avk::kCtrStride * 4, 4, avk::kLogShards,
                          hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipMemcpy2DAsync(c.med.data(), 4, e->mlog_count, avk::kCtrStride * 4, 4, avk::kLogShards,
                          hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipMemcpyAsync(c.upd.data(), e->upd_count, avk::kLogShards * 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipMemcpyAsync(&c.ovf, e->log_overflow, 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  c.soff.assign(avk::kLogShards, 0);
  c.doff.assign(avk::kLogShards, 0);
  c.moff.assign(avk::kLogShards, 0);
  for (uint32_t i = 0; i < avk::kLogShards; ++i) {
    c.moff[i] = (uint64_t)c.n_med;
    c.n_med += std::min<uint32_t>(c.med[i], e->mlog_cap);
    c.total += c.upd[i];
    c.soff[i] = (uint64_t)c.n_singles;
    c.n_singles += std::min<uint32_t>(c.singles[i], e->log_cap);
    c.doff[i] = (uint64_t)c.n_records;
    c.n_records += std::min<uint32_t>(c.dense[i], e->dlog_cap);
  }
  return AV_OK;
}

// A sweep-grid option changed the number of log writers: re-shard the log now if it is empty
// (every enqueued round has finished: read_log_counts synchronizes), else at the next clear_log.
int relayout_log_if_empty(av_engine* e) {
  LogCounts c;
  int rc = read_log_counts(e, c);
  if (rc != AV_OK) return rc;
  if (!c.ovf && c.total == 0 && c.n_singles == 0 && c.n_med == 0 && c.n_records == 0) set_log_layout(e);
  return AV_OK;
}

extern "C++" {
namespace {

// n bytes from device memory into the caller's host buffer. Pinned caller memory: one DMA. Pageable
// memory: chunks through two pinned staging buffers, the DMA of chunk i + 1 in flight while host
// threads copy chunk i out (a hipMemcpy into pageable memory is staged by the runtime at ~14.5 GB/s,
// DESIGN.md §4 delivery).
int copy_out_bytes(av_engine* e, void* out, const void* dev, size_t n) {
  if (!n) return AV_OK;
  hipPointerAttribute_t at{};
  bool pinned = false;
  if (hipPointerGetAttributes(&at, out) == hipSuccess) pinned = at.type == hipMemoryTypeHost;
  (void)hipGetLastError();
  constexpr size_t kChunk = (size_t)64 << 20;  // bytes
  if (pinned || n <= (size_t)4 << 20) {
    AV_HIP(hipMemcpyAsync(out, dev, n, hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipStreamSynchronize(e->stream));
    return AV_OK;
  }
  for (int i = 0; i < 2; ++i) {
    if (!e->stage[i]) AV_HIP(hipHostMalloc(&e->stage[i], kChunk, hipHostMallocDefault));
    if (!e->stage_ev[i]) AV_HIP(hipEventCreateWithFlags(&e->stage_ev[i], hipEventDisableTiming));
  }
  const size_t chunks = (n + kChunk - 1) / kChunk;
  const char* src_dev = static_cast<const char*>(dev);
  auto dma = [&](size_t c) -> int {
    const size_t w = std::min(kChunk, n - c * kChunk);
    AV_HIP(hipMemcpyAsync(e->stage[c & 1], src_dev + c * kChunk, w, hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipEventRecord(e->stage_ev[c & 1], e->stream));
    return AV_OK;
  };
  int rc = dma(0);
  if (rc != AV_OK) return rc;
  for (size_t c = 0; c < chunks; ++c) {
    if (c + 1 < chunks) {
      rc = dma(c + 1);  // its staging buffer's previous chunk (c - 1) was copied out already
      if (rc != AV_OK) return rc;
    }
    AV_HIP(hipEventSynchronize(e->stage_ev[c & 1]));
    const size_t w = std::min(kChunk, n - c * kChunk);
    const char* src = static_cast<const char*>(e->stage[c & 1]);
    char* dst = static_cast<char*>(out) + c * kChunk;
    parallel_chunks((int64_t)w, 1 << 21, [&](int, int64_t a, int64_t b) {
      std::memcpy(dst + a, src + a, (size_t)(b - a));
    });
  }
  return AV_OK;
}

int copy_out(av_engine* e, uint64_t* out, const uint64_t* dev, size_t n) { return copy_out_bytes(e, out, dev, n * 8); }

// ---- canonical StatusUpdate order on the device (log_ops.hip launch_encode_log) ----
constexpr uint32_t kChunkNodes = 4096;         // compact index granularity (nodes per index entry)
constexpr size_t kHdrBytes = sizeof(av_compact_header);

uint32_t bits_for(uint64_t n) {  // bits of the values 0 .. n - 1
  uint32_t b = 0;
  while (b < 32 && (1ull << b) < n) ++b;
  return b;
}

struct Encoded {
  int64_t updates = 0;
  int64_t bytes = 0;  // compact: the whole stream, header included
  av_compact_header hdr{};
};

// Rounds the pending log can hold (round_rel < this)
uint32_t log_rounds(const av_engine* e) { return (uint32_t)std::max<int64_t>(e->round - e->log_base, 1); }

avk::EncodeParams encode_params(av_engine* e) {
  avk::EncodeParams p{};
  p.log = e->log;
  p.mlog = e->mlog;
  p.dlog = e->dlog;
  p.log_count = e->log_count;
  p.log_cap = e->log_cap;
  p.mlog_cap = e->mlog_cap;
  p.dlog_cap = e->dlog_cap;
  p.shards = e->log_shards;
  p.K = (uint32_t)e->k;
  p.n0 = (uint32_t)e->n0;
  p.NL = e->NL;
  p.BL = e->BL;
  p.t0 = (uint32_t)e->t0;
  p.r_total = log_rounds(e);
  p.round_shift = e->round_shift;
  const uint32_t tb = bits_for((uint64_t)(e->t1 - e->t0)), sb = bits_for((uint64_t)e->k);
  p.target_bits = tb;
  p.code_bytes = sb + tb + 2 <= 16 ? 2u : 4u;
  p.err = e->enc_err;
  return p;
}

// Device bytes a compact stream of the pending log needs at most (c: the log's counts).
size_t compact_bound(const av_engine* e, const avk::EncodeParams& p, const LogCounts& c) {
  const uint64_t R = p.r_total, chunks = (e->NL + kChunkNodes - 1) / kChunkNodes;
  const uint64_t entries = (uint64_t)(c.n_singles + c.n_med + c.n_records);
  const uint64_t groups = std::min<uint64_t>(R * e->NL, entries);
  return kHdrBytes + (size_t)(R * chunks + 1) * 16 + (size_t)groups * 12 + (size_t)c.total * p.code_bytes + 256;
}

// Encode the pending log (counts c) into dev: packed words (compact = false; dev holds c.total u64)
// or the compact stream (dev: compact_bound bytes; the header is returned, not written). Enqueued on
// the engine stream; synchronizes once per encoder pass (a log spanning more (round, node) buckets
// than one pass holds takes several) and checks that every counted update was laid out.
int encode_log(av_engine* e, const LogCounts& c, bool compact, void* dev, Encoded* res) {
  *res = Encoded{};
  if (!e->enc_err) AV_HIP(dev_alloc(&e->enc_err, 1));
  if (!e->enc_tot) AV_HIP(dev_alloc(&e->enc_tot, 4));
  avk::EncodeParams p = encode_params(e);
  const uint32_t R = p.r_total;
  const uint32_t per = std::max<uint32_t>(1, std::min<uint32_t>(R, e->enc_buckets / std::max<uint32_t>(e->NL, 1)));
  const uint64_t entries = (uint64_t)(c.n_singles + c.n_med + c.n_records);
  AV_CHECK(entries < (1ull << 40), AV_ERR_UNSUPPORTED, "StatusUpdate log too large to order");
  p.nr = per;
  void* scratch = nullptr;
  int rc = engine_scratch(e, avk::encode_scratch_bytes(p, entries, per * e->NL), &scratch);
  if (rc != AV_OK) return rc;
  const uint32_t chunks = (e->NL + kChunkNodes - 1) / kChunkNodes;
  auto* base = static_cast<uint8_t*>(dev);
  uint64_t* cidx = compact ? reinterpret_cast<uint64_t*>(base + kHdrBytes) : nullptr;
  uint8_t* groups = compact ? base + kHdrBytes + (size_t)((uint64_t)R * chunks + 1) * 16 : nullptr;
  AV_HIP(hipMemsetAsync(e->enc_err, 0, 4, e->stream));
  uint64_t ubase = 0, cbase = 0;
  for (uint32_t r0 = 0; r0 < R; r0 += per) {
    p.r0 = r0;
    p.nr = std::min(per, R - r0);
    const bool last = r0 + p.nr >= R;
    AV_HIP(avk::launch_encode_log(p, entries, scratch, compact ? nullptr : static_cast<uint64_t*>(dev), groups, cidx,
                                  chunks, kChunkNodes, ubase, cbase, last, e->enc_tot, e->stream));
    uint64_t tot[4] = {0, 0, 0, 0};
    uint32_t err = 0;
    AV_HIP(hipMemcpyAsync(tot, e->enc_tot, sizeof(tot), hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipMemcpyAsync(&err, e->enc_err, 4, hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipStreamSynchronize(e->stream));
    AV_CHECK(err == 0, AV_ERR_HIP, "StatusUpdate log inconsistent (encoder flags %u)", err);
    ubase += tot[0];
    cbase += tot[1];
  }
  AV_CHECK((int64_t)ubase == c.total, AV_ERR_HIP, "StatusUpdate log inconsistent (%lld of %lld updates ordered)",
           (long long)ubase, (long long)c.total);
  res->updates = (int64_t)ubase;
  if (compact) {
    av_compact_header& h = res->hdr;
    h.magic = AV_COMPACT_MAGIC;
    h.version = AV_COMPACT_VERSION;
    h.log_base = e->log_base;
    h.n_updates = (int64_t)ubase;
    h.node_base = e->n0;
    h.target_base = e->t0;
    h.n_rounds = (int32_t)R;
    h.chunks = (int32_t)chunks;
    h.chunk_nodes = (int32_t)kChunkNodes;
    h.code_bytes = (int32_t)p.code_bytes;
    h.target_bits = (int32_t)p.target_bits;
    h.slot_bits = (int32_t)bits_for((uint64_t)e->k);
    h.round_shift = (int32_t)e->round_shift;
    h.bytes = (int64_t)(groups - base) + (int64_t)cbase;
    res->bytes = h.bytes;
  }
  return AV_OK;
}

// Grow a device buffer (contents not kept).
int grow_dev(void** p, size_t* have, size_t want) {
  if (want <= *have) return AV_OK;
  if (*p) AV_HIP(hipFree(*p));
  *p = nullptr;
  *have = 0;
  want = std::max(want + want / 8, (size_t)1 << 20);
  hipError_t he = hipMalloc(p, want);
  AV_CHECK(he == hipSuccess, he == hipErrorOutOfMemory ? AV_ERR_OOM : AV_ERR_HIP, "device buffer (%zu B): %s", want,
           hipGetErrorString(he));
  *have = want;
  return AV_OK;
}
int grow_pinned(void** p, size_t* have, size_t want) {
  if (want <= *have) return AV_OK;
  if (*p) AV_HIP(hipHostFree(*p));
  *p = nullptr;
  *have = 0;
  want = std::max(want + want / 8, (size_t)1 << 20);
  AV_HIP(hipHostMalloc(p, want, hipHostMallocMapped));
  *have = want;
  return AV_OK;
}

// Read the log's counters, failing (and clearing the log) if it overflowed.
int pending_counts(av_engine* e, LogCounts& c) {
  int rc = read_log_counts(e, c);
  if (rc != AV_OK) return rc;
  if (c.ovf) {
    rc = clear_log(e);
    if (rc != AV_OK) return rc;
    return fail(AV_ERR_OVERFLOW, "device StatusUpdate log overflowed (%lld updates, capacity %lld per shard)",
                (long long)c.total, (long long)e->log_cap);
  }
  return AV_OK;
}

}  // namespace
}  // extern "C++"

int av_fetch_updates(av_engine* e, uint64_t* out, int64_t cap, int64_t* n_out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(n_out && (cap == 0 || out), AV_ERR_INVALID_ARG, "null argument");
  LogCounts c;
  int rc = pending_counts(e, c);
  *n_out = c.total;
  if (rc != AV_OK) return rc;
  AV_CHECK(c.total <= cap, AV_ERR_OVERFLOW, "cap too small: %lld updates pending", (long long)c.total);
  if (c.total > 0) {
    // the compact slots' device buffers hold no in-flight copy source after this wait
    if (e->copy_stream) AV_HIP(hipStreamSynchronize(e->copy_stream));
    rc = grow_dev(&e->cdev[0], &e->cdev_bytes[0], (size_t)c.total * 8);
    if (rc != AV_OK) return rc;
    Encoded r;
    rc = encode_log(e, c, false, e->cdev[0], &r);
    if (rc != AV_OK) return rc;
    rc = copy_out(e, out, static_cast<const uint64_t*>(e->cdev[0]), (size_t)c.total);
    if (rc != AV_OK) return rc;
  }
  return clear_log(e);
}

int av_fetch_compact(av_engine* e, void* out, int64_t cap, int64_t* bytes) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(bytes && (cap == 0 || out), AV_ERR_INVALID_ARG, "null argument");
  *bytes = 0;
  LogCounts c;
  int rc = pending_counts(e, c);
  if (rc != AV_OK) return rc;
  if (e->copy_stream) AV_HIP(hipStreamSynchronize(e->copy_stream));
  const avk::EncodeParams p = encode_params(e);
  rc = grow_dev(&e->cdev[0], &e->cdev_bytes[0], compact_bound(e, p, c));
  if (rc != AV_OK) return rc;
  Encoded r;
  rc = encode_log(e, c, true, e->cdev[0], &r);
  if (rc != AV_OK) return rc;
  *bytes = r.bytes;
  AV_CHECK(r.bytes <= cap, AV_ERR_OVERFLOW, "cap too small: the stream takes %lld bytes", (long long)r.bytes);
  rc = copy_out_bytes(e, static_cast<uint8_t*>(out) + kHdrBytes, static_cast<const uint8_t*>(e->cdev[0]) + kHdrBytes,
                      (size_t)r.bytes - kHdrBytes);
  if (rc != AV_OK) return rc;
  std::memcpy(out, &r.hdr, kHdrBytes);
  return clear_log(e);
}

int av_fetch_compact_async(av_engine* e, int64_t* ticket) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(ticket, AV_ERR_INVALID_ARG, "null argument");
  if (!e->copy_stream) AV_HIP(hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking));
  const int s = (int)(e->cticket % av_engine::kSlots);
  if (!e->cev[s]) AV_HIP(hipEventCreateWithFlags(&e->cev[s], hipEventDisableTiming));
  LogCounts c;
  int rc = pending_counts(e, c);  // waits for the rounds enqueued before
  if (rc != AV_OK) return rc;
  // the slot's previous copy (ticket - kSlots) has read its device buffer and filled its host buffer
  if (e->cpend[s]) AV_HIP(hipEventSynchronize(e->cev[s]));
  e->cpend[s] = false;
  const avk::EncodeParams p = encode_params(e);
  e->cdev_hwm = std::max(e->cdev_hwm, compact_bound(e, p, c));
  rc = grow_dev(&e->cdev[s], &e->cdev_bytes[s], e->cdev_hwm);
  if (rc != AV_OK) return rc;
  Encoded r;
  rc = encode_log(e, c, true, e->cdev[s], &r);  // synchronizes the engine stream
  if (rc != AV_OK) return rc;
  e->chost_hwm = std::max(e->chost_hwm, (size_t)r.bytes + 16);
  rc = grow_pinned(&e->chost[s], &e->chost_bytes[s], e->chost_hwm);
  if (rc != AV_OK) return rc;
  if (e->copy_blocks) {  // a small copy kernel (the header's bytes are copied too, and overwritten on wait)
    void* hdev = nullptr;
    AV_HIP(hipHostGetDevicePointer(&hdev, e->chost[s], 0));
    AV_HIP(avk::launch_stream_out(e->cdev[s], hdev, (uint64_t)r.bytes, e->copy_blocks, e->copy_stream));
  } else {
    AV_HIP(hipMemcpyAsync(static_cast<uint8_t*>(e->chost[s]) + kHdrBytes,
                          static_cast<const uint8_t*>(e->cdev[s]) + kHdrBytes, (size_t)r.bytes - kHdrBytes,
                          hipMemcpyDeviceToHost, e->copy_stream));
  }
  AV_HIP(hipEventRecord(e->cev[s], e->copy_stream));
  e->chdr[s] = r.hdr;
  e->cpend[s] = true;
  *ticket = e->cticket++;
  return clear_log(e);
}

int av_fetch_compact_wait(av_engine* e, int64_t ticket, const void** stream, int64_t* bytes) {
  AV_ENTER(e);
  AV_CHECK(stream && bytes, AV_ERR_INVALID_ARG, "null argument");
  AV_CHECK(ticket >= 0 && ticket < e->cticket && ticket >= e->cticket - av_engine::kSlots, AV_ERR_INVALID_ARG,
           "ticket %lld is not one of the last %d issued", (long long)ticket, av_engine::kSlots);
  const int s = (int)(ticket % av_engine::kSlots);
  AV_CHECK(e->cpend[s], AV_ERR_INVALID_ARG, "ticket %lld has no copy", (long long)ticket);
  AV_HIP(hipEventSynchronize(e->cev[s]));
  std::memcpy(e->chost[s], &e->chdr[s], kHdrBytes);
  *stream = e->chost[s];
  *bytes = e->chdr[s].bytes;
  return AV_OK;
}

int av_compact_expand(const void* stream, int64_t bytes, uint64_t* out, int64_t cap, int64_t* n_out) {
  AV_CHECK(stream && n_out && (cap == 0 || out), AV_ERR_INVALID_ARG, "null argument");
  *n_out = 0;
  AV_CHECK(bytes >= (int64_t)kHdrBytes, AV_ERR_INVALID_ARG, "stream shorter than its header");
  av_compact_header h;
  std::memcpy(&h, stream, kHdrBytes);
  AV_CHECK(h.magic == AV_COMPACT_MAGIC && h.version == AV_COMPACT_VERSION, AV_ERR_INVALID_ARG, "not a compact stream");
  AV_CHECK(h.bytes == bytes && h.n_rounds >= 1 && h.chunks >= 1 && (h.code_bytes == 2 || h.code_bytes == 4) &&
               h.target_bits >= 0 && h.target_bits <= 22 && h.n_updates >= 0 && h.round_shift >= 52 &&
               h.round_shift <= 60 && h.n_rounds <= (1ll << (64 - h.round_shift)),
           AV_ERR_INVALID_ARG, "malformed compact stream header");
  const uint64_t n_idx = (uint64_t)h.n_rounds * (uint64_t)h.chunks + 1;
  const uint8_t* base = static_cast<const uint8_t*>(stream);
  const uint64_t gstart = kHdrBytes + n_idx * 16;
  AV_CHECK((uint64_t)bytes >= gstart, AV_ERR_INVALID_ARG, "compact stream index truncated");
  const uint64_t* idx = reinterpret_cast<const uint64_t*>(base + kHdrBytes);
  AV_CHECK(idx[2 * (n_idx - 1)] == (uint64_t)bytes - gstart && idx[2 * (n_idx - 1) + 1] == (uint64_t)h.n_updates,
           AV_ERR_INVALID_ARG, "compact stream index inconsistent");
  *n_out = h.n_updates;
  AV_CHECK(h.n_updates <= cap, AV_ERR_OVERFLOW, "cap too small: %lld updates", (long long)h.n_updates);
  const uint8_t* groups = base + gstart;
  const uint32_t tb = (uint32_t)h.target_bits, cw = (uint32_t)h.code_bytes;
  const uint32_t tmask = (1u << tb) - 1u;
  std::vector<int> bad(64, 0);
  parallel_chunks((int64_t)(n_idx - 1), 1, [&](int t, int64_t j0, int64_t j1) {
    for (int64_t j = j0; j < j1; ++j) {
      const uint64_t rr = (uint64_t)j / (uint64_t)h.chunks;
      const uint64_t b0 = idx[2 * j], b1 = idx[2 * j + 2];
      uint64_t u = idx[2 * j + 1];
      const uint64_t u1 = idx[2 * j + 3];
      if (b0 > b1 || b1 > (uint64_t)bytes - gstart || u > u1) {
        bad[t] = 1;
        return;
      }
      for (uint64_t at = b0; at < b1;) {
        if (at + 8 > b1) {
          bad[t] = 1;
          return;
        }
        uint32_t node, n;
        std::memcpy(&node, groups + at, 4);
        std::memcpy(&n, groups + at + 4, 4);
        const uint64_t len = 8 + (((uint64_t)n * cw + 3) & ~3ull);
        if (at + len > b1 || u + n > u1 || (uint64_t)node >= (1ull << (h.round_shift - 28))) {
          bad[t] = 1;
          return;
        }
        const uint64_t hi = (rr << h.round_shift) | ((uint64_t)node << 28);
        const uint8_t* cp = groups + at + 8;
        for (uint32_t i = 0; i < n; ++i) {
          uint32_t code;
          if (cw == 2) {
            uint16_t v;
            std::memcpy(&v, cp + 2 * i, 2);
            code = v;
          } else {
            std::memcpy(&code, cp + 4 * i, 4);
          }
          const uint64_t slot = code >> (tb + 2), tl = (code >> 2) & tmask;
          out[u + i] = hi | (slot << 24) | (((uint64_t)h.target_base + tl) << 2) | (code & 3u);
        }
        u += n;
        at += len;
      }
      if (u != u1) {
        bad[t] = 1;
        return;
      }
    }
  });
  for (int b : bad) AV_CHECK(!b, AV_ERR_INVALID_ARG, "malformed compact stream groups");
  return AV_OK;
}

int av_updates_digest(av_engine* e, uint64_t out[3]) { return av_updates_digest_range(e, 0, e ? e->N : 0, out); }

int av_updates_digest_range(av_engine* e, int64_t n0, int64_t n1, uint64_t out[3]) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out && n0 >= 0 && n0 <= n1 && n1 <= e->N, AV_ERR_INVALID_ARG, "bad argument");
  uint32_t ovf = 0;
  AV_HIP(hipMemcpyAsync(&ovf, e->log_overflow, 4, hipMemcpyDeviceToHost, e->stream));
  if (!e->digest) AV_HIP(dev_alloc(&e->digest, 3));
  AV_HIP(avk::launch_log_digest(e->log, e->log_count, e->log_cap, e->dlog, e->dlog_count, e->dlog_cap, e->mlog,
                                e->mlog_count, e->mlog_cap, e->log_shards, (uint32_t)e->k, (uint32_t)n0, (uint32_t)n1,
                                e->round_shift, e->digest, e->stream));
  unsigned long long d[3] = {0, 0, 0};
  AV_HIP(hipMemcpyAsync(d, e->digest, sizeof(d), hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  AV_CHECK(!ovf, AV_ERR_OVERFLOW, "device StatusUpdate log overflowed: the digest would miss updates");
  for (int i = 0; i < 3; ++i) out[i] = (uint64_t)d[i];
  return AV_OK;
}

int av_applied_votes(av_engine* e, int64_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  std::vector<unsigned long long> c(avk::kLogShards);
  AV_HIP(hipMemcpyAsync(c.data(), e->applied, avk::kLogShards * 8, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  unsigned long long t = 0;
  for (auto v : c) t += v;
  *out = (int64_t)t;
  return AV_OK;
}

static int sum_counter(av_engine* e, const unsigned long long* dev, int64_t* out) {
  std::vector<unsigned long long> c(avk::kLogShards);
  AV_HIP(hipMemcpyAsync(c.data(), dev, avk::kLogShards * 8, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  unsigned long long t = 0;
  for (auto v : c) t += v;
  *out = (int64_t)t;
  return AV_OK;
}

int av_finalized_count(av_engine* e, int64_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  return sum_counter(e, e->finalized, out);
}

int av_live_records(av_engine* e, int32_t honest_only, int64_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  AV_HIP(hipMemsetAsync(e->scratch_count, 0, 8, e->stream));
  AV_HIP(avk::launch_count_live(e->planes, e->valid, e->byz, (uint32_t)e->n0, e->BL, e->L, honest_only,
                                e->scratch_count, e->stream));
  unsigned long long v = 0;
  AV_HIP(hipMemcpyAsync(&v, e->scratch_count, 8, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  *out = (int64_t)v;
  return AV_OK;
}

int av_discard_updates(av_engine* e) {
  AV_ENTER(e);
  return clear_log(e);
}

int av_log_entries(av_engine* e, int64_t out[3]) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  LogCounts c;
  int rc = read_log_counts(e, c);
  if (rc != AV_OK) return rc;
  out[0] = c.n_singles;
  out[1] = c.n_med;
  out[2] = c.n_records;
  return AV_OK;
}

int av_resize_log(av_engine* e, const int64_t entries[3]) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(entries && entries[0] >= 0 && entries[1] >= 0 && entries[2] >= 0, AV_ERR_INVALID_ARG, "bad entries");
  LogCounts c;
  int rc = read_log_counts(e, c);
  if (rc != AV_OK) return rc;
  AV_CHECK(!c.ovf && c.total == 0 && c.n_singles == 0 && c.n_med == 0 && c.n_records == 0, AV_ERR_UNSUPPORTED,
           "av_resize_log: the log holds updates (fetch or discard them first)");
  // sized for the current grid's writer waves (log_writer_waves): a shard takes every sh-th writer, so
  // with w writers one shard serves up to ceil(w / sh) of them; each writer gets ceil(n / w) + 1 entries
  // (a writer owns one run of lanes, at most one more than the lanes' mean: "one entry per lane" holds
  // any round), >= 16 per shard. The allocation is that per-shard share times kLogShards, so that a
  // later re-layout to more shards keeps the total.
  const uint64_t sh = avk::kLogShards;
  const uint64_t w = std::max<uint64_t>(log_writer_waves(e), 1), lsh = log_shards_for(w);
  auto per = [&](int64_t n) {
    const uint64_t shard = (((uint64_t)n + w - 1) / w + 1) * ((w + lsh - 1) / lsh);
    return std::max<uint64_t>((shard * lsh + sh - 1) / sh, 16);
  };
  const uint64_t s1 = per(entries[0]) * sh, s2 = per(entries[1]) * sh, s3 = per(entries[2]) * sh;
  AV_CHECK(s1 / sh < (1ull << 32) && s2 / sh < (1ull << 32) && s3 / sh < (1ull << 32), AV_ERR_INVALID_ARG,
           "log too large");
  AV_HIP(hipStreamSynchronize(e->stream));
  AV_HIP(hipFree(e->log));
  AV_HIP(hipFree(e->mlog));
  AV_HIP(hipFree(e->dlog));
  e->log = nullptr;
  e->mlog = nullptr;
  e->dlog = nullptr;
  hipError_t he = dev_alloc(&e->log, s1);
  if (he == hipSuccess) he = dev_alloc(&e->mlog, s2 * avk::med_rec_words());
  if (he == hipSuccess) he = dev_alloc(&e->dlog, s3 * avk::dense_words((uint32_t)e->k));
  if (he != hipSuccess) {  // leave a usable minimal log behind
    (void)hipGetLastError();
    if (!e->log) (void)dev_alloc(&e->log, sh * 16);
    if (!e->mlog) (void)dev_alloc(&e->mlog, sh * 16 * avk::med_rec_words());
    if (!e->dlog) (void)dev_alloc(&e->dlog, sh * 16 * avk::dense_words((uint32_t)e->k));
    e->log_alloc = e->mlog_alloc = e->dlog_alloc = sh * 16;
    set_log_layout(e);
    return fail(he == hipErrorOutOfMemory ? AV_ERR_OOM : AV_ERR_HIP, "av_resize_log: %s", hipGetErrorString(he));
  }
  e->log_alloc = s1;
  e->mlog_alloc = s2;
  e->dlog_alloc = s3;
  set_log_layout(e);
  return AV_OK;
}

namespace {
int sum_byte_counters(av_engine* e, size_t first, int64_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  std::vector<unsigned long long> c(avk::kLogShards);
  AV_HIP(hipMemcpyAsync(c.data(), e->bytes + first, avk::kLogShards * 8, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  unsigned long long t = 0;
  for (auto v : c) t += v;
  *out = (int64_t)t;
  return AV_OK;
}
}  // namespace

int av_alg_bytes(av_engine* e, int64_t* out) { return sum_byte_counters(e, 0, out); }

int av_alg_bytes_reread(av_engine* e, int64_t* out) { return sum_byte_counters(e, avk::kLogShards, out); }

int av_changed_words(av_engine* e, int64_t* words, int64_t* segments) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(words, AV_ERR_INVALID_ARG, "null argument");
  int rc = sum_counter(e, e->changed, words);
  if (rc != AV_OK || !segments) return rc;
  return sum_counter(e, e->changed + avk::kLogShards, segments);
}

int av_materialize(av_engine* e) {
  AV_ENTER(e);
  AV_PEER_CHECK(e);
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  if (e->timing && (e->v_stale || e->k_pend)) {
    AV_HIP(hipEventCreate(&ev0));
    AV_HIP(hipEventCreate(&ev1));
    AV_HIP(hipEventRecord(ev0, e->stream));
  }
  int rc = materialize_votes(e);
  if (rc != AV_OK) return rc;
  if (ev0) {
    AV_HIP(hipEventRecord(ev1, e->stream));
    e->events.emplace_back(ev0, ev1);
  }
  return AV_OK;
}

int av_read_pref(av_engine* e, int64_t n0, int64_t n1, int64_t t0, int64_t t1, uint8_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out && n0 >= 0 && n0 <= n1 && n1 <= e->N && t0 >= e->t0 && t0 <= t1 && t1 <= e->t1,
           AV_ERR_INVALID_ARG, "bad range");
  const size_t rows = (size_t)(n1 - n0);
  std::vector<uint32_t> w(rows * e->BL);
  if (rows) {
    AV_HIP(hipMemcpy2DAsync(w.data(), (size_t)e->BL * 4, e->pref[e->cur] + (size_t)n0 * e->PS, (size_t)e->PS * 4,
                            (size_t)e->BL * 4, rows, hipMemcpyDeviceToHost, e->stream));
    AV_HIP(hipStreamSynchronize(e->stream));
  }
  const int64_t W = t1 - t0;
  for (size_t r = 0; r < rows; ++r)
    for (int64_t t = t0; t < t1; ++t) {
      const int64_t tl = t - e->t0;
      out[r * W + (t - t0)] = (uint8_t)((w[r * e->BL + (tl >> 5)] >> (tl & 31)) & 1u);
    }
  return AV_OK;
}

int av_read_pref_words(av_engine* e, int64_t n0, int64_t n1, uint32_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out && n0 >= 0 && n0 <= n1 && n1 <= e->N, AV_ERR_INVALID_ARG, "bad range");
  const size_t words = (size_t)(n1 - n0) * e->BL;
  if (!words) return AV_OK;
  AV_HIP(hipMemcpy2DAsync(out, (size_t)e->BL * 4, e->pref[e->cur] + (size_t)n0 * e->PS, (size_t)e->PS * 4,
                          (size_t)e->BL * 4, (size_t)(n1 - n0), hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_sample_peers(av_engine* e, int64_t round, int64_t n0, int64_t n1, int32_t* out) {
  AV_ENTER(e);
  AV_CHECK(out && n0 >= 0 && n0 <= n1 && n1 <= e->N && round >= 0, AV_ERR_INVALID_ARG, "bad range");
  const size_t n = (size_t)(n1 - n0) * e->k;
  if (!n) return AV_OK;
  Scratch s;
  AV_HIP(s.ensure(n * 4));
  AV_HIP(avk::launch_sample_peers(e->cfg.seed, (uint32_t)e->N, (uint32_t)n0, (uint32_t)n1, (uint32_t)round, e->k,
                                  e->cfg.peer_mode, static_cast<uint32_t*>(s.p), e->stream));
  AV_HIP(hipMemcpyAsync(out, s.p, n * 4, hipMemcpyDeviceToHost, e->stream));
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_set_option(av_engine* e, const char* name, int64_t value) {
  if (e) ref_invalidate(e);
  AV_CHECK(e && name, AV_ERR_INVALID_ARG, "null argument");
  const std::string n(name);
  if (n == "plane_nt") {
    e->plane_nt = value != 0;
  } else if (n == "ablate_phase") {  // diagnostics (kernels.h RoundParams::ablate_phase; results invalid)
    e->ablate_phase = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(31, value));
  } else if (n == "ablate_emit") {
    e->ablate_emit = (int)std::max<int64_t>(0, std::min<int64_t>(3, value));
  } else if (n == "k_hi_virtual") {  // A/B: virtual K4..K7 group (kernels.h kHiVirt)
    int rc = materialize_counts(e);
    if (rc != AV_OK) return rc;
    e->k_hi_virtual = value != 0;
  } else if (n == "uni_merge") {  // tuning: runs per wave in a uniform-input round (1 = off)
    AV_CHECK(value >= 1 && value <= 16, AV_ERR_INVALID_ARG, "bad uni_merge");
    e->uni_merge = (uint32_t)value;
  } else if (n == "uniform_rows") {  // A/B: uniform-row settled tests (kernels.h uni_*)
    e->uni_rows = value != 0;
    ref_invalidate(e);
  } else if (n == "ref_rows") {  // reference-row flags in converged sweep rounds (kernels.h)
    e->ref_rows = value != 0;
  } else if (n == "replay_fuse") {  // replay rounds per fused launch on capped engines (<= 1: one launch per round)
    AV_CHECK(value >= 0 && value <= 4096, AV_ERR_INVALID_ARG, "replay_fuse must be in [0, 4096]");
    e->replay_fuse = (int)value;
  } else if (n == "ablate_node") {
    e->ablate_node = (uint32_t)std::max<int64_t>(0, std::min<int64_t>(7, value));
  } else if (n == "ablate_gather") {
    e->ablate_gather = value != 0;
  } else if (n == "kernel") {  // 2 = k_round_sweep (default where it applies), 1 = k_round_fast
    AV_CHECK(value == 1 || value == 2, AV_ERR_INVALID_ARG, "kernel must be 1 or 2");
    e->kernel = (int)value;
  } else if (n == "store_policy") {
    AV_CHECK(value >= 0 && value <= 3, AV_ERR_INVALID_ARG, "store_policy must be in [0, 3]");
    e->store_policy = (uint32_t)value;
  } else if (n == "sweep_blocks") {  // 0 = one wave per tile, -1 = the default choice, -2 = resident grid
    AV_CHECK(value >= -2 && value < (1ll << 31), AV_ERR_INVALID_ARG, "bad sweep_blocks");
    if (value < 0) {
      AV_ENTER(e);
      e->sweep_blocks = default_sweep_blocks(e, value == -2);
      e->sweep_blocks_explicit = false;
    } else {
      e->sweep_blocks = (uint32_t)value;
      e->sweep_blocks_explicit = true;
    }
    AV_ENTER(e);
    int rc = relayout_log_if_empty(e);
    if (rc != AV_OK) return rc;
  } else if (n == "settled_fast") {
    e->settled_fast = value != 0;
  } else if (n == "replay_fast") {
    e->replay_fast = value != 0;
  } else if (n == "count_changed") {  // diagnostics: count changed published words in every sweep round
    e->count_changed = value != 0;
  } else if (n == "solo_barrier") {  // diagnostics: a one-rank barrier after every round (exchange_cost.py)
    AV_CHECK(e->peer_world <= 1 && !e->comm, AV_ERR_UNSUPPORTED, "solo_barrier: engine has an exchange");
    if (value && !e->arrive) {
      AV_ENTER(e);
      int rc = alloc_arrival(e);
      if (rc != AV_OK) return rc;
      e->peer_arrive.p[0] = e->arrive;
    }
    e->solo_barrier = value != 0;
    e->solo_used = e->solo_used || e->solo_barrier;
  } else if (n == "copy_blocks") {
    AV_CHECK(value >= 0 && value <= 4096, AV_ERR_INVALID_ARG, "copy_blocks must be in [0, 4096]");
    e->copy_blocks = (uint32_t)value;
  } else if (n == "enc_buckets") {  // (round, node) buckets per encoder pass (tests of the multi-pass path)
    AV_CHECK(value >= 1 && value <= (1ll << 30), AV_ERR_INVALID_ARG, "enc_buckets must be in [1, 2^30]");
    e->enc_buckets = (uint32_t)value;
  } else if (n == "dropin_fast") {
    e->dropin_fast = value != 0;
  } else if (n == "settled_lean") {
    e->settled_lean = value != 0;
  } else if (n == "wave_runs") {
    e->wave_runs = value != 0;
  } else if (n == "sweep_nopipe") {
    e->sweep_nopipe = value != 0;
  } else if (n == "tiles_per_wave") {
    AV_CHECK(value >= 0 && value <= 4096, AV_ERR_INVALID_ARG, "bad tiles_per_wave");
    e->tiles_per_wave = (uint32_t)value;
    // the default grid depends on the run length; an explicit sweep_blocks stays as set
    if (!e->sweep_blocks_explicit) e->sweep_blocks = default_sweep_blocks(e);
    AV_ENTER(e);
    int rc = relayout_log_if_empty(e);
    if (rc != AV_OK) return rc;
  } else if (n == "unsynced_shard") {
    e->unsynced_shard = value != 0;
  } else if (n == "warm_pref") {
    e->warm_pref = value != 0;
  } else if (n == "round_marker") {
    e->round_marker = value != 0;
  } else if (n == "virtual_votes") {  // 0: always store the vote planes (A/B)
    e->virtual_votes = value != 0;
  } else if (n == "count_lazy") {  // 0: always store the count planes (A/B)
    AV_ENTER(e);
    int rc = materialize_counts(e);
    if (rc != AV_OK) return rc;
    e->count_lazy = value != 0;
  } else if (n == "vv_min_bl") {
    AV_CHECK(value >= 1 && value < (1ll << 31), AV_ERR_INVALID_ARG, "bad vv_min_bl");
    e->vv_min_bl = (uint32_t)value;
  } else if (n == "responder") {  // 0 = R2 decision, 1 = IsAccepted literally, 2 = the example's responder
    AV_ENTER(e);
    AV_CHECK(value >= 0 && value <= 2, AV_ERR_INVALID_ARG, "responder must be 0, 1 or 2");
    AV_CHECK(value != 2 || (e->NL == (uint32_t)e->N && e->t0 == 0 && e->t1 == e->M && e->peer_world <= 1 && !e->comm),
             AV_ERR_UNSUPPORTED, "the example responder (re-adds) needs an unsharded engine");
    AV_CHECK(value == 0 || e->peer_world <= 1, AV_ERR_UNSUPPORTED, "responder variants on a peer-push engine");
    if (value == 2 && !e->readd) {
      AV_HIP(dev_alloc(&e->readd, e->L));
      AV_HIP(dev_alloc(&e->died_out, e->L));
      AV_HIP(hipMemsetAsync(e->readd, 0, (size_t)e->L * 4, e->stream));
      AV_HIP(hipMemsetAsync(e->died_out, 0, (size_t)e->L * 4, e->stream));
    }
    int rc = materialize_votes(e);
    if (rc != AV_OK) return rc;
    e->pub_mode = (int32_t)value;
    rc = refresh_pref(e);  // republish the current snapshot under the new rule
    if (rc != AV_OK) return rc;
    AV_HIP(hipStreamSynchronize(e->stream));
  } else if (n == "uni_votes") {
    e->uni_votes = value != 0 ? 1u : 0u;
  } else if (n == "wave_dense") {  // A/B: the dense log must hold one record per lane with updates
    AV_CHECK(value >= 0 && value <= 64, AV_ERR_INVALID_ARG, "bad wave_dense");
    e->wave_dense = (uint32_t)value;
  } else if (n == "dense_min") {  // tuning (A/B): fewer updates per dense record; the dense log may fill sooner
    AV_CHECK(value >= 1 && value <= 32 * (int64_t)e->k + 1, AV_ERR_INVALID_ARG, "bad dense_min");
    e->dense_min = (uint32_t)value;
  } else if (n == "fresh") {  // 0: a round after init reads every plane (A/B only)
    if (!value) e->fresh = false;
  } else if (n == "push_defer") {  // A/B: 0 = every push stored from the tile loop
    e->push_defer = value != 0;
  } else if (n == "tile_draw") {  // A/B: per-tile shared peer draws in runs whose nodes overflow the run's draw
    AV_CHECK(value == 0 || value == 1, AV_ERR_INVALID_ARG, "tile_draw must be 0 or 1");
    e->tile_draw = (uint32_t)value;
  } else if (n == "materialize_run") {  // A/B: tiles per wave of the deferred state's write-back
    AV_CHECK(value >= 1 && value <= 64, AV_ERR_INVALID_ARG, "materialize_run must be 1..64");
    e->mat_run = (uint32_t)value;
  } else if (n == "push_store") {  // A/B: 1 = plain stores (default), 0 = system scope, 2 = none (results invalid)
    AV_CHECK(value >= 0 && value <= 2, AV_ERR_INVALID_ARG, "push_store must be 0, 1 or 2");
    e->push_store = (uint32_t)value;
  } else if (n == "peer_mask") {  // before the exchange is set up: need-masked pushes (default 1)
    AV_CHECK(e->peer_world == 0, AV_ERR_INVALID_ARG, "peer_mask must be set before the exchange is set up");
    e->peer_mask = value != 0;
  } else if (n == "pref_uncached") {
    // A/B: the three snapshot buffers re-allocated uncached (hipDeviceMallocUncached: the L2 does not
    // keep their lines, a gather reads the bytes it asks for instead of a 128-B line fill) or back
    AV_CHECK(value == 0 || value == 1, AV_ERR_INVALID_ARG, "pref_uncached must be 0 or 1");
    AV_CHECK(!e->arrive && !e->group, AV_ERR_UNSUPPORTED, "pref_uncached: not with a peer exchange");
    if ((value != 0) != e->pref_uncached) {
      AV_HIP(hipStreamSynchronize(e->stream));
      for (int b = 0; b < 3; ++b) {
        uint32_t* nb = nullptr;
        AV_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&nb), e->pref_alloc_words * 4,
                                     value ? hipDeviceMallocUncached : hipDeviceMallocDefault));
        AV_HIP(hipMemcpy(nb, e->pref[b], e->pref_alloc_words * 4, hipMemcpyDeviceToDevice));
        AV_HIP(hipFree(e->pref[b]));
        e->pref[b] = nb;
      }
      e->pref_uncached = value != 0;
    }
  } else if (n == "peer_fine") {  // before av_peer_handles: fine-grained snapshot buffers (default 1)
    AV_CHECK(!e->arrive, AV_ERR_INVALID_ARG, "peer_fine must be set before av_peer_handles");
    e->peer_fine = value != 0;
  } else if (n == "barrier_timeout_ms") {
    AV_CHECK(value >= 1 && value <= 3600000, AV_ERR_INVALID_ARG, "bad barrier_timeout_ms");
    e->barrier_timeout_ms = (uint32_t)value;
    e->barrier_ticks = 0;  // recomputed at the next barrier
  } else if (n == "warm_skip") {  // may only be switched off (it is a proven invariant, not a hint)
    if (!value) e->c_monotone = false;
  } else {
    return fail(AV_ERR_INVALID_ARG, "unknown option '%s'", name);
  }
  return AV_OK;
}

int av_set_timing(av_engine* e, int32_t enable) {
  AV_ENTER(e);
  e->timing = enable != 0;
  return AV_OK;
}

int av_kernel_stats(av_engine* e, double* total_ms, int64_t* launches) {
  AV_ENTER(e);
  AV_CHECK(total_ms && launches, AV_ERR_INVALID_ARG, "null argument");
  AV_HIP(hipStreamSynchronize(e->stream));
  for (auto& ev : e->events) {
    float ms = 0.f;
    AV_HIP(hipEventElapsedTime(&ms, ev.first, ev.second));
    e->timed_ms += ms;
    e->timed_launches++;
    (void)hipEventDestroy(ev.first);
    (void)hipEventDestroy(ev.second);
  }
  e->events.clear();
  *total_ms = e->timed_ms;
  *launches = e->timed_launches;
  e->timed_ms = 0.0;
  e->timed_launches = 0;
  return AV_OK;
}

int av_layout_info(av_engine* e, int64_t* lanes, int64_t* local_nodes, int64_t* local_blocks, int32_t* capped) {
  AV_CHECK(e, AV_ERR_INVALID_ARG, "null engine");
  if (lanes) *lanes = e->L;
  if (local_nodes) *local_nodes = e->NL;
  if (local_blocks) *local_blocks = e->BL;
  if (capped) *capped = e->capped ? 1 : 0;
  return AV_OK;
}

int av_comm_unique_id(uint8_t out[128]) {
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  AV_CHECK(r == ncclSuccess, AV_ERR_RCCL, "ncclGetUniqueId: %s", ncclGetErrorString(r));
  std::memcpy(out, &id, 128);
  return AV_OK;
}

int av_comm_init(av_engine* e, int32_t world, int32_t rank, const uint8_t id[128]) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  AV_CHECK(id && world >= 1 && rank >= 0 && rank < world, AV_ERR_INVALID_ARG, "bad world/rank");
  AV_CHECK(e->N % world == 0 && (int64_t)e->NL * world == e->N && e->n0 == (int64_t)rank * e->NL,
           AV_ERR_UNSUPPORTED, "node shards must be equal, contiguous and rank-ordered (N %% world == 0)");
  AV_CHECK(e->t0 == 0 && e->t1 == e->M, AV_ERR_UNSUPPORTED, "node sharding needs the full target range");
  ncclUniqueId uid;
  std::memcpy(&uid, id, 128);
  ncclResult_t r = ncclCommInitRank(&e->comm, world, uid, rank);
  AV_CHECK(r == ncclSuccess, AV_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
  e->world = world;
  e->rank = rank;
  // make every rank's initial preference rows visible everywhere
  const size_t count = (size_t)e->NL * e->PS;
  uint32_t* cur = e->pref[e->cur];
  r = ncclAllGather(cur + (size_t)e->n0 * e->PS, cur, count, ncclUint32, e->comm, e->stream);
  AV_CHECK(r == ncclSuccess, AV_ERR_RCCL, "ncclAllGather: %s", ncclGetErrorString(r));
  AV_HIP(hipStreamSynchronize(e->stream));
  return AV_OK;
}

int av_peer_handles(av_engine* e, uint8_t out[AV_PEER_HANDLE_BYTES]) {
  AV_ENTER(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  static_assert(sizeof(hipIpcMemHandle_t) * 4 + 64 == AV_PEER_HANDLE_BYTES, "peer handle blob size");
  AV_CHECK(!e->solo_used, AV_ERR_UNSUPPORTED,
           "diagnostics option solo_barrier was used on this engine: it cannot join a peer exchange");
  if (!e->arrive) {  // zeroed before any peer can see it: the exchange of handles orders the two
    // Snapshot buffers that peers store into over xGMI are fine-grained: this
    // device's L2 keeps such lines only within a kernel (the system-scope
    // acquire at every kernel start drops them), so a round never reads a
    // stale L2 copy of a row a peer pushed during the previous round. Coarse-
    // grained memory would let a line read two rounds earlier (the 3-deep
    // rotation) survive in L2. Option "peer_fine" 0: keep the
    // coarse-grained buffers (A/B only).
    if (e->peer_fine) {
      AV_HIP(hipStreamSynchronize(e->stream));
      for (int b = 0; b < 3; ++b) {
        uint32_t* fine = nullptr;
        AV_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), e->pref_alloc_words * 4,
                                     hipDeviceMallocFinegrained));
        AV_HIP(hipMemcpy(fine, e->pref[b], e->pref_alloc_words * 4, hipMemcpyDeviceToDevice));
        AV_HIP(hipFree(e->pref[b]));
        e->pref[b] = fine;
      }
    }
    int rc = alloc_arrival(e);
    if (rc != AV_OK) return rc;
  }
  void* bufs[4] = {e->pref[0], e->pref[1], e->pref[2], e->arrive};
  for (int i = 0; i < 4; ++i) {
    hipIpcMemHandle_t h;
    AV_HIP(hipIpcGetMemHandle(&h, bufs[i]));
    std::memcpy(out + i * sizeof(h), &h, sizeof(h));
  }
  // the device's PCI bus id: peers check that they can reach it (av_peer_init)
  char bus[64] = {};
  AV_HIP(hipDeviceGetPCIBusId(bus, (int)sizeof(bus) - 1, e->cfg.device));
  std::memcpy(out + 4 * sizeof(hipIpcMemHandle_t), bus, 64);
  return AV_OK;
}

int av_peer_init(av_engine* e, int32_t world, int32_t rank, const uint8_t* handles) {
  if (e) ref_invalidate(e);
  AV_ENTER(e);
  AV_CHECK(handles && world >= 1 && world <= avk::kMaxPeers + 1 && rank >= 0 && rank < world, AV_ERR_INVALID_ARG,
           "bad world/rank (at most %d ranks)", avk::kMaxPeers + 1);
  AV_CHECK(e->N % world == 0 && (int64_t)e->NL * world == e->N && e->n0 == (int64_t)rank * e->NL,
           AV_ERR_UNSUPPORTED, "node shards must be equal, contiguous and rank-ordered (N %% world == 0)");
  AV_CHECK(e->t0 == 0 && e->t1 == e->M, AV_ERR_UNSUPPORTED, "node sharding needs the full target range");
  AV_CHECK(e->comm == nullptr && e->peer_world == 0, AV_ERR_UNSUPPORTED, "exchange already initialised");
  AV_CHECK(!e->solo_used, AV_ERR_UNSUPPORTED,
           "diagnostics option solo_barrier was used on this engine: it cannot join a peer exchange");
  AV_CHECK(e->arrive != nullptr, AV_ERR_INVALID_ARG, "call av_peer_handles before av_peer_init");
  for (int r = 0; r < world; ++r) {
    void* ptrs[4] = {e->pref[0], e->pref[1], e->pref[2], e->arrive};
    if (r != rank) {
      // a peer GPU this process can see must be reachable (xGMI peer access);
      // one it cannot see (restricted visibility) is left to the IPC mapping
      char bus[65] = {};
      std::memcpy(bus, handles + (size_t)r * AV_PEER_HANDLE_BYTES + 4 * sizeof(hipIpcMemHandle_t), 64);
      int pdev = -1;
      if (bus[0] && hipDeviceGetByPCIBusId(&pdev, bus) == hipSuccess && pdev != e->cfg.device) {
        int can = 0;
        AV_HIP(hipDeviceCanAccessPeer(&can, e->cfg.device, pdev));
        AV_CHECK(can, AV_ERR_UNSUPPORTED, "device %d cannot access peer device %d (%s)", e->cfg.device, pdev, bus);
        hipError_t pe = hipDeviceEnablePeerAccess(pdev, 0);
        AV_CHECK(pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled, AV_ERR_HIP,
                 "hipDeviceEnablePeerAccess(%d): %s", pdev, hipGetErrorString(pe));
        (void)hipGetLastError();
      } else {
        (void)hipGetLastError();
      }
      for (int i = 0; i < 4; ++i) {
        hipIpcMemHandle_t h;
        std::memcpy(&h, handles + (size_t)r * AV_PEER_HANDLE_BYTES + i * sizeof(h), sizeof(h));
        void* m = nullptr;
        AV_HIP(hipIpcOpenMemHandle(&m, h, hipIpcMemLazyEnablePeerAccess));
        e->peer_opened.push_back(m);
        ptrs[i] = m;
      }
    }
    for (int b = 0; b < 3; ++b) e->peer_pref[b][r] = static_cast<uint32_t*>(ptrs[b]);
    e->peer_arrive.p[r] = static_cast<uint32_t*>(ptrs[3]);
    e->peer_needin.p[r] = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(ptrs[3]) + kNeedinOff);
  }
  e->needin = e->peer_needin.p[rank];
  {
    uint32_t* tbl[3][avk::kMaxPeers] = {};
    for (int b = 0; b < 3; ++b) {
      int n = 0;
      for (int r = 0; r < world; ++r)
        if (r != rank) tbl[b][n++] = e->peer_pref[b][r];
    }
    AV_HIP(dev_alloc(&e->push_tbl, (size_t)3 * avk::kMaxPeers));
    AV_HIP(hipMemcpy(e->push_tbl, tbl, sizeof(tbl), hipMemcpyHostToDevice));
  }
  e->peer_world = world;
  e->peer_rank = rank;
  e->world = world;
  e->rank = rank;
  if (world > 1) {
    // every replica of every snapshot buffer identical from here on: each
    // rank pushes its own rows of the three buffers, then all ranks meet
    for (int b = 0; b < 3; ++b) {
      int rc = push_own_rows(e, b);
      if (rc != AV_OK) return rc;
    }
    int rc = mask_setup(e);
    if (rc == AV_OK) rc = need_gen(e, e->round / avk::kNeedWin);
    if (rc != AV_OK) return rc;
    rc = peer_barrier(e);
    if (rc != AV_OK) return rc;
  }
  return av_synchronize(e);
}

int av_peer_group_serial(av_engine** engines, int32_t world) {
  AV_CHECK(engines && world >= 2 && world <= avk::kMaxPeers + 1, AV_ERR_INVALID_ARG,
           "bad engines/world (2..%d ranks)", avk::kMaxPeers + 1);
  for (int r = 0; r < world; ++r) {
    av_engine* e = engines[r];
    AV_CHECK(e, AV_ERR_INVALID_ARG, "null engine");
    AV_CHECK(e->cfg.device == engines[0]->cfg.device, AV_ERR_UNSUPPORTED, "peer group: one device");
    AV_CHECK(e->N == engines[0]->N && e->M == engines[0]->M && e->k == engines[0]->k &&
                 e->cfg.seed == engines[0]->cfg.seed && e->cfg.byz_threshold == engines[0]->cfg.byz_threshold &&
                 e->cfg.peer_mode == engines[0]->cfg.peer_mode && e->round == engines[0]->round &&
                 e->cur == engines[0]->cur,
             AV_ERR_INVALID_ARG, "peer group: engines of one network at one round");
    AV_CHECK(e->N % world == 0 && (int64_t)e->NL * world == e->N && e->n0 == (int64_t)r * e->NL, AV_ERR_UNSUPPORTED,
             "node shards must be equal, contiguous and rank-ordered (N %% world == 0)");
    AV_CHECK(e->t0 == 0 && e->t1 == e->M, AV_ERR_UNSUPPORTED, "node sharding needs the full target range");
    AV_CHECK(e->comm == nullptr && e->peer_world == 0 && !e->arrive && !e->solo_used, AV_ERR_UNSUPPORTED,
             "exchange already initialised");
  }
  AV_HIP(hipSetDevice(engines[0]->cfg.device));
  for (int r = 0; r < world; ++r) AV_HIP(hipStreamSynchronize(engines[r]->stream));
  // the snapshot buffers the real exchange uses (av_peer_handles): fine-grained unless option
  // "peer_fine" is 0, so that the group's parity runs and per-rank timings see the same memory type
  for (int r = 0; r < world; ++r) {
    av_engine* e = engines[r];
    if (!e->peer_fine) continue;
    for (int b = 0; b < 3; ++b) {
      uint32_t* fine = nullptr;
      AV_HIP(hipExtMallocWithFlags(reinterpret_cast<void**>(&fine), e->pref_alloc_words * 4,
                                   hipDeviceMallocFinegrained));
      AV_HIP(hipMemcpy(fine, e->pref[b], e->pref_alloc_words * 4, hipMemcpyDeviceToDevice));
      AV_HIP(hipFree(e->pref[b]));
      e->pref[b] = fine;
    }
  }
  auto* g = new PeerGroup();
  if (hipStreamCreateWithFlags(&g->stream, hipStreamNonBlocking) != hipSuccess) {
    delete g;
    return fail(AV_ERR_HIP, "hipStreamCreate failed");
  }
  g->members.assign(engines, engines + world);
  g->alive = world;
  for (int r = 0; r < world; ++r) {
    av_engine* e = engines[r];
    ref_invalidate(e);
    e->group = g;
    e->own_stream = e->stream;
    e->stream = g->stream;
    for (int b = 0; b < 3; ++b)
      for (int q = 0; q < world; ++q) e->peer_pref[b][q] = engines[q]->pref[b];
    uint32_t* tbl[3][avk::kMaxPeers] = {};
    for (int b = 0; b < 3; ++b) {
      int n = 0;
      for (int q = 0; q < world; ++q)
        if (q != r) tbl[b][n++] = e->peer_pref[b][q];
    }
    AV_HIP(dev_alloc(&e->push_tbl, (size_t)3 * avk::kMaxPeers));
    AV_HIP(hipMemcpy(e->push_tbl, tbl, sizeof(tbl), hipMemcpyHostToDevice));
    e->peer_world = world;
    e->peer_rank = r;
    e->world = world;
    e->rank = r;
  }
  for (int r = 0; r < world; ++r) {
    AV_HIP(dev_alloc(&engines[r]->needin, needin_words(engines[r], world)));
    for (int q = 0; q < world; ++q) engines[q]->peer_needin.p[r] = engines[r]->needin;
  }
  // every replica of every snapshot buffer identical from here on
  for (int r = 0; r < world; ++r) {
    for (int b = 0; b < 3; ++b) {
      int rc = push_own_rows(engines[r], b);
      if (rc != AV_OK) return rc;
    }
    int rc = mask_setup(engines[r]);
    if (rc == AV_OK) rc = need_gen(engines[r], engines[r]->round / avk::kNeedWin);
    if (rc != AV_OK) return rc;
  }
  AV_HIP(hipStreamSynchronize(g->stream));
  return AV_OK;
}

int av_peer_sync(av_engine* e) {
  AV_ENTER(e);
  AV_PEER_CHECK(e);
  if (e->peer_world <= 1) return AV_OK;
  int rc = push_own_rows(e, e->cur);
  if (rc == AV_OK) rc = stale_clear(e, e->cur);
  if (rc == AV_OK) rc = peer_barrier(e);
  if (rc != AV_OK) return rc;
  AV_HIP(hipStreamSynchronize(e->stream));
  return peer_failed(e);
}

int av_pushed_words(av_engine* e, int64_t* out) {
  AV_ENTER(e);
  AV_PEER_SYNC_CHECK(e);
  AV_CHECK(out, AV_ERR_INVALID_ARG, "null argument");
  return sum_counter(e, e->changed + 2 * avk::kLogShards, out);
}

}  // extern "C"
