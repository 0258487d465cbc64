/*
 * avalanche_oracle.h — TEST INFRASTRUCTURE ONLY (parity checker, CPU baseline).
 *
 * A plain-C restatement of go-avalanche's VoteRecord / Processor semantics
 * (reference: /root/reference, itsdevbear/go-avalanche @ 2025-01-17) plus the
 * synchronous batched-round harness rules R1-R4 of SURVEY.md §8(a).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library. The product path (go-avalanche_amd/, libavhip.so) never does.
 *
 * Parity pinning: the restatement is checked against the transcribed golden
 * vectors of the reference's own tests (avalanche_test.go TestVoteRecord,
 * TestBlockRegister, TestMultiBlockRegister; see tests/golden/) and against an
 * independent pure-Python restatement (oracle/avalanche_ref.py). The Go
 * reference itself cannot be built here (no Go toolchain).
 */
#ifndef AVALANCHE_ORACLE_H
#define AVALANCHE_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* avalanche.go:10,17 */
#define AVO_FINALIZATION_SCORE 128
#define AVO_MAX_ELEMENT_POLL 4096

/* avalanche.go:42-56 (Status enum, iota order) */
#define AVO_STATUS_INVALID 0
#define AVO_STATUS_REJECTED 1
#define AVO_STATUS_ACCEPTED 2
#define AVO_STATUS_FINALIZED 3

/* Canonical dump word of a (node, target) slot that holds no live record:
 * 0xFFFE0000 | (published_decision << 16).  Live records dump as the packed
 * VoteRecord votes | consider<<8 | confidence<<16 (vote.go:25-29). */
#define AVO_ABSENT_WORD 0xFFFE0000u

/* RNG domains (counter word 3) shared by the synthetic workload definition. */
#define AVO_DOM_PEERS 1u
#define AVO_DOM_BYZ 2u
#define AVO_DOM_INIT 3u
#define AVO_DOM_PAIRS 4u
#define AVO_DOM_REPLAY 5u

/* What a node publishes for a target it no longer holds (see
 * published_pref_mode in avalanche_oracle.c) */
#define AVO_RESP_DECISION 0    /* R2 (default): the finalized decision */
#define AVO_RESP_IS_ACCEPTED 1 /* processor.go:125-130: false after deletion */
#define AVO_RESP_EXAMPLE 2     /* main.go:175-182: re-added as accepted when queried, answers yes */

#define AVO_PEERS_RANDOM 0
#define AVO_PEERS_ROUND_ROBIN 1

#define AVO_INIT_NONE 0      /* no records (targets added individually) */
#define AVO_INIT_REJECTED 1  /* every node adds every target, IsAccepted()=false */
#define AVO_INIT_ACCEPTED 2  /* ... IsAccepted()=true */
#define AVO_INIT_BERNOULLI 3 /* IsAccepted() = philox < init_param (u32 threshold) */
#define AVO_INIT_PAIRS 4     /* double-spend pairs (2p, 2p+1) complementary per node */

/* ---- Philox4x32-10 (Salmon, Moraes, Dror, Shaw, SC'11 / Random123) ---- */
void avo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

/* ---- VoteRecord (vote.go:24-109) ---- */
typedef struct {
  uint8_t votes;       /* vote.go:26 */
  uint8_t consider;    /* vote.go:27 */
  uint16_t confidence; /* vote.go:28 */
} avo_vote_record;

avo_vote_record avo_new_vote_record(int accepted);        /* vote.go:33-35 */
int avo_is_accepted_rec(const avo_vote_record* vr);       /* vote.go:38-40 */
uint16_t avo_get_confidence_rec(const avo_vote_record* vr); /* vote.go:43-45 */
int avo_has_finalized(const avo_vote_record* vr);         /* vote.go:48-50 */
int avo_register_vote(avo_vote_record* vr, uint32_t err); /* vote.go:54-75 */
int avo_status(const avo_vote_record* vr);                /* vote.go:77-91 */
uint32_t avo_pack(avo_vote_record vr);
avo_vote_record avo_unpack(uint32_t w);

/* Batched single-vote transitions (exhaustive table generation). */
void avo_transition_batch(const uint32_t* words_in, const uint32_t* errs, int64_t n,
                          uint32_t* words_out, uint8_t* changed, uint8_t* status);

/* The oracle's branch-free form of the same step (used by the batched sim
 * when the poll cap cannot bind); status[i] = appended Status, -1 = none. */
void avo_transition_batch_branchfree(const uint32_t* words_in, const uint32_t* errs, int64_t n, uint32_t* words_out,
                                     int8_t* status);

/* ---- Processor (processor.go:12-187) over M dense target slots ---- */
typedef struct avo_processor avo_processor;
avo_processor* avo_processor_new(int64_t n_targets);
void avo_processor_free(avo_processor* p);
/* AddTargetToReconcile (processor.go:45-58); `valid` = t.IsValid() */
int avo_processor_add(avo_processor* p, int64_t t, int accepted, int valid);
/* RegisterVotes (processor.go:61-122). valid[t] = targets[t].IsValid().
 * Appends (target, status) pairs; returns 1 (validation is `if false`). */
int avo_processor_register_votes(avo_processor* p, const int64_t* targets, const uint32_t* errs,
                                 int64_t n, const uint8_t* valid, int64_t* out_targets,
                                 int32_t* out_status, int64_t* n_out);
int avo_processor_is_accepted(const avo_processor* p, int64_t t);              /* :125-130 */
int avo_processor_get_confidence(const avo_processor* p, int64_t t, uint16_t* out); /* :133-140; -1 = panic */
int64_t avo_processor_get_invs(const avo_processor* p, const uint8_t* valid, int64_t* out, int64_t cap); /* :144-170 */
uint32_t avo_processor_dump_word(const avo_processor* p, int64_t t);
int64_t avo_processor_get_round(const avo_processor* p);          /* :40-42 */
void avo_processor_set_round(avo_processor* p, int64_t round);    /* the owner's p.round = ... */

/* ---- Batched-round harness ---- */
typedef struct {
  int64_t n_nodes;
  int64_t n_targets;
  int32_t k;
  int32_t peer_mode;
  uint64_t seed;
  uint32_t byz_threshold; /* node j Byzantine iff philox(j) < threshold */
  int32_t init_mode;
  uint32_t init_param;
} avo_sim_config;

typedef struct avo_sim avo_sim;
avo_sim* avo_sim_new(const avo_sim_config* cfg);
avo_sim* avo_sim_new_threads(const avo_sim_config* cfg, int32_t threads); /* OpenMP population */
void avo_sim_free(avo_sim* s);
void avo_sim_set_valid(avo_sim* s, int64_t t, int valid);
int64_t avo_sim_get_round(const avo_sim* s, int64_t node); /* node's Processor.GetRound */
void avo_sim_set_round(avo_sim* s, int64_t node, int64_t round);
int64_t avo_sim_round_index(const avo_sim* s);
void avo_sim_set_round_index(avo_sim* s, int64_t r); /* harness RNG counter (re-population at round r) */
/* One round. replay_errs: NULL (sim mode: votes from peers' published
 * preferences) or [n_nodes][k][n_targets] err words. Updates are written as
 * 5 int64 columns (round, node, slot, target, status) in reference append order.
 * Returns 0, or -1 if cap was too small (n_out then holds the required count). */
int avo_sim_round(avo_sim* s, const uint32_t* replay_errs, int64_t* updates, int64_t cap,
                  int64_t* n_out, int32_t threads, int64_t* applied_votes);
/* Node-shard variant: processes nodes [n0, n1) only, refreshing only their
 * published rows; other rows are installed with avo_sim_set_pref_rows. */
int avo_sim_round_range(avo_sim* s, int64_t n0, int64_t n1, const uint32_t* replay_errs, int64_t* updates,
                        int64_t cap, int64_t* n_out, int32_t threads, int64_t* applied_votes);
/* General form: nodes [n0, n1); updates == NULL collects no rows; digest (if
 * not NULL) = {count, sum, xor} of avo_mix64(avo_pack_update(round_rel, ...))
 * over the round's StatusUpdates (order-independent; the engine computes the
 * same over its device log, av_updates_digest). */
int avo_sim_round_ex(avo_sim* s, int64_t n0, int64_t n1, const uint32_t* replay_errs, int64_t* updates,
                     int64_t cap, int64_t* n_out, int32_t threads, int64_t* applied_votes, uint64_t digest[3],
                     uint32_t round_rel);
/* 1: every round takes the literal per-vote path (GetInvsForNextPoll +
 * RegisterVotes per slot); 0 (default): the branch-free per-node form when the
 * poll cap cannot bind. Both are the same restatement; tests compare them. */
void avo_sim_set_literal(avo_sim* s, int literal);
void avo_sim_set_responder(avo_sim* s, int32_t mode); /* AVO_RESP_* */
void avo_sim_set_polling(avo_sim* s, int64_t node, int polls);
/* One node's literal round against an external snapshot (pref_words
 * [n_nodes][ceil(m/32)] bitsets, byz_words [ceil(n/32)]): words[m] canonical
 * record words in/out; digest accumulates its StatusUpdates; returns the
 * applied votes. The sampled full-size check of the engine. */
int64_t avo_node_round_ext(uint64_t seed, int64_t n_nodes, int32_t k, int32_t peer_mode, int64_t node,
                           int64_t round, int64_t m, const uint32_t* pref_words, const uint32_t* byz_words,
                           const uint8_t* valid, uint32_t* words, uint64_t digest[3], uint32_t round_rel);
uint64_t avo_pack_update(uint32_t round_rel, int64_t node, int32_t slot, int64_t t, int32_t status);
uint64_t avo_mix64(uint64_t x);
void avo_sim_set_pref_rows(avo_sim* s, int64_t n0, int64_t n1, const uint8_t* rows);
void avo_sim_dump(const avo_sim* s, uint32_t* out /* [N][M] canonical words */);
void avo_sim_dump_range(const avo_sim* s, int64_t n0, int64_t n1, uint32_t* out /* [n1-n0][M] */, int32_t threads);
void avo_sim_pref(const avo_sim* s, uint8_t* out /* [N][M] published preference */);
int avo_sim_is_byzantine(const avo_sim* s, int64_t node);
/* Mutators used by the golden-fixture interpreter */
int avo_sim_add(avo_sim* s, int64_t node, int64_t t, int accepted);
int avo_sim_register_votes(avo_sim* s, int64_t node, const int64_t* targets, const uint32_t* errs,
                           int64_t n, int64_t* out_targets, int32_t* out_status, int64_t* n_out);

/* ---- synthetic workload definition (same formulas as the device side) ---- */
void avo_sample_peers(uint64_t seed, int64_t node, int64_t round, int64_t n_nodes, int32_t k,
                      int32_t mode, int64_t* out);
int avo_is_byzantine(uint64_t seed, int64_t node, uint32_t threshold);
void avo_byz_words(uint64_t seed, int64_t n_nodes, uint32_t threshold, uint32_t* out /* [ceil(n/32)] bits */);
int avo_initial_accept(uint64_t seed, int32_t mode, uint32_t param, int64_t node, int64_t t);
uint32_t avo_replay_err(uint64_t seed, int64_t node, int64_t round, int32_t slot, int64_t t);
void avo_gen_replay_errs(uint64_t seed, int64_t round, int64_t n0, int64_t n1, int64_t n_targets,
                         int32_t k, uint32_t* out /* [n1-n0][k][M] */);

#ifdef __cplusplus
}
#endif
#endif
