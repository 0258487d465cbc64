/*
 * avalanche_oracle.c — TEST INFRASTRUCTURE ONLY. See avalanche_oracle.h.
 *
 * Straight, per-record restatement of the reference semantics. Nothing here
 * is bit-sliced or batched: every function follows the Go code it cites line
 * by line so that it can serve as the parity checker for the HIP engine.
 */
#include "avalanche_oracle.h"

#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------------ */
/* Philox4x32-10: round function and Weyl key schedule as published with   */
/* Random123 (multipliers 0xD2511F53 / 0xCD9E8D57, bumps 0x9E3779B9 /       */
/* 0xBB67AE85). Pinned by the Random123 known-answer vectors in tests/.    */
/* ------------------------------------------------------------------------ */
void avo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void philox_dom(uint64_t seed, uint32_t a, uint32_t b, uint32_t c, uint32_t dom, uint32_t out[4]) {
  uint32_t ctr[4] = {a, b, c, dom};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  avo_philox4x32_10(ctr, key, out);
}

/* ------------------------------------------------------------------------ */
/* VoteRecord — vote.go                                                      */
/* ------------------------------------------------------------------------ */

/* vote.go:93-98 countBits8: Kernighan's loop counts the set bits of a u8,
 * i.e. its population count (the loop form is kept in oracle/avalanche_ref.py;
 * tests/test_oracle.py checks the two agree on all 256 values). */
static int count_bits8(uint8_t i) { return __builtin_popcount((unsigned)i); }

/* vote.go:33-35 NewVoteRecord: confidence = boolToUint16(accepted) */
avo_vote_record avo_new_vote_record(int accepted) {
  avo_vote_record vr;
  vr.votes = 0;
  vr.consider = 0;
  vr.confidence = accepted ? 1 : 0;
  return vr;
}

/* vote.go:38-40 */
int avo_is_accepted_rec(const avo_vote_record* vr) { return (vr->confidence & 0x01) == 1; }
/* vote.go:43-45 */
uint16_t avo_get_confidence_rec(const avo_vote_record* vr) { return (uint16_t)(vr->confidence >> 1); }
/* vote.go:48-50 */
int avo_has_finalized(const avo_vote_record* vr) {
  return avo_get_confidence_rec(vr) >= AVO_FINALIZATION_SCORE;
}

/* vote.go:54-75 regsiterVote */
int avo_register_vote(avo_vote_record* vr, uint32_t err) {
  /* :55-56 — u8 shift with wrap; neutral = int32(err) < 0 */
  vr->votes = (uint8_t)((uint8_t)(vr->votes << 1) | (err == 0 ? 1 : 0));
  vr->consider = (uint8_t)((uint8_t)(vr->consider << 1) | ((int32_t)err >= 0 ? 1 : 0));

  /* :58 */
  int yes = count_bits8((uint8_t)(vr->votes & vr->consider & 0xff)) > 6;

  /* :61-63 — (-votes-1) is ^votes in uint8 arithmetic */
  uint8_t not_votes = (uint8_t)(-(int)vr->votes - 1);
  if (!yes && count_bits8((uint8_t)(not_votes & vr->consider & 0xff)) <= 6) {
    return 0;
  }

  /* :66-69 */
  if (avo_is_accepted_rec(vr) == yes) {
    vr->confidence = (uint16_t)(vr->confidence + 2);
    return avo_get_confidence_rec(vr) == AVO_FINALIZATION_SCORE;
  }

  /* :72-74 */
  vr->confidence = yes ? 1 : 0;
  return 1;
}

/* vote.go:77-91 */
int avo_status(const avo_vote_record* vr) {
  int finalized = avo_has_finalized(vr);
  int accepted = avo_is_accepted_rec(vr);
  if (!finalized && accepted) return AVO_STATUS_ACCEPTED;
  if (!finalized && !accepted) return AVO_STATUS_REJECTED;
  if (finalized && accepted) return AVO_STATUS_FINALIZED;
  return AVO_STATUS_INVALID;
}

uint32_t avo_pack(avo_vote_record vr) {
  return (uint32_t)vr.votes | ((uint32_t)vr.consider << 8) | ((uint32_t)vr.confidence << 16);
}

avo_vote_record avo_unpack(uint32_t w) {
  avo_vote_record vr;
  vr.votes = (uint8_t)(w & 0xff);
  vr.consider = (uint8_t)((w >> 8) & 0xff);
  vr.confidence = (uint16_t)(w >> 16);
  return vr;
}

void avo_transition_batch(const uint32_t* words_in, const uint32_t* errs, int64_t n,
                          uint32_t* words_out, uint8_t* changed, uint8_t* status) {
  for (int64_t i = 0; i < n; ++i) {
    avo_vote_record vr = avo_unpack(words_in[i]);
    int c = avo_register_vote(&vr, errs[i]);
    words_out[i] = avo_pack(vr);
    if (changed) changed[i] = (uint8_t)c;
    if (status) status[i] = (uint8_t)avo_status(&vr);
  }
}

/* ------------------------------------------------------------------------ */
/* Processor — processor.go. The Go maps keyed by Hash become dense arrays   */
/* over target slots: present[t] <=> voteRecords[hash] exists.              */
/* decision[t] remembers the finalized outcome of a deleted record so the   */
/* harness can publish it (SURVEY.md §8(a) rule R2); the reference itself   */
/* forgets it.                                                              */
/* ------------------------------------------------------------------------ */
struct avo_processor {
  int64_t m;
  int64_t round; /* processor.go:15: only its owner changes it (avalanche_test.go:302) */
  uint8_t* present;
  uint8_t* decision;
  avo_vote_record* rec;
};

avo_processor* avo_processor_new(int64_t n_targets) {
  avo_processor* p = (avo_processor*)calloc(1, sizeof(avo_processor));
  p->m = n_targets;
  p->present = (uint8_t*)calloc((size_t)n_targets, 1);
  p->decision = (uint8_t*)calloc((size_t)n_targets, 1);
  p->rec = (avo_vote_record*)calloc((size_t)n_targets, sizeof(avo_vote_record));
  return p;
}

void avo_processor_free(avo_processor* p) {
  if (!p) return;
  free(p->present);
  free(p->decision);
  free(p->rec);
  free(p);
}

/* processor.go:40-42 GetRound, and the owner's `p.round = ...` */
int64_t avo_processor_get_round(const avo_processor* p) { return p->round; }
void avo_processor_set_round(avo_processor* p, int64_t round) { p->round = round; }

/* processor.go:45-58 AddTargetToReconcile */
int avo_processor_add(avo_processor* p, int64_t t, int accepted, int valid) {
  if (t < 0 || t >= p->m) return 0;
  if (!valid) return 0;              /* :46-48 isWorthyPolling */
  if (p->present[t]) return 0;       /* :50-53 */
  p->present[t] = 1;                 /* :55-56 */
  p->rec[t] = avo_new_vote_record(accepted);
  return 1;
}

/* processor.go:61-122 RegisterVotes (validation block :63-90 is `if false`) */
int avo_processor_register_votes(avo_processor* p, const int64_t* targets, const uint32_t* errs,
                                 int64_t n, const uint8_t* valid, int64_t* out_targets,
                                 int32_t* out_status, int64_t* n_out) {
  int64_t nu = 0;
  for (int64_t i = 0; i < n; ++i) { /* :94 */
    int64_t t = targets[i];
    if (t < 0 || t >= p->m || !p->present[t]) continue; /* :95-99 */
    if (!valid[t]) continue;                             /* :101-103 */
    avo_vote_record* vr = &p->rec[t];
    if (!avo_register_vote(vr, errs[i])) continue;       /* :105-108 */
    if (out_targets) out_targets[nu] = t;                /* :111 */
    if (out_status) out_status[nu] = avo_status(vr);
    nu++;
    if (avo_has_finalized(vr)) {                         /* :114-116 */
      p->present[t] = 0;
      p->decision[t] = (uint8_t)avo_is_accepted_rec(vr);
    }
  }
  if (n_out) *n_out = nu;
  return 1; /* :121 */
}

/* processor.go:125-130 */
int avo_processor_is_accepted(const avo_processor* p, int64_t t) {
  if (t >= 0 && t < p->m && p->present[t]) return avo_is_accepted_rec(&p->rec[t]);
  return 0;
}

/* processor.go:133-140 ; -1 stands for panic("VoteRecord not found") */
int avo_processor_get_confidence(const avo_processor* p, int64_t t, uint16_t* out) {
  if (t < 0 || t >= p->m || !p->present[t]) return -1;
  *out = avo_get_confidence_rec(&p->rec[t]);
  return 0;
}

/* processor.go:144-170. Go map order is randomised; the harness fixes it to
 * ascending target index. Truncated to cap (4096, :165-167). */
int64_t avo_processor_get_invs(const avo_processor* p, const uint8_t* valid, int64_t* out, int64_t cap) {
  int64_t n = 0;
  for (int64_t t = 0; t < p->m; ++t) {
    if (!p->present[t]) continue;
    if (avo_has_finalized(&p->rec[t])) continue; /* :147-150 */
    if (!valid[t]) continue;                     /* :155-157 */
    if (n < cap) out[n] = t;
    n++;
    if (n >= cap) break; /* invs[:4096] keeps the first cap in this order */
  }
  return n < cap ? n : cap;
}

uint32_t avo_processor_dump_word(const avo_processor* p, int64_t t) {
  if (p->present[t]) return avo_pack(p->rec[t]);
  return AVO_ABSENT_WORD | ((uint32_t)p->decision[t] << 16);
}

/* What a node answers for target t (the responder of main.go:168-192):
 *   AVO_RESP_DECISION (harness rule R2): its record's accepted bit, or the
 *     decision of a record it finalized and deleted;
 *   AVO_RESP_IS_ACCEPTED: processor.go:125-130 literally: false once deleted;
 *   AVO_RESP_EXAMPLE: the example's responder (main.go:175-182): it first
 *     AddTargetToReconcile(&tx{isAccepted: true}), so an absent record comes
 *     back accepted and the answer is yes. */
static int published_pref_mode(const avo_processor* p, int64_t t, int32_t mode) {
  if (p->present[t]) return avo_is_accepted_rec(&p->rec[t]);
  if (mode == AVO_RESP_IS_ACCEPTED) return 0;
  if (mode == AVO_RESP_EXAMPLE) return 1;
  return p->decision[t];
}

/* ------------------------------------------------------------------------ */
/* Synthetic workload definition                                            */
/* ------------------------------------------------------------------------ */

/* k distinct peers != node, uniform over the other N-1 nodes by 32x32->hi
 * multiply; Philox blocks of 4 draws, counter (node, round, block, PEERS). */
void avo_sample_peers(uint64_t seed, int64_t node, int64_t round, int64_t n_nodes, int32_t k,
                      int32_t mode, int64_t* out) {
  uint64_t others = (uint64_t)(n_nodes - 1);
  if (mode == AVO_PEERS_ROUND_ROBIN || (uint64_t)k >= others) {
    /* main.go:110-116: round-robin over all other nodes, skipping self */
    for (int32_t j = 0; j < k; ++j) {
      uint64_t q = (mode == AVO_PEERS_ROUND_ROBIN) ? ((uint64_t)round * (uint64_t)k + (uint64_t)j)
                                                    : (uint64_t)j;
      uint64_t idx = q % others;
      out[j] = (int64_t)(idx + (idx >= (uint64_t)node ? 1 : 0));
    }
    return;
  }
  int32_t cnt = 0;
  uint32_t blk = 0;
  while (cnt < k) {
    uint32_t x[4];
    philox_dom(seed, (uint32_t)node, (uint32_t)round, blk, AVO_DOM_PEERS, x);
    for (int i = 0; i < 4 && cnt < k; ++i) {
      uint64_t u = ((uint64_t)x[i] * others) >> 32;
      int64_t p = (int64_t)(u + (u >= (uint64_t)node ? 1 : 0));
      int dup = 0;
      for (int32_t j = 0; j < cnt; ++j) dup |= (out[j] == p);
      if (!dup) out[cnt++] = p;
    }
    blk++;
  }
}

void avo_byz_words(uint64_t seed, int64_t n_nodes, uint32_t threshold, uint32_t* out /* [ceil(n/32)] */) {
  for (int64_t w = 0; w < (n_nodes + 31) / 32; ++w) out[w] = 0u;
  if (!threshold) return;
  for (int64_t j = 0; j < n_nodes; ++j)
    if (avo_is_byzantine(seed, j, threshold)) out[j >> 5] |= 1u << (j & 31);
}

int avo_is_byzantine(uint64_t seed, int64_t node, uint32_t threshold) {
  uint32_t x[4];
  philox_dom(seed, (uint32_t)node, 0, 0, AVO_DOM_BYZ, x);
  return x[0] < threshold;
}

int avo_initial_accept(uint64_t seed, int32_t mode, uint32_t param, int64_t node, int64_t t) {
  uint32_t x[4];
  switch (mode) {
    case AVO_INIT_REJECTED: return 0;
    case AVO_INIT_ACCEPTED: return 1;
    case AVO_INIT_BERNOULLI:
      philox_dom(seed, (uint32_t)node, (uint32_t)(t >> 2), 0, AVO_DOM_INIT, x);
      return x[t & 3] < param;
    case AVO_INIT_PAIRS: {
      int64_t pair = t >> 1;
      philox_dom(seed, (uint32_t)node, (uint32_t)(pair >> 2), 0, AVO_DOM_PAIRS, x);
      return (int)((x[pair & 3] >> 31) ^ (uint32_t)(t & 1));
    }
    default: return 0;
  }
}

/* Replayed vote stream (C2): P(yes)=0.70, P(no)=0.25, P(neutral)=0.05.
 * no-errs {1, 2, 0x7FFFFFFF}; neutral errs {0x80000000, 0xFFFFFFFF}. */
uint32_t avo_replay_err(uint64_t seed, int64_t node, int64_t round, int32_t slot, int64_t t) {
  uint32_t x[4];
  philox_dom(seed, (uint32_t)node, (uint32_t)round, (uint32_t)(t >> 1),
             AVO_DOM_REPLAY | ((uint32_t)slot << 8), x);
  uint32_t v = x[(t & 1) * 2];
  uint32_t sel = x[(t & 1) * 2 + 1];
  if (v < 3006477107u) return 0u;
  if (v < 4080218931u) {
    static const uint32_t no_errs[3] = {1u, 2u, 0x7FFFFFFFu};
    return no_errs[sel % 3u];
  }
  return (sel & 1u) ? 0xFFFFFFFFu : 0x80000000u;
}

void avo_gen_replay_errs(uint64_t seed, int64_t round, int64_t n0, int64_t n1, int64_t n_targets,
                         int32_t k, uint32_t* out) {
  for (int64_t n = n0; n < n1; ++n)
    for (int32_t s = 0; s < k; ++s)
      for (int64_t t = 0; t < n_targets; ++t)
        out[((n - n0) * k + s) * n_targets + t] = avo_replay_err(seed, n, round, s, t);
}

/* ------------------------------------------------------------------------ */
/* Batched-round harness                                                    */
/* ------------------------------------------------------------------------ */
struct avo_sim {
  avo_sim_config cfg;
  int64_t round;
  avo_processor** procs;
  uint8_t* valid; /* [M] Target.IsValid() */
  uint8_t* pref;  /* [N][M] round-start published preference snapshot */
  uint8_t* byz;   /* [N] */
  int literal;    /* 1: always the literal per-vote path (cross-checks the branch-free one) */
  int32_t responder; /* AVO_RESP_* */
  uint8_t* polls;    /* [N] the node polls in the rounds (the example's run loop stops, main.go:160-162) */
};

avo_sim* avo_sim_new(const avo_sim_config* cfg) { return avo_sim_new_threads(cfg, 1); }

avo_sim* avo_sim_new_threads(const avo_sim_config* cfg, int32_t threads) {
  avo_sim* s = (avo_sim*)calloc(1, sizeof(avo_sim));
  s->cfg = *cfg;
  int64_t n = cfg->n_nodes, m = cfg->n_targets;
  s->procs = (avo_processor**)calloc((size_t)n, sizeof(avo_processor*));
  s->valid = (uint8_t*)malloc((size_t)m);
  memset(s->valid, 1, (size_t)m);
  s->pref = (uint8_t*)calloc((size_t)(n * m), 1);
  s->byz = (uint8_t*)calloc((size_t)n, 1);
  s->polls = (uint8_t*)malloc((size_t)n);
  memset(s->polls, 1, (size_t)n);
  int nt = threads > 0 ? threads : 1;
  (void)nt;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 64) num_threads(nt)
#endif
  for (int64_t j = 0; j < n; ++j) {
    s->procs[j] = avo_processor_new(m);
    s->byz[j] = (uint8_t)avo_is_byzantine(cfg->seed, j, cfg->byz_threshold);
    if (cfg->init_mode != AVO_INIT_NONE) {
      for (int64_t t = 0; t < m; ++t) {
        int acc = avo_initial_accept(cfg->seed, cfg->init_mode, cfg->init_param, j, t);
        avo_processor_add(s->procs[j], t, acc, 1);
        s->pref[j * m + t] = (uint8_t)acc;
      }
    }
  }
  return s;
}

void avo_sim_free(avo_sim* s) {
  if (!s) return;
  for (int64_t j = 0; j < s->cfg.n_nodes; ++j) avo_processor_free(s->procs[j]);
  free(s->procs);
  free(s->valid);
  free(s->pref);
  free(s->byz);
  free(s->polls);
  free(s);
}

int64_t avo_sim_get_round(const avo_sim* s, int64_t node) { return avo_processor_get_round(s->procs[node]); }
void avo_sim_set_round(avo_sim* s, int64_t node, int64_t round) { avo_processor_set_round(s->procs[node], round); }

void avo_sim_set_valid(avo_sim* s, int64_t t, int valid) { s->valid[t] = (uint8_t)(valid != 0); }
int64_t avo_sim_round_index(const avo_sim* s) { return s->round; }
/* The harness's round counter (R1: the peer draw's RNG counter): a network
 * created now behaves as if populated at round r (the engine's av_init_records
 * on an engine that has run r rounds). */
void avo_sim_set_round_index(avo_sim* s, int64_t r) { s->round = r; }
int avo_sim_is_byzantine(const avo_sim* s, int64_t node) { return s->byz[node]; }

int avo_sim_add(avo_sim* s, int64_t node, int64_t t, int accepted) {
  int r = avo_processor_add(s->procs[node], t, accepted, s->valid[t]);
  s->pref[node * s->cfg.n_targets + t] = (uint8_t)published_pref_mode(s->procs[node], t, s->responder);
  return r;
}

int avo_sim_register_votes(avo_sim* s, int64_t node, const int64_t* targets, const uint32_t* errs,
                           int64_t n, int64_t* out_targets, int32_t* out_status, int64_t* n_out) {
  int r = avo_processor_register_votes(s->procs[node], targets, errs, n, s->valid, out_targets,
                                       out_status, n_out);
  for (int64_t t = 0; t < s->cfg.n_targets; ++t)
    s->pref[node * s->cfg.n_targets + t] = (uint8_t)published_pref_mode(s->procs[node], t, s->responder);
  return r;
}

typedef struct {
  int64_t* rows; /* 5 columns */
  int64_t n, cap;
} upd_buf;

static void upd_push(upd_buf* b, int64_t r, int64_t node, int64_t slot, int64_t t, int64_t st) {
  if (b->n == b->cap) {
    b->cap = b->cap ? b->cap * 2 : 64;
    b->rows = (int64_t*)realloc(b->rows, (size_t)b->cap * 5 * sizeof(int64_t));
  }
  int64_t* row = b->rows + b->n * 5;
  row[0] = r; row[1] = node; row[2] = slot; row[3] = t; row[4] = st;
  b->n++;
}

/* Packed StatusUpdate word of the device log (include/avhip.h) and the
 * order-independent multiset digest both sides compute over a round's updates:
 * count, sum and xor of splitmix64(word). */
uint64_t avo_pack_update(uint32_t round_rel, int64_t node, int32_t slot, int64_t t, int32_t status) {
  return ((uint64_t)round_rel << 52) | ((uint64_t)node << 28) | ((uint64_t)slot << 24) | ((uint64_t)t << 2) |
         (uint64_t)status;
}

uint64_t avo_mix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}


/* ---- branch-free form of one node's round, poll cap not binding ---------- *
 * Same per-record arithmetic as avo_register_vote (vote.go:54-75) inside
 * RegisterVotes (processor.go:92-117), written without data-dependent
 * branches so that the compiler vectorizes it over the node's targets:
 *   popcount(x) > 6 for a u8 x  <=>  z = ~x & 0xFF has at most one set bit
 *   <=>  (z & (z - 1)) == 0.
 * Used when every live valid record is polled (live valid <= 4096: the cap of
 * processor.go:165-167 cannot bind), so the poll set of each slot is exactly
 * the live valid records in ascending index (R1) and each of them takes one
 * vote per slot. tests/test_oracle.py checks this form against the literal
 * path (avo_sim_set_literal) on random networks and against avo_register_vote
 * on every reachable record state. Records are u32 words votes | consider<<8
 * | confidence<<16 (the avo_vote_record layout on little-endian hosts). */
_Static_assert(sizeof(avo_vote_record) == 4, "avo_vote_record must be 4 bytes");

#if defined(__x86_64__) && defined(__GNUC__)
#define AVO_CLONES __attribute__((target_clones("avx2", "default")))
#else
#define AVO_CLONES
#endif

/* one slot over targets [0, m): votes from yes[t] (err == 0) / cons[t]
 * (int32(err) >= 0); ev[t] = 4 | status for records whose regsiterVote
 * returned true (an appended StatusUpdate), 0 otherwise. Returns the number of
 * regsiterVote applications (live valid records). */
AVO_CLONES static int64_t node_slot_branchfree(uint32_t* restrict rec, uint8_t* restrict present,
                                               uint8_t* restrict decision, const uint8_t* restrict valid,
                                               const uint8_t* restrict yes, const uint8_t* restrict cons,
                                               uint8_t* restrict ev, int64_t m, uint32_t bare) {
  int64_t applied = 0;
  for (int64_t t = 0; t < m; ++t) {
    const uint32_t w = rec[t];
    /* polled: live (present, not finalized) and IsValid (processor.go:95-103, :147-157); bare = a
     * VoteRecord outside any Processor (vote.go alone: votes at any count) */
    const uint32_t pol = (uint32_t)(present[t] & valid[t]) & ((uint32_t)((w >> 17) < AVO_FINALIZATION_SCORE) | bare);
    const uint32_t v = ((w << 1) | yes[t]) & 0xFFu;              /* vote.go:55 */
    const uint32_t c = (((w >> 8) << 1) | cons[t]) & 0xFFu;       /* vote.go:56 */
    const uint32_t zy = ~(v & c) & 0xFFu, zn = (v | ~c) & 0xFFu;  /* zeros of votes&consider, ^votes&consider */
    const uint32_t isyes = (zy & (zy - 1u)) == 0u;                /* vote.go:58 */
    const uint32_t isno = (zn & (zn - 1u)) == 0u;                 /* vote.go:61 */
    const uint32_t concl = isyes | isno;                          /* vote.go:61-63 */
    const uint32_t conf = w >> 16;
    const uint32_t agree = concl & ((conf & 1u) == isyes);        /* vote.go:66 */
    const uint32_t conf2 = agree ? ((conf + 2u) & 0xFFFFu) : (concl ? isyes : conf); /* :67 / :73 */
    const uint32_t changed = concl & (agree ? ((conf2 >> 1) == AVO_FINALIZATION_SCORE) : 1u); /* :68 / :74 */
    const uint32_t fin = changed & ((conf2 >> 1) >= AVO_FINALIZATION_SCORE);                  /* processor.go:114 */
    const uint32_t acc = conf2 & 1u;
    const uint32_t st = fin ? (acc ? AVO_STATUS_FINALIZED : AVO_STATUS_INVALID)
                            : (acc ? AVO_STATUS_ACCEPTED : AVO_STATUS_REJECTED); /* vote.go:77-91 */
    const uint32_t w2 = v | (c << 8) | (conf2 << 16);
    rec[t] = pol ? w2 : w;
    const uint32_t del = pol & fin;                              /* processor.go:114-116 */
    present[t] = (uint8_t)(del ? 0u : present[t]);
    decision[t] = (uint8_t)(del ? acc : decision[t]);
    ev[t] = (uint8_t)((pol & changed) ? (4u | st) : 0u);
    applied += pol;
  }
  return applied;
}

/* The slot's votes as the two bit classes regsiterVote reads (vote.go:55-56):
 * replayed err words, a Byzantine peer's flip-flop answer ((r ^ t) & 1 ? 1 :
 * 0, R4) or the honest peer's published preference (main.go:179-182:
 * IsAccepted ? 0 : 1; never neutral). */
AVO_CLONES static void fill_votes(const uint32_t* restrict errs, int byz, const uint8_t* restrict prow, uint64_t r,
                                  uint8_t* restrict yes, uint8_t* restrict cons, int64_t m) {
  if (errs) {
    for (int64_t t = 0; t < m; ++t) {
      yes[t] = (uint8_t)(errs[t] == 0u);
      cons[t] = (uint8_t)((int32_t)errs[t] >= 0);
    }
  } else if (byz) {
    for (int64_t t = 0; t < m; ++t) {
      yes[t] = (uint8_t)(((r ^ (uint64_t)t) & 1u) == 0u);
      cons[t] = 1u;
    }
  } else {
    for (int64_t t = 0; t < m; ++t) {
      yes[t] = (uint8_t)(prow[t] != 0u);
      cons[t] = 1u;
    }
  }
}

/* live valid records of a node (the size of its uncapped poll set) */
static int64_t node_live_valid(const avo_processor* p, const uint8_t* valid) {
  int64_t n = 0;
  for (int64_t t = 0; t < p->m; ++t) n += p->present[t] & valid[t] & !avo_has_finalized(&p->rec[t]);
  return n;
}

/* The branch-free step over independent records (one vote each, all live and
 * valid): the exhaustive cross-check of node_slot_branchfree against
 * avo_register_vote (tests/test_oracle.py). status[i] = appended Status or -1. */
void avo_transition_batch_branchfree(const uint32_t* words_in, const uint32_t* errs, int64_t n, uint32_t* words_out,
                                     int8_t* status) {
  uint8_t* one = (uint8_t*)malloc((size_t)n + 1);
  uint8_t* dec = (uint8_t*)calloc((size_t)n + 1, 1);
  uint8_t* yes = (uint8_t*)calloc((size_t)n + 1, 1);
  uint8_t* cons = (uint8_t*)calloc((size_t)n + 1, 1);
  uint8_t* ev = (uint8_t*)malloc((size_t)n + 1);
  uint8_t* valid = (uint8_t*)malloc((size_t)n + 1);
  memset(one, 1, (size_t)n + 1);
  memset(valid, 1, (size_t)n + 1);
  for (int64_t i = 0; i < n; ++i) {
    words_out[i] = words_in[i];
    yes[i] = (uint8_t)(errs[i] == 0u);
    cons[i] = (uint8_t)((int32_t)errs[i] >= 0);
  }
  node_slot_branchfree(words_out, one, dec, valid, yes, cons, ev, n, 1u);
  for (int64_t i = 0; i < n; ++i) status[i] = (int8_t)(ev[i] ? (ev[i] & 3) : -1);
  free(one); free(dec); free(yes); free(cons); free(ev); free(valid);
}

void avo_sim_set_literal(avo_sim* s, int literal) { s->literal = literal != 0; }

void avo_sim_set_responder(avo_sim* s, int32_t mode) {
  s->responder = mode;
  const int64_t n = s->cfg.n_nodes, m = s->cfg.n_targets;
  for (int64_t j = 0; j < n; ++j)
    for (int64_t t = 0; t < m; ++t) s->pref[j * m + t] = (uint8_t)published_pref_mode(s->procs[j], t, mode);
}

void avo_sim_set_polling(avo_sim* s, int64_t node, int polls) { s->polls[node] = (uint8_t)(polls != 0); }

/* One synchronous round (R1): every node draws k peers; for slot s it builds
 * the capped poll set (GetInvsForNextPoll, ascending index) and registers one
 * Response whose votes are the peer's round-start published preference
 * (main.go:179-182: IsAccepted ? 0 : 1), Byzantine peers answering
 * ((r ^ t) & 1) (R4), or the replayed err stream. */
int avo_sim_round(avo_sim* s, const uint32_t* replay_errs, int64_t* updates, int64_t cap,
                  int64_t* n_out, int32_t threads, int64_t* applied_votes) {
  return avo_sim_round_ex(s, 0, s->cfg.n_nodes, replay_errs, updates, cap, n_out, threads, applied_votes, NULL, 0);
}

/* The same round for nodes [n0, n1) only (a node shard). Only those rows of
 * the published snapshot are refreshed; the other rows are whatever the
 * caller installed with avo_sim_set_pref_rows (the exchange step). */
int avo_sim_round_range(avo_sim* s, int64_t n0, int64_t n1, const uint32_t* replay_errs, int64_t* updates,
                        int64_t cap, int64_t* n_out, int32_t threads, int64_t* applied_votes) {
  return avo_sim_round_ex(s, n0, n1, replay_errs, updates, cap, n_out, threads, applied_votes, NULL, 0);
}

int avo_sim_round_ex(avo_sim* s, int64_t n0, int64_t n1, const uint32_t* replay_errs, int64_t* updates,
                     int64_t cap, int64_t* n_out, int32_t threads, int64_t* applied_votes, uint64_t digest[3],
                     uint32_t round_rel) {
  const int64_t n_nodes = s->cfg.n_nodes, m = s->cfg.n_targets;
  const int32_t k = s->cfg.k;
  const int64_t r = s->round;
  /* rows are kept per node (reference append order) only when the caller asks for them */
  upd_buf* bufs = updates ? (upd_buf*)calloc((size_t)(n1 - n0), sizeof(upd_buf)) : NULL;
  int64_t applied = 0, total = 0;
  /* the example's responder re-creates every record it is queried for and
   * does not hold (main.go:175-177): marked during the round against the
   * round-start presence, applied after it */
  uint8_t* pres0 = NULL;
  uint8_t* readd = NULL;
  if (s->responder == AVO_RESP_EXAMPLE) {
    pres0 = (uint8_t*)malloc((size_t)(n_nodes * m));
    readd = (uint8_t*)calloc((size_t)(n_nodes * m), 1);
    for (int64_t j = 0; j < n_nodes; ++j) memcpy(pres0 + j * m, s->procs[j]->present, (size_t)m);
  }
  uint64_t dsum = 0, dxor = 0;
  int nt = threads > 0 ? threads : 1;
  (void)nt;
#ifdef _OPENMP
#pragma omp parallel num_threads(nt) reduction(+ : applied, total, dsum) reduction(^ : dxor)
#endif
  {
    /* per-thread scratch, reused for every node of the thread */
    int64_t* peers = (int64_t*)malloc((size_t)k * sizeof(int64_t));
    int64_t* invs = (int64_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int64_t));
    uint32_t* errs = (uint32_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(uint32_t));
    int64_t* ut = (int64_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int64_t));
    int32_t* us = (int32_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int32_t));
    uint8_t* yes = (uint8_t*)malloc((size_t)m + 8);
    uint8_t* cons = (uint8_t*)malloc((size_t)m + 8);
    uint8_t* ev = (uint8_t*)calloc((size_t)m + 8, 1);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 16)
#endif
    for (int64_t node = n0; node < n1; ++node) {
      avo_processor* p = s->procs[node];
      if (!s->polls[node]) continue;  /* a node whose run loop has ended still answers queries */
      avo_sample_peers(s->cfg.seed, node, r, n_nodes, k, s->cfg.peer_mode, peers);
      if (!s->literal && !readd && node_live_valid(p, s->valid) <= AVO_MAX_ELEMENT_POLL) {
        /* cap cannot bind this round (live valid records only decrease within it) */
        for (int32_t slot = 0; slot < k; ++slot) {
          const int64_t peer = peers[slot];
          fill_votes(replay_errs ? replay_errs + (node * k + slot) * m : NULL, s->byz[peer], s->pref + peer * m,
                     (uint64_t)r, yes, cons, m);
          applied += node_slot_branchfree((uint32_t*)p->rec, p->present, p->decision, s->valid, yes, cons, ev, m, 0u);
          const uint64_t* ev8 = (const uint64_t*)ev;
          for (int64_t t0 = 0; t0 < m; t0 += 8) {
            if (t0 + 8 <= m && ev8[t0 >> 3] == 0) continue;
            for (int64_t t = t0; t < m && t < t0 + 8; ++t) {
              if (!ev[t]) continue;
              total++;
              if (bufs) upd_push(&bufs[node - n0], r, node, slot, t, ev[t] & 3);
              const uint64_t h = avo_mix64(avo_pack_update(round_rel, node, slot, t, ev[t] & 3));
              dsum += h;
              dxor ^= h;
            }
          }
        }
        continue;
      }
      for (int32_t slot = 0; slot < k; ++slot) {
        int64_t ni = avo_processor_get_invs(p, s->valid, invs, AVO_MAX_ELEMENT_POLL);
        int64_t peer = peers[slot];
        const uint8_t* prow = s->pref + peer * m;
        for (int64_t i = 0; i < ni; ++i) {
          int64_t t = invs[i];
          uint32_t err;
          if (readd && !pres0[peer * m + t] && s->valid[t]) __atomic_store_n(&readd[peer * m + t], 1, __ATOMIC_RELAXED);
          if (replay_errs) {
            err = replay_errs[(node * k + slot) * m + t];
          } else if (s->byz[peer]) {
            err = ((uint64_t)(r ^ t) & 1u) ? 1u : 0u;
          } else {
            err = prow[t] ? 0u : 1u;
          }
          errs[i] = err;
        }
        int64_t nu = 0;
        applied += ni; /* every polled record is live and valid: one regsiterVote each */
        avo_processor_register_votes(p, invs, errs, ni, s->valid, ut, us, &nu);
        total += nu;
        for (int64_t i = 0; i < nu; ++i) {
          if (bufs) upd_push(&bufs[node - n0], r, node, slot, ut[i], us[i]);
          const uint64_t h = avo_mix64(avo_pack_update(round_rel, node, slot, ut[i], us[i]));
          dsum += h;
          dxor ^= h;
        }
      }
    }
    free(peers); free(invs); free(errs); free(ut); free(us); free(yes); free(cons); free(ev);
  }
  int rc = 0;
  if (n_out) *n_out = total;
  if (digest) {
    digest[0] = (uint64_t)total;
    digest[1] = dsum;
    digest[2] = dxor;
  }
  if (bufs) {
    if (total <= cap) {
      int64_t off = 0;
      for (int64_t node = n0; node < n1; ++node) {
        memcpy(updates + off * 5, bufs[node - n0].rows, (size_t)bufs[node - n0].n * 5 * sizeof(int64_t));
        off += bufs[node - n0].n;
      }
    } else {
      rc = -1;
    }
    for (int64_t node = n0; node < n1; ++node) free(bufs[node - n0].rows);
    free(bufs);
  }
  int64_t p0 = n0, p1 = n1;
  if (readd) {
    for (int64_t j = 0; j < n_nodes; ++j)
      for (int64_t t = 0; t < m; ++t)
        if (readd[j * m + t]) avo_processor_add(s->procs[j], t, 1, s->valid[t]); /* &tx{isAccepted: true} */
    free(pres0);
    free(readd);
    p0 = 0;  /* re-adds touch any node's rows */
    p1 = n_nodes;
  }
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nt)
#endif
  for (int64_t j = p0; j < p1; ++j)
    for (int64_t t = 0; t < m; ++t) s->pref[j * m + t] = (uint8_t)published_pref_mode(s->procs[j], t, s->responder);
  if (applied_votes) *applied_votes = applied;
  s->round++;
  return rc;
}


/* One node's round against an external round-start snapshot: the sampled
 * full-size check of the engine (tests/test_gpu_fullsize.py). words[m] are the
 * node's canonical record words (live: packed VoteRecord; absent: 0xFFFE0000 |
 * decision << 16), updated in place. pref_words: the published preferences as
 * [n_nodes][ceil(m/32)] u32 bitsets (bit t % 32 of word t / 32; the engine's
 * own table), byz_words: [ceil(n_nodes/32)] Byzantine bits, valid[m]. The
 * round follows avo_sim_round_ex's literal path (R1, GetInvsForNextPoll +
 * RegisterVotes per slot; Byzantine peers answer (r ^ t) & 1 ? 1 : 0);
 * digest += {count, sum, xor} of its StatusUpdates; returns the applied votes. */
int64_t avo_node_round_ext(uint64_t seed, int64_t n_nodes, int32_t k, int32_t peer_mode, int64_t node,
                           int64_t round, int64_t m, const uint32_t* pref_words, const uint32_t* byz_words,
                           const uint8_t* valid, uint32_t* words, uint64_t digest[3], uint32_t round_rel) {
  avo_processor* p = avo_processor_new(m);
  for (int64_t t = 0; t < m; ++t) {
    const uint32_t w = words[t];
    if ((w >> 17) >= AVO_FINALIZATION_SCORE) {
      p->present[t] = 0;
      p->decision[t] = (uint8_t)((w >> 16) & 1u);
    } else {
      p->present[t] = 1;
      p->rec[t] = avo_unpack(w);
    }
  }
  const int64_t bl = (m + 31) / 32;
  int64_t* peers = (int64_t*)malloc((size_t)k * sizeof(int64_t));
  int64_t* invs = (int64_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int64_t));
  uint32_t* errs = (uint32_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(uint32_t));
  int64_t* ut = (int64_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int64_t));
  int32_t* us = (int32_t*)malloc(AVO_MAX_ELEMENT_POLL * sizeof(int32_t));
  int64_t applied = 0;
  avo_sample_peers(seed, node, round, n_nodes, k, peer_mode, peers);
  for (int32_t slot = 0; slot < k; ++slot) {
    const int64_t ni = avo_processor_get_invs(p, valid, invs, AVO_MAX_ELEMENT_POLL);
    const int64_t peer = peers[slot];
    const int byz = (int)((byz_words[peer >> 5] >> (peer & 31)) & 1u);
    for (int64_t i = 0; i < ni; ++i) {
      const int64_t t = invs[i];
      if (byz)
        errs[i] = ((uint64_t)(round ^ t) & 1u) ? 1u : 0u;
      else
        errs[i] = ((pref_words[peer * bl + (t >> 5)] >> (t & 31)) & 1u) ? 0u : 1u;
    }
    int64_t nu = 0;
    applied += ni;
    avo_processor_register_votes(p, invs, errs, ni, valid, ut, us, &nu);
    for (int64_t i = 0; i < nu; ++i) {
      const uint64_t h = avo_mix64(avo_pack_update(round_rel, node, slot, ut[i], us[i]));
      digest[0] += 1;
      digest[1] += h;
      digest[2] ^= h;
    }
  }
  for (int64_t t = 0; t < m; ++t) words[t] = avo_processor_dump_word(p, t);
  free(peers); free(invs); free(errs); free(ut); free(us);
  avo_processor_free(p);
  return applied;
}

void avo_sim_set_pref_rows(avo_sim* s, int64_t n0, int64_t n1, const uint8_t* rows) {
  memcpy(s->pref + n0 * s->cfg.n_targets, rows, (size_t)((n1 - n0) * s->cfg.n_targets));
}

void avo_sim_dump(const avo_sim* s, uint32_t* out) { avo_sim_dump_range(s, 0, s->cfg.n_nodes, out, 1); }

void avo_sim_dump_range(const avo_sim* s, int64_t n0, int64_t n1, uint32_t* out, int32_t threads) {
  int64_t m = s->cfg.n_targets;
  int nt = threads > 0 ? threads : 1;
  (void)nt;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nt)
#endif
  for (int64_t j = n0; j < n1; ++j)
    for (int64_t t = 0; t < m; ++t) out[(j - n0) * m + t] = avo_processor_dump_word(s->procs[j], t);
}

void avo_sim_pref(const avo_sim* s, uint8_t* out) {
  memcpy(out, s->pref, (size_t)(s->cfg.n_nodes * s->cfg.n_targets));
}
