"""Parity of the BASELINE configs at their full sizes (VERDICT r1 "Next round"
item 1): the engine through the C ABI against the CPU oracle on the box's host
cores, with the code paths the bench times (recomputed vote registers and
deferred count planes at BL = 32 and 1M nodes for C4; BL = 8 at 10M nodes for
C5; flip-flop voters for C3).

* C4 (1M nodes x 1000 targets, Bernoulli(0.8)) and C3 (100k x 2000, 20 %
  Byzantine, double-spend pairs): every round's StatusUpdates are compared as
  an order-independent digest (count, sum and xor of splitmix64 over the
  packed words: av_updates_digest vs the oracle's avo_sim_round_ex; in some
  rounds the whole stream delivered to the host, in canonical order), the
  applied-vote count every round, and the full record state at several rounds
  including the finalization storm (C4 rounds 16-18). C3 also compares the
  full update rows of some rounds.
* C5 (10M x 256): the oracle cannot hold the whole network in these tests'
  time, so every round checks a random contiguous range of 2048 nodes exactly:
  their records before the round plus the engine's own published snapshot go
  through the oracle's literal per-node round (avo_node_round_ext), and the
  records after the round and the range's update digest must match. Plus the
  whole-network properties: N*M*k applied votes per all-live round, every
  record finalized by round 19, published preference == accepted bit.

Reference: vote.go:54-91, processor.go:92-117 under SURVEY.md §8(a) R1-R4.
"""
import os

import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

SEED = 0xA7A1A9C4
P80 = int(0.8 * 2**32)
BYZ20 = int(0.2 * 2**32)


def host_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


T = host_threads()


def compare_state(eng, sim, n, where, chunk=100_000):
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        got = eng.read_records(a, b)
        exp = sim.dump(a, b, threads=T)
        if not np.array_equal(got, exp):
            bad = np.argwhere(got != exp)[:5]
            msg = [(int(a + i), int(j), hex(int(got[i, j])), hex(int(exp[i, j]))) for i, j in bad]
            raise AssertionError(f"state mismatch {where}: {msg}")


def step(eng, sim, r, collect_rows=False, order=None):
    """One round on both sides; StatusUpdates compared (digest, or rows). order="words" / "compact":
    the round's whole stream is delivered to the host (av_fetch_updates, or the compact stream
    expanded by av_compact_expand) and must be strictly ascending packed words — the canonical
    (round, node, slot, target) order, processor.go:94,111 — whose digest equals the oracle's: a
    sorted sequence of distinct words is fixed by its set, so this pins the full-size stream's order
    and content without holding the oracle's rows."""
    eng.run_rounds(1)
    if order:
        from oracle import cabi
        if order == "compact":
            s = eng.fetch_compact()
            assert avhip.compact_header(s)["log_base"] == eng.round - 1
            raw = avhip.compact_expand(s)
            del s
        else:
            raw = eng.fetch_updates(decode=False)
        exp, applied = sim.run_round(threads=T, collect=False, round_rel=0)
        assert raw.size == exp[0], f"round {r}: {raw.size} words, oracle {exp[0]}"
        assert np.all(raw[1:] > raw[:-1]), f"round {r}: delivered words not in canonical order"
        assert cabi.update_digest(raw) == exp, f"round {r}: delivered stream differs from the oracle's"
        return applied, exp[0]
    if collect_rows:
        got = eng.fetch_updates()
        exp, applied = sim.run_round(threads=T)
        assert np.array_equal(got, exp), f"round {r}: update rows differ"
        return applied, len(exp)
    got = eng.updates_digest()
    eng.discard_updates()
    exp, applied = sim.run_round(threads=T, collect=False, round_rel=0)
    assert got == exp, f"round {r}: update digest {got} != oracle {exp}"
    return applied, exp[0]


# ------------------------------------------------------------------ C4
C4 = dict(n=1_000_000, m=1000)


@pytest.fixture(scope="module")
def c4_pair(oracle):
    n, m = C4["n"], C4["m"]
    # the log holds round 17's storm (528M updates, mostly dense lane records)
    eng = avhip.Engine(n, m, k=8, seed=SEED, log_capacity=600_000_000)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    sim = oracle.Sim(n, m, 8, seed=SEED, init_mode=avhip.INIT_BERNOULLI, init_param=P80, threads=T)
    st = {"applied": 0, "round": 0}
    yield eng, sim, st
    eng.close()
    sim.close()


# rounds whose whole stream is delivered to the host in canonical order (step's `order`)
C4_ORDER = {1: "words", 17: "compact"}
C4P_ORDER = {3: "compact", 12: "words"}


def run_c4(c4_pair, last, states):
    eng, sim, st = c4_pair
    n, m = C4["n"], C4["m"]
    while st["round"] <= last:
        r = st["round"]
        applied, _ = step(eng, sim, r, order=C4_ORDER.get(r))
        st["applied"] += applied
        st["round"] += 1
        if r < 16:  # all records live: every node polls every target k times (R1)
            assert applied == n * m * 8, r
        assert eng.applied_votes() == st["applied"], r
        if r in states:
            compare_state(eng, sim, n, f"C4 after round {r}")


def test_c4_fullsize_rounds_0_7(c4_pair):
    """Convergence rounds (0-3: cold consider planes, ~1e8 updates per round)
    and the first settled rounds (vv + deferred counts)."""
    run_c4(c4_pair, 7, {0, 3, 7})


def test_c4_fullsize_rounds_8_15(c4_pair):
    """Warm settled rounds: stale vote planes, pending count steps; round 15
    writes the pending steps back (a record may reach 128 in round 16)."""
    run_c4(c4_pair, 15, {12, 15})


def test_c4_fullsize_rounds_16_20(c4_pair):
    """The finalization storm (rounds 16-18: 400M / 528M / 72M records
    finalize and are deleted, processor.go:114-116) through the quiet end."""
    eng, sim, st = c4_pair
    run_c4(c4_pair, 20, {16, 17, 18, 20})
    n, m = C4["n"], C4["m"]
    assert eng.finalized_count() == n * m
    assert eng.live_records() == 0


# ------------------------------------------------------------------ C4p / C4pb
# The north star's "1M nodes x 1k conflicting targets": targets (2p, 2p+1) are
# double-spend pairs with complementary initial IsAccepted per node (SURVEY.md
# R4), honest (c4p) or with 20 % Byzantine flip-flop voters (c4pb, as C3).
# Flips go on round after round (no record settles), so every round takes the
# general step and emits StatusUpdates.
C4P = dict(n=1_000_000, m=1000)


def c4p_fixture(byz):
    n, m = C4P["n"], C4P["m"]
    eng = avhip.Engine(n, m, k=8, seed=SEED, byz_threshold=byz, log_capacity=600_000_000)
    eng.init_records(avhip.INIT_PAIRS, 0)
    return eng


@pytest.fixture(scope="module")
def c4pb_pair(oracle):
    n, m = C4P["n"], C4P["m"]
    eng = c4p_fixture(BYZ20)
    sim = oracle.Sim(n, m, 8, seed=SEED, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=T)
    st = {"applied": 0, "round": 0, "emitted": []}
    yield eng, sim, st
    eng.close()
    sim.close()


def run_c4p(pair, last, states):
    eng, sim, st = pair
    n, m = C4P["n"], C4P["m"]
    while st["round"] <= last:
        r = st["round"]
        applied, nupd = step(eng, sim, r, order=C4P_ORDER.get(r))
        print(f"C4p(b) round {r}: {nupd} StatusUpdates, digest equal", flush=True)
        st["applied"] += applied
        st["emitted"].append(nupd)
        st["round"] += 1
        if r < 16:  # nothing can finalize before round 16 (>= 134 votes): all N*M*k applied
            assert applied == n * m * 8, r
        assert eng.applied_votes() == st["applied"], r
        if r in states:
            compare_state(eng, sim, n, f"C4p(b) after round {r}")


def test_c4pb_fullsize_rounds_0_10(c4pb_pair):
    """1M x 500 double-spend pairs with 20 % Byzantine flip-flop voters: the
    update digest every round, the full state at rounds 3 and 10."""
    run_c4p(c4pb_pair, 10, {3, 10})
    # conflicting preferences keep flipping: every round emits StatusUpdates
    assert all(e > 0 for e in c4pb_pair[2]["emitted"]), c4pb_pair[2]["emitted"]


def test_c4pb_fullsize_rounds_11_20(c4pb_pair):
    """Through the first finalizations (round 16 on) to round 20."""
    run_c4p(c4pb_pair, 20, {16, 20})


@pytest.fixture(scope="module")
def c4p_pair(oracle):
    n, m = C4P["n"], C4P["m"]
    eng = c4p_fixture(0)
    sim = oracle.Sim(n, m, 8, seed=SEED, init_mode=avhip.INIT_PAIRS, threads=T)
    st = {"applied": 0, "round": 0, "emitted": []}
    yield eng, sim, st
    eng.close()
    sim.close()


def test_c4p_honest_rounds_0_7(c4p_pair):
    """The honest pairs network (c4p), rounds 0-7: digests every round, state at rounds 6 and 7
    (the bench times rounds 5-15 and 0-8 of it: VERDICT r3 'pin what the bench times')."""
    run_c4p(c4p_pair, 7, {6, 7})


def test_c4p_honest_rounds_8_20(c4p_pair):
    """Honest c4p through the rest of the bench's epoch (rounds 8-15: klazy rounds with the
    uniform-rows and deferred-count interplay at 1M nodes), the first round that applies the
    deferred count steps (16) and the first finalizations, to round 20."""
    run_c4p(c4p_pair, 20, {15, 16, 20})


# ------------------------------------------------------------------ C3
C3 = dict(n=100_000, m=2000)


@pytest.fixture(scope="module")
def c3_pair(oracle):
    n, m = C3["n"], C3["m"]
    eng = avhip.Engine(n, m, k=8, seed=SEED, byz_threshold=BYZ20, log_capacity=200_000_000)
    eng.init_records(avhip.INIT_PAIRS, 0)
    sim = oracle.Sim(n, m, 8, seed=SEED, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=T)
    st = {"applied": 0, "round": 0}
    yield eng, sim, st
    eng.close()
    sim.close()


def run_c3(c3_pair, last, states, rows):
    eng, sim, st = c3_pair
    while st["round"] <= last:
        r = st["round"]
        applied, nupd = step(eng, sim, r, collect_rows=r in rows)
        st["applied"] += applied
        st["round"] += 1
        assert eng.applied_votes() == st["applied"], r
        if r in states:
            compare_state(eng, sim, C3["n"], f"C3 after round {r}")


def test_c3_fullsize_rounds_0_25(c3_pair):
    """Flip-flop voters keep every tile unsettled; finalization starts at round 18."""
    run_c3(c3_pair, 25, states={5, 17, 25}, rows={0, 6, 19})


def test_c3_fullsize_rounds_26_52(c3_pair):
    """Through the last honest finalization (round 51 in the r01 convergence run)."""
    eng, _, _ = c3_pair
    run_c3(c3_pair, 52, states={40, 52}, rows={30})
    assert eng.live_records(honest_only=True) == 0


# ------------------------------------------------------------------ C5
def test_c5_fullsize_sampled_oracle(oracle):
    """C5 at full size (10M nodes x 256 targets, k = 8, Bernoulli(0.8), BL = 8):
    every round, 2048 consecutive nodes at a random offset are checked exactly
    against the oracle's literal per-node round on the engine's own snapshot;
    whole-network properties throughout."""
    n, m, k = 10_000_000, 256, 8
    eng = avhip.Engine(n, m, k=k, seed=SEED, log_capacity=1_500_000_000)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    byz = oracle.byz_words(SEED, n, 0)
    valid = np.ones(m, np.uint8)
    rng = np.random.default_rng(5)
    S = 2048
    live_after = []
    total_applied = 0
    for r in range(20):
        a = int(rng.integers(0, n - S))
        before = eng.read_records(a, a + S)
        pref = eng.read_pref_words()
        exp_digest = np.zeros(3, np.uint64)
        exp_applied = 0
        words = before.copy()
        for i in range(S):
            row = np.ascontiguousarray(words[i])
            exp_applied += oracle.node_round_ext(SEED, n, k, 0, a + i, eng.round, m, pref, byz, valid, row,
                                                 exp_digest)
            words[i] = row
        a0 = eng.applied_votes()
        eng.run_rounds(1)
        applied = eng.applied_votes() - a0
        total_applied += applied
        got_digest = eng.updates_digest(a, a + S)
        eng.discard_updates()
        after = eng.read_records(a, a + S)
        assert np.array_equal(after, words), f"round {r}: records of nodes [{a}, {a + S}) differ"
        assert got_digest == tuple(int(v) for v in exp_digest), f"round {r}: update digest of [{a}, {a + S})"
        if r < 16:
            assert applied == n * m * k, r
            assert exp_applied == S * m * k, r
        if r == 15:  # every record live; published preference == its accepted bit (R2)
            recs = eng.read_records(0, 50_000)
            assert ((recs >> 17) < 128).all()
            assert np.array_equal(eng.read_pref(0, 50_000), ((recs >> 16) & 1).astype(np.uint8))
        live_after.append(eng.live_records())
    # rounds to finalization: nothing before round 16 (>= 134 votes), all by round 19
    assert live_after[15] == n * m and live_after[18] > 0 and live_after[19] == 0, live_after
    assert eng.finalized_count() == n * m
    recs = eng.read_records(n - 50_000, n)
    assert (recs >> 16 == (avhip.ABSENT_WORD >> 16) | ((recs >> 16) & 1)).all()
    # a finalized node publishes its decision (R2)
    assert np.array_equal(eng.read_pref(n - 50_000, n), ((recs >> 16) & 1).astype(np.uint8))
    eng.close()


def test_c5_whole_network_rounds_0_5(oracle):
    """C5's whole network (10M nodes x 256 targets, BL = 8) against the oracle holding all of it
    (C5 parity was sampled only): rounds 0-5 (the fresh round, the storm rounds and the
    first settled ones) with every round's update digest over all nodes, the applied votes, one
    round's stream delivered in canonical order, and the full record state after rounds 2 and 5."""
    n, m, k = 10_000_000, 256, 8
    eng = avhip.Engine(n, m, k=k, seed=SEED, log_capacity=1_500_000_000)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    sim = oracle.Sim(n, m, k, seed=SEED, init_mode=avhip.INIT_BERNOULLI, init_param=P80, threads=T)
    try:
        for r in range(6):
            applied, nupd = step(eng, sim, r, order="compact" if r == 1 else None)
            print(f"C5 round {r}: {nupd} StatusUpdates equal", flush=True)
            assert applied == n * m * k, r
            if r in (2, 5):
                compare_state(eng, sim, n, f"C5 after round {r}", chunk=500_000)
    finally:
        eng.close()
        sim.close()
