"""StatusUpdate delivery and side-effect-free reads (VERDICT r1 items 4 and
the ADVICE findings): device-side canonical ordering of fetched updates
(dense records expanded and radix-sorted on the device), the update digest
the full-size tests rely on, the engine-kept log base round, reads that do
not write back the deferred vote/count planes, and Processor.GetRound as a
caller-set field (processor.go:40-42)."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)


def test_digest_matches_fetched_words(oracle):
    """av_updates_digest over a multi-round log (round_rel 0..2, singles and
    dense lane records) == the numpy digest of the fetched packed words, and
    the fetched words are the oracle's rows in canonical order."""
    n, m, k = 3000, 2000, 8
    eng = avhip.Engine(n, m, k=k, seed=9, byz_threshold=BYZ20, log_capacity=1 << 25)
    eng.init_records(avhip.INIT_PAIRS, 0)
    sim = oracle.Sim(n, m, k, seed=9, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=8)
    exp = np.concatenate([sim.run_round(threads=8)[0] for _ in range(3)])
    eng.run_rounds(3)
    d = eng.updates_digest()
    raw = eng.fetch_updates(decode=False)
    assert np.all(raw[1:] >= raw[:-1]), "fetched updates not in canonical order"
    assert d == oracle.update_digest(raw)
    assert np.array_equal(avhip.decode_updates(raw, 0), exp)


def test_digest_node_range(oracle):
    n, m, k = 500, 300, 8
    eng = avhip.Engine(n, m, k=k, seed=4)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    eng.run_rounds(2)
    part = eng.updates_digest(100, 250)
    raw = eng.fetch_updates(decode=False)
    node = (raw >> np.uint64(28)) & np.uint64(0xFFFFFF)
    assert part == oracle.update_digest(raw[(node >= 100) & (node < 250)])


def test_log_base_after_overflow(oracle):
    """an overflowed fetch moves the engine's log base to the
    current round; the binding reads the base from the engine, so the rows of
    later rounds decode to their true round numbers."""
    n, m, k = 40, 517, 8
    eng = avhip.Engine(n, m, k=k, seed=5, byz_threshold=BYZ20, log_capacity=64)
    eng.init_records(avhip.INIT_PAIRS, 0)
    sim = oracle.Sim(n, m, k, seed=5, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS)
    overflowed = compared = 0
    for r in range(18):
        eng.run_rounds(1)
        exp, _ = sim.run_round()
        try:
            got = eng.fetch_updates()
        except avhip.LogOverflow:
            overflowed += 1
            assert eng.log_base_round() == eng.round == r + 1
            continue
        assert np.array_equal(got, exp), r
        compared += overflowed > 0 and len(exp) > 0
    assert overflowed >= 1 and compared >= 3, (overflowed, compared)


def test_reads_do_not_write_back_deferred_planes():
    """A read between warm rounds (records, IsAccepted, GetConfidence, poll
    sets) leaves the stale vote planes and pending count steps in place: the
    next round moves the same bytes as without the read, and both engines end
    in the same state."""
    n, m, k = 20_000, 1000, 8
    engs = []
    for _ in range(2):
        e = avhip.Engine(n, m, k=k, seed=13)
        e.init_records(avhip.INIT_BERNOULLI, P80)
        e.run_rounds(6)
        engs.append(e)
    a, b = engs
    rec = a.read_records(100, 200)
    assert a.is_accepted(150, 7) == bool((rec[50, 7] >> 16) & 1)
    assert a.get_confidence(150, 7) == int(rec[50, 7] >> 17)
    a.get_invs(150)
    ba, bb = a.alg_bytes(), b.alg_bytes()
    a.run_rounds(1)
    b.run_rounds(1)
    assert a.alg_bytes() - ba == b.alg_bytes() - bb
    assert np.array_equal(a.read_records(), b.read_records())


def test_read_virtual_matches_oracle(oracle):
    """Reads through stale vote planes (BL >= 16) and pending count steps equal
    the oracle's records every round, across the finalization rounds."""
    n, m, k = 600, 1000, 8
    eng = avhip.Engine(n, m, k=k, seed=21)
    eng.init_records(avhip.INIT_ACCEPTED, 0)
    sim = oracle.Sim(n, m, k, seed=21, init_mode=avhip.INIT_ACCEPTED)
    for r in range(20):
        eng.run_rounds(1)
        sim.run_round()
        eng.discard_updates()
        assert np.array_equal(eng.read_records(), sim.dump()), r


def test_get_round_is_a_processor_field():
    """processor.go:40-42: GetRound returns the Processor's round field, which
    nothing in the Processor advances (the reference test sets it,
    avalanche_test.go:302); batched rounds leave it alone."""
    eng = avhip.Engine(10, 64, k=8)
    eng.init_records(avhip.INIT_ACCEPTED, 0)
    assert eng.get_round(3) == 0
    eng.run_rounds(2)
    assert eng.get_round(3) == 0 and eng.round == 2
    eng.set_round(3, eng.get_round(3) + 1)
    assert eng.get_round(3) == 1 and eng.get_round(4) == 0
    with pytest.raises(avhip.AvError):
        eng.get_round(10)
