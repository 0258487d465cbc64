"""The round after av_init_records ("fresh": every record a NewVoteRecord,
vote.go:33-35, so only the A plane is read) and the warm round that applies
pending count steps itself instead of a separate write-back pass
("kconsume", the first round in which a record can reach 128). Both are
compared with the engine running every plane through memory (option
"fresh" 0, "count_lazy" 0) and with the oracle."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)

CASES = [
    # n, m, k, byz, init_mode, invalid targets before round 0
    (300, 1000, 8, 0, avhip.INIT_BERNOULLI, ()),        # BL 32: fresh + virtual votes
    (500, 517, 8, BYZ20, avhip.INIT_PAIRS, (3, 516)),    # ragged last block, invalid targets: keep records
    (700, 200, 8, 0, avhip.INIT_ACCEPTED, ()),           # BL 7: fresh, no virtual votes
    (90, 333, 5, BYZ20, avhip.INIT_REJECTED, (0,)),      # k = 5
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c[0]}m{c[1]}k{c[2]}")
def test_fresh_round_vs_oracle(oracle, case):
    n, m, k, byz, init_mode, invalid = case
    eng = avhip.Engine(n, m, k=k, seed=17, byz_threshold=byz, log_capacity=1 << 22)
    eng.init_records(init_mode, P80)
    sim = oracle.Sim(n, m, k, seed=17, byz_threshold=byz, init_mode=init_mode, init_param=P80)
    for t in invalid:
        eng.set_valid(t, False)
        sim.set_valid(t, False)
    for r in range(20):
        eng.run_rounds(1)
        exp, _ = sim.run_round()
        assert np.array_equal(eng.fetch_updates(), exp), r
        if r in (0, 1, 15, 16, 19):
            assert np.array_equal(eng.read_records(), sim.dump()), r


def test_fresh_and_kconsume_identical_to_stored_planes():
    """C4 shape at 1/50 scale through finalization: the fresh round 0 and the
    consuming round 16 change nothing but the bytes moved; a re-initialised
    engine is fresh again."""
    n, m = 20_000, 1000
    out = []
    for opt in (0, 1):
        e = avhip.Engine(n, m, k=8, seed=0xA7A1A9C4, log_capacity=1 << 27)
        e.set_option("count_lazy", opt)
        for epoch in range(2):
            e.init_records(avhip.INIT_BERNOULLI, P80)
            if not opt:
                e.set_option("fresh", 0)
            e.run_rounds(20)
        out.append((e.read_records(), e.fetch_updates(), e.applied_votes(), e.finalized_count(), e.alg_bytes()))
        e.close()
    off, on = out
    for a, b in zip(off[:4], on[:4]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert on[4] < off[4]


@pytest.mark.parametrize("path", ["set_valid", "register_votes", "replay", "write_records", "add_targets", "none"])
def test_fresh_virtual_consider_writeback(oracle, path):
    """The fresh round leaves the consider planes of its tiles unstored
    (kernels.h kCAll: all-ones after 8 sim votes). Every operation that reads
    or writes the planes right after it must see them as all-ones (write-back
    in k_vv_materialize; k_read_records_v reads them virtually); the rounds
    after it must match the oracle bit for bit."""
    n, m, k, seed = 300, 1000, 8, 29
    eng = avhip.Engine(n, m, k=k, seed=seed, log_capacity=1 << 22)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    sim = oracle.Sim(n, m, k, seed=seed, init_mode=avhip.INIT_BERNOULLI, init_param=P80)
    rng = np.random.default_rng(seed)
    eng.run_rounds(1)  # fresh
    exp, _ = sim.run_round()
    assert np.array_equal(eng.fetch_updates(), exp)
    assert np.array_equal(eng.read_records(), sim.dump())  # virtual read of kCAll tiles
    if path == "set_valid":
        eng.set_valid(40, False)
        sim.set_valid(40, False)
    elif path == "register_votes":
        node = 17
        ts = rng.integers(0, m, size=64)
        errs = rng.choice(np.array([0, 1, 0x80000000, 0x7FFFFFFF], np.uint32), 64)
        st = eng.register_votes(node, ts, errs)
        got = sim.register_votes(node, ts, errs)
        assert [(int(t), int(s)) for t, s in zip(ts, st) if s >= 0] == got
    elif path == "replay":
        errs = rng.choice(np.array([0, 1, 0x80000000], np.uint32), size=(n, k, m)).astype(np.uint32)
        eng.replay_round_errs(errs)
        exp, _ = sim.run_round(replay_errs=errs)
        assert np.array_equal(eng.fetch_updates(), exp)
    elif path == "write_records":
        eng.write_records(eng.read_records()[:50], n0=0, t0=0)
    elif path == "add_targets":
        assert not eng.add_targets(5, [7, 8], [True, False]).any()  # live records: no-op
        assert not sim.add(5, 7, True) and not sim.add(5, 8, False)
    assert np.array_equal(eng.read_records(), sim.dump()), path
    for r in range(8):
        eng.run_rounds(1)
        exp, _ = sim.run_round()
        assert np.array_equal(eng.fetch_updates(), exp), (path, r)
    assert np.array_equal(eng.read_records(), sim.dump()), path
    eng.close()
