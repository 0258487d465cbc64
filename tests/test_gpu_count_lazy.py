"""Deferred count planes (kernels.h `klazy`): in a warm k=8 sim
round in which no record can finalize, a tile whose polled records all agreed
with their accepted bit on all 8 votes gains exactly +8 on every polled count
(vote.go:66-69); it leaves its K planes unstored and counts the pending steps
per tile. Any other access first applies them (k_kl_materialize). These tests
run honest networks (where tiles defer) with reads, validity flips, drop-in
votes and option switches interleaved, and compare with the oracle bit for
bit; and the same network with the option on and off."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

P80 = int(0.8 * 2**32)
P97 = int(0.97 * 2**32)


def rows(u):
    return [tuple(int(v) for v in r) for r in np.asarray(u).tolist()]


def same_state(eng, sim, where):
    got, exp = eng.read_records(), sim.dump()
    if not np.array_equal(got, exp):
        bad = np.argwhere(got != exp)[:5]
        raise AssertionError(f"{where}: {[(int(a), int(b), hex(int(got[a, b])), hex(int(exp[a, b]))) for a, b in bad]}")


CASES = [
    dict(n=200, m=1000, seed=3, p=P97, blocks=0, reads=(5, 11, 19, 27)),     # BL 32 (vv on too)
    dict(n=500, m=256, seed=5, p=P80, blocks=0, reads=(14, 16, 22)),         # BL 8
    dict(n=900, m=100, seed=9, p=P97, blocks=-2, reads=(8, 15, 26)),         # resident (pipelined) grid
    dict(n=64, m=33, seed=2, p=P97, blocks=5, reads=(2, 3, 4, 12, 13, 14)),  # ragged last block, 5 blocks
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c['n']}m{c['m']}")
def test_count_lazy_parity(oracle, case):
    n, m, k = case["n"], case["m"], 8
    eng = avhip.Engine(n, m, k=k, seed=case["seed"], log_capacity=1 << 22)
    eng.set_option("sweep_blocks", case["blocks"])
    eng.init_records(3, case["p"])
    sim = oracle.Sim(n, m, k, seed=case["seed"], init_mode=3, init_param=case["p"])
    rng = np.random.default_rng(case["seed"])
    for r in range(30):
        if r == 9:  # validity flip inside a deferred stretch: pending steps applied first
            eng.set_valid(m - 1, False)
            sim.set_valid(m - 1, False)
        if r == 12:
            eng.set_valid(m - 1, True)
            sim.set_valid(m - 1, True)
        if r == 21:  # drop-in RegisterVotes between rounds
            node = int(rng.integers(0, n))
            ts = rng.integers(0, m, size=30)
            errs = rng.choice(np.array([0, 1], np.uint32), 30)
            st = eng.register_votes(node, ts, errs)
            exp = sim.register_votes(node, ts, errs)
            assert [(int(t), int(s)) for t, s in zip(ts, st) if s >= 0] == exp
        eng.run_rounds(1)
        exp_u, _ = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), f"round {r}"
        if r in case["reads"]:
            same_state(eng, sim, f"round {r}")
    same_state(eng, sim, "end")
    eng.close()


def test_count_lazy_long_runs(oracle):
    """Deferred steps carried over whole run_rounds calls (no read in between),
    then the finalization rounds, where the engine applies them first."""
    n, m = 300, 640
    eng = avhip.Engine(n, m, k=8, seed=21, log_capacity=1 << 22)
    eng.init_records(3, P97)
    sim = oracle.Sim(n, m, 8, seed=21, init_mode=3, init_param=P97)
    exp = []
    for chunk in (3, 9, 4, 8):
        eng.run_rounds(chunk)
        exp += [sim.run_round()[0] for _ in range(chunk)]
    assert rows(eng.fetch_updates()) == rows(np.concatenate(exp))
    same_state(eng, sim, "after 24 rounds")
    eng.close()


def test_count_lazy_on_off_identical():
    """C4 shape at 1/50 scale: identical records, updates and counters with the
    option on and off through warm-up, the warm rounds and finalization; the
    deferring engine moves fewer bytes."""
    n, m = 20_000, 1000
    out = []
    for lazy in (0, 1):
        e = avhip.Engine(n, m, k=8, seed=0xA7A1A9C4, log_capacity=1 << 24)
        e.set_option("count_lazy", lazy)
        e.init_records(3, P80)
        e.run_rounds(12)
        b12 = e.alg_bytes()
        mid = e.read_records()
        e.run_rounds(10)
        out.append((mid, e.read_records(), e.fetch_updates(), e.applied_votes(), e.finalized_count(), b12))
        e.close()
    off, on = out
    for a, b in zip(off[:5], on[:5]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert on[5] < off[5]


def test_count_lazy_bytes():
    """Per-lane bytes of warm k=8 sim rounds of an all-accepted network (every
    tile uniform, vote planes recomputed): round 0 (fresh after init) leaves
    the vote planes virtual, so round 1 regathers them (7 words for the 8-word
    V read) and reads K (the tile is not yet known all-live) but stores
    neither K nor A nor V: 172 - 4 - 68 = 100 B; from round 2 K is not read
    either: 68 B (7 regathered + 8 gathered words, the A read and the
    published word). Round 1 is settled (all 8 votes equal the accepted bit),
    so from round 2 the vote register is the A plane itself (kVUniform):
    nothing is regathered, 40 B (8 gathered words, the A read, the published
    word). Plus the tile's kpend word: read, and written when it changes
    (every deferred round).
    With uniform rows (option uniform_rows, default on; every published row
    equals the reference row, so no vote is gathered) the settled round moves
    8 B per lane: the A read and the published word.
    With the K4..K7 group virtual (option k_hi_virtual, default on: every
    count < 16, kernels.h kHiVirt) round 1 reads 16 B less of K: 84 B.
    With uniform rows round 1's input is uniform too, so its tiles (not yet
    settled candidates) take the reference word as their 8 votes (option
    uni_votes, default on): one 4-B read instead of 32 B of gathers, 28 B less."""
    n, m = 4000, 1000
    for uni, hv, warm, settled in ((0, 0, 100, 40), (1, 0, 72, 8), (1, 1, 56, 8)):
        e = avhip.Engine(n, m, k=8, seed=1, log_capacity=1 << 22)
        e.set_option("uniform_rows", uni)
        e.set_option("k_hi_virtual", hv)
        e.init_records(avhip.INIT_ACCEPTED, 0)
        lanes = e.layout_info()["lanes"]
        tiles = (lanes + 63) // 64
        e.run_rounds(1)  # round 0 fresh: A read, C/K/A/pref written, V virtual
        b = e.alg_bytes()
        e.run_rounds(1)
        assert e.alg_bytes() - b == lanes * warm + tiles * 8, (uni, hv)
        b = e.alg_bytes()
        e.run_rounds(1)
        assert e.alg_bytes() - b == lanes * settled + tiles * 8, (uni, hv)
        assert e.updates_count() == 0
        e.close()


@pytest.mark.parametrize("init", [avhip.INIT_BERNOULLI, avhip.INIT_PAIRS])
def test_k_hi_virtual_on_off_identical(init):
    """C4 shape at 1/50 scale (and the conflicting-pairs form, whose storm
    keeps counts low for longer): identical records, StatusUpdates and
    counters with the virtual K4..K7 group on and off, through the storm, the
    settled rounds, kconsume and finalization, with a mid-run read (virtual
    read of flagged tiles) and a validity flip (write-back); fewer bytes on."""
    n, m = 20_000, 1000
    out = []
    for hv in (0, 1):
        e = avhip.Engine(n, m, k=8, seed=0xA7A1A9C4, log_capacity=1 << 27)
        e.set_option("k_hi_virtual", hv)
        e.init_records(init, P80)
        e.run_rounds(2)
        mid = e.read_records()
        b2 = e.alg_bytes()
        e.run_rounds(3)
        e.set_valid(17, False)
        e.run_rounds(2)
        e.set_valid(17, True)
        e.run_rounds(15)
        out.append((mid, e.read_records(), e.fetch_updates(), e.applied_votes(), e.finalized_count(), b2))
        e.close()
    off, on = out
    for a, b in zip(off[:5], on[:5]):
        assert np.array_equal(np.asarray(a), np.asarray(b))
    assert on[5] < off[5]
