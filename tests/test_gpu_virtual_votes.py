"""Recomputed vote registers (kernels.h `vv`): after a warm k=8
sim round a tile may leave its vote planes unstored, because a record's vote
register after 8 sim votes is exactly that round's 8 gathered votes
(vote.go:55). The next round regathers them from the previous snapshot; any
other access first writes them back (k_vv_materialize). These tests run long
stretches of rounds with no state read in between (stale tiles carried from
round to round), interleave every operation that must write the planes back,
and compare with the oracle bit for bit."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)


def rows(u):
    return [tuple(int(v) for v in r) for r in np.asarray(u).tolist()]


def same_state(eng, sim, where):
    got, exp = eng.read_records(), sim.dump()
    if not np.array_equal(got, exp):
        bad = np.argwhere(got != exp)[:5]
        raise AssertionError(f"{where}: {[(int(a), int(b), hex(int(got[a, b])), hex(int(exp[a, b]))) for a, b in bad]}")


CASES = [
    dict(n=64, m=200, seed=3, init=3, byz=BYZ20, min_bl=1, blocks=0),      # BL 7, forced on
    dict(n=300, m=517, seed=5, init=4, byz=BYZ20, min_bl=None, blocks=0),  # BL 17: on by default
    dict(n=700, m=333, seed=17, init=2, byz=BYZ20, min_bl=1, blocks=-2),   # resident grid (pipelined)
    dict(n=50, m=1000, seed=8, init=3, byz=0, min_bl=None, blocks=7),      # BL 32, 7-block grid
    dict(n=9, m=600, seed=2, init=1, byz=int(0.45 * 2**32), min_bl=None, blocks=0),  # tiles straddle nodes
]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"n{c['n']}m{c['m']}")
def test_virtual_votes_parity(oracle, case):
    n, m, k = case["n"], case["m"], 8
    eng = avhip.Engine(n, m, k=k, seed=case["seed"], byz_threshold=case["byz"], log_capacity=1 << 22)
    if case["min_bl"] is not None:
        eng.set_option("vv_min_bl", case["min_bl"])
    eng.set_option("sweep_blocks", case["blocks"])
    eng.init_records(case["init"], P80)
    sim = oracle.Sim(n, m, k, seed=case["seed"], byz_threshold=case["byz"], init_mode=case["init"], init_param=P80)
    rng = np.random.default_rng(case["seed"])
    for r in range(26):
        if r == 7:  # validity flip: planes written back, the wave holding t stores its planes
            eng.set_valid(5, False)
            sim.set_valid(5, False)
        if r == 10:
            eng.set_valid(5, True)
            sim.set_valid(5, True)
        if r == 12:  # drop-in RegisterVotes on one node between rounds
            node = int(rng.integers(0, n))
            ts = rng.integers(0, m, size=40)
            errs = rng.choice(np.array([0, 1, 0x80000000], np.uint32), 40)
            st = eng.register_votes(node, ts, errs)
            exp = sim.register_votes(node, ts, errs)
            assert [(int(t), int(s)) for t, s in zip(ts, st) if s >= 0] == exp
        eng.run_rounds(1)
        exp_u, _ = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), f"round {r}"
        if r in (3, 9, 17, 25):  # reads between long runs of rounds with stale tiles
            same_state(eng, sim, f"round {r}")
    eng.close()


def test_virtual_votes_on_off_identical():
    """Same network with and without recomputed vote registers: identical
    records, updates and counters through warm-up, the warm rounds and the
    finalization rounds (16-18); the vv engine moves fewer bytes."""
    n, m = 20_000, 1000
    out = []
    for vv in (0, 1):
        e = avhip.Engine(n, m, k=8, seed=0xA7A1A9C4, log_capacity=1 << 24)
        e.set_option("virtual_votes", vv)
        e.init_records(avhip.INIT_BERNOULLI, P80)
        e.run_rounds(20)
        out.append((e.read_records(), e.fetch_updates(), e.applied_votes(), e.finalized_count(), e.alg_bytes()))
        e.close()
    (r0, u0, a0, f0, b0), (r1, u1, a1, f1, b1) = out
    assert np.array_equal(r0, r1)
    assert np.array_equal(u0, u1)
    assert (a0, f0) == (a1, f1)
    assert f0 > 0
    assert b1 < b0


def test_virtual_votes_bytes():
    """Per-lane bytes of a warm k=8 sim round: 172 B with stored vote planes;
    140 B in the first round that leaves them unstored (no V write); 136 B
    once the tile is stale (7 regathered words instead of the 8 V planes);
    108 B once the tile was settled (the vote register is the A plane);
    80 B when, in addition, the round's input snapshot is uniform (option
    uni_votes: one reference word read instead of the 8 gathered votes)."""
    n, m = 4000, 1000
    for uv, per_lane in ((0, 108), (1, 80)):
        e = avhip.Engine(n, m, k=8, seed=1, log_capacity=1 << 22)
        e.set_option("count_lazy", 0)  # count planes stored every round (test_gpu_count_lazy.py)
        e.set_option("uni_votes", uv)
        e.init_records(avhip.INIT_ACCEPTED, 0)
        lanes = e.layout_info()["lanes"]
        e.run_rounds(2)  # round 0 fresh (V left virtual); round 1 warm and stale
        b = e.alg_bytes()
        e.run_rounds(1)
        assert e.alg_bytes() - b == lanes * per_lane + 0  # round 1 settled: uniform; no updates, no flips
        e.close()
