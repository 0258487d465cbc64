"""Uniform rows (kernels.h uni_*): every sweep round tags the snapshot it
publishes when some published word differs from the reference node's word of
the round's input snapshot; when the input snapshot carries no tag, every row
of it IS the reference row of the snapshot before, so each gathered vote is
that row's word whoever the peers are, and settled-candidate tiles are tested
with no peer draw and no gather (round_sweep.hip settled_run_uni).

Checked against the oracle (every StatusUpdate, the records, the published
rows) through convergence, the settled rounds and finalization, with API calls
that rewrite snapshots mid-run (drop-in votes, validity flips, adds), with
Byzantine voters (whose flip-flop rows keep every snapshot tagged), and against
the same engine with the option off; the byte counter shows the path was
taken (8 B per settled lane instead of 40)."""
import os

import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

P80 = int(0.8 * 2**32)
BYZ20 = int(0.2 * 2**32)
T = max(1, min(8, os.cpu_count() or 1))


def rows(u):
    return [tuple(int(v) for v in r) for r in np.asarray(u).tolist()]


@pytest.mark.parametrize("n,m,byz,init", [(3000, 1000, 0, avhip.INIT_BERNOULLI), (4000, 256, 0, avhip.INIT_BERNOULLI),
                                          (2500, 1000, BYZ20, avhip.INIT_BERNOULLI), (1500, 64, 0, avhip.INIT_ACCEPTED),
                                          (2000, 517, 0, avhip.INIT_PAIRS)],
                         ids=["bl32", "bl8", "bl32_byz", "bl2_accepted", "ragged_pairs"])
def test_uniform_rows_vs_oracle(oracle, n, m, byz, init):
    eng = avhip.Engine(n, m, k=8, seed=93, byz_threshold=byz, log_capacity=1 << 24)
    eng.init_records(init, P80)
    sim = oracle.Sim(n, m, 8, seed=93, byz_threshold=byz, init_mode=init, init_param=P80, threads=T)
    for r in range(26):
        if r == 9:  # a drop-in Response rewrites node 5's published row mid-run (tags invalidated)
            eng.register_votes(5, [0, 1, 2, 40 % m], [1, 1, 1, 1])
            sim.register_votes(5, [0, 1, 2, 40 % m], np.array([1, 1, 1, 1], np.uint32))
            eng.discard_updates()
        if r == 12:
            eng.set_valid(3, False)
            sim.set_valid(3, False)
        if r == 14:
            eng.set_valid(3, True)
            sim.set_valid(3, True)
        eng.run_rounds(1)
        exp, _ = sim.run_round(threads=T)
        assert rows(eng.fetch_updates()) == rows(exp), f"round {r}"
        if r in (5, 11, 15, 17, 23, 25):
            np.testing.assert_array_equal(eng.read_records(), sim.dump(threads=T), err_msg=f"round {r}")
    honest = [j for j in range(n) if not sim.is_byzantine(j)]
    np.testing.assert_array_equal(eng.read_pref()[honest], sim.pref()[honest])
    eng.close()


def test_uniform_rows_on_off_identical_and_taken():
    """20k x 1000 (C4's row shape), Bernoulli(0.8), honest: the same
    StatusUpdate digests, records, published rows and finalizations with the
    option on and off through the settled rounds and the finalization storm;
    with it on the settled rounds move about a fifth of the bytes."""
    n, m = 20_000, 1000
    out = []
    for on in (1, 0):
        eng = avhip.Engine(n, m, k=8, seed=5, log_capacity=1 << 26)
        eng.set_option("uniform_rows", on)
        eng.init_records(avhip.INIT_BERNOULLI, P80)
        digests, settled_bytes = [], 0
        for r in range(22):
            b0 = eng.alg_bytes()
            eng.run_rounds(1)
            if 7 <= r <= 13:
                settled_bytes += eng.alg_bytes() - b0
            digests.append(eng.updates_digest())
            eng.discard_updates()
        out.append((digests, eng.read_records(), eng.read_pref(), settled_bytes, eng.finalized_count()))
        eng.close()
    on, off = out
    assert on[0] == off[0]
    np.testing.assert_array_equal(on[1], off[1])
    np.testing.assert_array_equal(on[2], off[2])
    assert on[4] == off[4] > 0
    assert on[3] < 0.3 * off[3], (on[3], off[3])


def test_uniform_rows_add_targets_midrun(oracle):
    """An AddTargetToReconcile of dead records after finalization (a snapshot
    rewrite outside the sweep) drops the uniform tag; later rounds agree with
    the oracle."""
    n, m = 1200, 256
    eng = avhip.Engine(n, m, k=8, seed=7, log_capacity=1 << 24)
    eng.init_records(avhip.INIT_ACCEPTED, 0)
    sim = oracle.Sim(n, m, 8, seed=7, init_mode=avhip.INIT_ACCEPTED, init_param=0, threads=T)
    for r in range(24):
        if r == 20:  # every record finalized by now: re-add some as rejected
            got = eng.add_targets(11, [4, 5, 200], [False, False, False])
            exp = [sim.add(11, t, False) for t in (4, 5, 200)]
            assert list(map(bool, got)) == exp
        eng.run_rounds(1)
        e_exp, _ = sim.run_round(threads=T)
        assert rows(eng.fetch_updates()) == rows(e_exp), f"round {r}"
    np.testing.assert_array_equal(eng.read_records(), sim.dump(threads=T))
    eng.close()


@pytest.mark.parametrize("tpw,merge,m", [(4, 4, 1000), (8, 2, 1000), (4, 4, 125), (8, 2, 250), (2, 8, 125)])
def test_uni_merge_on_off_identical(tpw, merge, m):
    """Option uni_merge > 1 (a round with a uniform input: every merge-th wave takes its
    neighbours' runs, the others end at once) changes only the work split, never a result:
    digests, records and published rows equal to uni_merge = 1 at runs of tpw tiles (so that
    tpw * merge <= 16 and the merge really happens). m = 125 / 250 are C4's target
    shards at 8 / 4 ranks (BL 4 / 8): a merged run of 16 tiles holds 256 / 128 nodes."""
    n = 20_000
    out = []
    for um in (1, merge):
        eng = avhip.Engine(n, m, k=8, seed=7, log_capacity=1 << 26)
        eng.set_option("tiles_per_wave", tpw)
        eng.set_option("uni_merge", um)
        eng.init_records(avhip.INIT_BERNOULLI, P80)
        digests = []
        for _ in range(20):
            eng.run_rounds(1)
            digests.append(eng.updates_digest())
            eng.discard_updates()
        out.append((digests, eng.read_records(), eng.read_pref(), eng.finalized_count()))
        eng.close()
    a, b = out
    assert a[0] == b[0]
    np.testing.assert_array_equal(a[1], b[1])
    np.testing.assert_array_equal(a[2], b[2])
    assert a[3] == b[3] > 0


@pytest.mark.parametrize("m,byz", [(1000, 0), (125, 0), (1000, BYZ20)], ids=["bl32", "bl4", "bl32_byz"])
def test_uni_votes_on_off_identical_and_taken(m, byz):
    """Option uni_votes (round_sweep.hip load_tile): with a uniform input snapshot the tiles that
    are not settled candidates take the reference word as their 8 votes instead of gathering them.
    Same digests, records, published rows and finalizations as with it off, through convergence,
    the settled rounds and the finalization storm; with honest voters the converging rounds move
    fewer bytes (the path was taken), with Byzantine voters no snapshot is uniform (nothing changes)."""
    n = 20_000
    out = []
    for on in (1, 0):
        eng = avhip.Engine(n, m, k=8, seed=11, byz_threshold=byz, log_capacity=1 << 26)
        eng.set_option("uni_votes", on)
        eng.init_records(avhip.INIT_BERNOULLI, P80)
        digests, nbytes = [], 0
        for r in range(22):
            b0 = eng.alg_bytes()
            eng.run_rounds(1)
            nbytes += eng.alg_bytes() - b0
            digests.append(eng.updates_digest())
            eng.discard_updates()
        out.append((digests, eng.read_records(), eng.read_pref(), nbytes, eng.finalized_count()))
        eng.close()
    on, off = out
    assert on[0] == off[0]
    np.testing.assert_array_equal(on[1], off[1])
    np.testing.assert_array_equal(on[2], off[2])
    assert on[4] == off[4] > 0
    if byz:
        assert on[3] == off[3]
    else:
        assert on[3] < off[3], (on[3], off[3])
