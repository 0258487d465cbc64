"""Reference rows (kernels.h ref_node / rflag_*): in a converged network every
honest node publishes the same row, so a sweep round flags each node whose
published row equals the reference node's row, and the next round's settled
tiles read the reference row once instead of gathering 8 peer rows that are,
bit for bit, that row. Checked against the oracle (every StatusUpdate, the
records) through convergence, the settled rounds, finalization and API calls
that rewrite the snapshot (drop-in votes, validity flips), and against the same
engine with the option off; the byte counter shows the path was taken."""
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


@pytest.mark.parametrize("n,m,byz", [(3000, 1000, 0), (4000, 256, 0), (2500, 1000, BYZ20), (1500, 64, 0)],
                         ids=["bl32", "bl8", "bl32_byz", "bl2"])
def test_ref_rows_vs_oracle(oracle, n, m, byz):
    eng = avhip.Engine(n, m, k=8, seed=91, byz_threshold=byz, log_capacity=1 << 24)
    eng.set_option("uniform_rows", 0)  # uniform rows would take the settled tiles first
    eng.set_option("ref_rows", 1)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    sim = oracle.Sim(n, m, 8, seed=91, byz_threshold=byz, init_mode=avhip.INIT_BERNOULLI, init_param=P80, threads=T)
    for r in range(24):
        if r == 9:  # a drop-in Response rewrites node 5's published row mid-run (flags invalidated)
            eng.register_votes(5, [0, 1, 2, 40], [1, 1, 1, 1])
            sim.register_votes(5, [0, 1, 2, 40], np.array([1, 1, 1, 1], np.uint32))
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
        if r in (5, 11, 15, 17, 23):
            np.testing.assert_array_equal(eng.read_records(), sim.dump(threads=T), err_msg=f"round {r}")
    honest = [j for j in range(n) if not sim.is_byzantine(j)]
    np.testing.assert_array_equal(eng.read_pref()[honest], sim.pref()[honest])


def test_ref_rows_on_off_identical_and_taken():
    """20k x 1000 (C4's row shape): the same StatusUpdates, records and
    published rows with the option on and off; fewer bytes moved with it on
    in the settled rounds (the 8 gathered rows replaced by one reference row)."""
    n, m = 20_000, 1000
    out = []
    for on in (1, 0):
        eng = avhip.Engine(n, m, k=8, seed=5, log_capacity=1 << 26)
        eng.set_option("uniform_rows", 0)  # (test_gpu_uniform_rows.py): the settled rounds would gather nothing
        eng.set_option("ref_rows", on)
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
    assert on[3] < 0.7 * off[3], (on[3], off[3])
