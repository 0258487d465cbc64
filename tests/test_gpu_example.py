"""examples/basic-preconcensus (BASELINE config C1, main.go:91-192) and the
responder variants of SURVEY R2 on the engine, bit for bit against the
oracle: responder 1 publishes IsAccepted literally (false after deletion,
processor.go:125-130); responder 2 is the example's responder, which re-adds
a queried target it does not hold as accepted and answers yes
(main.go:175-182); nodes whose run loop returned (main.go:143-162) stop
polling but keep answering (av_set_polling)."""
import os
import subprocess

import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("responder", [1, 2])
def test_responder_modes_vs_oracle(oracle, responder):
    n, m, k = 24, 70, 3
    byz = int(0.2 * 2**32)
    eng = avhip.Engine(n, m, k=k, seed=6, byz_threshold=byz)
    eng.init_records(avhip.INIT_ACCEPTED, 0)
    eng.set_option("responder", responder)
    sim = oracle.Sim(n, m, k, seed=6, byz_threshold=byz, init_mode=avhip.INIT_ACCEPTED)
    sim.set_responder(responder)
    honest = [j for j in range(n) if not sim.is_byzantine(j)]
    for r in range(60):
        if r == 30:
            for j in (2, 5, 11):
                eng.set_polling(j, False)
                sim.set_polling(j, False)
        if r == 20:
            eng.set_valid(4, False)
            sim.set_valid(4, False)
        eng.run_rounds(1)
        exp, _ = sim.run_round()
        assert np.array_equal(eng.fetch_updates(), exp), r
        assert np.array_equal(eng.read_records(), sim.dump()), r
        assert np.array_equal(eng.read_pref()[honest], sim.pref()[honest]), r


def test_example_c1_vs_oracle(oracle):
    """100 nodes x 100 txs, every tx accepted by every node, round-robin
    polling skipping self with one poll per round (k = 1), the example's
    responder, each node's loop returning after it counted 100 Finalized
    updates: every round's StatusUpdates and the final records equal the
    oracle's, and all 100 nodes finish ("Nodes fully finalized: 100")."""
    n = m = 100
    eng = avhip.Engine(n, m, k=1, peer_mode=avhip.PEERS_ROUND_ROBIN)
    eng.init_records(avhip.INIT_ACCEPTED, 0)
    eng.set_option("responder", 2)
    sim = oracle.Sim(n, m, 1, peer_mode=1, init_mode=avhip.INIT_ACCEPTED)
    sim.set_responder(2)
    finalized = np.zeros(n, np.int64)
    rounds = 0
    while (finalized < m).any() and rounds < 2000:
        eng.run_rounds(1)
        got = eng.fetch_updates()
        exp, _ = sim.run_round()
        assert np.array_equal(got, exp), rounds
        np.add.at(finalized, got[got[:, 4] == avhip.STATUS_FINALIZED, 1], 1)
        for j in np.flatnonzero(finalized >= m):
            eng.set_polling(int(j), False)
            sim.set_polling(int(j), False)
        rounds += 1
    assert (finalized >= m).all() and rounds == 134
    assert np.array_equal(eng.read_records(), sim.dump())


def test_example_binary():
    """The C++ example (go-avalanche_amd/examples/basic_preconsensus.cpp) in
    its literal mode prints the example's final line."""
    exe = os.path.join(ROOT, "go-avalanche_amd", "bin", "basic_preconsensus")
    out = subprocess.run([exe, "-literal"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "Nodes fully finalized: 100" in out.stdout
