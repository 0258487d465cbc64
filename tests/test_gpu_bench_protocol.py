"""bench.py's own step sequence pinned against the oracle ("pin
what the bench times"): bench.Runner — the class measure() drives — runs its
exact protocol on a 100k-node x 1000-target C4-shaped network: one untimed warm
epoch (one round per call, log emptied after each), goto(warmup) (re-population
with av_init_records on an engine that has already run 16 rounds, then the
warmup rounds), then the timed steps as measure() runs them (run_rounds of a
whole segment: rounds 5-15 of the second epoch, a re-population, rounds 0-8 of
the third). Every segment's StatusUpdate digest and applied votes are compared
with the oracle (a fresh network per epoch whose round counter starts where
the engine's does: Sim.set_round_index), and the full record state after each
timed segment.

Reference: vote.go:54-91, processor.go:92-117 under SURVEY.md §8(a) R1-R4.
"""
import argparse
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import avhip  # noqa: E402

pytestmark = pytest.mark.gpu

SEED = 0xA7A1A9C4
P80 = int(0.8 * 2**32)


def _threads():
    try:
        return max(1, min(16, len(os.sched_getaffinity(0))))
    except AttributeError:
        return 1


@pytest.mark.parametrize("wl", ["c4_100k", "c4pb_100k"])
def test_bench_runner_protocol_vs_oracle(oracle, monkeypatch, wl):
    bench = pytest.importorskip("bench")
    n, m = 100_000, 1000
    shapes = {"c4_100k": (n, m, 8, avhip.INIT_BERNOULLI, P80, 0, False, "C4 shape at 100k nodes"),
              "c4pb_100k": (n, m, 8, avhip.INIT_PAIRS, 0, bench.BYZ20, False, "C4pb shape at 100k nodes")}
    monkeypatch.setitem(bench.WORKLOADS, wl, shapes[wl])
    _, _, k, init_mode, init_param, byz, _, _ = shapes[wl]
    args = argparse.Namespace(seed=SEED, shard="peers", plane_nt=None, kernel=None, rehearse_one_gpu=False)
    T = _threads()
    warmup, steps, epoch = 5, 20, bench.EPOCH

    # the oracle: one fresh network per epoch, started at the engine's round of that epoch
    state = {"sim": None, "sim_start": None, "checked": 0, "applied": 0}

    def on_segment(run, pos, seg):
        eng = run.eng
        end_round = eng.round  # engine rounds run so far (absolute)
        first = end_round - seg
        # pos = epoch position of the segment's first round; the epoch started at first - pos
        start = first - pos
        if state["sim_start"] != start:
            if state["sim"] is not None:
                state["sim"].close()
            sim = oracle.Sim(n, m, k, seed=SEED, byz_threshold=byz, init_mode=init_mode, init_param=init_param,
                             threads=T)
            sim.set_round_index(start)
            assert pos == 0, "an epoch's first segment starts at its round 0"
            state["sim"], state["sim_start"] = sim, start
        sim = state["sim"]
        assert sim.round == first, (sim.round, first)
        cnt, sm, xr, applied = 0, 0, 0, 0
        for _ in range(seg):
            (c, s_, x), a = sim.run_round(threads=T, collect=False, round_rel=sim.round - eng.log_base_round())
            cnt += c
            sm = (sm + s_) % (1 << 64)
            xr ^= x
            applied += a
        got = eng.updates_digest()
        assert got == (cnt, sm, xr), f"{wl} rounds {first}..{end_round - 1}: digest {got} != oracle {(cnt, sm, xr)}"
        assert eng.applied_votes() - state["applied"] == applied, f"{wl} rounds {first}..{end_round - 1}: applied"
        state["applied"] = eng.applied_votes()
        if seg > 1:  # a timed segment: the whole state after it
            recs = eng.read_records()
            exp = sim.dump(threads=T)
            assert np.array_equal(recs, exp), f"{wl}: state after rounds {first}..{end_round - 1} differs"
            state["checked"] += 1

    run = bench.Runner(wl, args, world=1, rank=0, local_rank=0, log_capacity=400_000_000)
    run.on_segment = on_segment
    try:
        # measure()'s sequence: device warm-up epoch, goto(warmup), the timed steps
        run.steps(epoch, timed=False)
        run.goto(warmup)
        elapsed, applied, emitted, segs = run.steps(steps, timed=True)
        assert segs == 2 and state["checked"] == 2
        assert applied == steps * n * m * k  # every record live in every timed round
        # the roofline pass repeats the same steps from a re-population
        run.goto(warmup)
        run.steps(3, timed=False)
    finally:
        run.close()
        if state["sim"] is not None:
            state["sim"].close()
