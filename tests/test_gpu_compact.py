"""StatusUpdate delivery through the hand-written device encoder (log_ops.hip:
counting sort by (round, node) bucket, per-bucket (slot, target) layout; no
library sort or scan): av_fetch_updates against the oracle, the compact stream
(av_fetch_compact) byte for byte against the test-side restatement of its
format (compact_ref.py) applied to the same engine's packed words, and the
pipelined delivery (av_fetch_compact_async / _wait) round by round against the
oracle. processor.go:61,111 (*[]StatusUpdate, appended in vote order :94)."""
import numpy as np
import pytest

import avhip
from compact_ref import encode

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)


def twin(n, m, k, seed, byz=0, init=(avhip.INIT_BERNOULLI, P80), opts=(), **kw):
    out = []
    for _ in range(2):
        e = avhip.Engine(n, m, k=k, seed=seed, byz_threshold=byz, **kw)
        for name, v in opts:
            e.set_option(name, v)
        e.init_records(*init)
        out.append(e)
    return out


def check_compact(a, b, rounds_run):
    """a: fetch_updates; b: fetch_compact; the same engine state and log."""
    base = a.log_base_round()
    words = a.fetch_updates(decode=False)
    assert np.all(words[1:] > words[:-1]), "packed words not strictly ascending (canonical order)"
    s = b.fetch_compact()
    h = avhip.compact_header(s)
    nl = a.node_range[1] - a.node_range[0]
    tl = a.target_range[1] - a.target_range[0]
    ref = encode(words, log_base=base, n_rounds=max(rounds_run, 1), node_base=a.node_range[0], n_local=nl,
                 target_base=a.target_range[0], n_targets_local=tl, k=a.k, round_shift=a.round_shift)
    assert h["n_updates"] == words.size and h["log_base"] == base
    assert s.size == ref.size and np.array_equal(s, ref), "compact stream differs from the format restatement"
    assert np.array_equal(avhip.compact_expand(s), words)
    return words


def test_sweep_pairs_byz_three_rounds(oracle):
    """k_round_sweep slot/dense/single records over three pending rounds, vs the oracle."""
    n, m, k = 3000, 2000, 8
    a, b = twin(n, m, k, 9, BYZ20, (avhip.INIT_PAIRS, 0))
    sim = oracle.Sim(n, m, k, seed=9, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=8)
    exp = np.concatenate([sim.run_round(threads=8)[0] for _ in range(3)])
    for e in (a, b):
        e.run_rounds(3)
    words = check_compact(a, b, 3)
    assert np.array_equal(avhip.decode_updates(words, 0), exp)


@pytest.mark.parametrize("cfg", [
    # n, m, k, opts, rounds: k_round_node under the cap (M > 4096); first-generation kernel at k = 16
    # (singles and dense records); a target shard; many index chunks (n > 4096)
    dict(n=600, m=5000, k=8, opts=(), rounds=2),
    dict(n=300, m=700, k=16, opts=(("kernel", 1),), rounds=3),
    dict(n=10_000, m=64, k=8, opts=(), rounds=4),
    dict(n=2000, m=1000, k=8, opts=(), rounds=2, target_range=(256, 800)),
], ids=["capped", "k16_first_gen", "chunks", "target_shard"])
def test_compact_matches_words(cfg):
    kw = {"target_range": cfg["target_range"]} if "target_range" in cfg else {}
    a, b = twin(cfg["n"], cfg["m"], cfg["k"], 21, BYZ20, opts=cfg["opts"], **kw)
    for e in (a, b):
        e.run_rounds(cfg["rounds"])
    w = check_compact(a, b, cfg["rounds"])
    assert w.size > 0


def test_global_cell_tables(oracle):
    """k * BL > 4096 cells (M = 20000 at k = 8: 5000): the per-bucket tables live in global memory."""
    n, m, k = 64, 20_000, 8
    a, b = twin(n, m, k, 5, 0, (avhip.INIT_BERNOULLI, P80))
    sim = oracle.Sim(n, m, k, seed=5, init_mode=avhip.INIT_BERNOULLI, init_param=P80, threads=8)
    exp = np.concatenate([sim.run_round(threads=8)[0] for _ in range(2)])
    for e in (a, b):
        e.run_rounds(2)
    words = check_compact(a, b, 2)
    assert np.array_equal(avhip.decode_updates(words, 0), exp)


def test_replay_fused_rounds():
    """C2-shaped replay (M = 10000, 4-byte codes), several fused rounds in one log."""
    a, b = twin(200, 10_000, 8, 3, 0, (avhip.INIT_BERNOULLI, 0x80000000))
    for e in (a, b):
        e.replay_prepare(6)
        e.replay_rounds(6)
    w = check_compact(a, b, 6)
    assert w.size > 0


def test_multi_pass_encoder(oracle):
    """A log spanning more (round, node) buckets than one encoder pass holds (option enc_buckets):
    several passes, the same words and stream."""
    n, m, k = 1000, 300, 8
    a, b = twin(n, m, k, 11, BYZ20, (avhip.INIT_PAIRS, 0), opts=(("enc_buckets", 2500),))
    sim = oracle.Sim(n, m, k, seed=11, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=8)
    exp = np.concatenate([sim.run_round(threads=8)[0] for _ in range(7)])
    for e in (a, b):
        e.run_rounds(7)
    words = check_compact(a, b, 7)
    assert np.array_equal(avhip.decode_updates(words, 0), exp)


def test_async_pipeline_vs_oracle(oracle):
    """Pipelined delivery: round r + 1 enqueued while round r's stream is copied; every ticket's
    stream expands to the oracle's updates of its round."""
    n, m, k = 5000, 1000, 8
    eng = avhip.Engine(n, m, k=k, seed=17, byz_threshold=BYZ20)
    eng.init_records(avhip.INIT_PAIRS, 0)
    sim = oracle.Sim(n, m, k, seed=17, byz_threshold=BYZ20, init_mode=avhip.INIT_PAIRS, threads=8)
    exp = [sim.run_round(threads=8)[0] for _ in range(6)]
    got = {}
    tickets = []
    for r in range(6):
        eng.run_rounds(1)
        tickets.append((r, eng.fetch_compact_async()))
        if len(tickets) >= 2:  # the previous ticket's copy ran beside this round
            rr, t = tickets[-2]
            got[rr] = eng.fetch_compact_wait(t)
    rr, t = tickets[-1]
    got[rr] = eng.fetch_compact_wait(t)
    for r in range(6):
        s = got[r]
        h = avhip.compact_header(s)
        assert h["log_base"] == r
        assert np.array_equal(avhip.decode_updates(avhip.compact_expand(s), h["log_base"]), exp[r]), r
    with pytest.raises(avhip.AvError):
        eng.fetch_compact_wait(tickets[0][1])  # superseded


def test_full_size_two_level_scan():
    """1M nodes x 64 targets with 17 rounds pending: 17M (round, node) buckets (the device scan
    recurses twice); the fetched words are strictly ascending and fold to the pre-fetch digest."""
    n, m, k = 1_000_000, 64, 8
    eng = avhip.Engine(n, m, k=k, seed=2, log_capacity=1 << 27)
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    eng.run_rounds(17)
    d = eng.updates_digest()
    raw = eng.fetch_updates(decode=False)
    assert raw.size == d[0] and raw.size > 0
    assert np.all(raw[1:] > raw[:-1])
    from oracle import cabi
    assert cabi.update_digest(raw) == d


def test_beyond_2_24_nodes(oracle):
    """N = 2^25 (33.5M nodes x 64 targets, k = 8): the update word's node field widens to 25 bits
    (round shift 53, include/avhip.h). Sampled nodes above 2^24 checked against the oracle's literal
    per-node round on the engine's own snapshot (records and update digest), and the fetched words
    decode to those nodes, in canonical order; the compact stream carries the shift."""
    n, m, k = 1 << 25, 64, 8
    eng = avhip.Engine(n, m, k=k, seed=23, log_capacity=1 << 27)
    assert eng.round_shift == 53
    eng.init_records(avhip.INIT_BERNOULLI, P80)
    byz = oracle.byz_words(23, n, 0)
    valid = np.ones(m, np.uint8)
    S = 1024
    for r, a in enumerate([n - S, (1 << 24) + 12345, 1000]):
        before = eng.read_records(a, a + S)
        pref = eng.read_pref_words()
        exp_digest = np.zeros(3, np.uint64)
        words = before.copy()
        for i in range(S):
            row = np.ascontiguousarray(words[i])
            oracle.node_round_ext(23, n, k, 0, a + i, eng.round, m, pref, byz, valid, row, exp_digest)
            words[i] = row
        eng.run_rounds(1)
        assert eng.updates_digest(a, a + S) == tuple(int(v) for v in exp_digest), r
        assert np.array_equal(eng.read_records(a, a + S), words), r
        if r == 0:
            raw = eng.fetch_updates(decode=False)
            assert np.all(raw[1:] > raw[:-1])
            node = (raw >> np.uint64(28)) & np.uint64((1 << 25) - 1)
            sel = raw[(node >= a) & (node < a + S)]
            rows = avhip.decode_updates(sel, 0, 53)
            assert rows.shape[0] == exp_digest[0] and rows[:, 1].max() >= (1 << 24) and np.all(rows[:, 0] == 0)
            assert oracle.update_digest(sel) == tuple(int(v) for v in exp_digest)
            del raw, node
        else:
            s = eng.fetch_compact()
            h = avhip.compact_header(s)
            assert h["round_shift"] == 53 and h["n_updates"] > 0 and h["log_base"] == eng.round - 1
            w2 = avhip.compact_expand(s)
            assert np.all(w2[1:] > w2[:-1]) and np.all((w2 >> np.uint64(53)) == 0)
            node = (w2 >> np.uint64(28)) & np.uint64((1 << 25) - 1)
            assert oracle.update_digest(w2[(node >= a) & (node < a + S)]) == tuple(int(v) for v in exp_digest)
            del s, w2, node
