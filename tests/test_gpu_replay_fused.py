"""Fused replay rounds (k_replay_node, round_node.hip): a capped engine (M >
4096, the poll cap of processor.go:165-167 binds) applies up to `replay_fuse`
consecutive replay rounds in one launch and hands nodes that reach count 120
to the per-round exact pass. Checked bit for bit against the oracle (every
StatusUpdate of every round, the records, the applied votes) and against the
same engine with fusion off, including the hand-off to the exact pass,
polled lanes past the first 4096 targets, Byzantine publishing and k < 8."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)


@pytest.fixture(params=[1, 0], ids=["fast", "nofast"], autouse=True)
def replay_fast(request, monkeypatch):
    """Every test runs with k_replay_fast (nodes whose poll set is their first
    128 lanes, round_node.hip) on and off (option replay_fast)."""
    orig = avhip.Engine.__init__

    def init(self, *a, **kw):
        orig(self, *a, **kw)
        self.set_option("replay_fast", request.param)

    monkeypatch.setattr(avhip.Engine, "__init__", init)
    return request.param


def rows(u):
    return [tuple(int(v) for v in r) for r in np.asarray(u).tolist()]


def pair(oracle, n, m, k, seed, byz=0, init_mode=avhip.INIT_BERNOULLI, fuse=16):
    eng = avhip.Engine(n, m, k=k, seed=seed, byz_threshold=byz)
    eng.set_option("replay_fuse", fuse)
    eng.init_records(init_mode, P80)
    sim = oracle.Sim(n, m, k, seed=seed, byz_threshold=byz, init_mode=init_mode, init_param=P80)
    assert eng.layout_info()["capped"]
    return eng, sim


def run_oracle(oracle, sim, seed, r0, R, n, m, k):
    exp, applied = [], 0
    for r in range(r0, r0 + R):
        u, a = sim.run_round(oracle.gen_replay_errs(seed, r, 0, n, m, k))
        exp += rows(u)
        applied += a
    return exp, applied


def push_counts(eng, sim, nodes, targets, votes):
    """`votes` drop-in Responses of all-yes votes on `targets` for every node
    (processor.go:92-117): accepted records climb towards count 120."""
    nd, off, tg = [], [0], []
    for _ in range(votes):
        for node in nodes:
            nd.append(node)
            tg.extend(targets)
            off.append(len(tg))
    eng.register_votes_batch(nd, off, tg, np.zeros(len(tg), np.uint32))
    for node_, a, b in zip(nd, off[:-1], off[1:]):
        sim.register_votes(node_, tg[a:b], np.zeros(b - a, np.uint32))


@pytest.mark.parametrize("chunks", [[20], [3, 1, 7, 9]], ids=["one_call", "ragged_calls"])
def test_fused_replay_handoff_to_exact_pass(oracle, chunks):
    """Records pushed to count ~110-119 finalize during a fused batch: the
    node leaves the fused kernel at that round and the exact pass (deletion at
    128, the next target moving into the 4096 poll set) runs the rest."""
    n, m, k, seed = 8, 4500, 8, 31
    eng, sim = pair(oracle, n, m, k, seed, init_mode=avhip.INIT_ACCEPTED)
    push_counts(eng, sim, nodes=[0, 3, 5], targets=list(range(0, 96)) + [4090, 4095], votes=118)
    push_counts(eng, sim, nodes=[1], targets=list(range(200, 232)), votes=126)
    eng.discard_updates()  # the drop-in votes' updates (the oracle returned its own)
    sim_r0 = 0
    eng.replay_prepare(sum(chunks))
    exp_all, got_all, applied = [], [], 0
    for c in chunks:
        eng.replay_rounds(c)
        exp, a = run_oracle(oracle, sim, seed, sim_r0, c, n, m, k)
        sim_r0 += c
        applied += a
        exp_all += exp
        got_all += rows(eng.fetch_updates())
    assert got_all == exp_all
    assert eng.finalized_count() > 0
    np.testing.assert_array_equal(eng.read_records(), sim.dump())


def test_fused_replay_light_lanes_polled(oracle):
    """Invalid targets below 4096 push the poll set past block 128: lanes the
    fused kernel loads light get polled (heavy light waves) across a batch."""
    n, m, k, seed = 6, 5200, 8, 41
    eng, sim = pair(oracle, n, m, k, seed)
    for t in list(range(5, 300, 3)) + list(range(4000, 4100)):
        eng.set_valid(t, False)
        sim.set_valid(t, False)
    eng.replay_prepare(12)
    eng.replay_rounds(12)
    exp, applied = run_oracle(oracle, sim, seed, 0, 12, n, m, k)
    assert rows(eng.fetch_updates()) == exp
    np.testing.assert_array_equal(eng.read_records(), sim.dump())
    assert eng.applied_votes() == applied


@pytest.mark.parametrize("k", [1, 3, 5, 8])
def test_fused_replay_k(oracle, k):
    n, m, seed = 7, 4400, 50 + k
    eng, sim = pair(oracle, n, m, k, seed, byz=BYZ20)
    eng.replay_prepare(9)
    eng.replay_rounds(9)
    exp, applied = run_oracle(oracle, sim, seed, 0, 9, n, m, k)
    assert rows(eng.fetch_updates()) == exp
    np.testing.assert_array_equal(eng.read_records(), sim.dump())
    assert eng.applied_votes() == applied


def test_fused_matches_unfused_c2_shape(oracle):
    """C2's shape (BL = 313, 5 waves per node) with 20 % Byzantine nodes:
    fused batches of 16 + 4 rounds and one launch per round give the same
    StatusUpdates, records, applied votes and published preferences (all
    three snapshot buffers are exercised by the following sim round)."""
    n, m, k, seed, R = 300, 10_000, 8, 77, 20
    out = []
    for fuse in (16, 0):
        eng = avhip.Engine(n, m, k=k, seed=seed, byz_threshold=BYZ20, log_capacity=1 << 22)
        eng.set_option("replay_fuse", fuse)
        eng.init_records(avhip.INIT_BERNOULLI, P80)
        eng.replay_prepare(R)
        eng.replay_rounds(R)
        u = eng.fetch_updates()
        pref = eng.read_pref()
        eng.run_rounds(1)  # a sim round reads the snapshot the replay batch left current
        u2 = eng.fetch_updates()
        out.append((u, eng.read_records(), eng.applied_votes(), pref, u2, eng.read_pref()))
        eng.close()
    (a, b) = out
    assert np.array_equal(a[0], b[0])
    assert np.array_equal(a[1], b[1])
    assert a[2] == b[2]
    assert np.array_equal(a[3], b[3])
    assert np.array_equal(a[4], b[4])
    assert np.array_equal(a[5], b[5])


def test_fused_replay_c2_full_size_digest(oracle):
    """configs[1] at full size through one fused batch of 16 rounds (the bench's
    epoch length): per-run multiset digest of every StatusUpdate and the final
    records equal the oracle's."""
    n, m, k, R, seed = 1000, 10_000, 8, 16, 0xA7A1A9C4
    eng, sim = pair(oracle, n, m, k, seed)
    eng.replay_prepare(R)
    eng.replay_rounds(R)
    threads = min(8, __import__("os").cpu_count() or 1)
    cnt = s = x = 0
    for r in range(R):
        (c, s_, x_), _ = sim.run_round(oracle.gen_replay_errs(seed, r, 0, n, m, k), threads=threads,
                                       collect=False, round_rel=r)
        cnt += c
        s = (s + s_) & (2**64 - 1)
        x ^= x_
    assert eng.updates_digest() == (cnt, s, x)
    np.testing.assert_array_equal(eng.read_records(), sim.dump(threads=threads))
    assert eng.applied_votes() == R * n * k * 4096
