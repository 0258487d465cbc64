"""GPU parity tests: the HIP engine (through the C ABI of libavhip.so) against
the CPU oracle on identical seeded inputs, and against the golden vectors
transcribed from the reference's tests. Bit-exact everywhere (integer path)."""
import os

import numpy as np
import pytest

import avhip
from golden_ops import NotFound, run_processor

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)


def rows(u):
    return [tuple(int(v) for v in r) for r in np.asarray(u).tolist()]


def make_pair(oracle, n, m, k, seed=7, peer_mode=0, byz=0, init_mode=3, init_param=P80, log_capacity=0,
              kernel=2, sweep_blocks=None):
    eng = avhip.Engine(n, m, k=k, seed=seed, peer_mode=peer_mode, byz_threshold=byz, log_capacity=log_capacity)
    eng.set_option("kernel", kernel)
    if sweep_blocks is not None:
        eng.set_option("sweep_blocks", sweep_blocks)
    eng.init_records(init_mode, init_param)
    sim = oracle.Sim(n, m, k, seed=seed, peer_mode=peer_mode, byz_threshold=byz, init_mode=init_mode,
                     init_param=init_param)
    return eng, sim


def assert_same_state(eng, sim, where=""):
    got, exp = eng.read_records(), sim.dump()
    if not np.array_equal(got, exp):
        bad = np.argwhere(got != exp)[:5]
        msg = [(int(a), int(b), hex(int(got[a, b])), hex(int(exp[a, b]))) for a, b in bad]
        raise AssertionError(f"state mismatch {where}: {msg}")


# ------------------------------------------------------------------ sampling / init
@pytest.mark.parametrize("n,k,mode", [(1000, 8, 0), (12, 8, 0), (9, 8, 0), (7, 3, 1), (300, 16, 0), (3, 4, 0)])
def test_sample_peers_parity(oracle, n, k, mode):
    eng = avhip.Engine(n, 64, k=k, seed=11, peer_mode=mode)
    for rnd in (0, 1, 17, 1000):
        got = eng.sample_peers(rnd)
        for node in range(n):
            assert got[node].tolist() == oracle.sample_peers(11, node, rnd, n, k, mode).tolist(), (node, rnd)


@pytest.mark.parametrize("mode,param", [(1, 0), (2, 0), (3, P80), (4, 0)])
def test_init_parity(oracle, mode, param):
    eng, sim = make_pair(oracle, 37, 150, 8, byz=BYZ20, init_mode=mode, init_param=param)
    assert_same_state(eng, sim)
    pref, exp = eng.read_pref(), sim.pref()
    honest = [j for j in range(37) if not sim.is_byzantine(j)]
    assert np.array_equal(pref[honest], exp[honest])


# ------------------------------------------------------------------ rounds, sim mode
SIM_CASES = [
    dict(n=12, m=40, k=8, seed=7, init_mode=3),
    dict(n=10, m=33, k=8, seed=9, init_mode=4, byz=BYZ20),
    dict(n=6, m=20, k=3, seed=3, init_mode=2, peer_mode=1),
    dict(n=8, m=70, k=5, seed=4, init_mode=1, byz=int(0.3 * 2**32)),
    dict(n=64, m=200, k=8, seed=0xA7A1A9C4, init_mode=3, byz=BYZ20),
    dict(n=300, m=517, k=8, seed=5, init_mode=4, byz=BYZ20),
    dict(n=40, m=96, k=16, seed=8, init_mode=3),
]


@pytest.mark.parametrize("kernel", [2, 1], ids=["sweep", "per_tile"])
@pytest.mark.parametrize("case", SIM_CASES, ids=lambda c: f"n{c['n']}m{c['m']}k{c['k']}")
def test_sim_rounds_parity(oracle, case, kernel):
    eng, sim = make_pair(oracle, case["n"], case["m"], case["k"], seed=case["seed"],
                         peer_mode=case.get("peer_mode", 0), byz=case.get("byz", 0), init_mode=case["init_mode"],
                         kernel=kernel)
    total_applied = 0
    for r in range(40):
        if r == 5:  # target invalidated mid-run (avalanche_test.go:534 pattern), later revalidated
            eng.set_valid(3, False)
            sim.set_valid(3, False)
        if r == 13:
            eng.set_valid(3, True)
            sim.set_valid(3, True)
        eng.run_rounds(1)
        exp_u, applied = sim.run_round()
        total_applied += applied
        got_u = eng.fetch_updates()
        assert rows(got_u) == rows(exp_u), f"round {r}"
        assert_same_state(eng, sim, f"round {r}")
        assert eng.applied_votes() == total_applied
    assert eng.round == 40


@pytest.mark.parametrize("blocks", [0, 1, 3, 7])
def test_sweep_grid_parity(oracle, blocks):
    """The persistent sweep kernel with a grid smaller than the tile count
    (every wave walks several tiles; counters flushed once per wave) and with
    one wave per tile (0), across the warm-up, the warm steady state and
    finalization (rounds 16-17: the exact per-vote path with deletion)."""
    n, m, k = 700, 333, 8
    eng, sim = make_pair(oracle, n, m, k, seed=17, byz=BYZ20, init_mode=2, sweep_blocks=blocks)
    total = 0
    for r in range(20):
        eng.run_rounds(1)
        exp_u, applied = sim.run_round()
        total += applied
        assert rows(eng.fetch_updates()) == rows(exp_u), f"round {r}"
        assert eng.applied_votes() == total, f"round {r}"
        if r % 4 == 3 or r >= 15:
            assert_same_state(eng, sim, f"round {r}")
    assert eng.finalized_count() > 0


@pytest.mark.parametrize("kernel", [2, 1], ids=["sweep", "per_tile"])
def test_tiny_network_peers_parity(oracle, kernel):
    """N - 1 <= k: every other node is polled (the sampler's degenerate branch)."""
    eng, sim = make_pair(oracle, 5, 90, 8, seed=2, init_mode=3, kernel=kernel)
    for r in range(20):
        eng.run_rounds(1)
        exp_u, _ = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), r
    assert_same_state(eng, sim)


@pytest.mark.parametrize("kernel", [2, 1], ids=["node", "capped_v1"])
def test_sim_capped_parity(oracle, kernel):
    """M > 4096: the workgroup-scan path enforces the 4096 poll cap."""
    eng, sim = make_pair(oracle, 20, 5000, 8, seed=3, byz=BYZ20, init_mode=3, kernel=kernel)
    for r in range(6):
        eng.run_rounds(1)
        exp_u, applied = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), r
        assert_same_state(eng, sim, f"round {r}")
    assert eng.layout_info()["capped"]


# ------------------------------------------------------------------ rounds, replay mode
@pytest.mark.parametrize("n,m,k,kernel", [(9, 300, 8, 2), (9, 300, 8, 1), (70, 1000, 5, 2), (6, 4500, 8, 2),
                                          (6, 4500, 8, 1), (5, 4097, 2, 2), (4, 8300, 8, 2), (3, 20000, 8, 2)])
def test_replay_parity(oracle, n, m, k, kernel):
    eng, sim = make_pair(oracle, n, m, k, seed=21, init_mode=3, kernel=kernel)
    applied_total = 0
    for r in range(12):
        errs = oracle.gen_replay_errs(21, r, 0, n, m, k)
        eng.replay_round_errs(errs)
        exp_u, applied = sim.run_round(errs)
        applied_total += applied
        assert rows(eng.fetch_updates()) == rows(exp_u), r
        assert_same_state(eng, sim, f"round {r}")
    assert eng.applied_votes() == applied_total


def test_device_replay_generator_parity(oracle):
    n, m, k, R = 10, 4300, 8, 6
    eng, sim = make_pair(oracle, n, m, k, seed=0xA7A1A9C4, init_mode=3)
    eng.replay_prepare(R)
    eng.replay_rounds(R)
    exp = []
    for r in range(R):
        u, _ = sim.run_round(oracle.gen_replay_errs(0xA7A1A9C4, r, 0, n, m, k))
        exp += rows(u)
    assert rows(eng.fetch_updates()) == exp
    assert_same_state(eng, sim)


def test_c2_full_size_replay_parity(oracle):
    """configs[1] at full size (1k nodes x 10k targets, k=8, replayed streams,
    4096 poll cap binding): device-generated stream, bit-exact vs the oracle."""
    n, m, k, R, seed = 1000, 10_000, 8, 4, 0xA7A1A9C4
    eng, sim = make_pair(oracle, n, m, k, seed=seed, init_mode=3, init_param=0x80000000, log_capacity=1 << 24)
    eng.replay_prepare(R)
    threads = min(8, __import__("os").cpu_count() or 1)
    applied = 0
    for r in range(R):
        eng.replay_rounds(1)
        exp_u, a = sim.run_round(oracle.gen_replay_errs(seed, r, 0, n, m, k), threads=threads)
        applied += a
        assert np.array_equal(eng.fetch_updates(), exp_u), r
    assert_same_state(eng, sim)
    assert eng.applied_votes() == applied == R * n * k * 4096


# ------------------------------------------------------------------ exhaustive single-vote transitions
def test_exhaustive_transitions_gpu(oracle):
    """Every reachable live record (votes subset of consider: 6561 pairs x count
    0..127 x accepted) receives one vote of each err class; result and emitted
    StatusUpdate must equal the oracle's regsiterVote (vote.go:54-91)."""
    v = np.arange(256, dtype=np.uint32)
    vv, cc = np.meshgrid(v, v, indexing="ij")
    ok = (vv & ~cc) == 0
    vc = (vv[ok] | (cc[ok] << 8)).astype(np.uint32)  # 6561 nodes
    t = np.arange(256, dtype=np.uint32)  # target t: count t>>1, accepted t&1
    words = vc[:, None] | (((t >> 1) << 1 | (t & 1)) << 16)[None, :]
    n, m = words.shape
    for err in [0, 1, 2, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF]:
        eng = avhip.Engine(n, m, k=1, seed=1)
        eng.init_records(avhip.INIT_REJECTED, 0)
        eng.write_records(words)
        assert np.array_equal(eng.read_records(), words)
        eng.replay_round_errs(np.full((n, 1, m), err, np.uint32))
        exp_w, changed, status = oracle.transition_batch(words.ravel(), np.full(words.size, err, np.uint32))
        exp_w = exp_w.reshape(n, m)
        fin = (exp_w >> 17) >= 128
        exp_dump = np.where(fin, avhip.ABSENT_WORD | (((exp_w >> 16) & 1) << 16), exp_w).astype(np.uint32)
        assert np.array_equal(eng.read_records(), exp_dump), hex(err)
        idx = np.flatnonzero(changed)
        exp_u = [(0, int(i // m), 0, int(i % m), int(status[i])) for i in idx]
        assert rows(eng.fetch_updates()) == exp_u, hex(err)
        eng.close()


# ------------------------------------------------------------------ golden vectors through the C ABI
class EngineProc:
    def __init__(self, fx):
        self.accepted = {int(h): v["accepted"] for h, v in fx["targets"].items()}
        self.eng = avhip.Engine(2, max(self.accepted) + 1, k=1)

    def add(self, h):
        return bool(self.eng.add_targets(0, [h], [self.accepted[h]])[0])

    def register(self, node, votes):
        st = self.eng.register_votes(0, [h for _, h in votes], [e for e, _ in votes])
        return [(h, int(s)) for (_, h), s in zip(votes, st) if s >= 0]

    def is_accepted(self, h):
        return self.eng.is_accepted(0, h)

    def confidence(self, h):
        try:
            return self.eng.get_confidence(0, h)
        except avhip.VoteRecordNotFound:
            raise NotFound()

    def invs(self):
        return self.eng.get_invs(0).tolist()

    def get_round(self):
        return self.eng.get_round(0)

    def inc_round(self):
        self.eng.set_round(0, self.eng.get_round(0) + 1)


@pytest.mark.parametrize("which", [0, 1])
def test_processor_golden_gpu(golden, which):
    fx = golden["processor"][which]
    run_processor(fx, EngineProc(fx))


def test_vote_record_golden_gpu(golden):
    """TestVoteRecord (avalanche_test.go:13-91) through the engine. The bare
    VoteRecord keeps voting after finalization; a Processor deletes it
    (processor.go:114-116), so the engine runs the live stretches: up to the
    first finalization, then from the flip at :70 (state rebuilt from the vote
    history and the golden values) to the final finalization at :91."""
    fx = golden["vote_record"]
    steps = fx["steps"]
    eng = avhip.Engine(2, 1, k=1)
    assert eng.add_targets(0, [0], [fx["start_accepted"]])[0]
    votes = cons = 0
    resumed = False
    for i, st in enumerate(steps):
        err = st["err"]
        votes = ((votes << 1) & 0xFF) | (err == 0)
        cons = ((cons << 1) & 0xFF) | (err < 0x80000000)
        exp = (st["accepted"], st["finalized"], st["confidence"])
        dead = (int(eng.read_records()[0, 0]) >> 17) >= 128
        if dead:
            if st["finalized"]:
                continue  # bare record past finalization: no Processor equivalent
            # flip back to live (line 70): rebuild the bare record and resume
            eng.write_records(np.array([[votes | (cons << 8) | ((st["confidence"] << 1 | st["accepted"]) << 16)]],
                                       np.uint32))
            resumed = True
            continue
        eng.register_votes(0, [0], [err])
        w = int(eng.read_records()[0, 0])
        if (w >> 17) >= 128:
            got = (bool((w >> 16) & 1), True, 128)
        else:
            got = (bool((w >> 16) & 1), False, w >> 17)
        assert got == exp, f"step {i} (line {st['line']}): {got} != {exp}"
    assert resumed and (int(eng.read_records()[0, 0]) >> 17) >= 128


# ------------------------------------------------------------------ sharding identities
def test_target_shard_identity():
    """Two target-sharded engines == one engine, bit for bit (the multi-GPU
    target-sharding path, exercised on one device)."""
    n, m, k, R = 500, 1000, 8, 30
    full = avhip.Engine(n, m, k=k, seed=3, byz_threshold=BYZ20)
    full.init_records(avhip.INIT_PAIRS, 0)
    parts = [avhip.Engine(n, m, k=k, seed=3, byz_threshold=BYZ20, target_range=r) for r in [(0, 512), (512, 1000)]]
    for p in parts:
        p.init_records(avhip.INIT_PAIRS, 0)
    for r in range(R):
        full.run_rounds(1)
        for p in parts:
            p.run_rounds(1)
        u = np.concatenate([p.fetch_updates() for p in parts])
        u = u[np.lexsort((u[:, 3], u[:, 2], u[:, 1], u[:, 0]))]
        assert np.array_equal(full.fetch_updates(), u), r
    merged = np.concatenate([p.read_records() for p in parts], axis=1)
    assert np.array_equal(full.read_records(), merged)
    assert full.applied_votes() == sum(p.applied_votes() for p in parts)


def test_node_shard_needs_comm():
    e = avhip.Engine(10, 64, node_range=(0, 5))
    with pytest.raises(avhip.AvError):
        e.run_rounds(1)


# ------------------------------------------------------------------ full-size properties
def dense_words(k):  # kernels.h dense_words: u64 words of a dense lane record
    return (k + 5) // 2


MED_MAX = 6  # kernels.h kMedMax (folded medium records, AVK_MED_S4 = 0 builds only)


def emitted_bytes(u, k=8, med=False):
    """Log bytes the round kernels write for decoded updates `u`, per (round,
    node, 32-target block) with c updates. med=False (first-generation
    kernels): c >= dense_words(k) is one dense record of dense_words(k) u64
    words, else c single 8-B words. med=True (the k = 8 sweep,
    round_common.h emit_store_med, slot records): 1 update a single word;
    >= 2 updates in at most 4 slots (3 when one of them deletes its record:
    status Finalized / Invalid) one 32-B slot record; otherwise a dense record."""
    if len(u) == 0:
        return 0
    key = np.stack([u[:, 0], u[:, 1], u[:, 3] // 32], axis=1)
    _, inv, counts = np.unique(key, axis=0, return_inverse=True, return_counts=True)
    inv = inv.reshape(-1)
    dw = dense_words(k)
    if med:
        g = len(counts)
        _, first = np.unique(np.stack([inv, u[:, 2]], axis=1), axis=0, return_index=True)
        ns = np.bincount(inv[first], minlength=g)  # slots with updates per block
        died = np.bincount(inv, weights=np.isin(u[:, 4], [avhip.STATUS_FINALIZED, avhip.STATUS_INVALID]),
                           minlength=g) > 0
        slot_rec = (ns <= 3) | ((ns == 4) & ~died)
        return int(np.where(counts == 1, 8, np.where(slot_rec, 32, 8 * dw)).sum())
    return int(np.where(counts >= dw, 8 * dw, 8 * counts).sum())


def test_c4_shape_properties():
    """C4 shape at 1/10 scale (100k nodes x 1000 targets, k=8, Bernoulli(0.8)):
    rounds 0-15 keep every record live (finalization needs >= 134 votes), so
    applied votes == N*M*k per round; both round kernels give identical
    results; the published preference equals the records' accepted bit."""
    n, m, k = 100_000, 1000, 8
    digests = []
    # round 0: kernel 1 reads and writes all 25 planes (236 B per 32-record
    # lane); the sweep's fresh round reads only A and leaves the vote planes
    # and consider planes virtual (236 - 96 - 32 - 32 = 76 B). Warm bytes per lane over rounds 1-15:
    # kernel 1 176 each; the sweep's depend on which tiles settled
    # (test_gpu_virtual_votes.py, test_gpu_count_lazy.py check them exactly)
    for kernel, cold_bytes, warm_bytes in ((1, 236, 15 * 176), (2, 76, None)):
        e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4)
        e.set_option("kernel", kernel)
        e.set_option("count_lazy", 0)  # per-lane bytes with stored count planes (test_gpu_count_lazy.py)
        e.set_option("k_hi_virtual", 0)  # (the virtual K4..K7 group's bytes: test_gpu_count_lazy.py)
        e.init_records(avhip.INIT_BERNOULLI, P80)
        lanes = e.layout_info()["lanes"]
        e.run_rounds(1)  # round 0: consider planes fill up
        b1 = e.alg_bytes()
        e.run_rounds(15)  # warm: the all-ones consider planes are skipped
        b16 = e.alg_bytes()
        assert e.applied_votes() == n * m * k * 16
        u = e.fetch_updates()
        r0 = u[:, 0] == 0
        med = kernel == 2  # the sweep logs medium records (emit_updates_med)
        assert b1 == lanes * cold_bytes + emitted_bytes(u[r0], med=med)
        if warm_bytes is not None:
            assert b16 - b1 == lanes * warm_bytes + emitted_bytes(u[~r0], med=med)
        else:
            # (80 B: a settled tile whose input snapshot is uniform takes the reference word as its
            # votes, option uni_votes; 136 B: a stale tile regathers 7 words)
            assert lanes * 15 * 80 <= b16 - b1 - emitted_bytes(u[~r0], med=med) <= lanes * 15 * 136
        assert not np.isin(u[:, 4], [avhip.STATUS_FINALIZED, avhip.STATUS_INVALID]).any()
        recs = e.read_records(0, n, 0, m)
        assert ((recs >> 17) < 128).all()
        pref = e.read_pref(0, n, 0, m)
        assert np.array_equal(pref, ((recs >> 16) & 1).astype(np.uint8))
        digests.append((hash(recs.tobytes()), hash(u.tobytes())))
        e.close()
    assert digests[0] == digests[1]


def test_run_to_finalization_properties(oracle):
    """Honest network, all accepted: every record finalizes Finalized exactly
    once, at vote 134 (round 16 at k=8), and then the engine goes quiet."""
    n, m, k = 2000, 300, 8
    e = avhip.Engine(n, m, k=k, seed=5)
    e.init_records(avhip.INIT_ACCEPTED, 0)
    e.run_rounds(20)
    u = e.fetch_updates()
    assert len(u) == n * m
    assert (u[:, 4] == avhip.STATUS_FINALIZED).all()
    assert (u[:, 0] == 16).all() and (u[:, 2] == 5).all()  # 16*8 + 6 = 134th vote
    assert e.applied_votes() == n * m * 134
    assert (e.read_records() == (avhip.ABSENT_WORD | 1 << 16)).all()


def test_update_log_overflow_reported(oracle):
    """A device StatusUpdate log too small for a round: the round's state stays
    exact, the overflow is reported (av_update_log_overflowed, then
    AV_ERR_OVERFLOW from fetch), and the log works again after the fetch."""
    n, m, k = 300, 517, 8
    eng, sim = make_pair(oracle, n, m, k, seed=5, byz=BYZ20, init_mode=4, log_capacity=64)
    eng.run_rounds(3)
    for _ in range(3):
        sim.run_round()
    assert eng.log_overflowed()
    with pytest.raises(avhip.LogOverflow):
        eng.fetch_updates()
    assert not eng.log_overflowed()
    assert_same_state(eng, sim, "after overflow")


@pytest.mark.parametrize("kernel", [2, 1], ids=["node", "capped_v1"])
def test_capped_finalization_parity(oracle, kernel):
    """M > 4096 with more live records than the cap, run through finalization:
    records deleted at count 128 make room for the next ones inside a round
    (the per-vote poll-set re-selection path)."""
    n, m, k = 12, 4500, 8
    eng, sim = make_pair(oracle, n, m, k, seed=13, init_mode=2, kernel=kernel)
    for r in range(22):
        eng.run_rounds(1)
        exp_u, applied = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), r
        if r >= 15:
            assert_same_state(eng, sim, f"round {r}")
    assert eng.finalized_count() > 0


def _oracle_poll_sets(sim, valid, t0=0):
    dump = sim.dump()
    live = (dump >> 17) < 128
    sets = []
    for row in live & valid[None, :]:
        sets.append((np.flatnonzero(row)[:avhip.MAX_ELEMENT_POLL] + t0).tolist())
    return sets


@pytest.mark.parametrize("n,m", [(40, 700), (9, 5000)])
def test_poll_sets_batch_parity(oracle, n, m):
    """av_get_invs_batch (GetInvsForNextPoll of every node, processor.go:144-170,
    device compaction) == the oracle's live valid records in target order, capped
    at 4096, == per-node av_get_invs; through finalization and invalid targets."""
    eng, sim = make_pair(oracle, n, m, 8, seed=23, byz=BYZ20, init_mode=2)
    valid = np.ones(m, bool)
    for r in range(19):
        if r == 3:
            for t in (0, 5, m - 1):
                eng.set_valid(t, False)
                sim.set_valid(t, False)
                valid[t] = False
        eng.run_rounds(1)
        sim.run_round()
        if r in (0, 15, 16, 18):
            offs, tg = eng.get_invs_batch()
            got = [tg[offs[i]:offs[i + 1]].tolist() for i in range(n)]
            assert got == _oracle_poll_sets(sim, valid), r
            for node in (0, n // 2, n - 1):
                assert eng.get_invs(node).tolist() == got[node]
            offs2, tg2 = eng.get_invs_batch(2, 5)
            assert [tg2[offs2[i]:offs2[i + 1]].tolist() for i in range(3)] == got[2:5]
    eng.fetch_updates()


def test_target_shard_identity_8way():
    """Eight target shards (BL = 4 per shard: the 8-GPU C4 decomposition) ==
    one engine, bit for bit, through finalization and deletion (rounds 16-19)."""
    n, m, k, R = 3000, 1000, 8, 20
    full = avhip.Engine(n, m, k=k, seed=31, byz_threshold=BYZ20, log_capacity=1 << 23)
    full.init_records(avhip.INIT_ACCEPTED, 0)
    from avhip import sharding
    parts = [avhip.Engine(n, m, k=k, seed=31, byz_threshold=BYZ20, target_range=sharding.target_shard(m, 8, r),
                          log_capacity=1 << 22) for r in range(8)]
    for p in parts:
        p.init_records(avhip.INIT_ACCEPTED, 0)
    for r in range(R):
        full.run_rounds(1)
        for p in parts:
            p.run_rounds(1)
        u = np.concatenate([p.fetch_updates() for p in parts])
        u = u[np.lexsort((u[:, 3], u[:, 2], u[:, 1], u[:, 0]))]
        assert np.array_equal(full.fetch_updates(), u), r
    merged = np.concatenate([p.read_records() for p in parts], axis=1)
    assert np.array_equal(full.read_records(), merged)
    assert full.applied_votes() == sum(p.applied_votes() for p in parts)
    assert full.finalized_count() == sum(p.finalized_count() for p in parts) > 0


@pytest.mark.parametrize("g,tpw,tile_draw", [(2, 16, 1), (4, 8, 1), (8, 4, 1), (4, 16, 1), (8, 16, 1), (8, 16, 0),
                                              (2, 16, 0)])
def test_target_shard_runs(g, tpw, tile_draw):
    """G target shards of a C4-shaped network (BL = 16 / 8 / 4 lanes per node)
    with runs of tpw tiles per wave (a run of 64 * tpw / BL nodes: past 32 the
    run's draw falls back to per-tile draws, shared by 2 producer lanes per node
    with option tile_draw, else one draw per lane) == one engine, bit for bit,
    through the settled rounds and finalization."""
    n, m, k, R = 20_000, 1000, 8, 20
    full = avhip.Engine(n, m, k=k, seed=77, log_capacity=1 << 24)
    full.init_records(avhip.INIT_BERNOULLI, P80)
    from avhip import sharding
    parts = []
    for r in range(g):
        p = avhip.Engine(n, m, k=k, seed=77, target_range=sharding.target_shard(m, g, r), log_capacity=1 << 23)
        p.set_option("tiles_per_wave", tpw)
        p.set_option("tile_draw", tile_draw)
        p.init_records(avhip.INIT_BERNOULLI, P80)
        parts.append(p)
    for r in range(R):
        full.run_rounds(1)
        for p in parts:
            p.run_rounds(1)
        u = np.concatenate([p.fetch_updates() for p in parts])
        u = u[np.lexsort((u[:, 3], u[:, 2], u[:, 1], u[:, 0]))]
        assert np.array_equal(full.fetch_updates(), u), r
    merged = np.concatenate([p.read_records() for p in parts], axis=1)
    assert np.array_equal(full.read_records(), merged)
    assert full.applied_votes() == sum(p.applied_votes() for p in parts)
    assert full.finalized_count() == sum(p.finalized_count() for p in parts) > 0
    for p in parts + [full]:
        p.close()


def test_cross_kernel_full_c4():
    """configs C4 at full size (1M nodes x 1000 targets, k=8, Bernoulli(0.8)):
    the sweep kernel and the first-generation per-tile kernel agree on every
    round's StatusUpdate count and on the records and published preferences of
    sampled nodes, rounds 0-15; round 15's update streams agree exactly."""
    n, m, k, R = 1_000_000, 1000, 8, 16
    engs = []
    for kernel in (2, 1):
        e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, log_capacity=1 << 26)
        e.set_option("kernel", kernel)
        e.init_records(avhip.INIT_BERNOULLI, P80)
        engs.append(e)
    rng = np.random.default_rng(0)
    sample = np.unique(np.concatenate([[0, 1, n - 1], rng.integers(0, n, 64)]))
    for r in range(R):
        for e in engs:
            e.run_rounds(1)
        counts = [e.updates_count() for e in engs]
        assert counts[0] == counts[1], (r, counts)
        if r == R - 1:
            a, b = (e.fetch_updates() for e in engs)
            assert np.array_equal(a, b)
        else:
            for e in engs:
                e.discard_updates()
        if r % 5 == 0 or r == R - 1:
            for node in sample[:8]:
                ra, rb = (e.read_records(int(node), int(node) + 1, 0, m) for e in engs)
                assert np.array_equal(ra, rb), (r, int(node))
    for node in sample:
        ra, rb = (e.read_records(int(node), int(node) + 1, 0, m) for e in engs)
        assert np.array_equal(ra, rb), int(node)
        pa, pb = (e.read_pref(int(node), int(node) + 1, 0, m) for e in engs)
        assert np.array_equal(pa, pb), int(node)
    assert engs[0].applied_votes() == engs[1].applied_votes() == n * m * k * R
    for e in engs:
        e.close()


def test_sweep_parity_c3_shape(oracle):
    """The C3 shape (double-spend pairs, 20 % Byzantine flip-flop voters) at
    2000 nodes x 2000 targets, 30 rounds: sweep kernel vs oracle, bit-exact."""
    n, m, k = 2000, 2000, 8
    eng, sim = make_pair(oracle, n, m, k, seed=0xA7A1A9C4, byz=BYZ20, init_mode=4, log_capacity=1 << 24)
    threads = min(8, os.cpu_count() or 1)
    total = 0
    for r in range(30):
        eng.run_rounds(1)
        exp_u, applied = sim.run_round(threads=threads)
        total += applied
        assert np.array_equal(eng.fetch_updates(), exp_u), r
    assert_same_state(eng, sim)
    assert eng.applied_votes() == total


@pytest.mark.parametrize("seed", range(40))
def test_random_config_fuzz(oracle, seed):
    """Randomized network shapes through the round kernels vs the oracle:
    N, M (BL from 1 to > 64 per node, tiles straddling nodes, M > 4096 with
    the cap), k in 1..10, init modes, Byzantine share, peer mode, target
    validity flips, both kernel generations and both sweep grids."""
    rng = np.random.default_rng(1000 + seed)
    n = int(rng.integers(3, 400))
    m = int(rng.choice([int(rng.integers(1, 40)), int(rng.integers(40, 2100)), int(rng.integers(4097, 6000))]))
    if m > 4096:
        n = min(n, 40)
    k = int(rng.integers(1, 11))
    init_mode = int(rng.integers(1, 5))
    byz = int(rng.choice([0, int(0.2 * 2**32), int(0.45 * 2**32)]))
    peer_mode = int(rng.random() < 0.15)
    kernel = int(rng.choice([1, 2]))
    blocks = int(rng.choice([-1, 0, -2]))
    eng, sim = make_pair(oracle, n, m, k, seed=int(rng.integers(1, 2**31)), peer_mode=peer_mode, byz=byz,
                         init_mode=init_mode, init_param=int(rng.integers(0, 2**32)), log_capacity=1 << 22,
                         kernel=kernel)
    if kernel == 2 and blocks != -1:
        eng.set_option("sweep_blocks", blocks)
    rounds = int(rng.integers(5, 40))
    for r in range(rounds):
        if rng.random() < 0.1:
            t = int(rng.integers(0, m))
            v = bool(rng.integers(0, 2))
            eng.set_valid(t, v)
            sim.set_valid(t, v)
        eng.run_rounds(1)
        exp_u, _ = sim.run_round()
        assert rows(eng.fetch_updates()) == rows(exp_u), (r, n, m, k)
    assert_same_state(eng, sim, f"n={n} m={m} k={k} kernel={kernel} blocks={blocks}")
