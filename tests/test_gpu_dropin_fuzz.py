"""Randomised op sequences on the one-node Processor surface (drop-in path) and
interleaved batched rounds, engine vs oracle, bit-exact after every op.

Covers what the reference's RegisterVotes loop does with messy input
(processor.go:92-117): duplicate hashes inside one Response (applied in order),
unknown hashes (skipped), invalid targets (skipped), votes on records deleted
earlier in the same Response, re-adding after finalization (:45-58)."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

ERRS = np.array([0, 0, 0, 0, 1, 2, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF], np.uint32)


def check(eng, sim, where):
    got, exp = eng.read_records(), sim.dump()
    assert np.array_equal(got, exp), where


@pytest.mark.parametrize("seed,k", [(1, 4), (2, 4), (3, 4), (4, 8), (5, 8)])
def test_dropin_fuzz(oracle, seed, k):
    rng = np.random.default_rng(seed)
    n, m = 5, 150
    eng = avhip.Engine(n, m, k=k, seed=seed)  # no records (AV_INIT_NONE)
    sim = oracle.Sim(n, m, k, seed=seed, init_mode=0)
    valid = np.ones(m, bool)
    for step in range(400):
        op = rng.integers(0, 10)
        node = int(rng.integers(0, n))
        if op < 2:  # AddTargetToReconcile, list with duplicates
            ts = rng.integers(0, m, size=int(rng.integers(1, 20)))
            acc = rng.integers(0, 2, size=ts.size)
            got = eng.add_targets(node, ts, acc)
            exp = [sim.add(node, int(t), int(a)) for t, a in zip(ts, acc)]
            assert got.tolist() == exp, (step, "add")
        elif op < 8:  # RegisterVotes, long Responses with duplicates and unknown hashes
            size = int(rng.integers(1, 600))
            ts = rng.integers(-5, m + 5, size=size)
            ts[rng.random(size) < 0.3] = int(rng.integers(0, m))  # hammer one record
            errs = rng.choice(ERRS, size)
            st = eng.register_votes(node, ts, errs)
            known = (ts >= 0) & (ts < m)
            exp = sim.register_votes(node, ts[known], errs[known])
            got = [(int(t), int(s)) for t, s in zip(ts, st) if s >= 0]
            assert got == exp, (step, "register")
        elif op == 8:  # Target.IsValid flips
            t = int(rng.integers(0, m))
            v = bool(rng.integers(0, 2))
            eng.set_valid(t, v)
            sim.set_valid(t, v)
            valid[t] = v
        else:  # a batched round in between (published preferences must be consistent)
            eng.run_rounds(1)
            exp_u, _ = sim.run_round()
            got_u = eng.fetch_updates()
            assert np.array_equal(got_u, exp_u), (step, "round")
        check(eng, sim, step)
        if step % 50 == 0:
            for t in range(0, m, 7):
                w = int(sim.dump()[node, t])
                live = (w >> 17) < 128
                assert eng.is_accepted(node, t) == (live and bool((w >> 16) & 1))
                if live:
                    assert eng.get_confidence(node, t) == w >> 17
                else:
                    with pytest.raises(avhip.VoteRecordNotFound):
                        eng.get_confidence(node, t)
            dump = sim.dump()[node]
            exp_invs = [t for t in range(m) if (int(dump[t]) >> 17) < 128 and valid[t]][:4096]
            assert eng.get_invs(node).tolist() == exp_invs, (step, "invs")


def test_node_sharded_rccl_world1(oracle):
    """The node-sharded RCCL path (av_comm_init + in-place ncclAllGather every
    round) with a single rank equals the plain engine bit for bit."""
    n, m, k, R = 64, 200, 8, 20
    plain = avhip.Engine(n, m, k=k, seed=9, byz_threshold=int(0.2 * 2**32))
    comm = avhip.Engine(n, m, k=k, seed=9, byz_threshold=int(0.2 * 2**32), node_range=(0, n))
    for e in (plain, comm):
        e.init_records(avhip.INIT_PAIRS, 0)
    comm.comm_init(1, 0, avhip.comm_unique_id())
    plain.run_rounds(R)
    comm.run_rounds(R)
    assert np.array_equal(plain.read_records(), comm.read_records())
    assert np.array_equal(plain.fetch_updates(), comm.fetch_updates())


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_register_votes_batch_vs_oracle(oracle, seed):
    """av_register_votes_batch: many Responses of many nodes in one call (a
    node may appear several times; its Responses apply in order), with
    duplicates, unknown hashes, invalid targets, neutral votes and records
    finalizing inside the batch == the oracle's RegisterVotes per Response."""
    rng = np.random.default_rng(seed)
    n, m = 40, 300
    eng = avhip.Engine(n, m, k=8, seed=seed)
    eng.init_records(avhip.INIT_BERNOULLI, int(0.6 * 2**32))
    sim = oracle.Sim(n, m, 8, seed=seed, init_mode=3, init_param=int(0.6 * 2**32))
    for t in (7, 100):
        eng.set_valid(t, False)
        sim.set_valid(t, False)
    # push records close to 128 so that batches finalize some of them
    for _ in range(16):
        eng.run_rounds(1)
        sim.run_round()
    eng.discard_updates()
    for batch in range(12):
        n_resp = int(rng.integers(1, 60))
        nodes = rng.integers(0, n, size=n_resp)
        sizes = rng.integers(0, 200, size=n_resp)
        offsets = np.concatenate([[0], np.cumsum(sizes)])
        targets = rng.integers(-3, m + 3, size=int(offsets[-1]))
        errs = rng.choice(ERRS, size=targets.size)
        got = eng.register_votes_batch(nodes, offsets, targets, errs)
        for i in range(n_resp):
            a, b = int(offsets[i]), int(offsets[i + 1])
            exp = sim.register_votes(int(nodes[i]), targets[a:b], errs[a:b])
            have = [(int(targets[v]), int(got[v])) for v in range(a, b) if got[v] >= 0]
            assert have == exp, (batch, i)
        check(eng, sim, f"batch {batch}")


def test_register_votes_batch_device_grouping(oracle):
    """Batches of >= 65536 votes are grouped by lane on the device (radix sort
    of (lane, position) + run-length encode, log_ops.hip launch_group_votes):
    the same statuses and records as the oracle's RegisterVotes per Response,
    with nodes repeated across the batch (their Responses apply in order)."""
    rng = np.random.default_rng(77)
    n, m = 300, 700
    eng = avhip.Engine(n, m, k=8, seed=77)
    eng.init_records(avhip.INIT_BERNOULLI, int(0.6 * 2**32))
    sim = oracle.Sim(n, m, 8, seed=77, init_mode=3, init_param=int(0.6 * 2**32))
    eng.set_valid(11, False)
    sim.set_valid(11, False)
    for _ in range(14):
        eng.run_rounds(1)
        sim.run_round()
    eng.discard_updates()
    for batch in range(2):
        n_resp = 900
        nodes = rng.integers(0, n, size=n_resp)
        sizes = rng.integers(0, 200, size=n_resp)
        offsets = np.concatenate([[0], np.cumsum(sizes)])
        assert offsets[-1] >= 1 << 16
        targets = rng.integers(-3, m + 3, size=int(offsets[-1]))
        errs = rng.choice(ERRS, size=targets.size)
        got = eng.register_votes_batch(nodes, offsets, targets, errs)
        for i in range(n_resp):
            a, b = int(offsets[i]), int(offsets[i + 1])
            exp = sim.register_votes(int(nodes[i]), targets[a:b], errs[a:b])
            have = [(int(targets[v]), int(got[v])) for v in range(a, b) if got[v] >= 0]
            assert have == exp, (batch, i)
        check(eng, sim, f"device batch {batch}")
        eng.run_rounds(1)
        exp_u, _ = sim.run_round()
        assert np.array_equal(eng.fetch_updates(), exp_u)


@pytest.mark.parametrize("seed,n_resp,unsorted", [(5, 200, False), (6, 290, False), (7, 250, True)],
                         ids=["fast", "fast_many", "one_unsorted"])
def test_register_votes_batch_fast_path(oracle, seed, n_resp, unsorted):
    """The batch fast path (engine.cpp av_register_votes_batch: each
    Response's targets strictly ascending — a poll set's order, rule R1 — so
    k_dropin_resp applies each lane's run in place, one workgroup per node,
    its Responses in call order, no grouping) == the oracle's RegisterVotes
    per Response, and == the same engine forced onto the sort-grouped path
    (option dropin_fast = 0). Nodes repeat across the batch. unsorted: one
    Response out of order sends the whole batch down the general path."""
    rng = np.random.default_rng(seed)
    n, m = 300, 1000
    engs = []
    for fast in (1, 0):
        e = avhip.Engine(n, m, k=8, seed=seed)
        e.set_option("dropin_fast", fast)
        e.init_records(avhip.INIT_BERNOULLI, int(0.6 * 2**32))
        e.set_valid(11, False)
        engs.append(e)
    sim = oracle.Sim(n, m, 8, seed=seed, init_mode=3, init_param=int(0.6 * 2**32))
    sim.set_valid(11, False)
    for _ in range(15):  # counts near 120: batches finalize records
        for e in engs:
            e.run_rounds(1)
        sim.run_round()
    for e in engs:
        e.discard_updates()
    for batch in range(3):
        nodes = np.concatenate([rng.permutation(n)[:n_resp // 2], rng.integers(0, n, n_resp - n_resp // 2)])
        parts = []
        for _ in range(n_resp):
            k = int(rng.integers(0, 700))
            parts.append(np.sort(rng.choice(np.arange(-3, m + 3), size=k, replace=False)))
        if unsorted:
            parts[n_resp // 2] = parts[n_resp // 2][::-1].copy()
        offsets = np.concatenate([[0], np.cumsum([len(q) for q in parts])])
        targets = np.concatenate(parts).astype(np.int64)
        errs = rng.choice(ERRS, size=targets.size)
        got = [e.register_votes_batch(nodes, offsets, targets, errs) for e in engs]
        assert np.array_equal(got[0], got[1]), batch
        for i in range(n_resp):
            a, b = int(offsets[i]), int(offsets[i + 1])
            exp = sim.register_votes(int(nodes[i]), targets[a:b], errs[a:b])
            have = [(int(targets[v]), int(got[0][v])) for v in range(a, b) if got[0][v] >= 0]
            assert have == exp, (batch, i)
        check(engs[0], sim, f"fast batch {batch}")
        assert np.array_equal(engs[0].read_records(), engs[1].read_records())
    for e in engs:
        e.run_rounds(1)
    exp_u, _ = sim.run_round()
    for e in engs:
        assert np.array_equal(e.fetch_updates(), exp_u)
        e.close()
