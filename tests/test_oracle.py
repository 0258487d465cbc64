"""CPU tests: pin the oracle (C restatement + Python restatement) against the
golden vectors transcribed from the reference's own tests, and against each
other on exhaustive single-vote transitions and seeded multi-round sims."""
import numpy as np
import pytest

from golden_ops import NotFound, run_processor, run_vote_record
from oracle import avalanche_ref as ref


# ---------------------------------------------------------------- adapters
class CRecord:
    def __init__(self, oracle, accepted):
        self.o = oracle
        self.w = np.array([1 << 16 if accepted else 0], np.uint32)

    def state(self):
        w = int(self.w[0])
        conf = w >> 16
        return (bool(conf & 1), (conf >> 1) >= 128, conf >> 1)

    def vote(self, err):
        self.w, _, _ = self.o.transition_batch(self.w, np.array([err], np.uint32))
        return self.state()


class PyRecord:
    def __init__(self, accepted):
        self.r = ref.VoteRecord(accepted)

    def state(self):
        return (self.r.is_accepted(), self.r.has_finalized(), self.r.get_confidence())

    def vote(self, err):
        self.r.register_vote(err)
        return self.state()


class CProc:
    """C oracle Processor of node 0 in a 2-node sim, hash == target index."""

    def __init__(self, oracle, fx):
        self.accepted = {int(h): v["accepted"] for h, v in fx["targets"].items()}
        self.m = max(self.accepted) + 1
        self.sim = oracle.Sim(2, self.m, 1, init_mode=0)

    def words(self):
        return self.sim.dump()[0]

    def add(self, h):
        return self.sim.add(0, h, self.accepted[h])

    def register(self, node, votes):
        return self.sim.register_votes(0, [h for _, h in votes], [e for e, _ in votes])

    def is_accepted(self, h):
        w = int(self.words()[h])
        return (w >> 17) < 128 and bool((w >> 16) & 1)

    def confidence(self, h):
        w = int(self.words()[h])
        if (w >> 17) >= 128:
            raise NotFound()
        return w >> 17

    def invs(self):
        w = self.words()
        return [t for t in range(self.m) if (int(w[t]) >> 17) < 128][:4096]

    def get_round(self):
        return self.sim.get_round(0)

    def inc_round(self):
        self.sim.set_round(0, self.sim.get_round(0) + 1)


class PyProc:
    def __init__(self, fx):
        self.targets = {int(h): ref.Target(int(h), v["accepted"], v["valid"]) for h, v in fx["targets"].items()}
        self.p = ref.Processor()

    def add(self, h):
        return self.p.add_target_to_reconcile(self.targets[h])

    def register(self, node, votes):
        ups = []
        self.p.register_votes(node, [(h, e) for e, h in votes], ups)
        return ups

    def is_accepted(self, h):
        return self.p.is_accepted(h)

    def confidence(self, h):
        try:
            return self.p.get_confidence(h)
        except KeyError:
            raise NotFound()

    def invs(self):
        return self.p.get_invs_for_next_poll()

    def get_round(self):
        return self.p.get_round()

    def inc_round(self):
        self.p.round += 1


# ---------------------------------------------------------------- golden vectors
def test_philox_kat(golden, oracle):
    for v in golden["philox4x32_10_kat"]:
        assert list(oracle.philox(v["ctr"], v["key"])) == v["out"]
        assert ref.philox4x32_10(v["ctr"], v["key"]) == v["out"]


def test_vote_record_golden_c(golden, oracle):
    run_vote_record(golden["vote_record"], lambda acc: CRecord(oracle, acc))


def test_vote_record_golden_py(golden):
    run_vote_record(golden["vote_record"], PyRecord)


@pytest.mark.parametrize("which", [0, 1])
def test_processor_golden_c(golden, oracle, which):
    fx = golden["processor"][which]
    run_processor(fx, CProc(oracle, fx))


@pytest.mark.parametrize("which", [0, 1])
def test_processor_golden_py(golden, which):
    fx = golden["processor"][which]
    run_processor(fx, PyProc(fx))


def test_golden_fixture_matches_generator(golden, tmp_path):
    """The committed fixture is exactly what make_golden.py produces."""
    import importlib.util
    import json
    import os

    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(here, "golden", "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    assert json.loads(json.dumps(mg.vote_record())) == golden["vote_record"]
    assert json.loads(json.dumps([mg.block_register(), mg.multi_block_register()])) == golden["processor"]


# ---------------------------------------------------------------- exhaustive transitions
REPR_ERRS = np.array([0, 1, 2, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFF], np.uint32)


def reachable_words():
    """All (votes, consider) with votes subset of consider (3^8 = 6561) x confidence in
    {0..257} plus u16 wrap edges."""
    v = np.arange(256, dtype=np.uint32)
    vv, cc = np.meshgrid(v, v, indexing="ij")
    ok = (vv & ~cc) == 0
    vc = (vv[ok] | (cc[ok] << 8)).astype(np.uint32)
    assert vc.size == 6561
    conf = np.concatenate([np.arange(258, dtype=np.uint32), np.array([65532, 65533, 65534, 65535], np.uint32)])
    return (vc[:, None] | (conf[None, :] << 16)).ravel()


def numpy_transition(words, errs):
    """Third, vectorised restatement of vote.go:54-75 used only for this check."""
    pc = np.array([bin(i).count("1") for i in range(256)], np.int64)
    votes = words & 0xFF
    cons = (words >> 8) & 0xFF
    conf = (words >> 16).astype(np.int64)
    votes = ((votes << 1) & 0xFF) | (errs == 0)
    cons = ((cons << 1) & 0xFF) | (errs.view(np.int32) >= 0)
    yes = pc[votes & cons] > 6
    concl = yes | (pc[(~votes) & cons & 0xFF] > 6)
    agree = concl & ((conf & 1).astype(bool) == yes)
    flip = concl & ~agree
    new_conf = np.where(agree, (conf + 2) & 0xFFFF, np.where(flip, yes.astype(np.int64), conf))
    changed = np.where(agree, (new_conf >> 1) == 128, flip)
    out = (votes | (cons << 8) | (new_conf << 16)).astype(np.uint32)
    return out, changed


def test_exhaustive_transitions_c_vs_numpy(oracle):
    w = reachable_words()
    for e in REPR_ERRS:
        errs = np.full(w.shape, e, np.uint32)
        got, ch, _ = oracle.transition_batch(w, errs)
        exp, ch2 = numpy_transition(w.astype(np.int64), errs)
        assert np.array_equal(got, exp)
        assert np.array_equal(ch.astype(bool), ch2)


def test_sampled_transitions_c_vs_python(oracle):
    rng = np.random.default_rng(1)
    w = rng.choice(reachable_words(), 20000)
    errs = rng.choice(REPR_ERRS, w.size)
    got, ch, st = oracle.transition_batch(w, errs)
    for i in range(w.size):
        r = ref.VoteRecord.from_word(int(w[i]))
        c = r.register_vote(int(errs[i]))
        assert r.word() == int(got[i]) and c == bool(ch[i]) and r.status() == int(st[i])


# ---------------------------------------------------------------- synthetic workload + sims
def test_sampling_c_vs_python(oracle):
    for n_nodes, k, mode in [(1000, 8, 0), (12, 8, 0), (9, 8, 0), (5, 3, 1), (50, 16, 0), (3, 4, 0)]:
        for node in range(min(n_nodes, 6)):
            for rnd in range(4):
                got = oracle.sample_peers(11, node, rnd, n_nodes, k, mode).tolist()
                assert got == ref.sample_peers(11, node, rnd, n_nodes, k, mode)
                if mode == 0 and k < n_nodes - 1:
                    assert len(set(got)) == k and node not in got


def test_replay_errs_c_vs_python(oracle):
    e = oracle.gen_replay_errs(5, 3, 2, 4, 37, 3)
    for n in range(2, 4):
        for s in range(3):
            for t in range(37):
                assert int(e[n - 2, s, t]) == ref.replay_err(5, n, 3, s, t)


SIM_CASES = [
    dict(n=12, m=40, k=8, seed=7, init_mode=3, init_param=int(0.8 * 2**32)),
    dict(n=10, m=33, k=8, seed=9, init_mode=4, byz=int(0.2 * 2**32)),
    dict(n=6, m=20, k=3, seed=3, init_mode=2, peer_mode=1),
    dict(n=8, m=70, k=5, seed=4, init_mode=1, byz=int(0.3 * 2**32)),
]


@pytest.mark.parametrize("case", SIM_CASES)
def test_sim_c_vs_python(oracle, case):
    kw = dict(seed=case["seed"], peer_mode=case.get("peer_mode", 0), byz_threshold=case.get("byz", 0),
              init_mode=case["init_mode"], init_param=case.get("init_param", 0x80000000))
    c = oracle.Sim(case["n"], case["m"], case["k"], **kw)
    p = ref.Sim(case["n"], case["m"], case["k"], **kw)
    assert np.array_equal(c.dump(), p.dump())
    for r in range(24):
        if r == 5:  # a target stops being valid mid-run (avalanche_test.go:534 pattern)
            c.set_valid(3, False)
            p.set_valid(3, False)
        if r == 11:
            c.set_valid(3, True)
            p.set_valid(3, True)
        u1, _ = c.run_round()
        u2 = p.run_round()
        assert [tuple(x) for x in u1.tolist()] == [tuple(x) for x in u2], r
        assert np.array_equal(c.dump(), p.dump()), r


def test_sim_replay_capped_c_vs_python(oracle):
    """M > 4096: the poll cap (processor.go:165-167) binds; replayed votes incl. neutral."""
    n, m, k = 3, 4200, 2
    c = oracle.Sim(n, m, k, seed=2, init_mode=3)
    p = ref.Sim(n, m, k, 2, init_mode=3)
    for r in range(3):
        errs = oracle.gen_replay_errs(2, r, 0, n, m, k)
        u1, applied = c.run_round(errs)
        u2 = p.run_round(errs)
        assert applied == n * k * 4096
        assert [tuple(x) for x in u1.tolist()] == [tuple(x) for x in u2]
        assert np.array_equal(c.dump(), p.dump())


def test_oracle_threads_deterministic(oracle):
    a = oracle.Sim(64, 100, 8, seed=1, byz_threshold=int(0.2 * 2**32))
    b = oracle.Sim(64, 100, 8, seed=1, byz_threshold=int(0.2 * 2**32))
    for _ in range(20):
        u1, n1 = a.run_round(threads=1)
        u2, n2 = b.run_round(threads=4)
        assert np.array_equal(u1, u2) and n1 == n2
    assert np.array_equal(a.dump(), b.dump())


def test_branchfree_step_vs_literal_exhaustive(oracle):
    """The oracle's branch-free step (the batched sim's fast form) equals the
    literal avo_register_vote (vote.go:54-75) on every reachable record state
    and every err class, including the finalizing step (count 127 -> 128)."""
    w = reachable_words()
    for e in REPR_ERRS:
        errs = np.full(w.shape, e, np.uint32)
        exp, ch, st = oracle.transition_batch(w, errs)
        got, gst = oracle.transition_batch_branchfree(w, errs)
        assert np.array_equal(got, exp), hex(e)
        assert np.array_equal(gst, np.where(ch.astype(bool), st.astype(np.int8), -1)), hex(e)


BF_CASES = [
    dict(n=300, m=517, k=8, seed=5, init_mode=4, byz=int(0.2 * 2**32)),
    dict(n=64, m=200, k=8, seed=3, init_mode=2),
    dict(n=40, m=96, k=5, seed=8, init_mode=3, init_param=int(0.8 * 2**32), peer_mode=1),
    dict(n=9, m=33, k=8, seed=4, init_mode=1, byz=int(0.45 * 2**32)),
    dict(n=20, m=4500, k=8, seed=6, init_mode=2),   # M > 4096: cap binds -> literal path per node
    dict(n=30, m=300, k=8, seed=9, init_mode=3, replay=True),
]


@pytest.mark.parametrize("case", BF_CASES, ids=lambda c: f"n{c['n']}m{c['m']}k{c['k']}")
def test_sim_branchfree_vs_literal(oracle, case):
    """The batched sim's branch-free per-node form == the literal per-vote
    path (GetInvsForNextPoll + RegisterVotes per slot) through finalization,
    validity flips and replayed neutral votes."""
    kw = dict(seed=case["seed"], peer_mode=case.get("peer_mode", 0), byz_threshold=case.get("byz", 0),
              init_mode=case["init_mode"], init_param=case.get("init_param", 0x80000000))
    a = oracle.Sim(case["n"], case["m"], case["k"], threads=3, **kw)
    b = oracle.Sim(case["n"], case["m"], case["k"], **kw)
    b.set_literal()
    for r in range(22):
        if r == 4:
            a.set_valid(2, False)
            b.set_valid(2, False)
        if r == 9:
            a.set_valid(2, True)
            b.set_valid(2, True)
        errs = oracle.gen_replay_errs(case["seed"], r, 0, case["n"], case["m"], case["k"]) if case.get("replay") else None
        ua, na = a.run_round(errs, threads=3)
        ub, nb = b.run_round(errs)
        assert na == nb and np.array_equal(ua, ub), r
    assert np.array_equal(a.dump(), b.dump())


def test_digest_mode_matches_rows(oracle):
    kw = dict(seed=11, byz_threshold=int(0.2 * 2**32), init_mode=4)
    a = oracle.Sim(200, 300, 8, **kw)
    b = oracle.Sim(200, 300, 8, **kw)
    for r in range(6):
        u, na = a.run_round(threads=2)
        d, nb = b.run_round(threads=2, collect=False, round_rel=3)
        words = ((np.uint64(3) << np.uint64(52)) | (u[:, 1].astype(np.uint64) << np.uint64(28))
                 | (u[:, 2].astype(np.uint64) << np.uint64(24)) | (u[:, 3].astype(np.uint64) << np.uint64(2))
                 | u[:, 4].astype(np.uint64))
        assert na == nb and d == oracle.update_digest(words), r
        assert int(words[0]) == oracle.pack_update(3, int(u[0, 1]), int(u[0, 2]), int(u[0, 3]), int(u[0, 4]))
    assert np.array_equal(a.dump(), b.dump())


@pytest.mark.parametrize("responder", [1, 2])
def test_sim_responder_modes_c_vs_python(oracle, responder):
    """Responder variants: 1 = IsAccepted literally (a deleted
    record answers no, processor.go:125-130); 2 = the example's responder
    (main.go:175-182: a queried target it does not hold is re-added as
    accepted and answered yes). Some nodes stop polling (the example's run
    loop returns, main.go:160-162) but keep answering."""
    n, m, k = 24, 70, 3
    kw = dict(seed=6, byz_threshold=int(0.2 * 2**32), init_mode=2)
    c = oracle.Sim(n, m, k, **kw)
    p = ref.Sim(n, m, k, 6, byz_threshold=int(0.2 * 2**32), init_mode=2)
    c.set_responder(responder)
    p.set_responder(responder)
    for r in range(60):
        if r == 30:
            for j in (2, 5, 11):
                c.set_polling(j, False)
                p.polls[j] = False
        if r == 20:
            c.set_valid(4, False)
            p.set_valid(4, False)
        u1, _ = c.run_round()
        u2 = p.run_round()
        assert [tuple(x) for x in u1.tolist()] == [tuple(x) for x in u2], r
        assert np.array_equal(c.dump(), p.dump()), r
        assert np.array_equal(c.pref(), np.array(p.pref, np.uint8)), r


def run_example_oracle(oracle, n=100, m=100, max_rounds=2000):
    """examples/basic-preconcensus (main.go:91-192) as synchronous rounds:
    every node adds every tx as accepted (main.go:49-54), polls one peer per
    round in round-robin order skipping itself (main.go:110-116, k = 1), the
    responder re-adds what it does not hold (main.go:175-177), and a node's
    loop returns once it counted txCount Finalized updates (main.go:143-162)."""
    sim = oracle.Sim(n, m, 1, peer_mode=1, init_mode=2)
    sim.set_responder(2)
    finalized = np.zeros(n, np.int64)
    rounds, all_updates = 0, []
    while (finalized < m).any() and rounds < max_rounds:
        u, _ = sim.run_round()
        all_updates.append(u)
        fin = u[u[:, 4] == 3]
        np.add.at(finalized, fin[:, 1], 1)
        for j in np.flatnonzero(finalized >= m):
            sim.set_polling(int(j), False)
        rounds += 1
    return sim, rounds, finalized, all_updates


def test_example_c1_oracle():
    from oracle import cabi

    sim, rounds, finalized, _ = run_example_oracle(cabi)
    assert (finalized >= 100).all()  # "Nodes fully finalized: 100"
    assert rounds == 134  # every record finalizes at its 134th vote (vote.go:66-69), one vote per round
