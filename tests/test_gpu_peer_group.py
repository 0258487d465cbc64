"""The peer-push exchange of node-sharded engines with every
rank an engine of this process on device 0 (av_peer_group_serial): the rounds
of all ranks run on one stream in rank order, which stands in for the device
barrier, so that 2, 4 and 8 ranks can be checked bit for bit against the CPU
oracle running the whole network on a one-GPU box. The pushes themselves are
the same kernel stores as over IPC (test_gpu_peer_push.py runs the rank
processes). The reference's network crossing this replaces is
`networkNodes[nodeID].query(invs)` (examples/basic-preconcensus/main.go:132),
whose answers come from each peer's IsAccepted (processor.go:125-130)."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)

CASES = {
    # name: (N, M, k, byz, init_mode, init_param, rounds, options)
    "c4_shape": (512, 1000, 8, 0, 3, P80, 22, {}),
    "byz_pairs": (256, 200, 8, BYZ20, 4, 0, 30, {}),
    "pairs_bl8": (512, 256, 8, 0, 4, 0, 20, {}),
    "k5_first_gen": (192, 130, 5, BYZ20, 3, P80, 12, {"kernel": 1}),
    "c4_shape_reinit": (512, 1000, 8, 0, 3, P80, 22, {"_reinit": 9}),
    "c4_shape_uniform_off": (512, 1000, 8, 0, 3, P80, 22, {"uniform_rows": 0}),
}


def make_group(case, world, extra=()):
    n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
    per = n // world
    engs = [avhip.Engine(n, m, k=k, seed=11, byz_threshold=byz, node_range=(r * per, (r + 1) * per),
                         log_capacity=1 << 22) for r in range(world)]
    for e in engs:
        for name, v in list(opts.items()) + list(extra):
            if not name.startswith("_"):
                e.set_option(name, v)
        e.init_records(init_mode, init_param)
    avhip.peer_group_serial(engs)
    return engs


def run_case(case, world, extra=()):
    n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
    engs = make_group(case, world, extra)
    if "_reinit" in opts:  # bench.py's epoch start: the network re-populated (every rank)
        avhip.run_group_rounds(engs, opts["_reinit"])
        for e in engs:
            e.synchronize()
            e.discard_updates()
            e.init_records(init_mode, init_param)
        avhip.run_group_rounds(engs, rounds - opts["_reinit"])
    else:
        avhip.run_group_rounds(engs, rounds)
    rec = np.concatenate([e.read_records() for e in engs])
    upd = np.concatenate([e.fetch_updates() for e in engs])
    upd = upd[np.lexsort(upd.T[::-1])] if len(upd) else upd
    own = np.concatenate([e.read_pref(*e.node_range) for e in engs])
    for e in engs:
        e.close()
    return rec, upd, own


def oracle_run(oracle, case):
    n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
    sim = oracle.Sim(n, m, k, seed=11, byz_threshold=byz, init_mode=init_mode, init_param=init_param)
    if "_reinit" in opts:
        sim.set_round_index(opts["_reinit"])
        rounds -= opts["_reinit"]
    exp = np.concatenate([sim.run_round()[0] for _ in range(rounds)])
    return sim, exp[np.lexsort(exp.T[::-1])]


@pytest.mark.parametrize("mode", ["masked", "full", "direct"])
@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("case", sorted(CASES))
def test_peer_group_vs_oracle(oracle, case, world, mode):
    # masked: need-masked pushes (where the layout allows), queued per wave; full: every changed word to
    # every peer, queued; direct: every changed word stored from the tile loop (push_defer 0)
    extra = {"masked": (("peer_mask", 1),), "full": (("peer_mask", 0),),
             "direct": (("peer_mask", 0), ("push_defer", 0))}[mode]
    rec, upd, own = run_case(case, world, extra=extra)
    sim, exp = oracle_run(oracle, case)
    assert np.array_equal(rec, sim.dump()), "VoteRecord state differs from the oracle"
    assert np.array_equal(upd, exp), "StatusUpdate stream differs from the oracle"
    # every rank's own published rows = the network's round-start preferences (honest nodes: a
    # Byzantine node publishes its flip-flop pattern, which the oracle applies at vote time instead)
    honest = np.array([not sim.is_byzantine(j) for j in range(own.shape[0])])
    assert np.array_equal(own[honest], sim.pref()[honest]), "published preferences differ from the oracle"


def test_peer_group_round_order_enforced():
    """A rank may not run ahead of the group (its peers' replicas would be read
    before they are complete)."""
    engs = make_group("c4_shape", 2)
    engs[0].run_rounds(1)
    with pytest.raises(avhip.AvError):
        engs[0].run_rounds(1)  # rank 1 has not run round 0 yet
    engs[1].run_rounds(1)
    engs[0].run_rounds(1)
    for e in engs:
        e.close()


@pytest.mark.parametrize("case", ["c4_shape", "pairs_bl8"])
def test_masked_pushes_fewer_words_same_results(case):
    """8 ranks, the need-masked exchange against full pushes of every changed
    word: identical records, updates and (after av_peer_sync) identical
    replicas of the whole network's rows on every rank, with fewer words
    pushed (a rank's 1/8 of the nodes draws ~1 - e^-1 = 63 % of the rows)."""
    out = {}
    for mask in (0, 1):
        n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
        engs = make_group(case, 8, extra=(("peer_mask", mask),))
        avhip.run_group_rounds(engs, rounds)
        rec = np.concatenate([e.read_records() for e in engs])
        upd = np.concatenate([e.fetch_updates(decode=False) for e in engs])
        pushed = sum(e.pushed_words() for e in engs)
        for e in engs:
            e.peer_sync()
        reps = [e.read_pref_words() for e in engs]
        for r in reps[1:]:
            assert np.array_equal(r, reps[0]), "replicas differ after av_peer_sync"
        out[mask] = (rec, np.sort(upd), pushed, reps[0])
        for e in engs:
            e.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][3], out[1][3])
    # never more words than full pushes; in a network whose rows keep changing (conflicting pairs)
    # about the drawn share (a converging one pushes its withheld changes once a peer draws the row)
    assert 0 < out[1][2] <= out[0][2], (out[1][2], out[0][2])
    if case == "pairs_bl8":
        assert out[1][2] < 0.8 * out[0][2], (out[1][2], out[0][2])
