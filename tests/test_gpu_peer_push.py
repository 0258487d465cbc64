"""Node-sharded engines with the peer-push exchange (av_peer_handles /
av_peer_init): one process per rank, all on device 0 here (the
IPC mappings are the same calls whether the peer is this GPU or another one
over xGMI), compared bit for bit with the CPU oracle running the whole network.
Covers the sweep kernel's changed-word push (warm rounds, recomputed vote
registers, finalization) and the full-row push after rounds of the other
kernels (capped path, first-generation kernel)."""
import multiprocessing as mp
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BYZ20 = int(0.2 * 2**32)
P80 = int(0.8 * 2**32)

CASES = {
    # name: (N, M, k, byz, init_mode, init_param, rounds, options)
    "c4_shape_vv": (512, 1000, 8, 0, 3, P80, 22, {}),
    "byz_pairs": (256, 200, 8, BYZ20, 4, 0, 30, {}),
    "k5_first_gen": (192, 130, 5, BYZ20, 3, P80, 12, {"kernel": 1}),
    "capped": (64, 4200, 8, 0, 3, P80, 6, {}),
    # bench.py's epoch protocol: the network re-populated (av_init_records, collective) after 9
    # rounds; the new rows must reach every replica (compared: the rounds after the re-population)
    "c4_shape_reinit": (512, 1000, 8, 0, 3, P80, 22, {"_reinit": 9}),
    "byz_pairs_reinit": (256, 200, 8, BYZ20, 4, 0, 20, {"_reinit": 7}),
    # uniform rows on / off across ranks (mismatch slots pushed to the replicas)
    "c4_shape_uniform_off": (512, 1000, 8, 0, 3, P80, 22, {"uniform_rows": 0}),
    # the need-masked exchange (default on where the layout allows it: here BL 32 and 8) and off
    "c4_shape_unmasked": (512, 1000, 8, 0, 3, P80, 22, {"peer_mask": 0}),
    "pairs_bl8_masked": (512, 256, 8, BYZ20, 4, 0, 24, {}),
}


def _rank_main(case, world, rank, d, q):
    try:
        import avhip

        n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
        per = n // world
        e = avhip.Engine(n, m, k=k, seed=11, byz_threshold=byz, node_range=(rank * per, (rank + 1) * per),
                         device=0, log_capacity=1 << 22)
        for name, v in opts.items():
            if not name.startswith("_"):
                e.set_option(name, v)
        e.init_records(init_mode, init_param)
        tmp = os.path.join(d, f"h{rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(e.peer_handles())
        os.rename(tmp, os.path.join(d, f"h{rank}.bin"))
        t0 = time.time()
        paths = [os.path.join(d, f"h{r}.bin") for r in range(world)]
        while not all(os.path.exists(p) for p in paths):
            if time.time() - t0 > 60:
                raise TimeoutError("peer handles did not arrive")
            time.sleep(0.05)
        handles = []
        for p in paths:
            with open(p, "rb") as f:
                handles.append(f.read())
        e.peer_init(world, rank, handles)
        try:  # a record write outside a round would desynchronise the replicas
            e.add_targets(rank * per, [0], [1])
            raise AssertionError("add_targets accepted on a peer-push engine")
        except avhip.AvError:
            pass
        if "_reinit" in opts:  # bench.py's epoch start: a fresh network at round r1 (collective)
            e.run_rounds(opts["_reinit"])
            e.synchronize()
            e.discard_updates()
            e.init_records(init_mode, init_param)
            e.run_rounds(rounds - opts["_reinit"])
        else:
            # two calls: stale vote planes and snapshot rotation carried across them
            e.run_rounds(rounds // 2)
            e.run_rounds(rounds - rounds // 2)
        e.synchronize()
        np.save(os.path.join(d, f"rec{rank}.npy"), e.read_records())
        np.save(os.path.join(d, f"upd{rank}.npy"), e.fetch_updates())
        # need-masked pushes leave rows no local node reads behind: complete every replica first
        e.peer_sync()
        np.save(os.path.join(d, f"pref{rank}.npy"), e.read_pref())
        e.close()
        q.put((rank, "ok"))
    except Exception as ex:  # report, never hang the parent
        q.put((rank, f"error: {ex!r}"))


def run_ranks(case, world, tmp_path):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(case, world, r, str(tmp_path), q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + 100
    while len(res) < world and time.time() < deadline:
        try:
            r, msg = q.get(timeout=1)
            res[r] = msg
        except Exception:
            pass
    for p in procs:
        p.join(timeout=max(1, deadline - time.time()))
    for p in procs:
        if p.is_alive():
            p.kill()
    assert len(res) == world, f"ranks did not finish: {res}"
    assert all(v == "ok" for v in res.values()), res
    rec = np.concatenate([np.load(tmp_path / f"rec{r}.npy") for r in range(world)])
    upd = np.concatenate([np.load(tmp_path / f"upd{r}.npy") for r in range(world)])
    upd = upd[np.lexsort(upd.T[::-1])] if len(upd) else upd
    prefs = [np.load(tmp_path / f"pref{r}.npy") for r in range(world)]
    return rec, upd, prefs


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("case", sorted(CASES))
def test_peer_push_vs_oracle(oracle, case, world, tmp_path):
    n, m, k, byz, init_mode, init_param, rounds, opts = CASES[case]
    rec, upd, prefs = run_ranks(case, world, tmp_path)
    sim = oracle.Sim(n, m, k, seed=11, byz_threshold=byz, init_mode=init_mode, init_param=init_param)
    if "_reinit" in opts:  # a fresh network populated at round r1 (oracle Sim.set_round_index)
        sim.set_round_index(opts["_reinit"])
        rounds -= opts["_reinit"]
    exp = [sim.run_round()[0] for _ in range(rounds)]
    exp = np.concatenate(exp)
    exp = exp[np.lexsort(exp.T[::-1])]
    assert np.array_equal(rec, sim.dump()), "VoteRecord state differs from the oracle"
    assert np.array_equal(upd, exp), "StatusUpdate stream differs from the oracle"
    # every rank's replica of the published preferences is the whole network's
    for p in prefs:
        assert np.array_equal(p, prefs[0])


def test_peer_push_world1(tmp_path):
    """A one-rank peer exchange is the unsharded engine (no pushes, no barrier)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_world1_main, args=(q,))
    p.start()
    msg = q.get(timeout=90)
    p.join(timeout=30)
    assert msg == "ok", msg


def _world1_main(q):
    try:
        import avhip

        e = avhip.Engine(64, 64, node_range=(0, 64), device=0)
        e.init_records(3, P80)
        e.peer_init(1, 0, [e.peer_handles()])
        e.run_rounds(2)
        e.close()
        q.put("ok")
    except Exception as ex:
        q.put(f"error: {ex!r}")


def _absent_main(world, rank, d, q):
    """Rank 1 maps the exchange and then never takes part in a round."""
    try:
        import avhip

        n, m = 128, 64
        per = n // world
        e = avhip.Engine(n, m, k=8, seed=3, node_range=(rank * per, (rank + 1) * per), device=0)
        e.init_records(3, P80)
        e.set_option("barrier_timeout_ms", 1500)
        tmp = os.path.join(d, f"h{rank}.tmp")
        with open(tmp, "wb") as f:
            f.write(e.peer_handles())
        os.rename(tmp, os.path.join(d, f"h{rank}.bin"))
        t0 = time.time()
        paths = [os.path.join(d, f"h{r}.bin") for r in range(world)]
        while not all(os.path.exists(p) for p in paths):
            if time.time() - t0 > 60:
                raise TimeoutError("peer handles did not arrive")
            time.sleep(0.05)
        handles = [open(p, "rb").read() for p in paths]
        e.peer_init(world, rank, handles)
        done = os.path.join(d, "rank0.done")
        if rank == 1:  # absent: wait (engine mapped) until rank 0 has seen the failure
            while not os.path.exists(done) and time.time() - t0 < 90:
                time.sleep(0.05)
            e.close()
            q.put((rank, "ok"))
            return
        e.run_rounds(1)  # its barrier waits for rank 1, which never arrives
        seen = []
        for name, call in [("synchronize", e.synchronize), ("run_rounds", lambda: e.run_rounds(1)),
                           ("read_records", e.read_records), ("fetch_updates", e.fetch_updates),
                           ("applied_votes", e.applied_votes)]:
            try:
                call()
                seen.append(f"{name}: accepted")
            except avhip.PeerExchangeFailed:
                seen.append(f"{name}: refused")
        open(done, "w").close()
        e.close()
        q.put((rank, "ok" if all(s.endswith("refused") for s in seen) else f"error: {seen}"))
    except Exception as ex:
        open(os.path.join(d, "rank0.done"), "w").close()
        q.put((rank, f"error: {ex!r}"))


def test_peer_barrier_timeout_fails_engine(tmp_path):
    """A rank that never arrives at the round barrier: the barrier gives up
    after its timeout and every later round and result of the engine is
    refused with AV_ERR_PEER (sticky), instead of running rounds unordered."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_absent_main, args=(2, r, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    deadline = time.time() + 100
    while len(res) < 2 and time.time() < deadline:
        try:
            r, msg = q.get(timeout=1)
            res[r] = msg
        except Exception:
            pass
    for p in procs:
        p.join(timeout=max(1, deadline - time.time()))
        if p.is_alive():
            p.kill()
    assert res == {0: "ok", 1: "ok"}, res
