"""CPU (gloo, world_size 2) rehearsal of the N>1 path.

The node-sharded exchange protocol of libavhip.so (each rank updates its node
range, then the published-preference rows are all-gathered) is replayed with
the oracle as the per-rank compute and torch.distributed/gloo as the
transport; the result must equal the single-process oracle bit for bit. The
shard planners are the ones bench.py uses."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from avhip import sharding

N, M, K, ROUNDS, SEED, BYZ = 48, 90, 8, 22, 0xBEEF, int(0.2 * 2**32)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cabi

    n0, n1 = sharding.node_shard(N, world, rank)
    sim = cabi.Sim(N, M, K, seed=SEED, byz_threshold=BYZ, init_mode=4)
    ups = []
    for _ in range(ROUNDS):
        u, _ = sim.run_round_range(n0, n1)
        ups.append(u)
        rows = sim.pref()[n0:n1]
        full = sharding.allgather_pref_rows(rows, world)
        sim.set_pref_rows(0, full)
    np.save(os.path.join(out_dir, f"dump{rank}.npy"), sim.dump()[n0:n1])
    np.save(os.path.join(out_dir, f"ups{rank}.npy"), np.concatenate(ups))
    dist.barrier()
    dist.destroy_process_group()


def test_node_sharded_exchange_gloo(tmp_path, oracle):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ref = oracle.Sim(N, M, K, seed=SEED, byz_threshold=BYZ, init_mode=4)
    ref_ups = np.concatenate([ref.run_round()[0] for _ in range(ROUNDS)])
    dumps = np.concatenate([np.load(tmp_path / f"dump{r}.npy") for r in range(world)])
    assert np.array_equal(dumps, ref.dump())
    ups = np.concatenate([np.load(tmp_path / f"ups{r}.npy") for r in range(world)])
    ups = ups[np.lexsort((ups[:, 3], ups[:, 2], ups[:, 1], ups[:, 0]))]
    assert np.array_equal(ups, ref_ups)


@pytest.mark.parametrize("m", [1, 31, 32, 1000, 4096])
def test_target_shard_plan(m):
    for world in range(1, 9):
        shards = [sharding.target_shard(m, world, r) for r in range(world)]
        cover = []
        for t0, t1 in shards:
            assert t0 % 32 == 0 and t0 <= t1 <= m
            cover += list(range(t0, t1))
        assert cover == list(range(m))


def test_node_shard_plan():
    assert [sharding.node_shard(1_000_000, 8, r) for r in (0, 7)] == [(0, 125_000), (875_000, 1_000_000)]
    with pytest.raises(ValueError):
        sharding.node_shard(10, 3, 0)


def _push_rank_main(rank, world, port, out_dir):
    """The peer-push exchange (av_peer_init) restated over gloo:
    three rotating replicas of the published preferences per rank; after its
    round a rank compares its new rows with what its own replica of the output
    buffer holds (identical on every rank by induction) and sends only the
    changed entries, which every rank writes into its replica."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cabi

    n0, n1 = sharding.node_shard(N, world, rank)
    sim = cabi.Sim(N, M, K, seed=SEED, byz_threshold=BYZ, init_mode=4)
    bufs = [sim.pref().copy(), np.zeros((N, M), np.uint8), np.zeros((N, M), np.uint8)]
    cur, ups, pushed = 0, [], []
    for _ in range(ROUNDS):
        u, _ = sim.run_round_range(n0, n1)
        ups.append(u)
        nb = (cur + 1) % 3
        new = sim.pref()[n0:n1]
        idx = np.argwhere(new != bufs[nb][n0:n1])
        mine = (idx[:, 0] + n0, idx[:, 1], new[idx[:, 0], idx[:, 1]])
        allp = [None] * world
        dist.all_gather_object(allp, mine)
        for rows, cols, vals in allp:
            bufs[nb][rows, cols] = vals
        pushed.append(sum(len(v[0]) for v in allp))
        cur = nb
        sim.set_pref_rows(0, bufs[cur])
    np.save(os.path.join(out_dir, f"dump{rank}.npy"), sim.dump()[n0:n1])
    np.save(os.path.join(out_dir, f"ups{rank}.npy"), np.concatenate(ups))
    np.save(os.path.join(out_dir, f"bufs{rank}.npy"), np.stack(bufs))
    np.save(os.path.join(out_dir, f"pushed{rank}.npy"), np.array(pushed))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_peer_push_protocol_gloo(tmp_path, oracle, world):
    mp.spawn(_push_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ref = oracle.Sim(N, M, K, seed=SEED, byz_threshold=BYZ, init_mode=4)
    ref_ups = np.concatenate([ref.run_round()[0] for _ in range(ROUNDS)])
    dumps = np.concatenate([np.load(tmp_path / f"dump{r}.npy") for r in range(world)])
    assert np.array_equal(dumps, ref.dump())
    ups = np.concatenate([np.load(tmp_path / f"ups{r}.npy") for r in range(world)])
    ups = ups[np.lexsort((ups[:, 3], ups[:, 2], ups[:, 1], ups[:, 0]))]
    assert np.array_equal(ups, ref_ups)
    bufs = [np.load(tmp_path / f"bufs{r}.npy") for r in range(world)]
    for b in bufs[1:]:
        assert np.array_equal(b, bufs[0])  # every replica of every buffer identical
    assert np.array_equal(bufs[0][ROUNDS % 3], ref.pref())
    pushed = np.load(tmp_path / "pushed0.npy")
    assert pushed.max() < N * M  # never more than a full exchange
