#!/usr/bin/env python3
"""Fixed per-round cost of the peer-push exchange, measured in
the one-GPU rehearsal: `world` rank processes, each a node shard of one
network (every rank on device 0). Each rank times R back-to-back warm rounds
of its shard twice, in the same contended setup (all ranks running at once,
started together):
  1. `unsynced`: the shard alone (option unsynced_shard: no pushes, no barrier);
  2. `exchange`: the same shard with the peer exchange (av_peer_init: changed
     words pushed into the peers' replicas + the device barrier per round).
The exchange's cost per round = slowest rank's (2) - slowest rank's (1): the
same shards, the same GPU sharing, only the exchange differs. (The previous
form subtracted the unsharded engine's round / world, which charged the
contention of the shared GPU to the exchange.)

    python tools/barrier_cost.py [--world 2] [--nodes 8192] [--targets 1000] [--rounds 200]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))

P80 = int(0.8 * 2**32)


def _run(eng, warm, rounds):
    eng.run_rounds(warm)
    eng.synchronize()
    eng.discard_updates()
    t0 = time.perf_counter()
    eng.run_rounds(rounds)
    eng.synchronize()
    dt = time.perf_counter() - t0
    eng.discard_updates()
    eng.set_timing(True)
    eng.run_rounds(rounds)
    ms, nl = eng.kernel_stats()
    eng.set_timing(False)
    eng.discard_updates()
    return dt / rounds * 1e3, ms / max(1, nl)


def _meet(d, name, world, rank, timeout=60):
    """File barrier across the rank processes (host side, between phases)."""
    open(os.path.join(d, f"{name}.{rank}"), "w").close()
    t0 = time.time()
    while not all(os.path.exists(os.path.join(d, f"{name}.{r}")) for r in range(world)):
        if time.time() - t0 > timeout:
            raise TimeoutError(f"ranks did not meet at {name}")
        time.sleep(0.005)


def _engine(args, world, rank):
    import avhip

    per = args.nodes // world
    e = avhip.Engine(args.nodes, args.targets, k=8, seed=3, node_range=(rank * per, (rank + 1) * per), device=0,
                     log_capacity=1 << 24)
    for o in args.option:
        name, v = o.split("=")
        e.set_option(name, int(v))
    e.init_records(avhip.INIT_BERNOULLI, P80)
    return e


def _rank(args, world, rank, d, q):
    try:
        out = {}
        # 1. the shard alone, every rank at once (no exchange)
        e = _engine(args, world, rank)
        e.set_option("unsynced_shard", 1)
        _meet(d, "a", world, rank)
        ms, kms = _run(e, args.warm, args.rounds)
        e.close()
        out["unsynced"] = {"ms_per_round": ms, "kernel_ms_per_launch": kms}
        # 2. the same shard with the peer exchange
        e = _engine(args, world, rank)
        with open(os.path.join(d, f"h{rank}.tmp"), "wb") as f:
            f.write(e.peer_handles())
        os.rename(os.path.join(d, f"h{rank}.tmp"), os.path.join(d, f"h{rank}.bin"))
        paths = [os.path.join(d, f"h{r}.bin") for r in range(world)]
        t0 = time.time()
        while not all(os.path.exists(p) for p in paths):
            if time.time() - t0 > 60:
                raise TimeoutError("peer handles did not arrive")
            time.sleep(0.02)
        e.peer_init(world, rank, [open(p, "rb").read() for p in paths])
        _meet(d, "b", world, rank)
        ms, kms = _run(e, args.warm, args.rounds)
        out["exchange"] = {"ms_per_round": ms, "kernel_ms_per_launch": kms,
                           "changed_words_per_round": e.changed_words()[0] / (args.warm + 2 * args.rounds)}
        e.close()
        q.put((rank, out))
    except Exception as ex:
        q.put((rank, {"error": repr(ex)[:300]}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--nodes", type=int, default=8192)
    ap.add_argument("--targets", type=int, default=1000)
    ap.add_argument("--warm", type=int, default=8)
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--option", action="append", default=[], help="name=value engine option for the rank engines")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        procs = [ctx.Process(target=_rank, args=(args, args.world, r, d, q)) for r in range(args.world)]
        for p in procs:
            p.start()
        res = {}
        deadline = time.time() + 150
        while len(res) < args.world and time.time() < deadline:
            try:
                r, v = q.get(timeout=1.0)
                res[r] = v
            except Exception:
                pass
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    out = {"options": args.option, "world": args.world, "nodes": args.nodes, "targets": args.targets,
           "rounds": args.rounds, "ranks": res}
    ok = [v for v in res.values() if "exchange" in v]
    if len(ok) == args.world:
        ex = max(v["exchange"]["ms_per_round"] for v in ok)
        un = max(v["unsynced"]["ms_per_round"] for v in ok)
        out["exchange_fixed_cost_us"] = (ex - un) * 1e3
        out["note"] = ("slowest rank's per-round wall time with the exchange minus the same shards without it "
                       "(unsynced_shard), all ranks on one GPU at once in both phases")
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
