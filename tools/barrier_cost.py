#!/usr/bin/env python3
"""Fixed per-round cost of the peer-push exchange, measured in
the one-GPU rehearsal: `world` rank processes, each a node shard of a small
network with the peer exchange (av_peer_init; every rank on device 0), time
R back-to-back warm rounds; the same network on one engine without an
exchange is the baseline. On a small network the round kernels take a few
microseconds, so the difference per round is the exchange's fixed cost: the
folded arrival in the round kernel's last wave, the 1-wave wait kernel and its
launch gap (plus the interleaving of the ranks' kernels on one GPU, which the
8-GPU case does not have).

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
    return dt / rounds * 1e3, ms / max(1, nl)


def _rank(args, world, rank, d, q):
    try:
        import avhip

        per = args.nodes // world
        e = avhip.Engine(args.nodes, args.targets, k=8, seed=3, node_range=(rank * per, (rank + 1) * per), device=0,
                         log_capacity=1 << 24)
        for o in args.option:
            name, v = o.split("=")
            e.set_option(name, int(v))
        e.init_records(avhip.INIT_BERNOULLI, P80)
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
        ms, kms = _run(e, args.warm, args.rounds)
        e.close()
        q.put((rank, {"ms_per_round": ms, "kernel_ms_per_launch": kms}))
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
    import avhip

    e = avhip.Engine(args.nodes, args.targets, k=8, seed=3, device=0, log_capacity=1 << 24)
    e.init_records(avhip.INIT_BERNOULLI, P80)
    base_ms, base_kms = _run(e, args.warm, args.rounds)
    e.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        procs = [ctx.Process(target=_rank, args=(args, args.world, r, d, q)) for r in range(args.world)]
        for p in procs:
            p.start()
        res = {}
        deadline = time.time() + 120
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
    out = {"options": args.option, "world": args.world, "nodes": args.nodes, "targets": args.targets, "rounds": args.rounds,
           "single_engine": {"ms_per_round": base_ms, "kernel_ms_per_launch": base_kms}, "ranks": res}
    ok = [v for v in res.values() if "ms_per_round" in v]
    if len(ok) == args.world:
        out["exchange_fixed_cost_us"] = (max(v["ms_per_round"] for v in ok) - base_ms / args.world) * 1e3
        out["note"] = ("per-round wall time of the slowest rank minus the unsharded engine's per-round time / world "
                       "(the ranks' shards share one GPU here)")
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
