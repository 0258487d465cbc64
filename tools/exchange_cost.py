#!/usr/bin/env python3
"""The peer exchange's fixed cost per round on ONE GPU with no contention
(DESIGN.md §5): rank 0's node shard of a network at G ranks (C4: 1M x 1000,
G = 8 -> 125k nodes) runs back-to-back rounds
  * `alone`: with no exchange (option unsynced_shard);
  * `barrier`: followed, every round, by the exchange's barrier kernel at world 1
    (option solo_barrier: the same 1-wave kernel, its system-scope release and
    its wait, and one more dependent kernel boundary per round; no pushes, no
    other rank to wait for);
so the difference is what the barrier adds per round on a rank of an 8-GPU
run before any cross-GPU latency or skew. Both over the same epoch rounds
(by round kind: storm 1-3, klazy/settled 4-15), wall clock per round of a
back-to-back stretch, several alternating repetitions.

    python tools/exchange_cost.py [--nodes 1000000] [--targets 1000] [--ranks 8] [--reps 3] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))

P80 = int(0.8 * 2**32)


def stretch(e, first, count):
    """Wall ms per round of rounds [first, first + count) of a fresh epoch, back to back."""
    e.init_records(3, P80)
    if first:
        e.run_rounds(first)
    e.synchronize()
    e.discard_updates()
    t0 = time.perf_counter()
    e.run_rounds(count)
    e.synchronize()
    dt = time.perf_counter() - t0
    e.discard_updates()
    return dt / count * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1_000_000)
    ap.add_argument("--targets", type=int, default=1000)
    ap.add_argument("--ranks", type=int, default=8)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    import avhip

    per = args.nodes // args.ranks
    e = avhip.Engine(args.nodes, args.targets, k=8, seed=3, node_range=(0, per), device=0,
                     log_capacity=min(per * args.targets * 2, (1 << 31) - 1))
    e.set_option("unsynced_shard", 1)
    stretch(e, 0, 16)  # warm-up epoch
    res = {"alone": {}, "barrier": {}}
    for _ in range(args.reps):
        for variant in ("alone", "barrier"):
            e.set_option("solo_barrier", 1 if variant == "barrier" else 0)
            for name, (a, n) in {"storm_1_3": (1, 3), "settled_4_15": (4, 12), "epoch_0_15": (0, 16)}.items():
                res[variant].setdefault(name, []).append(stretch(e, a, n))
    e.close()
    out = {"nodes": args.nodes, "targets": args.targets, "ranks": args.ranks, "shard_nodes": per, "ms_per_round": res,
           "barrier_us_per_round": {k: (min(res["barrier"][k]) - min(res["alone"][k])) * 1e3 for k in res["alone"]},
           "note": "min over repetitions; barrier = the exchange's 1-wave barrier kernel at world 1 after every round"}
    print(json.dumps(out))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
