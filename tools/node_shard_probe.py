#!/usr/bin/env python3
"""Per-rank round-kernel time of a NODE shard of C4 (rank 0's N/G nodes, all
targets), measured alone on one GPU with the diagnostics option
"unsynced_shard" (no exchange: timing only, results invalid). Compare with
tools/ab_tune.py's target shards: the node shard keeps BL = 32 rows and reads
N*k/G peer rows instead of N*k.

    python tools/node_shard_probe.py [--shards 1,2,4,8] [--rounds 6] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import avhip  # noqa: E402
from avhip import sharding  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--rounds", type=int, default=14)
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--json", default=None)
    ap.add_argument("--kinds", default="nodes,targets")
    ap.add_argument("--option", action="append", default=[], help="name=value, set on every engine")
    args = ap.parse_args()
    N, M, K, init_mode, init_param, byz, replay, _ = WORKLOADS[args.workload]
    out = {}

    def timed(e, rounds):
        # bench.py's protocol: device warm-up pass, re-init, 2 warmup rounds,
        # then `rounds` back-to-back rounds timed around a synchronize
        e.init_records(init_mode, init_param)
        e.run_rounds(2 + rounds)
        e.synchronize()
        e.discard_updates()
        e.init_records(init_mode, init_param)
        e.run_rounds(2)
        e.synchronize()
        e.discard_updates()
        t0 = time.perf_counter()
        e.run_rounds(rounds)
        e.synchronize()
        return (time.perf_counter() - t0) / rounds * 1e3

    for g in [int(x) for x in args.shards.split(",")]:
        for kind in args.kinds.split(","):
            if kind == "nodes":
                e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz,
                                 node_range=sharding.node_shard(N, g, 0), log_capacity=1 << 26)
                e.set_option("unsynced_shard", 1)
            else:
                e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz,
                                 target_range=sharding.target_shard(M, g, 0), log_capacity=1 << 26)
            for o in args.option:
                name, v = o.split("=")
                e.set_option(name, int(v))
            ms = [timed(e, args.rounds) for _ in range(3)]
            e.close()
            key = f"{args.workload}_{kind}shard{g}" + "".join("_" + o for o in args.option)
            out[key] = {"ms_per_round": ms, "median_ms": statistics.median(ms)}
            print(key, out[key], flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
