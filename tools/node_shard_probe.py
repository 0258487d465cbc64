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
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    N, M, K, init_mode, init_param, byz, replay, _ = WORKLOADS[args.workload]
    out = {}
    for g in [int(x) for x in args.shards.split(",")]:
        for vv in (1, 0):
            e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz,
                             node_range=sharding.node_shard(N, g, 0), log_capacity=1 << 26)
            e.set_option("unsynced_shard", 1)
            e.set_option("virtual_votes", vv)
            e.init_records(init_mode, init_param)
            e.run_rounds(3)
            e.synchronize()
            e.discard_updates()
            ts = []
            for _ in range(args.rounds):
                e.set_timing(True)
                e.run_rounds(1)
                ms, n = e.kernel_stats()
                e.set_timing(False)
                ts.append(ms / max(n, 1))
            e.close()
            key = f"{args.workload}_nodeshard{g}_vv{vv}"
            out[key] = {"nodes": list(sharding.node_shard(N, g, 0)), "median_ms": statistics.median(ts),
                        "min_ms": min(ts)}
            print(key, out[key], flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
