#!/usr/bin/env python3
"""C2 replay epochs with and without fused replay rounds (k_replay_node):
HIP-event time of one 16-round replay batch, per option set.

    python tools/fuse_probe.py [--option name=value ...] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import avhip  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def epoch(e, init_mode, init_param, rounds, first):
    e.init_records(init_mode, init_param)
    if first:
        e.replay_prepare(first)
        e.replay_rounds(first)
    e.replay_prepare(rounds)
    e.synchronize()
    e.discard_updates()
    e.set_timing(True)
    t0 = time.perf_counter()
    e.replay_rounds(rounds)
    e.synchronize()
    wall = time.perf_counter() - t0
    ms, n = e.kernel_stats()
    e.set_timing(False)
    u = e.updates_count()
    e.discard_updates()
    return {"kernel_ms": ms, "launches": n, "wall_ms": wall * 1e3, "updates": u}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--first", type=int, default=5, help="untimed rounds before the timed batch")
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--repeat", type=int, default=1, help="measured batches (the median is reported)")
    ap.add_argument("--fuse", default="16,0", help="replay_fuse values")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    out = []
    for fuse in [int(x) for x in args.fuse.split(",")]:
        e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=min(n * m // 2 + (1 << 20), 1 << 31))
        e.set_option("replay_fuse", fuse)
        for o in args.option:
            name, v = o.split("=")
            e.set_option(name, int(v))
        epoch(e, init_mode, init_param, args.rounds, args.first)  # warm-up
        reps = [epoch(e, init_mode, init_param, args.rounds, args.first) for _ in range(args.repeat)]
        reps.sort(key=lambda x: x["kernel_ms"])
        r = dict(reps[len(reps) // 2])  # the median batch
        r.update({"fuse": fuse, "options": args.option, "rounds": args.rounds, "repeat": args.repeat,
                  "kernel_ms_per_round": r["kernel_ms"] / args.rounds,
                  "kernel_ms_per_round_all": [x["kernel_ms"] / args.rounds for x in reps]})
        print(json.dumps(r), flush=True)
        out.append(r)
        e.close()
    if args.json:
        with open(args.json, "w") as f:
            json.dump({"workload": desc, "runs": out}, f, indent=1)


if __name__ == "__main__":
    main()
