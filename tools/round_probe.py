#!/usr/bin/env python3
"""One epoch of a BASELINE workload on one GPU, round by round: per-round
round-kernel time (HIP events), applied votes and StatusUpdates. Run it under
rocprofv3 (--kernel-trace / --pmc) to attribute counters to rounds: after the
init kernels, the i-th round-kernel dispatch is round i (write-back passes
named k_kl_materialize / k_vv_materialize sit between them).

    python tools/round_probe.py --workload c4 --rounds 16 [--option name=value ...] [--json out.json]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import avhip  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    ap.add_argument("--rounds", type=int, default=16)
    ap.add_argument("--warm-epochs", type=int, default=1, help="untimed epochs first (device clock warm-up)")
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xA7A1A9C4)
    ap.add_argument("--json", default=None)
    ap.add_argument("--nodes", type=int, default=None, help="override the workload's node count (size scaling)")
    args = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    if args.nodes:
        n = args.nodes
    e = avhip.Engine(n, m, k=k, seed=args.seed, byz_threshold=byz, log_capacity=min(n * m // 2 + (1 << 20), 1 << 31))
    for o in args.option:
        name, v = o.split("=")
        e.set_option(name, int(v))
    lanes = e.layout_info()["lanes"]
    for _ in range(args.warm_epochs):
        e.init_records(init_mode, init_param)
        if replay:
            e.replay_prepare(args.rounds)
            e.replay_rounds(args.rounds)
        else:
            e.run_rounds(args.rounds)
        e.synchronize()
        e.discard_updates()
    e.init_records(init_mode, init_param)
    if replay:
        e.replay_prepare(args.rounds)
    rows = []
    for r in range(args.rounds):
        a0, b0 = e.applied_votes(), e.alg_bytes()
        e.set_timing(True)
        if replay:
            e.replay_rounds(1)
        else:
            e.run_rounds(1)
        ms, _ = e.kernel_stats()
        e.set_timing(False)
        u = e.updates_count()
        e.discard_updates()
        rows.append({"round": r, "kernel_ms": ms, "applied": e.applied_votes() - a0, "updates": u,
                     "bytes_per_lane": (e.alg_bytes() - b0) / lanes})
        print(json.dumps(rows[-1]), flush=True)
    out = {"workload": desc, "lanes": lanes, "tiles": (lanes + 63) // 64, "options": args.option, "rounds": rows,
           "kernel_ms_total": sum(x["kernel_ms"] for x in rows)}
    print(json.dumps({k_: v for k_, v in out.items() if k_ != "rounds"}))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
