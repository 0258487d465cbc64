#!/usr/bin/env python3
"""Run a BASELINE config until every honest node has finalized every target
(or a round limit), one GPU, and report rounds-to-finalization plus the
per-round kernel throughput.

    python tools/run_to_finalization.py --workload c3 [--max-rounds 512] [--json out.json]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c3", choices=["c3", "c4", "c5"])
    ap.add_argument("--max-rounds", type=int, default=512)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xA7A1A9C4)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    assert not replay
    # log sized for the heaviest round (every record can emit up to 2 updates per round at k=8);
    # capped at 2^31 entries (16 GB) — a round beyond that is reported as overflow
    log_cap = min(2 * n * m + (1 << 20), 1 << 31)
    e = avhip.Engine(n, m, k=k, seed=args.seed, byz_threshold=byz, log_capacity=log_cap)
    e.init_records(init_mode, init_param)
    honest_records = e.live_records(honest_only=True)
    per_round = []
    t_start = time.perf_counter()
    done_round = None
    for r in range(args.max_rounds):
        a0, f0 = e.applied_votes(), e.finalized_count()
        e.set_timing(True)
        e.run_rounds(1)
        ms, _ = e.kernel_stats()
        e.set_timing(False)
        emitted = e.updates_count()  # StatusUpdates this round (log sized for the heaviest round)
        e.discard_updates()  # convergence only needs the counters
        live = e.live_records(honest_only=True)
        per_round.append({"round": r, "kernel_ms": ms, "applied": e.applied_votes() - a0,
                          "finalized": e.finalized_count() - f0, "emitted": emitted, "honest_live": live})
        if live == 0:
            done_round = r
            break
    wall = time.perf_counter() - t_start
    total_applied = e.applied_votes()
    kern = sum(x["kernel_ms"] for x in per_round)
    out = {
        "workload": desc,
        "n_nodes": n, "n_targets": m, "k": k,
        "honest_records": honest_records,
        "rounds_to_finalization": None if done_round is None else done_round + 1,
        "rounds_run": len(per_round),
        "honest_live_at_end": per_round[-1]["honest_live"],
        "applied_votes": total_applied,
        "kernel_ms_total": kern,
        "updates_per_s_kernel": total_applied / (kern * 1e-3) if kern else None,
        "wall_s": wall,
        "per_round": per_round,
    }
    print(json.dumps({k_: v for k_, v in out.items() if k_ != "per_round"}, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
