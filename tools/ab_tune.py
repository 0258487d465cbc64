#!/usr/bin/env python3
"""Interleaved A/B timing of round-kernel variants in ONE process (guide §5.4
rule 24) on the C4 workload, plus the per-GPU kernel time of a target shard
of the same network (what each rank runs at 2/4/8-way target sharding).

    python tools/ab_tune.py [--rounds 6] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))

import torch  # noqa: E402,F401

import avhip  # noqa: E402
from avhip import sharding  # noqa: E402

N, M, K = 1_000_000, 1000, 8
P80 = int(0.8 * 2**32)


def one_round_ms(e):
    e.set_timing(True)
    e.run_rounds(1)
    ms, n = e.kernel_stats()
    e.set_timing(False)
    return ms / max(n, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    out = {}

    # --- A/B: non-temporal planes on/off, consider-plane skip on/off (both engines warm)
    warm = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, log_capacity=1 << 28)
    cold = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, log_capacity=1 << 28)
    for e in (warm, cold):
        e.init_records(avhip.INIT_BERNOULLI, P80)
    cold.set_option("warm_skip", 0)
    for e in (warm, cold):
        e.run_rounds(2)
        e.synchronize()
        try:
            e.fetch_updates(decode=False)
        except avhip.LogOverflow:
            pass
    lanes = warm.layout_info()["lanes"]
    times = {"skip": [], "skip+nt": [], "noskip": [], "noskip+nt": []}
    for _ in range(args.rounds):
        for name, e, nt in (("skip", warm, 0), ("skip+nt", warm, 1), ("noskip", cold, 0), ("noskip+nt", cold, 1)):
            e.set_option("plane_nt", nt)
            times[name].append(one_round_ms(e))
    for name, ts in times.items():
        per_lane = 176 if name.startswith("skip") else 236
        med = statistics.median(ts)
        out[name] = {"median_ms": med, "min_ms": min(ts),
                     "alg_GBs": lanes * per_lane / (med * 1e-3) / 1e9}
    warm.close()
    cold.close()

    # --- per-rank kernel time at G-way target sharding (rank 0's shard, warm), nt on/off interleaved
    for g in (1, 2, 4, 8):
        t0, t1 = sharding.target_shard(M, g, 0)
        e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, target_range=(t0, t1), log_capacity=1 << 27)
        e.init_records(avhip.INIT_BERNOULLI, P80)
        e.run_rounds(2)
        e.synchronize()
        try:
            e.fetch_updates(decode=False)
        except avhip.LogOverflow:
            pass
        variants = {"": (0, 0), "+nt": (1, 0), "+nt+ablate_gather": (1, 1)}
        ts = {v: [] for v in variants}
        b0 = e.alg_bytes()
        for _ in range(args.rounds):
            for v, (nt, abl) in variants.items():
                e.set_option("plane_nt", nt)
                e.set_option("ablate_gather", abl)
                ts[v].append(one_round_ms(e))
        e.set_option("ablate_gather", 0)
        bpl = (e.alg_bytes() - b0) / (len(variants) * args.rounds)
        for v in variants:
            med = statistics.median(ts[v])
            out[f"shard{g}{v}"] = {
                "targets": [t0, t1], "median_ms": med, "alg_GBs": bpl / (med * 1e-3) / 1e9,
                "updates_per_s_per_gpu": N * (t1 - t0) * K / (med * 1e-3)}
        e.close()
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
