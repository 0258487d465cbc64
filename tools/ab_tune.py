#!/usr/bin/env python3
"""Interleaved A/B timing of round-kernel variants in ONE process (guide §5.4
rule 24) on the C4 workload, and the per-GPU kernel time of a target shard of
the same network (what each rank runs at 2/4/8-way target sharding).

    python tools/ab_tune.py [--rounds 6] [--json out.json] [--variants sweep,per_tile,...]

Variants: sweep (k_round_sweep, persistent grid), sweep_w1 (sweep kernel,
one wave per tile), per_tile (k_round_fast), ablate (sweep, peer gather
replaced by a coalesced read: timing only, results invalid).
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

sys.path.insert(0, ROOT)
from bench import WORKLOADS  # noqa: E402

VARIANTS = {
    "sweep": dict(kernel=2),
    "sweep_w1": dict(kernel=2, sweep_blocks=0),
    "sweep_res": dict(kernel=2, sweep_blocks=-2),
    "per_tile": dict(kernel=1),
    "ablate": dict(kernel=2, ablate_gather=1),
    "w1_sc1": dict(kernel=2, sweep_blocks=0, store_policy=2),
    "w1_ntsc1": dict(kernel=2, sweep_blocks=0, store_policy=3),
    "res_sc1": dict(kernel=2, sweep_blocks=-2, store_policy=2),
    "w1_plain": dict(kernel=2, sweep_blocks=0, plane_nt=0),
    "vv0": dict(kernel=2, virtual_votes=0),
    "vv_all": dict(kernel=2, vv_min_bl=1),
    "kl0": dict(kernel=2, count_lazy=0),
}


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
    ap.add_argument("--variants", default="sweep,sweep_w1,per_tile,ablate")
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    args = ap.parse_args()
    N, M, K, init_mode, init_param, byz, replay, _ = WORKLOADS[args.workload]
    assert not replay, "sim-mode workloads only"
    names = args.variants.split(",")
    out = {}
    for g in [int(x) for x in args.shards.split(",")]:
        t0, t1 = sharding.target_shard(M, g, 0)
        # one engine per variant, all at the same round with the same state
        # (rounds 2.. stay below 15: no record can finalize, every tile is warm)
        engs = {}
        for v in names:
            e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz, target_range=(t0, t1),
                             log_capacity=1 << 27)
            opts = VARIANTS[v]
            e.set_option("kernel", opts["kernel"])
            e.set_option("ablate_gather", opts.get("ablate_gather", 0))
            for opt in ("sweep_blocks", "store_policy", "plane_nt", "virtual_votes", "vv_min_bl", "count_lazy"):
                if opt in opts:
                    e.set_option(opt, opts[opt])
            e.init_records(init_mode, init_param)
            e.run_rounds(2)
            e.synchronize()
            e.discard_updates()
            engs[v] = e
        lanes = engs[names[0]].layout_info()["lanes"]
        ts = {v: [] for v in names}
        bpl = {}
        for _ in range(min(args.rounds, 12)):
            for v, e in engs.items():
                b0 = e.alg_bytes()
                ts[v].append(one_round_ms(e))
                bpl[v] = (e.alg_bytes() - b0) / lanes
                e.discard_updates()
        for v in names:
            med = statistics.median(ts[v])
            out[f"{args.workload}_shard{g}_{v}"] = {
                "targets": [t0, t1], "median_ms": med, "min_ms": min(ts[v]),
                "alg_GBs": bpl[v] * lanes / (med * 1e-3) / 1e9, "alg_bytes_per_lane": bpl[v],
                "updates_per_s_per_gpu": N * (t1 - t0) * K / (med * 1e-3)}
        for e in engs.values():
            e.close()
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
