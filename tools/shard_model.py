#!/usr/bin/env python3
"""Multi-GPU projection of the bench window from one-GPU measurements
(DESIGN.md §5). For a workload and the bench window (steps W..W+K-1 of
16-round epochs):

1. the whole network on one engine, one round at a time: kernel ms per round
   (HIP events) and the published words / 64-B row segments that changed
   (option count_changed: the words a peer-push round stores into each peer);
2. for G in 2, 4, 8, rank 0's share alone on this GPU:
   * node shard (N/G nodes, all targets) with option unsynced_shard (no
     exchange; its uniform-rows path runs on its own mismatch slot, as a rank
     of a peer-push run does once the slots are pushed): kernel ms per round;
   * target shard (all nodes, M/G targets): kernel ms per round (no exchange
     exists for it).
Projection per round at G ranks:
   node + peer push: max(node-shard kernel, the rank's pushes: changed
   segments / G * 64 B over one xGMI link per peer) + the barrier's fixed cost;
   target shard: the target-shard kernel.
The barrier's fixed cost per round is --barrier-us (tools/exchange_cost.py
measures it; plus the cross-GPU flag latency, which one GPU cannot show).

    python tools/shard_model.py [--workload c4] [--warmup 5] [--steps 20] [--barrier-us 6] [--json out.json]
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
from avhip import sharding  # noqa: E402
from bench import EPOCH, WORKLOADS, XGMI_LINK_GBS  # noqa: E402


def window_rounds(eng, init, warmup, steps, count_changed=False):
    """Per-round kernel ms (and changed words / segments) over the bench window of fresh epochs."""
    rows = []
    if count_changed:
        eng.set_option("count_changed", 1)
    pos = warmup
    eng.init_records(*init)
    eng.run_rounds(warmup)  # untimed
    eng.synchronize()
    eng.discard_updates()
    for _ in range(steps):
        if pos % EPOCH == 0:
            eng.synchronize()
            eng.discard_updates()
            eng.init_records(*init)
        w0, g0 = eng.changed_words()
        eng.set_timing(True)
        eng.run_rounds(1)
        ms, _ = eng.kernel_stats()
        eng.set_timing(False)
        w1, g1 = eng.changed_words()
        eng.discard_updates()
        rows.append({"round": pos % EPOCH, "ms": ms, "words": w1 - w0, "segments": g1 - g0})
        pos += 1
    if count_changed:
        eng.set_option("count_changed", 0)
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--barrier-us", type=float, default=6.0)
    ap.add_argument("--option", action="append", default=[], help="name=value on the rank-0 share engines")
    ap.add_argument("--kinds", default="nodes,targets")
    ap.add_argument("--no-one-gpu", action="store_true", help="skip the whole-network pass (projections need it)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    N, M, K, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    assert not replay, "sim workloads only"
    init = (init_mode, init_param)
    cap = min(int(1.25 * N * M) + (1 << 20), (1 << 31) - 1)
    if args.no_one_gpu:
        one = [{"round": (args.warmup + i) % EPOCH, "ms": 0.0, "words": 0, "segments": 0} for i in range(args.steps)]
    else:
        e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=cap)
        window_rounds(e, init, args.warmup, args.steps)  # device warm-up
        plain = window_rounds(e, init, args.warmup, args.steps)
        one = window_rounds(e, init, args.warmup, args.steps, count_changed=True)
        e.close()
        for a, b in zip(one, plain):  # kernel time without the counting; words / segments from the counting pass
            a["ms_counting"], a["ms"] = a["ms"], b["ms"]
    t1 = sum(r["ms"] for r in one)
    out = {"workload": desc, "window": f"{args.warmup}+{args.steps}", "one_gpu": one, "one_gpu_ms": t1,
           "link_GBs_per_direction": XGMI_LINK_GBS, "barrier_us": args.barrier_us, "ranks": {}}
    print(json.dumps({"one_gpu_ms": t1}), flush=True)
    for g in [int(x) for x in args.ranks.split(",")]:
        def share(kind):
            kw = dict(node_range=sharding.node_shard(N, g, 0)) if kind == "nodes" else \
                dict(target_range=sharding.target_shard(M, g, 0))
            if kind not in args.kinds.split(","):
                return [{"ms": 0.0} for _ in range(args.steps)]
            en = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=max(1 << 24, cap // g), **kw)
            if kind == "nodes":
                en.set_option("unsynced_shard", 1)
            for o in args.option:
                name, v = o.split("=")
                en.set_option(name, int(v))
            window_rounds(en, init, args.warmup, args.steps)
            rows = window_rounds(en, init, args.warmup, args.steps)
            en.close()
            return rows

        ns, ts = share("nodes"), share("targets")
        per = []
        for a, b, c in zip(one, ns, ts):
            push_ms = a["segments"] / g * 64.0 / (XGMI_LINK_GBS * 1e9) * 1e3
            per.append({"round": a["round"], "node_kernel_ms": b["ms"], "push_ms": push_ms,
                        "node_ms": max(b["ms"], push_ms) + args.barrier_us * 1e-3, "target_ms": c["ms"]})
        tn = sum(p["node_ms"] for p in per)
        tt = sum(p["target_ms"] for p in per)
        eff = (lambda t: t1 / (g * t) if t > 0 and t1 > 0 else None)
        out["ranks"][g] = {"per_round": per, "node_push_ms": tn, "target_ms": tt,
                           "node_push_efficiency": eff(tn), "target_efficiency": eff(tt)}
        print(json.dumps({"g": g, "node_push_ms": tn, "target_ms": tt, "eff_node": eff(tn), "eff_target": eff(tt),
                          "options": args.option}), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
