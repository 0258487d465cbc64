#!/usr/bin/env python3
"""Multi-GPU decompositions of the bench window, measured rank by rank on one
MI355X and projected to G GPUs.

For a workload and the bench window (steps W..W+K-1 of 16-round epochs):

* one GPU, the whole network: kernel ms per round (HIP events);
* for each G and decomposition, every rank of the decomposition as an engine
  of this process on this GPU, all ranks of an exchange in one serial peer
  group (av_peer_group_serial: each rank's round kernel pushes into the other
  ranks' buffers exactly as over xGMI; the stream's order replaces the
  barrier), so that a rank's kernel time is that of the rank alone on a GPU and
  every result is exact (the group is the network):
    - targets  : target shards (no exchange), rank 0 alone;
    - nodes    : node shards, every changed word pushed to every peer;
    - masked   : node shards, need-masked pushes (engine option peer_mask);
    - 2d GnxGt : Gt target shards, each split in Gn node shards with the
                 need-masked exchange inside its column (rank (0, t) group).
  per round and rank: kernel ms (for the exchanges it includes the pushes,
  stored into this GPU's memory, and the need-window work) and words pushed
  (av_pushed_words, all peers).
Projection of a round at G GPUs: max over ranks of max(kernel ms, the rank's
busiest link: pushed words / peers * 4 B / XGMI_LINK_GBS) + the barrier's fixed
cost (--barrier-us, tools/exchange_cost.py); the pushes are issued inside the
round kernel, so link time and kernel time overlap. Efficiency = one-GPU window
ms / (G * projected window ms).

    python tools/group_model.py [--workload c4] [--ranks 2,4,8] [--kinds targets,nodes,masked,2d] [--json out]
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
from avhip import sharding  # noqa: E402
from bench import EPOCH, WORKLOADS, XGMI_LINK_GBS  # noqa: E402

SEED = 0xA7A1A9C4


def log_cap(n, m):
    # one round's updates at a time (discarded after every round): ~0.1 per record in a storm round
    return min(int(0.3 * n * m) + (1 << 20), (1 << 31) - 1)


def window(engs, init, warmup, steps, on_round):
    """Run the bench window on a list of engines that step together (a serial peer group in rank
    order, or a single engine): untimed warmup, then `steps` rounds, each timed per engine."""
    def reinit():
        for e in engs:
            e.synchronize()
            e.discard_updates()
        for e in engs:
            e.init_records(*init)
    pos = warmup
    reinit()
    for _ in range(warmup):
        for e in engs:
            e.run_rounds(1)
        for e in engs:
            e.synchronize()
            e.discard_updates()
    for e in engs:
        e.set_timing(True)
        e.kernel_stats()
    for _ in range(steps):
        if pos % EPOCH == 0:
            for e in engs:
                e.set_timing(False)
            reinit()
            for e in engs:
                e.set_timing(True)
        p0 = [e.pushed_words() if len(engs) > 1 else 0 for e in engs]
        for e in engs:
            e.run_rounds(1)
        ms = [e.kernel_stats()[0] for e in engs]
        p1 = [e.pushed_words() if len(engs) > 1 else 0 for e in engs]
        for e in engs:
            e.discard_updates()
        on_round(pos % EPOCH, ms, [b - a for a, b in zip(p0, p1)])
        pos += 1
    for e in engs:
        e.set_timing(False)


ALL_OPTIONS = []  # --all-option: set on every engine (one-GPU, target shards, groups)


def run_single(n, m, k, byz, init, warmup, steps, options=(), **kw):
    e = avhip.Engine(n, m, k=k, seed=SEED, byz_threshold=byz, log_capacity=log_cap(kw.get("nl", n), m), **{
        k2: v for k2, v in kw.items() if k2 != "nl"})
    for name, v in list(ALL_OPTIONS) + list(options):
        e.set_option(name, v)
    rows = []
    window([e], init, warmup, steps, lambda r, ms, pw: None)  # device warm-up
    window([e], init, warmup, steps, lambda r, ms, pw: rows.append({"round": r, "ms": ms[0]}))
    e.close()
    return rows


def run_group(n, m, k, byz, init, warmup, steps, g, mask, t_range=None, options=()):
    per = n // g
    engs = []
    for r in range(g):
        kw = dict(node_range=(r * per, (r + 1) * per))
        mm = m
        if t_range is not None:  # 2-D: this column's target shard as a network of its own width
            mm = t_range[1] - t_range[0]
        engs.append(avhip.Engine(n, mm, k=k, seed=SEED, byz_threshold=byz, log_capacity=log_cap(per, mm), **kw))
    for e in engs:
        e.set_option("peer_mask", mask)
        for name, v in list(ALL_OPTIONS) + list(options):
            e.set_option(name, v)
        e.init_records(*init)
    avhip.peer_group_serial(engs)
    rows = []
    window(engs, init, warmup, steps, lambda r, ms, pw: None)
    window(engs, init, warmup, steps, lambda r, ms, pw: rows.append({"round": r, "ms": ms, "pushed": pw}))
    for e in engs:
        e.close()
    return rows


def project(rows, peers, barrier_us):
    out = []
    for row in rows:
        per_rank = []
        for ms, pw in zip(row["ms"], row["pushed"]):
            link = (pw / peers * 4.0 / (XGMI_LINK_GBS * 1e9) * 1e3) if peers else 0.0
            per_rank.append(max(ms, link))
        out.append({"round": row["round"], "kernel_ms_max": max(row["ms"]),
                    "link_ms_max": max((pw / peers * 4.0 / (XGMI_LINK_GBS * 1e9) * 1e3) if peers else 0.0
                                       for pw in row["pushed"]),
                    "pushed_words": sum(row["pushed"]),
                    "ms": max(per_rank) + (barrier_us * 1e-3 if peers else 0.0)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--kinds", default="targets,nodes,masked,2d")
    ap.add_argument("--barrier-us", type=float, default=6.0)
    ap.add_argument("--target-option", action="append", default=[],
                    help="name=value on the target-shard engines (an extra 'targets+' row)")
    ap.add_argument("--variant", action="append", default=[],
                    help="name:opt=v,opt=v -- an extra masked node-shard row with engine options (A/B)")
    ap.add_argument("--all-option", action="append", default=[],
                    help="name=value on every engine, e.g. warm_pref=1: each rank's gather sources read "
                         "(untimed) before its timed kernel, as its own GPU's caches would hold them")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    ALL_OPTIONS.extend((o.split("=")[0], int(o.split("=")[1])) for o in args.all_option)
    topts = [(o.split("=")[0], int(o.split("=")[1])) for o in args.target_option]
    N, M, K, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    assert not replay, "sim workloads only"
    init = (init_mode, init_param)
    kinds = args.kinds.split(",")
    t0 = time.time()
    one = run_single(N, M, K, byz, init, args.warmup, args.steps)
    t1 = sum(r["ms"] for r in one)
    out = {"workload": desc, "window": f"{args.warmup}+{args.steps}", "all_options": args.all_option, "one_gpu": one, "one_gpu_ms": t1,
           "link_GBs_per_direction": XGMI_LINK_GBS, "barrier_us": args.barrier_us, "ranks": {},
           "model": "round = max over ranks of max(kernel ms, busiest link ms) + barrier; link ms = words pushed "
                    "/ peers * 4 B / link GB/s (one xGMI link per peer, pushes overlap the kernel)"}
    print(json.dumps({"one_gpu_ms": t1, "s": round(time.time() - t0, 1)}), flush=True)

    def record(g, name, rows_proj, extra=None):
        tot = sum(r["ms"] for r in rows_proj)
        ent = {"ms": tot, "efficiency": t1 / (g * tot) if tot > 0 else None, "per_round": rows_proj}
        if extra:
            ent.update(extra)
        out["ranks"].setdefault(str(g), {})[name] = ent
        print(json.dumps({"g": g, "kind": name, "ms": round(tot, 4), "eff": round(ent["efficiency"], 3),
                          "s": round(time.time() - t0, 1)}), flush=True)
        if args.json:
            with open(args.json, "w") as f:
                json.dump(out, f, indent=1)

    for g in [int(x) for x in args.ranks.split(",")]:
        if "targets" in kinds:
            rows = run_single(N, M, K, byz, init, args.warmup, args.steps,
                              target_range=sharding.target_shard(M, g, 0))
            record(g, "targets", [{"round": r["round"], "ms": r["ms"], "kernel_ms_max": r["ms"]} for r in rows])
            if topts:
                rows = run_single(N, M, K, byz, init, args.warmup, args.steps, options=topts,
                                  target_range=sharding.target_shard(M, g, 0))
                record(g, "targets+" + ",".join(args.target_option),
                       [{"round": r["round"], "ms": r["ms"], "kernel_ms_max": r["ms"]} for r in rows])
        for name, mask in (("nodes", 0), ("masked", 1)):
            if name in kinds and N % g == 0:
                rows = run_group(N, M, K, byz, init, args.warmup, args.steps, g, mask)
                record(g, name, project(rows, g - 1, args.barrier_us))
        for var in args.variant:
            vname, vopts = var.split(":")
            opts = [(o.split("=")[0], int(o.split("=")[1])) for o in vopts.split(",") if o]
            if N % g == 0:
                rows = run_group(N, M, K, byz, init, args.warmup, args.steps, g, 1, options=opts)
                record(g, "masked+" + vname, project(rows, g - 1, args.barrier_us))
        if "2d" in kinds and g >= 4:
            for gn in (2, 4) if g == 8 else (2,):
                gt = g // gn
                tr = sharding.target_shard(M, gt, 0)
                rows = run_group(N, M, K, byz, init, args.warmup, args.steps, gn, 1, t_range=tr)
                record(g, f"2d_{gn}x{gt}", project(rows, gn - 1, args.barrier_us),
                       {"note": f"{gn} node shards x {gt} target shards; rank (0, 0)'s column, masked exchange "
                                f"over {gn - 1} link(s) per rank"})
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
