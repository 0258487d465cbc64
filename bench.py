#!/usr/bin/env python3
"""Throughput bench of the batched Avalanche vote-record update path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

One *step* = one synchronous round of go-avalanche's poll loop for every
simulated node: k peers sampled per node, k Responses
registered, VoteRecord updates (vote.go:54-91) and StatusUpdate emission
(processor.go:111). Inputs (records, preferences, replayed votes) are resident
in HBM before the timed region starts.

metric : vote-record updates/s = regsiterVote applications on live records
         (vote.go:54) per second, whole job (all ranks). triples/s (node, target,
         round) = updates/s / k is reported beside it.
workload : C4 of BASELINE.json (the north_star's 1M nodes x 1k targets) — k=8,
         IsAccepted() ~ Bernoulli(0.8), honest, synthetic (seeded), rounds
         W..W+K-1 (< 17: every record stays live). With N GPUs the same network
         is split by target blocks (no per-round exchange; strong scaling) or,
         with --shard nodes, by nodes with an RCCL all-gather of the published
         preferences every round. At N=1 the line also carries configs[1] (C2:
         replayed vote streams, 4096 poll cap binding) under "secondary".
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (device plumbing + torch.distributed only)
import torch.distributed as dist  # noqa: E402

import avhip  # noqa: E402
from avhip import sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
P80 = int(0.8 * 2**32)
BYZ20 = int(0.2 * 2**32)

WORKLOADS = {
    # name: (nodes, targets, k, init_mode, init_param, byz_threshold, replay, description)
    "c4": (1_000_000, 1000, 8, avhip.INIT_BERNOULLI, P80, 0, False,
           "C4: 1M nodes x 1000 targets, k=8, Bernoulli(0.8) initial acceptance, honest, sim mode"),
    "c2": (1000, 10_000, 8, avhip.INIT_BERNOULLI, 0x80000000, 0, True,
           "C2: 1k nodes x 10k targets, k=8, replayed vote streams (70/25/5 yes/no/neutral), 4096 poll cap binds"),
    "c3": (100_000, 2000, 8, avhip.INIT_PAIRS, 0, BYZ20, False,
           "C3: 100k nodes x 1000 double-spend pairs, k=8, 20% Byzantine flip-flop voters"),
    "c5": (10_000_000, 256, 8, avhip.INIT_BERNOULLI, P80, 0, False,
           "C5: 10M nodes x 256 targets, k=8, Bernoulli(0.8), honest"),
}


PARALLELISM = {
    "peers": "node-sharded, changed preference words pushed to peers over xGMI + device barrier per round",
    "nodes": "node-sharded, RCCL all-gather of preference rows per round",
    "targets": "target-sharded, no exchange",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=14)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    # peers: node shards + peer-push exchange; nodes: node shards +
    # RCCL all-gather of the preference rows; targets: target shards, no exchange
    ap.add_argument("--shard", default="peers", choices=["peers", "targets", "nodes"])
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xA7A1A9C4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--plane-nt", type=int, default=None, help="override the plane_nt tuning option")
    ap.add_argument("--kernel", type=int, default=None, choices=[1, 2],
                    help="round kernel generation (A/B only; default: the engine's choice)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank on device 0, gloo for the host-side "
                         "barrier/reductions (target sharding only; not a measurement)")
    return ap.parse_args()


def cpu_baseline(wl, seed, budget_s):
    """Oracle ("port": C restatement of the reference semantics) on host cores,
    on a bounded sample of the same workload: fewer nodes, same targets/k."""
    from oracle import cabi

    n, m, k, init_mode, init_param, byz, replay, _ = WORKLOADS[wl]
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    threads = max(1, min(threads, 16))
    ns = min(n, 80000 if wl != "c2" else 400)
    sim = cabi.Sim(ns, m, k, seed=seed, byz_threshold=byz, init_mode=init_mode, init_param=init_param)
    applied = 0
    dt = 0.0
    rounds = 0
    while dt < budget_s and rounds < 16:
        errs = cabi.gen_replay_errs(seed, rounds, 0, ns, m, k) if replay else None  # input, untimed
        ts = time.perf_counter()
        _, a = sim.run_round(errs, threads=threads)
        dt += time.perf_counter() - ts
        applied += a
        rounds += 1
    sim.close()
    return {"value": applied / dt, "unit": "vote-record updates/s", "cores": threads, "kind": "port",
            "sample": f"oracle/avalanche_oracle.c Sim, {ns} nodes x {m} targets, k={k}, {rounds} rounds "
                      f"({applied} regsiterVote applications, {dt:.1f}s, OpenMP over nodes)"}


def measure(wl, args, world, rank, local_rank, steps, warmup):
    """Build the workload's engine (this rank's shard), run `warmup` untimed and
    `steps` timed rounds; return whole-job numbers (max time, summed work) and
    rank-local kernel numbers."""
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[wl]
    if args.shard == "targets" and world > 1 and m > 4096:
        raise SystemExit("target sharding needs M <= 4096 (poll cap couples targets); use --shard nodes")
    kw = dict(k=k, seed=args.seed, byz_threshold=byz, device=local_rank)
    if world > 1 and args.shard == "targets":
        kw["target_range"] = sharding.target_shard(m, world, rank)
    elif world > 1:
        kw["node_range"] = sharding.node_shard(n, world, rank)
    # StatusUpdates per timed round reach ~15% of the records under C3's flip-flop voters
    est_updates = int((1.0 if byz else 0.25) * n * m) + (1 << 20)
    eng = avhip.Engine(n, m, log_capacity=min(est_updates, 1 << 29), **kw)
    if args.plane_nt is not None:
        eng.set_option("plane_nt", args.plane_nt)
    if args.kernel is not None:
        eng.set_option("kernel", args.kernel)
    eng.init_records(init_mode, init_param)
    if world > 1 and args.shard == "nodes":
        obj = [avhip.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(world, rank, obj[0])
    elif world > 1 and args.shard == "peers":
        # map every rank's preference snapshots (IPC over xGMI); if any rank
        # cannot, every rank falls back to target sharding (same network)
        blobs = [None] * world
        dist.all_gather_object(blobs, eng.peer_handles())
        err = None
        try:
            eng.peer_init(world, rank, blobs)
        except avhip.AvError as ex:
            err = repr(ex)[:200]
        errs = [None] * world
        dist.all_gather_object(errs, err)
        if any(errs):
            eng.close()
            args.shard = "targets"
            args.shard_fallback = next(e for e in errs if e)
            return measure(wl, args, world, rank, local_rank, steps, warmup)
    if replay:  # both passes' rounds (the roofline pass re-runs warmup + steps)
        eng.replay_prepare(3 * (warmup + steps))
    run = eng.replay_rounds if replay else eng.run_rounds
    info = eng.layout_info()

    # ---- device warm-up (untimed): after process start the GPU runs these
    # kernels up to ~15 % slower for the first ~20-30 ms of sustained load,
    # whatever the launch pattern (tools/gap_probe.py --events-first, DESIGN.md
    # §4); one untimed pass of the same rounds, then the records start over
    run(warmup + steps)
    eng.synchronize()
    eng.discard_updates()
    eng.init_records(init_mode, init_param)

    # ---- warmup (untimed), then empty the StatusUpdate log. Discarded on the
    # device, not fetched: sorting round 0-1's ~10^8 updates on the host took
    # ~4.7 s, long enough for the idle GPU to lose the warm-up above (the timed
    # rounds then ran at 0.70-0.82 ms instead of 0.65; profiles/r01 trace)
    run(warmup)
    eng.synchronize()
    eng.discard_updates()
    applied0 = eng.applied_votes()

    # ---- timed region (no per-launch events: their queue packets add ~10 us between kernels)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(steps)
    eng.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log_overflow = eng.log_overflowed()  # updates past the device log's capacity were counted, not stored
    applied = eng.applied_votes() - applied0
    emitted = eng.updates_count()

    # ---- roofline pass: the same work again (records re-initialized, warmup,
    # `steps` rounds), every launch bracketed by HIP events on the engine's stream
    eng.discard_updates()
    eng.init_records(init_mode, init_param)
    run(warmup)
    eng.synchronize()
    eng.discard_updates()
    bytes1 = eng.alg_bytes()
    eng.set_timing(True)
    run(steps)
    eng.synchronize()
    eng.set_timing(False)
    kern_ms, launches = eng.kernel_stats()
    # algorithmic bytes per launch, counted by the round kernel itself (planes
    # actually streamed, gathered vote words, published words, StatusUpdates)
    alg_bytes = (eng.alg_bytes() - bytes1) / max(launches, 1)
    kavg_ms = kern_ms / max(launches, 1)
    replicas = None
    if world > 1 and args.shard in ("peers", "nodes"):
        # every rank's replica of the published preferences must be the same:
        # hash a slice of every rank's node range as this rank sees it
        import hashlib

        hs = hashlib.sha256()
        for r in range(world):
            a = sharding.node_shard(n, world, r)[0]
            hs.update(eng.read_pref(a, min(a + 2048, n)).tobytes())
        digests = [None] * world
        dist.all_gather_object(digests, hs.hexdigest())
        replicas = len(set(digests)) == 1
    eng.close()

    if world > 1:
        st = torch.tensor([elapsed, float(applied), float(emitted)], dtype=torch.float64,
                          device="cpu" if args.rehearse_one_gpu else "cuda")
        tmax = st[0:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tot = st[1:3].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, applied, emitted = float(tmax), float(tot[0]), float(tot[1])
    value = applied / elapsed
    # roofline of this rank's round kernel: algorithmic bytes per
    # launch as counted by the kernel (per 32-record lane at k=8: 236 B cold,
    # 172 B warm, 136 B with recomputed vote registers; + the StatusUpdate log)
    # / its HIP-event average launch time.
    achieved = alg_bytes / (kavg_ms * 1e-3) / 1e9
    gen2 = k <= 8 and args.kernel != 1
    kname = (("k_round_node" if gen2 else "k_round_capped") if info["capped"]
             else ("k_round_sweep" if gen2 else "k_round_fast")) + f"<{k},{'true' if replay else 'false'}>"
    return {
        "desc": desc, "n": n, "m": m, "k": k, "value": value, "elapsed": elapsed, "applied": applied,
        "emitted": emitted, "info": info, "kavg_ms": kavg_ms, "alg_bytes": alg_bytes, "achieved": achieved,
        "kernel": kname, "log_overflow": log_overflow, "replicas_identical": replicas,
    }


def allgather_probe(world, local_rank, total_bytes=1_000_000 * 128, reps=5):
    per = total_bytes // world // 4 * 4
    src = torch.ones(per // 4, dtype=torch.int32, device=f"cuda:{local_rank}")
    dst = torch.empty(world * (per // 4), dtype=torch.int32, device=f"cuda:{local_rank}")
    dist.all_gather_into_tensor(dst, src)  # warm
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        dist.all_gather_into_tensor(dst, src)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local_rank}")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t)
    inbound = per * (world - 1)
    return {"bytes_total": per * world, "ms": dt * 1e3, "inbound_GBs_per_gpu": inbound / dt / 1e9,
            "note": "C4 node-sharded round exchange (1M x 1000 bits), torch.distributed all_gather_into_tensor"}


def roofline(r, traffic=None):
    return {"bound": "hbm", "achieved": r["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": r["achieved"] / HBM_PEAK_GBS, "traffic": traffic, "kernel": r["kernel"],
            "kernel_ms_avg": r["kavg_ms"], "alg_bytes_per_launch": r["alg_bytes"]}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse_one_gpu:
        if args.shard == "nodes":
            raise SystemExit("--rehearse-one-gpu: not with --shard nodes (RCCL needs distinct GPUs)")
        local_rank = 0
    torch.cuda.set_device(local_rank)
    if world > 1 and args.rehearse_one_gpu:
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))

    r = measure(args.workload, args, world, rank, local_rank, args.steps, args.warmup)
    secondary = None
    if world > 1 and not args.rehearse_one_gpu and not args.no_secondary:
        # the exchange a node-sharded C4 round would need: every rank's published-
        # preference rows (N/G x 128 B) all-gathered over xGMI (RCCL through
        # torch.distributed); recorded for the node- vs target-sharding choice
        # (DESIGN.md §5), not part of the timed value
        try:
            secondary = {"xgmi_allgather": allgather_probe(world, local_rank)}
        except Exception as exc:  # a diagnostic: never costs the measured line
            secondary = {"xgmi_allgather": {"error": repr(exc)[:200]}}
    if world == 1 and not args.no_secondary and args.workload != "c2":
        c2 = measure("c2", args, world, rank, local_rank, 14, 2)
        secondary = {"c2": {"workload": c2["desc"], "value": c2["value"], "unit": "vote-record updates/s",
                            "ms_per_step": c2["elapsed"] / 14 * 1e3, "rounds": "2..15",
                            "roofline": roofline(c2)}}

    if rank == 0:
        traffic = None
        pmc_path = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.workload}.json")
        if world == 1 and os.path.exists(pmc_path):
            with open(pmc_path) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        line = {
            "metric": "vote-record updates/sec (node·target·round) at 1/2/4/8 GPU; % HBM roofline",
            "value": r["value"],
            "unit": "vote-record updates/s (1 update = 1 regsiterVote on a live record; k=8 per node·target·round)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "device_warmup_rounds": args.warmup + args.steps,
            "ms_per_step": r["elapsed"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded Philox4x32-10 network; no dataset)",
            "config": {
                "workload": r["desc"],
                "n_nodes": r["n"], "n_targets": r["m"], "k": r["k"],
                "rounds": f"{args.warmup}..{args.warmup + args.steps - 1}",
                "parallelism": (PARALLELISM[args.shard] + f" x{world}") if world > 1 else "single GPU",
                "layout": "bit-sliced: 25 u32 planes per 32 records; tile of 64 lanes contiguous",
                "capped_poll_path": r["info"]["capped"],
            },
            "triples_per_s": r["value"] / r["k"],
            "updates_emitted": int(r["emitted"]),
            "update_log_overflow": r["log_overflow"],
            "roofline": roofline(r, traffic),
        }
        if r["replicas_identical"] is not None:
            line["config"]["replicas_identical"] = r["replicas_identical"]
        if getattr(args, "shard_fallback", None):
            line["config"]["shard_fallback"] = "peer exchange unavailable: " + args.shard_fallback
        if secondary:
            line["secondary"] = secondary
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(args.workload, args.seed, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
