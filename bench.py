#!/usr/bin/env python3
"""Throughput bench of the batched Avalanche vote-record update path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c2|c3|c5|c4p|c4pb]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

`python bench.py --gpus N` (N > 1) with no launcher around it starts its own N
rank processes: a fresh `python -m torch.distributed.run` child (before any GPU
call), whose rank 0 prints the line; the exit status is the child's.

One *step* = one synchronous round of go-avalanche's poll loop for every
simulated node: k peers sampled per node, k Responses
registered, VoteRecord updates (vote.go:54-91) and StatusUpdate emission
(processor.go:111). Inputs (records, preferences, replayed votes) are resident
in HBM before the timed region starts.

metric : vote-record updates/s = regsiterVote applications on live records
         (vote.go:54) per second, whole job (all ranks). triples/s (node, target,
         round) = updates/s / k is reported beside it.
workload : C4 of BASELINE.json (the north_star's 1M nodes x 1k targets) — k=8,
         IsAccepted() ~ Bernoulli(0.8), honest, synthetic (seeded).
window : BASELINE.md fixes C4 at its all-live rounds (no record can finalize
         before round 16 at k = 8: 7 warm-up votes + 128 agreeing ones). The
         step sequence is therefore a chain of 16-round *epochs*: step p is
         round p % 16 of a fresh network, the records re-initialised (untimed,
         outside the timed segments) at every epoch start. `--warmup W` runs
         steps 0..W-1 untimed, `--steps K` times steps W..W+K-1 — whatever W
         and K are, every timed round has every record live. A timed stretch
         that crosses an epoch boundary is timed as two segments, each
         bracketed by barrier + synchronize; their times add up.
         Every StatusUpdate of the timed rounds is stored in the device log
         (sized for the window); an overflow is a hard failure (exit 3, no
         number printed).
multi-GPU : N ranks split the same network (strong scaling): target shards
         (default: no exchange at all), or node shards with the
         peer-push exchange or an RCCL all-gather (`--shard peers|nodes`).

The line carries the round kernel's roofline: SURVEY.md
§8(d)'s algorithmic bytes per launch (9.125 B per live (node, target, round)
+ 20 B per StatusUpdate) over the kernel's HIP-event time, the bytes the
bit-sliced kernel actually moves, and — from the committed rocprofv3 PMC
summary of this bench window and these kernel sources, when it matches — the
HBM traffic and the instruction-issue fractions that bind the round.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402  (device plumbing + torch.distributed only)
import torch.distributed as dist  # noqa: E402

import numpy as np  # noqa: E402

import avhip  # noqa: E402
from avhip import sharding  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
P80 = int(0.8 * 2**32)
BYZ20 = int(0.2 * 2**32)
EPOCH = 16  # all-live rounds of a fresh network at k = 8 (finalization needs >= 134 votes)
S8D_TRIPLE_BYTES = {False: 9.125, True: 10.125}  # sim / replay, per live (node, target, round)
S8D_UPDATE_BYTES = 20.0                           # per emitted StatusUpdate

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
    # the north star's "1M nodes x 1k conflicting targets": 500 double-spend pairs per node with
    # complementary initial IsAccepted, honest / 20 % Byzantine flip-flop voters
    "c4p": (1_000_000, 1000, 8, avhip.INIT_PAIRS, 0, 0, False,
            "C4p: 1M nodes x 1000 targets as 500 conflicting double-spend pairs, k=8, honest"),
    "c4pb": (1_000_000, 1000, 8, avhip.INIT_PAIRS, 0, BYZ20, False,
             "C4pb: 1M nodes x 500 double-spend pairs, k=8, 20% Byzantine flip-flop voters"),
}

# --shard auto (the default): the decomposition tools/group_model.py measured best per workload and
# rank count (profiles/r05/s7): target shards, except the conflicting workloads at 8
# ranks, whose rounds all change their rows: node shards with the need-masked peer push
AUTO_SHARD = {8: {"c4p": "peers", "c4pb": "peers"}}


def shard_for(wl, world, requested):
    if requested != "auto":
        return requested
    if world <= 1:
        return "targets"
    return AUTO_SHARD.get(world, {}).get(wl, "targets")


NODE_SHARD_TPW = {"c4p": 8, "c4pb": 8}


def eng_tpw_set(args):
    return getattr(args, "tiles_per_wave", None) is not None


PARALLELISM = {
    "peers": "node-sharded, changed preference words pushed to peers over xGMI + device barrier per round",
    "nodes": "node-sharded, RCCL all-gather of preference rows per round",
    "targets": "target-sharded, no exchange",
}

KERNEL_SRC = [os.path.join(ROOT, "go-avalanche_amd", "csrc", f) for f in
              ("round_sweep.hip", "round_node.hip", "kernels.hip", "log_ops.hip", "round_common.h", "round_slots.h",
               "kernels.h", "dev_scan.h", "engine.cpp")]


class BenchFailure(SystemExit):
    pass


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=sorted(WORKLOADS))
    # targets: target shards, no exchange (default: DESIGN.md §5 measures it ahead of the node
    # shards at G = 2 and 4, even at 8); peers: node shards + peer-push exchange; nodes: node
    # shards + RCCL all-gather of the preference rows
    ap.add_argument("--shard", default="auto", choices=["auto", "peers", "targets", "nodes"])
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xA7A1A9C4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--plane-nt", type=int, default=None, help="override the plane_nt tuning option")
    ap.add_argument("--kernel", type=int, default=None, choices=[1, 2],
                    help="round kernel generation (A/B only; default: the engine's choice)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a 1-GPU box: every rank on device 0, gloo for the host-side "
                         "barrier/reductions (not a measurement)")
    ap.add_argument("--no-roofline-pass", action="store_true",
                    help="skip the HIP-event pass (rocprofv3 PMC runs: one window only)")
    ap.add_argument("--no-exchange-pass", action="store_true",
                    help="skip the one-GPU changed-word pass (rocprofv3 PMC runs: the roofline pass stays the "
                         "process's last round-kernel dispatches, tools/pmc_bench.py)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="where the full per-round / per-workload detail goes (the line stays compact)")
    return ap.parse_args(argv)


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def rank_launch_cmd(argv, gpus, port):
    """The command that runs this bench as `gpus` rank processes of one node
    (torch.distributed.run, rendezvous on 127.0.0.1), with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def launch_ranks(argv, gpus):
    """`bench.py --gpus N` started without a launcher (WORLD_SIZE unset): run
    the N ranks as ONE fresh child process (never exec: nothing here has
    touched the GPU, and this process only waits), pass its output through and
    return its exit status."""
    cmd = rank_launch_cmd(argv, gpus, free_port())
    print("bench: launching " + " ".join(cmd[1:7]) + f" ... ({gpus} ranks)", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def src_digest():
    h = hashlib.sha256()
    for p in KERNEL_SRC:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_cpus():
    """The host cores this process may use: the affinity mask, capped by the
    cgroup CPU quota (cpu.max) when one is set — a 1-GPU box exposes every
    CPU of the machine in its affinity mask but grants a share of them."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    threads = affinity if quota is None else max(1, min(affinity, int(round(quota))))
    return {"threads": threads, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(wl, seed, budget_s):
    """Oracle ("port": the C restatement of the reference semantics,
    oracle/avalanche_oracle.c) on host cores, on a bounded sample of the same
    workload: fewer nodes, same targets/k, the same all-live rounds."""
    from oracle import cabi

    n, m, k, init_mode, init_param, byz, replay, _ = WORKLOADS[wl]
    hc = host_cpus()
    threads = hc["threads"]
    # ~10-20 s of CPU work (the branch-free oracle runs ~6e9 updates/s on 16 cores)
    ns = min(n, 500_000 if wl != "c2" else 1000)
    sim = cabi.Sim(ns, m, k, seed=seed, byz_threshold=byz, init_mode=init_mode, init_param=init_param,
                   threads=threads)
    applied = 0
    dt = 0.0
    rounds = 0
    while dt < budget_s and rounds < EPOCH:
        errs = cabi.gen_replay_errs(seed, rounds, 0, ns, m, k) if replay else None  # input, untimed
        ts = time.perf_counter()
        _, a = sim.run_round(errs, threads=threads, collect=False)
        dt += time.perf_counter() - ts
        applied += a
        rounds += 1
    sim.close()
    return {"value": applied / dt, "unit": "vote-record updates/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": hc,
            "sample_short": f"oracle C restatement (branch-free bit-plane path, AVX2 target clone), {ns} x {m}, "
                            f"rounds 0..{rounds - 1}, {dt:.1f}s, {threads} threads",
            "sample": f"oracle/avalanche_oracle.c (C restatement of vote.go/processor.go, the parity oracle; its "
                      f"branch-free bit-plane round, vectorised by an AVX2 target clone — not the reference's Go "
                      f"map path, which has no toolchain here), "
                      f"{ns} nodes x {m} targets, k={k}, rounds 0..{rounds - 1} ({applied} regsiterVote "
                      f"applications, {dt:.1f}s, OpenMP over nodes, {threads} threads on {cpu_model()})"}


class Runner:
    """One engine (this rank's shard of a workload) stepped through the epoch
    chain: step p is round p % EPOCH of a fresh network."""

    def __init__(self, wl, args, world, rank, local_rank, log_capacity):
        self.wl = wl
        n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[wl]
        self.n, self.m, self.k, self.replay, self.desc = n, m, k, replay, desc
        self.init = (init_mode, init_param)
        self.world, self.rank = world, rank
        if args.shard == "targets" and world > 1 and m > 4096:
            raise SystemExit("target sharding needs M <= 4096 (poll cap couples targets); use --shard nodes")
        kw = dict(k=k, seed=args.seed, byz_threshold=byz, device=local_rank)
        if world > 1 and args.shard == "targets":
            kw["target_range"] = sharding.target_shard(m, world, rank)
        elif world > 1:
            kw["node_range"] = sharding.node_shard(n, world, rank)
        self.eng = eng = avhip.Engine(n, m, log_capacity=log_capacity, **kw)
        if args.plane_nt is not None:
            eng.set_option("plane_nt", args.plane_nt)
        if args.kernel is not None:
            eng.set_option("kernel", args.kernel)
        eng.init_records(*self.init)
        self.pos = 0  # step index of the next round
        self.shard = args.shard
        self.fallback = None
        if world > 1 and args.shard == "nodes":
            obj = [avhip.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            eng.comm_init(world, rank, obj[0])
        elif world > 1 and args.shard == "peers":
            # runs of 8 tiles for the conflicting workloads' node shards (no settled rounds, which are
            # what the engine's 16-tile default for >= 4 ranks is for): +1-3 % at 4 and 8 ranks
            # (tools/group_model.py, profiles/r05/s16/gm_ptpw_*.log)
            if wl in NODE_SHARD_TPW and not eng_tpw_set(args):
                eng.set_option("tiles_per_wave", NODE_SHARD_TPW[wl])
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
                self.fallback = next(e for e in errs if e)
        self.info = eng.layout_info() if self.fallback is None else None
        # tests (test_gpu_bench_protocol.py): called after every segment, before the log is emptied
        self.on_segment = None

    def close(self):
        self.eng.close()

    def reset(self):
        """Start a fresh epoch (untimed): records re-initialised, log emptied."""
        self.eng.synchronize()
        self.eng.discard_updates()
        self.eng.init_records(*self.init)
        self.pos = 0

    def _run(self, rounds):
        if self.replay:
            self.eng.replay_prepare(rounds)  # untimed: callers prepare before a timed segment
            self.eng.replay_rounds(rounds)
        else:
            self.eng.run_rounds(rounds)

    def steps(self, count, timed, entries=None):
        """Run `count` steps from the current position. timed: every segment
        inside one epoch is bracketed by barrier + synchronize and its wall
        time summed. Untimed steps run one round at a time with the log
        emptied after each (a conflicting workload emits ~1e8 StatusUpdates
        per round); `entries` (a dict) collects each untimed round's log
        entries per kind by round of the epoch. Returns (seconds, applied,
        emitted, segments)."""
        eng = self.eng
        elapsed, applied, emitted, segs = 0.0, 0, 0, 0
        while count > 0:
            if self.pos % EPOCH == 0 and self.pos > 0:
                self.reset()
            seg = min(EPOCH - self.pos % EPOCH, count)
            if not timed and not self.replay:
                seg = 1
            eng.synchronize()
            eng.discard_updates()
            a0 = eng.applied_votes()
            if self.replay:
                eng.replay_prepare(seg)
            if timed:
                if self.world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            if self.replay:
                eng.replay_rounds(seg)
            else:
                eng.run_rounds(seg)
                if timed:
                    # the deferred state the segment's rounds leave behind (stale vote planes, pending
                    # count steps: DESIGN.md §3) is written back inside the timed region, so every
                    # timed round's records are paid for (vote.go:54-75 state observable afterwards)
                    eng.materialize()
            if timed:
                eng.synchronize()
                torch.cuda.synchronize()
                if self.world > 1:
                    dist.barrier()
                elapsed += time.perf_counter() - t0
            else:
                eng.synchronize()
            if eng.log_overflowed():
                raise BenchFailure(f"bench: StatusUpdate log overflowed in {self.wl} steps "
                                   f"{self.pos}..{self.pos + seg - 1}: updates were not stored; no number reported")
            if entries is not None and not timed and seg == 1:
                entries[self.pos % EPOCH] = eng.log_entries()
            if self.on_segment is not None:
                self.on_segment(self, self.pos, seg)
            emitted += eng.updates_count()
            applied += eng.applied_votes() - a0
            self.pos += seg
            count -= seg
            segs += 1
        return elapsed, applied, emitted, segs

    def goto(self, pos):
        """Untimed: bring the engine to step `pos` of a fresh chain."""
        self.reset()
        self.steps(pos, timed=False)


ENTRY_BYTES = (8, 32, 48)  # singles, slot records, dense records (k = 8; kernels.h)


def window_segments(warmup, steps):
    """The timed window's segments as lists of epoch rounds (steps W..W+K-1, split at epoch starts)."""
    segs, cur = [], []
    for pos in range(warmup, warmup + steps):
        if pos % EPOCH == 0 and cur:
            segs.append(cur)
            cur = []
        cur.append(pos % EPOCH)
    if cur:
        segs.append(cur)
    return segs


def compact_delivery(d):
    """The delivery measurement in the line: StatusUpdates per second consumed on the device
    (av_updates_digest) and fetched to the host as packed words (pageable / pinned destination), and
    the vote-record updates per second of rounds 0-3 with every round's updates delivered to host
    memory: votes_per_s_with_fetch = the pipelined compact stream (round r + 1 computes while round
    r's stream is copied), _words = the same with every stream expanded into the caller's packed
    words, _unpipelined = one round then its packed-word fetch into pinned memory."""
    cp = d.get("compact") or {}
    return {"digest_updates_per_s": d["digest_updates_per_s"],
            "fetch_updates_per_s": {"pageable": d["pageable"]["updates_per_s"], "pinned": d["pinned"]["updates_per_s"]},
            "votes_per_s_with_fetch": cp.get("votes_per_s"),
            "votes_per_s_with_fetch_words": cp.get("votes_per_s_expanded"),
            "votes_per_s_with_fetch_unpipelined": d["pinned"]["delivered_votes_per_s"],
            "compact_bytes_per_update": cp.get("bytes_per_update")}


def compact_pipeline(run, rounds=4, most_updates=0):
    """Rounds 0..rounds-1 of a fresh epoch with every round's StatusUpdates delivered to host memory
    as the compact stream (av_fetch_compact_async / _wait): round r + 1 is enqueued while round r's
    stream is copied on the copy stream. Wall clock from the first round's enqueue to the last
    stream in host memory. Then the same with every stream also expanded into the caller's packed
    words (av_compact_expand, host threads; ctypes releases the GIL) on a consumer thread, which
    reads stream r while streams r + 1 and r + 2 are encoded and copied (the engine keeps three).
    Two first passes (untimed) grow the engine's delivery buffers: Byzantine rows follow the absolute
    round's parity (byz_pattern), so the same epoch rounds emit different amounts a pass later."""
    from concurrent.futures import ThreadPoolExecutor

    eng = run.eng
    out = {}
    # the caller's packed-word buffer, allocated and touched before the timed rounds
    words = np.empty(max(most_updates, 1) + (1 << 20), np.uint64)
    words.fill(0)
    pool = ThreadPoolExecutor(max_workers=1)
    for mode in ("warm", "warm", "stream", "expanded"):
        run.goto(0)
        eng.synchronize()
        a0 = eng.applied_votes()
        nbytes = nupd = 0
        pend, jobs = [], []

        def consume(t):
            nonlocal nbytes, nupd
            view = eng.fetch_compact_wait(t, copy=False)
            h = avhip.compact_header(view)
            nbytes += h["bytes"]
            nupd += h["n_updates"]
            if mode == "expanded":
                jobs.append(pool.submit(avhip.compact_expand_into, view, words))

        def settle(keep):
            # the stream whose slot the next av_fetch_compact_async reuses is expanded by now
            while len(jobs) > keep:
                jobs.pop(0).result()
        t0 = time.perf_counter()
        for _ in range(rounds):
            eng.run_rounds(1)
            settle(1)
            pend.append(eng.fetch_compact_async())
            if len(pend) >= 2:
                consume(pend.pop(0))
        while pend:
            consume(pend.pop(0))
        settle(0)
        dt = time.perf_counter() - t0
        run.pos += rounds
        applied = eng.applied_votes() - a0
        out[mode] = {"s": dt, "applied": applied, "updates": nupd, "bytes": nbytes}
    pool.shutdown()
    st, ex = out["stream"], out["expanded"]
    return {"rounds": rounds, "updates": st["updates"], "bytes": st["bytes"],
            "bytes_per_update": st["bytes"] / max(1, st["updates"]),
            "votes_per_s": st["applied"] / st["s"], "ms": st["s"] * 1e3,
            "GB_per_s": st["bytes"] / st["s"] / 1e9, "updates_per_s": st["updates"] / st["s"],
            "votes_per_s_expanded": ex["applied"] / ex["s"], "ms_expanded": ex["s"] * 1e3,
            "note": "compact stream (include/avhip.h av_compact_header: ~2 B per update, canonical order) "
                    "copied into engine-owned pinned host memory handed to the caller (zero-copy view, valid "
                    "three tickets); expanded: also av_compact_expand into the caller's packed uint64 words on a "
                    "consumer thread"}


def size_log(eng, per_round, warmup, steps):
    """Log entries per kind for the largest timed segment (the warm-up epoch's per-round counts
    summed over the segment's rounds, 1.3x + 64 per shard of slack), in place of the worst case per
    update: the device log holds what one timed segment emits, and at least any one round of the
    epoch (the delivery pass fetches rounds 0-3 one at a time, whatever the window). Returns the
    log's bytes."""
    need = [max(per_round.get(r, (0, 0, 0))[k] for r in range(EPOCH)) for k in range(3)]
    for seg in window_segments(warmup, steps):
        tot = [sum(per_round.get(r, (0, 0, 0))[k] for r in seg) for k in range(3)]
        need = [max(a, b) for a, b in zip(need, tot)]
    ent = [int(1.3 * v) + 64 * 1024 for v in need]
    eng.synchronize()
    eng.discard_updates()
    eng.resize_log(*ent)
    return sum(e * b for e, b in zip(ent, ENTRY_BYTES))


def log_capacity(n, m, world, rank, shard):
    """StatusUpdate log entries for one rank's engine: every update of one timed
    segment (up to 16 rounds: C4 ~2e8 in rounds 0-2, the conflicting C4p/C4pb
    ~1e9 over rounds 0-8) of the rank's share of the network. 36 B of device
    memory per entry at k = 8 (singles 8, slot records 16, dense records 12 B of
    capacity per update): 45 GB at 1M x 1000 and 77 GB for C5 on one GPU."""
    n_loc, m_loc = n, m
    if world > 1:
        if shard == "targets":
            t0, t1 = sharding.target_shard(m, world, rank)
            m_loc = t1 - t0
        else:
            n_loc = -(-n // world)
    return min(int(1.25 * n_loc * m_loc) + (1 << 20), (1 << 31) - 1)


def measure(wl, args, world, rank, local_rank, steps, warmup):
    """This rank's shard of workload `wl`: device warm-up (one untimed epoch),
    `warmup` untimed steps, `steps` timed steps; then a second pass over the
    same steps with HIP events around every round kernel (roofline)."""
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[wl]
    args = argparse.Namespace(**vars(args))  # this workload's copy (its decomposition)
    args.shard = shard_for(wl, world, args.shard)
    # replay (C2) keeps the per-update worst case; the sim workloads start small and are re-sized
    # after the warm-up epoch (size_log)
    log_cap = log_capacity(n, m, world, rank, args.shard) if replay else 1 << 20
    run = Runner(wl, args, world, rank, local_rank, log_cap)
    if run.fallback is not None:
        args.shard = "targets"
        args.shard_fallback = run.fallback
        return measure(wl, args, world, rank, local_rank, steps, warmup)
    eng = run.eng
    # ---- device warm-up (untimed): after process start the GPU runs these
    # kernels up to ~15 % slower for the first ~20-30 ms of sustained load
    # (tools/gap_probe.py --events-first): one untimed epoch,
    # one round at a time in a log of two single words and one record per lane
    # (what one round can emit at most), counting each round's entries; then the
    # log is sized for the largest timed segment
    log_bytes = None
    if not replay:
        lanes = eng.layout_info()["lanes"]
        eng.resize_log(2 * lanes, lanes, lanes)
        per_round = {}
        run.steps(EPOCH, timed=False, entries=per_round)
        log_bytes = size_log(eng, per_round, warmup, steps)
    else:
        run.steps(EPOCH, timed=False)
    # ---- warmup steps (untimed), then the timed steps
    run.goto(warmup)
    elapsed, applied, emitted, segs = run.steps(steps, timed=True)
    # (the timed segments end with the deferred state's write-back, av_materialize: inside the
    # window; the roofline pass below times it on its own as writeback_ms)
    writeback_ms = None

    # ---- delivery (one GPU, sim workloads; detail only): rounds 0-3 of a fresh epoch (the fresh and
    # storm rounds, the most updates) one at a time, each followed by av_fetch_updates of its whole
    # update stream into pageable host memory: the reference's *[]StatusUpdate out-parameter
    # (processor.go:61,111) filled every round
    delivery = None
    if world == 1 and not replay and not args.no_roofline_pass:  # (before the roofline pass, which
        # must stay the process's last round-kernel dispatches for tools/pmc_bench.py)
        rows = []
        for dest in ("pageable", "pinned"):
            run.goto(0)
            buf = None
            if dest == "pinned":  # allocated before the rounds (page-locking 0.8 GB takes ~70 ms)
                most = max(r["updates"] for r in rows) + (1 << 20)
                buf = torch.empty(most, dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
            for _ in range(4):
                rnd = run.pos % EPOCH
                eng.synchronize()
                a0 = eng.applied_votes()
                t0 = time.perf_counter()
                eng.run_rounds(1)
                eng.synchronize()
                t1 = time.perf_counter()
                nu = eng.updates_count()
                # the on-device consumer: av_updates_digest folds every pending update (all three
                # record kinds) in device memory, nothing crosses PCIe
                eng.updates_digest()
                t1d = time.perf_counter()
                if buf is None or buf.size < nu:
                    if dest == "pinned":
                        buf = torch.empty(max(nu, 1), dtype=torch.int64, pin_memory=True).numpy().view(np.uint64)
                    else:
                        buf = np.empty(max(nu, 1), np.uint64)
                got = eng.fetch_into(buf)
                t2 = time.perf_counter()
                run.pos += 1
                rows.append({"dest": dest, "round": rnd, "updates": got, "applied": eng.applied_votes() - a0,
                             "round_ms": (t1 - t0) * 1e3,
                             "digest_ms": (t1d - t1) * 1e3, "fetch_ms": (t2 - t1d) * 1e3})
            buf = None

        def rate(dest):
            rs = [r for r in rows if r["dest"] == dest]
            upd = sum(r["updates"] for r in rs)
            ms = sum(r["round_ms"] + r["fetch_ms"] for r in rs)
            return {"updates": upd, "ms": ms, "updates_per_s": upd / (sum(r["fetch_ms"] for r in rs) * 1e-3),
                    "GB_per_s": 8.0 * upd / (sum(r["fetch_ms"] for r in rs) * 1e-3) / 1e9,
                    "delivered_votes_per_s": sum(r["applied"] for r in rs) / (ms * 1e-3)}
        pg, pn = rate("pageable"), rate("pinned")
        dg = [r for r in rows if r["dest"] == "pageable"]
        compact = compact_pipeline(run, rounds=4, most_updates=max(r["updates"] for r in rows))
        delivery = {"rounds": rows, "pageable": pg, "pinned": pn, "compact": compact,
                    "delivered_updates_per_s": pg["delivered_votes_per_s"],
                    "status_updates_per_s": pg["updates_per_s"],
                    "digest_updates_per_s": sum(r["updates"] for r in dg) / (sum(r["digest_ms"] for r in dg) * 1e-3),
                    "note": "per round (rounds 0-3 of a fresh epoch), wall clock: the round; av_updates_digest (the "
                            "on-device consumer); av_fetch_updates (device expansion, canonical radix sort, copy "
                            "to the host: 8 B per update) into pageable memory (through pinned staging) or "
                            "straight into a pinned buffer (one DMA)"}
    # ---- roofline pass: the same steps again, every round's kernels bracketed
    # by HIP events on the engine's stream; sim rounds one step at a time so
    # that every round's kernel time, model bytes and re-read bytes are known
    kern_ms = launches = 0
    moved = reread = 0
    applied2 = emitted2 = 0
    per_round = []
    if not args.no_roofline_pass:
        # the same steps of fresh epochs; the peer draws follow the engine's
        # absolute round counter, so the StatusUpdate count differs slightly
        # from the timed pass (the applied votes do not: every record is live)
        run.goto(warmup)
        eng.set_timing(True)
        left = steps
        wb_ms = 0.0

        def writeback():
            # the write-back that ends a timed segment, timed alone (its own launches)
            nonlocal wb_ms
            if replay:
                return
            eng.materialize()
            wb_ms += eng.kernel_stats()[0]  # (the loop read and reset the round events already)
        while left > 0:
            rnd = run.pos % EPOCH
            if rnd == 0 and run.pos > 0 and left < steps:
                writeback()  # the previous epoch's segment ended here
            seg = min(EPOCH - rnd, left) if replay else 1
            b0, r0 = eng.alg_bytes(), eng.alg_bytes_reread()
            _, a, em, _ = run.steps(seg, timed=False)
            ms, nl = eng.kernel_stats()
            db, dr = eng.alg_bytes() - b0, eng.alg_bytes_reread() - r0
            per_round.append({"round": rnd, "rounds": seg, "kernel_ms": ms, "launches": nl, "model_bytes": db,
                              "reread_bytes": dr, "applied": a, "emitted": em})
            kern_ms += ms
            launches += nl
            moved += db
            reread += dr
            applied2 += a
            emitted2 += em
            left -= seg
        writeback()  # the window's last segment
        writeback_ms = None if replay else wb_ms
        eng.set_timing(False)
        if applied2 != applied:
            raise BenchFailure(f"bench: roofline pass applied {applied2} votes, the timed pass {applied}")
    # ---- exchange pass (one GPU, sim workloads): the same steps again with the changed published
    # words counted per round (option count_changed), the input of the multi-GPU push model
    changed = None
    if world == 1 and not replay and not args.no_roofline_pass and not args.no_exchange_pass:
        run.goto(warmup)
        eng.set_option("count_changed", 1)
        changed = []
        for _ in range(steps):
            rnd = run.pos % EPOCH
            w0, g0 = eng.changed_words()
            run.steps(1, timed=False)
            w1, g1 = eng.changed_words()
            changed.append({"round": rnd, "words": w1 - w0, "segments": g1 - g0})
        eng.set_option("count_changed", 0)
    replicas = None
    needed_rows = None
    if world > 1 and args.shard in ("peers", "nodes"):
        # the exchange's own invariant, checked before any resynchronisation: every peer row a local
        # node draws in the next round (R1: the draw is a function of (seed, node, round)) is, in this
        # rank's replica, the row its owner holds now (a push lost in a round shows here)
        needed_rows = exchange_rows_match(eng, n, world, rank)
        # then every rank's whole replica must be the same once the withheld rows are pushed:
        # hash a slice of every rank's node range as this rank sees it
        if args.shard == "peers":
            eng.peer_sync()  # need-masked pushes leave rows no local node reads behind (collective)
        hs = hashlib.sha256()
        for r in range(world):
            a = sharding.node_shard(n, world, r)[0]
            hs.update(eng.read_pref(a, min(a + 2048, n)).tobytes())
        digests = [None] * world
        dist.all_gather_object(digests, hs.hexdigest())
        replicas = len(set(digests)) == 1
    info = run.info
    run.close()

    # the general step: the fresh and storm rounds of the window (bench round kinds
    # 'fresh' / 'storm', every tile through the slot network), updates over their HIP-event kernel time
    gen = [pr for pr in per_round if round_kind(pr["round"], replay) in ("fresh", "storm")]
    gen_applied = float(sum(pr["applied"] for pr in gen))
    gen_ms = float(sum(pr["kernel_ms"] for pr in gen))
    if world > 1:
        st = torch.tensor([elapsed, gen_ms, float(applied), float(emitted), gen_applied], dtype=torch.float64,
                          device="cpu" if args.rehearse_one_gpu else "cuda")
        tmax = st[0:2].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tot = st[2:5].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        elapsed, gen_ms = float(tmax[0]), float(tmax[1])
        applied_all, emitted_all, gen_applied = float(tot[0]), float(tot[1]), float(tot[2])
    else:
        applied_all, emitted_all = applied, emitted
    value_general = gen_applied / (gen_ms * 1e-3) if gen and gen_ms > 0 else None
    kavg_ms = kern_ms / launches if launches else None
    gen2 = k <= 8 and args.kernel != 1
    if info["capped"] and replay and gen2:
        # consecutive replay rounds fused per launch (engine option replay_fuse, default 16): one
        # launch covers a timed segment's rounds, so kernel_ms_avg is per launch, not per round
        kname = f"k_replay_node<{k}> (+ k_round_capped exact pass)"
    else:
        kname = (("k_round_node" if gen2 else "k_round_capped") if info["capped"]
                 else ("k_round_sweep" if gen2 else "k_round_fast")) + f"<{k},{'true' if replay else 'false'}>"
    # SURVEY.md §8(d) bytes of this rank's launches in the roofline pass: every
    # applied vote is one live (node, target, round) triple / k; + 20 B per
    # emitted StatusUpdate
    s8d = (applied2 / k * S8D_TRIPLE_BYTES[replay] + emitted2 * S8D_UPDATE_BYTES) / launches if launches else None
    for pr in per_round:
        pr["s8d_bytes"] = pr["applied"] / k * S8D_TRIPLE_BYTES[replay] + pr["emitted"] * S8D_UPDATE_BYTES
    return {
        "wl": wl, "desc": desc, "n": n, "m": m, "k": k, "elapsed": elapsed, "applied": applied_all,
        "emitted": emitted_all, "value": applied_all / elapsed, "segments": segs, "info": info,
        "kavg_ms": kavg_ms, "launches": launches, "s8d_bytes": s8d,
        "moved_bytes": moved / launches if launches else None, "kernel": kname, "replicas_identical": replicas,
        "reread_bytes": reread / launches if launches else None, "per_round": per_round, "replay": replay,
        "kernel_ms_total": kern_ms, "steps": steps,
        "lanes": info["lanes"] if info else None,
        "rounds_per_launch": steps / launches if launches else None,
        "first_round": warmup % EPOCH,
        "writeback_ms": writeback_ms, "changed": changed,
        "value_general": value_general, "general_rounds": sorted({pr["round"] for pr in gen}),
        "needed_rows_match": needed_rows,
        "log_bytes": log_bytes, "delivery": delivery, "shard": args.shard,
        "shard_fallback": getattr(args, "shard_fallback", None),
    }


def exchange_rows_match(eng, n, world, rank, sample=2048):
    """Node-sharded ranks: every peer row the first `sample` local nodes draw in the next round must
    equal, in this rank's replica, its owner's current row. Each rank hashes its replica's copy of
    those rows per owner and sends (rows, hash); each owner re-hashes the rows from its own (the
    authoritative) copy. Collective; True iff every request matches on every rank."""
    a, b = sharding.node_shard(n, world, rank)
    peers = eng.sample_peers(eng.round, a, min(b, a + sample))
    rows = np.unique(peers.reshape(-1))
    owners = [sharding.node_shard(n, world, q) for q in range(world)]
    mine = eng.read_pref_words(0, n)  # this rank's replica, as stored
    req = {}
    for q, (q0, q1) in enumerate(owners):
        if q == rank:
            continue
        rq = rows[(rows >= q0) & (rows < q1)]
        req[q] = (rq.tolist(), hashlib.sha256(np.ascontiguousarray(mine[rq]).tobytes()).hexdigest())
    allreq = [None] * world
    dist.all_gather_object(allreq, req)
    ok = True
    for p in range(world):
        if p == rank or allreq[p] is None or rank not in allreq[p]:
            continue
        rq, h = allreq[p][rank]
        ok &= hashlib.sha256(np.ascontiguousarray(mine[np.asarray(rq, np.int64)]).tobytes()).hexdigest() == h
    oks = [None] * world
    dist.all_gather_object(oks, bool(ok))
    return all(oks)


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


PMC_DIR = os.path.join(ROOT, "profiles", "r06")


def load_pmc(wl, window, world):
    """The committed rocprofv3 PMC summary of this bench window (tools/
    pmc_bench.py), used only if it was measured on these kernel sources."""
    path = os.path.join(PMC_DIR, f"pmc_{wl}.json")
    if world != 1 or not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    if d.get("src_sha") != src_digest() or d.get("window") != window:
        return None
    return d


# round kinds of a fresh sim network at k = 8 (engine: launch_one_round): round 0 reads only A
# (fresh), rounds 1-3 carry the convergence storm, 4-15 may defer count planes (klazy; a tile that
# stays unanimous takes the settled path: no count can reach 120 before round 16, the first 6 votes
# of a fresh record never step it), 16 applies the deferred steps (kconsume, outside the all-live
# epoch)
def round_kind(r, replay):
    if replay:
        return "replay (fused rounds per launch)"
    return "fresh" if r == 0 else "storm" if r <= 3 else "klazy" if r <= 15 else "kconsume"


def binding(fr):
    """The resource closest to its peak; 'latency' when none is above half of
    its peak while waves wait on memory most of their cycles (SQ_WAIT_ANY)."""
    c = {k: v for k, v in fr.items() if k in ("fabric", "hbm_compulsory", "valu_issue", "salu_issue") and v is not None}
    top = max(c, key=c.get)
    if c[top] < 0.5 and (fr.get("wait_any") or 0.0) >= 0.5:
        return "latency"
    return top


def roofline(r, window=None, world=1):
    """Roofline of the round kernel.

    achieved/frac: the bit-sliced kernel's byte model (state
    planes read/written per round type, every gathered preference word, the
    published word, the StatusUpdate log; counted by the kernel itself per
    tile, av_alg_bytes) per launch / the HIP-event launch time, against the
    8 TB/s HBM peak. alg_bytes_s8d/frac_s8d: SURVEY.md §8(d)'s 4-B-per-record
    model, which this layout beats (3.1 B per record), hence > 1.
    hbm_bytes_compulsory: the model minus the preference words re-read by
    other lanes of the same round = a lower bound on the HBM bytes.
    traffic (PMC, when the committed profile matches sources and window):
    FETCH_SIZE + WRITE_SIZE, calibrated = bytes crossing the L2 <-> fabric
    boundary, Infinity-Cache hits included (MI355X_MICROARCH.md §HBM), i.e. an
    upper bound on the HBM bytes. Per round kind: the same fractions, issue
    rates and the binding resource."""
    if r["kavg_ms"] is None:
        return None
    t = r["kavg_ms"] * 1e-3
    ach = r["moved_bytes"] / t / 1e9
    comp = r["moved_bytes"] - r["reread_bytes"]
    out = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
           "traffic": None, "traffic_kind": "fabric (L2<->EA requests incl. Infinity-Cache hits: upper bound on HBM)",
           "kernel": r["kernel"], "kernel_ms_avg": r["kavg_ms"], "launches": r["launches"],
           # the timed pass (wall clock, barrier + synchronize) and the HIP-event pass run the same
           # rounds separately: the difference per step is launch gaps and host work (+- noise)
           "kernel_ms_per_step": r["kernel_ms_total"] / r["steps"],
           "host_gap_ms_per_step": r["elapsed"] / r["steps"] * 1e3 - r["kernel_ms_total"] / r["steps"],
           "rounds_per_launch": r["rounds_per_launch"],
           "model": "bit-sliced byte model per round type (DESIGN.md §3), counted by the kernel (av_alg_bytes)",
           "model_bytes": r["moved_bytes"],
           "hbm_bytes_compulsory": comp, "frac_hbm_compulsory": comp / t / 1e9 / HBM_PEAK_GBS,
           "alg_bytes_s8d": r["s8d_bytes"], "frac_s8d": r["s8d_bytes"] / t / 1e9 / HBM_PEAK_GBS,
           "note": "frac = model bytes / kernel time / 8 TB/s; frac_s8d = SURVEY.md §8(d) bytes (9.125 B per live "
                   "node-target-round + 20 B per StatusUpdate), a model this layout beats"}
    pmc = load_pmc(r["wl"], window, world) if window else None
    pr_pmc = {}
    if pmc:
        out["traffic"] = pmc.get("fabric_bytes_per_launch")
        out["pmc_source"] = pmc.get("source")
        for row in pmc.get("per_round", []):
            pr_pmc.setdefault(row["round"], []).append(row)
    # per round kind (sim: one round per launch; replay: one fused launch per row)
    kinds = {}
    for pr in r["per_round"]:
        kd = kinds.setdefault(round_kind(pr["round"], r["replay"]),
                              {"rounds": [], "ms": 0.0, "launches": 0, "model": 0, "reread": 0, "pmc": []})
        kd["rounds"].append(pr["round"])
        kd["ms"] += pr["kernel_ms"]
        kd["launches"] += pr["launches"]
        kd["model"] += pr["model_bytes"]
        kd["reread"] += pr["reread_bytes"]
    if pmc and len(pmc.get("per_round", [])) == len(r["per_round"]):
        for pr, row in zip(r["per_round"], pmc["per_round"]):
            kinds[round_kind(pr["round"], r["replay"])]["pmc"].append((pr, row))
    rt = {}
    for name, kd in kinds.items():
        ts = kd["ms"] * 1e-3
        fr = {"model": kd["model"] / ts / 1e9 / HBM_PEAK_GBS,
              "hbm_compulsory": (kd["model"] - kd["reread"]) / ts / 1e9 / HBM_PEAK_GBS,
              "fabric": None, "valu_issue": None, "salu_issue": None, "wait_any": None}
        if kd["pmc"]:
            cyc = sum(row["cycles"] for _, row in kd["pmc"])
            fab = sum(row["fabric_bytes"] for _, row in kd["pmc"])
            fr["fabric"] = fab / ts / 1e9 / HBM_PEAK_GBS
            fr["valu_issue"] = sum(row["valu"] for _, row in kd["pmc"]) * 2.0 / (1024.0 * cyc)
            fr["salu_issue"] = sum(row["salu"] for _, row in kd["pmc"]) / (256.0 * cyc)
            fr["wait_any"] = (sum(row["wait_any"] for _, row in kd["pmc"]) /
                              max(1.0, sum(row["wave_cycles"] for _, row in kd["pmc"])))
        ent = {"rounds": sorted(set(kd["rounds"])), "launches": kd["launches"],
               "kernel_ms_avg": kd["ms"] / max(1, kd["launches"]),
               "model_bytes_per_launch": kd["model"] / max(1, kd["launches"]),
               "model_bytes_per_lane": kd["model"] / max(1, kd["launches"]) / r["lanes"] if r["lanes"] else None,
               "fracs": fr}
        ent["binding"] = binding(fr) if kd["pmc"] else None
        rt[name] = ent
    out["round_kinds"] = rt
    # the whole window's binding resource (PMC window sums)
    if pmc:
        iss = pmc["issue"]
        fr = {"fabric": (out["traffic"] or 0.0) / t / 1e9 / HBM_PEAK_GBS,
              "hbm_compulsory": out["frac_hbm_compulsory"], "valu_issue": iss["frac_valu"],
              "salu_issue": iss["frac_salu"], "wait_any": iss["wait_any_frac"]}
        out["binding_fracs"] = fr
        out["binding"] = binding(fr)
        out["issue"] = iss
    return out


# xGMI between two MI355X of one node: 7 links per GPU, one per peer, ~153.6 GB/s per link both
# directions together (MI355X_MICROARCH.md / the platform figure): 76.8 GB/s per direction
XGMI_LINK_GBS = 76.8


def exchange_model(changed, n, ps, ranks=(2, 4, 8)):
    """The peer-push exchange at G ranks from the one-GPU exchange pass: rank r owns
    1/G of the nodes, so it changes ~1/G of the round's published words and stores each changed
    64-B row segment into each of its G - 1 peers' replicas, one peer per xGMI link (all links
    busy at once): per-link bytes per round = segments / G * 64 B. Beside it the all-gather of
    every rank's rows (what `--shard nodes` does with RCCL): (N / G) * row bytes per link."""
    if not changed:
        return None
    out = {"link_GBs_per_direction": XGMI_LINK_GBS, "rounds": [c["round"] for c in changed],
           "changed_words": [c["words"] for c in changed], "changed_segments": [c["segments"] for c in changed]}
    for g in ranks:
        push = [c["segments"] / g * 64.0 / (XGMI_LINK_GBS * 1e9) * 1e3 for c in changed]
        out[f"g{g}"] = {"push_ms_per_round_mean": sum(push) / len(push), "push_ms_per_round_max": max(push),
                        "push_bytes_per_link_max": max(c["segments"] for c in changed) / g * 64.0,
                        "allgather_ms_per_round": n / g * ps * 4.0 / (XGMI_LINK_GBS * 1e9) * 1e3}
    return out


def compact_roofline(rf):
    """The line's roofline: the contract's keys, the kernel and its launches, the binding resource and
    per round kind (ms per launch, frac, binding). Everything else: the detail file."""
    if rf is None:
        return None
    keep = ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms_avg", "launches",
            "frac_hbm_compulsory", "frac_s8d", "binding")
    out = {k: rf[k] for k in keep if k in rf}
    out["kinds"] = {name: {"ms": kd["kernel_ms_avg"], "frac": kd["fracs"]["model"], "binding": kd["binding"]}
                    for name, kd in rf.get("round_kinds", {}).items()}
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher around us: start the ranks as one fresh child process and wait
        sys.exit(launch_ranks(argv, args.gpus))
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

    window = f"{args.warmup}+{args.steps}"
    detail = {"window": window, "n_gpus": world, "workloads": {}}
    try:
        r = measure(args.workload, args, world, rank, local_rank, args.steps, args.warmup)
        secondary = {}
        if not args.no_secondary:
            if world > 1 and not args.rehearse_one_gpu:
                # the exchange a node-sharded C4 round would need with an all-gather:
                # every rank's published-preference rows (N/G x 128 B) over xGMI
                # (RCCL through torch.distributed); a diagnostic, not the timed value
                try:
                    secondary["xgmi_allgather"] = allgather_probe(world, local_rank)
                except Exception as exc:
                    secondary["xgmi_allgather"] = {"error": repr(exc)[:200]}
            others = ["c4p", "c4pb", "c3", "c5"] + (["c2"] if world == 1 else [])
            for wl in others:
                if wl == args.workload:
                    continue
                try:
                    sr = measure(wl, args, world, rank, local_rank, args.steps, args.warmup)
                except avhip.AvError as ex:  # a secondary workload's failure leaves the headline's line
                    secondary[wl] = {"error": repr(ex)[:300]}
                    continue
                rf = roofline(sr, window, world)
                secondary[wl] = {"value": sr["value"], "value_general": sr["value_general"],
                                 "ms_per_step": sr["elapsed"] / args.steps * 1e3,
                                 "frac": rf["frac"] if rf else None, "binding": rf.get("binding") if rf else None}
                if sr["writeback_ms"] is not None:
                    secondary[wl]["writeback_ms"] = sr["writeback_ms"]
                if sr["delivery"]:
                    secondary[wl]["delivery"] = compact_delivery(sr["delivery"])
                if world > 1:
                    secondary[wl]["replicas_identical"] = sr["replicas_identical"]
                    secondary[wl]["needed_rows_match"] = sr["needed_rows_match"]
                    secondary[wl]["shard"] = sr["shard"]
                detail["workloads"][wl] = {"workload": sr["desc"], "value": sr["value"], "delivery": sr["delivery"],
                                           "ms_per_step": sr["elapsed"] / args.steps * 1e3,
                                           "updates_emitted": int(sr["emitted"]), "roofline": rf,
                                           "per_round": sr["per_round"], "writeback_ms": sr["writeback_ms"],
                                           "exchange_model": exchange_model(sr["changed"], sr["n"],
                                                                            avhip_pref_stride(sr))}
    except BenchFailure as ex:
        if rank == 0:
            print(str(ex), file=sys.stderr, flush=True)
        raise SystemExit(3)

    if rank == 0:
        first = r["first_round"]
        rf = roofline(r, window, world)
        line = {
            "metric": "vote-record updates/sec (node·target·round) at 1/2/4/8 GPU; % HBM roofline",
            "value": r["value"],
            # updates/s of the fresh and storm rounds alone (the general step: every tile through the
            # slot network, no settled shortcut), HIP-event kernel time; `value` is the whole window
            "value_general": r["value_general"],
            "general_rounds": r["general_rounds"],
            "unit": "vote-record updates/s (1 update = 1 regsiterVote on a live record; k=8 per node·target·round)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": r["elapsed"] / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded Philox4x32-10 network; no dataset)",
            "config": {
                "workload": r["desc"],
                "n_nodes": r["n"], "n_targets": r["m"], "k": r["k"],
                "rounds": f"step p = round p % 16 of a fresh network (all records live), timed from round {first}, "
                          f"{r['segments']} segment(s)",
                "parallelism": (PARALLELISM[r["shard"]] + f" x{world}") if world > 1 else "single GPU",
            },
            "updates_emitted": int(r["emitted"]),
            "roofline": compact_roofline(rf),
            "writeback_ms": r["writeback_ms"],
            # device memory of the StatusUpdate log (sized for the largest timed segment, size_log)
            "log_gb": r["log_bytes"] / 1e9 if r["log_bytes"] else None,
            "detail": os.path.relpath(args.detail, ROOT),
        }
        if r["delivery"]:
            line["delivery"] = compact_delivery(r["delivery"])
        if r["replicas_identical"] is not None:
            line["config"]["replicas_identical"] = r["replicas_identical"]
            line["config"]["needed_rows_match"] = r["needed_rows_match"]
        if r.get("shard_fallback"):
            line["config"]["shard_fallback"] = "peer exchange unavailable: " + r["shard_fallback"]
        # the north star's own workload (BASELINE.json: "1M nodes x 1k conflicting targets"): C4p, 500
        # double-spend pairs per node, every round through the slot network (no settled shortcut)
        ns = r if args.workload == "c4p" else secondary.get("c4p")
        if ns and ns.get("value") is not None:
            line["north_star_value"] = ns["value"]
            line["north_star"] = {"workload": WORKLOADS["c4p"][7], "value": ns["value"],
                                  "value_general": ns.get("value_general"),
                                  "target": 1e10, "note": "BASELINE.json north_star: >= 1e10 bit-exact vote-record "
                                  "updates/s for 1M nodes x 1k conflicting targets (target on 8 GPUs)"}
        if secondary:
            line["secondary"] = secondary
        detail["workloads"][args.workload] = {"workload": r["desc"], "value": r["value"], "delivery": r["delivery"],
                                              "ms_per_step": r["elapsed"] / args.steps * 1e3,
                                              "updates_emitted": int(r["emitted"]), "roofline": rf,
                                              "per_round": r["per_round"], "writeback_ms": r["writeback_ms"],
                                              "exchange_model": exchange_model(r["changed"], r["n"],
                                                                               avhip_pref_stride(r))}
        if not args.no_cpu_baseline and world == 1:
            cb = cpu_baseline(args.workload, args.seed, args.cpu_seconds)
            detail["cpu_baseline"] = cb
            line["cpu_baseline"] = {k: cb[k] for k in ("value", "unit", "cores", "kind")}
            line["cpu_baseline"]["sample"] = cb["sample_short"]
        os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
        with open(args.detail, "w") as f:
            json.dump(detail, f, indent=1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def avhip_pref_stride(r):
    """Words per preference row (kernels.h pref_stride) of a measured workload."""
    bl = r["info"]["local_blocks"] if r["info"] else (r["m"] + 31) // 32
    return bl if bl <= 1 else ((bl + 31) // 32 * 32 if bl > 32 else 1 << (bl - 1).bit_length())


if __name__ == "__main__":
    main()
