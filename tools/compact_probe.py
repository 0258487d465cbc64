#!/usr/bin/env python3
"""Phases of the compact StatusUpdate delivery (av_fetch_compact_async / _wait,
av_compact_expand) per round of a fresh epoch, on one GPU: the round itself,
the encode call (log counters, the device counting sort and layout, the copy
issued), the copy's wait, and the host expansion into packed words; then the
pipelined loop (round r + 1 beside round r's copy), after a warm-up pass that
grows the engine's buffers.

    python tools/compact_probe.py [--workload c4p] [--rounds 4] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import avhip  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4p")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--json", default=None)
    ap.add_argument("--option", action="append", default=[], help="engine option name=value")
    ap.add_argument("--no-phases", action="store_true")
    a = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[a.workload]
    e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=1 << 20)
    for o in a.option:
        k_, v_ = o.split("=")
        e.set_option(k_, int(v_))
    lanes = e.layout_info()["lanes"]
    e.resize_log(2 * lanes, lanes, lanes)
    words = np.empty(150_000_000, np.uint64)
    words.fill(0)
    out = {"workload": a.workload, "options": a.option, "phases": [], "pipelined": []}
    print(json.dumps({"options": a.option}), flush=True)
    for rep in range(0 if a.no_phases else a.reps):
        e.init_records(init_mode, init_param)
        e.discard_updates()
        for r in range(a.rounds):
            t0 = time.perf_counter()
            e.run_rounds(1)
            e.synchronize()
            t1 = time.perf_counter()
            tk = e.fetch_compact_async()
            t2 = time.perf_counter()
            v = e.fetch_compact_wait(tk, copy=False)
            t3 = time.perf_counter()
            got = avhip.compact_expand_into(v, words)
            t4 = time.perf_counter()
            h = avhip.compact_header(v)
            row = {"rep": rep, "round": r, "updates": got, "bytes": h["bytes"], "round_ms": (t1 - t0) * 1e3,
                   "encode_ms": (t2 - t1) * 1e3, "copy_ms": (t3 - t2) * 1e3, "expand_ms": (t4 - t3) * 1e3,
                   "copy_GBs": h["bytes"] / max(t3 - t2, 1e-9) / 1e9}
            out["phases"].append(row)
            print(json.dumps(row), flush=True)
    from concurrent.futures import ThreadPoolExecutor
    pool = ThreadPoolExecutor(max_workers=1)
    for expand in (False, True):
        for rep in range(a.reps):
            e.init_records(init_mode, init_param)
            e.discard_updates()
            e.synchronize()
            a0 = e.applied_votes()
            pend, jobs, nb = [], [], 0

            def consume(t):
                nonlocal nb
                v = e.fetch_compact_wait(t, copy=False)
                nb += v.size
                if expand:
                    jobs.append(pool.submit(avhip.compact_expand_into, v, words))
            t0 = time.perf_counter()
            for r in range(a.rounds):
                e.run_rounds(1)
                while len(jobs) > 1:
                    jobs.pop(0).result()
                pend.append(e.fetch_compact_async())
                if len(pend) >= 2:
                    consume(pend.pop(0))
            while pend:
                consume(pend.pop(0))
            while jobs:
                jobs.pop(0).result()
            dt = time.perf_counter() - t0
            row = {"expand": expand, "rep": rep, "ms": dt * 1e3, "bytes": nb, "GBs": nb / dt / 1e9,
                   "votes_per_s": (e.applied_votes() - a0) / dt}
            out["pipelined"].append(row)
            print(json.dumps(row), flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
