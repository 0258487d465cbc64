#!/usr/bin/env python3
"""Latency of the drop-in RegisterVotes path (processor.go:61-122) on one GPU:
av_register_votes (one Response of one node per call) against
av_register_votes_batch (many Responses of many nodes per call), on the C2
shape (1k nodes x 10k targets, 4096-vote Responses = the poll cap).

    python tools/dropin_latency.py [--json out.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import avhip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    n, m, votes = 1000, 10_000, 4096
    e = avhip.Engine(n, m, k=8)
    e.init_records(avhip.INIT_BERNOULLI, 0x80000000)
    rng = np.random.default_rng(1)
    errs_pool = np.array([0, 0, 0, 1, 0x80000000], np.uint32)
    out = {"shape": f"{n} nodes x {m} targets, {votes}-vote Responses"}
    # single: one Response per call
    t = np.arange(votes, dtype=np.int64)
    reps = 200
    for _ in range(10):
        e.register_votes(0, t, rng.choice(errs_pool, votes))
    t0 = time.perf_counter()
    for i in range(reps):
        e.register_votes(i % n, t, rng.choice(errs_pool, votes))
    dt = (time.perf_counter() - t0) / reps
    out["single"] = {"us_per_call": dt * 1e6, "votes_per_call": votes, "votes_per_s": votes / dt}
    # poll-set order (ascending targets: the fast path) and shuffled targets (sort-grouped path)
    for n_resp, shuffled in ((64, False), (1000, False), (8000, False), (8000, True)):
        nodes = np.arange(n_resp, dtype=np.int64) % n
        offsets = np.arange(n_resp + 1, dtype=np.int64) * votes
        targets = np.tile(t, n_resp)
        if shuffled:
            targets = np.concatenate([rng.permutation(t) for _ in range(n_resp)])
        errs = rng.choice(errs_pool, targets.size)
        e.register_votes_batch(nodes, offsets, targets, errs)
        r = 5
        t0 = time.perf_counter()
        for _ in range(r):
            e.register_votes_batch(nodes, offsets, targets, errs)
        dt = (time.perf_counter() - t0) / r
        out[f"batch_{n_resp}" + ("_shuffled" if shuffled else "")] = {"us_per_call": dt * 1e6, "responses": n_resp, "votes_per_call": int(targets.size),
                                  "us_per_response": dt * 1e6 / n_resp, "votes_per_s": targets.size / dt}
    print(json.dumps(out, indent=1))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
