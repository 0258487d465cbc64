#!/usr/bin/env python3
"""StatusUpdate delivery time in C4's finalization storm.

Runs C4 (1M x 1000, k=8) on one GPU to round 15 (untimed), then for each of
rounds 16..19: the round kernel (HIP events), and av_fetch_updates — the
device side (log counts, compaction of singles + dense records, dense-record
expansion, radix sort of the packed words on the device) plus the copy of the
sorted words to host memory — timed by wall clock around the call, the words
returned raw (decode=False: the caller's own decoding is not part of the
delivery). Reports words/s and host-copy GB/s.

    python tools/delivery_probe.py [--json out.json]
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
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--rounds", default="16,17,18,19")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[a.workload]
    want = [int(x) for x in a.rounds.split(",")]
    e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=min(2 * n * m + (1 << 20), 1 << 31))
    e.init_records(init_mode, init_param)
    rows = []
    for r in range(max(want) + 1):
        if r not in want:
            e.run_rounds(1)
            e.synchronize()
            e.discard_updates()
            continue
        e.set_timing(True)
        e.run_rounds(1)
        e.synchronize()
        kms, _ = e.kernel_stats()
        e.set_timing(False)
        cnt = e.updates_count()
        t0 = time.perf_counter()
        words = e.fetch_updates(decode=False)
        dt = time.perf_counter() - t0
        assert words.size == cnt
        assert words.size < 2 or bool((words[1:] >= words[:-1]).all())  # canonical order
        rows.append({"round": r, "kernel_ms": kms, "updates": int(cnt), "fetch_ms": dt * 1e3,
                     "words_per_s": cnt / dt if dt > 0 else None,
                     "host_GBps": cnt * 8 / dt / 1e9 if dt > 0 else None})
        print(json.dumps(rows[-1]), flush=True)
        del words
    out = {"workload": desc, "rounds": rows,
           "note": "fetch_ms: av_fetch_updates wall time (device compaction + dense expansion + radix sort + "
                   "copy of the sorted packed words to pageable host memory), decode=False"}
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
