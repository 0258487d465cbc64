#!/usr/bin/env python3
"""The deferred state's write-back (av_materialize, k_materialize) at the bench's segment ends:
HIP-event time of the write-back after rounds 0..E-1 of a fresh network (E = 16: the end of the
first timed segment, rounds 5-15; E = 9: the second, rounds 0-8), per option value.

    python tools/wb_probe.py [--workloads c4,c4p,c5] [--ends 16,9] [--runs 1,4,16] [--json out.json]
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
from bench import WORKLOADS  # noqa: E402


def one(e, init, end):
    e.synchronize()
    e.discard_updates()
    e.init_records(*init)
    for _ in range(end):
        e.run_rounds(1)
        e.synchronize()
        e.discard_updates()
    e.set_timing(True)
    e.kernel_stats()
    e.materialize()
    ms, n = e.kernel_stats()
    e.set_timing(False)
    return ms, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workloads", default="c4,c4p,c5")
    ap.add_argument("--ends", default="16,9")
    ap.add_argument("--runs", default="1,4,16")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    out = []
    for wl in args.workloads.split(","):
        n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[wl]
        e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=0)
        lanes = e.layout_info()["lanes"]
        e.resize_log(2 * lanes, lanes, lanes)
        for end in [int(x) for x in args.ends.split(",")]:
            for run in [int(x) for x in args.runs.split(",")]:
                e.set_option("materialize_run", run)
                one(e, (init_mode, init_param), end)  # warm-up
                ms, nl = one(e, (init_mode, init_param), end)
                row = {"workload": wl, "end": end, "run": run, "ms": ms, "launches": nl}
                out.append(row)
                print(json.dumps(row), flush=True)
        e.close()
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
