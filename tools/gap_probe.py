#!/usr/bin/env python3
"""Inter-kernel gaps of back-to-back rounds with and without per-launch HIP
timing events (run under rocprofv3 --kernel-trace; diagnostics only).

    rocprofv3 --kernel-trace -d DIR -o gap -- python3 tools/gap_probe.py [--workload c4]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402,F401

import avhip  # noqa: E402
from bench import WORKLOADS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c4")
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--events-first", action="store_true", help="run the evented pass first")
ap.add_argument("--option", action="append", default=[], help="engine option name=value (repeatable)")
a = ap.parse_args()
n, m, k, mode, param, byz, replay, _ = WORKLOADS[a.workload]
for timing in ((True, False) if a.events_first else (False, True)):
    e = avhip.Engine(n, m, k=k, byz_threshold=byz, log_capacity=1 << 26)
    for o in a.option:
        name, val = o.split("=")
        e.set_option(name, int(val))
    e.init_records(mode, param)
    if replay:
        e.replay_prepare(a.rounds + 2)
    run = e.replay_rounds if replay else e.run_rounds
    run(2)
    e.synchronize()
    e.discard_updates()
    e.set_timing(timing)
    t0 = time.perf_counter()
    run(a.rounds)
    e.synchronize()
    dt = time.perf_counter() - t0
    print(f"timing={timing}: {dt / a.rounds * 1e3:.4f} ms per round (wall)", flush=True)
    e.close()
