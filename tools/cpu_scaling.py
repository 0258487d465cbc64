#!/usr/bin/env python3
"""CPU baseline scaling probe: the oracle (oracle/avalanche_oracle.c, OpenMP
over nodes) on a C4 slice at a given thread count, to check how many host
threads the box actually grants (affinity mask vs cgroup CPU quota)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import cabi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, required=True)
    ap.add_argument("--nodes", type=int, default=200_000)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    sim = cabi.Sim(a.nodes, 1000, 8, seed=0xA7A1A9C4, init_mode=3, init_param=int(0.8 * 2**32), threads=a.threads)
    sim.run_round(threads=a.threads, collect=False)  # warm
    t0 = time.perf_counter()
    applied = 0
    for _ in range(a.rounds):
        applied += sim.run_round(threads=a.threads, collect=False)[1]
    dt = time.perf_counter() - t0
    sim.close()
    print(f"threads {a.threads}: {applied / dt:.3e} updates/s ({dt:.2f} s)", flush=True)


if __name__ == "__main__":
    main()
