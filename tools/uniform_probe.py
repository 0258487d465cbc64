#!/usr/bin/env python3
"""After each round of a workload's epoch: how many published rows differ from the reference
node's row of this snapshot and of the one before (DESIGN.md §3 uniform rows: a round tags its
output when a published word differs from the previous snapshot's reference word)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import avhip  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--ref", type=int, default=0)
    args = ap.parse_args()
    n, m, k, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    e = avhip.Engine(n, m, k=k, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=min(n * m // 2 + (1 << 20), 1 << 31))
    e.init_records(init_mode, init_param)
    prev = e.read_pref_words()
    for r in range(args.rounds):
        e.run_rounds(1)
        u = e.updates_count()
        e.discard_updates()
        cur = e.read_pref_words()
        ref_now, ref_prev = cur[args.ref], prev[args.ref]
        out = {"round": r, "updates": u,
               "rows_differing_from_own_ref": int((cur != ref_now).any(axis=1).sum()),
               "rows_differing_from_prev_ref": int((cur != ref_prev).any(axis=1).sum()),
               "ref_row_changed": bool((ref_now != ref_prev).any())}
        print(json.dumps(out), flush=True)
        prev = cur


if __name__ == "__main__":
    main()
