#!/usr/bin/env python3
"""Does the serial group model (tools/group_model.py: G ranks' round kernels run
one after another on ONE GPU) charge each rank a cold Infinity Cache (MALL)?

In the serial group, rank i's kernel runs right after rank i-1's, which streamed
its own planes and gathered from its own snapshot replica; on a real 8-GPU node
every rank has its GPU's MALL to itself. This probe times one shard's round
kernel (HIP events, the engine stream) alone on one GPU, round after round,
twice: as is, and with a 2 GB read-modify-write sweep of an unrelated buffer
between rounds (evicts the MALL and the L2s). If the flushed time matches the
serial group's per-rank time, the group model's excess over the shard alone is
the time-shared cache, not the exchange.

    python tools/mall_probe.py --workload c4p --shards 1,8 --kinds nodes,targets [--rounds 6]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import avhip  # noqa: E402
from avhip import sharding  # noqa: E402
from bench import WORKLOADS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4p")
    ap.add_argument("--shards", default="1,8")
    ap.add_argument("--kinds", default="nodes,targets")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--flush-mb", type=int, default=2048)
    ap.add_argument("--option", action="append", default=[])
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    N, M, K, init_mode, init_param, byz, replay, desc = WORKLOADS[args.workload]
    junk = torch.empty(args.flush_mb << 18, dtype=torch.float32, device="cuda").fill_(1.0)
    out = {"workload": desc, "flush_mb": args.flush_mb, "runs": {}}

    def rounds(e, flush):
        e.init_records(init_mode, init_param)
        e.run_rounds(2)  # the fresh round and the first storm round untimed (bench warm-up)
        e.synchronize()
        e.discard_updates()
        ms = []
        for _ in range(args.rounds):
            if flush:
                junk.mul_(1.0000001)
                torch.cuda.synchronize()
            e.set_timing(True)
            e.run_rounds(1)
            kms, _ = e.kernel_stats()
            e.set_timing(False)
            e.synchronize()
            e.discard_updates()
            ms.append(kms)
        return ms

    for g in [int(x) for x in args.shards.split(",")]:
        for kind in args.kinds.split(","):
            if g == 1 and kind == "targets":
                continue
            kw = {}
            if g > 1:
                kw = ({"node_range": sharding.node_shard(N, g, 0)} if kind == "nodes"
                      else {"target_range": sharding.target_shard(M, g, 0)})
            e = avhip.Engine(N, M, k=K, seed=0xA7A1A9C4, byz_threshold=byz, log_capacity=1 << 27, **kw)
            if g > 1 and kind == "nodes":
                e.set_option("unsynced_shard", 1)
            for o in args.option:
                name, v = o.split("=")
                e.set_option(name, int(v))
            rounds(e, False)  # device warm-up
            for flush in (False, True, False, True):
                ms = rounds(e, flush)
                key = f"{kind if g > 1 else 'whole'}{g}_{'flushed' if flush else 'warm'}"
                out["runs"].setdefault(key, []).append(statistics.median(ms))
                print(json.dumps({"run": key, "median_ms": statistics.median(ms), "ms": ms}), flush=True)
            e.close()
    print(json.dumps({k: statistics.median(v) for k, v in out["runs"].items()}))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
