#!/usr/bin/env python3
"""Read-request sizes at the L2's memory side (TCC EA) over exactly the bench
window's round-kernel dispatches (the roofline pass, as tools/pmc_bench.py):
how many 32-, 64- and 128-B requests the L2 sends to the fabric per launch,
the bytes they stand for, and the share of requests that go on to DRAM (the
rest are Infinity-Cache hits). Attributes a workload's fabric bytes beyond the
kernel's byte model (C5 moved 1.6x its model).

Inputs: rocprofv3 --pmc passes of `python3 bench.py --workload W --no-cpu-baseline
--no-secondary --no-exchange-pass`:
  --req  TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum
  --dram TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum GRBM_GUI_ACTIVE

    python tools/pmc_ea.py --req DIR --dram DIR --launches 20 [--model-bytes B] --out out.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_bench import window  # noqa: E402


def sums(d, launches):
    tot = {}
    win = window(d, launches)
    for _, _, c in win:
        for k, v in c.items():
            tot[k] = tot.get(k, 0.0) + v
    return {k: v / launches for k, v in tot.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--req", required=True)
    ap.add_argument("--dram", default=None)
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--model-bytes", type=float, default=None, help="the kernel's model bytes per launch")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    r = sums(args.req, args.launches)
    n32, n64, n128 = (r.get(f"TCC_EA0_RDREQ_{w}B_sum", 0.0) for w in (32, 64, 128))
    tot = r.get("TCC_EA0_RDREQ_sum", 0.0)
    out = {"per_launch": r, "rdreq_32B": n32, "rdreq_64B": n64, "rdreq_128B": n128, "rdreq": tot,
           "read_bytes_by_size": 32 * n32 + 64 * n64 + 128 * n128,
           "note": "requests per launch of the round kernel over the bench window; read bytes = 32/64/128 B "
                   "per request of each size"}
    if args.dram:
        d = sums(args.dram, args.launches)
        out["dram"] = d
        if tot:
            out["dram_share_of_rdreq"] = d.get("TCC_EA0_RDREQ_DRAM_sum", 0.0) / tot
    if args.model_bytes:
        out["model_bytes"] = args.model_bytes
    txt = json.dumps(out, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
