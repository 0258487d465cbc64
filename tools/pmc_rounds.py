#!/usr/bin/env python3
"""Per-round PMC table from a rocprofv3 --pmc run of tools/round_probe.py:
the round-kernel dispatches in order (after `--skip` warm-up epochs' worth of
them), each counter per dispatch and per 64-lane tile.

    python tools/pmc_rounds.py DIR [DIR ...] --tiles T [--skip S] [--json out.json]
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def load(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    per = collections.OrderedDict()
    for f in files:
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if "k_round_sweep" not in name and "k_round_node" not in name and "materialize" not in name:
                continue
            mk = re.search(r"(k_\w+)(<[^>]*>)?", name)
            key = (int(r["Dispatch_Id"]), mk.group(0) if mk else name)
            per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--tiles", type=int, required=True)
    ap.add_argument("--skip", type=int, default=0, help="round-kernel dispatches to skip (warm-up epochs)")
    ap.add_argument("--json", default=None)
    args = ap.parse_args()
    merged = None
    for d in args.dirs:
        per = load(d)
        rounds = [(k, v) for k, v in sorted(per.items()) if "round" in k[1]][args.skip:]
        if merged is None:
            merged = [dict(kernel=k[1], **v) for k, v in rounds]
        else:
            for row, (k, v) in zip(merged, rounds):
                row.update(v)
    out = []
    for i, row in enumerate(merged):
        r = {"round": i, "kernel": row["kernel"]}
        for c, v in row.items():
            if c == "kernel":
                continue
            r[c] = v
            if c.startswith("SQ_INSTS"):
                r[c + "_per_tile"] = v / args.tiles
        out.append(r)
        print(json.dumps(r))
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
