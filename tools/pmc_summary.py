#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch of the round kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE/WRITE_SIZE are in KiB; the per-width ratio measured/true is taken
from bin/pmc_calib's known-byte kernels profiled in the same kind of pass, and
applied to the round kernel's own mix of access widths.

    python tools/pmc_summary.py --calib-fetch DIR --calib-write DIR \
        --fetch DIR --write DIR --kernel k_round_fast --out profiles/pmc_traffic_c4.json
"""
import argparse
import csv
import glob
import json
import os
import statistics
import subprocess


def per_dispatch(d, counter):
    """{kernel_name: [value per dispatch]} from a rocprofv3 counter_collection csv."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    out = {}
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                out.setdefault(row["Kernel_Name"], {}).setdefault(row["Dispatch_Id"], 0.0)
                out[row["Kernel_Name"]][row["Dispatch_Id"]] += float(row["Counter_Value"])
    return {k: list(v.values()) for k, v in out.items()}


def pick(d, needle):
    hits = {k: v for k, v in d.items() if needle in k}
    if not hits:
        raise SystemExit(f"kernel {needle} not found in {list(d)[:8]}")
    name = max(hits, key=lambda k: len(hits[k]))
    return name, hits[name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--kernel", default="k_round_fast")
    ap.add_argument("--calib-bytes", type=int, default=1 << 30)
    ap.add_argument("--skip", type=int, default=2, help="leading dispatches to ignore (warmup rounds)")
    # algorithmic byte mix of one warm sim-mode lane at k=8
    ap.add_argument("--read-x4", type=float, default=64.0)
    ap.add_argument("--read-x1", type=float, default=40.0)  # C7, A, 8 gathered words
    ap.add_argument("--write-x4", type=float, default=64.0)
    ap.add_argument("--write-x1", type=float, default=8.0)  # A, published word
    ap.add_argument("--lanes", type=int, default=32_000_000)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    cf, cw = per_dispatch(a.calib_fetch, "FETCH_SIZE"), per_dispatch(a.calib_write, "WRITE_SIZE")
    ratio = {}
    for key, d, cnt in (("read_x4", cf, "calib_read_dwordx4"), ("read_x1", cf, "calib_read_dword"),
                        ("write_x4", cw, "calib_write_dwordx4"), ("write_x1", cw, "calib_write_dword")):
        _, vals = pick(d, cnt)
        ratio[key] = statistics.median(vals) * 1024 / a.calib_bytes  # measured / true
    kf, kw = per_dispatch(a.fetch, "FETCH_SIZE"), per_dispatch(a.write, "WRITE_SIZE")
    kname, fvals = pick(kf, a.kernel)
    _, wvals = pick(kw, a.kernel)
    fvals, wvals = fvals[a.skip:], wvals[a.skip:]
    raw_read = statistics.median(fvals) * 1024
    raw_write = statistics.median(wvals) * 1024
    rsum, wsum = a.read_x4 + a.read_x1, a.write_x4 + a.write_x1
    read_scale = (a.read_x4 * ratio["read_x4"] + a.read_x1 * ratio["read_x1"]) / rsum
    write_scale = (a.write_x4 * ratio["write_x4"] + a.write_x1 * ratio["write_x1"]) / wsum
    read, write = raw_read / read_scale, raw_write / write_scale
    try:
        commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    except Exception:
        commit = None
    out = {
        "kernel": kname,
        "dispatches": len(fvals),
        "calibration_measured_over_true": ratio,
        "raw_fetch_bytes_per_launch": raw_read,
        "raw_write_bytes_per_launch": raw_write,
        "hbm_read_bytes_per_launch": read,
        "hbm_write_bytes_per_launch": write,
        "hbm_bytes_per_launch": read + write,
        "alg_bytes_per_launch_planes_gathers": a.lanes * (rsum + wsum),
        "note": "FETCH_SIZE/WRITE_SIZE (KiB) from separate --pmc passes; per-width measured/true ratios from "
                "bin/pmc_calib (1 GiB coalesced dword / dwordx4 streams) applied to the kernel's byte mix",
        "commit": commit,
    }
    print(json.dumps(out, indent=1))
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
