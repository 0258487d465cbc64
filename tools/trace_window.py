#!/usr/bin/env python3
"""The headline workload's roofline-pass dispatches in a rocprofv3 kernel trace of `python bench.py`
(`--kernel-trace --output-format csv`): the bench runs the headline first, and its roofline pass is
the `launches` sweep-round dispatches before the last write-back (`k_materialize`) that precedes its
exchange pass, whose warm rounds are the first dispatches of the counting kernel build
(`k_round_sweep<8, 0, 1, false, true>`). Prints their mean
duration (to compare with the line's `roofline.kernel_ms_avg`) and writes the window's rows.

    python tools/trace_window.py TRACE.csv [--launches 20] [--out window.csv]
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--launches", type=int, default=20)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sweep = [i for i, r in enumerate(rows) if "k_round_sweep<" in r["Kernel_Name"]]
    cc = [i for i in sweep if "k_round_sweep<8, 0, 1, false, true>" in rows[i]["Kernel_Name"]]
    if not cc:
        raise SystemExit("no counting-build dispatch (exchange pass) in the trace")
    # the roofline pass ends with its last segment's write-back (k_materialize) before the exchange
    # pass (whose first rounds, before count_changed is set, are ordinary sweep dispatches)
    mats = [i for i, r in enumerate(rows) if "k_materialize" in r["Kernel_Name"] and i < cc[0]]
    end = mats[-1] if mats else cc[0]
    before = [i for i in sweep if i < end]
    win = before[-args.launches:]
    durs = [(int(rows[i]["End_Timestamp"]) - int(rows[i]["Start_Timestamp"])) / 1e6 for i in win]
    print(f"{len(win)} dispatches, mean {sum(durs) / len(durs):.4f} ms, total {sum(durs):.4f} ms")
    for i, d in zip(win, durs):
        print(f"  {rows[i]['Kernel_Name'][:60]:60s} {d:.4f} ms")
    if args.out:
        with open(args.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            for i in win:
                w.writerow(rows[i])


if __name__ == "__main__":
    main()
