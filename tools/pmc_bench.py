#!/usr/bin/env python3
"""PMC summary of exactly the bench window, for bench.py's roofline
(profiles/r04/pmc_<workload>.json, used only while its src_sha matches the
kernel sources): window averages and one row per roofline-pass step.

bench.py runs, per workload: one untimed device warm-up epoch, goto(warmup),
the timed steps, goto(warmup) again and the roofline pass — the same rounds
as the timed steps, each bracketed by HIP events. The roofline pass is the
last `steps` round-kernel dispatches of the process (run with --no-secondary),
so this averages the counters over exactly those dispatches.

Inputs are rocprofv3 --pmc passes of `python3 bench.py --workload W
--no-cpu-baseline --no-secondary --no-exchange-pass --steps S --warmup W` (one pass per counter
group, MI355X_MICROARCH.md §HBM / the 8-SQ-counter limit):
  --sq    SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
          SQ_INSTS_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
  --fetch FETCH_SIZE      --write WRITE_SIZE
  --calib-fetch / --calib-write: bin/pmc_calib under FETCH_SIZE / WRITE_SIZE
Fabric bytes = FETCH_SIZE (KiB) / measured-over-true read ratio + WRITE_SIZE /
write ratio (the calibration kernels move a known 1 GiB with dword and dwordx4
accesses; both read widths measure 0.5, both write widths 1.0 on gfx950).
These are the L2's memory-side (EA) requests: Infinity-Cache hits are
included (MI355X_MICROARCH.md §HBM), so they bound the HBM bytes from above.

Issue fractions (MI355X_MICROARCH.md: a wave64 VALU instruction occupies its
SIMD for 2 cycles; one scalar unit per CU issues one SALU instruction per
cycle): frac_valu = VALU x 2 / (1024 SIMDs x cycles), frac_salu = SALU /
(256 CUs x cycles), cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs).
"""
import argparse
import csv
import glob
import importlib.util
import json
import os
import statistics

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROUND_KERNELS = ("k_round_sweep", "k_round_node", "k_replay_node", "k_round_fast", "k_round_capped", "k_replay_fast")
# launched before the round kernel of the same launch (counted with the next primary dispatch)
PRE = ("k_replay_fast",)
# the kernel a launch of the bench's roofline pass is counted by (k_round_capped also runs as the
# exact pass behind k_round_node / k_replay_node)
PRIMARY = ("k_round_sweep", "k_round_node", "k_replay_node", "k_round_fast")


def dispatches(d):
    """[(dispatch_id, kernel_name, {counter: value})] of every dispatch in a pass dir."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection csv under {d}")
    rows = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                key = int(r["Dispatch_Id"])
                ent = rows.setdefault(key, [r["Kernel_Name"], {}])
                ent[1][r["Counter_Name"]] = ent[1].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return [(k, v[0], v[1]) for k, v in sorted(rows.items())]


def window(d, launches):
    """The round-kernel dispatches of the roofline pass: from the launches-th
    last primary round kernel on (C2: k_replay_node launches with the exact
    passes between them; otherwise one round kernel per step)."""
    rounds = [x for x in dispatches(d) if any(k in x[1] for k in ROUND_KERNELS)]
    prim = [i for i, x in enumerate(rounds) if any(k in x[1] for k in PRIMARY)]
    if len(prim) < launches:
        raise SystemExit(f"{d}: {len(prim)} round-kernel launches, need {launches}")
    return rounds[prim[-launches]:]


def groups(win):
    """The window's dispatches grouped per launch of the bench's roofline pass:
    PRE kernels with the primary that follows them, the exact passes
    (k_round_capped) with the primary before them."""
    out, pending = [], []
    for x in win:
        if any(k in x[1] for k in PRE):
            pending.append(x)
        elif any(k in x[1] for k in PRIMARY):
            out.append(pending + [x])
            pending = []
        elif out:
            out[-1].append(x)
    return out


def step_rounds(warmup, steps, replay, epoch=16):
    """bench.py's roofline-pass segmentation: the first round of each launch."""
    rows, pos, left = [], warmup, steps
    while left > 0:
        rnd = pos % epoch
        seg = min(epoch - rnd, left) if replay else 1
        rows.append(rnd)
        pos += seg
        left -= seg
    return rows


def mean_of(win, counter, launches):
    """Per launch: the counter summed over the window's dispatches / launches."""
    vals = [c[counter] for _, _, c in win if counter in c]
    if len(vals) != len(win):
        raise SystemExit(f"counter {counter} missing in some dispatches")
    return sum(vals) / launches


def calib_ratio(d, needle, counter, true_bytes):
    vals = [c[counter] for _, name, c in dispatches(d) if needle in name and counter in c]
    if not vals:
        raise SystemExit(f"{needle} not found under {d}")
    return statistics.median(vals) * 1024 / true_bytes


def bench_src_digest():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.src_digest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--launches", type=int, default=None,
                    help="roofline-pass launches (default: steps; C2 fuses replay rounds: 2 at the defaults)")
    ap.add_argument("--sq", required=True)
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--calib-fetch", required=True)
    ap.add_argument("--calib-write", required=True)
    ap.add_argument("--calib-bytes", type=int, default=1 << 30)
    ap.add_argument("--replay", action="store_true", help="replay workload (C2): fused launches per segment")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    rf = calib_ratio(a.calib_fetch, "calib_read_dwordx4", "FETCH_SIZE", a.calib_bytes)
    rf1 = calib_ratio(a.calib_fetch, "calib_read_dword", "FETCH_SIZE", a.calib_bytes)
    rw = calib_ratio(a.calib_write, "calib_write_dwordx4", "WRITE_SIZE", a.calib_bytes)
    rw1 = calib_ratio(a.calib_write, "calib_write_dword", "WRITE_SIZE", a.calib_bytes)
    read_ratio, write_ratio = (rf + rf1) / 2, (rw + rw1) / 2

    n = a.launches or a.steps
    wf, ww, wq = window(a.fetch, n), window(a.write, n), window(a.sq, n)
    gf, gw, gq = groups(wf), groups(ww), groups(wq)
    rounds = step_rounds(a.warmup, a.steps, a.replay)
    if not (len(gf) == len(gw) == len(gq) == len(rounds) == n):
        raise SystemExit(f"window groups {len(gf)}/{len(gw)}/{len(gq)} vs {len(rounds)} roofline-pass launches")

    def tot(g, c):
        return sum(x[2][c] for x in g)

    per_round = []
    for r, f_, w_, q_ in zip(rounds, gf, gw, gq):
        per_round.append({
            "round": r, "kernels": [x[1].split("(")[0].split("::")[-1] for x in q_],
            "fabric_bytes": tot(f_, "FETCH_SIZE") * 1024 / read_ratio + tot(w_, "WRITE_SIZE") * 1024 / write_ratio,
            "cycles": tot(q_, "GRBM_GUI_ACTIVE") / 8.0, "valu": tot(q_, "SQ_INSTS_VALU"), "salu": tot(q_, "SQ_INSTS_SALU"),
            "wait_any": tot(q_, "SQ_WAIT_ANY"), "wave_cycles": tot(q_, "SQ_WAVE_CYCLES"),
            "waves": tot(q_, "SQ_WAVES"), "vmem_rd": tot(q_, "SQ_INSTS_VMEM_RD"), "lds": tot(q_, "SQ_INSTS_LDS"),
        })
    names = sorted({n for _, n, _ in wq})
    read = mean_of(wf, "FETCH_SIZE", n) * 1024 / read_ratio
    write = mean_of(ww, "WRITE_SIZE", n) * 1024 / write_ratio
    cyc = mean_of(wq, "GRBM_GUI_ACTIVE", n) / 8.0
    valu, salu = mean_of(wq, "SQ_INSTS_VALU", n), mean_of(wq, "SQ_INSTS_SALU", n)
    out = {
        "workload": a.workload,
        "window": f"{a.warmup}+{a.steps}",
        "src_sha": bench_src_digest(),
        "kernels": names,
        "dispatches": len(wq),
        "launches": n,
        "calibration_measured_over_true": {"read_x4": rf, "read_x1": rf1, "write_x4": rw, "write_x1": rw1},
        "fabric_read_bytes_per_launch": read,
        "fabric_write_bytes_per_launch": write,
        "fabric_bytes_per_launch": read + write,
        "per_round": per_round,
        "issue": {
            "cycles_per_launch": cyc,
            "valu_per_launch": valu,
            "salu_per_launch": salu,
            "vmem_rd_per_launch": mean_of(wq, "SQ_INSTS_VMEM_RD", n),
            "vmem_wr_per_launch": mean_of(wq, "SQ_INSTS_VMEM_WR", n),
            "lds_per_launch": mean_of(wq, "SQ_INSTS_LDS", n),
            "waves_per_launch": mean_of(wq, "SQ_WAVES", n),
            "wait_any_frac": mean_of(wq, "SQ_WAIT_ANY", n) / max(1.0, mean_of(wq, "SQ_WAVE_CYCLES", n)),
            "frac_valu": valu * 2.0 / (1024.0 * cyc),
            "frac_salu": salu / (256.0 * cyc),
            "note": "wave64 VALU = 2 SIMD cycles, 1024 SIMDs; SALU = 1 cycle on one scalar unit per CU, 256 CUs; "
                    "cycles = GRBM_GUI_ACTIVE / 8 XCDs",
        },
        "source": {"sq": a.sq, "fetch": a.fetch, "write": a.write},
        "note": "per launch of the bench's roofline pass (its round-kernel dispatches, summed, / launches: the same "
                "rounds as the timed steps); FETCH_SIZE / WRITE_SIZE corrected by bin/pmc_calib's measured/true ratios "
                "= fabric bytes (L2 <-> EA, Infinity-Cache hits included)",
    }
    print(json.dumps(out, indent=1))
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
