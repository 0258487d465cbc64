"""bench.py's host logic (no GPU): round kinds of the C4 epoch, the binding
resource, the roofline built from a roofline pass's per-round rows, the PMC
summary gate (source digest + window) and the CPU-count rule."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

bench = pytest.importorskip("bench")


def test_round_kinds_follow_the_count_bound():
    # round 0 fresh, 1-3 storm, 4-15 klazy (no count can reach 120 before round 16: the first 6
    # votes of a fresh record never step it), 16 on kconsume
    kinds = [bench.round_kind(r, False) for r in range(17)]
    assert kinds[0] == "fresh" and set(kinds[1:4]) == {"storm"}
    assert set(kinds[4:16]) == {"klazy"} and kinds[16] == "kconsume"
    assert bench.round_kind(3, True).startswith("replay")


def test_binding_picks_the_resource_or_latency():
    assert bench.binding({"fabric": 0.8, "valu_issue": 0.3, "salu_issue": 0.2, "wait_any": 0.6}) == "fabric"
    assert bench.binding({"fabric": 0.3, "valu_issue": 0.41, "salu_issue": 0.3, "wait_any": 0.55}) == "latency"
    assert bench.binding({"fabric": 0.3, "valu_issue": 0.41, "salu_issue": 0.3, "wait_any": 0.2}) == "valu_issue"
    assert bench.binding({"fabric": None, "hbm_compulsory": 0.7, "valu_issue": None, "salu_issue": None}) == \
        "hbm_compulsory"


def _r(per_round, lanes=1000):
    kern = sum(p["kernel_ms"] for p in per_round)
    n = len(per_round)
    moved = sum(p["model_bytes"] for p in per_round)
    return {"wl": "c4", "kavg_ms": kern / n, "moved_bytes": moved / n,
            "reread_bytes": sum(p["reread_bytes"] for p in per_round) / n, "kernel": "k", "launches": n,
            "kernel_ms_total": kern, "steps": n, "elapsed": kern * 1e-3 * 1.01, "rounds_per_launch": 1.0,
            "s8d_bytes": 9.125e9, "per_round": per_round, "replay": False, "lanes": lanes}


def test_roofline_is_model_bytes_over_kernel_time():
    rows = [{"round": r, "kernel_ms": 0.1 if r >= 4 else 1.0, "launches": 1,
             "model_bytes": 8e8 if r >= 4 else 4e9, "reread_bytes": 0 if r >= 4 else 1e9} for r in range(6)]
    r = _r(rows)
    out = bench.roofline(r, window=None)
    t = r["kavg_ms"] * 1e-3
    assert out["frac"] == pytest.approx(r["moved_bytes"] / t / 1e9 / bench.HBM_PEAK_GBS)
    assert out["frac"] <= 1.0 and out["traffic"] is None
    kinds = out["round_kinds"]
    assert kinds["klazy"]["rounds"] == [4, 5] and kinds["storm"]["rounds"] == [1, 2, 3]
    # 8e8 B in 0.1 ms = 8 TB/s: the klazy rows sit exactly at the peak
    assert kinds["klazy"]["fracs"]["model"] == pytest.approx(1.0)
    assert kinds["storm"]["fracs"]["hbm_compulsory"] == pytest.approx(3e9 / 1e-3 / 1e9 / bench.HBM_PEAK_GBS)
    assert out["host_gap_ms_per_step"] > 0


def test_pmc_summary_used_only_when_digest_and_window_match(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "PMC_DIR", str(tmp_path))
    good = {"src_sha": bench.src_digest(), "window": "5+20", "fabric_bytes_per_launch": 1.0}
    (tmp_path / "pmc_c4.json").write_text(json.dumps(good))
    assert bench.load_pmc("c4", "5+20", 1)["fabric_bytes_per_launch"] == 1.0
    assert bench.load_pmc("c4", "0+5", 1) is None      # another window
    assert bench.load_pmc("c4", "5+20", 2) is None     # multi-rank lines carry no single-GPU PMC
    (tmp_path / "pmc_c4.json").write_text(json.dumps(dict(good, src_sha="0" * 16)))
    assert bench.load_pmc("c4", "5+20", 1) is None     # other kernel sources


def test_committed_pmc_summaries_are_well_formed():
    d = bench.PMC_DIR
    files = [f for f in os.listdir(d) if f.startswith("pmc_") and f.endswith(".json")] if os.path.isdir(d) else []
    for f in files:
        pm = json.load(open(os.path.join(d, f)))
        assert pm["window"] == "5+20" and len(pm["src_sha"]) == 16
        assert pm["fabric_bytes_per_launch"] > 0 and 0 < pm["issue"]["frac_valu"] < 1
        assert all(src.startswith(os.path.relpath(d, ROOT) + "/") for src in pm["source"].values())


def test_cpu_baseline_threads_respect_the_quota():
    hc = bench.host_cpus()
    assert 1 <= hc["threads"] <= hc["affinity_cpus"]
    if hc["cgroup_cpu_quota"]:
        assert hc["threads"] <= max(1, round(hc["cgroup_cpu_quota"]))


def test_gpus_n_without_launcher_spawns_ranks(monkeypatch):
    """`python3 bench.py --gpus 2` with no torch.distributed.run around it starts ONE child
    process running the same bench under torch.distributed.run with 2 ranks (rendezvous on
    127.0.0.1), before any GPU call, and exits with the child's status."""
    calls = []

    def fake_call(cmd):
        calls.append(cmd)
        return 7

    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench.subprocess, "call", fake_call)
    monkeypatch.setattr(bench.torch.cuda, "set_device", lambda *a: pytest.fail("GPU touched before the spawn"))
    with pytest.raises(SystemExit) as ex:
        bench.main(["--gpus", "2", "--steps", "3", "--rehearse-one-gpu"])
    assert ex.value.code == 7
    assert len(calls) == 1
    cmd = calls[0]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "2", "--steps", "3", "--rehearse-one-gpu"]


def test_launcher_present_runs_in_process(monkeypatch):
    """Under a launcher (WORLD_SIZE set) nothing is spawned; a mismatch is refused."""
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: pytest.fail("spawned under a launcher"))
    with pytest.raises(SystemExit) as ex:
        bench.main(["--gpus", "2"])
    assert "WORLD_SIZE=4" in str(ex.value.code)


def test_exchange_model_per_link_bytes():
    changed = [{"round": 0, "words": 1000, "segments": 100}, {"round": 1, "words": 0, "segments": 0}]
    m = bench.exchange_model(changed, n=1_000_000, ps=32)
    # g8: 100 segments / 8 ranks * 64 B per link
    assert m["g8"]["push_bytes_per_link_max"] == pytest.approx(100 / 8 * 64)
    assert m["g8"]["push_ms_per_round_max"] == pytest.approx(100 / 8 * 64 / (bench.XGMI_LINK_GBS * 1e9) * 1e3)
    assert m["g2"]["allgather_ms_per_round"] == pytest.approx(500_000 * 128 / (bench.XGMI_LINK_GBS * 1e9) * 1e3)
    assert bench.exchange_model(None, 10, 1) is None


def test_line_roofline_is_compact():
    rows = [{"round": r, "kernel_ms": 0.1 if r >= 4 else 1.0, "launches": 1,
             "model_bytes": 8e8 if r >= 4 else 4e9, "reread_bytes": 0} for r in range(6)]
    full = bench.roofline(_r(rows), window=None)
    c = bench.compact_roofline(full)
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in c
    assert set(c["kinds"]) == {"fresh", "storm", "klazy"}
    assert len(json.dumps(c)) < 900


def test_log_capacity_follows_the_shard():
    full = bench.log_capacity(1_000_000, 1000, 1, 0, "targets")
    assert full == int(1.25 * 1_000_000 * 1000) + (1 << 20)
    # target shards: the rank's targets (whole 32-target blocks), not the network's
    parts = [bench.log_capacity(1_000_000, 1000, 4, r, "targets") for r in range(4)]
    assert all(p < full / 3 for p in parts)
    assert sum(p - (1 << 20) for p in parts) == int(1.25 * 1_000_000 * 1000)
    # node shards: the rank's nodes
    assert bench.log_capacity(1_000_000, 1000, 8, 3, "peers") == int(1.25 * 125_000 * 1000) + (1 << 20)
    # capped below 2^31 entries per engine
    assert bench.log_capacity(10_000_000, 256, 1, 0, "targets") == (1 << 31) - 1


def test_window_segments_split_at_epochs():
    """The timed window's segments (the log is sized for the largest): steps
    W..W+K-1 are rounds p % 16 of fresh epochs, split where an epoch starts."""
    import bench
    assert bench.window_segments(5, 20) == [list(range(5, 16)), list(range(0, 9))]
    assert bench.window_segments(0, 16) == [list(range(16))]
    assert bench.window_segments(16, 3) == [[0, 1, 2]]
    assert bench.window_segments(15, 2) == [[15], [0]]


def test_shard_auto_per_workload():
    """--shard auto: target shards except the conflicting workloads at 8 ranks
    (node shards with the need-masked push), as measured."""
    import bench
    assert bench.shard_for("c4", 1, "auto") == "targets"
    assert bench.shard_for("c4", 8, "auto") == "targets"
    assert bench.shard_for("c4p", 8, "auto") == "peers"
    assert bench.shard_for("c4pb", 8, "auto") == "peers"
    assert bench.shard_for("c4p", 4, "auto") == "targets"
    assert bench.shard_for("c4p", 8, "nodes") == "nodes"


def test_compact_delivery_fields():
    """The line's `delivery` summary: the on-device digest rate, the host fetch rates into pageable
    and pinned memory, the vote-record rate with every round's compact stream delivered pipelined
    (and expanded into packed words), and the unpipelined packed-word rate."""
    import bench
    d = {"digest_updates_per_s": 1e10,
         "pageable": {"updates_per_s": 3e9, "delivered_votes_per_s": 2e11},
         "pinned": {"updates_per_s": 5e9, "delivered_votes_per_s": 4e11},
         "compact": {"votes_per_s": 1.9e12, "votes_per_s_expanded": 1.1e12, "bytes_per_update": 2.1}}
    c = bench.compact_delivery(d)
    assert c == {"digest_updates_per_s": 1e10, "fetch_updates_per_s": {"pageable": 3e9, "pinned": 5e9},
                 "votes_per_s_with_fetch": 1.9e12, "votes_per_s_with_fetch_words": 1.1e12,
                 "votes_per_s_with_fetch_unpipelined": 4e11, "compact_bytes_per_update": 2.1}


def test_size_log_covers_any_single_round():
    """the log holds at least the fullest single round of the epoch (the delivery pass
    fetches rounds 0-3 one at a time), whatever the timed window."""
    import bench

    class E:
        def synchronize(self):
            pass

        def discard_updates(self):
            pass

        def resize_log(self, *ent):
            self.ent = ent
    per_round = {r: (10, 20, 30) for r in range(16)}
    per_round[1] = (5_000_000, 6_000_000, 7_000_000)
    e = E()
    bench.size_log(e, per_round, 5, 10)  # window rounds 5..14: no storm round inside
    assert all(v >= int(1.3 * w) for v, w in zip(e.ent, per_round[1]))


def test_node_shard_run_length_only_for_conflicting_workloads():
    import bench
    assert bench.NODE_SHARD_TPW == {"c4p": 8, "c4pb": 8}
    assert "c4" not in bench.NODE_SHARD_TPW
