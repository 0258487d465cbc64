"""Engine bookkeeping around the round kernels, checked against host-side
restatements: the StatusUpdate log's shard layout (every writer wave gets a
shard of its own, so the usable capacity is the requested one), the
changed-published-word counter (av_changed_words: what a peer-push round sends,
DESIGN.md §5) against a host diff of the published snapshots, and the deferred
state's write-back (av_materialize) leaving every result unchanged.

The log is the reference's `*[]StatusUpdate` out-parameter (processor.go:61,
111); the published snapshot is what the responder answers from (IsAccepted,
processor.go:125-130, main.go:179-182)."""
import numpy as np
import pytest

import avhip

pytestmark = pytest.mark.gpu

P80 = int(0.8 * 2**32)
BYZ20 = int(0.2 * 2**32)


def digest_round0(n, m, init, cap, opts=()):
    e = avhip.Engine(n, m, k=8, seed=0xA7A1A9C4, log_capacity=cap)
    for name, v in opts:
        e.set_option(name, v)
    e.init_records(init, P80)
    e.run_rounds(1)
    e.synchronize()
    out = (e.log_overflowed(), e.updates_digest(), e.updates_count())
    e.close()
    return out


@pytest.mark.parametrize("init", [avhip.INIT_BERNOULLI, avhip.INIT_PAIRS])
@pytest.mark.parametrize("opts", [(), (("tiles_per_wave", 16),), (("sweep_blocks", 40),)],
                         ids=["default", "tpw16", "blocks40"])
def test_log_capacity_is_usable(init, opts):
    """A small engine (4000 x 1000: 1000 tiles, a few hundred sweep waves) holds
    one round's updates in a log 1.3x their number: the shards follow the
    sweep's writer waves (1000 shards for ~250 waves left 3/4 of
    the capacity unreachable and overflowed here)."""
    n, m = 4000, 1000
    ovf, dig, cnt = digest_round0(n, m, init, 1 << 24, opts)
    assert not ovf and cnt > 100_000
    ovf2, dig2, cnt2 = digest_round0(n, m, init, int(cnt * 1.3), opts)
    assert not ovf2, f"log of {int(cnt * 1.3)} entries overflowed with {cnt} updates"
    assert (dig2, cnt2) == (dig, cnt)


def test_log_default_capacity_conflicting_round():
    """The default capacity (8 entries per 32-record lane, at least 2^20) holds a
    conflicting round of a small engine (double-spend pairs, ~0.1 updates per
    record) with no explicit size."""
    ovf, _, cnt = digest_round0(8000, 1000, avhip.INIT_PAIRS, 0)
    assert not ovf and cnt > 200_000


def test_log_relayout_waits_for_empty_log():
    """A grid option changed while updates are pending keeps their layout (fetch
    reads them back intact); the re-sharding happens once the log is empty."""
    n, m = 4000, 1000
    e = avhip.Engine(n, m, k=8, seed=7, log_capacity=1 << 24)
    ref = avhip.Engine(n, m, k=8, seed=7, log_capacity=1 << 24)
    for x in (e, ref):
        x.init_records(avhip.INIT_PAIRS, 0)
        x.run_rounds(2)
    e.set_option("tiles_per_wave", 16)  # log not empty: layout kept until the fetch
    a, b = e.fetch_updates(decode=False), ref.fetch_updates(decode=False)
    assert np.array_equal(a, b)
    for x in (e, ref):
        x.run_rounds(1)
    a, b = e.fetch_updates(decode=False), ref.fetch_updates(decode=False)
    assert np.array_equal(a, b)
    e.close()
    ref.close()


def host_changed(snaps, r, bl):
    """Published words of round r's output S_{r+1} that differ from the buffer it
    overwrites (S_{r-2}; zeros before round 2 on a fresh engine), and the 16-word
    row segments holding one."""
    new = snaps[r + 1]
    old = snaps[r - 2] if r >= 2 else np.zeros_like(new)
    d = new != old
    words = int(d.sum())
    pad = (-bl) % 16
    seg = np.pad(d, ((0, 0), (0, pad))).reshape(d.shape[0], -1, 16).any(axis=2)
    return words, int(seg.sum())


@pytest.mark.parametrize("case", [
    dict(init=avhip.INIT_BERNOULLI, byz=0, m=1000),   # storm, then settled (klazy, kpend >= 2 shortcut)
    dict(init=avhip.INIT_PAIRS, byz=BYZ20, m=1000),   # Byzantine rows: pattern words every round
    dict(init=avhip.INIT_BERNOULLI, byz=0, m=512),    # BL 16
], ids=["c4", "c4pb", "bl16"])
def test_changed_words_match_host_diff(case):
    """Option count_changed: per sweep round, av_changed_words' words and 64-B
    segments equal a host diff of the published snapshots S_{r+1} vs S_{r-2}
    (the `known` shortcut of publish() decides what is counted and
    pushed without loading the overwritten word)."""
    n, m = 3000, case["m"]
    e = avhip.Engine(n, m, k=8, seed=11, byz_threshold=case["byz"], log_capacity=1 << 24)
    e.set_option("count_changed", 1)
    e.init_records(case["init"], P80)
    bl = e.layout_info()["local_blocks"]
    snaps = [e.read_pref_words()]
    seen_zero = False
    for r in range(14):
        w0, g0 = e.changed_words()
        e.run_rounds(1)
        w1, g1 = e.changed_words()
        e.discard_updates()
        snaps.append(e.read_pref_words())
        hw, hg = host_changed(snaps, r, bl)
        assert (w1 - w0, g1 - g0) == (hw, hg), f"round {r}"
        seen_zero |= hw == 0
    if case["byz"] == 0 and m == 1000:
        assert seen_zero  # the honest network settles: the shortcut path ran
    e.close()


@pytest.mark.parametrize("run", [1, 4, 16])
def test_materialize_leaves_results_unchanged(oracle, run):
    """av_materialize in the middle of a deferred stretch (stale vote planes,
    pending count steps): records, digests and every later round identical to
    an engine that never wrote back, and to the oracle; k_materialize taking 1,
    4 or 16 tiles per wave (option materialize_run)."""
    n, m = 2000, 1000
    a = avhip.Engine(n, m, k=8, seed=5, log_capacity=1 << 24)
    a.set_option("materialize_run", run)
    b = avhip.Engine(n, m, k=8, seed=5, log_capacity=1 << 24)
    sim = oracle.Sim(n, m, 8, seed=5, init_mode=avhip.INIT_BERNOULLI, init_param=P80)
    for x in (a, b):
        x.init_records(avhip.INIT_BERNOULLI, P80)
        x.run_rounds(8)
    for _ in range(8):
        sim.run_round()
    before = a.read_records()
    dig = a.updates_digest()
    a.materialize()
    assert np.array_equal(a.read_records(), before)
    assert a.updates_digest() == dig
    assert np.array_equal(before, sim.dump())
    for x in (a, b):
        x.run_rounds(12)  # through kconsume and finalization
    for _ in range(12):
        sim.run_round()
    assert np.array_equal(a.read_records(), b.read_records())
    assert np.array_equal(a.read_records(), sim.dump())
    assert a.updates_digest() == b.updates_digest()
    a.close()
    b.close()


def test_solo_barrier_is_sticky():
    """Once the diagnostics option solo_barrier has run (it allocates the
    arrival slots and advances the barrier sequence), the engine refuses to
    join a peer exchange even after the option is cleared: its
    snapshot buffers were never moved to fine-grained memory and its sequence
    numbers would not match its peers'."""
    e = avhip.Engine(256, 64, k=8, seed=3)
    e.init_records(avhip.INIT_BERNOULLI, P80)
    e.set_option("solo_barrier", 1)
    e.run_rounds(2)
    e.set_option("solo_barrier", 0)
    with pytest.raises(avhip.AvError):
        e.peer_handles()
    e.close()


@pytest.mark.parametrize("n,m", [(6000, 1000), (5000, 2000)], ids=["even", "uneven_writers"])
def test_resize_log_one_entry_per_lane(n, m):
    """A log of two single words and one record per lane holds any single round
    (a lane's updates of a round are one record, or at most two single words),
    here the storm round of conflicting pairs, whose lanes mostly log exactly
    two words; av_log_entries counts them by kind; a log holding updates is not
    re-sized. 5000 x 2000 (BL 63: 1231 writer waves over 256 shards) gives
    some shards one writer more than others: the sizing serves the fullest
    shard (C3's bench log overflowed at one entry per lane before)."""
    e = avhip.Engine(n, m, k=8, seed=9, log_capacity=1 << 20)
    lanes = e.layout_info()["lanes"]
    e.resize_log(2 * lanes, lanes, lanes)
    ref = avhip.Engine(n, m, k=8, seed=9, log_capacity=1 << 26)
    for x in (e, ref):
        x.init_records(avhip.INIT_PAIRS, 0)
    for r in range(4):
        for x in (e, ref):
            x.run_rounds(1)
        ent = e.log_entries()
        assert not e.log_overflowed()
        assert 0 < sum(ent) <= e.updates_count() and ent[0] <= 2 * lanes and max(ent[1:]) <= lanes
        if r == 1:
            with pytest.raises(avhip.AvError):
                e.resize_log(2 * lanes, lanes, lanes)
        assert np.array_equal(e.fetch_updates(decode=False), ref.fetch_updates(decode=False))
    # sized below one round's needs: the overflow is reported, never silent
    e.resize_log(16, 16, 16)
    e.run_rounds(1)
    assert e.log_overflowed()
    with pytest.raises(avhip.LogOverflow):
        e.fetch_updates()
    e.close()
    ref.close()
