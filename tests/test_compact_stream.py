"""The compact StatusUpdate stream's host side (av_compact_expand, include/avhip.h)
on CPU: streams laid out by the test-side restatement (compact_ref.py) of the
format expand to exactly the packed words they were made from (canonical
(round, node, slot, target) order, processor.go:94,111), for 2- and 4-byte
codes, several rounds and index chunks, empty and one-update streams; malformed
streams are refused. No GPU: av_compact_expand is host code."""
import ctypes as C

import numpy as np
import pytest

import avhip
from compact_ref import encode


def random_words(rng, *, n_rounds, node_base, n_local, target_base, n_targets_local, k, density):
    rows = []
    for r in range(n_rounds):
        for nl in range(n_local):
            if rng.random() >= density:
                continue
            nu = int(rng.integers(1, 12))
            for _ in range(nu):
                rows.append((r, node_base + nl, int(rng.integers(0, k)),
                             target_base + int(rng.integers(0, n_targets_local)), int(rng.integers(0, 4))))
    if not rows:
        return np.zeros(0, np.uint64)
    a = np.array(rows, np.uint64)
    w = (a[:, 0] << np.uint64(52)) | (a[:, 1] << np.uint64(28)) | (a[:, 2] << np.uint64(24)) | \
        (a[:, 3] << np.uint64(2)) | a[:, 4]
    # (round, node, slot, target) is unique per update: drop duplicate keys, keep one status
    key = w >> np.uint64(2)
    _, first = np.unique(key, return_index=True)
    return np.sort(w[first])


CASES = [
    # rounds, node_base, nodes, target_base, targets, k, density
    (1, 0, 100, 0, 1000, 8, 0.6),       # C4-like: 2-B codes
    (3, 500, 9000, 64, 300, 8, 0.05),   # three rounds, three index chunks per round, a target shard
    (2, 0, 50, 0, 10_000, 8, 0.9),      # C2-like: 4-B codes (3 + 14 + 2 bits)
    (1, 7, 20, 0, 4096, 16, 0.5),       # k = 16: 4 slot bits, 4-B codes
    (4, 0, 30, 0, 33, 1, 0.7),          # k = 1: no slot bits
    (1, 0, 64, 0, 2000, 8, 0.0),        # no updates at all
]


@pytest.mark.parametrize("case", CASES)
def test_expand_inverts_encode(case):
    R, nb, nl, tb, tl, k, dens = case
    rng = np.random.default_rng(hash(case) & 0xFFFF)
    w = random_words(rng, n_rounds=R, node_base=nb, n_local=nl, target_base=tb, n_targets_local=tl, k=k,
                     density=dens)
    s = encode(w, log_base=17, n_rounds=R, node_base=nb, n_local=nl, target_base=tb, n_targets_local=tl, k=k)
    h = avhip.compact_header(s)
    assert h["n_updates"] == w.size and h["bytes"] == s.size and h["log_base"] == 17
    assert h["code_bytes"] == (2 if (k - 1).bit_length() + (tl - 1).bit_length() + 2 <= 16 else 4)
    got = avhip.compact_expand(s)
    assert np.array_equal(got, w)
    if w.size:  # ~2-4 B per update against 8 B per packed word
        assert s.size < 8 * w.size + 80 + 16 * (R * -(-nl // 4096) + 1)


def test_one_update():
    w = np.array([(0 << 52) | (5 << 28) | (3 << 24) | (77 << 2) | 2], np.uint64)
    s = encode(w, log_base=0, n_rounds=1, node_base=0, n_local=10, target_base=0, n_targets_local=100, k=8)
    assert np.array_equal(avhip.compact_expand(s), w)


def _expand_rc(s, cap=None):
    b = np.ascontiguousarray(s, np.uint8)
    n = C.c_int64(0)
    out = np.zeros(max(1, cap or 1 << 16), np.uint64)
    rc = avhip.lib().av_compact_expand(b.ctypes.data_as(C.c_void_p), b.size, out.ctypes.data_as(C.c_void_p),
                                       out.size if cap is None else cap, C.byref(n))
    return rc, n.value


def test_malformed_streams_are_refused():
    rng = np.random.default_rng(3)
    w = random_words(rng, n_rounds=2, node_base=0, n_local=40, target_base=0, n_targets_local=500, k=8, density=0.5)
    s = encode(w, log_base=0, n_rounds=2, node_base=0, n_local=40, target_base=0, n_targets_local=500, k=8)
    assert _expand_rc(s) == (0, w.size)
    bad = s.copy()
    bad[0] ^= 1  # magic
    assert _expand_rc(bad)[0] == -1
    assert _expand_rc(s[:-4])[0] == -1  # truncated: the header's byte count disagrees
    bad = s.copy()
    hdr = avhip.COMPACT_HEADER.itemsize
    idx_end = hdr + 16 * (2 * 1 + 1)
    bad[idx_end + 4] ^= 0x7F  # first group's count corrupted
    assert _expand_rc(bad)[0] == -1
    rc, n = _expand_rc(s, cap=max(0, w.size - 1))  # caller buffer too small
    assert rc == avhip.AV_ERR_OVERFLOW and n == w.size


def test_wide_node_field():
    """Networks of >= 2^24 nodes: the words' round field starts at bit 53 (include/avhip.h)."""
    rs = 53
    rows = np.array([(0, (1 << 24) + 5, 3, 17, 2), (1, 3, 0, 1, 1), (1, (1 << 25) - 1, 7, 63, 0)], np.uint64)
    w = (rows[:, 0] << np.uint64(rs)) | (rows[:, 1] << np.uint64(28)) | (rows[:, 2] << np.uint64(24)) | \
        (rows[:, 3] << np.uint64(2)) | rows[:, 4]
    s = encode(w, log_base=9, n_rounds=2, node_base=0, n_local=1 << 25, target_base=0, n_targets_local=64, k=8,
               round_shift=rs)
    assert avhip.compact_header(s)["round_shift"] == rs
    got = avhip.compact_expand(s)
    assert np.array_equal(got, w)
    assert np.array_equal(avhip.decode_updates(got, 9, rs), rows.astype(np.int64) + np.array([9, 0, 0, 0, 0]))
