"""ctypes binding of libavhip.so (include/avhip.h) — the MI355X batched
Avalanche voting engine.

This is a thin host-side mirror of the C ABI used by bench.py and the tests.
It never falls back to anything else: if libavhip.so cannot be loaded, or a
call fails, an exception is raised.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

try:  # share torch's HIP runtime (same soname) when torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the binding itself
    torch = None

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# AVHIP_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("AVHIP_LIB") or os.path.join(_PKG_ROOT, "lib", "libavhip.so")
HEADER_PATH = os.path.join(os.path.dirname(_PKG_ROOT), "include", "avhip.h")

AV_OK = 0
AV_ERR_NOT_FOUND = -4
AV_ERR_OVERFLOW = -5
AV_ERR_PEER = -8

STATUS_INVALID, STATUS_REJECTED, STATUS_ACCEPTED, STATUS_FINALIZED = 0, 1, 2, 3
PEERS_RANDOM, PEERS_ROUND_ROBIN = 0, 1
INIT_NONE, INIT_REJECTED, INIT_ACCEPTED, INIT_BERNOULLI, INIT_PAIRS = 0, 1, 2, 3, 4
ABSENT_WORD = 0xFFFE0000
FINALIZATION_SCORE = 128
MAX_ELEMENT_POLL = 4096


class AvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"avhip error {code}: {msg}")
        self.code = code


class VoteRecordNotFound(AvError):
    """The reference panics with "VoteRecord not found" (processor.go:136)."""


class LogOverflow(AvError):
    pass


class PeerExchangeFailed(AvError):
    """A rank missed a peer barrier: the engine refuses further rounds and results."""


class Config(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int64),
        ("n_targets", C.c_int64),
        ("k", C.c_int32),
        ("peer_mode", C.c_int32),
        ("seed", C.c_uint64),
        ("byz_threshold", C.c_uint32),
        ("device", C.c_int32),
        ("node_begin", C.c_int64),
        ("node_end", C.c_int64),
        ("target_begin", C.c_int64),
        ("target_end", C.c_int64),
        ("update_log_capacity", C.c_int64),
    ]


# every symbol declared in include/avhip.h (non-inline)
PEER_HANDLE_BYTES = 320  # include/avhip.h AV_PEER_HANDLE_BYTES

EXPORTED = [
    "av_abi_version", "av_config_init", "av_create", "av_destroy", "av_strerror", "av_last_error",
    "av_init_records", "av_add_targets", "av_set_valid", "av_register_votes", "av_is_accepted",
    "av_get_confidence", "av_get_invs", "av_get_invs_batch", "av_run_rounds", "av_replay_round_errs", "av_replay_prepare",
    "av_replay_rounds", "av_synchronize", "av_round_index", "av_updates_count", "av_fetch_updates",
    "av_update_log_overflowed", "av_applied_votes", "av_alg_bytes", "av_alg_bytes_reread", "av_finalized_count", "av_live_records", "av_discard_updates", "av_read_records", "av_write_records", "av_read_pref", "av_sample_peers",
    "av_set_option", "av_set_timing", "av_kernel_stats", "av_layout_info", "av_comm_unique_id", "av_comm_init",
    "av_peer_handles", "av_peer_init", "av_get_round", "av_set_round", "av_log_base_round", "av_updates_digest",
    "av_updates_digest_range", "av_read_pref_words", "av_set_polling",
    "av_register_votes_batch", "av_changed_words", "av_materialize", "av_peer_group_serial", "av_peer_sync",
    "av_pushed_words", "av_log_entries", "av_resize_log", "av_fetch_compact", "av_fetch_compact_async",
    "av_fetch_compact_wait", "av_compact_expand", "av_update_round_shift",
]

_lib = None
_vp = C.c_void_p


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OSError(f"libavhip.so not built at {LIB_PATH} (run __graft_entry__.build() or make -C go-avalanche_amd)")
    L = C.CDLL(LIB_PATH)
    i64, i32, u32 = C.c_int64, C.c_int32, C.c_uint32
    P = C.POINTER
    sig = {
        "av_abi_version": (i32, []),
        "av_config_init": (None, [P(Config)]),
        "av_create": (i32, [P(Config), P(_vp)]),
        "av_destroy": (i32, [_vp]),
        "av_strerror": (C.c_char_p, [i32]),
        "av_last_error": (C.c_char_p, []),
        "av_init_records": (i32, [_vp, i32, u32]),
        "av_add_targets": (i32, [_vp, i64, _vp, _vp, i64, _vp]),
        "av_set_valid": (i32, [_vp, i64, i32]),
        "av_register_votes": (i32, [_vp, i64, _vp, _vp, i64, _vp]),
        "av_is_accepted": (i32, [_vp, i64, i64, P(i32)]),
        "av_get_confidence": (i32, [_vp, i64, i64, P(C.c_uint16)]),
        "av_get_invs": (i32, [_vp, i64, _vp, i64, P(i64)]),
        "av_get_invs_batch": (i32, [_vp, i64, i64, _vp, _vp, i64, P(i64)]),
        "av_run_rounds": (i32, [_vp, i32]),
        "av_replay_round_errs": (i32, [_vp, _vp]),
        "av_replay_prepare": (i32, [_vp, i32]),
        "av_replay_rounds": (i32, [_vp, i32]),
        "av_synchronize": (i32, [_vp]),
        "av_round_index": (i32, [_vp, P(i64)]),
        "av_updates_count": (i32, [_vp, P(i64)]),
        "av_fetch_updates": (i32, [_vp, _vp, i64, P(i64)]),
        "av_update_log_overflowed": (i32, [_vp, P(i32)]),
        "av_applied_votes": (i32, [_vp, P(i64)]),
        "av_alg_bytes": (i32, [_vp, P(i64)]),
        "av_alg_bytes_reread": (i32, [_vp, P(i64)]),
        "av_changed_words": (i32, [_vp, P(i64), P(i64)]),
        "av_materialize": (i32, [_vp]),
        "av_finalized_count": (i32, [_vp, P(i64)]),
        "av_live_records": (i32, [_vp, i32, P(i64)]),
        "av_discard_updates": (i32, [_vp]),
        "av_read_records": (i32, [_vp, i64, i64, i64, i64, _vp]),
        "av_write_records": (i32, [_vp, i64, i64, i64, i64, _vp]),
        "av_read_pref": (i32, [_vp, i64, i64, i64, i64, _vp]),
        "av_sample_peers": (i32, [_vp, i64, i64, i64, _vp]),
        "av_set_option": (i32, [_vp, C.c_char_p, i64]),
        "av_set_timing": (i32, [_vp, i32]),
        "av_kernel_stats": (i32, [_vp, P(C.c_double), P(i64)]),
        "av_layout_info": (i32, [_vp, P(i64), P(i64), P(i64), P(i32)]),
        "av_comm_unique_id": (i32, [_vp]),
        "av_comm_init": (i32, [_vp, i32, i32, _vp]),
        "av_peer_handles": (i32, [_vp, _vp]),
        "av_peer_init": (i32, [_vp, i32, i32, _vp]),
        "av_get_round": (i32, [_vp, i64, P(i64)]),
        "av_set_round": (i32, [_vp, i64, i64]),
        "av_log_base_round": (i32, [_vp, P(i64)]),
        "av_updates_digest": (i32, [_vp, _vp]),
        "av_updates_digest_range": (i32, [_vp, i64, i64, _vp]),
        "av_read_pref_words": (i32, [_vp, i64, i64, _vp]),
        "av_set_polling": (i32, [_vp, i64, i32]),
        "av_register_votes_batch": (i32, [_vp, i64, _vp, _vp, _vp, _vp, _vp]),
        "av_peer_group_serial": (i32, [_vp, i32]),
        "av_peer_sync": (i32, [_vp]),
        "av_pushed_words": (i32, [_vp, P(i64)]),
        "av_log_entries": (i32, [_vp, _vp]),
        "av_resize_log": (i32, [_vp, _vp]),
        "av_fetch_compact": (i32, [_vp, _vp, i64, P(i64)]),
        "av_fetch_compact_async": (i32, [_vp, P(i64)]),
        "av_fetch_compact_wait": (i32, [_vp, i64, P(_vp), P(i64)]),
        "av_compact_expand": (i32, [_vp, i64, _vp, i64, P(i64)]),
        "av_update_round_shift": (i32, [_vp, P(i32)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc):
    if rc == AV_OK:
        return
    msg = lib().av_last_error().decode(errors="replace")
    if rc == AV_ERR_NOT_FOUND:
        raise VoteRecordNotFound(rc, msg)
    if rc == AV_ERR_OVERFLOW:
        raise LogOverflow(rc, msg)
    if rc == AV_ERR_PEER:
        raise PeerExchangeFailed(rc, msg)
    raise AvError(rc, msg)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_vp)


def decode_updates(u: np.ndarray, base_round: int = 0, round_shift: int = 52) -> np.ndarray:
    """Packed update words -> int64[n, 5] (round, node, slot, target, status); round_shift = the
    engine's (av_update_round_shift: 52 below 2^24 nodes)."""
    u = np.asarray(u, np.uint64)
    out = np.empty((u.size, 5), np.int64)
    out[:, 0] = (u >> np.uint64(round_shift)).astype(np.int64) + base_round
    out[:, 1] = ((u >> np.uint64(28)) & np.uint64((1 << (round_shift - 28)) - 1)).astype(np.int64)
    out[:, 2] = ((u >> np.uint64(24)) & np.uint64(0xF)).astype(np.int64)
    out[:, 3] = ((u >> np.uint64(2)) & np.uint64(0x3FFFFF)).astype(np.int64)
    out[:, 4] = (u & np.uint64(3)).astype(np.int64)
    return out


COMPACT_MAGIC = 0x31435641  # include/avhip.h AV_COMPACT_MAGIC
COMPACT_HEADER = np.dtype([("magic", "<u4"), ("version", "<u4"), ("log_base", "<i8"), ("n_updates", "<i8"),
                           ("bytes", "<i8"), ("node_base", "<i8"), ("target_base", "<i8"), ("n_rounds", "<i4"),
                           ("chunks", "<i4"), ("chunk_nodes", "<i4"), ("code_bytes", "<i4"),
                           ("target_bits", "<i4"), ("slot_bits", "<i4"), ("round_shift", "<i4"),
                           ("reserved", "<i4")])
assert COMPACT_HEADER.itemsize == 80


def compact_header(stream) -> dict:
    """The av_compact_header of a compact StatusUpdate stream, as a dict."""
    h = np.frombuffer(memoryview(stream)[:COMPACT_HEADER.itemsize], COMPACT_HEADER)[0]
    return {k: int(h[k]) for k in COMPACT_HEADER.names}


def compact_expand(stream) -> np.ndarray:
    """av_compact_expand: a compact stream -> the packed update words av_fetch_updates returns."""
    b = np.frombuffer(stream, np.uint8)
    n = compact_header(b)["n_updates"]
    out = np.zeros(max(n, 1), np.uint64)
    got = C.c_int64(0)
    _check(lib().av_compact_expand(_ptr(b), b.size, _ptr(out), out.size, C.byref(got)))
    return out[: got.value]


def compact_expand_into(stream, words: np.ndarray) -> int:
    """av_compact_expand into the caller's uint64 buffer; returns the number of updates."""
    assert words.dtype == np.uint64 and words.flags.c_contiguous
    b = np.frombuffer(stream, np.uint8) if not isinstance(stream, np.ndarray) else stream
    got = C.c_int64(0)
    _check(lib().av_compact_expand(_ptr(b), b.size, _ptr(words), words.size, C.byref(got)))
    return got.value


def comm_unique_id() -> bytes:
    buf = (C.c_uint8 * 128)()
    _check(lib().av_comm_unique_id(C.cast(buf, _vp)))
    return bytes(buf)


def peer_group_serial(engines):
    """Make the node-shard engines of one network (rank order) one in-process
    peer group on one device (av_peer_group_serial): every rank's round pushes
    into the others' buffers; run round r of every rank in rank order."""
    arr = (_vp * len(engines))(*[e._h for e in engines])
    _check(lib().av_peer_group_serial(C.cast(arr, _vp), len(engines)))
    for e in engines:
        e._group = engines  # destroyed together (Engine.close closes the whole group)


def run_group_rounds(engines, rounds=1):
    """`rounds` synchronous rounds of a serial peer group: round r of rank 0, 1, .."""
    for _ in range(rounds):
        for e in engines:
            e.run_rounds(1)


class Engine:
    """One engine = N nodes x M targets of VoteRecords (or a shard) in HBM."""

    def __init__(self, n_nodes, n_targets, k=8, seed=0xA7A1A9C4, peer_mode=PEERS_RANDOM, byz_threshold=0,
                 device=0, node_range=None, target_range=None, log_capacity=0):
        cfg = Config()
        lib().av_config_init(C.byref(cfg))
        cfg.n_nodes, cfg.n_targets, cfg.k = n_nodes, n_targets, k
        cfg.peer_mode, cfg.seed, cfg.byz_threshold, cfg.device = peer_mode, seed, byz_threshold, device
        if node_range is not None:
            cfg.node_begin, cfg.node_end = node_range
        if target_range is not None:
            cfg.target_begin, cfg.target_end = target_range
        cfg.update_log_capacity = log_capacity
        h = _vp()
        _check(lib().av_create(C.byref(cfg), C.byref(h)))
        self._h = h
        self.n_nodes, self.n_targets, self.k = n_nodes, n_targets, k
        self.node_range = (cfg.node_begin, cfg.node_end) if node_range else (0, n_nodes)
        self.target_range = (cfg.target_begin, cfg.target_end) if target_range else (0, n_targets)

    def close(self):
        """Destroy the engine; a member of a serial peer group takes the whole group with it (the
        members store into each other's buffers: av_peer_group_serial)."""
        group = getattr(self, "_group", None)
        if group:
            for e in group:
                e._group = None
            for e in group:
                if e is not self:
                    e.close()
        if getattr(self, "_h", None):
            lib().av_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # ---- population ----
    def init_records(self, mode=INIT_BERNOULLI, param=0x80000000):
        _check(lib().av_init_records(self._h, mode, param))

    def add_targets(self, node, targets, accepted):
        t = np.ascontiguousarray(targets, np.int64)
        a = np.ascontiguousarray(accepted, np.uint8)
        out = np.zeros(max(1, t.size), np.uint8)
        _check(lib().av_add_targets(self._h, node, _ptr(t), _ptr(a), t.size, _ptr(out)))
        return out[: t.size].astype(bool)

    def set_valid(self, target, valid):
        _check(lib().av_set_valid(self._h, target, int(bool(valid))))

    # ---- one-node Processor methods ----
    def register_votes(self, node, targets, errs):
        t = np.ascontiguousarray(targets, np.int64)
        e = np.ascontiguousarray(errs, np.uint32)
        st = np.zeros(max(1, t.size), np.int32)
        _check(lib().av_register_votes(self._h, node, _ptr(t), _ptr(e), t.size, _ptr(st)))
        return st[: t.size]

    def register_votes_batch(self, nodes, offsets, targets, errs):
        """Many Responses in one call: Response i = node nodes[i], votes
        offsets[i]..offsets[i+1]-1. Returns the per-vote status (-1 = none)."""
        nd = np.ascontiguousarray(nodes, np.int64)
        of = np.ascontiguousarray(offsets, np.int64)
        t = np.ascontiguousarray(targets, np.int64)
        e = np.ascontiguousarray(errs, np.uint32)
        # the C entry point reads targets/errs up to offsets[n]: check the lengths here (not with
        # assert, which `python -O` strips)
        if of.size != nd.size + 1:
            raise ValueError(f"offsets has {of.size} entries, expected len(nodes) + 1 = {nd.size + 1}")
        if of[0] != 0 or np.any(np.diff(of) < 0):
            raise ValueError("offsets must start at 0 and be non-decreasing")
        if not (t.size == e.size == of[-1]):
            raise ValueError(f"targets ({t.size}) and errs ({e.size}) must both have offsets[-1] = {of[-1]} entries")
        st = np.zeros(max(1, t.size), np.int32)
        _check(lib().av_register_votes_batch(self._h, nd.size, _ptr(nd), _ptr(of), _ptr(t), _ptr(e), _ptr(st)))
        return st[: t.size]

    def is_accepted(self, node, target):
        out = C.c_int32(0)
        _check(lib().av_is_accepted(self._h, node, target, C.byref(out)))
        return bool(out.value)

    def get_confidence(self, node, target):
        out = C.c_uint16(0)
        _check(lib().av_get_confidence(self._h, node, target, C.byref(out)))
        return out.value

    def get_invs(self, node):
        buf = np.zeros(MAX_ELEMENT_POLL, np.int64)
        n = C.c_int64(0)
        _check(lib().av_get_invs(self._h, node, _ptr(buf), buf.size, C.byref(n)))
        return buf[: n.value].copy()

    def get_invs_batch(self, n0=None, n1=None):
        """Poll sets of nodes [n0, n1) as CSR (offsets int64[n+1], targets int32[total])."""
        n0 = self.node_range[0] if n0 is None else n0
        n1 = self.node_range[1] if n1 is None else n1
        offs = np.zeros(n1 - n0 + 1, np.int64)
        total = C.c_int64(0)
        rc = lib().av_get_invs_batch(self._h, n0, n1, _ptr(offs), None, 0, C.byref(total))
        if rc not in (AV_OK, AV_ERR_OVERFLOW):
            _check(rc)
        tg = np.zeros(max(total.value, 1), np.int32)
        _check(lib().av_get_invs_batch(self._h, n0, n1, _ptr(offs), _ptr(tg), tg.size, C.byref(total)))
        return offs, tg[: total.value]

    # ---- rounds ----
    def run_rounds(self, rounds=1):
        _check(lib().av_run_rounds(self._h, rounds))

    def replay_round_errs(self, errs):
        e = np.ascontiguousarray(errs, np.uint32)
        nl = self.node_range[1] - self.node_range[0]
        tl = self.target_range[1] - self.target_range[0]
        assert e.shape == (nl, self.k, tl), e.shape
        _check(lib().av_replay_round_errs(self._h, _ptr(e)))

    def replay_prepare(self, rounds):
        _check(lib().av_replay_prepare(self._h, rounds))

    def replay_rounds(self, rounds):
        _check(lib().av_replay_rounds(self._h, rounds))

    def synchronize(self):
        _check(lib().av_synchronize(self._h))

    def get_round(self, node):
        """Processor.GetRound of `node` (processor.go:40-42): a caller-set field."""
        out = C.c_int64(0)
        _check(lib().av_get_round(self._h, node, C.byref(out)))
        return out.value

    def set_round(self, node, rnd):
        _check(lib().av_set_round(self._h, node, rnd))

    def set_polling(self, node, polls):
        """Whether `node` polls in the rounds (the example's loop returns, main.go:160-162)."""
        _check(lib().av_set_polling(self._h, node, int(bool(polls))))

    @property
    def round(self):
        out = C.c_int64(0)
        _check(lib().av_round_index(self._h, C.byref(out)))
        return out.value

    # ---- outputs ----
    def updates_count(self):
        out = C.c_int64(0)
        _check(lib().av_updates_count(self._h, C.byref(out)))
        return out.value

    def log_base_round(self):
        """Round the pending log's round fields count from (kept by the engine:
        a fetch, a discard or an overflowed fetch moves it)."""
        out = C.c_int64(0)
        _check(lib().av_log_base_round(self._h, C.byref(out)))
        return out.value

    def fetch_updates(self, decode=True):
        """All StatusUpdates since the previous fetch in canonical order
        (sorted on the device)."""
        n = self.updates_count()
        buf = np.zeros(max(1, n), np.uint64)
        got = C.c_int64(0)
        base = self.log_base_round()
        _check(lib().av_fetch_updates(self._h, _ptr(buf), buf.size, C.byref(got)))
        buf = buf[: got.value]
        return decode_updates(buf, base, self.round_shift) if decode else buf

    @property
    def round_shift(self):
        """The update words' round field position (av_update_round_shift)."""
        out = C.c_int32(0)
        _check(lib().av_update_round_shift(self._h, C.byref(out)))
        return out.value

    def fetch_into(self, buf):
        """All pending StatusUpdates, packed and sorted canonical, into the caller's uint64 buffer
        (av_fetch_updates); returns how many."""
        assert buf.dtype == np.uint64 and buf.flags.c_contiguous
        got = C.c_int64(0)
        _check(lib().av_fetch_updates(self._h, _ptr(buf), buf.size, C.byref(got)))
        return got.value

    def fetch_compact(self):
        """All pending StatusUpdates as a compact stream (av_fetch_compact), as a uint8 array."""
        need = C.c_int64(0)
        rc = lib().av_fetch_compact(self._h, None, 0, C.byref(need))
        if rc not in (AV_OK, AV_ERR_OVERFLOW):
            _check(rc)
        buf = np.zeros(max(need.value, COMPACT_HEADER.itemsize), np.uint8)
        got = C.c_int64(0)
        _check(lib().av_fetch_compact(self._h, _ptr(buf), buf.size, C.byref(got)))
        return buf[: got.value]

    def fetch_compact_into(self, buf):
        """av_fetch_compact into the caller's uint8 buffer; returns the stream's bytes."""
        assert buf.dtype == np.uint8 and buf.flags.c_contiguous
        got = C.c_int64(0)
        _check(lib().av_fetch_compact(self._h, _ptr(buf), buf.size, C.byref(got)))
        return got.value

    def fetch_compact_async(self):
        """av_fetch_compact_async: encode the pending updates, start their copy, clear the log; a ticket."""
        t = C.c_int64(0)
        _check(lib().av_fetch_compact_async(self._h, C.byref(t)))
        return t.value

    def fetch_compact_wait(self, ticket, copy=True):
        """av_fetch_compact_wait: the ticket's stream. copy=False: a zero-copy view of the engine's
        pinned buffer (valid until the fetch_compact_async call two tickets later)."""
        p = _vp()
        n = C.c_int64(0)
        _check(lib().av_fetch_compact_wait(self._h, ticket, C.byref(p), C.byref(n)))
        view = np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint8)), shape=(n.value,))
        return view.copy() if copy else view

    def updates_digest(self, n0=None, n1=None):
        """(count, sum, xor) of splitmix64 over the pending packed updates (not
        cleared), of nodes [n0, n1) if given."""
        out = np.zeros(3, np.uint64)
        if n0 is None:
            _check(lib().av_updates_digest(self._h, _ptr(out)))
        else:
            _check(lib().av_updates_digest_range(self._h, n0, n1, _ptr(out)))
        return tuple(int(v) for v in out)

    def read_pref_words(self, n0=0, n1=None):
        """Round-start published rows as stored: uint32[n1-n0, BL] bitsets."""
        n1 = self.n_nodes if n1 is None else n1
        bl = self.layout_info()["local_blocks"]
        out = np.zeros((n1 - n0, bl), np.uint32)
        _check(lib().av_read_pref_words(self._h, n0, n1, _ptr(out)))
        return out

    def applied_votes(self):
        out = C.c_int64(0)
        _check(lib().av_applied_votes(self._h, C.byref(out)))
        return out.value

    def finalized_count(self):
        out = C.c_int64(0)
        _check(lib().av_finalized_count(self._h, C.byref(out)))
        return out.value

    def live_records(self, honest_only=False):
        out = C.c_int64(0)
        _check(lib().av_live_records(self._h, int(honest_only), C.byref(out)))
        return out.value

    def log_overflowed(self) -> bool:
        v = C.c_int32()
        _check(lib().av_update_log_overflowed(self._h, C.byref(v)))
        return bool(v.value)

    def discard_updates(self):
        _check(lib().av_discard_updates(self._h))

    def alg_bytes(self):
        out = C.c_int64(0)
        _check(lib().av_alg_bytes(self._h, C.byref(out)))
        return out.value

    def alg_bytes_reread(self):
        """Part of alg_bytes() that re-reads preference words already gathered in the same round."""
        out = C.c_int64(0)
        _check(lib().av_alg_bytes_reread(self._h, C.byref(out)))
        return out.value

    def changed_words(self):
        """(words, 64-B segments) of published words that changed in sweep rounds (pushed to every
        peer on a peer-push engine; counted on any engine with option count_changed=1)."""
        w, g = C.c_int64(0), C.c_int64(0)
        _check(lib().av_changed_words(self._h, C.byref(w), C.byref(g)))
        return w.value, g.value

    def log_entries(self):
        """Pending log entries per kind: (singles, slot records, dense records)."""
        out = np.zeros(3, np.int64)
        _check(lib().av_log_entries(self._h, _ptr(out)))
        return tuple(int(v) for v in out)

    def resize_log(self, singles, slots, dense):
        """Re-allocate the empty device log for that many entries of each kind."""
        v = np.array([singles, slots, dense], np.int64)
        _check(lib().av_resize_log(self._h, _ptr(v)))

    def pushed_words(self):
        """Words stored into peer replicas by sweep rounds (all peers together)."""
        out = C.c_int64(0)
        _check(lib().av_pushed_words(self._h, C.byref(out)))
        return out.value

    def peer_sync(self):
        """Collective: every rank's own rows pushed whole (replicas complete for reads)."""
        _check(lib().av_peer_sync(self._h))

    def materialize(self):
        """Write back the deferred state (stale vote planes, pending count steps) now."""
        _check(lib().av_materialize(self._h))

    def read_records(self, n0=None, n1=None, t0=None, t1=None):
        n0 = self.node_range[0] if n0 is None else n0
        n1 = self.node_range[1] if n1 is None else n1
        t0 = self.target_range[0] if t0 is None else t0
        t1 = self.target_range[1] if t1 is None else t1
        out = np.zeros((n1 - n0, t1 - t0), np.uint32)
        _check(lib().av_read_records(self._h, n0, n1, t0, t1, _ptr(out)))
        return out

    def write_records(self, words, n0=None, t0=None):
        w = np.ascontiguousarray(words, np.uint32)
        n0 = self.node_range[0] if n0 is None else n0
        t0 = self.target_range[0] if t0 is None else t0
        _check(lib().av_write_records(self._h, n0, n0 + w.shape[0], t0, t0 + w.shape[1], _ptr(w)))

    def read_pref(self, n0=0, n1=None, t0=None, t1=None):
        n1 = self.n_nodes if n1 is None else n1
        t0 = self.target_range[0] if t0 is None else t0
        t1 = self.target_range[1] if t1 is None else t1
        out = np.zeros((n1 - n0, t1 - t0), np.uint8)
        _check(lib().av_read_pref(self._h, n0, n1, t0, t1, _ptr(out)))
        return out

    def sample_peers(self, rnd, n0=0, n1=None):
        n1 = self.n_nodes if n1 is None else n1
        out = np.zeros((n1 - n0, self.k), np.int32)
        _check(lib().av_sample_peers(self._h, rnd, n0, n1, _ptr(out)))
        return out

    # ---- measurement / tuning ----
    def set_option(self, name, value):
        _check(lib().av_set_option(self._h, name.encode(), int(value)))

    def set_timing(self, enable=True):
        _check(lib().av_set_timing(self._h, int(enable)))

    def kernel_stats(self):
        ms, n = C.c_double(0), C.c_int64(0)
        _check(lib().av_kernel_stats(self._h, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def layout_info(self):
        lanes, nl, bl, capped = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int32()
        _check(lib().av_layout_info(self._h, C.byref(lanes), C.byref(nl), C.byref(bl), C.byref(capped)))
        return {"lanes": lanes.value, "local_nodes": nl.value, "local_blocks": bl.value, "capped": bool(capped.value)}

    def peer_handles(self) -> bytes:
        """IPC handles of this rank's preference snapshots (av_peer_handles)."""
        buf = (C.c_uint8 * PEER_HANDLE_BYTES)()
        _check(lib().av_peer_handles(self._h, C.cast(buf, _vp)))
        return bytes(buf)

    def peer_init(self, world, rank, handles):
        """Map every rank's snapshots (handles: the rank-ordered list of
        peer_handles() blobs) and switch to the peer-push exchange."""
        blob = b"".join(handles)
        assert len(blob) == world * PEER_HANDLE_BYTES
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        _check(lib().av_peer_init(self._h, world, rank, C.cast(buf, _vp)))

    def comm_init(self, world, rank, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        _check(lib().av_comm_init(self._h, world, rank, C.cast(buf, _vp)))
