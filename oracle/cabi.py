"""TEST INFRASTRUCTURE ONLY — ctypes binding of the C oracle (liboracle).

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "lib", "libavoracle.so")
_lib = None

u32p = np.ctypeslib.ndpointer(np.uint32, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")


class SimConfig(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_int64),
        ("n_targets", C.c_int64),
        ("k", C.c_int32),
        ("peer_mode", C.c_int32),
        ("seed", C.c_uint64),
        ("byz_threshold", C.c_uint32),
        ("init_mode", C.c_int32),
        ("init_param", C.c_uint32),
    ]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.avo_philox4x32_10.argtypes = [u32p, u32p, u32p]
        L.avo_transition_batch.argtypes = [u32p, u32p, C.c_int64, u32p, u8p, u8p]
        L.avo_processor_new.restype = C.c_void_p
        L.avo_processor_new.argtypes = [C.c_int64]
        L.avo_processor_free.argtypes = [C.c_void_p]
        L.avo_sim_new.restype = C.c_void_p
        L.avo_sim_new.argtypes = [C.POINTER(SimConfig)]
        L.avo_sim_new_threads.restype = C.c_void_p
        L.avo_sim_new_threads.argtypes = [C.POINTER(SimConfig), C.c_int32]
        L.avo_sim_round_ex.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                       C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int64), C.c_void_p,
                                       C.c_uint32]
        L.avo_sim_dump_range.argtypes = [C.c_void_p, C.c_int64, C.c_int64, u32p, C.c_int32]
        L.avo_pack_update.restype = C.c_uint64
        L.avo_pack_update.argtypes = [C.c_uint32, C.c_int64, C.c_int32, C.c_int64, C.c_int32]
        L.avo_transition_batch_branchfree.argtypes = [u32p, u32p, C.c_int64, u32p,
                                                      np.ctypeslib.ndpointer(np.int8, flags="C_CONTIGUOUS")]
        L.avo_node_round_ext.restype = C.c_int64
        L.avo_node_round_ext.argtypes = [C.c_uint64, C.c_int64, C.c_int32, C.c_int32, C.c_int64, C.c_int64,
                                         C.c_int64, u32p, u32p, u8p, u32p, C.c_void_p, C.c_uint32]
        L.avo_byz_words.argtypes = [C.c_uint64, C.c_int64, C.c_uint32, u32p]
        L.avo_sim_get_round.restype = C.c_int64
        L.avo_sim_get_round.argtypes = [C.c_void_p, C.c_int64]
        L.avo_sim_set_round.argtypes = [C.c_void_p, C.c_int64, C.c_int64]
        L.avo_sim_set_responder.argtypes = [C.c_void_p, C.c_int32]
        L.avo_sim_set_polling.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.avo_sim_set_literal.argtypes = [C.c_void_p, C.c_int]
        L.avo_mix64.restype = C.c_uint64
        L.avo_mix64.argtypes = [C.c_uint64]
        L.avo_sim_free.argtypes = [C.c_void_p]
        L.avo_sim_set_valid.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.avo_sim_round_index.restype = C.c_int64
        L.avo_sim_round_index.argtypes = [C.c_void_p]
        L.avo_sim_set_round_index.restype = None
        L.avo_sim_set_round_index.argtypes = [C.c_void_p, C.c_int64]
        L.avo_sim_round.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64,
                                    C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int64)]
        L.avo_sim_round_range.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p, C.c_int64,
                                          C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int64)]
        L.avo_sim_set_pref_rows.argtypes = [C.c_void_p, C.c_int64, C.c_int64, u8p]
        L.avo_sim_dump.argtypes = [C.c_void_p, u32p]
        L.avo_sim_pref.argtypes = [C.c_void_p, u8p]
        L.avo_sim_is_byzantine.argtypes = [C.c_void_p, C.c_int64]
        L.avo_sim_add.argtypes = [C.c_void_p, C.c_int64, C.c_int64, C.c_int]
        L.avo_sim_register_votes.argtypes = [C.c_void_p, C.c_int64, i64p, u32p, C.c_int64, i64p, i32p,
                                             C.POINTER(C.c_int64)]
        L.avo_sample_peers.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, C.c_int32, i64p]
        L.avo_is_byzantine.argtypes = [C.c_uint64, C.c_int64, C.c_uint32]
        L.avo_initial_accept.argtypes = [C.c_uint64, C.c_int32, C.c_uint32, C.c_int64, C.c_int64]
        L.avo_replay_err.restype = C.c_uint32
        L.avo_replay_err.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int32, C.c_int64]
        L.avo_gen_replay_errs.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, u32p]
        _lib = L
    return _lib


def philox(ctr, key):
    out = np.zeros(4, np.uint32)
    lib().avo_philox4x32_10(np.asarray(ctr, np.uint32), np.asarray(key, np.uint32), out)
    return out


def transition_batch(words: np.ndarray, errs: np.ndarray):
    words = np.ascontiguousarray(words, np.uint32)
    errs = np.ascontiguousarray(errs, np.uint32)
    out = np.empty_like(words)
    changed = np.empty(words.shape, np.uint8)
    status = np.empty(words.shape, np.uint8)
    lib().avo_transition_batch(words, errs, words.size, out, changed, status)
    return out, changed, status


def pack_update(round_rel, node, slot, t, status):
    return lib().avo_pack_update(round_rel, node, slot, t, status)


def update_digest(words):
    """(count, sum, xor) of avo_mix64 over packed update words (numpy, same as the C side)."""
    z = np.asarray(words, np.uint64) + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    z = z ^ (z >> np.uint64(31))
    return int(z.size), int(z.sum(dtype=np.uint64)), int(np.bitwise_xor.reduce(z)) if z.size else 0


def transition_batch_branchfree(words: np.ndarray, errs: np.ndarray):
    words = np.ascontiguousarray(words, np.uint32)
    errs = np.ascontiguousarray(errs, np.uint32)
    out = np.empty_like(words)
    status = np.empty(words.shape, np.int8)
    lib().avo_transition_batch_branchfree(words, errs, words.size, out, status)
    return out, status


def byz_words(seed, n_nodes, threshold):
    out = np.zeros((n_nodes + 31) // 32, np.uint32)
    lib().avo_byz_words(seed, n_nodes, threshold, out)
    return out


def node_round_ext(seed, n_nodes, k, peer_mode, node, rnd, m, pref_words, byz_words, valid, words, digest,
                   round_rel=0):
    """One node's literal round against the engine's snapshot (avo_node_round_ext).
    words (uint32[m]) is updated in place; digest (uint64[3]) accumulates."""
    assert words.dtype == np.uint32 and words.flags["C_CONTIGUOUS"] and digest.dtype == np.uint64
    return lib().avo_node_round_ext(seed, n_nodes, k, peer_mode, node, rnd, m,
                                    np.ascontiguousarray(pref_words, np.uint32),
                                    np.ascontiguousarray(byz_words, np.uint32), np.ascontiguousarray(valid, np.uint8),
                                    words, digest.ctypes.data_as(C.c_void_p), round_rel)


def sample_peers(seed, node, rnd, n_nodes, k, mode=0):
    out = np.zeros(k, np.int64)
    lib().avo_sample_peers(seed, node, rnd, n_nodes, k, mode, out)
    return out


def gen_replay_errs(seed, rnd, n0, n1, n_targets, k):
    out = np.empty((n1 - n0, k, n_targets), np.uint32)
    lib().avo_gen_replay_errs(seed, rnd, n0, n1, n_targets, k, out)
    return out


class Sim:
    """Batched-round harness over one restated Processor per node."""

    def __init__(self, n_nodes, n_targets, k=8, seed=0xA7A1A9C4, peer_mode=0, byz_threshold=0,
                 init_mode=3, init_param=0x80000000, threads=1):
        self.cfg = SimConfig(n_nodes, n_targets, k, peer_mode, seed, byz_threshold, init_mode, init_param)
        self.n, self.m, self.k = n_nodes, n_targets, k
        self._h = lib().avo_sim_new_threads(C.byref(self.cfg), threads)

    def close(self):
        if self._h:
            lib().avo_sim_free(self._h)
            self._h = None

    __del__ = close

    @property
    def round(self):
        return lib().avo_sim_round_index(self._h)

    def set_round_index(self, r):
        """Start this (freshly populated) network's rounds at round r: the engine's
        av_init_records on an engine that has already run r rounds."""
        lib().avo_sim_set_round_index(self._h, r)

    def get_round(self, node):
        return lib().avo_sim_get_round(self._h, node)

    def set_round(self, node, rnd):
        lib().avo_sim_set_round(self._h, node, rnd)

    def set_responder(self, mode):
        """0: publish the decision (R2); 1: IsAccepted literally (processor.go:125-130);
        2: the example's responder, re-adding queried targets (main.go:175-182)."""
        lib().avo_sim_set_responder(self._h, mode)

    def set_polling(self, node, polls):
        lib().avo_sim_set_polling(self._h, node, int(polls))

    def set_literal(self, literal=True):
        """Force the literal per-vote path (cross-check of the branch-free one)."""
        lib().avo_sim_set_literal(self._h, int(literal))

    def set_valid(self, t, valid):
        lib().avo_sim_set_valid(self._h, t, int(valid))

    def add(self, node, t, accepted):
        return bool(lib().avo_sim_add(self._h, node, t, int(accepted)))

    def register_votes(self, node, targets, errs):
        targets = np.ascontiguousarray(targets, np.int64)
        errs = np.ascontiguousarray(errs, np.uint32)
        ot = np.zeros(max(1, len(targets)), np.int64)
        os_ = np.zeros(max(1, len(targets)), np.int32)
        n = C.c_int64(0)
        lib().avo_sim_register_votes(self._h, node, targets, errs, len(targets), ot, os_, C.byref(n))
        return list(zip(ot[: n.value].tolist(), os_[: n.value].tolist()))

    def run_round(self, replay_errs=None, threads=1, collect=True, round_rel=0):
        """Returns (updates int64[n,5] (round,node,slot,target,status), applied_votes).
        collect=False: no rows; returns (digest (count, sum, xor) of the round's
        packed updates with round field `round_rel`, applied_votes)."""
        n = C.c_int64(0)
        applied = C.c_int64(0)
        rp = None
        if replay_errs is not None:
            replay_errs = np.ascontiguousarray(replay_errs, np.uint32)
            assert replay_errs.shape == (self.n, self.k, self.m)
            rp = replay_errs.ctypes.data_as(C.c_void_p)
        dig = np.zeros(3, np.uint64)
        if not collect:
            lib().avo_sim_round_ex(self._h, 0, self.n, rp, None, 0, C.byref(n), threads, C.byref(applied),
                                   dig.ctypes.data_as(C.c_void_p), round_rel)
            return tuple(int(v) for v in dig), applied.value
        cap = self.n * self.m * 2 + 16
        buf = np.empty((cap, 5), np.int64)
        rc = lib().avo_sim_round_ex(self._h, 0, self.n, rp, buf.ctypes.data_as(C.c_void_p), cap, C.byref(n),
                                    threads, C.byref(applied), dig.ctypes.data_as(C.c_void_p), round_rel)
        assert rc == 0, "oracle update buffer too small"
        return buf[: n.value].copy(), applied.value

    def run_round_range(self, n0, n1, threads=1):
        """Sim-mode round for the node shard [n0, n1) only (node-sharded rehearsal)."""
        n = C.c_int64(0)
        applied = C.c_int64(0)
        cap = (n1 - n0) * self.m * 2 + 16
        buf = np.empty((cap, 5), np.int64)
        rc = lib().avo_sim_round_range(self._h, n0, n1, None, buf.ctypes.data_as(C.c_void_p), cap, C.byref(n),
                                       threads, C.byref(applied))
        assert rc == 0
        return buf[: n.value].copy(), applied.value

    def set_pref_rows(self, n0, rows):
        rows = np.ascontiguousarray(rows, np.uint8)
        lib().avo_sim_set_pref_rows(self._h, n0, n0 + rows.shape[0], rows)

    def dump(self, n0=0, n1=None, threads=1):
        n1 = self.n if n1 is None else n1
        out = np.empty((n1 - n0, self.m), np.uint32)
        lib().avo_sim_dump_range(self._h, n0, n1, out, threads)
        return out

    def pref(self):
        out = np.empty((self.n, self.m), np.uint8)
        lib().avo_sim_pref(self._h, out)
        return out

    def is_byzantine(self, node):
        return bool(lib().avo_sim_is_byzantine(self._h, node))
