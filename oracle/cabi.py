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
        L.avo_sim_free.argtypes = [C.c_void_p]
        L.avo_sim_set_valid.argtypes = [C.c_void_p, C.c_int64, C.c_int]
        L.avo_sim_round_index.restype = C.c_int64
        L.avo_sim_round_index.argtypes = [C.c_void_p]
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
                 init_mode=3, init_param=0x80000000):
        self.cfg = SimConfig(n_nodes, n_targets, k, peer_mode, seed, byz_threshold, init_mode, init_param)
        self.n, self.m, self.k = n_nodes, n_targets, k
        self._h = lib().avo_sim_new(C.byref(self.cfg))

    def close(self):
        if self._h:
            lib().avo_sim_free(self._h)
            self._h = None

    __del__ = close

    @property
    def round(self):
        return lib().avo_sim_round_index(self._h)

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

    def run_round(self, replay_errs=None, threads=1):
        """Returns (updates int64[n,5] (round,node,slot,target,status), applied_votes)."""
        n = C.c_int64(0)
        applied = C.c_int64(0)
        rp = None
        if replay_errs is not None:
            replay_errs = np.ascontiguousarray(replay_errs, np.uint32)
            assert replay_errs.shape == (self.n, self.k, self.m)
            rp = replay_errs.ctypes.data_as(C.c_void_p)
        cap = self.n * self.m * 2 + 16
        buf = np.empty((cap, 5), np.int64)
        rc = lib().avo_sim_round(self._h, rp, buf.ctypes.data_as(C.c_void_p), cap, C.byref(n), threads,
                                 C.byref(applied))
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

    def dump(self):
        out = np.empty((self.n, self.m), np.uint32)
        lib().avo_sim_dump(self._h, out)
        return out

    def pref(self):
        out = np.empty((self.n, self.m), np.uint8)
        lib().avo_sim_pref(self._h, out)
        return out

    def is_byzantine(self, node):
        return bool(lib().avo_sim_is_byzantine(self._h, node))
