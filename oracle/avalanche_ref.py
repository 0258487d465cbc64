"""TEST INFRASTRUCTURE ONLY — independent pure-Python restatement of go-avalanche.

Second, independent restatement (besides the C oracle in avalanche_oracle.c) of
the reference's VoteRecord and Processor semantics, written against the Go
source with Python dicts standing in for Go maps. Used only to cross-check the
C oracle at small sizes and to run the golden fixtures; never imported by the
product path.

Reference: /root/reference (itsdevbear/go-avalanche @ 2025-01-17).
"""
from __future__ import annotations

import numpy as np

FINALIZATION_SCORE = 128  # avalanche.go:10
MAX_ELEMENT_POLL = 4096  # avalanche.go:17

STATUS_INVALID, STATUS_REJECTED, STATUS_ACCEPTED, STATUS_FINALIZED = 0, 1, 2, 3  # avalanche.go:42-56

ABSENT_WORD = 0xFFFE0000


def _popcount8(x: int) -> int:
    return bin(x & 0xFF).count("1")


class VoteRecord:
    """vote.go:24-109."""

    __slots__ = ("votes", "consider", "confidence")

    def __init__(self, accepted: bool):  # vote.go:33-35
        self.votes = 0
        self.consider = 0
        self.confidence = 1 if accepted else 0

    @classmethod
    def from_word(cls, w: int) -> "VoteRecord":
        vr = cls(False)
        vr.votes = w & 0xFF
        vr.consider = (w >> 8) & 0xFF
        vr.confidence = (w >> 16) & 0xFFFF
        return vr

    def word(self) -> int:
        return self.votes | (self.consider << 8) | (self.confidence << 16)

    def is_accepted(self) -> bool:  # vote.go:38-40
        return (self.confidence & 1) == 1

    def get_confidence(self) -> int:  # vote.go:43-45
        return self.confidence >> 1

    def has_finalized(self) -> bool:  # vote.go:48-50
        return self.get_confidence() >= FINALIZATION_SCORE

    def register_vote(self, err: int) -> bool:  # vote.go:54-75
        err &= 0xFFFFFFFF
        self.votes = ((self.votes << 1) & 0xFF) | (1 if err == 0 else 0)
        signed = err - (1 << 32) if err >= (1 << 31) else err
        self.consider = ((self.consider << 1) & 0xFF) | (1 if signed >= 0 else 0)
        yes = _popcount8(self.votes & self.consider) > 6
        if not yes and _popcount8((~self.votes) & self.consider) <= 6:
            return False
        if self.is_accepted() == yes:
            self.confidence = (self.confidence + 2) & 0xFFFF
            return self.get_confidence() == FINALIZATION_SCORE
        self.confidence = 1 if yes else 0
        return True

    def status(self) -> int:  # vote.go:77-91
        fin, acc = self.has_finalized(), self.is_accepted()
        if not fin and acc:
            return STATUS_ACCEPTED
        if not fin and not acc:
            return STATUS_REJECTED
        if fin and acc:
            return STATUS_FINALIZED
        return STATUS_INVALID


class Target:
    """avalanche.go:74-91 Target interface (Hash/Type/IsAccepted/Score/IsValid)."""

    def __init__(self, hash_: int, accepted: bool = True, valid: bool = True, type_: str = "tx", score: int = 1):
        self.hash = hash_
        self.accepted = accepted
        self.valid = valid
        self.type = type_
        self.score = score


class Processor:
    """processor.go:12-187 with Go maps as dicts. Iteration order of
    GetInvsForNextPoll is fixed to ascending hash."""

    def __init__(self):
        self.targets: dict[int, Target] = {}
        self.vote_records: dict[int, VoteRecord] = {}
        self.decision: dict[int, bool] = {}  # harness extension for rule R2
        self.round = 0

    def get_round(self) -> int:  # processor.go:40-42
        return self.round

    def add_target_to_reconcile(self, t: Target) -> bool:  # processor.go:45-58
        if not t.valid:
            return False
        if t.hash in self.vote_records:
            return False
        self.targets[t.hash] = t
        self.vote_records[t.hash] = VoteRecord(t.accepted)
        return True

    def register_votes(self, node_id: int, votes, updates: list) -> bool:  # processor.go:61-122
        for h, err in votes:
            vr = self.vote_records.get(h)
            if vr is None:
                continue
            if not self.targets[h].valid:
                continue
            if not vr.register_vote(err):
                continue
            updates.append((h, vr.status()))
            if vr.has_finalized():
                del self.vote_records[h]
                self.decision[h] = vr.is_accepted()
        return True

    def is_accepted(self, h: int) -> bool:  # processor.go:125-130
        vr = self.vote_records.get(h)
        return vr.is_accepted() if vr is not None else False

    def get_confidence(self, h: int) -> int:  # processor.go:133-140
        vr = self.vote_records.get(h)
        if vr is None:
            raise KeyError("VoteRecord not found")
        return vr.get_confidence()

    def get_invs_for_next_poll(self) -> list[int]:  # processor.go:144-170
        invs = []
        for h in sorted(self.vote_records):
            r = self.vote_records[h]
            if r.has_finalized():
                continue
            if not self.targets[h].valid:
                continue
            invs.append(h)
        return invs[:MAX_ELEMENT_POLL]

    def published(self, h: int, responder: int = 0) -> bool:
        """What this node answers for h: its record's IsAccepted; without a
        record: 0 = the finalized decision (R2), 1 = IsAccepted literally
        (false, processor.go:125-130), 2 = the example's responder (it re-adds
        &tx{isAccepted: true} first and answers yes, main.go:175-182)."""
        vr = self.vote_records.get(h)
        if vr is not None:
            return vr.is_accepted()
        if responder == 1:
            return False
        if responder == 2:
            return True
        return bool(self.decision.get(h, False))

    def dump_word(self, h: int) -> int:
        vr = self.vote_records.get(h)
        if vr is not None:
            return vr.word()
        return ABSENT_WORD | (int(self.decision.get(h, False)) << 16)


# --------------------------------------------------------------------------
# Philox4x32-10 and the synthetic workload definition (independent restatement)
# --------------------------------------------------------------------------
_M = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    c = [x & _M for x in ctr]
    k0, k1 = key[0] & _M, key[1] & _M
    for r in range(10):
        if r:
            k0 = (k0 + 0x9E3779B9) & _M
            k1 = (k1 + 0xBB67AE85) & _M
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & _M, p1 & _M, ((p0 >> 32) ^ c[3] ^ k1) & _M, p0 & _M]
    return c


DOM_PEERS, DOM_BYZ, DOM_INIT, DOM_PAIRS, DOM_REPLAY = 1, 2, 3, 4, 5
PEERS_RANDOM, PEERS_ROUND_ROBIN = 0, 1
INIT_NONE, INIT_REJECTED, INIT_ACCEPTED, INIT_BERNOULLI, INIT_PAIRS = 0, 1, 2, 3, 4


def _ph(seed, a, b, c, dom):
    return philox4x32_10([a, b, c, dom], [seed & _M, (seed >> 32) & _M])


def sample_peers(seed, node, rnd, n_nodes, k, mode=PEERS_RANDOM):
    others = n_nodes - 1
    if mode == PEERS_ROUND_ROBIN or k >= others:
        out = []
        for j in range(k):
            q = rnd * k + j if mode == PEERS_ROUND_ROBIN else j
            idx = q % others
            out.append(idx + (1 if idx >= node else 0))
        return out
    out, blk = [], 0
    while len(out) < k:
        x = _ph(seed, node, rnd, blk, DOM_PEERS)
        for v in x:
            if len(out) == k:
                break
            u = (v * others) >> 32
            p = u + (1 if u >= node else 0)
            if p not in out:
                out.append(p)
        blk += 1
    return out


def is_byzantine(seed, node, threshold):
    return _ph(seed, node, 0, 0, DOM_BYZ)[0] < threshold


def initial_accept(seed, mode, param, node, t):
    if mode == INIT_REJECTED:
        return False
    if mode == INIT_ACCEPTED:
        return True
    if mode == INIT_BERNOULLI:
        return _ph(seed, node, t >> 2, 0, DOM_INIT)[t & 3] < param
    if mode == INIT_PAIRS:
        pair = t >> 1
        return bool(((_ph(seed, node, pair >> 2, 0, DOM_PAIRS)[pair & 3] >> 31) ^ (t & 1)))
    return False


def replay_err(seed, node, rnd, slot, t):
    x = _ph(seed, node, rnd, t >> 1, DOM_REPLAY | (slot << 8))
    v, sel = x[(t & 1) * 2], x[(t & 1) * 2 + 1]
    if v < 3006477107:
        return 0
    if v < 4080218931:
        return (1, 2, 0x7FFFFFFF)[sel % 3]
    return 0xFFFFFFFF if sel & 1 else 0x80000000


class Sim:
    """Synchronous batched rounds, SURVEY.md §8(a) R1-R4, over one Processor per node."""

    def __init__(self, n_nodes, n_targets, k, seed, peer_mode=PEERS_RANDOM, byz_threshold=0,
                 init_mode=INIT_BERNOULLI, init_param=0x80000000):
        self.n, self.m, self.k, self.seed = n_nodes, n_targets, k, seed
        self.peer_mode, self.byz_threshold = peer_mode, byz_threshold
        self.round = 0
        self.targets = [Target(t, valid=True) for t in range(n_targets)]
        self.procs = [Processor() for _ in range(n_nodes)]
        self.byz = [is_byzantine(seed, j, byz_threshold) for j in range(n_nodes)]
        if init_mode != INIT_NONE:
            for j, p in enumerate(self.procs):
                for t in range(n_targets):
                    p.add_target_to_reconcile(Target(t, accepted=initial_accept(seed, init_mode, init_param, j, t)))
                    p.targets[t] = self.targets[t]  # validity is a property of the shared target
        self.responder = 0
        self.polls = [True] * n_nodes
        self.pref = self._snapshot()

    def set_valid(self, t, valid):
        self.targets[t].valid = bool(valid)

    def set_responder(self, mode):
        self.responder = mode
        self.pref = self._snapshot()

    def _snapshot(self):
        return [[p.published(t, self.responder) for t in range(self.m)] for p in self.procs]

    def run_round(self, replay_errs=None):
        r, updates = self.round, []
        held = [set(p.vote_records) for p in self.procs]  # round-start records (responder 2)
        readd = set()
        for node, p in enumerate(self.procs):
            if not self.polls[node]:  # the example's run loop has returned (main.go:160-162)
                continue
            peers = sample_peers(self.seed, node, r, self.n, self.k, self.peer_mode)
            for slot in range(self.k):
                invs = p.get_invs_for_next_poll()
                peer = peers[slot]
                votes = []
                for t in invs:
                    if self.responder == 2 and t not in held[peer] and self.targets[t].valid:
                        readd.add((peer, t))  # AddTargetToReconcile(&tx{isAccepted: true}) (main.go:175-177)
                    if replay_errs is not None:
                        err = int(replay_errs[node, slot, t])
                    elif self.byz[peer]:
                        err = 1 if ((r ^ t) & 1) else 0
                    else:
                        err = 0 if self.pref[peer][t] else 1
                    votes.append((t, err))
                ups = []
                p.register_votes(peer, votes, ups)
                updates.extend((r, node, slot, h, st) for h, st in ups)
        for peer, t in sorted(readd):
            self.procs[peer].add_target_to_reconcile(Target(t, accepted=True))
            self.procs[peer].targets[t] = self.targets[t]
        self.pref = self._snapshot()
        self.round += 1
        return updates

    def dump(self):
        return np.array([[p.dump_word(t) for t in range(self.m)] for p in self.procs], dtype=np.uint32)
