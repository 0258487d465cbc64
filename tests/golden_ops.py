"""Interpreter for the transcribed reference-test fixtures (tests/golden/).

A fixture is run against any object implementing the small Processor surface
below, so the same golden vectors pin the C oracle, the Python restatement and
(in -m gpu tests) the HIP engine through the C ABI.
"""
from __future__ import annotations


class NotFound(Exception):
    pass


def run_vote_record(fx, make_record):
    """fx = golden["vote_record"]; make_record(accepted) -> object with
    vote(err) -> (accepted, finalized, confidence)  and  state() -> same tuple."""
    for chk in fx["initial_checks"]:
        rec = make_record(chk["accepted_arg"])
        assert rec.state() == (chk["accepted"], chk["finalized"], chk["confidence"]), chk
    rec = make_record(fx["start_accepted"])
    for i, st in enumerate(fx["steps"]):
        got = rec.vote(st["err"])
        exp = (st["accepted"], st["finalized"], st["confidence"])
        assert got == exp, f"step {i} (avalanche_test.go:{st['line']}): got {got}, want {exp}"


def run_processor(fx, proc):
    """proc implements add(hash)->bool, register(node, votes[[err, hash]...]) -> [(hash, status)],
    is_accepted(hash)->bool, confidence(hash)->int (raise NotFound), invs()->[hash],
    get_round()->int, inc_round() (the test's p.round++)."""
    for i, op in enumerate(fx["ops"]):
        where = f"{fx['name']} op {i} (avalanche_test.go:{op['line']})"
        kind = op["op"]
        if kind == "is_accepted":
            assert proc.is_accepted(op["hash"]) == op["expect"], where
        elif kind == "add":
            assert proc.add(op["hash"]) == op["expect"], where
        elif kind == "poll_count":
            assert len(proc.invs()) == op["expect"], where
        elif kind == "poll_contains":
            assert op["hash"] in proc.invs(), where
        elif kind == "register":
            got = [list(x) for x in proc.register(op["node"], op["votes"])]
            assert got == op["expect_updates"], f"{where}: got {got}"
        elif kind == "confidence":
            assert proc.confidence(op["hash"]) == op["expect"], where
        elif kind == "get_round":
            assert proc.get_round() == op["expect"], where
        elif kind == "inc_round":
            proc.inc_round()
        else:
            raise AssertionError(f"unknown op {kind}")
