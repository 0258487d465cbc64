"""The reference's Processor tests (avalanche_test.go) restated in C++ against
the host mirror go-avalanche_amd/host/avalanche.hpp, run on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "go-avalanche_amd", "bin", "avalanche_gpu_tests")


def test_cpp_mirror_binary_built():
    assert os.path.exists(BIN), "run __graft_entry__.build()"


@pytest.mark.gpu
def test_example_basic_preconsensus():
    """examples/basic-preconcensus (C1) on the engine: every node finalizes every tx."""
    exe = os.path.join(ROOT, "go-avalanche_amd", "bin", "basic_preconsensus")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "Nodes fully finalized: 100" in r.stdout


@pytest.mark.gpu
def test_cpp_mirror_reference_tests():
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    for name in ("TestBlockRegister", "TestMultiBlockRegister", "SuitableNodeAndInvalidTarget", "NetworkRounds",
                 "PipelinedRounds"):
        assert f"PASS {name}" in r.stdout
