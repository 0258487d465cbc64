import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "go-avalanche_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "reference_tests.json")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine through the C ABI)")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from oracle import cabi

    cabi.lib()
    return cabi
