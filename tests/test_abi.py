"""CPU tests of the drop-in boundary: libavhip.so loads and exports every
symbol include/avhip.h declares (no compute calls: there is no GPU here)."""
import ctypes
import os
import re

import avhip

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "avhip.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^(?:int|void|const char\*)\s+(av_\w+)\(", src, re.M)))


def test_header_declares_binding_symbols():
    assert header_symbols() == sorted(avhip.EXPORTED)


def test_library_exports_every_header_symbol():
    lib = ctypes.CDLL(avhip.LIB_PATH)
    missing = [s for s in header_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_abi_version_and_strings():
    L = avhip.lib()
    assert L.av_abi_version() == 1
    assert L.av_strerror(-4) == b"VoteRecord not found"
    assert L.av_strerror(0) == b"ok"


def test_create_rejects_bad_config_without_gpu():
    # argument validation happens before any device call
    import pytest

    with pytest.raises(avhip.AvError):
        avhip.Engine(1, 10)  # n_nodes must be >= 2
    with pytest.raises(avhip.AvError):
        avhip.Engine(10, 10, k=17)
    with pytest.raises(avhip.AvError):
        avhip.Engine(10, 5000, target_range=(0, 2048))  # cap couples targets


def test_update_word_decoding():
    import numpy as np

    u = np.array([(3 << 52) | (12345 << 28) | (7 << 24) | (999 << 2) | 2], np.uint64)
    assert avhip.decode_updates(u, 10).tolist() == [[13, 12345, 7, 999, 2]]
