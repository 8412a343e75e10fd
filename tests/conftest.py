import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def golden_cases():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)["cases"]


def golden_inputs(case):
    """(llr int8 [B, N], expected hard uint8 [B, N]) for a golden case."""
    from golden.gen_golden import awgn_i8, random_codewords
    from ldpcgputegra_amd import load_table
    n = load_table(case["code"]).n
    if "llr_file" in case:
        llr = np.load(os.path.join(GOLDEN, case["llr_file"]))
    else:
        cw = random_codewords(case["code"], case["batch"], case["info_seed"]) if "info_seed" in case else None
        llr = awgn_i8(n, case["batch"], case["seed"], np.array(case["table"], dtype=np.uint32), codeword=cw)
    packed = np.load(os.path.join(GOLDEN, case["name"] + ".npz"))["hard_packed"]
    hard = np.unpackbits(packed, axis=-1, count=n)
    return llr, hard


@pytest.fixture(scope="session")
def gpu_available():
    from ldpcgputegra_amd import _lib
    import ctypes as C
    c = C.c_int()
    _lib.lib().ldpc_device_count(C.byref(c))
    return c.value > 0
