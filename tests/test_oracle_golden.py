"""The CPU oracle (oracle/ldpc_oracle.c) against the reference's own outputs.

The golden vectors were produced by the unmodified reference SSE decoders
(code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp, .../NMS/...) compiled from
/root/reference (tests/golden/gen_golden.py).  Bit-exact hard decisions.
"""
import hashlib

import numpy as np
import pytest
from conftest import golden_cases, golden_inputs

import oracle as O
from ldpcgputegra_amd import load_table

CASES = golden_cases()
FAST = [c for c in CASES if not c["code"].startswith("dvbs2")]
DVB = [c for c in CASES if c["code"].startswith("dvbs2")]


@pytest.mark.parametrize("case", FAST, ids=[c["name"] for c in FAST])
def test_oracle_matches_reference_short_codes(case):
    llr, expected = golden_inputs(case)
    assert hashlib.sha256(llr.tobytes()).hexdigest() == case["llr_sha256"]
    got = O.decode_i8(load_table(case["code"]), llr, case["iters"], case["algo"], case["param"],
                      var_min=case["var_min"], msg_max=case["msg_max"])
    assert np.array_equal(got, expected)


@pytest.mark.parametrize("case", DVB, ids=[c["name"] for c in DVB])
def test_oracle_matches_reference_dvbs2(case):
    llr, expected = golden_inputs(case)
    # the regenerated inputs are exactly the ones the reference decoded
    assert hashlib.sha256(llr.tobytes()).hexdigest() == case["llr_sha256"]
    # 4 of the 16 codewords keep the CPU suite fast; all 16 run on the GPU box
    got = O.decode_i8(load_table(case["code"]), llr[:4], case["iters"], case["algo"], case["param"])
    assert np.array_equal(got, expected[:4])


def test_golden_covers_edge_cases():
    its = {c["iters"] for c in CASES}
    assert {0, 1, 2, 50} <= its
    assert any(c["algo"] == 1 for c in CASES)                      # NMS
    assert any(c["var_min"] == -128 for c in CASES)                # abs8(-128) path
    assert any(c["msg_max"] == 127 for c in CASES)
    assert any(c["code"] == "1944x972" for c in CASES)             # N % 16 != 0 (scalar transpose)
    assert any(c["code"] == "dvbs2_r1_2" and c["bit_errors"] == 0 for c in CASES)
    assert any(c["code"] == "dvbs2_r1_2" and c["bit_errors"] > 10000 for c in CASES)


def test_quantizer_matches_reference_rule():
    # CFastFixConversion::generate: trunc toward zero, then clamp to [-31, 31]
    y = np.array([-5.0, -3.9, -0.124, -0.126, 0.0, 0.124, 0.126, 0.9999, 3.874, 3.876, 100.0], np.float32)
    q = O.quantize(y)
    assert q.tolist() == [-31, -31, 0, -1, 0, 0, 1, 7, 30, 31, 31]


def test_float_oracle_basic_properties():
    t = load_table("576x288")
    rng = np.random.default_rng(0)
    llr = (-1.0 + 0.6 * rng.standard_normal((4, t.n))).astype(np.float32)
    hard, soft, its = O.decode_f32(t, llr, 20, O.OMS, 0.0)
    assert np.array_equal(hard, (soft > 0).astype(np.uint8))
    assert (its == 20).all()
    # zero iterations returns the channel LLRs unchanged
    h0, s0, _ = O.decode_f32(t, llr, 0)
    assert np.array_equal(s0, llr)
