"""The C-ABI's host decoder (ldpc_ctx_create with device = -1, csrc/host.cpp):
the drop-in on a machine without an MI355X.  Runs here, on
the CPU: every golden vector of the reference (tests/golden, produced by the
reference's own SSE decoder, code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp)
through ldpc_decode_i8 on the AVX2 path and, for a subset, the portable
per-lane path; early termination and the float decoder against the oracle;
device-buffer entry points rejected cleanly."""
import ctypes as C
import os

import numpy as np
import pytest
from conftest import golden_cases, golden_inputs

import oracle as O
from ldpcgputegra_amd import ALGO_MS, ALGO_NMS, ALGO_OMS, Code, Decoder, LdpcError, _lib, channel, default_params
from ldpcgputegra_amd import load_table

CASES = golden_cases()
_decs = {}


def host(code):
    if code not in _decs:
        _decs[code] = Decoder(Code(code), device=-1, max_batch=4096)
    return _decs[code]


def params_of(case):
    algo = ALGO_NMS if case["algo"] == 1 else ALGO_OMS
    return default_params(algo=algo, offset=case["param"], factor=case["param"], var_min=case["var_min"],
                          msg_max=case["msg_max"], msg_min=-case["msg_max"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_host_decoder_matches_reference_golden(case):
    llr, expected = golden_inputs(case)
    d = host(case["code"])
    got = d.decode_i8(llr, case["iters"], params_of(case))
    assert d.last_kernel == "host"
    assert np.array_equal(got, expected), "%d bits differ" % int((got != expected).sum())


@pytest.mark.parametrize("case", [c for c in CASES if c["code"] in ("576x288", "2048x384") or
                                  (c["code"] == "dvbs2_r1_2" and c["iters"] <= 20)][:12],
                         ids=lambda c: c["name"])
@pytest.mark.parametrize("env", [{"LDPC_HOST_PORTABLE": "1"}, {"LDPC_HOST_LANES": "16"}],
                         ids=["portable", "sse16"])
def test_host_portable_path_matches_golden(case, env, monkeypatch):
    """The per-lane portable loop and the 16-lane SSE4.1 blocks (the paths a
    host without AVX2 runs) equal the reference's golden vectors too."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    llr, expected = golden_inputs(case)
    got = host(case["code"]).decode_i8(llr, case["iters"], params_of(case))
    assert np.array_equal(got, expected)


@pytest.mark.parametrize("lanes", ["16", "32"])
def test_host_simd_early_termination_ragged(lanes, monkeypatch):
    """Early termination on both SIMD widths over a ragged batch of 50
    (blocks of 16 / 32 with a partial last block) equals the oracle."""
    monkeypatch.setenv("LDPC_HOST_LANES", lanes)
    t = load_table("576x288")
    llr = channel.awgn_i8_host(t.n, 50, seed=8, table=channel.i8_table(channel.sigma_from_ebn0(2.0, 0.5)))
    exp, _, its = O.decode_i8(t, llr, 25, early_term=True, return_soft=True)
    assert its.min() < 25
    got = host("576x288").decode_i8(llr, 25, default_params(early_term=1))
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("code,ebn0", [("576x288", 2.0), ("dvbs2_r1_2", 1.1)])
@pytest.mark.parametrize("algo", [ALGO_OMS, ALGO_NMS])
def test_host_early_termination_vs_oracle(code, ebn0, algo):
    """Per-codeword stop after the first iteration whose hard decisions satisfy
    H (the oracle's semantics), on a ragged 40-codeword batch (two blocks)."""
    t = load_table(code)
    llr = channel.awgn_i8_host(t.n, 40, seed=5, table=channel.i8_table(channel.sigma_from_ebn0(ebn0, t.k_info / t.n)))
    iters = 25
    o_algo, param = (O.NMS, 29) if algo == ALGO_NMS else (O.OMS, 1)
    exp, _, its = O.decode_i8(t, llr, iters, o_algo, param, early_term=True, return_soft=True,
                              threads=O.host_threads())
    assert its.min() < iters
    got = host(code).decode_i8(llr, iters, default_params(algo=algo, factor=29, early_term=1))
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("code,algo,beta,batch,iters", [("648x324", ALGO_MS, 0.0, 1, 10), ("648x324", ALGO_OMS, 0.15, 9, 20),
                                                        ("576x288", ALGO_NMS, 0.75, 5, 20)])
def test_host_float_decoder_vs_oracle(code, algo, beta, batch, iters):
    """configs[0] shape (802.11n N=648 r1/2, one codeword, 10 it, float
    min-sum on the host CPU) and other float variants: hard decisions equal
    the oracle's float restatement."""
    t = load_table(code)
    rng = np.random.default_rng(3)
    llr = (-1.0 + channel.sigma_from_ebn0(1.5, 0.5) * rng.standard_normal((batch, t.n))).astype(np.float32)
    exp, _, _ = O.decode_f32(t, llr, iters, O.NMS if algo == ALGO_NMS else O.OMS, beta)
    got = host(code).decode_f32(llr, iters, default_params(algo=algo, beta=beta))
    assert np.array_equal(got, exp)


def test_host_context_rejects_device_entry_points():
    d = host("576x288")
    p = default_params()
    L = _lib.lib()
    buf = (C.c_byte * 576)()
    assert L.ldpc_decode_i8_async(d._ctx, None, buf, buf, None, None, 1, 5, C.byref(p)) == _lib.LDPC_EUNSUPPORTED
    assert L.ldpc_awgn_i8_async(d._ctx, None, buf, 1, 0, 1, (C.c_uint32 * 64)(*([1] * 64)), None) == \
        _lib.LDPC_EUNSUPPORTED
    with pytest.raises(LdpcError):
        d.set_kernel(8)
    q = d.quantize(np.array([0.13, -0.13, 4.0, -4.0, np.nan], np.float32))
    assert q.tolist() == [1, -1, 31, -31, -31]


def test_host_sse4_object_has_no_vex():
    """the 16-lane SSE4.1 check loop is the path for hosts without
    AVX2, so it must not be VEX-encoded (it was compiled under an avx2 target
    attribute until r06).  host_sse4.cpp is now its own translation unit built
    with -msse4.1 only; the build check disassembles it."""
    import subprocess
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    objdir = os.path.join(root, "build", "obj")
    if not os.path.exists(os.path.join(objdir, "host_sse4.o")):
        pytest.skip("objects not built here")
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "check_host_isa.py"), objdir],
                         capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
