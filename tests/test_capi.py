"""C-ABI surface (no GPU needed): every symbol of include/ldpc_mi355x.h is
exported, parameter validation and error codes follow the documented
contract, the host channel generator matches its numpy restatement."""
import ctypes as C
import os
import re

import numpy as np
import pytest
from conftest import ROOT

from ldpcgputegra_amd import _lib, channel, load_table
from golden.gen_golden import awgn_i8


def header_functions():
    txt = open(os.path.join(ROOT, "include", "ldpc_mi355x.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z0-9_]+)\s*\(", txt)))


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 25
    for n in names:
        assert hasattr(L, n), n
    # and the python binding declares a signature for each of them
    assert sorted(_lib.SIGNATURES) == names


def test_abi_version_and_strerror():
    L = _lib.lib()
    assert L.ldpc_abi_version() == 1
    assert L.ldpc_strerror(0) == b"ok"
    assert L.ldpc_strerror(-2) == b"unsupported configuration"


def test_default_params_match_reference_defaults():
    p = _lib.default_params()
    # code/x86/main_p.cpp:90-104,133-141
    assert (p.algo, p.offset, p.factor) == (0, 1, 29)
    assert (p.var_min, p.var_max, p.msg_min, p.msg_max) == (-127, 127, -31, 31)
    assert abs(p.beta - 0.15) < 1e-7 and p.early_term == 0


def test_ctx_create_without_device_fails_cleanly(gpu_available):
    if gpu_available:
        pytest.skip("device present")
    from ldpcgputegra_amd import Code, LdpcError, Decoder
    with pytest.raises(LdpcError) as ei:
        Decoder(Code("576x288"), max_batch=16)
    assert ei.value.status == _lib.LDPC_EDEVICE


def test_null_arguments_rejected():
    L = _lib.lib()
    assert L.ldpc_code_load(None, None) == _lib.LDPC_EINVAL
    h = C.c_void_p()
    assert L.ldpc_code_load(b"/nonexistent.ldpc", C.byref(h)) == _lib.LDPC_EIO
    assert L.ldpc_ctx_create(None, 0, 16, C.byref(h)) == _lib.LDPC_EINVAL


def test_sigma_formula():
    # CChanelAWGN_MKL::configure: sqrt(10^(-(EbN0 + 10log10 R)/10) / 2)
    for eb, r in [(1.0, 0.5), (2.5, 0.8), (0.0, 1 / 3)]:
        ref = np.sqrt(10 ** (-(eb + 10 * np.log10(r)) / 10) / 2)
        assert abs(channel.sigma_from_ebn0(eb, r) - ref) < 1e-12


@pytest.mark.parametrize("sat", [31, 15])
def test_host_generator_matches_numpy_spec(sat):
    t = channel.i8_table(0.8, 8, sat)
    assert t[63] == sat
    a = channel.awgn_i8_host(576, 8, seed=99, table=t, first_cw=5)
    b = awgn_i8(576, 8, 99, t, first_cw=5)
    assert np.array_equal(a, b)
    assert a.min() >= -sat and a.max() <= sat


def test_generator_distribution_matches_quantised_gaussian():
    sigma = 0.9
    t = channel.i8_table(sigma, 8, 31)
    q = channel.awgn_i8_host(64800, 4, seed=3, table=t).astype(np.int64).ravel()
    # sample of the reference chain: y = -1 + sigma z -> clamp(trunc(8 y), +-31)
    rng = np.random.default_rng(1)
    y = -1.0 + sigma * rng.standard_normal(q.size)
    r = np.clip(np.trunc(8 * y), -31, 31)
    for v in (-31, -8, -1, 0, 1, 5, 31):
        assert abs((q == v).mean() - (r == v).mean()) < 3e-3, v
    assert abs(q.mean() - r.mean()) < 0.05


def test_codeword_bits_flip_sign():
    t = channel.i8_table(0.7)
    zero = channel.awgn_i8_host(576, 2, 11, t)
    cw = np.zeros((2, 576), np.uint8)
    cw[:, ::3] = 1
    flipped = channel.awgn_i8_host(576, 2, 11, t, codeword=cw)
    assert np.array_equal(flipped[:, ::3], -zero[:, ::3])
    assert np.array_equal(np.delete(flipped, np.s_[::3], 1), np.delete(zero, np.s_[::3], 1))
