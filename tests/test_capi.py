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


def test_channel_options_qpsk_esn0_normalize():
    """CChanelAWGN_MKL's options (code/x86/CChanel/CChanelAWGN_MKL.cpp:97-143):
    Es/N0 input (Eb/N0 = Es/N0 - 10 log10(2R)), QPSK amplitude 0.707106781 and
    the 2/sigma^2 normalisation.  Every threshold of the integer-exact
    generator's table sits where clamp(trunc(factor * norm * (-amp + sigma z)))
    steps by one level, and the defaults reproduce the plain BPSK table."""
    import math
    from scipy.stats import norm as N
    from ldpcgputegra_amd import channel
    r = 0.5
    assert channel.sigma_from_snr(1.0, r) == channel.sigma_from_ebn0(1.0, r)
    assert channel.sigma_from_snr(1.0, r, es_n0=True) == pytest.approx(
        channel.sigma_from_ebn0(1.0 - 10 * math.log10(2 * r), r))
    s = channel.sigma_from_ebn0(1.2, r)
    assert np.array_equal(channel.i8_table(s), channel.i8_table(s, amp=channel.BPSK, normalize=False))
    for amp, normalize, factor, sat in ((channel.QPSK, False, 8, 31), (1.0, True, 8, 31), (channel.QPSK, True, 4, 15)):
        t = channel.i8_table(s, factor, sat, amp=amp, normalize=normalize)
        assert t[63] == sat
        nm = 2.0 / (s * s) if normalize else 1.0
        q = lambda y: int(np.clip(np.trunc(factor * nm * y), -sat, sat))   # noqa: E731
        th = t[:2 * sat].astype(np.float64)
        assert np.all(np.diff(th) >= 0)
        for k in range(2 * sat):
            if th[k] <= 0 or th[k] >= 2.0 ** 32 - 1:
                continue
            z = N.ppf(th[k] / 2.0 ** 32)
            y = -amp + s * z
            # the threshold is p rounded to 2^-32: in y that is s * 2^-32 / pdf(z)
            eps = max(1e-7, 4 * s * 2.0 ** -32 / N.pdf(z))
            if factor * nm * eps > 0.25:
                continue                                       # deep tail: resolution coarser than a level
            assert q(y + eps) - q(y - eps) == 1, (amp, normalize, k)
            assert q(y + eps) == -sat + k + 1
