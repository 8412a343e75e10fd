"""Synthetic AWGN channel (host side) for tests, BER sweeps and bench.py.

Integer-exact quantised generator shared bit-for-bit by the host
(``ldpc_awgn_i8_host``), the GPU kernel (``ldpc_awgn_i8_async``) and
tests/golden/gen_golden.py:

    u  = splitmix64((cw*N + i) ^ (seed * 0xD1B54A32D192ED03)) >> 32
    q0 = -sat + #{k < 2 sat : u >= table[k]}      (bit 0 sent as -1)
    q  = bit ? -q0 : q0

``table`` holds the 2*sat quantisation thresholds of
``clamp(trunc(factor * y), -sat, sat)``, y = -1 + sigma*z, z ~ N(0, 1), i.e.
exactly the distribution the reference produces with CChanelAWGN_MKL::generate
+ CFastFixConversion::generate (code/x86/CChanel/CChanelAWGN_MKL.cpp:128-143,
code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65), with a
deterministic counter-based RNG in place of MKL's MT2203 stream (not
available here; channel parity is therefore statistical, not bitwise).
"""
import ctypes as C

import numpy as np

from . import _lib


def sigma_from_ebn0(ebn0_db, rate):
    """CChanelAWGN_MKL::configure (code/x86/CChanel/CChanelAWGN_MKL.cpp:102-105)."""
    return float(_lib.lib().ldpc_awgn_sigma(float(ebn0_db), float(rate)))


def sigma_from_snr(snr_db, rate, es_n0=False):
    """CChanelAWGN_MKL::configure with its es_n0 option (:97-104)."""
    return float(_lib.lib().ldpc_awgn_sigma_ex(float(snr_db), float(rate), int(bool(es_n0))))


QPSK = 0.707106781   # CChanelAWGN_MKL.cpp:124
BPSK = 1.0


def i8_table(sigma, factor=8, sat=31, amp=BPSK, normalize=False):
    """Thresholds of q = clamp(trunc(factor * norm * (-amp + sigma z)), +-sat):
    BPSK / QPSK amplitude, norm = 2 / sigma^2 with the reference's normalize
    option (CChanelAWGN_MKL.cpp:114-143), else 1."""
    t = np.empty(64, dtype=np.uint32)
    norm = 2.0 / (sigma * sigma) if normalize else 1.0
    _lib.check(_lib.lib().ldpc_awgn_i8_table_ex(float(sigma), float(amp), float(norm), int(factor), int(sat),
                                                t.ctypes.data))
    return t


def awgn_i8_host(n, batch, seed, table, first_cw=0, codeword=None):
    out = np.empty((batch, n), dtype=np.int8)
    cw = None
    if codeword is not None:
        codeword = np.ascontiguousarray(codeword, dtype=np.uint8)
        cw = codeword.ctypes.data
    t = np.ascontiguousarray(table, dtype=np.uint32)
    _lib.check(_lib.lib().ldpc_awgn_i8_host(n, batch, first_cw, seed, t.ctypes.data, cw, out.ctypes.data))
    return out
