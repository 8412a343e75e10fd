"""CPU model of the packed-pair check arithmetic of pk16.h (test
infrastructure, no GPU), which coop3.hip's slab waves use (first written for
the since-removed coop2 kernel).

The kernel keeps two codewords per VGPR (one per 16-bit half): V in the "R
form" 256 x + 255, messages in the "C form" 256 m, and a check's messages for
a codeword pair as two dwords -- MA (a 2-bit code per edge and codeword) and
MB (the cst1 / cst2 bytes) -- decoded with v_perm_b32 through the byte table
[+cst1, -cst1, +cst2, -cst2].  This file emulates every instruction the
kernel's check update uses (v_pk_{add,sub}_i16 with and without clamp,
v_pk_{min,max}_i16, v_pk_ashrrev_i16, v_perm_b32, v_bfi_b32, shifts) on numpy
arrays and compares the result bit for bit with the reference's int8 check
update (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:201-254 for the first
degree group, :293-314 for later groups), over several
rounds so that the decoded old messages are exercised as well.
"""
import numpy as np
import pytest

M32 = 0xFFFFFFFF
RNEG127, R127, R0, C510 = 0x81FF81FF, 0x7FFF7FFF, 0x00FF00FF, 0x01FE01FE
HIBYTES, SIGNS = 0xFF00FF00, 0x80008000


# ---- instruction models on int64 arrays holding 32-bit registers ----------
def split(x):
    x = np.asarray(x, np.int64)
    lo, hi = x & 0xFFFF, (x >> 16) & 0xFFFF
    return lo - ((lo & 0x8000) << 1), hi - ((hi & 0x8000) << 1)


def join(lo, hi):
    return (np.asarray(lo, np.int64) & 0xFFFF) | ((np.asarray(hi, np.int64) & 0xFFFF) << 16)


def _pk(f):
    def op(a, b):
        (al, ah), (bl, bh) = split(a), split(b)
        return join(f(al, bl), f(ah, bh))
    return op


def _sat(v):
    return np.clip(v, -32768, 32767)


pk_sub_sat = _pk(lambda x, y: _sat(x - y))   # v_pk_sub_i16 ... clamp
pk_add_sat = _pk(lambda x, y: _sat(x + y))   # v_pk_add_i16 ... clamp
pk_sub = _pk(lambda x, y: x - y)             # v_pk_sub_i16 (wraps)
pk_max = _pk(np.maximum)                     # v_pk_max_i16
pk_min = _pk(np.minimum)                     # v_pk_min_i16


def pk_sra15(a):                             # v_pk_ashrrev_i16 15
    lo, hi = split(a)
    return join(np.where(lo < 0, -1, 0), np.where(hi < 0, -1, 0))


def bfi(m, a, b):                            # v_bfi_b32
    m = np.asarray(m, np.int64)
    return (m & a) | (~m & M32 & b)


def perm(s0, s1, sel):                       # v_perm_b32 (selectors 0..7, 0x0c, >= 0x0d)
    s0, s1, sel = np.broadcast_arrays(*(np.asarray(v, np.int64) for v in (s0, s1, sel)))
    src = np.stack([(s1 >> (8 * i)) & 0xFF for i in range(4)] + [(s0 >> (8 * i)) & 0xFF for i in range(4)])
    out = np.zeros(s0.shape, np.int64)
    for i in range(4):
        si = (sel >> (8 * i)) & 0xFF
        b = np.take_along_axis(src, np.minimum(si, 7)[None], 0)[0]
        b = np.where(si == 0x0C, 0, np.where(si >= 0x0D, 0xFF, b))
        out |= b << (8 * i)
    return out


# ---- the kernel's helpers (coop2.hip) --------------------------------------
def unpack_v(raw):
    return perm(raw, raw, 0x010D000D)


def pack_v(r):
    return perm(r, r, 0x0C0C0301)


def abs_r(r):
    return pk_max(r, pk_sub(C510, r))


def msg_tab(MB):
    p0, p1 = perm(MB, MB, 0x0C010C00), perm(MB, MB, 0x0C030C02)
    return perm(pk_sub(0, p0), p0, 0x06020400), perm(pk_sub(0, p1), p1, 0x06020400)


def old_msg(MA, tab, j):
    sh = (MA << (8 - 2 * j)) & M32 if j <= 4 else MA >> (2 * j - 8)
    return perm(tab[1], tab[0], (sh & 0x03000300) | 0x040C000C)


def abs_sat(r):                              # |x| of R(x) or of the saturated 0x8000, capped at R(127)
    return pk_max(r, pk_sub_sat(C510, r))


def signed_csts(k1, k2, sacc, D):
    """eps * k1, eps * k2 (C form), eps = -1 where the sign parity of the
    check's contributions (and the odd-degree flip) is odd."""
    Pm = pk_sra15(sacc ^ (SIGNS if D & 1 else 0))
    return pk_sub(k1 ^ Pm, Pm), pk_sub(k2 ^ Pm, Pm)


def new_v(j, c, a, min1, e1, e2, MA):
    """pk16.h new_v: V' = sign(c) * min(|c| + eps * cst, 127) -- the reference's
    max(sat(c + m), -127) with m = (c < 0) ^ par ? -cst : cst -- and edge j's
    code (bit 0: c < 0, bit 1: got cst2) into MA."""
    neq = pk_sra15(pk_sub(min1, a))
    T = pk_add_sat(a, bfi(neq, e2, e1))
    sc = pk_sra15(c)
    MA = MA | (sc & (0x00010001 << (2 * j))) | (neq & (0x00020002 << (2 * j)))
    return bfi(sc, pk_sub(C510, T), T), MA


def new_v_later(j, c, a, min1, e1, e2, MA):
    """The later degree group (a = |min(c, msg_max)| is not |c|): c clamped at
    -127 first, V' = max(sat(c + m), -127), same code / MB encoding."""
    neq = pk_sra15(pk_sub(min1, a))
    sc = pk_sra15(c)
    m = bfi(neq, e2, e1)
    MA = MA | (sc & (0x00010001 << (2 * j))) | (neq & (0x00020002 << (2 * j)))
    return pk_max(pk_add_sat(c, pk_sub(m ^ sc, sc)), RNEG127), MA


def kernel_check(vraw, MA, MB, off, mm, later):
    """One check for a vector of codeword pairs: vraw[j] = u16 V pair of edge
    j.  Returns (new V u16 pairs, MA, MB).  The kernel splits a first-group
    check into pre / chain / post; the chain only supplies the x edge's V, so
    the per-edge algebra is the same for every edge.  The first group works on
    the unclamped contributions (only their sign and saturated magnitude are
    used); MB holds eps * cst1, eps * cst2 (signed bytes) and MA bit 0 of an
    edge the sign of its contribution, so that the old message decodes as
    (-1)^sign * eps * cst through the same byte table."""
    D = len(vraw)
    rmm, coff = (mm * 256 + 255) * 0x10001, off * 256 * 0x10001
    tab = msg_tab(MB)
    c, a = [], []
    min1 = np.full(MA.shape, R127, np.int64)
    min2 = min1.copy()
    sacc = np.zeros(MA.shape, np.int64)
    for j in range(D):
        cj = pk_sub_sat(unpack_v(vraw[j]), old_msg(MA, tab, j))
        if later:
            cj = pk_max(cj, RNEG127)
            aj = abs_r(pk_min(cj, rmm))
        else:   # |c| unclipped (coop3: msg_max clips min1 / min2 instead, the same edges win)
            aj = abs_sat(cj)
        c.append(cj)
        a.append(aj)
        sacc = sacc ^ cj
        min2, min1 = pk_max(min1, pk_min(aj, min2)), pk_min(min1, aj)
    if later:
        k1, k2 = pk_min(pk_max(pk_sub(min2, coff), R0), rmm), pk_min(pk_max(pk_sub(min1, coff), R0), rmm)
    else:
        k1, k2 = pk_max(pk_sub(pk_min(min2, rmm), coff), R0), pk_max(pk_sub(pk_min(min1, rmm), coff), R0)
    k1, k2 = k1 & HIBYTES, k2 & HIBYTES
    e1, e2 = signed_csts(k1, k2, sacc, D)
    MAn = np.zeros(MA.shape, np.int64)
    vnew = []
    for j in range(D):
        vn, MAn = (new_v_later if later else new_v)(j, c[j], a[j], min1, e1, e2, MAn)
        vnew.append(pack_v(vn))
    return vnew, MAn, perm(e2, e1, 0x07030501)


# ---- reference and pair helpers --------------------------------------------
def ref_check(v, m, off, mm, later):
    """SURVEY.md 8(a) per-check recurrence (the oracle's semantics) on [B, D]."""
    B, D = v.shape
    c = np.maximum(np.clip(v - m, -128, 127), -127)
    a = np.abs(np.minimum(c, mm)) if later else np.minimum(np.abs(c), mm)
    min1 = np.full(B, 127)
    min2 = np.full(B, 127)
    for j in range(D):
        min2 = np.minimum(min2, np.maximum(a[:, j], min1))
        min1 = np.minimum(min1, a[:, j])
    cst1 = np.minimum(np.maximum(min2 - off, 0), mm)
    cst2 = np.minimum(np.maximum(min1 - off, 0), mm)
    par = ((c < 0).sum(axis=1) + D) & 1
    r = np.where(a == min1[:, None], cst1[:, None], cst2[:, None])
    mn = np.where((c < 0) ^ (par[:, None] == 1), -r, r)
    return np.maximum(np.clip(c + mn, -128, 127), -127), mn


def to_pairs(x):
    x = np.asarray(x, np.int64) & 0xFF
    return x[0::2] | (x[1::2] << 8)


def from_u16(raw):
    b = np.stack([raw & 0xFF, (raw >> 8) & 0xFF], axis=1).reshape(-1)
    return b - ((b & 0x80) << 1)


def hi_bytes(r):
    lo, hi = split(r)
    return np.stack([lo >> 8, hi >> 8], axis=1).reshape(-1)


def draw(rng, shape, lo=-127):
    v = rng.integers(lo, 128, shape)
    small = rng.random(shape) < 0.5          # small magnitudes: ties at min1 / min2
    v[small] = rng.integers(-3, 4, int(small.sum()))
    return v


# ---- tests -----------------------------------------------------------------
def test_saturating_forms_exhaustive():
    v = np.repeat(np.arange(-128, 128), 127)
    m = np.tile(np.arange(-63, 64), 256)
    R = join(256 * v + 255, 256 * v[::-1] + 255)
    C = join(256 * m, 256 * m[::-1])
    c = pk_max(pk_sub_sat(R, C), RNEG127)
    exp = np.maximum(np.clip(v - m, -128, 127), -127)
    lo, hi = split(c)
    assert np.array_equal(lo >> 8, exp) and np.array_equal(hi >> 8, exp[::-1])
    assert np.all((lo & 0xFF) == 0xFF) and np.all((hi & 0xFF) == 0xFF)     # stays in R form
    ok = exp >= -127
    n = pk_max(pk_add_sat(c, C), RNEG127)
    lo, _ = split(n)
    assert np.array_equal((lo >> 8)[ok], np.maximum(np.clip(exp + m, -128, 127), -127)[ok])
    a = abs_r(c)
    lo, _ = split(a)
    assert np.array_equal(lo >> 8, np.abs(exp)) and np.all((lo & 0xFF) == 0xFF)


def test_v_pairs_round_trip():
    raw = np.arange(1 << 16)
    assert np.array_equal(pack_v(unpack_v(raw)), raw)


@pytest.mark.parametrize("later", [False, True])
@pytest.mark.parametrize("off,mm", [(0, 31), (1, 31), (3, 31), (0, 63), (1, 63)])
def test_packed_check_update_is_bit_exact(later, off, mm):
    rng = np.random.default_rng(97 * off + mm + 7 * later)
    n, D = 3000, (6 if later else 7)
    v = draw(rng, (2 * n, D), lo=-128)       # the channel may deliver -128
    m = np.zeros((2 * n, D), np.int64)       # messages start at 0: MA = MB = 0
    MA = np.zeros(n, np.int64)
    MB = np.zeros(n, np.int64)
    for _ in range(4):
        tab = msg_tab(MB)
        for j in range(D):                   # the kernel decodes the reference's messages
            assert np.array_equal(hi_bytes(old_msg(MA, tab, j)), m[:, j])
        v_ref, m = ref_check(v, m, off, mm, later)
        vnew, MA, MB = kernel_check([to_pairs(v[:, j]) for j in range(D)], MA, MB, off, mm, later)
        for j in range(D):
            assert np.array_equal(from_u16(vnew[j]), v_ref[:, j]), "edge %d" % j
        v = np.where(rng.random(v.shape) < 0.5, v_ref, draw(rng, v.shape))
    tab = msg_tab(MB)
    for j in range(D):
        assert np.array_equal(hi_bytes(old_msg(MA, tab, j)), m[:, j])
