"""Code tables: numpy reader, C-ABI loader and DVB-S2 Annex-B builder agree,
and reproduce the reference's PosNoeudsVariable tables (sha256 recorded by
tools/extract_codes.py in codes/manifest.json)."""
import hashlib
import json
import os

import numpy as np
import pytest

from ldpcgputegra_amd import Code, available, codes, load_table

MANIFEST = json.load(open(os.path.join(codes.CODE_DIR, "manifest.json")))


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_table_matches_reference_hash(name):
    t = load_table(name)
    m = MANIFEST[name]
    assert (t.n, t.m, t.e) == (m["n"], m["m"], m["e"])
    assert [list(g) for g in t.groups] == m["groups"]
    assert hashlib.sha256(t.edge_var.astype("<u4").tobytes()).hexdigest() == m["edge_var_sha256"]


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_c_loader_matches_numpy_reader(name):
    t = load_table(name)
    c = Code(name)
    t2 = c.table()
    assert (c.n, c.m, c.e) == (t.n, t.m, t.e)
    assert t2.groups == t.groups
    assert np.array_equal(t2.edge_var, t.edge_var)


def test_dvbs2_structure():
    t = load_table("dvbs2_r1_2")
    assert (t.n, t.m, t.e) == (64800, 32400, 226799)
    assert t.groups == [(7, 32399), (6, 1)]
    c = Code("dvbs2_r1_2")
    info = c.plan_info()
    assert info["staircase"]
    assert info["min_hazard"] >= 60          # measured: 62 (SURVEY / plan.cpp)


def gf2_rank(h):
    h = h.copy()
    r = 0
    for c in range(h.shape[1]):
        piv = np.nonzero(h[r:, c])[0]
        if piv.size == 0:
            continue
        p = r + piv[0]
        h[[r, p]] = h[[p, r]]
        rows = np.nonzero(h[:, c])[0]
        rows = rows[rows != r]
        h[rows] ^= h[r]
        r += 1
        if r == h.shape[0]:
            break
    return r


def test_80211n_648_structure():
    """The 802.11n N=648 R=1/2 table (tools/make_qc_codes.py, entered from
    the standard; absent from the reference): degrees, full rank, the
    dual-diagonal parity part, and a systematic encoder that satisfies H."""
    t = load_table("80211n_648")
    assert (t.n, t.m, t.e) == (648, 324, 2376)
    assert t.groups == [(8, 108), (7, 216)]
    H = np.zeros((t.m, t.n), dtype=np.uint8)
    for i, (_, vs) in enumerate(t.checks()):
        H[i, vs] = 1
    assert H.sum() == t.e                          # no repeated edge
    assert gf2_rank(H) == t.m
    colw = H.sum(axis=0)
    assert colw.min() >= 2 and colw[t.n - t.m:].max() <= 3   # parity columns: weight 3 (first), 2 (diagonal)
    # systematic encoding by elimination on the parity part: H = [A | B], B p = A u
    A, B = H[:, : t.n - t.m], H[:, t.n - t.m:]
    assert gf2_rank(B) == t.m
    rng = np.random.default_rng(5)
    u = rng.integers(0, 2, t.n - t.m, dtype=np.uint8)
    aug = np.concatenate([B, (A.astype(np.int64) @ u % 2).astype(np.uint8)[:, None]], axis=1)
    # Gauss-Jordan on [B | A u]
    r = 0
    for c in range(t.m):
        p = r + np.nonzero(aug[r:, c])[0][0]
        aug[[r, p]] = aug[[p, r]]
        rows = np.nonzero(aug[:, c])[0]
        aug[rows[rows != r]] ^= aug[r]
        r += 1
    cw = np.concatenate([u, aug[:, -1]])
    assert not (H.astype(np.int64) @ cw % 2).any()


def test_generic_codes_have_no_staircase():
    assert not Code("576x288").plan_info()["staircase"]


def test_code_from_table_object_roundtrip():
    t = load_table("576x288")
    c = Code(t)
    assert np.array_equal(c.table().edge_var, t.edge_var)


def test_available_lists_shipped_codes():
    names = available()
    for n in ("576x288", "1944x972", "dvbs2_r1_2", "dvbs2_r2_3", "dvbs2_r8_9", "dvbs2_r9_10"):
        assert n in names


def test_bad_tables_rejected():
    from ldpcgputegra_amd import LdpcError, Table
    t = load_table("576x288")
    bad = t.edge_var.copy()
    bad[1] = bad[0]                                   # repeated variable in one check
    with pytest.raises(LdpcError):
        Code(Table(t.n, t.m, t.groups, bad))
    bad2 = t.edge_var.copy()
    bad2[5] = t.n                                     # out of range
    with pytest.raises(LdpcError):
        Code(Table(t.n, t.m, t.groups, bad2))
    with pytest.raises(FileNotFoundError):
        Code("no_such_code")


@pytest.mark.parametrize("name", ["dvbs2_r1_2", "dvbs2_r2_3", "dvbs2_r8_9", "dvbs2_r9_10"])
def test_dvbs2_encoder_codewords_satisfy_h(name):
    c = Code(name)
    t = load_table(name)
    rng = np.random.default_rng(3)
    info = rng.integers(0, 2, size=(3, c.k_info), dtype=np.uint8)
    cw = c.encode(info)
    assert np.array_equal(cw[:, :c.k_info], info)
    assert (t.syndrome(cw) == 0).all()
    assert cw[:, c.k_info:].any()


def test_encoder_requires_dvbs2_table():
    from ldpcgputegra_amd import LdpcError
    with pytest.raises(LdpcError):
        Code("576x288").encode(np.zeros((1, 288), np.uint8))


@pytest.mark.parametrize("name,k,q,profile", [("dvbs2shape_r3_4", 48600, 45, {12: 15, 3: 120}),
                                             ("dvbs2shape_r5_6", 54000, 30, {13: 15, 3: 135})])
def test_dvbs2_shaped_tables(name, k, q, profile):
    """configs[4]'s rates 3/4 and 5/6 are absent from the reference (and ETSI
    Annex B is not available offline): tools/make_dvbs2_shaped.py writes tables
    with their Annex-B structure.  Check that structure: N, K, q, rows of 360
    information bits with the standard's degree profile, regular checks of
    degree dc (+ staircase), the file regenerates identically, and random
    information words encode to codewords (H c = 0)."""
    import subprocess
    import sys
    path = os.path.join(os.path.dirname(__file__), "..", "ldpcgputegra_amd", "codes", name + ".txt")
    rows = [list(map(int, l.split())) for l in open(path) if l.strip() and not l.startswith("#")]
    from collections import Counter
    assert Counter(len(r) for r in rows) == Counter(profile)
    assert len(rows) * 360 == k
    t = load_table(name)
    assert (t.n, t.k_info) == (64800, k) and t.m == 360 * q
    dc = sum(d * c for d, c in profile.items()) * 360 // t.m
    assert t.groups == [(dc + 2, t.m - 1), (dc + 1, 1)]
    before = open(path).read()
    subprocess.check_call([sys.executable, os.path.join(os.path.dirname(path), "..", "..", "tools",
                                                        "make_dvbs2_shaped.py")], stderr=subprocess.DEVNULL)
    assert open(path).read() == before
    code = Code(name)
    info = np.random.default_rng(7).integers(0, 2, size=(4, k), dtype=np.uint8)
    cw = code.encode(info)
    assert np.array_equal(cw[:, :k], info)
    assert (t.syndrome(cw) == 0).all()
