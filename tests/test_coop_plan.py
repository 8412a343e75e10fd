"""The workgroup-cooperative kernel's schedule (coop.hip build_plan) satisfies
the rules its pipeline relies on, re-derived here in numpy from the H table:

  * windows tile the first degree group in schedule order (<= S checks each,
    empty windows allowed), the tail check (second group) has a window of
    its own;
  * no information variable is shared inside a window or by two consecutive
    windows, cyclically (the kernel loads window u+1 before window u stores);
  * the number of forwarded reads (latest writer 2 .. R+1 windows back) matches.
"""
import numpy as np
import pytest

from ldpcgputegra_amd import Code, load_table


def checks(t):
    out, e = [], 0
    for d, c in t.groups:
        for _ in range(c):
            out.append(t.edge_var[e:e + d].tolist())
            e += d
    return out


@pytest.mark.parametrize("code", ["dvbs2_r1_2", "dvbs2_r2_3"])
@pytest.mark.parametrize("S,R,dist", [(24, 3, 1), (28, 3, 1), (28, 4, 1), (32, 3, 1), (24, 3, 2)])
def test_coop_plan_rules(code, S, R, dist):
    t = load_table(code)
    plan = Code(code).coop_plan(S, R, dist)
    assert plan is not None
    ch = checks(t)
    M, D0 = t.m, t.groups[0][0]
    X = D0 - 2
    wins, tail = plan["windows"], plan["tail"]
    nw = len(wins)
    # tiling
    nxt = 0
    for u, (first, cnt) in enumerate(wins):
        assert 0 <= cnt <= S
        if u == tail:
            assert (first, cnt) == (M - 1, 1)
            continue
        if cnt:
            assert first == nxt and first + cnt <= M - 1
            nxt = first + cnt
    assert nxt == M - 1
    info = [set(ch[c][:X]) if c < M - 1 else set(ch[c][:X]) for c in range(M)]
    wvars = []
    for first, cnt in wins:
        s = set()
        for c in range(first, first + cnt):
            assert not (s & info[c]), "info variable shared inside a window"
            s |= info[c]
        wvars.append(s)
    for u in range(nw):
        for d in range(1, dist + 1):
            assert not (wvars[u] & wvars[u - d]), "windows %d apart share a variable (u=%d)" % (d, u)
    # forwarded reads: latest earlier touch dist+1 .. R+dist windows back (cyclic)
    last = {}
    for u, (first, cnt) in enumerate(wins):
        for c in range(first, first + cnt):
            for v in ch[c][:X]:
                last[v] = u
    nf = 0
    for u, (first, cnt) in enumerate(wins):
        for c in range(first, first + cnt):
            for v in ch[c][:X]:
                d = (u - last[v]) % nw or nw
                if dist + 1 <= d <= R + dist:
                    nf += 1
                last[v] = u
    assert nf == plan["n_fwd"]
    # windows are mostly full and forwarding is rare
    assert (M - 1) / (nw * S) > (0.85 if dist == 1 else 0.8)
    assert plan["n_fwd"] < 0.05 * (M * X)


def test_coop_plan_absent_for_non_staircase():
    assert Code("576x288").coop_plan() is None
