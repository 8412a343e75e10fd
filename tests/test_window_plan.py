"""The windowed2 schedule (plan.cpp ldpc_plan_windows) satisfies the rules
the kernel's read-ahead relies on, checked independently in numpy:
  * windows tile the schedule in order, <= S checks, one degree group each;
  * only slot 0 may lack a chain input (staircase link from the previous check);
  * inside a window only the chain link shares a variable;
  * a variable read by window u (its chain input excepted) is not written by
    windows u-P..u-1 of the same group."""
import numpy as np
import pytest

from ldpcgputegra_amd import Code, load_table


def chain_in(t, starts, degs, ci):
    p = (ci - 1) % t.m
    pv = t.edge_var[starts[p]:starts[p] + degs[p]]
    x = t.edge_var[starts[ci] + degs[ci] - 2]
    return pv[-1] == x and len(set(pv.tolist()) & set(t.edge_var[starts[ci]:starts[ci] + degs[ci]].tolist())) == 1


@pytest.mark.parametrize("code", ["dvbs2_r1_2", "dvbs2_r2_3"])
@pytest.mark.parametrize("S,P", [(16, 2), (32, 1)])
def test_window_plan_rules(code, S, P):
    t = load_table(code)
    plan = Code(code).window_plan(S, P)
    assert plan, "staircase code must have a plan"
    degs = np.concatenate([np.full(c, d) for d, c in t.groups])
    grp = np.concatenate([np.full(c, g) for g, (d, c) in enumerate(t.groups)])
    starts = np.concatenate([[0], np.cumsum(degs)[:-1]])
    nxt = 0
    writer = {}
    gstart = 0
    for u, (first, cnt) in enumerate(plan):
        assert first == nxt and 1 <= cnt <= S
        nxt = first + cnt
        g = grp[first]
        assert (grp[first:first + cnt] == g).all()
        if u > 0 and grp[plan[u - 1][0]] != g:
            gstart = u
        seen = {}
        for k in range(cnt):
            ci = first + k
            has_x = chain_in(t, starts, degs, ci)
            if k > 0:
                assert has_x, "chain break inside a window"
            vs = t.edge_var[starts[ci]:starts[ci] + degs[ci]]
            for j, v in enumerate(vs.tolist()):
                is_chain = has_x and j == degs[ci] - 2
                if is_chain:
                    continue
                assert v not in seen, "variable shared inside a window"
                lw = writer.get(v, -10 ** 9)
                assert not (lw >= gstart and lw >= u - P), "read-ahead hazard"
            for v in vs.tolist():
                seen[v] = k
        for k in range(cnt):
            for v in t.edge_var[starts[first + k]:starts[first + k] + degs[first + k]].tolist():
                writer[v] = u
    assert nxt == t.m
    # windows are mostly full
    assert np.mean([c for _, c in plan]) > 0.9 * S
