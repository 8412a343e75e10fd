"""numpy model of the windowed kernel's schedule (ldpcgputegra_amd/csrc/windowed.hip).

Test infrastructure: it re-derives, on the CPU, exactly the decomposition the
HIP kernel uses -- windows of 16 consecutive checks, per-check pre / chain /
post phases, the staircase chain value forwarded from check to check, the
read-ahead of V two windows early, and the compressed per-check messages --
so that the algebra can be checked against the oracle without a GPU.
"""
import numpy as np

S = 16


def clamp(x, lo, hi):
    return np.minimum(np.maximum(x, lo), hi)


def windows_of(table):
    """Same windows as plan.cpp: <= 16 consecutive checks of one degree group."""
    degs = np.concatenate([np.full(c, d) for d, c in table.groups])
    grp = np.concatenate([np.full(c, g) for g, (d, c) in enumerate(table.groups)])
    starts = np.concatenate([[0], np.cumsum(degs)[:-1]])
    wins, c = [], 0
    while c < table.m:
        n = 0
        while c + n < table.m and n < S and grp[c + n] == grp[c]:
            n += 1
        wins.append((c, n))
        c += n
    return wins, degs, grp, starts


def decode(table, llr, iters, offset=1, vmin=-127, mm=31):
    """OMS only.  Returns (hard, soft) like the oracle."""
    B, N = llr.shape
    V = llr.astype(np.int64).copy()
    wins, degs, grp, starts = windows_of(table)
    ev = table.edge_var.astype(np.int64)
    # compressed messages per check: (cst1, cst2, jmin, signs[D])
    c1 = np.zeros((table.m, B), np.int64)
    c2 = np.zeros((table.m, B), np.int64)
    jm = np.zeros((table.m, B), np.int64)
    sg = np.zeros((table.m, B, degs.max()), np.int64)

    def cst(x):
        return np.minimum(np.maximum(x - offset, 0), mm)

    carry = None
    for _ in range(iters):
        # group passes; the pipeline reads V two windows ahead inside a group
        for g in range(len(table.groups)):
            gw = [w for w in wins if grp[w[0]] == g]
            D = table.groups[g][0]
            X, O = D - 2, D - 1
            later = g > 0
            loaded = {}

            def load(i):
                first, n = gw[i]
                idx = np.stack([ev[starts[first + k]:starts[first + k] + D] for k in range(n)])  # [n, D]
                return idx, V[:, idx].copy()                                                    # [B, n, D]

            for i in range(min(2, len(gw))):
                loaded[i] = load(i)
            for i, (first, n) in enumerate(gw):
                if i + 2 < len(gw):
                    loaded[i + 2] = load(i + 2)          # read ahead, before this window stores
                idx, vv = loaded.pop(i)
                chk = np.arange(first, first + n)
                r_old = np.where(jm[chk].T[:, :, None] == np.arange(D), c1[chk].T[:, :, None],
                                 c2[chk].T[:, :, None])
                m_old = np.where(sg[chk][:, :, :D].transpose(1, 0, 2) == 1, -r_old, r_old)   # [B, n, D]
                c = clamp(vv - m_old, vmin, 127)
                a = np.abs(np.minimum(c, mm)) if later else np.minimum(np.abs(c), mm)
                keep = np.arange(D) != X
                # chain: serial over the window's checks
                info = np.arange(D) < X
                i1 = np.where(info, a, 127).min(axis=2)
                s2 = (np.where(info, c < 0, False).sum(axis=2) & 1) ^ (D & 1)
                T = cst(i1)
                has_x = np.array([table_has_chain_in(table, ev, starts, degs, first + k) for k in range(n)])
                ys = np.zeros((B, n), np.int64)
                carry_in = carry
                m_x0 = m_old[:, :, X].copy()
                co0 = c[:, :, O].copy()
                for k in range(n):
                    yin = carry if (has_x[k] and carry is not None) else vv[:, k, X]
                    cx = clamp(yin - m_old[:, k, X], vmin, 127)
                    ax = np.abs(np.minimum(cx, mm)) if later else np.abs(cx)
                    r = clamp(ax - offset, 0, T[:, k])
                    neg = (cx < 0) ^ s2[:, k]
                    ys[:, k] = clamp(c[:, k, O] + np.where(neg == 1, -r, r), vmin, 127)
                    carry = ys[:, k]
                    c[:, k, X] = cx
                if not later and vmin == -127 and mm <= 63:
                    check_zchain(vv[:, :, X], m_x0, co0, T, s2, has_x, carry_in, ys, offset, n)
                a =np.abs(np.minimum(c, mm)) if later else np.minimum(np.abs(c), mm)
                # post
                m1 = a.min(axis=2)
                srt = np.sort(a, axis=2)
                m2 = srt[:, :, 1]
                k1, k2 = cst(m2), cst(m1)
                par = ((c < 0).sum(axis=2) & 1) ^ (D & 1)
                r = np.where(a == m1[:, :, None], k1[:, :, None], k2[:, :, None])
                neg = par[:, :, None] ^ (c < 0)
                vn = clamp(c + np.where(neg == 1, -r, r), vmin, 127)
                assert np.array_equal(vn[:, :, O], ys), "chain value != post value"
                for k in range(n):
                    V[:, idx[k]] = vn[:, k]
                jmin = np.argmax(a == m1[:, :, None], axis=2)
                c1[chk], c2[chk], jm[chk] = k1.T, k2.T, jmin.T
                sg[chk, :, :D] = neg.transpose(1, 0, 2)
    return (V > 0).astype(np.uint8), V.astype(np.int8)


def dz(u, off, T):
    """sign(u) * clamp(|u| - off, 0, T) == med3(u - med3(u, -off, off), -T, T)."""
    s = u - clamp(u, -off, off)
    return clamp(s, -T, T)


def check_zchain(vx, mx, co, T, s2, has_x, carry_in, ys, off, n):
    """The kernel's sign-normalised chain (windowed.hip, "z-domain"):
    y_k = co_k + eps_k dz(y_{k-1} - mx_k), eps_k = -1 if kpar_k else +1.
    With rho_k = eps_k rho_{k-1} and z_k = rho_k y_k:
      z_k = C_k + dz(u_k),  u_k = z_{k-1} + tau_k,
      C_k = rho_k co_k,  tau_k = -rho_{k-1} mx_k,
    so every step is med3 / sub / med3 / add.  Chain values are left
    unclamped (|y| <= 127 + T); clamping would not change any dz input that
    matters because |y - mx| >= 127 - msg_max > T + off there."""
    B = vx.shape[0]
    eps = np.where(s2 == 1, -1, 1)                  # [B, n]
    y_in = np.where(has_x[0] and carry_in is not None, carry_in if carry_in is not None else 0, vx[:, 0])
    rho_prev = np.ones(B, np.int64)
    z_prev = y_in * rho_prev
    for k in range(n):
        rho = eps[:, k] * rho_prev
        tau = -rho_prev * mx[:, k]
        u = z_prev + tau
        z = rho * co[:, k] + dz(u, off, T[:, k])
        y = rho * z
        assert np.array_equal(clamp(y, -127, 127), ys[:, k]), "z-domain chain mismatch at slot %d" % k
        # the kernel recovers the chain input of slot k from u: y_{k-1} = rho_{k-1} (u_k - tau_k)
        z_prev, rho_prev = z, rho


def table_has_chain_in(table, ev, starts, degs, ci):
    prev = (ci - 1) % table.m
    a = set(ev[starts[prev]:starts[prev] + degs[prev]].tolist())
    x = ev[starts[ci] + degs[ci] - 2]
    return int(x) in a and ev[starts[prev] + degs[prev] - 1] == x
