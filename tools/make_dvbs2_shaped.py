#!/usr/bin/env python3
"""DVB-S2-SHAPED stand-ins for the normal-frame rates 3/4 and 5/6.

BASELINE.json configs[4] mixes DVB-S2 rates {1/2, 3/4, 5/6}.  The reference
ships no r3/4 or r5/6 table (code/x86/Constantes/ holds 64800x{32400,7200,6480}
only, code/gpu_fixed/matrix/ adds 64800x21600) and ETSI EN 302 307 Annex B is
not reachable offline, so the real address tables cannot be entered here.
This tool writes tables with the Annex-B STRUCTURE of those rates -- the
same N, K, q, rows of 360 information bits, degree profile and staircase
parity (so exactly the decoder workload: edges, check degrees, window plans)
-- with seeded random addresses:

  rate 3/4: N=64800 K=48600 q=45, 15 rows of 12 addresses + 120 rows of 3
            (5400 degree-12 + 43200 degree-3 information bits; checks of
            degree 12 + 2)
  rate 5/6: N=64800 K=54000 q=30, 15 rows of 13 addresses + 135 rows of 3
            (5400 degree-13 + 48600 degree-3; checks of degree 20 + 2)

Every residue mod q gets the same number of addresses (regular check
degree), the addresses of a row have distinct residues and are at least
MIN_SPREAD apart (cyclically: no 4-cycle through the staircase, and the
reuse distance of a variable in the layered order that the windowed / coop
kernels' plans need), and a greedy test rejects
addresses closing a 4-cycle between two rows.  They are NOT the ETSI codes:
their BER curves differ from the standard's; decoder parity on them is
checked against the oracle and (the table being an input) is independent
of that.  Files: ldpcgputegra_amd/codes/dvbs2shape_r3_4.txt, _r5_6.txt.
usage: python tools/make_dvbs2_shaped.py
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SHAPES = {  # name: (K, q, [(rows, addresses per row), ...])
    "dvbs2shape_r3_4": (48600, 45, [(15, 12), (120, 3)]),
    "dvbs2shape_r5_6": (54000, 30, [(15, 13), (135, 3)]),
}
N = 64800
MIN_SPREAD = 64


def make(K, q, layout, seed):
    M = N - K
    assert M == 360 * q
    rows = [d for cnt, d in layout for _ in range(cnt)]
    assert len(rows) * 360 == K
    total = sum(rows)
    per_res = total // q
    assert per_res * q == total, "regular check degree needs total % q == 0"
    rng = np.random.default_rng(seed)
    for attempt in range(200):
        left = np.full(q, per_res)
        tab = []                                 # per row: list of (residue, t)
        by_res = [[] for _ in range(q)]          # residue -> [(row, t)]
        ok = True
        for a, d in enumerate(rows):
            row = []
            # residues with the most addresses left first (keeps the end feasible)
            for _ in range(d):
                used = {r for r, _ in row}
                cand = [r for r in range(q) if left[r] > 0 and r not in used]
                if not cand:
                    ok = False
                    break
                mx = max(left[r] for r in cand)
                pool = [r for r in cand if left[r] >= mx - 1]
                placed = False
                for r in rng.permutation(pool):
                    for t in rng.permutation(360)[:128]:
                        x = r + q * t
                        # addresses of a row at least MIN_SPREAD apart (cyclically): an information
                        # bit's checks are its row's addresses + m q, so this is the
                        # distance between two touches of one variable in the layered order
                        # (the windowed / coop plans need it; the real tables have >= 51)
                        if any(min((x - (r2 + q * t2)) % M, ((r2 + q * t2) - x) % M) < MIN_SPREAD
                               for r2, t2 in row):
                            continue
                        # 4-cycle with row b: residues r, r2 both in rows a and b
                        # with equal t differences (mod 360)
                        bad = False
                        for r2, t2 in row:
                            for b, tb in by_res[r]:
                                for b2, tb2 in by_res[r2]:
                                    if b2 == b and (t - tb - t2 + tb2) % 360 == 0:
                                        bad = True
                                        break
                                if bad:
                                    break
                            if bad:
                                break
                        if bad:
                            continue
                        row.append((int(r), int(t)))
                        left[r] -= 1
                        placed = True
                        break
                    if placed:
                        break
                if not placed:
                    ok = False
                    break
            if not ok:
                break
            for r, t in row:
                by_res[r].append((a, t))
            tab.append(sorted(r + q * t for r, t in row))
        if ok:
            return tab
    raise RuntimeError("no table found")


def main():
    out_dir = os.path.join(ROOT, "ldpcgputegra_amd", "codes")
    for i, (name, (K, q, layout)) in enumerate(SHAPES.items()):
        tab = make(K, q, layout, seed=302307 + i)
        path = os.path.join(out_dir, name + ".txt")
        with open(path, "w") as f:
            f.write("# SYNTHETIC DVB-S2-shaped table (tools/make_dvbs2_shaped.py): the Annex-B structure of this rate\n")
            f.write("# (N, K, q, degree profile, staircase parity) with seeded random addresses -- NOT the ETSI EN 302 307\n")
            f.write("# table, which is absent from the reference and not available offline\n")
            f.write("# N=%d K=%d q=%d rows=%d\n" % (N, K, q, len(tab)))
            for row in tab:
                f.write(" ".join(str(x) for x in row) + "\n")
        print("wrote", path, file=sys.stderr)


if __name__ == "__main__":
    main()
