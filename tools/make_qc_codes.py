#!/usr/bin/env python3
"""Write quasi-cyclic codes the reference does not ship as runtime code files.

BASELINE.json configs 1-2 name the IEEE 802.11n N=648 rate-1/2 code, which
is absent from /root/reference (SURVEY.md 8(a), 8(d) "Config 1").  Its
parity-check matrix is the standard's base matrix (IEEE Std 802.11n-2009,
Annex R, Table R.1, sub-block size Z=27) expanded with cyclically shifted
identities: base entry s at (r, c) puts ones at
H[r*Z + i][c*Z + (i + s) % Z], i = 0..Z-1; '-' is a zero block.

Layered order follows the reference's convention for its other 802.11n
table (code/x86/Constantes/1944x972/constantes_sse.h: checks grouped by
degree, highest degree first; base-matrix row order inside a group; edges of
a check in ascending variable order).  The table is entered from the public
standard and is NOT pinned by any reference file ("parity unpinned" for the
table itself; the decoders' parity on it is checked against the oracle like
every other H).  tests/test_codes.py checks its structure (full rank, the
dual-diagonal parity part, degrees).

Usage: python tools/make_qc_codes.py   (rewrites codes/648x324.ldpc and its
manifest entry)
"""
import hashlib
import json
import os
import struct

import numpy as np

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ldpcgputegra_amd", "codes")

Z648 = 27
BASE_648_R12 = """
 0 -  -  -  0  0  -  -  0  -  -  0  1  0  -  -  -  -  -  -  -  -  -  -
22 0  -  - 17  -  0  0 12  -  -  -  -  0  0  -  -  -  -  -  -  -  -  -
 6 -  0  - 10  -  -  - 24  -  0  -  -  -  0  0  -  -  -  -  -  -  -  -
 2 -  -  0 20  -  -  - 25  0  -  -  -  -  -  0  0  -  -  -  -  -  -  -
23 -  -  -  3  -  -  -  0  -  9 11  -  -  -  -  0  0  -  -  -  -  -  -
24 - 23  1 17  -  3  - 10  -  -  -  -  -  -  -  -  0  0  -  -  -  -  -
25 -  -  -  8  -  -  -  7 18  -  -  0  -  -  -  -  -  0  0  -  -  -  -
13 24 -  -  0  -  8  -  6  -  -  -  -  -  -  -  -  -  -  0  0  -  -  -
 7 20 - 16 22 10  -  - 23  -  -  -  -  -  -  -  -  -  -  -  0  0  -  -
11 -  -  - 19  -  -  - 13  -  3 17  -  -  -  -  -  -  -  -  -  0  0  -
25 -  8  - 23 18  - 14  9  -  -  -  -  -  -  -  -  -  -  -  -  -  0  0
 3 -  -  - 16  -  -  2 25  5  -  -  1  -  -  -  -  -  -  -  -  -  -  0
"""


def parse_base(text):
    return [[-1 if t == "-" else int(t) for t in line.split()] for line in text.strip().splitlines()]


def expand(base, z):
    """Rows of H as sorted variable lists, in base-row order."""
    rows = []
    for r, brow in enumerate(base):
        for i in range(z):
            rows.append(sorted(c * z + (i + s) % z for c, s in enumerate(brow) if s >= 0))
    return rows


def layered(rows):
    """Reference convention: group checks by degree (descending), stable."""
    degs = sorted({len(r) for r in rows}, reverse=True)
    groups, edges = [], []
    for d in degs:
        sel = [r for r in rows if len(r) == d]
        groups.append([d, len(sel)])
        for r in sel:
            edges.extend(r)
    return groups, np.array(edges, dtype=np.uint32)


def write(name, n, m, groups, ev, source):
    with open(os.path.join(OUT, name + ".ldpc"), "wb") as f:
        f.write(b"LDPCH001")
        f.write(struct.pack("<IIII", n, m, ev.size, len(groups)))
        for d, c in groups:
            f.write(struct.pack("<II", d, c))
        f.write(ev.astype("<u4").tobytes())
    mpath = os.path.join(OUT, "manifest.json")
    man = json.load(open(mpath))
    man[name] = dict(n=n, m=m, e=int(ev.size), groups=groups,
                     edge_var_sha256=hashlib.sha256(ev.astype("<u4").tobytes()).hexdigest(), source=source)
    with open(mpath, "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    base = parse_base(BASE_648_R12)
    assert len(base) == 12 and all(len(r) == 24 for r in base)
    rows = expand(base, Z648)
    groups, ev = layered(rows)
    write("648x324", 24 * Z648, 12 * Z648, groups, ev,
          "IEEE 802.11n-2009 Annex R Table R.1 (Z=27, R=1/2); not in the reference")
    print("648x324: groups %s, E=%d" % (groups, ev.size))


if __name__ == "__main__":
    main()
