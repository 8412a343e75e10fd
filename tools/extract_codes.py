#!/usr/bin/env python3
"""Convert the reference's compile-time H tables into runtime code files.

Run ONCE in the development container (it reads /root/reference, which does
not exist on the GPU box).  Output is pure data under
``ldpcgputegra_amd/codes/``:

* ``<name>.ldpc``   -- binary layered H table (format: ldpcgputegra_amd/codes/README.md)
* ``dvbs2_*.txt``   -- DVB-S2 Annex-B address tables (one row per 360-bit
  group), from which ``ldpc_code_from_dvbs2_table`` rebuilds H.

The reference stores H as a C header: ``PosNoeudsVariable[]`` (flattened
edge -> variable index list in *layered* order) plus ``DEG_k`` /
``DEG_k_COMPUTATIONS`` macros (e.g.
``code/x86/Constantes/64800x32400.dvb-s2/constantes_sse.h:6-36``,
``code/gpu_fixed/matrix/64800x21600/constantes_gpu.h:6-23``).  We parse those
numbers as text; no reference source is copied.

For DVB-S2 tables the Annex-B rows are *recovered from H*: the checks of
information bit ``360*g`` are exactly the addresses of row ``g`` (the encoder
rule ``(x + (v % 360) * q) % M`` of ``code/x86/CEncoder/GenericEncoder.cpp:60``
with ``v % 360 == 0``).  The script verifies that rebuilding H from the
recovered rows reproduces the reference table edge-for-edge.
"""
import hashlib
import json
import os
import re
import struct
import sys

import numpy as np

REF = "/root/reference/code"
OUT = os.path.join(os.path.dirname(__file__), "..", "ldpcgputegra_amd", "codes")

# name -> (macro header, table header)
SOURCES = {
    "576x288": ("x86/Constantes/576x288/constantes_sse.h",) * 2,
    "1944x972": ("x86/Constantes/1944x972/constantes_sse.h",) * 2,
    "2304x1152": ("x86/Constantes/2304x1152/constantes_sse.h",) * 2,
    "2048x384": ("x86/Constantes/2048x384/constantes_sse.h",) * 2,
    "4000x2000": ("x86/Constantes/4000x2000/constantes_sse.h",) * 2,
    "dvbs2_r1_2": ("x86/Constantes/64800x32400.dvb-s2/constantes_sse.h",) * 2,
    "dvbs2_r8_9": ("x86/Constantes/64800x7200.dvb-s2/constantes_sse.h",) * 2,
    "dvbs2_r9_10": ("x86/Constantes/64800x6480.dvb-s2/constantes_sse.h",) * 2,
    "dvbs2_r2_3": ("gpu_fixed/matrix/64800x21600/constantes_gpu.h",
                   "gpu_fixed/matrix/64800x21600/constantes_decoder.h"),
    "200x100": ("gpu_fixed/matrix/200x100/constantes_sse.h",) * 2,
    "816x408": ("gpu_fixed/matrix/816x408/constantes_gpu.h",
                "gpu_fixed/matrix/816x408/constantes_decoder.h"),
    "1024x518": ("gpu_fixed/matrix/1024x518/constantes_gpu.h",
                 "gpu_fixed/matrix/1024x518/constantes_decoder.h"),
    "1200x600": ("gpu_fixed/matrix/1200x600/constantes_gpu.h",
                 "gpu_fixed/matrix/1200x600/constantes_decoder.h"),
    "1248x624": ("gpu_fixed/matrix/1248x624/constantes_sse.h",) * 2,
    "4896x2448": ("gpu_fixed/matrix/4896x2448/constantes_gpu.h",
                  "gpu_fixed/matrix/4896x2448/constantes_decoder.h"),
    "8000x4000": ("gpu_fixed/matrix/8000x4000/constantes_gpu.h",
                  "gpu_fixed/matrix/8000x4000/constantes_decoder.h"),
    "9972x4986": ("gpu_fixed/matrix/9972x4986/constantes_gpu.h",
                  "gpu_fixed/matrix/9972x4986/constantes_decoder.h"),
    "20000x10000": ("gpu_fixed/matrix/20000x10000/constantes_gpu.h",
                    "gpu_fixed/matrix/20000x10000/constantes_decoder.h"),
    "16200x7560": ("gpu_fixed/matrix/16200x7560/constantes_sse.h",) * 2,
}

DVBS2 = {"dvbs2_r1_2", "dvbs2_r8_9", "dvbs2_r9_10", "dvbs2_r2_3"}

MAGIC = b"LDPCH001"


def _macro(text, name):
    m = re.search(r"^\s*#define\s+%s\s+(\d+)" % re.escape(name), text, re.M)
    return int(m.group(1)) if m else None


def parse(name):
    mac_path, tab_path = (os.path.join(REF, p) for p in SOURCES[name])
    mac = open(mac_path).read()
    n, m, e = _macro(mac, "_N"), _macro(mac, "_K"), _macro(mac, "_M")
    ngroups = _macro(mac, "NB_DEGRES")
    groups = [(_macro(mac, "DEG_%d" % (g + 1)), _macro(mac, "DEG_%d_COMPUTATIONS" % (g + 1)))
              for g in range(ngroups)]
    tab = open(tab_path).read()
    body = tab[tab.index("PosNoeudsVariable"):]
    body = body[body.index("{") + 1: body.index("}")]
    body = re.sub(r"/\*.*?\*/", " ", body, flags=re.S)
    vals = np.array([int(x) for x in re.findall(r"\d+", body)], dtype=np.uint32)
    assert vals.size == e, (name, vals.size, e)
    assert sum(d * c for d, c in groups) == e, (name, groups, e)
    assert sum(c for _, c in groups) == m, (name, groups, m)
    assert int(vals.max()) < n
    return dict(n=n, m=m, e=e, groups=groups, edge_var=vals)


def write_ldpc(path, code):
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<IIII", code["n"], code["m"], code["e"], len(code["groups"])))
        for d, c in code["groups"]:
            f.write(struct.pack("<II", d, c))
        f.write(code["edge_var"].astype("<u4").tobytes())


def dvbs2_rows_from_h(code):
    """Recover the Annex-B rows: the checks of info bit 360*g (see module doc)."""
    n, m = code["n"], code["m"]
    k = n - m
    assert k % 360 == 0 and m % 360 == 0
    q = m // 360
    # check index of every edge, in the reference's layered order:
    # rows 1..m-1 first, then row 0 (order rule of SURVEY.md 8(a) a7).
    degs = np.concatenate([np.full(c, d) for d, c in code["groups"]])
    starts = np.concatenate([[0], np.cumsum(degs)[:-1]])
    layered_rows = np.array(list(range(1, m)) + [0])
    edge_row = np.repeat(layered_rows, degs)
    ev = code["edge_var"]
    rows = []
    for g in range(k // 360):
        rows.append(sorted(int(r) for r in edge_row[ev == 360 * g]))
    return q, rows


def dvbs2_h_from_rows(n, m, q, rows):
    """Independent python model of ldpc_code_from_dvbs2_table (used to verify)."""
    k = n - m
    info = [[] for _ in range(m)]
    for g, row in enumerate(rows):
        for kk in range(360):
            v = 360 * g + kk
            for x in row:
                info[(x + kk * q) % m].append(v)
    edges, groups = [], {}
    order = list(range(1, m)) + [0]
    for r in order:
        lst = sorted(info[r])
        if r > 0:
            lst += [k + r - 1, k + r]
        else:
            lst += [k]
        edges.extend(lst)
    return np.array(edges, dtype=np.uint32)


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = {}
    for name in SOURCES:
        code = parse(name)
        write_ldpc(os.path.join(OUT, name + ".ldpc"), code)
        h = hashlib.sha256(code["edge_var"].astype("<u4").tobytes()).hexdigest()
        manifest[name] = dict(n=code["n"], m=code["m"], e=code["e"],
                              groups=code["groups"], edge_var_sha256=h)
        if name in DVBS2:
            q, rows = dvbs2_rows_from_h(code)
            rebuilt = dvbs2_h_from_rows(code["n"], code["m"], q, rows)
            assert np.array_equal(rebuilt, code["edge_var"]), name
            with open(os.path.join(OUT, name + ".txt"), "w") as f:
                f.write("# DVB-S2 (ETSI EN 302 307 Annex B) parity address table\n")
                f.write("# N=%d K=%d q=%d rows=%d\n" % (code["n"], code["n"] - code["m"], q, len(rows)))
                for row in rows:
                    f.write(" ".join(str(x) for x in row) + "\n")
            manifest[name]["dvbs2"] = dict(q=q, rows=len(rows))
        print(name, code["n"], code["m"], code["e"], code["groups"], file=sys.stderr)
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
