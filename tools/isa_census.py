#!/usr/bin/env python3
"""ISA census of a kernel: instruction classes per region between barriers.

usage: isa_census.py <lib.so | obj.o | file.s> [kernel-substring] [--min-valu N]
Prints, for every region between two s_barrier of the chosen kernel(s), its
ISA line span and the counts of VALU (v_*), packed-16 VALU (v_pk_*), SALU
(s_*), LDS (ds_*), VMEM (buffer/global) and s_nop instructions, plus a
per-mnemonic histogram of the largest straight-line region of each kind
(--hist).  Used for coop3's per-period VALU census.
"""
import argparse
import collections
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import check_vmcnt  # noqa: E402


def classify(mn):
    if mn.startswith("v_"):
        return "valu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("buffer_", "global_", "scratch_", "flat_")):
        return "vmem"
    if mn == "s_nop":
        return "nop"
    if mn.startswith("s_"):
        return "salu"
    return "other"


def regions(lines):
    cur, start = [], 0
    for i, l in enumerate(lines):
        mn = l.split()[0] if l.split() else ""
        if mn == "s_barrier":
            yield start, i, cur
            cur, start = [], i + 1
        else:
            cur.append(mn)
    yield start, len(lines), cur


def coop3_census(funcs, kernel="coop3_decodeILi6ELi2ELb0ELb0ELb0E"):
    """One steady period of coop3 (DVB-S2 r1/2, WS = 6): the slab waves' fast
    period split at its branches (the shared prefix, the post variants for
    slab wave 0 / the others, the pre), a memory-wave period (between two
    period-closing vmcnt waits) and a chain block of 8 steps; VALU also as lane-ops per
    check x codeword (a slab lane = one check x 2 codewords; the memory and
    chain waves serve a window's 48 checks x 16 codewords)."""
    name = next(k for k in funcs if kernel in k)
    L = funcs[name]
    mn = [l.split()[0] if l.split() else "" for l in L]
    out = {"kernel": name}
    st = [i for i, l in enumerate(L) if mn[i] == "s_setprio" and l.split()[1] == "1"]
    s0 = st[len(st) // 2]
    b = s0
    while not mn[b].startswith("s_cbranch"):
        b -= 1
    e = s0
    while mn[e] != "s_barrier":
        e += 1
    marks = [b] + [i for i in range(b + 1, e) if mn[i].startswith(("s_cbranch", "s_branch"))] + [e]
    parts = []
    for x, y in zip(marks, marks[1:]):
        c = collections.Counter(classify(m) for m in mn[x + 1:y])
        parts.append(dict(lines=[x, y], valu=c["valu"], salu=c["salu"], lds=c["lds"], nop=c["nop"]))
    out["slab_fast_period_blocks"] = parts
    w = [i for i, l in enumerate(L) if "vmcnt(" in l and check_vmcnt.closes_period(L, i)]
    for x, y in zip(w, w[1:]):
        if not any(mn[i].startswith(("s_cbranch_scc", "s_cbranch_vcc", "s_branch")) for i in range(x + 1, y)):
            c = collections.Counter(classify(m) for m in mn[x + 1:y])
            out["memory_wave_period"] = dict(lines=[x, y], valu=c["valu"], salu=c["salu"], lds=c["lds"],
                                             vmem=c["vmem"], nop=c["nop"],
                                             valu_lane_ops_per_check_cw=round(c["valu"] * 64 / (48 * 16), 2))
            break
    mad = [i for i, m in enumerate(mn) if m == "v_pk_mad_i16"]
    if len(mad) >= 16:
        x, y = mad[8], mad[16]
        c = collections.Counter(classify(m) for m in mn[x:y])
        out["chain_8_steps"] = dict(valu=c["valu"], lds=c["lds"], salu=c["salu"])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("kernel", nargs="?", default="coop3_decodeILi6ELi2ELb0ELb0ELb0E")
    ap.add_argument("--min-valu", type=int, default=100)
    ap.add_argument("--hist", action="store_true")
    ap.add_argument("--coop3", action="store_true", help="coop3 steady-period census as JSON")
    a = ap.parse_args()
    funcs = check_vmcnt.functions(check_vmcnt.disassemble(a.path))
    if a.coop3:
        import json
        print(json.dumps(coop3_census(funcs, a.kernel), indent=1))
        return
    for name, lines in funcs.items():
        if a.kernel not in name:
            continue
        print("==", name)
        for s, e, mns in regions(lines):
            c = collections.Counter(classify(m) for m in mns)
            if c["valu"] < a.min_valu:
                continue
            pk = sum(1 for m in mns if m.startswith("v_pk_"))
            br = sum(1 for m in mns if m.startswith("s_cbranch") or m == "s_branch")
            print("  lines %6d-%6d  valu %4d (pk %3d)  salu %3d  lds %3d  vmem %3d  nop %3d  branches %d"
                  % (s, e, c["valu"], pk, c["salu"], c["lds"], c["vmem"], c["nop"], br))
            if a.hist:
                h = collections.Counter(m for m in mns if m.startswith("v_"))
                print("    " + ", ".join("%s %d" % kv for kv in h.most_common()))


if __name__ == "__main__":
    main()
