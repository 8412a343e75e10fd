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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("kernel", nargs="?", default="coop3_decodeILi6ELi2ELb0ELb0ELb0E")
    ap.add_argument("--min-valu", type=int, default=100)
    ap.add_argument("--hist", action="store_true")
    a = ap.parse_args()
    funcs = check_vmcnt.functions(check_vmcnt.disassemble(a.path))
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
