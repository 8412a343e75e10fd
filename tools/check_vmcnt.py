#!/usr/bin/env python3
"""Build-time guard for coop3's hand-counted `s_waitcnt vmcnt(36)`.

coop3's memory wave (csrc/coop3_kernel.h, `mperiod`) issues, per period, for each of
the WS slab-wave sets (6 for DVB-S2 r1/2's kernel, 4 for r2/3 and the shaped r3/4,
2 for first-group degrees 22 .. 30), in this order: NLD line loads (all sets),
NGI LDS-DMA gathers (`buffer_load_dwordx4 ... lds`, inline asm the compiler does
not count), NLD line writebacks and NSI stores -- (2 NLD + NGI + NSI) WS
vector-memory instructions, NLD = ceil((D0 - 2) / 8), NGI = NSI = 1 up to
degree 16, 2 above -- and closes the period with vmcnt((3 NLD + NGI + 2 NSI) WS)
right before its barrier:
everything up to the previous period's gathers (and so its line loads) has
landed.  That count is only right while the compiler emits exactly those 24
instructions per period (no split, no extra load, no scratch spill).  This
script disassembles the built coop3 kernels and checks it: every straight-line
region between two consecutive period-closing waits (`s_waitcnt vmcnt(36)`
followed by the `s_barrier` with no vector-memory instruction between; no
scalar / VCC branch inside the region: those are the guarded first / last
periods) must hold exactly --ops vector-memory instructions, at least
--min-regions such regions must exist per kernel, and no coop3 kernel may touch
scratch.  (The compiler's own waits for the line loads it tracks are stricter
than needed and not period boundaries.)

usage: check_vmcnt.py [--ops N] [--vmcnt N] <coop3.o | libldpc_mi355x.so | file.s>
exit 0 = ok, 1 = mismatch (the message names the kernel and region).
"""
import argparse
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
VMEM = re.compile(r"^\s*(buffer_|global_|scratch_|flat_)\w+")
BRANCH = re.compile(r"^\s*s_(cbranch_(scc|vcc)\w*|branch|setpc|swappc)\b")


def disassemble(path):
    """ISA text of the gfx950 code object(s) inside a host object / library."""
    if path.endswith(".s"):
        return open(path).read()
    tmp = tempfile.mkdtemp(prefix="vmcnt_")
    try:
        src = os.path.join(tmp, os.path.basename(path))
        shutil.copy(path, src)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", src], cwd=tmp, check=True,
                       capture_output=True)
        out = []
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" in f and "gfx950" in f:
                r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950",
                                    os.path.join(tmp, f)], check=True, capture_output=True, text=True)
                out.append(r.stdout)
        if not out:
            raise SystemExit("check_vmcnt: no gfx950 code object in %s" % path)
        return "\n".join(out)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def functions(isa):
    """{symbol: [instruction lines]} of the disassembly."""
    funcs, name = {}, None
    for line in isa.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            name = m.group(1)
            funcs.setdefault(name, [])
        elif name and line.strip():
            funcs[name].append(line)
    return funcs


def kind(line):
    """L: a load into VGPRs, G: an LDS-DMA load (`... lds`), S: a store."""
    if "_store" in line.split("//")[0]:
        return "S"
    if re.search(r"\blds\b", line.split("//")[0]):
        return "G"
    return "L"


def closes_period(lines, i, reach=12):
    """The wait at line i is followed by an s_barrier within `reach` lines,
    with no vector-memory instruction or branch before it."""
    for l in lines[i + 1:i + 1 + reach]:
        if re.match(r"^\s*s_barrier\b", l):
            return True
        if VMEM.match(l) or BRANCH.match(l):
            return False
    return False


# coop3_decode<D0, WS, R, STAMP, ET, NMS>: the slab-wave count WS and the line
# ops per lane group NLD = ceil((D0 - 2) / 8) set the period's op count
# ((2 NLD + 2) WS), their order and the closing wait ((3 NLD + 3) WS)
WS_NAME = re.compile(r"coop3_decodeILi(\d+)ELi(\d+)ELi\d+E")


def counts(name):
    """(ops, vmcnt, expected order) of a coop3 kernel from its template arguments."""
    m = WS_NAME.search(name)
    d0, ws = (int(m.group(1)), int(m.group(2))) if m else (7, 6)
    nld = (d0 - 2 + 7) // 8
    half = d0 >= 22                                          # two lanes per check: 4 slab waves of 4 slots
    mp = 10 if half else 2 * ((d0 + 7) // 8 + 1)            # message pieces per check (G3::MP)
    ws = 2 if half else ws                                   # the memory wave's 8-slot sets (G3::NSET)
    ngi, nsi = (8 * (mp + 1) + 63) // 64, (mp + 2 + 7) // 8   # gather / store instructions per 8-slot set
    return ((2 * nld + ngi + nsi) * ws, (3 * nld + ngi + 2 * nsi) * ws,
            "L" * (nld * ws) + "G" * (ngi * ws) + "S" * ((nld + nsi) * ws))


def check(isa, ops=None, vmcnt=None, min_regions=1, pattern="coop3_decode"):
    """List of error strings (empty = ok) and the number of regions checked.
    ops / vmcnt: force the counts (default: 4 WS / 6 WS from each kernel's
    template arguments)."""
    errs, checked = [], 0
    kernels = {k: v for k, v in functions(isa).items() if pattern in k}
    if not kernels:
        return ["no %s kernel in the disassembly" % pattern], 0
    base_ops, base_vmcnt = ops, vmcnt
    for name, lines in kernels.items():
        k_ops, k_vmcnt, want = counts(name)
        ops = base_ops if base_ops is not None else k_ops
        vmcnt = base_vmcnt if base_vmcnt is not None else k_vmcnt
        wait = re.compile(r"^\s*s_waitcnt\s+.*vmcnt\(%d\)" % vmcnt)
        if any(re.match(r"^\s*scratch_", l) for l in lines):
            errs.append("%s: scratch access (a spill adds vector-memory ops the vmcnt does not count)" % name)
        marks = [i for i, l in enumerate(lines) if wait.match(l) and closes_period(lines, i)]
        if not marks:
            errs.append("%s: no s_waitcnt vmcnt(%d)" % (name, vmcnt))
            continue
        good = 0
        for a, b in zip(marks, marks[1:]):
            body = lines[a + 1:b]
            if any(BRANCH.match(l) for l in body):
                continue
            n = sum(1 for l in body if VMEM.match(l))
            if n != ops:
                errs.append("%s: %d vector-memory instructions between the vmcnt(%d) waits at ISA lines %d and %d, "
                            "the wait assumes %d per period" % (name, n, vmcnt, a, b, ops))
            else:
                # the count is right only in this order: NLD WS line loads,
                # WS LDS-DMA gathers, then the (NLD + 1) WS writebacks / stores
                seq = "".join(kind(l) for l in body if VMEM.match(l))
                if seq != want:
                    errs.append("%s: vector-memory order %s between the waits at ISA lines %d and %d, the vmcnt(%d) "
                                "argument assumes %s (line loads, gathers, stores)" % (name, seq, a, b, vmcnt, want))
            good += 1
        if good < min_regions:
            errs.append("%s: only %d straight-line memory-wave periods found (want >= %d)" % (name, good,
                                                                                             min_regions))
        checked += good
    return errs, checked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--ops", type=int, default=None, help="force the vector-memory ops per period (default 4 WS)")
    ap.add_argument("--vmcnt", type=int, default=None, help="force the period's closing wait (default 6 WS)")
    ap.add_argument("--min-regions", type=int, default=1)
    a = ap.parse_args()
    errs, n = check(disassemble(a.path), a.ops, a.vmcnt, a.min_regions)
    if errs:
        for e in errs:
            print("check_vmcnt: " + e, file=sys.stderr)
        return 1
    print("check_vmcnt: ok (%d memory-wave periods checked: (2 NLD + NGI + NSI) WS vector-memory ops in order, "
          "vmcnt((3 NLD + NGI + 2 NSI) WS); degree 7: WS 6, NLD 1; 10: WS 4, NLD 1; 14: WS 4, NLD 2; 22: 2 sets, "
          "NLD 3, NGI = NSI = 2; 27, 30: 2 sets, NLD 4, NGI = NSI = 2)" % n)
    return 0


if __name__ == "__main__":
    sys.exit(main())
