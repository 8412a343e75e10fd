#!/usr/bin/env python3
"""Build-time guard for coop3's hand-counted `s_waitcnt vmcnt(36)`.

coop3's memory wave (csrc/coop3.hip, `mperiod`) issues, per period, for each of
the WS = 6 slab-wave sets, in this order: one line load, one LDS-DMA gather
(`buffer_load_dwordx4 ... lds`, inline asm the compiler does not count), one
line writeback and one store -- 4 * WS = 24 vector-memory instructions -- and
closes the period with vmcnt(24 + 2 * WS = 36) right before its barrier:
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

usage: check_vmcnt.py [--ops 24] [--vmcnt 36] <coop3.o | libldpc_mi355x.so | file.s>
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


def closes_period(lines, i, reach=8):
    """The wait at line i is followed by an s_barrier within `reach` lines,
    with no vector-memory instruction or branch before it."""
    for l in lines[i + 1:i + 1 + reach]:
        if re.match(r"^\s*s_barrier\b", l):
            return True
        if VMEM.match(l) or BRANCH.match(l):
            return False
    return False


ET_NAME = re.compile(r"coop3_decodeILi\d+ELi\d+ELb[01]ELb1E")


def check(isa, ops, vmcnt, min_regions=1, pattern="coop3_decode", et_ops=24, et_vmcnt=36):
    """List of error strings (empty = ok) and the number of regions checked.
    Early-termination kernels (template flag ET) are checked against
    et_ops / et_vmcnt (the same counts today)."""
    errs, checked = [], 0
    kernels = {k: v for k, v in functions(isa).items() if pattern in k}
    if not kernels:
        return ["no %s kernel in the disassembly" % pattern], 0
    base_ops, base_vmcnt = ops, vmcnt
    for name, lines in kernels.items():
        ops, vmcnt = (et_ops, et_vmcnt) if ET_NAME.search(name) else (base_ops, base_vmcnt)
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
                # the count is right only in this order: WS line loads, WS
                # LDS-DMA gathers, then the 2 WS writebacks / stores
                seq = "".join(kind(l) for l in body if VMEM.match(l))
                ws = ops // 4
                want = "L" * ws + "G" * ws + "S" * (2 * ws)
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
    ap.add_argument("--ops", type=int, default=24, help="vector-memory ops per memory-wave period (4 * WS)")
    ap.add_argument("--vmcnt", type=int, default=36, help="the period's closing wait (4 * WS + 2 * WS)")
    ap.add_argument("--et-ops", type=int, default=24, help="ET kernels' vector-memory ops per period")
    ap.add_argument("--et-vmcnt", type=int, default=36, help="ET kernels' period-closing wait")
    ap.add_argument("--min-regions", type=int, default=1)
    a = ap.parse_args()
    errs, n = check(disassemble(a.path), a.ops, a.vmcnt, a.min_regions, et_ops=a.et_ops, et_vmcnt=a.et_vmcnt)
    if errs:
        for e in errs:
            print("check_vmcnt: " + e, file=sys.stderr)
        return 1
    print("check_vmcnt: ok (%d memory-wave periods of %d / %d vector-memory ops, vmcnt(%d) / vmcnt(%d) with ET)"
          % (n, a.ops, a.et_ops, a.vmcnt, a.et_vmcnt))
    return 0


if __name__ == "__main__":
    sys.exit(main())
