#!/usr/bin/env python3
"""Build-time check of the host decoder's per-ISA objects (host_simd.h): the
SSE4.1 object -- the path for hosts WITHOUT AVX2 -- must hold no VEX-encoded
instruction (a `v`-prefixed x86 mnemonic such as vpminsb / vmovdqa would fault
with SIGILL exactly there), and the AVX2 object must actually use 256-bit
registers.

usage: check_host_isa.py [objdir]   (default: <repo>/build/obj)
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def mnemonics(obj):
    out = subprocess.run(["objdump", "-d", "--no-show-raw-insn", obj], capture_output=True, text=True, check=True).stdout
    for line in out.splitlines():
        m = re.match(r"\s*[0-9a-f]+:\s+(\S+)\s*(.*)", line)
        if m:
            yield m.group(1), m.group(2)


def check(objdir):
    sse4 = os.path.join(objdir, "host_sse4.o")
    avx2 = os.path.join(objdir, "host_avx2.o")
    for p in (sse4, avx2):
        if not os.path.exists(p):
            raise SystemExit("check_host_isa: %s missing (build first)" % p)
    vex = sorted({mn for mn, _ in mnemonics(sse4) if mn.startswith("v") and mn not in ("verr", "verw")})
    if vex:
        raise SystemExit("check_host_isa: VEX instructions in the SSE4.1 object: %s" % ", ".join(vex[:12]))
    ymm = sum(1 for _, ops in mnemonics(avx2) if "%ymm" in ops)
    if ymm == 0:
        raise SystemExit("check_host_isa: the AVX2 object uses no ymm register")
    print("check_host_isa: ok (host_sse4.o: no VEX instruction; host_avx2.o: %d ymm instructions)" % ymm)


if __name__ == "__main__":
    check(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "build", "obj"))
