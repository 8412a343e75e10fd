"""The build-time guard of coop3's hand-counted `s_waitcnt vmcnt(6 WS)`
(tools/check_vmcnt.py, run by __graft_entry__.build()): the built kernels
(degree 7: WS = 6, vmcnt(36); degree 10: WS = 4, vmcnt(24)) pass it, and a
count that does not match what the ISA issues per memory-wave period fails it
-- a wrong expectation, an ISA with one extra load, and one in another order."""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_vmcnt  # noqa: E402

LIB = os.path.join(ROOT, "ldpcgputegra_amd", "libldpc_mi355x.so")


def test_built_coop3_matches_its_vmcnt():
    isa = check_vmcnt.disassemble(LIB)
    errs, n = check_vmcnt.check(isa)
    assert errs == [] and n >= 12
    names = [k for k in check_vmcnt.functions(isa) if "coop3_decode" in k]
    assert any("coop3_decodeILi7ELi6E" in k for k in names) and any("coop3_decodeILi10ELi4E" in k for k in names)


def test_wrong_count_fails_the_build_check():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_vmcnt.py"), "--ops", "23", LIB],
                         capture_output=True, text=True)
    assert out.returncode == 1 and "the wait assumes 23 per period" in out.stderr


def test_an_extra_load_in_a_period_is_caught():
    funcs = check_vmcnt.functions(check_vmcnt.disassemble(LIB))
    name = next(k for k in funcs if "coop3_decodeILi7ELi6E" in k)
    lines = funcs[name]
    waits = [i for i, l in enumerate(lines) if "vmcnt(36)" in l and check_vmcnt.closes_period(lines, i)]
    # duplicate one vector-memory instruction inside a straight-line period
    for a, b in zip(waits, waits[1:]):
        if not any(check_vmcnt.BRANCH.match(l) for l in lines[a + 1:b]):
            k = next(i for i in range(a + 1, b) if check_vmcnt.VMEM.match(lines[i]))
            lines.insert(k, lines[k])
            break
    isa = "0000000000000000 <%s>:\n" % name + "\n".join(lines)
    errs, _ = check_vmcnt.check(isa)
    assert len(errs) == 1 and "25 vector-memory instructions" in errs[0], errs


def test_a_reordered_period_is_caught():
    """Same count, another order (a store before the gathers): the wait's
    argument assumes loads, then gathers, then stores."""
    funcs = check_vmcnt.functions(check_vmcnt.disassemble(LIB))
    name = next(k for k in funcs if "coop3_decodeILi10ELi4E" in k)
    lines = funcs[name]
    waits = [i for i, l in enumerate(lines) if "vmcnt(24)" in l and check_vmcnt.closes_period(lines, i)]
    for a, b in zip(waits, waits[1:]):
        if not any(check_vmcnt.BRANCH.match(l) for l in lines[a + 1:b]):
            vm = [i for i in range(a + 1, b) if check_vmcnt.VMEM.match(lines[i])]
            st = next(i for i in vm if check_vmcnt.kind(lines[i]) == "S")
            lines.insert(vm[0], lines.pop(st))   # first store moved to the period's start
            break
    isa = "0000000000000000 <%s>:\n" % name + "\n".join(lines)
    errs, _ = check_vmcnt.check(isa)
    assert len(errs) == 1 and "vector-memory order" in errs[0], errs
