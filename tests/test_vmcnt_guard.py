"""The build-time guard of coop3's hand-counted `s_waitcnt vmcnt(36)`
(tools/check_vmcnt.py, run by __graft_entry__.build()): the built kernels pass
it, and a count that does not match what the ISA issues per memory-wave period
fails it -- both a wrong expectation and an ISA with one extra load."""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tools"))
import check_vmcnt  # noqa: E402

LIB = os.path.join(ROOT, "ldpcgputegra_amd", "libldpc_mi355x.so")


def test_built_coop3_matches_its_vmcnt():
    errs, n = check_vmcnt.check(check_vmcnt.disassemble(LIB), 24, 36)
    assert errs == [] and n >= 6


def test_wrong_count_fails_the_build_check():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "check_vmcnt.py"), "--ops", "23", LIB],
                         capture_output=True, text=True)
    assert out.returncode == 1 and "the wait assumes 23 per period" in out.stderr


def test_an_extra_load_in_a_period_is_caught():
    funcs = check_vmcnt.functions(check_vmcnt.disassemble(LIB))
    name = next(k for k in funcs if "coop3_decode" in k and not check_vmcnt.ET_NAME.search(k))
    lines = funcs[name]
    waits = [i for i, l in enumerate(lines) if "vmcnt(36)" in l and check_vmcnt.closes_period(lines, i)]
    # duplicate one vector-memory instruction inside a straight-line period
    for a, b in zip(waits, waits[1:]):
        if not any(check_vmcnt.BRANCH.match(l) for l in lines[a + 1:b]):
            k = next(i for i in range(a + 1, b) if check_vmcnt.VMEM.match(lines[i]))
            lines.insert(k, lines[k])
            break
    isa = "0000000000000000 <%s>:\n" % name + "\n".join(lines)
    errs, _ = check_vmcnt.check(isa, 24, 36)
    assert len(errs) == 1 and "25 vector-memory instructions" in errs[0], errs
