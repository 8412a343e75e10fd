"""coop3's LDS line cache plan (ldpcgputegra_amd/csrc/linecache.cpp), host
side: built for DVB-S2 r1/2 within the kernel's slot budget and self-checked
by the planner's replay (lc_check_plan: every pre read / post write of the
coop3 schedule finds its line in the slot its record names, no slot is
refilled before its dirty line is written back, a line is reloaded only after
its store completed, and the lines left dirty at a segment end are exactly
the epilogue's).  No GPU needed."""
import pytest

from ldpcgputegra_amd.codes import Code, available


def test_dvbs2_r1_2_plan_fits_and_replays():
    lc = Code("dvbs2_r1_2").coop3_line_cache()
    assert lc is not None, "no line-cache plan (LDPC_LC_DEBUG=1 names the planner line)"
    assert 2 <= lc["slots"] <= lc["max_slots"]
    # ~8 accesses per residency: 162000 info-edge accesses per iteration (x2, pre and post)
    assert 12000 <= lc["residencies"] <= 21000
    assert 0 < lc["epilogue"] <= lc["prologue"] < lc["slots"]


def test_dvbs2_r2_3_plan_fits_and_replays():
    """First-group degree 10 (r2/3: 8 information edges per check, windows of
    30 checks at S = 32): the plan fits the degree-10 kernel's larger line
    cache and replays; the swizzle spreads its bank groups too."""
    lc = Code("dvbs2_r2_3").coop3_line_cache()
    assert lc is not None and 2 <= lc["slots"] <= lc["max_slots"] == 848
    assert 0 < lc["epilogue"] <= lc["prologue"] < lc["slots"]
    b = Code("dvbs2_r2_3").coop3_lc_banks()
    assert b["swizzled"] < 0.02 * b["plain"]


def test_dvbs2shape_r3_4_plan_fits_and_replays():
    """First-group degree 14 (the shaped r3/4: 12 information edges per
    check, two line loads per lane group and period): the greedy slot
    assignment does not fit the 784 slots, the packed chains + slot
    elimination do; the plan replays, and the schedule's self-check (no
    variable in neighbouring windows, every distance-2 writer / reader pair in
    slab wave 0 -- the pair the forwarding codes with 5 edge bits mark) holds."""
    lc = Code("dvbs2shape_r3_4").coop3_line_cache()
    assert lc is not None and 2 <= lc["slots"] <= lc["max_slots"] == 784


@pytest.mark.parametrize("name,slots", [("dvbs2shape_r5_6", 944), ("dvbs2_r8_9", 896), ("dvbs2_r9_10", 896)])
def test_degree_22_to_30_plans_fit_and_replay(name, slots):
    """First-group degree 22 / 27 / 30 (the shaped r5/6, the reference's
    r8/9 and r9/10: 20 .. 28 information edges per check, S = 16 windows at
    plan distance 2, 3 / 4 line loads per lane group and period): ~700 .. 840
    lines live at once, so the plan needs the packed chains, the slot
    elimination and its one-hold ejections to fit the kernel's line cache
    (r06: 944 / 896 / 896 slots beside the two-lanes-per-check kernel's
    160-B message records); it replays, and the swizzle spreads the bank
    groups of the two-lane accesses (instruction j of a slab wave: 2 slots x
    info entries j and XH + j per 32-lane half)."""
    lc = Code(name).coop3_line_cache()
    assert lc is not None and 2 <= lc["slots"] <= lc["max_slots"] == slots
    assert 0 < lc["epilogue"] <= lc["prologue"] < lc["slots"]
    b = Code(name).coop3_lc_banks()
    assert b["swizzled"] < 0.1 * b["plain"]


@pytest.mark.parametrize("name", ["576x288", "1944x972"])
def test_codes_without_coop3_have_no_plan(name):
    if name not in available():
        pytest.skip("code table absent")
    assert Code(name).coop3_line_cache() is None


def test_dvbs2_r1_2_swizzle_spreads_bank_groups():
    """The planner's per-residency XOR swizzle (a line's row i at piece i ^ z of
    its slot) puts the 4 pieces a 32-lane half of a pre read / post write
    touches in distinct bank groups: the modelled extra LDS cycles per
    iteration and workgroup drop from ~75k (every line unswizzled) to under 2 %
    of that, and the swizzled plan still replays (lc_check_plan checks every
    access at its swizzled position)."""
    b = Code("dvbs2_r1_2").coop3_lc_banks()
    assert b["plain"] > 50000
    assert b["swizzled"] < 0.02 * b["plain"]


def test_swizzle_off_reproduces_plain(monkeypatch):
    monkeypatch.setenv("LDPC_LC_SWIZZLE", "0")
    b = Code("dvbs2_r1_2").coop3_lc_banks()
    assert b["swizzled"] == b["plain"] > 0
