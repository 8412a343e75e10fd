"""GPU parity of the configs[4] path exactly as bench.py --mixed runs it, and of
the coop kernel (5) with its XCD block remap on.

bench.py --mixed decodes ONE 4096-codeword batch per GPU mixing DVB-S2 r1/2
and the DVB-S2-shaped r3/4, r5/6 (codeword c has rate c % 3: 1366 / 1365 /
1365 codewords), each rate at its own Eb/N0, 50 iterations at most, early
termination on.  The per-rate sub-batches run coop3 at grid 88 (r1/2 at
first-group degree 7, the shaped r3/4 at degree 14, the shaped r5/6 at degree
22) -- grid % 8 == 0, so the XCD-aware workgroup remap is ON; the tests here
check exactly those launches (and the coop kernel's, forced) against the oracle's
early-termination semantics: SURVEY.md §8(f) row 2's per-codeword stop on the
posterior hard-decision syndrome after every iteration (oracle/ldpc_oracle.c,
check_syndrome_ok).  That is the build's own definition, NOT the reference's
commented `arret` test (code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:255,
551-553: the extrinsic sign parity of every check during the iteration,
stopping the whole 16-frame call), so iterations-used parity is unpinned by
the reference; the per-check recurrence (:172-546) is pinned.  The
shaped codes have no reference build (their tables are not the reference's),
so the oracle -- pinned against the reference on every code it ships -- is the
checker.
"""
import os

import numpy as np
import pytest

import oracle as O
from ldpcgputegra_amd import Code, Decoder, channel, default_params, load_table

pytestmark = pytest.mark.gpu


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def _bench_mixed_inputs(torch, names, B, seed, ebn0):
    """The LLR batch bench_mixed() builds (bench.py): rate c % len(names) per
    codeword, each rate's all-zero codeword through its own device channel."""
    ids = np.arange(B, dtype=np.int32) % len(names)
    n = Code(names[0]).n
    llr = torch.empty((B, n), dtype=torch.int8, device="cuda")
    for c, name in enumerate(names):
        code = Code(name)
        sel = torch.from_numpy(np.where(ids == c)[0]).cuda()
        tmp = torch.empty((sel.numel(), n), dtype=torch.int8, device="cuda")
        gen = Decoder(code, max_batch=max(1, sel.numel()))
        table = channel.i8_table(channel.sigma_from_ebn0(ebn0[name], code.k_info / code.n), 8, 31)
        gen.awgn_i8_device(tmp, first_cw=c * B, seed=seed, table=table)
        llr[sel] = tmp
        gen.close()
    torch.cuda.synchronize()
    return ids, llr


def test_configs4_mixed_batch_as_benched_vs_oracle():
    """The whole configs[4] step of bench.py --mixed (MIXED_SETS["configs4"],
    MIXED_EBN0, batch 4096, 50 it, early termination, seed 2024): every
    codeword's hard decisions and iterations used equal the oracle's decode
    under its own code; every rate ran on coop3 (first-group degree 7, 14 and
    22: the r5/6 sub-batch on the 2-slab-wave kernel) with the XCD remap on
    (grid 88 for 1365 / 1366 codewords)."""
    torch = _torch()
    import bench
    from ldpcgputegra_amd.decoder import MixedDecoder
    names = bench.MIXED_SETS["configs4"]
    B, iters = 4096, 50
    ids, llr = _bench_mixed_inputs(torch, names, B, 2024, bench.MIXED_EBN0)
    mx = MixedDecoder([Code(n) for n in names], max_batch=B)
    hard = torch.empty((B, llr.shape[1]), dtype=torch.uint8, device="cuda")
    its = torch.empty(B, dtype=torch.int32, device="cuda")
    mx.decode_i8_device(llr, hard, ids, iters, params=default_params(early_term=1), iters_used=its)
    torch.cuda.synchronize()
    got_h, got_i, host = hard.cpu().numpy(), its.cpu().numpy(), llr.cpu().numpy()
    kernels = mx.last_kernels()
    assert kernels == ["coop3", "coop3", "coop3"], kernels
    thr = O.host_threads()
    for c, name in enumerate(names):
        sel = np.where(ids == c)[0]
        assert sel.size in (1365, 1366)
        eh, _, eit = O.decode_i8(load_table(name), host[sel], iters, early_term=True, return_soft=True, threads=thr)
        assert np.array_equal(got_i[sel], eit), (name, int((got_i[sel] != eit).sum()))
        bad = np.nonzero((got_h[sel] != eh).any(axis=1))[0]
        assert bad.size == 0, (name, bad[:16])
        assert eit.min() < iters                       # early termination is exercised
    mx.close()


@pytest.mark.parametrize("code", ["dvbs2shape_r3_4", "dvbs2shape_r5_6", "dvbs2_r2_3"])
@pytest.mark.parametrize("early", [False, True])
def test_coop_xcd_remap_vs_oracle(code, early):
    """kernel 5 (coop) at batch 128 (grid 8: remap on), fixed iterations and
    early termination: soft output, hard decisions and iterations used all
    equal the oracle's."""
    torch = _torch()
    t = load_table(code)
    B, iters = 128, 20
    ebn0 = {"dvbs2shape_r3_4": 2.8, "dvbs2shape_r5_6": 3.5, "dvbs2_r2_3": 2.2}[code]
    llr = channel.awgn_i8_host(t.n, B, seed=17, table=channel.i8_table(channel.sigma_from_ebn0(ebn0, t.k_info / t.n)))
    thr = O.host_threads()
    eh, es, eit = O.decode_i8(t, llr, iters, early_term=early, return_soft=True, threads=thr)
    if early:
        assert eit.min() < iters
    dec = Decoder(Code(code), max_batch=B, kernel=5)
    d_hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(B, dtype=torch.int32, device="cuda")
    dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters, params=default_params(early_term=int(early)),
                         soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_kernel == "coop"
    assert np.array_equal(d_its.cpu().numpy(), eit)
    assert np.array_equal(d_soft.cpu().numpy(), es)
    assert np.array_equal(d_hard.cpu().numpy(), eh)
    dec.close()


@pytest.mark.parametrize("kernel,env", [(5, {"LDPC_COOP_ET_KERNEL": "0"})])
def test_per_iteration_early_termination_padded_pitch(kernel, env):
    """The per-iteration early-termination launches (coop with
    LDPC_COOP_ET_KERNEL=0) address V by its padded row pitch (LDPC_VPITCH_PAD,
    default 64 codewords): results equal the oracle's (regression: they used to
    fail with LDPC_EDEVICE).  coop3 has only its in-kernel early termination."""
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    B, iters = 64, 30
    llr = channel.awgn_i8_host(t.n, B, seed=23, table=channel.i8_table(channel.sigma_from_ebn0(1.1, 0.5)))
    eh, es, eit = O.decode_i8(t, llr, iters, early_term=True, return_soft=True, threads=O.host_threads())
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        dec = Decoder(Code("dvbs2_r1_2"), max_batch=B, kernel=kernel)
        d_hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
        d_its = torch.empty(B, dtype=torch.int32, device="cuda")
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters, params=default_params(early_term=1),
                             soft=d_soft, iters_used=d_its)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    assert np.array_equal(d_its.cpu().numpy(), eit)
    assert np.array_equal(d_soft.cpu().numpy(), es)
    assert np.array_equal(d_hard.cpu().numpy(), eh)
    dec.close()


@pytest.mark.parametrize("factor,early", [(29, False), (24, True), (32, False)])
def test_coop3_nms_vs_oracle(factor, early):
    """NMS (CDecoder_NMS_fixed_SSE.cpp:188-240: cst = (min * factor) >> 5) on
    the fast DVB-S2 r1/2 kernel: coop3 runs it (no fallback reported) and its
    soft output, hard decisions and iterations used equal the oracle's."""
    from ldpcgputegra_amd import ALGO_NMS
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    B, iters = 200, 25
    llr = channel.awgn_i8_host(t.n, B, seed=factor, table=channel.i8_table(channel.sigma_from_ebn0(1.1, 0.5)))
    eh, es, eit = O.decode_i8(t, llr, iters, O.NMS, factor, early_term=early, return_soft=True,
                              threads=O.host_threads())
    dec = Decoder(Code("dvbs2_r1_2"), max_batch=B)
    d_hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(B, dtype=torch.int32, device="cuda")
    dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters,
                         params=default_params(algo=ALGO_NMS, factor=factor, early_term=int(early)),
                         soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_kernel == "coop3" and dec.last_skipped is None
    assert np.array_equal(d_its.cpu().numpy(), eit)
    assert np.array_equal(d_soft.cpu().numpy(), es)
    assert np.array_equal(d_hard.cpu().numpy(), eh)
    dec.close()


def _env(**kv):
    """Set environment variables (the C side reads them per call); returns the
    restore function."""
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})

    def restore():
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return restore


def _mixed_decode(torch, names, llr, ids, iters):
    from ldpcgputegra_amd.decoder import MixedDecoder
    B = llr.shape[0]
    mx = MixedDecoder([Code(n) for n in names], max_batch=B)
    hard = torch.empty((B, llr.shape[1]), dtype=torch.uint8, device="cuda")
    its = torch.empty(B, dtype=torch.int32, device="cuda")
    mx.decode_i8_device(llr, hard, ids, iters, params=default_params(early_term=1), iters_used=its)
    torch.cuda.synchronize()
    out = (hard.cpu().numpy(), its.cpu().numpy(), mx.last_kernels(), mx.last_et_stages())
    mx.close()
    del hard, its
    return out


def test_configs4_mixed_staged_vs_oracle():
    """The mixed decoder stages a rate's early termination by the same rule as
    a single-code decode (coop3 sub-batch >= LDPC_COOP3_ET_STAGE_MIN): with
    the threshold at 512 and bench.py --mixed's inputs at batch 1536, r1/2's
    512 codewords run staged (K = 20, then compactions every 5 iterations) and
    every codeword of every rate equals the oracle's per-codeword early
    termination (hard decisions and iterations used)."""
    torch = _torch()
    import bench
    names = bench.MIXED_SETS["configs4"]
    B, iters = 1536, 50
    ids, llr = _bench_mixed_inputs(torch, names, B, 2024, bench.MIXED_EBN0)
    restore = _env(LDPC_COOP3_ET_STAGE_MIN=512)
    try:
        got_h, got_i, kernels, stages = _mixed_decode(torch, names, llr, ids, iters)
    finally:
        restore()
    assert kernels == ["coop3", "coop3", "coop3"], kernels
    assert stages[0] == 20, stages
    host = llr.cpu().numpy()
    thr = O.host_threads()
    for c, name in enumerate(names):
        sel = np.where(ids == c)[0]
        eh, _, eit = O.decode_i8(load_table(name), host[sel], iters, early_term=True, return_soft=True, threads=thr)
        assert np.array_equal(got_i[sel], eit), (name, int((got_i[sel] != eit).sum()))
        assert np.array_equal(got_h[sel], eh), name
    assert got_i[ids == 0].max() > 20 and got_i[ids == 0].min() <= 20   # stages before and after K


def test_configs4_mixed_staged_batch_as_benched():
    """bench.py --mixed --batch 24576 (8192 codewords per rate): r1/2 runs
    staged by default, and the whole batch equals the same mixed decode with
    staging off (one in-kernel early-termination launch per rate, itself
    oracle-checked above) bit for bit -- hard decisions and iterations used;
    a seeded sample of 96 codewords per rate equals the oracle."""
    torch = _torch()
    import bench
    names = bench.MIXED_SETS["configs4"]
    B, iters = 24576, 50
    ids, llr = _bench_mixed_inputs(torch, names, B, 2024, bench.MIXED_EBN0)
    got_h, got_i, kernels, stages = _mixed_decode(torch, names, llr, ids, iters)
    assert kernels == ["coop3", "coop3", "coop3"], kernels
    assert stages[0] > 0, stages
    restore = _env(LDPC_COOP3_ET_STAGE_MIN=1 << 30)
    try:
        ref_h, ref_i, _, stages1 = _mixed_decode(torch, names, llr, ids, iters)
    finally:
        restore()
    assert stages1[0] == 0
    assert np.array_equal(got_i, ref_i), int((got_i != ref_i).sum())
    assert np.array_equal(got_h, ref_h)
    del ref_h
    host = llr.cpu().numpy()
    rng = np.random.default_rng(5)
    thr = O.host_threads()
    for c, name in enumerate(names):
        sel = np.sort(rng.choice(np.where(ids == c)[0], 96, replace=False))
        eh, _, eit = O.decode_i8(load_table(name), host[sel], iters, early_term=True, return_soft=True, threads=thr)
        assert np.array_equal(got_i[sel], eit), name
        assert np.array_equal(got_h[sel], eh), name
