"""GPU parity: the HIP decoder (through the C-ABI) against the reference's
golden vectors and the CPU oracle.

int8 paths: bit-exact hard decisions AND bit-exact final V (soft) vs the
oracle.  Float path: the north star allows 1e-6 LLR; the kernels use the same
exact IEEE ops (sub/add/min/max/abs, no FMA) as the oracle, so the test
tolerance is FLOAT_TOL = 1e-6 absolute and in practice the results are
bit-identical.
"""
import os

import numpy as np
import pytest
from conftest import golden_cases, golden_inputs

import oracle as O
from ldpcgputegra_amd import ALGO_MS, ALGO_NMS, ALGO_OMS, Code, Decoder, LdpcError, channel, default_params, load_table

pytestmark = pytest.mark.gpu
FLOAT_TOL = 1e-6
CASES = golden_cases()
_decoders = {}


def decoder(code, kernel=0, max_batch=4096):
    key = (code, kernel, max_batch)
    if key not in _decoders:
        _decoders[key] = Decoder(Code(code), max_batch=max_batch, kernel=kernel)
    return _decoders[key]


def kernels_for(code):
    """Kernel families that can run this code: 1 generic, 2 windowed,
    3 windowed2 (S=16), 5 coop (workgroup-cooperative), 7 lds (LDS-resident
    short codes), 8 coop3 (slab waves doing pre + post, i16 chain; first-group
    degree 7 or 10).  (4 = windowed2 S=32 and 6 = coop2 were superseded and removed.)"""
    ks = [1]
    c = Code(code)
    if c.plan_info()["windowed"]:
        ks.append(2)
    if c.window_plan(16, 2):
        ks.append(3)
    if c.coop_plan() is not None and c.max_deg in (7, 10, 14, 22):
        ks.append(5)
    if c.coop3_line_cache() is not None:
        ks.append(8)
    if c.layer_info()["lds_i8"]:
        ks.append(7)
    return ks


def params_of(case):
    algo = ALGO_NMS if case["algo"] == 1 else ALGO_OMS
    return default_params(algo=algo, offset=case["param"], factor=case["param"], var_min=case["var_min"],
                          msg_max=case["msg_max"], msg_min=-case["msg_max"])


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gpu_matches_reference_golden(case):
    llr, expected = golden_inputs(case)
    for k in kernels_for(case["code"]):
        dec = decoder(case["code"], k, max_batch=64)
        try:
            got = dec.decode_i8(llr, case["iters"], params_of(case))
        except Exception as e:   # windowed kernel may not support exotic params
            if k >= 2 and "not applicable" in str(e):
                continue
            raise
        assert np.array_equal(got, expected), "kernel %d: %d bits differ" % (k, int((got != expected).sum()))


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


@pytest.mark.parametrize("code", ["576x288", "648x324", "1944x972", "2048x384", "1024x518", "1200x600", "200x100",
                                  "dvbs2_r1_2", "dvbs2_r2_3", "dvbs2_r9_10", "16200x7560", "dvbs2shape_r3_4",
                                  "dvbs2shape_r5_6"])
@pytest.mark.parametrize("batch", [1, 37, 64])
def test_soft_output_bit_exact_vs_oracle(code, batch):
    torch = _torch()
    t = load_table(code)
    iters = 6 if t.n > 10000 else 15
    sigma = channel.sigma_from_ebn0(1.5, t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, batch, seed=batch, table=channel.i8_table(sigma))
    ref_hard, ref_soft, _ = O.decode_i8(t, llr, iters, O.OMS, 1, return_soft=True)
    for k in kernels_for(code):
        dec = decoder(code, k, max_batch=64)
        d_llr = torch.from_numpy(llr).cuda()
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
        dec.decode_i8_device(d_llr, d_hard, iters, soft=d_soft)
        torch.cuda.synchronize()
        assert np.array_equal(d_soft.cpu().numpy(), ref_soft), "kernel %d" % k
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard), "kernel %d" % k


@pytest.mark.parametrize("code", ["576x288", "1944x972", "200x100", "dvbs2_r1_2", "dvbs2shape_r3_4"])
@pytest.mark.parametrize("batch,ld", [(1, 1), (37, 50), (64, 64), (48, 128)])
def test_node_major_input_vs_oracle(code, batch, ld):
    """ldpc_decode_i8_nm_async: node-major input [N][ld] (the reference's
    interleaved layout, CGPU_Decoder_MS_SIMD_v2.cu:120-251) gives the oracle's
    hard and soft outputs bit-exactly on every kernel family; ld 50 exercises
    the unaligned byte path, 64/128 the 16-byte path, 48 < 128 a ragged tail."""
    torch = _torch()
    t = load_table(code)
    iters = 6 if t.n > 10000 else 15
    sigma = channel.sigma_from_ebn0(1.5, t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, batch, seed=7 + batch, table=channel.i8_table(sigma))
    ref_hard, ref_soft, _ = O.decode_i8(t, llr, iters, O.OMS, 1, return_soft=True)
    nm = np.full((t.n, ld), 77, dtype=np.int8)   # junk beyond `batch` must be ignored
    nm[:, :batch] = llr.T
    for k in kernels_for(code):
        dec = decoder(code, k, max_batch=64)
        d_nm = torch.from_numpy(nm).cuda()
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
        dec.decode_i8_nm_device(d_nm, d_hard, iters, batch=batch, soft=d_soft)
        torch.cuda.synchronize()
        assert np.array_equal(d_soft.cpu().numpy(), ref_soft), "kernel %d" % k
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard), "kernel %d" % k


@pytest.mark.parametrize("kernel", [5, 8])
def test_node_major_input_xcd_remap_early_termination(kernel):
    """The node-major path at a batch that turns the XCD-aware
    workgroup remap on (200 codewords: stride 256, grid 16, grid % 8 == 0)
    with a pitch ld = 300 > batch and a ragged last group, early termination
    and iterations used: soft output, hard decisions and iterations equal the
    oracle's on coop (5) and coop3 (8)."""
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    batch, ld, iters = 200, 300, 25
    llr = channel.awgn_i8_host(t.n, batch, seed=31, table=channel.i8_table(channel.sigma_from_ebn0(1.1, 0.5)))
    ref_hard, ref_soft, ref_its = O.decode_i8(t, llr, iters, O.OMS, 1, early_term=True, return_soft=True,
                                              threads=O.host_threads())
    assert ref_its.min() < iters
    nm = np.full((t.n, ld), -5, dtype=np.int8)
    nm[:, :batch] = llr.T
    dec = decoder("dvbs2_r1_2", kernel, max_batch=256)
    d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
    dec.decode_i8_nm_device(torch.from_numpy(nm).cuda(), d_hard, iters, batch=batch,
                            params=default_params(early_term=1), soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_kernel == {5: "coop", 8: "coop3"}[kernel]
    assert np.array_equal(d_its.cpu().numpy(), ref_its)
    assert np.array_equal(d_soft.cpu().numpy(), ref_soft)
    assert np.array_equal(d_hard.cpu().numpy(), ref_hard)


def test_config1_single_codeword_float_sweep():
    """BASELINE.json configs[0] shape on the GPU path: 802.11n N=648 r1/2, one
    codeword, 10 iterations, float min-sum, Eb/N0 0.5 .. 3.0 dB (SURVEY.md
    8(d) "Config 1"), every point equal to the oracle's float decode."""
    torch = _torch()
    t = load_table("648x324")
    rng = np.random.default_rng(21)
    for ebn0 in (0.5, 1.0, 1.5, 2.0, 2.5, 3.0):
        sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
        llr = (-1.0 + sigma * rng.standard_normal((1, t.n))).astype(np.float32)
        ref_hard, ref_soft, _ = O.decode_f32(t, llr, 10, O.OMS, 0.0)
        for k in (0, 1, 7, 9):
            dec = decoder("648x324", k, 64)
            d_hard = torch.empty((1, t.n), dtype=torch.uint8, device="cuda")
            d_soft = torch.empty((1, t.n), dtype=torch.float32, device="cuda")
            dec.decode_f32_device(torch.from_numpy(llr).cuda(), d_hard, 10, params=default_params(algo=ALGO_MS),
                                  soft=d_soft)
            torch.cuda.synchronize()
            assert np.max(np.abs(d_soft.cpu().numpy() - ref_soft)) <= FLOAT_TOL, (ebn0, k)
            assert np.array_equal(d_hard.cpu().numpy(), ref_hard), (ebn0, k)


@pytest.mark.parametrize("code,batch,is_float", [("816x408", 4096, False), ("648x324", 4096, True),
                                                 ("648x324", 3000, False), ("200x100", 9000, True)])
def test_lds_kernel_large_batches(code, batch, is_float):
    """Kernel 7 packs several codewords per wave at large batches (with and
    without two lanes per check): bit-exact soft output vs the oracle."""
    torch = _torch()
    t = load_table(code)
    iters = 8
    dec = decoder(code, 7, batch)
    if is_float:
        rng = np.random.default_rng(11)
        sigma = channel.sigma_from_ebn0(1.5, t.k_info / t.n)
        llr = (-1.0 + sigma * rng.standard_normal((batch, t.n))).astype(np.float32)
        _, ref_soft, _ = O.decode_f32(t, llr, iters, O.OMS, 0.0)
        d_soft = torch.empty((batch, t.n), dtype=torch.float32, device="cuda")
        dec.decode_f32_device(torch.from_numpy(llr).cuda(), None, iters, params=default_params(algo=ALGO_MS),
                              soft=d_soft)
    else:
        llr = channel.awgn_i8_host(t.n, batch, seed=9, table=channel.i8_table(0.8))
        _, ref_soft, _ = O.decode_i8(t, llr, iters, O.OMS, 1, return_soft=True)
        d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), None, iters, soft=d_soft)
    torch.cuda.synchronize()
    assert dec.last_kernel == "lds"
    assert np.array_equal(d_soft.cpu().numpy(), ref_soft)


@pytest.mark.parametrize("algo,param", [(ALGO_OMS, 0), (ALGO_OMS, 3), (ALGO_NMS, 24), (ALGO_MS, 0)])
def test_algorithms_vs_oracle(algo, param):
    t = load_table("1944x972")
    llr = channel.awgn_i8_host(t.n, 40, seed=7, table=channel.i8_table(0.75))
    o_algo = O.NMS if algo == ALGO_NMS else O.OMS
    o_param = param if algo != ALGO_MS else 0
    exp = O.decode_i8(t, llr, 12, o_algo, o_param)
    p = default_params(algo=algo, offset=param, factor=param)
    for k in (1, 7):
        got = decoder("1944x972", k, 64).decode_i8(llr, 12, p)
        assert np.array_equal(got, exp), "kernel %d" % k


ET_EBN0 = {"dvbs2_r1_2": 1.0, "dvbs2shape_r3_4": 2.8, "dvbs2shape_r5_6": 3.5}


@pytest.mark.parametrize("code", ["576x288", "648x324", "dvbs2_r1_2", "dvbs2shape_r3_4", "dvbs2shape_r5_6"])
def test_early_termination_vs_oracle(code):
    torch = _torch()
    t = load_table(code)
    batch = 24
    sigma = channel.sigma_from_ebn0(ET_EBN0.get(code, 2.0), t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, batch, seed=3, table=channel.i8_table(sigma))
    ref_hard, ref_soft, ref_its = O.decode_i8(t, llr, 30, O.OMS, 1, early_term=True, return_soft=True)
    assert ref_its.min() < 30                                # some codewords stop early
    for k in kernels_for(code):
        dec = decoder(code, k, max_batch=64)
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
        d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, 30, params=default_params(early_term=1),
                             soft=d_soft, iters_used=d_its)
        torch.cuda.synchronize()
        assert np.array_equal(d_its.cpu().numpy(), ref_its), "kernel %d" % k
        assert np.array_equal(d_soft.cpu().numpy(), ref_soft), "kernel %d" % k


@pytest.mark.parametrize("q,nms,step,ebn0", [(20, False, 10, 1.0), (40, False, 2, 1.0), (30, True, 3, 1.6)])
def test_coop3_staged_early_termination_vs_oracle(monkeypatch, q, nms, step, ebn0):
    """Staged early termination (launch_coop3: K iterations on the whole
    batch, then every `step` iterations the codewords still decoding
    compacted into dense groups of the other of two state buffers and
    decoded on from there, each stage's codewords moved back), forced at a
    small batch (LDPC_COOP3_ET_STAGE_MIN=0): hard and soft outputs and
    iterations equal the oracle's per-codeword early termination."""
    torch = _torch()
    code, batch, iters = "dvbs2_r1_2", 200, 30
    t = load_table(code)
    sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, batch, seed=17, table=channel.i8_table(sigma))
    algo, param = (O.NMS, 26) if nms else (O.OMS, 1)
    ref_hard, ref_soft, ref_its = O.decode_i8(t, llr, iters, algo, param, early_term=True, return_soft=True)
    k1 = int(np.percentile(ref_its, q))   # the first stage: some codewords converge in it, some after it
    assert 0 < k1 < iters and (ref_its > k1).any() and (ref_its <= k1).any()
    monkeypatch.setenv("LDPC_COOP3_ET_STAGE_MIN", "0")
    monkeypatch.setenv("LDPC_COOP3_ET_K", str(k1))
    monkeypatch.setenv("LDPC_COOP3_ET_STEP", str(step))   # step 2 / 3: several compactions
    dec = decoder(code, 8, max_batch=256)
    d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
    p = default_params(early_term=1, algo=ALGO_NMS, factor=param) if nms else default_params(early_term=1)
    dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters, params=p, soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert np.array_equal(d_its.cpu().numpy(), ref_its)
    assert np.array_equal(d_soft.cpu().numpy(), ref_soft)
    assert np.array_equal(d_hard.cpu().numpy(), ref_hard)


def test_coop3_staged_early_termination_past_64_stages(monkeypatch):
    """More iterations than 64 stages hold (K = 2, one iteration per stage,
    90 iterations: K + 64 < 90): the 64th stage takes every iteration left,
    so codewords still decoding are decoded up to the last iteration and
    record it (regression: the stage loop used to stop at 64 stages, leaving
    them under-decoded with iters_used = -1).  Eb/N0 0.9 dB: a quarter of the codewords
    never converge, one converges only after the 64th stage began."""
    torch = _torch()
    code, batch, iters = "dvbs2_r1_2", 48, 90
    t = load_table(code)
    llr = channel.awgn_i8_host(t.n, batch, seed=29, table=channel.i8_table(channel.sigma_from_ebn0(0.9, 0.5)))
    ref_hard, ref_soft, ref_its = O.decode_i8(t, llr, iters, early_term=True, return_soft=True,
                                              threads=O.host_threads())
    assert (ref_its == iters).any() and (ref_its < iters).any()
    monkeypatch.setenv("LDPC_COOP3_ET_STAGE_MIN", "0")
    monkeypatch.setenv("LDPC_COOP3_ET_K", "2")
    monkeypatch.setenv("LDPC_COOP3_ET_STEP", "1")
    dec = decoder(code, 8, max_batch=64)
    d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
    dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters, params=default_params(early_term=1),
                         soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_et_stage == 2
    assert np.array_equal(d_its.cpu().numpy(), ref_its)
    assert np.array_equal(d_soft.cpu().numpy(), ref_soft)
    assert np.array_equal(d_hard.cpu().numpy(), ref_hard)


def has_kernel(code, k):
    try:
        decoder(code, k, 64)
        return True
    except LdpcError:
        return False


@pytest.mark.parametrize("code,algo,beta,batch", [("1944x972", ALGO_MS, 0.0, 33), ("576x288", ALGO_OMS, 0.15, 33),
                                                  ("576x288", ALGO_NMS, 0.75, 33), ("dvbs2_r1_2", ALGO_MS, 0.0, 33),
                                                  ("648x324", ALGO_MS, 0.0, 1024), ("648x324", ALGO_OMS, 0.15, 37),
                                                  ("648x324", ALGO_NMS, 0.75, 37), ("576x288", ALGO_MS, 0.0, 1030)])
def test_float_decoder_vs_oracle(code, algo, beta, batch):
    """648x324 at batch 1024 / 20 it / float min-sum is BASELINE.json configs[1]."""
    torch = _torch()
    t = load_table(code)
    rng = np.random.default_rng(5)
    sigma = channel.sigma_from_ebn0(1.2, t.k_info / t.n)
    llr = (-1.0 + sigma * rng.standard_normal((batch, t.n))).astype(np.float32)
    iters = 5 if t.n > 10000 else 20
    o_algo = O.NMS if algo == ALGO_NMS else O.OMS
    ref_hard, ref_soft, _ = O.decode_f32(t, llr, iters, o_algo, beta)
    ks = [1] + ([7] if Code(code).layer_info()["lds_f32"] else []) + ([9] if has_kernel(code, 9) else [])
    if code in ("648x324", "576x288"):
        assert 9 in ks                                       # the edge-parallel kernel covers both shapes
    for k in ks:
        dec = decoder(code, k, max(64, batch))
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.float32, device="cuda")
        dec.decode_f32_device(torch.from_numpy(llr).cuda(), d_hard, iters,
                              params=default_params(algo=algo, beta=beta), soft=d_soft)
        torch.cuda.synchronize()
        soft = d_soft.cpu().numpy()
        assert np.max(np.abs(soft - ref_soft)) <= FLOAT_TOL, "kernel %d" % k
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard), "kernel %d" % k


@pytest.mark.parametrize("code,algo,beta,batch,iters", [
    ("dvbs2_r1_2", ALGO_MS, 0.0, 40, 6), ("dvbs2_r1_2", ALGO_OMS, 0.15, 17, 3), ("dvbs2_r1_2", ALGO_NMS, 0.75, 64, 4),
    ("dvbs2_r2_3", ALGO_MS, 0.0, 33, 3), ("dvbs2shape_r3_4", ALGO_NMS, 0.75, 20, 3),
    ("dvbs2shape_r5_6", ALGO_MS, 0.0, 20, 3), ("dvbs2_r8_9", ALGO_OMS, 0.15, 20, 3), ("dvbs2_r9_10", ALGO_MS, 0.0, 80, 2),
    ("dvbs2_r1_2", ALGO_MS, 0.0, 3, 1)])
def test_stairf_vs_oracle(code, algo, beta, batch, iters, monkeypatch):
    """Float staircase kernel (11, stairf.hip): the float default for the
    DVB-S2 codes (no early termination) against the oracle's serial float
    decode (oracle/ldpc_oracle.c), every DVB-S2 check degree it is built for,
    every group width (LDPC_STAIRF_S 2 / 4 / 8 / 16: 32 / 16 / 8 / 4 codewords per wave;
    a code whose check count 16 does not divide runs its fallback width);
    iteration counts that are not multiples of its prefetch block; batches that
    leave part of a wave empty; bit-identical soft output."""
    torch = _torch()
    t = load_table(code)
    rng = np.random.default_rng(21)
    sigma = channel.sigma_from_ebn0(1.0, t.k_info / t.n)
    llr = (-1.0 + sigma * rng.standard_normal((batch, t.n))).astype(np.float32)
    o_algo = O.NMS if algo == ALGO_NMS else O.OMS
    ref_hard, ref_soft, _ = O.decode_f32(t, llr, iters, o_algo, beta)
    for k, width in ((0, None), (11, 2), (11, 4), (11, 8), (11, 16)):
        if width:
            monkeypatch.setenv("LDPC_STAIRF_S", str(width))
        dec = decoder(code, k, max(64, batch))
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.float32, device="cuda")
        dec.decode_f32_device(torch.from_numpy(llr).cuda(), d_hard, iters,
                              params=default_params(algo=algo, beta=beta), soft=d_soft)
        torch.cuda.synchronize()
        assert dec.last_kernel == "stairf"
        soft = d_soft.cpu().numpy()
        assert np.array_equal(soft.view(np.uint32), ref_soft.view(np.uint32)), \
            "kernel %d width %s: %d values differ" % (k, width, int((soft != ref_soft).sum()))
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard)


@pytest.mark.parametrize("code,algo,beta,ebn0,iters", [("dvbs2_r1_2", ALGO_MS, 0.0, 2.0, 9),
                                                       ("dvbs2_r1_2", ALGO_NMS, 0.75, 2.0, 12),
                                                       ("dvbs2_r2_3", ALGO_OMS, 0.15, 2.6, 12)])
def test_stairf_early_termination_vs_oracle(code, algo, beta, ebn0, iters, monkeypatch):
    """Float staircase kernel with early termination (one launch per
    iteration, then a syndrome pass over the live codewords): iterations used,
    soft output and hard decisions equal the oracle's per-codeword stop
    (oracle/ldpc_oracle.c: syndrome after every iteration), at every group
    width; some codewords stop early, some run to the limit."""
    torch = _torch()
    t = load_table(code)
    batch = 70
    rng = np.random.default_rng(23)
    llr = (-1.0 + channel.sigma_from_ebn0(ebn0, t.k_info / t.n) * rng.standard_normal((batch, t.n))).astype(np.float32)
    o_algo = O.NMS if algo == ALGO_NMS else O.OMS
    ref_hard, ref_soft, ref_its = O.decode_f32(t, llr, iters, o_algo, beta, early_term=True, threads=O.host_threads())
    assert ref_its.min() < iters
    for k, width in ((0, None), (11, 2), (11, 4), (11, 8), (11, 16)):
        if width:
            monkeypatch.setenv("LDPC_STAIRF_S", str(width))
        dec = decoder(code, k, 128)
        d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((batch, t.n), dtype=torch.float32, device="cuda")
        d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
        dec.decode_f32_device(torch.from_numpy(llr).cuda(), d_hard, iters,
                              params=default_params(algo=algo, beta=beta, early_term=1), soft=d_soft, iters_used=d_its)
        torch.cuda.synchronize()
        assert dec.last_kernel == "stairf"
        assert np.array_equal(d_its.cpu().numpy(), ref_its), "width %s" % width
        soft = d_soft.cpu().numpy()
        assert np.array_equal(soft.view(np.uint32), ref_soft.view(np.uint32)), "width %s" % width
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard), "width %s" % width


@pytest.mark.parametrize("code,batch", [("648x324", 1024), ("576x288", 37)])
def test_ldsep_auto_early_termination_vs_oracle(code, batch):
    """The float default for the short QC codes is the edge-parallel kernel
    (9, ldsep.hip): with early termination its hard decisions, soft output and
    iterations used equal the oracle's (syndrome after every iteration,
    oracle/ldpc_oracle.c check_syndrome_ok_f)."""
    torch = _torch()
    t = load_table(code)
    rng = np.random.default_rng(8)
    llr = (-1.0 + channel.sigma_from_ebn0(2.0, 0.5) * rng.standard_normal((batch, t.n))).astype(np.float32)
    ref_hard, ref_soft, ref_its = O.decode_f32(t, llr, 20, O.OMS, 0.0, early_term=True)
    assert ref_its.min() < 20
    dec = decoder(code, 0, batch)
    d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((batch, t.n), dtype=torch.float32, device="cuda")
    d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
    dec.decode_f32_device(torch.from_numpy(llr).cuda(), d_hard, 20, params=default_params(algo=ALGO_MS, early_term=1),
                          soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_kernel == "ldsep"
    assert np.array_equal(d_its.cpu().numpy(), ref_its)
    assert np.max(np.abs(d_soft.cpu().numpy() - ref_soft)) <= FLOAT_TOL
    assert np.array_equal(d_hard.cpu().numpy(), ref_hard)


def test_device_channel_matches_host_generator():
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    dec = decoder("dvbs2_r1_2", 0, 64)
    # BPSK, and QPSK with the 2/sigma^2 normalisation (CChanelAWGN_MKL options)
    for table in (channel.i8_table(0.87), channel.i8_table(0.87, 8, 31, amp=channel.QPSK, normalize=True)):
        d = torch.empty((7, t.n), dtype=torch.int8, device="cuda")
        dec.awgn_i8_device(d, first_cw=123, seed=42, table=table)
        torch.cuda.synchronize()
        assert np.array_equal(d.cpu().numpy(), channel.awgn_i8_host(t.n, 7, 42, table, first_cw=123))


def test_error_counter():
    torch = _torch()
    dec = decoder("576x288", 1, 64)
    hard = np.zeros((5, 576), np.uint8)
    hard[1, 3] = 1
    hard[1, 100] = 1
    hard[3, 287] = 1
    hard[4, 300] = 1            # beyond k = 288: not counted (CErrorAnalyzer counts N-M bits)
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    dec.count_errors_device(torch.from_numpy(hard).cuda(), 288, counts)
    torch.cuda.synchronize()
    assert counts.cpu().tolist() == [3, 2]
    # against a reference codeword, dword path (n, k multiples of 4) and byte path
    rng = np.random.default_rng(4)
    for code, n, k in (("576x288", 576, 288), ("9972x4986", 9972, 4986)):   # k % 4 == 2: byte path
        dec = decoder(code, 1, 64)                 # the row length is the context's code length
        ref = rng.integers(0, 2, (6, n), dtype=np.uint8)
        hard = ref.copy()
        hard[0, :k] ^= 1                       # k errors
        hard[2, k - 1] ^= 1
        hard[5, k:] ^= 1                       # beyond k: not counted
        counts.zero_()
        dec.count_errors_device(torch.from_numpy(hard).cuda(), k, counts, ref=torch.from_numpy(ref).cuda())
        torch.cuda.synchronize()
        assert counts.cpu().tolist() == [k + 1, 2]


def test_dvbs2_full_batch_vs_reference():
    """BASELINE configs[2] (DVB-S2 r1/2, 4096 codewords, 50 it) in full: every
    hard decision of the default kernel equals the reference's own SSE
    decoder (oracle/_ref, code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:114-574,
    all host threads); the soft output of a 256-codeword slice (16 whole
    workgroups, spread over the batch) equals the oracle's; plus shard
    invariance on a ragged split and convergence past the waterfall."""
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    B = 4096
    dec = decoder("dvbs2_r1_2", 0, B)
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, 0.5))
    llr = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    dec.awgn_i8_device(llr, 0, 77, table)
    h1 = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    s1 = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    h2 = torch.empty_like(h1)
    dec.decode_i8_device(llr, h1, 50, soft=s1)
    assert dec.last_kernel == "coop3"
    dec.decode_i8_device(llr[:1000], h2[:1000], 50)           # ragged shard
    dec.decode_i8_device(llr[1000:], h2[1000:], 50)
    torch.cuda.synchronize()
    assert torch.equal(h1, h2)
    host_llr = llr.cpu().numpy()
    got = h1.cpu().numpy()
    thr = O.host_threads()
    if O.ref_available("dvbs2_r1_2"):
        exp = O.ref_decode_mt("dvbs2_r1_2", host_llr, 50, 1, thr)
    else:
        exp = O.decode_i8(t, host_llr, 50, threads=thr)
    diff = np.nonzero((got != exp).any(axis=1))[0]
    assert diff.size == 0, "codewords differing from the reference: %s" % diff[:16]
    fe = int((got[:, :t.k_info].sum(axis=1) > 0).sum())
    assert 0 < fe < 100, fe                                   # 1.0 dB: in the waterfall, mostly converged
    sel = np.concatenate([np.arange(16 * g * 16, 16 * g * 16 + 16) for g in range(16)])
    _, ref_soft, _ = O.decode_i8(t, host_llr[sel], 50, return_soft=True, threads=thr)
    assert np.array_equal(s1.cpu().numpy()[sel], ref_soft)


@pytest.mark.parametrize("kernel", [5, 8])
@pytest.mark.parametrize("batch,ebn0", [(40, 1.1), (64, 1.1), (1024, 1.0)])
def test_coop2_early_termination_vs_oracle(batch, ebn0, kernel):
    """coop (5) and coop3 (8), both with in-kernel early termination, on whole and
    partial workgroups and, at batch 1024 (grid 64), with the XCD block remap
    on, as bench.py --mixed runs it: hard decisions, soft output and iterations
    used all equal the oracle's (syndrome after every iteration)."""
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    dec = decoder("dvbs2_r1_2", kernel, max(64, batch))
    sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, batch, seed=batch + 5, table=channel.i8_table(sigma))
    thr = O.host_threads()
    ref_hard, ref_soft, ref_its = O.decode_i8(t, llr, 50, early_term=True, return_soft=True, threads=thr)
    assert ref_its.min() < 50
    d_hard = torch.empty((batch, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(batch, dtype=torch.int32, device="cuda")
    for rep in range(2):                      # the second run reuses the context's live / snapshot buffers
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, 50, params=default_params(early_term=1),
                             soft=d_soft, iters_used=d_its)
        torch.cuda.synchronize()
        assert dec.last_kernel == {5: "coop", 8: "coop3"}[kernel]
        assert np.array_equal(d_its.cpu().numpy(), ref_its), rep
        assert np.array_equal(d_soft.cpu().numpy(), ref_soft), rep
        assert np.array_equal(d_hard.cpu().numpy(), ref_hard), rep


def test_mixed_rate_batch_with_early_termination():
    """BASELINE config 5 shape: one batch mixing DVB-S2 rates 1/2, 2/3, 8/9,
    9/10 (3/4 and 5/6 tables are absent from the reference), random
    codewords, early termination.  Every codeword must equal the oracle's
    decode under its own code (hard decisions and iterations used)."""
    torch = _torch()
    from ldpcgputegra_amd.decoder import MixedDecoder
    names = ["dvbs2_r1_2", "dvbs2_r2_3", "dvbs2_r8_9", "dvbs2_r9_10"]
    ebn0 = {"dvbs2_r1_2": 1.0, "dvbs2_r2_3": 2.2, "dvbs2_r8_9": 4.0, "dvbs2_r9_10": 4.4}
    mx = MixedDecoder(names, max_batch=64)
    B = 24
    ids = np.array([i % 4 for i in range(B)], np.int32)
    np.random.default_rng(4).shuffle(ids)
    llr = np.empty((B, 64800), np.int8)
    for c, name in enumerate(names):
        code = Code(name)
        sel = np.where(ids == c)[0]
        info = np.random.default_rng(c).integers(0, 2, size=(sel.size, code.k_info), dtype=np.uint8)
        cw = code.encode(info)
        table = channel.i8_table(channel.sigma_from_ebn0(ebn0[name], code.k_info / code.n))
        llr[sel] = channel.awgn_i8_host(code.n, sel.size, seed=31 + c, table=table, codeword=cw)
    d_hard = torch.empty((B, 64800), dtype=torch.uint8, device="cuda")
    d_its = torch.empty(B, dtype=torch.int32, device="cuda")
    mx.profile(True)   # per-code decode-kernel timing (ldpc_mixed_kernel_time)
    mx.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, ids, 20, params=default_params(early_term=1),
                        iters_used=d_its)
    torch.cuda.synchronize()
    kt = mx.kernel_time(reset=True)
    assert [n for _, n in kt] == [1, 1, 1, 1] and all(ms > 0 for ms, _ in kt), kt
    assert [n for _, n in mx.kernel_time()] == [0, 0, 0, 0]   # reset
    mx.profile(False)
    hard, its = d_hard.cpu().numpy(), d_its.cpu().numpy()
    for c, name in enumerate(names):
        sel = np.where(ids == c)[0]
        eh, _, eit = O.decode_i8(load_table(name), llr[sel], 20, early_term=True, return_soft=True)
        assert np.array_equal(hard[sel], eh), name
        assert np.array_equal(its[sel], eit), name


def test_device_calls_ordered_with_torch_default_stream():
    """Device-pointer calls made while torch is on its default stream are
    fenced against it: a torch op issued right after the generator / decoder
    sees their complete output (regression: the NULL stream used to mean the
    context's own non-blocking stream, unordered with torch's work, which
    corrupted bench.py --mixed's per-rate inputs)."""
    torch = _torch()
    from ldpcgputegra_amd.decoder import MixedDecoder
    names = ("dvbs2_r1_2", "dvbs2_r8_9")
    codes = [Code(n) for n in names]
    n, per = codes[0].n, 64
    ids = np.arange(2 * per, dtype=np.int32) % 2
    llr = torch.zeros((2 * per, n), dtype=torch.int8, device="cuda")
    host = np.empty((2 * per, n), dtype=np.int8)
    for c, code in enumerate(codes):
        sel = np.where(ids == c)[0]
        table = channel.i8_table(channel.sigma_from_ebn0(1.0 + 3 * c, code.k_info / n), 8, 31)
        gen = Decoder(code, max_batch=per)
        for rep in range(3):   # reused allocator blocks: a stale tmp would show
            tmp = torch.empty((per, n), dtype=torch.int8, device="cuda")
            gen.awgn_i8_device(tmp, first_cw=c * 1000, seed=11, table=table)
            llr[torch.from_numpy(sel).cuda()] = tmp
        gen.close()
        host[sel] = channel.awgn_i8_host(n, per, 11, table, first_cw=c * 1000)
    assert np.array_equal(llr.cpu().numpy(), host)
    mx = MixedDecoder(codes, max_batch=2 * per)
    hard = torch.empty((2 * per, n), dtype=torch.uint8, device="cuda")
    its = torch.empty(2 * per, dtype=torch.int32, device="cuda")
    p = default_params(early_term=1)
    mx.decode_i8_device(llr, hard, ids, 20, params=p, iters_used=its)
    got_h, got_i = hard.cpu().numpy(), its.cpu().numpy()   # no explicit synchronize
    for c, code in enumerate(codes):
        sel = np.where(ids == c)[0]
        dec = Decoder(code, max_batch=per)
        x = llr[torch.from_numpy(sel).cuda()].contiguous()
        h2 = torch.empty((per, n), dtype=torch.uint8, device="cuda")
        i2 = torch.empty(per, dtype=torch.int32, device="cuda")
        dec.decode_i8_device(x, h2, 20, params=p, iters_used=i2)
        assert np.array_equal(h2.cpu().numpy(), got_h[sel])
        assert np.array_equal(i2.cpu().numpy(), got_i[sel])
        dec.close()
    mx.close()


@pytest.mark.gpu
def test_quantize_f32_i8_vs_oracle():
    """ldpc_quantize_f32_i8[_async] vs CFastFixConversion::generate's rule
    (code/x86/CFixPointConversion/CFastFixConversion.cpp:55-65, restated as
    oracle_quantize): truncation toward zero at +-0.124 / 0.126 (x 8), the
    saturation limits, other factors / limits, and a large random vector."""
    torch = _torch()
    dec = Decoder(Code("576x288"), max_batch=8)
    edge = np.array([-5.0, -3.9, -0.124, -0.126, 0.0, -0.0, 0.124, 0.126, 0.9999, 3.874, 3.876, 100.0,
                     1e30, -1e30], np.float32)
    assert dec.quantize(edge).tolist() == O.quantize(edge).tolist()
    rng = np.random.default_rng(5)
    y = (rng.standard_normal(1 << 20) * 6).astype(np.float32)
    for factor, lo, hi in ((8, -31, 31), (4, -127, 127), (16, -128, 127), (1, -7, 9)):
        ref = O.quantize(y, factor, lo, hi)
        assert np.array_equal(dec.quantize(y, factor, lo, hi), ref), (factor, lo, hi)
        yd = torch.from_numpy(y).cuda()
        qd = torch.empty(y.shape, dtype=torch.int8, device="cuda")
        dec.quantize_device(yd, qd, factor, lo, hi)
        assert np.array_equal(qd.cpu().numpy(), ref), (factor, lo, hi)


def test_dvbs2_large_batch_vs_reference():
    """A batch of 16464 codewords (1029 workgroups: four per CU and a ragged
    last one): coop3 has no batch cap -- every hard decision equals the
    reference SSE decoder's (10 iterations)."""
    torch = _torch()
    t = load_table("dvbs2_r1_2")
    B = 16384 + 80
    dec = decoder("dvbs2_r1_2", 0, B)
    table = channel.i8_table(channel.sigma_from_ebn0(1.2, 0.5))
    llr = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    dec.awgn_i8_device(llr, 5, 91, table)
    hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    dec.decode_i8_device(llr, hard, 10)
    assert dec.last_kernel == "coop3" and dec.last_skipped is None
    got = hard.cpu().numpy()
    host_llr = llr.cpu().numpy()
    thr = O.host_threads()
    if O.ref_available("dvbs2_r1_2"):
        exp = O.ref_decode_mt("dvbs2_r1_2", host_llr, 10, 1, thr)
    else:
        exp = O.decode_i8(t, host_llr, 10, threads=thr)
    diff = np.nonzero((got != exp).any(axis=1))[0]
    assert diff.size == 0, "codewords differing from the reference: %s" % diff[:16]


def test_fast_kernel_fallback_is_reported():
    """Parameters the fast DVB-S2 kernels do not take (msg_max > 63) fall back
    to a general kernel -- bit-exact with the oracle -- and the context reports
    the skipped kernel (ldpc_ctx_last_skipped = coop3 for r1/2 and r2/3)."""
    t = load_table("dvbs2_r1_2")
    llr = channel.awgn_i8_host(t.n, 16, seed=4, table=channel.i8_table(channel.sigma_from_ebn0(1.0, 0.5)))
    p = default_params(msg_max=100, msg_min=-100)
    dec = decoder("dvbs2_r1_2", 0, 64)
    got = dec.decode_i8(llr, 6, p)
    assert dec.last_kernel not in ("coop3", "coop") and dec.last_skipped == "coop3"
    assert np.array_equal(got, O.decode_i8(t, llr, 6, O.OMS, 1, msg_max=100))
    dec.decode_i8(llr, 6)
    assert dec.last_kernel == "coop3" and dec.last_skipped is None
    t2 = load_table("dvbs2_r2_3")
    llr2 = channel.awgn_i8_host(t2.n, 16, seed=4, table=channel.i8_table(channel.sigma_from_ebn0(2.0, 2 / 3)))
    d2 = decoder("dvbs2_r2_3", 0, 64)
    got2 = d2.decode_i8(llr2, 6, p)
    assert d2.last_kernel not in ("coop3", "coop") and d2.last_skipped == "coop3"
    assert np.array_equal(got2, O.decode_i8(t2, llr2, 6, O.OMS, 1, msg_max=100))


def test_host_path_chunked_vs_device():
    """The host-buffer API (ldpc_decode_i8 / _f32) decodes a batch in chunks on
    copy/decode lanes (decode_host): its output equals the device API's on the
    same LLRs for pageable and pinned (ldpc_host_alloc) buffers, 1 .. 5 chunks
    and a ragged last chunk; configs[2]'s full 4096-codeword batch included
    (the device path is pinned against the reference by
    test_dvbs2_full_batch_vs_reference)."""
    torch = _torch()
    from ldpcgputegra_amd import pinned_empty
    t = load_table("dvbs2_r1_2")
    B = 4096
    dec = decoder("dvbs2_r1_2", 0, B)
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, 0.5))
    llr = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    dec.awgn_i8_device(llr, 0, 78, table)
    hd = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    dec.decode_i8_device(llr, hd, 50)
    exp = hd.cpu().numpy()
    host = llr.cpu().numpy()
    assert np.array_equal(dec.decode_i8(host, 50), exp)                      # pageable, 4 chunks
    pin_in, pin_out = pinned_empty((B, t.n), np.int8), pinned_empty((B, t.n), np.uint8)
    pin_in[:] = host
    try:
        for chunks, b in (("1", 1000), ("3", 1000), ("5", 1400), ("2", B)):
            os.environ["LDPC_HOST_CHUNKS"] = chunks
            dec.decode_i8(pin_in[:b], 50, out=pin_out[:b])
            assert np.array_equal(pin_out[:b], exp[:b]), (chunks, b)
    finally:
        del os.environ["LDPC_HOST_CHUNKS"]
    f = load_table("648x324")
    fd = decoder("648x324", 0, 1000)
    y = (-1.0 + 0.8 * np.random.default_rng(3).standard_normal((1000, f.n))).astype(np.float32)
    hf = torch.empty((1000, f.n), dtype=torch.uint8, device="cuda")
    fd.decode_f32_device(torch.from_numpy(y).cuda(), hf, 20)
    assert np.array_equal(fd.decode_f32(y, 20), hf.cpu().numpy())


def test_host_async_two_contexts_ping_pong():
    """ldpc_decode_i8_host_async: two contexts on two streams keep two host
    batches in flight (the reference's streams x frames model,
    paper/ldpcGpuTegra.tex:279-289); six batches of alternating inputs (pinned
    and pageable, a ragged 1000-codeword batch) give exactly the device API's
    hard decisions, and ldpc_ctx_synchronize is a no-op with nothing queued."""
    torch = _torch()
    from ldpcgputegra_amd import pinned_empty
    t = load_table("dvbs2_r1_2")
    B = 1024
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, 0.5))
    decs = [Decoder(Code("dvbs2_r1_2"), max_batch=B) for _ in range(2)]
    decs[0].synchronize()
    streams = [torch.cuda.Stream() for _ in range(2)]
    ins = [pinned_empty((B, t.n), np.int8), np.empty((B, t.n), np.int8)]
    outs = [pinned_empty((B, t.n), np.uint8), np.empty((B, t.n), np.uint8)]
    exp = []
    for i in range(2):
        ins[i][:] = channel.awgn_i8_host(t.n, B, 79, table, first_cw=i * B)
        d_h = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
        decoder("dvbs2_r1_2", 0, B).decode_i8_device(torch.from_numpy(ins[i]).cuda(), d_h, 30)
        torch.cuda.synchronize()
        exp.append(d_h.cpu().numpy())
    for k in range(6):
        j = k % 2
        if k >= 2:
            decs[j].synchronize()
            assert np.array_equal(outs[j][:nb[j]], exp[j][:nb[j]]), k
        nb = nb if k else [B, B]
        nb[j] = 1000 if k == 4 else B
        outs[j][:] = 2
        decs[j].decode_i8_host_async(ins[j][:nb[j]], outs[j][:nb[j]], 30, stream=streams[j].cuda_stream)
    for j in range(2):
        decs[j].synchronize()
        assert np.array_equal(outs[j][:nb[j]], exp[j][:nb[j]]), j
        assert decs[j].last_kernel == "coop3"
        decs[j].close()


def test_context_per_device_and_bad_device():
    """One context per device id (the multi-GPU layout): every
    visible device decodes the same codewords bit-identically; a device id
    beyond the visible ones is rejected with LDPC_EINVAL, not a crash."""
    torch = _torch()
    from ldpcgputegra_amd import LdpcError
    from ldpcgputegra_amd import _lib
    import ctypes as C
    cnt = C.c_int()
    _lib.check(_lib.lib().ldpc_device_count(C.byref(cnt)))
    assert cnt.value >= 1
    t = load_table("576x288")
    llr = channel.awgn_i8_host(t.n, 40, seed=12, table=channel.i8_table(0.8))
    exp = O.decode_i8(t, llr, 12)
    for dev in range(cnt.value):
        d = Decoder(Code("576x288"), device=dev, max_batch=64)
        assert np.array_equal(d.decode_i8(llr, 12), exp), dev
        d.close()
    with pytest.raises(LdpcError):
        Decoder(Code("576x288"), device=cnt.value, max_batch=64)


@pytest.mark.parametrize("code,dtype,kernel", [("648x324", "f32", 9), ("648x324", "f32", 7), ("576x288", "f32", 9),
                                               ("dvbs2_r1_2", "i8", 8), ("576x288", "i8", 7)])
def test_decode_count_matches_separate_count(code, dtype, kernel):
    """ldpc_decode_*_count_async (decode + CErrorAnalyzer-style count in one
    call; fused into the ldsep epilogue) gives the hard decisions of the plain
    decode and the counts ldpc_count_errors_async gives on them, for the
    all-zero reference and for an explicit reference codeword array."""
    import torch
    t = load_table(code)
    B = 96 if t.n < 10000 else 32
    iters = 10
    sigma = channel.sigma_from_ebn0(0.5, t.k_info / t.n)
    dec = Decoder(Code(code), max_batch=B, kernel=kernel)
    if dtype == "f32":
        rng = np.random.default_rng(4)
        llr = torch.from_numpy((-1.0 + sigma * rng.standard_normal((B, t.n))).astype(np.float32)).cuda()
        p = default_params(algo=ALGO_MS, beta=0.0)
    else:
        llr = torch.from_numpy(channel.awgn_i8_host(t.n, B, seed=4, table=channel.i8_table(sigma))).cuda()
        p = default_params()
    ref = torch.from_numpy(np.random.default_rng(9).integers(0, 2, (B, t.n), dtype=np.uint8)).cuda()
    for r in (None, ref):
        hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
        hard2 = torch.empty_like(hard)
        c1 = torch.zeros(2, dtype=torch.int64, device="cuda")
        c2 = torch.zeros(2, dtype=torch.int64, device="cuda")
        dec.decode_count_device(llr, hard, iters, t.k_info, c1, ref=r, params=p)
        (dec.decode_f32_device if dtype == "f32" else dec.decode_i8_device)(llr, hard2, iters, params=p)
        dec.count_errors_device(hard2, t.k_info, c2, ref=r)
        torch.cuda.synchronize()
        assert dec.last_kernel == Decoder.KERNEL_NAMES[kernel]
        assert torch.equal(hard, hard2)
        assert c1.tolist() == c2.tolist() and c1[1] > 0, (c1.tolist(), c2.tolist())
