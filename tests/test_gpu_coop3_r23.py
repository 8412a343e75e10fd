"""coop3 beyond DVB-S2 r1/2: first-group degree 10 (DVB-S2 r2/3, the
reference's code/gpu_fixed/matrix/64800x21600 table) and 14 (the DVB-S2-shaped
r3/4 of configs[4]) -- coop3_decode<10 | 14, 4, 2>: 4 slab waves (one per SIMD)
over windows of <= 32 checks, 8 / 12 information edges per check, two 16-bit
edge-code words per codeword (96-B message records), 1 / 2 line loads per lane
group and period -- and first-group degree 22, 27, 30 (the shaped r5/6 of
configs[4], the reference's r8/9 and r9/10, code/x86/Constantes/64800x7200 /
64800x6480) -- coop3_decode<22 | 27 | 30, 4, 2>: two lanes per check (4 slab
waves of 4 slots over windows of 16 checks, each lane reducing half of the 20 /
25 / 28 information edges, a DPP min / sign merge), 160-B message records,
gathers and stores in two instructions per slot set, 3 / 4 line loads per lane
group and period -- against the oracle
(the reference's recurrence, CDecoder_OMS_fixed_SSE.cpp:172-546; NMS
CDecoder_NMS_fixed_SSE.cpp:188-240; early termination per codeword on the
posterior hard-decision syndrome after each iteration, SURVEY.md §8(f) row 2 --
the build's definition, not the reference's commented `arret` test (:255,
551-553: extrinsic sign parity per 16-frame call), so iterations used are
unpinned by the reference).  The reference ships no r2/3 or shaped decoder build
(its x86 tree has constantes_sse.h only for 64800x{32400,7200,6480}), so the
oracle -- pinned on the 88 reference golden cases, which include r8/9 and
r9/10 and run on coop3 in test_gpu_parity.py -- is the checker: soft output,
hard decisions and iterations used, bit for bit."""
import numpy as np
import pytest

import oracle as O
from ldpcgputegra_amd import ALGO_NMS, Code, Decoder, channel, default_params, load_table

pytestmark = pytest.mark.gpu
CODES = ["dvbs2_r2_3", "dvbs2shape_r3_4", "dvbs2shape_r5_6", "dvbs2_r8_9", "dvbs2_r9_10"]
EBN0 = {"dvbs2_r2_3": (1.9, 2.3, 1.8, 2.2), "dvbs2shape_r3_4": (2.35, 2.6, 2.3, 2.8),   # OMS ET, NMS ET, staged, full
        "dvbs2shape_r5_6": (3.4, 3.3, 3.4, 3.5), "dvbs2_r8_9": (4.3, 4.1, 4.3, 4.6), "dvbs2_r9_10": (4.4, 4.5, 4.4, 5.0)}


def _run(CODE, llr, iters, params, batch=None, max_batch=None):
    import torch
    t = load_table(CODE)
    B = llr.shape[0]
    dec = Decoder(Code(CODE), max_batch=max_batch or max(B, 64), kernel=8)
    d_hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
    d_soft = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
    d_its = torch.empty(B, dtype=torch.int32, device="cuda")
    dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, iters, params=params, soft=d_soft, iters_used=d_its)
    torch.cuda.synchronize()
    assert dec.last_kernel == "coop3"
    out = d_hard.cpu().numpy(), d_soft.cpu().numpy(), d_its.cpu().numpy(), dec.last_et_stage
    dec.close()
    return out


def _llr(CODE, B, ebn0, seed):
    t = load_table(CODE)
    return channel.awgn_i8_host(t.n, B, seed=seed, table=channel.i8_table(channel.sigma_from_ebn0(ebn0, t.k_info / t.n)))


@pytest.mark.parametrize("CODE", CODES)
@pytest.mark.parametrize("batch,iters", [(1, 3), (37, 10), (200, 25)])
def test_r23_fixed_iterations_vs_oracle(CODE, batch, iters):
    """Fixed iterations, OMS offset 1: ragged batch (37), one codeword, and a
    batch that turns the XCD workgroup remap on (200: grid 16)."""
    t = load_table(CODE)
    llr = _llr(CODE, batch, EBN0[CODE][0], 11 + batch)
    eh, es, _ = O.decode_i8(t, llr, iters, return_soft=True, threads=O.host_threads())
    h, s, its, _ = _run(CODE, llr, iters, default_params())
    assert np.array_equal(s, es)
    assert np.array_equal(h, eh)
    assert (its == iters).all()


@pytest.mark.parametrize("CODE", CODES)
@pytest.mark.parametrize("nms", [False, True])
def test_r23_early_termination_vs_oracle(CODE, nms):
    """In-kernel early termination (one launch): soft, hard and iterations
    used equal the oracle's per-codeword stop; OMS and NMS factor 24."""
    t = load_table(CODE)
    B, iters = 200, 30
    llr = _llr(CODE, B, EBN0[CODE][1] if nms else EBN0[CODE][0], 5)   # NMS 24/32 converges later than OMS
    algo, param = (O.NMS, 24) if nms else (O.OMS, 1)
    eh, es, eit = O.decode_i8(t, llr, iters, algo, param, early_term=True, return_soft=True, threads=O.host_threads())
    assert eit.min() < iters and eit.max() > eit.min()
    p = default_params(early_term=1, algo=ALGO_NMS, factor=24) if nms else default_params(early_term=1)
    h, s, its, st = _run(CODE, llr, iters, p)
    assert st == 0
    assert np.array_equal(its, eit)
    assert np.array_equal(s, es)
    assert np.array_equal(h, eh)


@pytest.mark.parametrize("CODE", CODES)
def test_r23_nms_fixed_vs_oracle(CODE):
    t = load_table(CODE)
    llr = _llr(CODE, 64, EBN0[CODE][1], 8)
    eh, es, _ = O.decode_i8(t, llr, 12, O.NMS, 29, return_soft=True, threads=O.host_threads())
    h, s, _, _ = _run(CODE, llr, 12, default_params(algo=ALGO_NMS, factor=29))
    assert np.array_equal(s, es) and np.array_equal(h, eh)


@pytest.mark.parametrize("CODE", CODES)
def test_r23_staged_early_termination_vs_oracle(CODE, monkeypatch):
    """Staged early termination (compaction of the codewords still decoding
    into 16-codeword groups, messages in the 96 .. 160-B record layouts), forced at a
    small batch: equal to the oracle."""
    t = load_table(CODE)
    B, iters = 200, 30
    llr = _llr(CODE, B, EBN0[CODE][2], 17)
    eh, es, eit = O.decode_i8(t, llr, iters, early_term=True, return_soft=True, threads=O.host_threads())
    k1 = int(np.percentile(eit, 30))
    assert 0 < k1 < iters and (eit > k1).any()
    monkeypatch.setenv("LDPC_COOP3_ET_STAGE_MIN", "0")
    monkeypatch.setenv("LDPC_COOP3_ET_K", str(k1))
    monkeypatch.setenv("LDPC_COOP3_ET_STEP", "3")
    h, s, its, st = _run(CODE, llr, iters, default_params(early_term=1), max_batch=256)
    assert st == k1
    assert np.array_equal(its, eit)
    assert np.array_equal(s, es)
    assert np.array_equal(h, eh)


@pytest.mark.parametrize("CODE", CODES)
def test_r23_full_batch_fixed_50_sampled_vs_oracle(CODE):
    """configs[2]'s shape on the higher rates: batch 4096, 50 iterations, at
    bench.py's --mixed Eb/N0 of the rate: a seeded sample of 256 codewords
    (spread over every XCD's workgroups) equals the oracle's decode, hard
    decisions and soft output."""
    t = load_table(CODE)
    B, iters = 4096, 50
    llr = _llr(CODE, B, EBN0[CODE][3], 2024)
    h, s, _, _ = _run(CODE, llr, iters, default_params(), max_batch=B)
    sel = np.sort(np.random.default_rng(1).choice(B, 256, replace=False))
    eh, es, _ = O.decode_i8(t, llr[sel], iters, return_soft=True, threads=O.host_threads())
    assert np.array_equal(s[sel], es)
    assert np.array_equal(h[sel], eh)


@pytest.mark.parametrize("CODE", ["dvbs2_r1_2", "dvbs2_r2_3", "dvbs2shape_r5_6"])
def test_wave_priorities_do_not_change_results(CODE, monkeypatch):
    """The chain / memory wave priorities (coop3_chain_prio / coop3_mem_prio,
    overridden by LDPC_COOP3_PRIO / LDPC_COOP3_MPRIO per launch) only reorder
    issue: every level gives the oracle's soft output, fixed iterations and
    early termination alike."""
    t = load_table(CODE)
    ebn0 = {"dvbs2_r1_2": 1.0}.get(CODE) or EBN0[CODE][0]
    llr = _llr(CODE, 37, ebn0, 23)
    eh, es, _ = O.decode_i8(t, llr, 10, return_soft=True, threads=O.host_threads())
    _, ees, eit = O.decode_i8(t, llr, 30, early_term=True, return_soft=True, threads=O.host_threads())
    for chain, mem in [(0, 0), (3, 2), (1, 3)]:
        monkeypatch.setenv("LDPC_COOP3_PRIO", str(chain))
        monkeypatch.setenv("LDPC_COOP3_MPRIO", str(mem))
        h, s, _, _ = _run(CODE, llr, 10, default_params())
        assert np.array_equal(s, es) and np.array_equal(h, eh), (chain, mem)
        _, s2, its, _ = _run(CODE, llr, 30, default_params(early_term=1))
        assert np.array_equal(s2, ees) and np.array_equal(its, eit), (chain, mem)
