"""BER curve identity: the MI355X decoder's BER/FER at each Eb/N0 equals the
reference code/x86 SSE decoder's on the same int8 LLRs (BASELINE.json north
star: "BER curve identical to code/x86").

The LLRs come from the device AWGN generator (all-zero codeword, BPSK,
``q = clamp(trunc(8 y), +-31)`` as code/x86/CFixPointConversion/
CFastFixConversion.cpp:55-65), are copied to the host and decoded twice:
on the GPU through the C-ABI (default kernel selection: coop3 for DVB-S2
r1/2) and by the reference's own CDecoder_OMS_fixed_SSE (oracle/_ref, built
from the unmodified sources; 16-frame decode() calls as code/x86/main_p.cpp:485),
or by the oracle's C restatement when _ref was not built.  Errors are
counted over the K_info systematic positions as
code/x86/CErrorAnalyzer/CErrorAnalyzer.cpp:123-154.

The per-point frame count is LDPC_BER_FRAMES (default 256), the Eb/N0 points
LDPC_BER_EBN0 (comma-separated dB; default 0.7 .. 1.2 plus SURVEY.md §8(d)
Config 3's 1.5); with LDPC_BER_CURVE_OUT set, the curve is written there as
JSON (the committed artefacts profiles/r04_ber_curve.json, and r01d's before
it, came from that).
"""
import json
import os

import numpy as np
import pytest

import oracle as O
from ldpcgputegra_amd import Code, Decoder, channel

pytestmark = pytest.mark.gpu

EBN0 = tuple(float(x) for x in os.environ.get("LDPC_BER_EBN0", "0.7,0.8,0.9,1.0,1.1,1.2,1.5").split(","))


def test_dvbs2_ber_curve_identical_to_reference():
    import torch
    name, iters = "dvbs2_r1_2", 50
    frames = int(os.environ.get("LDPC_BER_FRAMES", "256"))
    frames = max(16, frames // 16 * 16)
    code = Code(name)
    k_info = code.k_info
    dec = Decoder(code, max_batch=min(frames, 4096))
    kind = "reference" if O.ref_available(name) else "port"
    threads = min(16, os.cpu_count() or 1)
    rows = []
    for pi, ebn0 in enumerate(EBN0):
        table = channel.i8_table(channel.sigma_from_ebn0(ebn0, code.k_info / code.n))
        gpu_hard = []
        host_llr = []
        for b0 in range(0, frames, dec.max_batch):
            B = min(dec.max_batch, frames - b0)
            d = torch.empty((B, code.n), dtype=torch.int8, device="cuda")
            dec.awgn_i8_device(d, first_cw=pi * 1_000_000 + b0, seed=2024, table=table)
            host_llr.append(d.cpu().numpy())
            gpu_hard.append(dec.decode_i8(host_llr[-1], iters))
        llr = np.concatenate(host_llr)
        got = np.concatenate(gpu_hard)
        if kind == "reference":
            exp = O.ref_decode_mt(name, llr, iters, 1, threads)
        else:
            exp = O.decode_i8_mt(load_table_of(code), llr, iters, 1, threads)
        diff = int((got != exp).sum())
        be_g = got[:, :k_info].sum(axis=1)     # all-zero codeword: a 1 is an error
        be_r = exp[:, :k_info].sum(axis=1)
        rows.append(dict(ebn0_db=ebn0, sigma=channel.sigma_from_ebn0(ebn0, code.k_info / code.n), frames=frames,
                         gpu_ber=float(be_g.sum()) / (frames * k_info), gpu_fer=float((be_g > 0).mean()),
                         ref_ber=float(be_r.sum()) / (frames * k_info), ref_fer=float((be_r > 0).mean()),
                         differing_bits=diff))
        assert diff == 0, "Eb/N0 %.2f dB: %d hard-decision bits differ from the %s decoder" % (ebn0, diff, kind)
    out = os.environ.get("LDPC_BER_CURVE_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(dict(code=name, iters=iters, algo="int8 OMS offset 1", checker=kind, kernel=dec.last_kernel,
                           checker_threads=threads, points=rows), f, indent=1)
    # the curve must actually span the waterfall (otherwise the identity says little)
    assert rows[0]["ref_fer"] > rows[-1]["ref_fer"] or rows[0]["ref_fer"] == 0


def load_table_of(code):
    from ldpcgputegra_amd import load_table
    return load_table(code.name)
