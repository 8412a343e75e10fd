#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ (run in the dev container).

Expected outputs come from the REFERENCE itself: the unmodified
code/x86 SSE decoders (CDecoder_OMS_fixed_SSE / CDecoder_NMS_fixed_SSE)
compiled from /root/reference by oracle/Makefile (`make -C oracle ref`) and
driven through oracle/ref_harness.cpp, 16 frames per decode() call exactly as
code/x86/main_p.cpp:485 does.

Inputs are int8 LLRs from the integer-exact AWGN generator defined in
ldpcgputegra_amd/channel.py, re-implemented here in numpy (``awgn_i8``) so the
fixtures do not depend on the product library; the script cross-checks it
against the library's host generator.  For short codes the full LLR arrays are
stored; for N = 64800 the (seed, threshold table) and the SHA-256 of the
regenerated LLRs are stored instead, together with the bit-packed reference
hard decisions.

Usage:  python tests/golden/gen_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

OUT = os.path.dirname(os.path.abspath(__file__))

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & M64
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & M64
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & M64
    return x ^ (x >> np.uint64(31))


def random_codewords(code, batch, info_seed):
    """Random info bits (numpy PCG64, seed info_seed) DVB-S2-encoded by the product encoder."""
    from ldpcgputegra_amd import Code
    c = Code(code)
    info = np.random.default_rng(info_seed).integers(0, 2, size=(batch, c.k_info), dtype=np.uint8)
    return c.encode(info)


def awgn_i8(n, batch, seed, table, first_cw=0, codeword=None):
    """numpy restatement of ldpc_awgn_i8_host (codeword None = all-zero)."""
    sat = int(table[63])
    idx = (np.arange(batch, dtype=np.uint64)[:, None] + np.uint64(first_cw)) * np.uint64(n) + \
        np.arange(n, dtype=np.uint64)[None, :]
    key = np.uint64((int(seed) * 0xD1B54A32D192ED03) & 0xFFFFFFFFFFFFFFFF)
    u = (splitmix64(idx ^ key) >> np.uint64(32)).astype(np.uint64)
    th = np.asarray(table[:2 * sat], dtype=np.uint64)
    cnt = (u[..., None] >= th).sum(axis=-1)
    q = (cnt - sat).astype(np.int8)
    if codeword is not None:
        q = np.where(codeword.astype(bool), -q, q).astype(np.int8)
    return q


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    import oracle as O
    from ldpcgputegra_amd import channel, load_table

    cases = []

    def add(name, code, llr, iters, algo, param, vmin=-127, mmax=31, store_llr=True, gen=None, cw=None):
        hard = O.ref_decode(code, llr, iters, algo, param, vmin=vmin, mmax=mmax, mmin=-mmax)
        rec = dict(name=name, code=code, iters=iters, algo=algo, param=param, var_min=vmin, msg_max=mmax,
                   batch=int(llr.shape[0]), llr_sha256=sha(llr), hard_sha256=sha(hard),
                   bit_errors=int((hard != (0 if cw is None else cw)).sum()))
        arrays = dict(hard_packed=np.packbits(hard, axis=-1))
        if store_llr:
            rec["llr_file"] = "llr_%s.npy" % rec["llr_sha256"][:16]
            np.save(os.path.join(OUT, rec["llr_file"]), llr)
        else:
            rec.update(gen)
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
        cases.append(rec)
        print(name, rec["bit_errors"], file=sys.stderr)

    def gen_llr(code, ebn0, batch, seed):
        t = load_table(code)
        sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
        table = channel.i8_table(sigma, 8, 31)
        llr = awgn_i8(t.n, batch, seed, table)
        assert np.array_equal(llr, channel.awgn_i8_host(t.n, batch, seed, table)), "generator mismatch"
        return llr, dict(seed=seed, ebn0=ebn0, sigma=sigma, table=[int(x) for x in table])

    # --- short codes: full inputs stored
    for code, ebn0s in [("576x288", (1.0, 2.0, 3.0)), ("1944x972", (1.0, 1.5, 2.0)),
                        ("2304x1152", (1.5,)), ("2048x384", (3.0,)), ("4000x2000", (1.5,))]:
        for ebn0 in ebn0s:
            llr, _ = gen_llr(code, ebn0, 16, seed=1000 + int(ebn0 * 10))
            tag = "%s_eb%02d" % (code, int(ebn0 * 10))
            for it in (0, 1, 2, 20, 50):
                add("%s_oms1_it%d" % (tag, it), code, llr, it, O.OMS, 1)
            add("%s_oms2_it20" % tag, code, llr, 20, O.OMS, 2)
            add("%s_oms0_it20" % tag, code, llr, 20, O.OMS, 0)
            add("%s_nms29_it20" % tag, code, llr, 20, O.NMS, 29)
    # --- saturation stress: uniform int8 LLRs in [-127, 127], and a -128 floor
    rng = np.random.default_rng(1234)
    for code in ("576x288", "1944x972"):
        n = load_table(code).n
        llr = rng.integers(-127, 128, size=(16, n), dtype=np.int16).astype(np.int8)
        add("%s_stress127_oms1_it10" % code, code, llr, 10, O.OMS, 1)
        add("%s_stress127_nms29_it10" % code, code, llr, 10, O.NMS, 29)
        add("%s_stress127_msg127_it10" % code, code, llr, 10, O.OMS, 3, mmax=127)
        llr2 = rng.integers(-128, 128, size=(16, n), dtype=np.int16).astype(np.int8)
        add("%s_stress128_vmin128_it10" % code, code, llr2, 10, O.OMS, 1, vmin=-128)
    # --- DVB-S2 r1/2 at 50 iterations: converged / waterfall / failing
    for ebn0 in (0.7, 0.9, 1.2):
        llr, gen = gen_llr("dvbs2_r1_2", ebn0, 16, seed=5000 + int(ebn0 * 10))
        add("dvbs2_r1_2_eb%02d_oms1_it50" % int(ebn0 * 10), "dvbs2_r1_2", llr, 50, O.OMS, 1, store_llr=False,
            gen=gen)
    llr, gen = gen_llr("dvbs2_r1_2", 0.9, 16, seed=5009)
    add("dvbs2_r1_2_eb09_nms29_it20", "dvbs2_r1_2", llr, 20, O.NMS, 29, store_llr=False, gen=gen)
    # random (non-zero) codewords through the DVB-S2 encoder: sign handling
    # with both bit values (the reference's -encoder mode, GenericEncoder)
    for code, ebn0, it in (("dvbs2_r1_2", 0.9, 50), ("dvbs2_r8_9", 4.0, 30)):
        t = load_table(code)
        sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
        table = channel.i8_table(sigma, 8, 31)
        cw = random_codewords(code, 16, info_seed=77)
        llr = awgn_i8(t.n, 16, 7001, table, codeword=cw)
        assert np.array_equal(llr, channel.awgn_i8_host(t.n, 16, 7001, table, codeword=cw))
        gen = dict(seed=7001, ebn0=ebn0, sigma=sigma, table=[int(x) for x in table], info_seed=77)
        add("%s_eb%02d_randcw_oms1_it%d" % (code, int(ebn0 * 10), it), code, llr, it, O.OMS, 1, store_llr=False,
            gen=gen, cw=cw)
    for code, ebn0 in (("dvbs2_r8_9", 4.0), ("dvbs2_r9_10", 4.4)):
        llr, gen = gen_llr(code, ebn0, 16, seed=6000)
        add("%s_eb%02d_oms1_it30" % (code, int(ebn0 * 10)), code, llr, 30, O.OMS, 1, store_llr=False, gen=gen)

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py", reference="code/x86 CDecoder_{OMS,NMS}_fixed_SSE",
                       cases=cases), f, indent=1)


if __name__ == "__main__":
    main()
