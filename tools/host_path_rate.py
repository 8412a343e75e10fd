#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (ldpc_decode_i8 /
ldpc_decode_f32: pageable host LLRs in, host hard decisions out, synchronous,
as the reference's CDecoder::decode(char*, char*, int) is called).  Not the
bench value (bench.py keeps inputs resident in HBM); recorded in DESIGN.md.
usage (GPU box): python tools/host_path_rate.py"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpcgputegra_amd import ALGO_MS, Code, Decoder, channel, default_params  # noqa: E402


def rate(code_name, batch, iters, is_float, reps=5):
    code = Code(code_name)
    dec = Decoder(code, max_batch=batch)
    sigma = channel.sigma_from_ebn0(1.0, code.k_info / code.n)
    if is_float:
        llr = (-1.0 + sigma * np.random.default_rng(1).standard_normal((batch, code.n))).astype(np.float32)
        run = lambda: dec.decode_f32(llr, iters, default_params(algo=ALGO_MS))   # noqa: E731
    else:
        llr = channel.awgn_i8_host(code.n, batch, 1, channel.i8_table(sigma))
        run = lambda: dec.decode_i8(llr, iters)   # noqa: E731
    run()
    dec.profile(True)
    dec.kernel_time(reset=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    el = (time.perf_counter() - t0) / reps
    kms, n = dec.kernel_time(reset=True)
    return dict(code=code_name, batch=batch, iters=iters, dtype="f32" if is_float else "int8",
                kernel=dec.last_kernel, ms_per_call=round(el * 1e3, 3), kernel_ms=round(kms / max(n, 1), 3),
                host_path_mbps=round(batch * code.n / el / 1e6, 1))


if __name__ == "__main__":
    for args in (("dvbs2_r1_2", 4096, 50, False), ("648x324", 1024, 20, True)):
        print(json.dumps(rate(*args)), flush=True)
