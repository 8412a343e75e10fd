#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-buffer boundary (ldpc_decode_i8 /
ldpc_decode_f32: host LLRs in, host hard decisions out, synchronous, as the
reference's CDecoder::decode(char*, char*, int) is called), with pageable
and with pinned (ldpc_host_alloc) buffers, against the resident rate (the
same decode on device buffers).  Not the bench value (bench.py keeps inputs
resident in HBM); recorded in DESIGN.md.
Streaming mode (`stream`): two contexts on two streams ping-pong pinned host
batches with ldpc_decode_i8_host_async (H2D of batch k+1 and D2H of batch k-1
under the decode of batch k: the reference's W streams x F frames in flight,
paper/ldpcGpuTegra.tex:279-289), >= 20 batches timed in steady state.
usage (GPU box): python tools/host_path_rate.py [chunks ... | stream [batches]]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpcgputegra_amd import ALGO_MS, Code, Decoder, channel, default_params, pinned_empty  # noqa: E402


def rate(code_name, batch, iters, is_float, pinned, reps=5):
    import torch
    code = Code(code_name)
    dec = Decoder(code, max_batch=batch)
    sigma = channel.sigma_from_ebn0(1.0, code.k_info / code.n)
    dt = np.float32 if is_float else np.int8
    if is_float:
        src = (-1.0 + sigma * np.random.default_rng(1).standard_normal((batch, code.n))).astype(np.float32)
        p = default_params(algo=ALGO_MS)
    else:
        src = channel.awgn_i8_host(code.n, batch, 1, channel.i8_table(sigma))
        p = default_params()
    llr = pinned_empty(src.shape, dt) if pinned else np.empty(src.shape, dt)
    llr[:] = src
    hard = pinned_empty((batch, code.n), np.uint8) if pinned else np.empty((batch, code.n), np.uint8)
    run = (lambda: dec.decode_f32(llr, iters, p, out=hard)) if is_float else (lambda: dec.decode_i8(llr, iters, p, out=hard))
    run()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    el = (time.perf_counter() - t0) / reps
    # resident: the same decode on device buffers
    d_llr, d_hard = torch.from_numpy(src).cuda(), torch.empty((batch, code.n), dtype=torch.uint8, device="cuda")
    dev = (lambda: dec.decode_f32_device(d_llr, d_hard, iters, p)) if is_float else (
        lambda: dec.decode_i8_device(d_llr, d_hard, iters, p))
    dev()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dev()
    torch.cuda.synchronize()
    el_dev = (time.perf_counter() - t0) / reps
    return dict(code=code_name, batch=batch, iters=iters, dtype="f32" if is_float else "int8",
                buffers="pinned" if pinned else "pageable", chunks=os.environ.get("LDPC_HOST_CHUNKS", "default"),
                kernel=dec.last_kernel, ms_per_call=round(el * 1e3, 3), resident_ms=round(el_dev * 1e3, 3),
                host_path_mbps=round(batch * code.n / el / 1e6, 1),
                resident_mbps=round(batch * code.n / el_dev / 1e6, 1), host_over_resident=round(el_dev / el, 3))


def stream_rate(code_name="dvbs2_r1_2", batch=4096, iters=50, batches=24, warm=2):
    """Steady-state PCIe-inclusive rate of two contexts ping-ponging pinned
    host batches, against the resident rate of the same decodes."""
    import torch
    code = Code(code_name)
    sigma = channel.sigma_from_ebn0(1.0, code.k_info / code.n)
    p = default_params()
    decs = [Decoder(code, max_batch=batch) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    llr = [pinned_empty((batch, code.n), np.int8) for _ in range(2)]
    hard = [pinned_empty((batch, code.n), np.uint8) for _ in range(2)]
    for i in range(2):
        llr[i][:] = channel.awgn_i8_host(code.n, batch, 1, channel.i8_table(sigma), first_cw=i * batch)

    def submit(k):
        decs[k % 2].decode_i8_host_async(llr[k % 2], hard[k % 2], iters, p, stream=streams[k % 2].cuda_stream)

    for k in range(warm):
        submit(k)
    for d in decs:
        d.synchronize()
    t0 = time.perf_counter()
    for k in range(batches):
        if k >= 2:
            decs[k % 2].synchronize()   # batch k-2 done: its buffers may be refilled / read
        submit(k)
    for d in decs:
        d.synchronize()
    el = (time.perf_counter() - t0) / batches
    # the outputs equal a resident decode of the same inputs
    d_llr = torch.from_numpy(np.ascontiguousarray(llr[(batches - 1) % 2])).cuda()
    d_hard = torch.empty((batch, code.n), dtype=torch.uint8, device="cuda")
    decs[0].decode_i8_device(d_llr, d_hard, iters, p)
    torch.cuda.synchronize()
    same = bool(np.array_equal(d_hard.cpu().numpy(), hard[(batches - 1) % 2]))
    t0 = time.perf_counter()
    for _ in range(5):
        decs[0].decode_i8_device(d_llr, d_hard, iters, p)
    torch.cuda.synchronize()
    el_dev = (time.perf_counter() - t0) / 5
    for d in decs:
        d.close()
    return dict(mode="stream", code=code_name, batch=batch, iters=iters, dtype="int8", buffers="pinned",
                contexts=2, batches_timed=batches, kernel="coop3" if code_name == "dvbs2_r1_2" else None,
                ms_per_batch=round(el * 1e3, 3), resident_ms=round(el_dev * 1e3, 3),
                host_path_mbps=round(batch * code.n / el / 1e6, 1),
                resident_mbps=round(batch * code.n / el_dev / 1e6, 1), host_over_resident=round(el_dev / el, 3),
                outputs_equal_resident=same)


if __name__ == "__main__":
    if sys.argv[1:2] == ["stream"]:
        print(json.dumps(stream_rate(batches=int(sys.argv[2]) if len(sys.argv) > 2 else 24)), flush=True)
        sys.exit(0)
    for ch in (sys.argv[1:] or ["2"]):
        os.environ["LDPC_HOST_CHUNKS"] = ch
        for args in (("dvbs2_r1_2", 4096, 50, False), ("648x324", 1024, 20, True)):
            for pinned in (False, True):
                print(json.dumps(rate(*args, pinned)), flush=True)
