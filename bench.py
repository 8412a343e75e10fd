#!/usr/bin/env python3
"""Throughput benchmark: layered int8 offset-min-sum decode of DVB-S2
N=64800 r=1/2 at 50 iterations (BASELINE.json configs[2]: batch 4096 per GPU).

A "step" = one pass of the hot path over one batch: frame-major int8 LLRs
already resident in HBM -> interleave -> layered decode (50 it) -> hard
decisions (frame-major) -> bit/frame error count.  Inputs come from the
integer-exact AWGN generator on the device (synthetic, all-zero codeword, as
the reference's CFakeEncoder + channel) and are generated before timing.

Multi-GPU: one process per GPU (torch.distributed.run); every rank decodes
its own contiguous shard of codewords (first codeword = rank * batch) with no
data-path collective ("scaling": "weak"); only the timing (max over ranks)
and the 3 error counters are reduced after the timed region.

Prints ONE JSON line on rank 0 (contract in the task statement / DESIGN.md).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def source_hash():
    from ldpcgputegra_amd._lib import source_hash as h
    return h()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default 10; f32: 400 -- a 0.05 ms step, so that the host's fixed "
                         "synchronisation cost around the timed region stays below 1 %%)")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--dtype", default="i8", choices=("i8", "f32"),
                    help="i8: configs[2] (default); f32: configs[1], float min-sum (defaults 648x324, batch 1024, 20 it)")
    ap.add_argument("--mixed", action="store_true",
                    help="configs[4]: mixed-rate DVB-S2 batch with early termination (rates: --mixed-codes)")
    ap.add_argument("--mixed-codes", default="configs4", choices=("configs4", "reference"),
                    help="configs4: 1/2 + DVB-S2-shaped 3/4, 5/6 (default); reference: 1/2, 2/3, 8/9, 9/10")
    ap.add_argument("--code", default=None, help="default dvbs2_r1_2 (i8) / 648x324 (f32)")
    ap.add_argument("--batch", type=int, default=None, help="codewords per GPU (default 4096 i8 / 1024 f32)")
    ap.add_argument("--iters", type=int, default=None, help="default 50 (i8) / 20 (f32)")
    ap.add_argument("--ebn0", type=float, default=1.0, help="Eb/N0 (dB) of the synthetic channel")
    ap.add_argument("--kernel", type=int, default=0,
                    help="0 auto, 1 generic, 2 windowed, 3 windowed2 S=16, 5 coop, 7 lds, 8 coop3, 9 ldsep (float)")
    ap.add_argument("--seed", type=int, default=2024)
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU baseline time budget (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = this process's CPU share (cgroup quota / affinity)")
    ap.add_argument("--traffic-file", default=os.path.join(ROOT, "profiles", "traffic.json"))
    a = ap.parse_args()
    f32 = a.dtype == "f32"
    if a.code is None:
        a.code = "648x324" if f32 else "dvbs2_r1_2"
    if a.batch is None:
        a.batch = 1024 if f32 else 4096
    if a.iters is None:
        a.iters = 20 if f32 else 50
    if a.steps is None:
        a.steps = 400 if f32 and not a.mixed else 10
    return a


def hbm_peak_gbs():
    # MI355X HBM3E peak (MI355X_MICROARCH.md "Chip-level parameters": 8.0 TB/s spec)
    return 8000.0


def lds_peak_gbs():
    # LDS array: 256 B/clk/CU (ds_read_b64 / b128, MI355X_MICROARCH.md "LDS"),
    # 256 CUs at the 2.4 GHz peak engine clock
    return 256 * 256 * 2.4


def host_cpu_info():
    """CPU model, physical cores, logical CPUs and the CPU share this process
    may use (the GPU box grants a cgroup quota of 16 CPUs per GPU on a larger
    host: threads beyond it are throttled, not run)."""
    info = {"model": None, "physical_cores": None, "logical_cpus": os.cpu_count(), "cpu_quota": None}
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        kv = {}
        for line in out.splitlines():
            if ":" in line:
                k, v = line.split(":", 1)
                kv[k.strip()] = v.strip()
        info["model"] = kv.get("Model name")
        if kv.get("Core(s) per socket") and kv.get("Socket(s)"):
            info["physical_cores"] = int(kv["Core(s) per socket"]) * int(kv["Socket(s)"])
    except (OSError, ValueError, subprocess.SubprocessError):
        pass
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    info["cpu_quota"] = O.host_threads()
    return info


def cpu_baseline(code_name, iters, budget_s, threads, seed):
    """Time the reference's own SSE decoder (oracle/_ref, kind "reference";
    one decoder object per thread decoding 16 frames per call, as
    code/x86/main_p.cpp:473-576) or, if it was not built, the oracle port, on
    `threads` host threads (default: the whole CPU share of this process)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from ldpcgputegra_amd import channel, load_table
    t = load_table(code_name)
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, t.k_info / t.n))
    kind = "reference" if O.ref_available(code_name) else "port"

    def rate(thr, budget):
        blk = 16 * thr                     # one 16-frame decode() call per thread per round
        llr = channel.awgn_i8_host(t.n, blk, seed, table)
        done, t0 = 0, time.perf_counter()
        while True:
            if kind == "reference":
                O.ref_decode_mt(code_name, llr, iters, 1, thr)
            else:
                O.decode_i8_mt(t, llr, iters, 1, thr)
            done += blk
            el = time.perf_counter() - t0
            if el >= budget:
                return done, el

    host = host_cpu_info()
    done1, el1 = rate(1, max(1.0, budget_s * 0.2))            # per-thread rate, for the all-core projection
    done, el = rate(threads, budget_s)
    mbps = done * t.n / el / 1e6
    per_thread = done1 * t.n / el1 / 1e6
    return dict(value=round(mbps, 3), unit="Mbit/s", cores=threads, kind=kind,
                threads=threads, cpu_model=host["model"], host_physical_cores=host["physical_cores"],
                host_logical_cpus=host["logical_cpus"], cpu_quota=host["cpu_quota"],
                per_thread_mbps=round(per_thread, 3),
                all_physical_cores_projection_mbps=(round(per_thread * host["physical_cores"], 1)
                                                    if host["physical_cores"] else None),
                sample="%s %d it int8 OMS offset 1: %d codewords (%d threads x 16-frame decode() calls) in %.2f s; "
                       "1 thread: %d codewords in %.2f s. Threads = this process's CPU share (cgroup quota %s of "
                       "%s logical CPUs); the all-core figure is per-thread rate x physical cores, a projection, "
                       "not a measurement" % (code_name, iters, done, threads, el, done1, el1, host["cpu_quota"],
                                              host["logical_cpus"]))


def cpu_baseline_product_host(code_name, iters, budget_s, threads, seed):
    """The product's own host decoder (a device -1 context of the C-ABI,
    csrc/host.cpp: AVX2, 32 codewords per block, one block per thread at a
    time) on the same threads and inputs as cpu_baseline -- the drop-in for a
    machine without a GPU, timed like the reference's per-thread loop
    (code/x86/main_p.cpp:664-765).  Product code, not the oracle."""
    from ldpcgputegra_amd import Code, Decoder, channel, load_table
    t = load_table(code_name)
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, t.k_info / t.n))

    def rate(thr, budget):
        os.environ["LDPC_HOST_THREADS"] = str(thr)
        blk = 32 * thr                     # one 32-codeword block per thread per round
        llr = channel.awgn_i8_host(t.n, blk, seed, table)
        dec = Decoder(Code(code_name), device=-1, max_batch=blk)
        dec.decode_i8(llr[:32], 1)         # untimed: first touch
        done, t0 = 0, time.perf_counter()
        while True:
            dec.decode_i8(llr, iters)
            done += blk
            el = time.perf_counter() - t0
            if el >= budget:
                dec.close()
                return done, el

    old = os.environ.get("LDPC_HOST_THREADS")
    try:
        done1, el1 = rate(1, max(1.0, budget_s * 0.25))
        done, el = rate(threads, budget_s)
    finally:
        if old is None:
            os.environ.pop("LDPC_HOST_THREADS", None)
        else:
            os.environ["LDPC_HOST_THREADS"] = old
    return dict(value=round(done * t.n / el / 1e6, 3), unit="Mbit/s", cores=threads, kind="product-host",
                threads=threads, per_thread_mbps=round(done1 * t.n / el1 / 1e6, 3),
                sample="%s %d it int8 OMS offset 1 on the product's device -1 host decoder: %d codewords "
                       "(%d threads x 32-codeword blocks) in %.2f s; 1 thread: %d codewords in %.2f s"
                       % (code_name, iters, done, threads, el, done1, el1))


def cpu_baseline_f32(code_name, iters, budget_s, threads, seed):
    """The reference has no float decoder (its decode(float*) is a no-op,
    code/x86/CDecoder/template/CDecoder_fixed_SSE.cpp:35-40): time the
    oracle's scalar float restatement (kind "port") on `threads` threads."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from ldpcgputegra_amd import channel, load_table
    t = load_table(code_name)
    sigma = channel.sigma_from_ebn0(1.0, t.k_info / t.n)
    rng = np.random.default_rng(seed)
    blk = 64 * threads
    llr = (-1.0 + sigma * rng.standard_normal((blk, t.n))).astype(np.float32)
    done, t0 = 0, time.perf_counter()
    while True:
        O.decode_f32(t, llr, iters, O.OMS, 0.0, threads=threads)
        done += blk
        el = time.perf_counter() - t0
        if el >= budget_s:
            break
    host = host_cpu_info()
    return dict(value=round(done * t.n / el / 1e6, 3), unit="Mbit/s", cores=threads, kind="port", threads=threads,
                cpu_model=host["model"], host_physical_cores=host["physical_cores"], cpu_quota=host["cpu_quota"],
                sample="%s %d it float min-sum (oracle restatement, scalar, one decoder per thread): %d codewords "
                       "in %.2f s on %d threads" % (code_name, iters, done, el, threads))


# configs[4]: rates {1/2, 3/4, 5/6}.  The reference ships no r3/4 or r5/6 table
# and ETSI Annex B is not available offline: those two are DVB-S2-SHAPED
# stand-ins (tools/make_dvbs2_shaped.py: the Annex-B structure -- N, K, q,
# degree profile, staircase -- with seeded random addresses, so the decoder
# workload of the real rates but not their BER).  --mixed-codes reference runs
# the rates the reference does ship (1/2, 2/3, 8/9, 9/10).
MIXED_SETS = {
    "configs4": ("dvbs2_r1_2", "dvbs2shape_r3_4", "dvbs2shape_r5_6"),
    "reference": ("dvbs2_r1_2", "dvbs2_r2_3", "dvbs2_r8_9", "dvbs2_r9_10"),
}
MIXED_EBN0 = {"dvbs2_r1_2": 1.0, "dvbs2_r2_3": 2.2, "dvbs2_r8_9": 4.6, "dvbs2_r9_10": 5.0,
              "dvbs2shape_r3_4": 2.8, "dvbs2shape_r5_6": 3.5}


def cpu_baseline_mixed(names, frames, iters, budget_s, threads, seed):
    """configs[4] on the host, every rate MEASURED (code/x86/main_p.cpp:664-765's
    timer mode: the same resident LLRs decoded again and again), at FIXED
    `iters` iterations (code/x86's decoder has no early termination: its
    arret test is commented out, CDecoder_OMS_fixed_SSE.cpp:551-553), budget_s
    / len(names) seconds per rate on `threads` threads:
    * rates the reference can be built for (oracle/_ref: r1/2, r8/9, r9/10):
      the reference's own SSE decoder, 16-frame decode() calls (kind
      "reference");
    * the others (r2/3, the DVB-S2-shaped r3/4 and r5/6: no constantes_sse.h
      in code/x86): the product's own host decoder (a device -1 context,
      csrc/host.cpp, 32-codeword AVX2 blocks; kind "product-host") -- the
      reference cannot decode them at all.
    The step's host time = sum over rates of frames / measured rate."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from ldpcgputegra_amd import Code, Decoder, channel, load_table
    per_rate, tot = [], 0.0
    old_threads = os.environ.get("LDPC_HOST_THREADS")
    for name, f in zip(names, frames):
        t = load_table(name)
        llr_table = channel.i8_table(channel.sigma_from_ebn0(MIXED_EBN0.get(name, 3.0), t.k_info / t.n))
        budget = budget_s / len(names)
        if O.ref_available(name):
            kind, blk = "reference", 16 * threads
            llr = channel.awgn_i8_host(t.n, blk, seed, llr_table)
            O.ref_decode_mt(name, llr, iters, 1, threads)   # untimed: library load, first touch, thread start
            run = lambda: O.ref_decode_mt(name, llr, iters, 1, threads)   # noqa: E731
            dec = None
        else:
            kind, blk = "product-host", 32 * threads
            os.environ["LDPC_HOST_THREADS"] = str(threads)
            llr = channel.awgn_i8_host(t.n, blk, seed, llr_table)
            dec = Decoder(Code(name), device=-1, max_batch=blk)
            dec.decode_i8(llr[:32], 1)                       # untimed: first touch
            run = lambda: dec.decode_i8(llr, iters)         # noqa: E731
        done, t0 = 0, time.perf_counter()
        while True:
            run()
            done += blk
            el = time.perf_counter() - t0
            if el >= budget:
                break
        if dec is not None:
            dec.close()
        cw_s = done / el
        tot += f / cw_s
        per_rate.append(dict(code=name, kind=kind, codewords_per_s=round(cw_s, 1), mbps=round(cw_s * t.n / 1e6, 3),
                             sample="%d codewords in %.2f s" % (done, el)))
    if old_threads is None:
        os.environ.pop("LDPC_HOST_THREADS", None)
    else:
        os.environ["LDPC_HOST_THREADS"] = old_threads
    host = host_cpu_info()
    n = load_table(names[0]).n
    kinds = sorted({r["kind"] for r in per_rate})
    return dict(value=round(sum(frames) * n / tot / 1e6, 3), unit="Mbit/s", cores=threads,
                kind="reference" if kinds == ["reference"] else "port", kinds=kinds,
                threads=threads, cpu_model=host["model"], host_physical_cores=host["physical_cores"],
                cpu_quota=host["cpu_quota"], per_rate=per_rate,
                sample="every rate measured at fixed %d iterations (no early termination in code/x86) on %d threads, "
                       "~%.1f s per rate: the reference SSE decoder (16-frame decode() calls) for %s; the product's "
                       "host decoder (device -1 context, 32-codeword blocks) for %s, which code/x86 has no table for; "
                       "step host time = sum of frames / measured rate" % (
                           iters, threads, budget_s / len(names),
                           ", ".join(r["code"] for r in per_rate if r["kind"] == "reference") or "none",
                           ", ".join(r["code"] for r in per_rate if r["kind"] != "reference") or "none"))


def bench_mixed(a, rank, world, local, torch, dist):
    """configs[4]: one batch of B codewords per GPU mixing DVB-S2 normal-frame
    rates (MIXED_SETS[a.mixed_codes]), codeword c using rate c % len(codes),
    each rate at its own Eb/N0 (MIXED_EBN0), int8 OMS with early termination
    (per-codeword syndrome after every iteration), at most a.iters iterations.  A step = the mixed decode of the whole batch
    (per-rate gather, concurrent per-rate decodes on their own streams,
    scatter) with LLRs resident in HBM."""
    import numpy as np
    from ldpcgputegra_amd import Code, channel, default_params
    from ldpcgputegra_amd.decoder import Decoder, MixedDecoder
    from ldpcgputegra_amd.shard import mixed_layout, reduce_results, reduce_sums
    B = a.batch
    names = MIXED_SETS[a.mixed_codes]
    codes = [Code(n) for n in names]
    N = codes[0].n
    mx = MixedDecoder(codes, device=local, max_batch=B)
    # global codeword g = rank * B + i has rate g % len(codes); rate c's noise
    # indices are disjoint across ranks and rates (shard.mixed_layout), so N
    # ranks decode exactly the codewords one process decodes at batch N * B
    ids, noise_first = mixed_layout(rank, world, B, len(codes))
    llr = torch.empty((B, N), dtype=torch.int8, device="cuda")
    for c, code in enumerate(codes):      # all-zero codeword per rate (CFakeEncoder), own channel
        sel = torch.from_numpy(np.where(ids == c)[0]).cuda()
        if sel.numel() == 0:
            continue
        tmp = torch.empty((sel.numel(), N), dtype=torch.int8, device="cuda")
        gen = Decoder(code, device=local, max_batch=max(1, sel.numel()))
        table = channel.i8_table(channel.sigma_from_ebn0(MIXED_EBN0[code.name], code.k_info / code.n), 8, 31)
        gen.awgn_i8_device(tmp, first_cw=noise_first[c], seed=a.seed, table=table)
        llr[sel] = tmp
        gen.close()
    hard = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    its = torch.empty(B, dtype=torch.int32, device="cuda")
    params = default_params(early_term=1)

    def step():
        mx.decode_i8_device(llr, hard, ids, a.iters, params=params, iters_used=its)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    mx.kernel_time(reset=True)
    mx.profile(True)   # HIP events around each code's decode launch (on its own stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    kt = mx.kernel_time(reset=True)
    mx.profile(False)
    h, it = hard.cpu().numpy(), its.cpu().numpy()
    # per rate over ALL ranks: frames, bit errors, frame errors, iterations,
    # algorithmic bytes (sums) and the decode launch time (max)
    sums = []
    for c, code in enumerate(codes):
        sel = ids == c
        e = h[sel][:, :code.k_info].sum(axis=1)          # all-zero codeword: every 1 is an error
        sums += [int(sel.sum()), int(e.sum()), int((e > 0).sum()), int(it[sel].sum()),
                 float((4.0 * code.e * it[sel] + 2.0 * N).sum())]
    sums = reduce_sums(sums, device="cuda")
    kms = [kt[c][0] / kt[c][1] if kt[c][1] else 0.0 for c in range(len(codes))]
    kms_max = [reduce_results(k, 0, 0, 0, device="cuda")[0] for k in kms]
    per_rate, alg_bytes, be_tot, fe_tot, bits = [], 0.0, 0, 0, 0
    for c, code in enumerate(codes):
        fr, be_c, fe_c, it_c, ab_c = sums[5 * c:5 * c + 5]
        fr = int(fr)
        per_rate.append(dict(code=code.name, ebn0_db=MIXED_EBN0[code.name], frames=fr,
                             avg_iters=it_c / max(fr, 1), ber=be_c / max(fr * code.k_info, 1),
                             fer=fe_c / max(fr, 1),
                             kernel=mx.last_kernels()[c],
                             et_first_stage=mx.last_et_stages()[c],   # > 0: staged early termination (coop3)
                             kernel_ms=round(kms_max[c], 4) if kms_max[c] else None))
        alg_bytes += ab_c
        be_tot += int(be_c)
        fe_tot += int(fe_c)
        bits += fr * code.k_info
    el, _, _, _ = reduce_results(el, 0, 0, 0, device="cuda")
    if rank == 0:
        frames = world * B * a.steps
        value = frames * N / el / 1e6
        achieved = alg_bytes * a.steps / el / 1e9
        out = {
            "metric": "decoded Mbit/s, configs[4]: mixed-rate DVB-S2 (%s) int8 + early termination"
                      % ", ".join(n.split("_", 1)[1].replace("_", "/") for n in names),
            "value": round(value, 3), "unit": "Mbit/s", "n_gpus": world,
            "ranks_seen": dist.get_world_size() if dist.is_initialized() else 1, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            # per 4096 codewords: comparable with the fixed-50 configs[2] step at batch 4096
            "ms_per_4096_codewords": round(el / a.steps * 1e3 * 4096 / B, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int8",
            "data": "synthetic (device AWGN generator, all-zero codeword per rate)" + (
                "; r3/4 and r5/6 are DVB-S2-shaped stand-ins (Annex-B structure, seeded random addresses: "
                "tools/make_dvbs2_shaped.py), not the ETSI tables" if a.mixed_codes == "configs4" else ""),
            "config": {"workload": "mixed-rate DVB-S2 N=64800 batch %d per GPU, <= %d iters, early termination"
                                   % (B, a.iters), "codes": list(names), "batch_per_gpu": B,
                       "global_batch": B * world, "iters_max": a.iters, "code_set": a.mixed_codes,
                       "parallelism": "codeword shards x%d (no collective)" % world},
            "per_rate": per_rate,
            "ber": be_tot / max(bits, 1), "fer": fe_tot / max(world * B, 1),
            # whole-step rate (several kernels on concurrent streams): no single dominant launch;
            # traffic = HBM bytes per step over all its kernels (PMC, profiles/traffic.json)
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": hbm_peak_gbs(), "unit": "GB/s",
                         "frac": round(achieved / hbm_peak_gbs(), 4), "traffic": None,
                         # the longest per-rate decode launch (they run concurrently; per_rate has each)
                         "kernel_ms": max((r["kernel_ms"] for r in per_rate if r["kernel_ms"]), default=None),
                         "algorithmic_bytes_per_step": alg_bytes},
            "cpu_baseline": None,
        }
        src = source_hash()
        out["build"] = {"src_sha16": src}
        try:
            tr = json.load(open(a.traffic_file))
            ent = tr.get("mixed_%s_b%d_it%d" % (a.mixed_codes, B, a.iters), {})
            if ent.get("src_sha16") == src:
                out["roofline"]["traffic"] = ent.get("hbm_bytes_per_step")
        except (OSError, ValueError):
            pass
        if world == 1 and a.cpu_seconds > 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            out["cpu_baseline"] = cpu_baseline_mixed(list(names), [r["frames"] for r in per_rate], a.iters,
                                                     a.cpu_seconds, a.cpu_threads or O.host_threads(), a.seed)
        print(json.dumps(out), flush=True)
    mx.close()


def launch_ranks(a):
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launcher:
    start one as a CHILD process -- before this process has touched the GPU
    (no torch import yet) -- with N ranks on 127.0.0.1, rank 0's JSON line
    passing through on the shared stdout, and return its exit status."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    sys.stdout.flush()
    return subprocess.run(cmd, env=dict(os.environ, MASTER_ADDR="127.0.0.1")).returncode


def rank_list(value, world, dist):
    """[value of rank 0, ..., value of rank world-1] (any backend)."""
    if world == 1:
        return [value]
    out = [None] * world
    dist.all_gather_object(out, value)
    return out


def main():
    a = parse()
    if a.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        sys.exit("bench.py: WORLD_SIZE=%d but --gpus %d" % (world, a.gpus))
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # "gloo" rehearses N ranks on fewer GPUs (ranks share devices round-robin);
    # the driver's runs use RCCL ("nccl"), one GPU per rank
    backend = os.environ.get("LDPC_BENCH_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    elif world > torch.cuda.device_count():
        sys.exit("bench.py: %d ranks but %d visible GPUs (LDPC_BENCH_BACKEND=gloo shares devices)"
                 % (world, torch.cuda.device_count()))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    if a.mixed:
        bench_mixed(a, rank, world, local, torch, dist)
        if world > 1:
            dist.destroy_process_group()
        return

    from ldpcgputegra_amd import ALGO_MS, Code, Decoder, channel, default_params
    from ldpcgputegra_amd.shard import reduce_results, shard_range
    code = Code(a.code)
    dec = Decoder(code, device=local, max_batch=a.batch, kernel=a.kernel)
    B, N = a.batch, code.n
    sigma = channel.sigma_from_ebn0(a.ebn0, code.k_info / code.n)
    table = channel.i8_table(sigma, 8, 31)
    f32 = a.dtype == "f32"
    hard = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    counts = torch.zeros(2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    first_cw, _ = shard_range(rank, world, B * world)      # contiguous shard per rank
    if f32:
        # float BPSK channel output y = -1 + sigma n of the all-zero codeword
        # (positive LLR <-> bit 1, code/x86/CChanel/CChanelAWGN_MKL.cpp:139), used
        # directly as the decoder input (no 2/sigma^2 scaling, as the reference)
        g = torch.Generator(device="cuda").manual_seed(a.seed * 1000003 + first_cw)
        llr = -1.0 + sigma * torch.randn((B, N), generator=g, device="cuda", dtype=torch.float32)
        params = default_params(algo=ALGO_MS, beta=0.0)
    else:
        llr = torch.empty((B, N), dtype=torch.int8, device="cuda")
        dec.awgn_i8_device(llr, first_cw=first_cw, seed=a.seed, table=table, stream=stream)
        params = default_params()
    def step():   # decode + error count (fused into the float kernel's epilogue; int8: a count launch after)
        dec.decode_count_device(llr, hard, a.iters, code.k_info, counts, params=params, stream=stream)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    counts.zero_()
    # The kernel's average launch duration, from HIP events over the timed
    # region.  When a step is ONE launch (the float edge-parallel kernel, error
    # count fused into its epilogue) a single event pair brackets the whole
    # region: per-launch event pairs cost ~7.5 us of GPU time per 46 us step
    # (profiles/r06l_f32_events.txt), which would inflate the step they time.
    # Otherwise (int8: decode + count launches) an event pair per decode launch.
    region = f32 and dec.last_kernel == "ldsep"
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    dec.profile(not region)
    dec.kernel_time(reset=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(a.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = el_local = time.perf_counter() - t0
    kms, launches = dec.kernel_time(reset=True)
    dec.profile(False)
    if region:
        kms, launches = ev0.elapsed_time(ev1), a.steps

    be_l, fe_l = counts.tolist()
    el, be, fe, _ = reduce_results(el, be_l, fe_l, B * a.steps, device="cuda")
    kernel_ms, _, _, _ = reduce_results(kms / max(launches, 1), 0, 0, 0, device="cuda")
    per_rank = rank_list({"device": local, "kernel_ms": round(kms / max(launches, 1), 4),
                          "elapsed_s": round(el_local, 6)}, world, dist)
    ranks_seen = dist.get_world_size() if dist.is_initialized() else 1

    if rank == 0:
        frames = world * B * a.steps
        value = frames * N / el / 1e6
        E = code.e
        if f32:   # SURVEY.md 8(d), per launch: f32 msg rd+wr, V rd+wr per edge; f32 llr in, u8 hard out
            alg_bytes = B * (16.0 * E * a.iters + 5.0 * N)
        else:
            alg_bytes = B * (4.0 * E * a.iters + 2.0 * N)
        achieved = alg_bytes / (kernel_ms * 1e-3) / 1e9     # GB/s
        peak = hbm_peak_gbs()
        # PMC traffic of this exact build: profiles/traffic.json entries carry
        # the source hash of the library they were measured on (tools/
        # summarize_profiles.py); a different build gets null, not a stale number
        traffic, traffic_note = None, None
        src = source_hash()
        try:
            tr = json.load(open(a.traffic_file))
            key = "%s_b%d_it%d_%s" % (a.code, B, a.iters, dec.last_kernel)
            ent = tr.get(key, {})
            if ent.get("src_sha16") == src:
                traffic = ent.get("hbm_bytes_per_launch")
                traffic_note = "PMC FETCH/WRITE passes on this build: %s" % ent.get("source")
            elif ent:
                traffic_note = ("no PMC pass for this build (src %s); last measured on src %s: %s"
                                % (src, ent.get("src_sha16"), ent.get("source")))
        except (OSError, ValueError):
            pass
        out = {
            "metric": (("decoded Mbit/s, configs[1]: %s float min-sum, %d iters" if a.code == "648x324" else
                        "decoded Mbit/s, %s float min-sum, %d iters") % (a.code, a.iters) if f32 else
                       "decoded Mbit/s + BER@SNR, DVB-S2 N=64800 r=1/2, 50 iters, 1/2/4/8 MI355X"),
            "value": round(value, 3),
            "unit": "Mbit/s",
            "n_gpus": world,
            "ranks_seen": ranks_seen,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32" if f32 else "int8",
            "data": "synthetic (device AWGN generator, all-zero codeword, Eb/N0 %.2f dB)" % a.ebn0,
            "config": {
                "workload": ("%s layered float min-sum, %d iters, batch %d codewords per GPU" % (a.code, a.iters, B)
                             if f32 else
                             "%s layered int8 offset-min-sum (offset 1), %d iters, batch %d codewords per GPU"
                             % (a.code, a.iters, B)),
                "code": a.code, "batch_per_gpu": B, "global_batch": B * world, "iters": a.iters,
                "ebn0_db": a.ebn0, "kernel": dec.last_kernel,
                "parallelism": "codeword shards x%d (no collective)" % world,
            },
            "ber": be / max(frames * code.k_info, 1),
            "fer": fe / max(frames, 1),
            "info_mbps": round(value * code.k_info / N, 3),
            "roofline": {
                "bound": "hbm", "achieved": round(achieved, 2), "peak": peak, "unit": "GB/s",
                "frac": round(achieved / peak, 4), "traffic": traffic, "traffic_source": traffic_note,
                "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": alg_bytes,
            },
            "build": {"src_sha16": src},
        }
        if dec.last_kernel == "coop3":
            # priced against HBM as the contract asks; what limits the kernel is
            # the per-period issue and latency of its slab, chain and memory
            # waves (cycle stamps and SQ counters)
            out["roofline"]["note"] = ("HBM is not the limiter: real traffic (PMC) is ~0.66x the algorithmic bytes "
                                       "at ~3.5 TB/s; the period is set by VALU issue + LDS latency of the slab "
                                       "waves, the chain wave's serial steps and the memory wave's issue")
        if dec.last_kernel == "stairf":
            out["roofline"]["note"] = ("float staircase kernel: HBM-bound once the chip is full (16384 codewords at "
                                       "width 2: 4.73 TB/s of real traffic); below that per-wave VALU issue and the "
                                       "chain's dependent steps (DESIGN.md, stairf)")
        if dec.last_kernel in ("lds", "ldsep"):
            # the LDS-resident kernel keeps V and the messages in LDS: HBM sees
            # only LLRs in / hard decisions out (the measured traffic), so the
            # algorithmic bytes are LDS bytes, priced against the LDS array's
            # peak (256 B/clk/CU, MI355X_MICROARCH.md "LDS"); what bounds it is
            # the latency of each layer's dependent LDS round trips at one
            # wave per SIMD (lds kernel)
            lds_peak = lds_peak_gbs()
            out["roofline"] = {
                "bound": "lds", "achieved": round(achieved, 2), "peak": lds_peak, "unit": "GB/s",
                "frac": round(achieved / lds_peak, 4), "traffic": traffic, "traffic_source": traffic_note,
                "hbm_achieved": round(traffic / (kernel_ms * 1e-3) / 1e9, 2) if traffic else None,
                "kernel_ms": round(kernel_ms, 4), "algorithmic_bytes_per_launch": alg_bytes,
                "kernel_ms_source": ("one HIP event pair over the timed region / launches (one launch per step)"
                                     if region else "HIP event pair per decode launch, averaged"),
                "note": ("algorithmic bytes are on-chip traffic (V in LDS, messages in VGPRs: neither leaves the CU); "
                         "bound in practice: VALU issue at one wave per SIMD (DPP butterflies per check, DESIGN.md)"
                         if dec.last_kernel == "ldsep" else
                         "algorithmic bytes are LDS traffic (V and messages never leave LDS); bound in practice: "
                         "dependent LDS round trips per layer at one wave per SIMD (latency, not bandwidth)"),
            }
        if world == 1 and a.cpu_seconds > 0:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle as O
            thr = a.cpu_threads or O.host_threads()
            out["cpu_baseline"] = (cpu_baseline_f32(a.code, a.iters, a.cpu_seconds, thr, a.seed) if f32 else
                                   cpu_baseline(a.code, a.iters, a.cpu_seconds, thr, a.seed))
            if not f32:   # beside the reference: the product's own host decoder (device -1)
                out["cpu_baseline_product_host"] = cpu_baseline_product_host(a.code, a.iters, a.cpu_seconds * 0.5,
                                                                             thr, a.seed)
        else:
            out["cpu_baseline"] = None
        if world > 1:   # one entry per rank: its device and its own decode-kernel time
            out["per_rank"] = per_rank
            out["backend"] = backend
        if dec.last_skipped:   # a faster kernel did not apply to these parameters
            out["config"]["kernel_skipped"] = dec.last_skipped
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
