"""BASELINE configs[3] (DVB-S2 r1/2, batch 32768 split across 8 MI355X as
independent codeword shards) exercised as far as one MI355X allows.

SURVEY.md §8(e): the path shards embarrassingly -- 8 contiguous ranges of 4096
codewords, every GPU regenerating its own LLRs from (seed, first codeword),
no collective.  The reference has no multi-GPU path (its concurrency model is
several decoder objects on their own streams, code/gpu_fixed/test.cpp:347-393,
paper/ldpcGpuTegra.tex:279-289), so what must hold is shard invariance:

* the 32768-codeword batch decoded as 8 shards on 8 separate decoder contexts
  (one per would-be GPU, inputs regenerated per shard exactly as bench.py's
  ranks do) equals the same batch decoded as ONE 32768-codeword coop3 launch,
  bit for bit (hard decisions and final V);
* one shard equals the reference's own SSE decoder (oracle/_ref,
  code/x86/CDecoder/OMS/CDecoder_OMS_fixed_SSE.cpp:114-574) on every bit;
* bench.py --gpus 8 (gloo, the 8 ranks sharing the one device) reports 8 ranks
  and the BER / FER of one process decoding the same 4096 codewords.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as O
from ldpcgputegra_amd import Code, Decoder, channel, load_table

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SHARDS, SHARD_B, ITERS, SEED = 8, 4096, 50, 2024


def _torch():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_configs3_eight_shards_equal_one_launch_and_reference():
    torch = _torch()
    from ldpcgputegra_amd.shard import shard_range
    t = load_table("dvbs2_r1_2")
    code = Code("dvbs2_r1_2")
    total = SHARDS * SHARD_B
    table = channel.i8_table(channel.sigma_from_ebn0(1.0, t.k_info / t.n), 8, 31)
    # one launch over the whole batch (LLRs from one generator call)
    big = Decoder(code, max_batch=total)
    llr = torch.empty((total, t.n), dtype=torch.int8, device="cuda")
    big.awgn_i8_device(llr, first_cw=0, seed=SEED, table=table)
    h_all = torch.empty((total, t.n), dtype=torch.uint8, device="cuda")
    s_all = torch.empty((total, t.n), dtype=torch.int8, device="cuda")
    big.decode_i8_device(llr, h_all, ITERS, soft=s_all)
    torch.cuda.synchronize()
    assert big.last_kernel == "coop3"
    big.close()
    # 8 shards on 8 contexts, each regenerating its own inputs (bench.py's ranks)
    h_sh = torch.empty_like(h_all)
    s_sh = torch.empty_like(s_all)
    decs = []
    for r in range(SHARDS):
        first, count = shard_range(r, SHARDS, total)
        assert (first, count) == (r * SHARD_B, SHARD_B)
        d = Decoder(code, max_batch=count)
        x = torch.empty((count, t.n), dtype=torch.int8, device="cuda")
        d.awgn_i8_device(x, first_cw=first, seed=SEED, table=table)
        assert torch.equal(x, llr[first:first + count])         # same inputs as the one-launch batch
        d.decode_i8_device(x, h_sh[first:first + count], ITERS, soft=s_sh[first:first + count])
        decs.append(d)
    torch.cuda.synchronize()
    assert all(d.last_kernel == "coop3" for d in decs)
    assert torch.equal(h_sh, h_all)
    assert torch.equal(s_sh, s_all)
    # whole-job error counts (info bits of the all-zero codeword) as bench.py reports them
    be = int(h_all[:, :t.k_info].sum(dtype=torch.int64))
    fe = int((h_all[:, :t.k_info].sum(dim=1, dtype=torch.int64) > 0).sum())
    assert 0 < fe < total // 50, (be, fe)
    # one shard (the last: codewords 28672 .. 32767) against the reference itself
    first = (SHARDS - 1) * SHARD_B
    host_llr = llr[first:].cpu().numpy()
    got = h_all[first:].cpu().numpy()
    thr = O.host_threads()
    if O.ref_available("dvbs2_r1_2"):
        exp = O.ref_decode_mt("dvbs2_r1_2", host_llr, ITERS, 1, thr)
    else:
        exp = O.decode_i8(t, host_llr, ITERS, threads=thr)
    diff = np.nonzero((got != exp).any(axis=1))[0]
    assert diff.size == 0, "codewords differing from the reference: %s" % diff[:16]
    for d in decs:
        d.close()


def _bench_json(args, env):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                         timeout=600, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


def test_configs3_eight_rank_gloo_rehearsal():
    """`python bench.py --gpus 8` exactly as the driver starts it (bench.py
    launches torch.distributed.run itself), gloo backend so the 8 ranks can
    share the box's one MI355X, 512 codewords per rank at 50 iterations: 8
    ranks seen, 8 per-rank entries, and whole-job BER / FER equal to one
    process decoding the same 4096 codewords."""
    env = dict(os.environ, LDPC_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    common = ["--iters", str(ITERS), "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"]
    eight = _bench_json(["--gpus", "8", "--batch", "512"] + common, env)
    one = _bench_json(["--batch", "4096"] + common, {k: v for k, v in env.items()})
    assert eight["n_gpus"] == 8 and eight["ranks_seen"] == 8 and eight["backend"] == "gloo"
    assert len(eight["per_rank"]) == 8 and all(r["kernel_ms"] > 0 for r in eight["per_rank"])
    assert eight["config"]["global_batch"] == 4096 == one["config"]["global_batch"]
    assert eight["config"]["kernel"] == "coop3" == one["config"]["kernel"]
    assert one["fer"] > 0
    assert eight["ber"] == one["ber"] and eight["fer"] == one["fer"]
