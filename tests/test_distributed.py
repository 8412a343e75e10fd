"""N > 1 path on the CPU: world_size-2 gloo processes shard a batch of
codewords exactly as bench.py does (contiguous shards, inputs regenerated from
(seed, first codeword)), decode their shard with the PRODUCT decoder on the
host (a device -1 context of the C-ABI: csrc/host.cpp, the drop-in on a
machine without a GPU), and reduce only counters and time.  Shard invariance:
the union of the shards equals the oracle's single-process decode bit for
bit (the oracle is only the checker here)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from ldpcgputegra_amd.shard import reduce_results, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_dir):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path.insert(0, root)
    import torch.distributed as dist
    from ldpcgputegra_amd import Code, Decoder, channel, load_table
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = load_table("576x288")
    table = channel.i8_table(channel.sigma_from_ebn0(1.5, 0.5))
    first, count = shard_range(rank, world, total)
    llr = channel.awgn_i8_host(t.n, count, seed=9, table=table, first_cw=first)
    dec = Decoder(Code("576x288"), device=-1, max_batch=count)   # product host decoder, one context per rank
    hard = dec.decode_i8(llr, 10)
    assert dec.last_kernel == "host"
    dec.close()
    be = int(hard[:, :t.k_info].sum())
    fe = int((hard[:, :t.k_info].sum(axis=1) > 0).sum())
    el, BE, FE, FR = reduce_results(0.1 * (rank + 1), be, fe, count)
    np.save(os.path.join(out_dir, "hard_%d.npy" % rank), hard)
    np.save(os.path.join(out_dir, "red_%d.npy" % rank), np.array([el, BE, FE, FR]))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_batch():
    for total in (1, 7, 4096, 32768):
        for world in (1, 2, 3, 8):
            got = [shard_range(r, world, total) for r in range(world)]
            assert got[0][0] == 0
            for (f, c), (f2, _) in zip(got, got[1:]):
                assert f + c == f2
            assert sum(c for _, c in got) == total
            assert max(c for _, c in got) - min(c for _, c in got) <= 1


def test_two_rank_gloo_shards_match_single_process(tmp_path):
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import oracle as O
    from ldpcgputegra_amd import channel, load_table
    total = 10
    mp.start_processes(_worker, args=(2, _free_port(), total, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    hard = np.concatenate([np.load(tmp_path / ("hard_%d.npy" % r)) for r in range(2)])
    t = load_table("576x288")
    table = channel.i8_table(channel.sigma_from_ebn0(1.5, 0.5))
    ref = O.decode_i8(t, channel.awgn_i8_host(t.n, total, seed=9, table=table), 10)
    assert np.array_equal(hard, ref)
    red = [np.load(tmp_path / ("red_%d.npy" % r)) for r in range(2)]
    assert np.array_equal(red[0], red[1])                   # every rank sees the reduced values
    el, be, fe, fr = red[0]
    assert el == pytest.approx(0.2)                         # max over ranks
    assert fr == total and be == ref[:, :t.k_info].sum()


@pytest.mark.gpu
def test_two_rank_bench_on_gpu_matches_single_process():
    """bench.py's N > 1 path on hardware: torch.distributed.run with 2 ranks
    (gloo, both on the box's one MI355X, LDPC_BENCH_BACKEND=gloo as the
    driver's 8-GPU runs use RCCL), 256 DVB-S2 r1/2 codewords per rank, each
    rank decoding its own contiguous shard on its own decoder context.  The
    JSON line reports n_gpus 2 and whole-job BER / FER equal to one process
    decoding the same 512 codewords (the shards cover exactly those)."""
    import json
    import subprocess
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    args = ["--batch", "256", "--iters", "10", "--steps", "2", "--warmup", "1", "--cpu-seconds", "0"]
    env = dict(os.environ, LDPC_BENCH_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    # plain `python bench.py --gpus 2`, as the driver runs it: bench.py starts
    # torch.distributed.run itself (a child process, before any GPU call)
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"] + args,
                         capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-2000:]
    two = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    args[1] = "512"
    out1 = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, capture_output=True, text=True,
                          timeout=300, cwd=root)
    assert out1.returncode == 0, out1.stderr[-2000:]
    one = json.loads([l for l in out1.stdout.splitlines() if l.startswith("{")][-1])
    assert two["n_gpus"] == 2 and two["config"]["global_batch"] == 512 and one["config"]["global_batch"] == 512
    assert two["ranks_seen"] == 2 and len(two["per_rank"]) == 2 and all(r["kernel_ms"] > 0 for r in two["per_rank"])
    assert one["n_gpus"] == 1 and one["ranks_seen"] == 1
    assert two["ber"] == one["ber"] and two["fer"] == one["fer"] and one["fer"] > 0
    assert two["value"] > 0


def test_bench_rank_count_checks():
    """bench.py refuses a rank count it cannot honour instead of silently
    decoding on fewer GPUs: WORLD_SIZE != --gpus, and more nccl ranks than
    visible devices (here: none) -- both exit non-zero before any decode."""
    import subprocess
    import sys
    root = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
    bench = os.path.join(root, "bench.py")
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, bench, "--gpus", "1", "--cpu-seconds", "0"], capture_output=True,
                         text=True, timeout=120, env=env, cwd=root)
    assert out.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in out.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["LDPC_BENCH_BACKEND"] = "nccl"
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    out = subprocess.run([sys.executable, bench, "--gpus", "2", "--cpu-seconds", "0"], capture_output=True,
                         text=True, timeout=300, env=env, cwd=root)
    assert out.returncode != 0 and "2 ranks but 0 visible GPUs" in out.stderr
