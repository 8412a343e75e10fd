"""Debug (GPU box): configs[1] step time with and without the per-launch HIP
events bench.py records (the float kernel is ~0.05 ms, so launch gaps matter)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from ldpcgputegra_amd import ALGO_MS, Code, Decoder, channel, default_params  # noqa: E402

code = Code("648x324")
B, it = 1024, 20
dec = Decoder(code, device=0, max_batch=B)
sigma = channel.sigma_from_ebn0(1.0, code.k_info / code.n)
g = torch.Generator(device="cuda").manual_seed(1)
llr = -1.0 + sigma * torch.randn((B, code.n), generator=g, device="cuda", dtype=torch.float32)
hard = torch.empty((B, code.n), dtype=torch.uint8, device="cuda")
counts = torch.zeros(2, dtype=torch.int64, device="cuda")
p = default_params(algo=ALGO_MS, beta=0.0)
stream = torch.cuda.current_stream().cuda_stream
for ev in (True, False, True, False):
    dec.profile(ev)
    for _ in range(20):
        dec.decode_count_device(llr, hard, it, code.k_info, counts, params=p, stream=stream)
    torch.cuda.synchronize()
    dec.kernel_time(reset=True)
    K = 400
    t0 = time.perf_counter()
    for _ in range(K):
        dec.decode_count_device(llr, hard, it, code.k_info, counts, params=p, stream=stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    ms, n = dec.kernel_time(reset=True)
    print("events %s: %.4f ms per step, kernel %s ms" % (ev, el / K * 1e3, round(ms / n, 4) if n else None), flush=True)
    # host issue cost alone (no GPU wait): time to enqueue K steps
    t0 = time.perf_counter()
    for _ in range(K):
        dec.decode_count_device(llr, hard, it, code.k_info, counts, params=p, stream=stream)
    el_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    print("   host enqueue %.4f ms per step" % (el_issue / K * 1e3), flush=True)
