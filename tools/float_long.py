"""Float decode time of the long staircase codes (DVB-S2) per kernel.

python tools/float_long.py [codes] -- prints one JSON line per (code, batch,
kernel): decode-kernel ms per launch (HIP events, ldpc_ctx_profile), info
Mbit/s.  Kernel 11 = stairf (float staircase), 1 = generic.  WIDTHS=4,8,16 (group widths),
BATCHES=1024,4096, ITERS=20, GENERIC=1 adds one generic-kernel line.
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpcgputegra_amd import ALGO_MS, Code, Decoder, channel, default_params  # noqa: E402


def run(code, batch, kernel, iters, reps, width=None):
    if width:
        os.environ["LDPC_STAIRF_S"] = str(width)
    c = Code(code)
    dec = Decoder(c, max_batch=batch, kernel=kernel)
    rng = np.random.default_rng(1)
    sigma = channel.sigma_from_ebn0(1.0, c.k_info / c.n)
    llr = torch.from_numpy((-1.0 + sigma * rng.standard_normal((batch, c.n))).astype(np.float32)).cuda()
    hard = torch.empty((batch, c.n), dtype=torch.uint8, device="cuda")
    p = default_params(algo=ALGO_MS)
    dec.decode_f32_device(llr, hard, iters, params=p)
    torch.cuda.synchronize()
    dec.profile(True)
    dec.kernel_time(reset=True)
    for _ in range(reps):
        dec.decode_f32_device(llr, hard, iters, params=p)
    torch.cuda.synchronize()
    ms, n = dec.kernel_time(reset=True)
    ms /= max(n, 1)
    ber = float((hard.cpu().numpy()[:, : c.k_info] != 0).mean())
    print(json.dumps(dict(code=code, batch=batch, kernel=dec.last_kernel, width=width, iters=iters,
                          kernel_ms=round(ms, 4),
                          info_mbit_s=round(batch * c.k_info / ms / 1e3, 1), ber=ber)), flush=True)


if __name__ == "__main__":
    codes = sys.argv[1:] or ["dvbs2_r1_2"]
    iters = int(os.environ.get("ITERS", 20))
    widths = [int(w) for w in os.environ.get("WIDTHS", "8").split(",")]
    batches = [int(b) for b in os.environ.get("BATCHES", "1024,4096").split(",")]
    for code in codes:
        for batch in batches:
            for w in widths:
                run(code, batch, 11, iters, 3, w)
    if os.environ.get("GENERIC"):
        run(codes[0], 1024, 1, iters, 1)
