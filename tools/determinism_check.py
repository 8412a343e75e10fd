"""Run-to-run determinism of the configs[4] mixed-rate decode (GPU box).

Builds bench.py --mixed's input batch (same seed, rates and Eb/N0), then
decodes it several times through MixedDecoder and, per rate, through a plain
Decoder on the rate's contiguous sub-batch, with early termination; prints
per-rate hashes of hard decisions / iterations used so a run-to-run or
mixed-vs-single difference shows which path varies.
usage: python tools/determinism_check.py [reps]
"""
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from bench import MIXED_CODES, MIXED_EBN0  # noqa: E402
from ldpcgputegra_amd import Code, channel, default_params  # noqa: E402
from ldpcgputegra_amd.decoder import Decoder, MixedDecoder  # noqa: E402


def h(t):
    return hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()[:12]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    B, seed, iters = 4096, 2024, 50
    codes = [Code(n) for n in MIXED_CODES]
    N = codes[0].n
    ids = np.arange(B, dtype=np.int32) % len(codes)
    llr = torch.empty((B, N), dtype=torch.int8, device="cuda")
    subs = []
    for c, code in enumerate(codes):
        sel = torch.from_numpy(np.where(ids == c)[0]).cuda()
        tmp = torch.empty((sel.numel(), N), dtype=torch.int8, device="cuda")
        gen = Decoder(code, device=0, max_batch=sel.numel())
        table = channel.i8_table(channel.sigma_from_ebn0(MIXED_EBN0[code.name], code.k_info / code.n), 8, 31)
        gen.awgn_i8_device(tmp, first_cw=c * B, seed=seed, table=table)
        llr[sel] = tmp
        subs.append((sel, tmp.clone()))
        gen.close()
    torch.cuda.synchronize()
    params = default_params(early_term=1)
    mx = MixedDecoder(codes, device=0, max_batch=B)
    hard = torch.empty((B, N), dtype=torch.uint8, device="cuda")
    its = torch.empty(B, dtype=torch.int32, device="cuda")
    for r in range(reps):
        hard.zero_()
        mx.decode_i8_device(llr, hard, ids, iters, params=params, iters_used=its)
        torch.cuda.synchronize()
        row = []
        for c, (sel, _) in enumerate(subs):
            row.append("%s:%s/%s it=%.3f" % (codes[c].name[6:], h(hard[sel]), h(its[sel]),
                                            its[sel].float().mean().item()))
        print("mixed  rep %d  " % r + "  ".join(row), flush=True)
    for c, (sel, x) in enumerate(subs):
        dec = Decoder(codes[c], device=0, max_batch=x.shape[0])
        for p_name, p in (("early", params), ("fixed", default_params())):
            for r in range(reps):
                hh = torch.empty((x.shape[0], N), dtype=torch.uint8, device="cuda")
                ii = torch.zeros(x.shape[0], dtype=torch.int32, device="cuda")
                dec.decode_i8_device(x, hh, iters, params=p, iters_used=ii)
                torch.cuda.synchronize()
                print("single %s %s rep %d kernel %s: %s/%s it=%.3f" % (codes[c].name, p_name, r, dec.last_kernel,
                                                                    h(hh), h(ii), ii.float().mean().item()),
                      flush=True)
        dec.close()
    mx.close()


if __name__ == "__main__":
    main()
