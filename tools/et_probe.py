#!/usr/bin/env python3
"""coop3 kernel time by batch size, with and without in-kernel early
termination (DVB-S2 r1/2, Eb/N0 1.0 dB, <= 50 it): how a lone workgroup's
iteration compares with a full chip's, i.e. what sets configs[4]'s critical
path (bench.py --mixed).  GPU box:  [CODE=dvbs2shape_r5_6 EBN0=3.5 ITERS=50]
python tools/et_probe.py [batch ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ldpcgputegra_amd import Code, Decoder, channel, default_params  # noqa: E402


def main():
    import torch
    batches = [int(x) for x in sys.argv[1:]] or [16, 128, 1366, 4096]
    code = Code(os.environ.get("CODE", "dvbs2_r1_2"))
    dec = Decoder(code, max_batch=max(batches))
    table = channel.i8_table(channel.sigma_from_ebn0(float(os.environ.get("EBN0", "1.0")), code.k_info / code.n))
    iters = int(os.environ.get("ITERS", "50"))
    for B in batches:
        llr = torch.empty((B, code.n), dtype=torch.int8, device="cuda")
        hard = torch.empty((B, code.n), dtype=torch.uint8, device="cuda")
        used = torch.empty((B,), dtype=torch.int32, device="cuda")
        dec.awgn_i8_device(llr, first_cw=0, seed=2024, table=table)
        for et in (0, 1):
            p = default_params(early_term=et)
            dec.decode_i8_device(llr, hard, iters, p, iters_used=used)
            torch.cuda.synchronize()
            dec.profile(True)
            dec.kernel_time(reset=True)
            reps = 3
            for _ in range(reps):
                dec.decode_i8_device(llr, hard, iters, p, iters_used=used)
            torch.cuda.synchronize()
            tot, n = dec.kernel_time(reset=True)
            ms = tot / max(1, n)
            dec.profile(False)
            u = used.float()
            print(json.dumps(dict(code=code.name, batch=B, early_term=et, kernel=dec.last_kernel, kernel_ms=round(ms, 3),
                                  ms_per_iter_max=round(ms / max(1.0, u.max().item()), 4),
                                  iters_avg=round(u.mean().item(), 2), iters_max=int(u.max().item()),
                                  fer=round((u >= iters).float().mean().item(), 5) if et else None)), flush=True)


if __name__ == "__main__":
    main()
