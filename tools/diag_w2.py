#!/usr/bin/env python3
"""windowed2 vs oracle on a code: first iteration with a soft-output
mismatch, and where (info / parity variables, codewords).
usage (GPU box): python tools/diag_w2.py <code> [batch] [ebn0]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from ldpcgputegra_amd import Code, Decoder, channel, load_table  # noqa: E402

name = sys.argv[1]
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 64
ebn0 = float(sys.argv[3]) if len(sys.argv) > 3 else 1.5
import torch  # noqa: E402
t = load_table(name)
llr = channel.awgn_i8_host(t.n, batch, seed=batch, table=channel.i8_table(channel.sigma_from_ebn0(ebn0, t.k_info / t.n)))
for k in (1, 3, 4):
    dec = Decoder(Code(name), max_batch=64, kernel=k)
    for it in range(1, 7):
        _, ref, _ = O.decode_i8(t, llr, it, O.OMS, 1, return_soft=True)
        d = torch.empty((batch, t.n), dtype=torch.int8, device="cuda")
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), None, it, soft=d)
        torch.cuda.synchronize()
        got = d.cpu().numpy()
        bad = np.argwhere(got != ref)
        if bad.size:
            cw = np.unique(bad[:, 0])
            vs = np.unique(bad[:, 1])
            print("kernel", k, "iter", it, "diffs", len(bad), "codewords", cw[:10], "vars", vs[:20],
                  "info vars", int((vs < t.k_info).sum()), "got", got[bad[0][0], bad[0][1]], "ref", ref[bad[0][0], bad[0][1]])
            break
    else:
        print("kernel", k, "ok through 6 iterations")
