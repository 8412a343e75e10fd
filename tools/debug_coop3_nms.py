#!/usr/bin/env python3
"""Debug probe (GPU): where coop3's degree-14 decode first differs from the
oracle -- per configuration, the first iteration count with a difference and
the differing variables (info / parity) and codewords."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import torch  # noqa: E402
from ldpcgputegra_amd import ALGO_NMS, Code, Decoder, channel, default_params, load_table  # noqa: E402


def run(code, B, ebn0, seed, algo, param, iters_list, early=0):
    t = load_table(code)
    llr = channel.awgn_i8_host(t.n, B, seed=seed, table=channel.i8_table(channel.sigma_from_ebn0(ebn0, t.k_info / t.n)))
    dec = Decoder(Code(code), max_batch=max(B, 64), kernel=8)
    k = t.k_info
    for it in iters_list:
        oa = O.NMS if algo == ALGO_NMS else O.OMS
        eh, es, _ = O.decode_i8(t, llr, it, oa, param, early_term=bool(early), return_soft=True,
                                threads=O.host_threads())
        d_hard = torch.empty((B, t.n), dtype=torch.uint8, device="cuda")
        d_soft = torch.empty((B, t.n), dtype=torch.int8, device="cuda")
        p = default_params(algo=algo, factor=param, early_term=early) if algo == ALGO_NMS else \
            default_params(offset=param, early_term=early)
        d_its = torch.empty(B, dtype=torch.int32, device="cuda")
        dec.decode_i8_device(torch.from_numpy(llr).cuda(), d_hard, it, params=p, soft=d_soft, iters_used=d_its)
        torch.cuda.synchronize()
        s = d_soft.cpu().numpy()
        diff = np.argwhere(s != es)
        print("%s B=%d eb=%.2f algo=%d param=%d it=%d et=%d: %d differing values" % (code, B, ebn0, algo, param, it,
                                                                                    early, len(diff)), flush=True)
        if len(diff):
            cws = np.unique(diff[:, 0])
            vs = diff[:, 1]
            print("  codewords", cws[:16].tolist(), "vars (info <", k, "):", np.sort(vs)[:24].tolist(),
                  "n info", int((vs < k).sum()), "n parity", int((vs >= k).sum()), flush=True)
            i0 = diff[0]
            print("  first:", i0.tolist(), "gpu", int(s[i0[0], i0[1]]), "oracle", int(es[i0[0], i0[1]]), flush=True)
            return
    dec.close()


if __name__ == "__main__":
    code = sys.argv[1] if len(sys.argv) > 1 else "dvbs2shape_r3_4"
    run(code, 64, 1.8, 8, 0, 1, [4, 8, 12, 20])                  # OMS, values far from saturation
    run(code, 64, 2.6, 8, ALGO_NMS, 29, [8, 12], early=1)        # one iteration per segment
    run("dvbs2_r2_3", 64, 2.6, 8, ALGO_NMS, 29, [8, 12])
    run(code, 64, 2.6, 8, ALGO_NMS, 29, [7, 8])
    os.environ["LDPC_LC_SWIZZLE"] = "0"
    run(code, 64, 2.6, 8, ALGO_NMS, 29, [8])                     # (new contexts: plan without the swizzle)
