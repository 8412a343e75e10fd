"""Debug (GPU box): where the two-lanes-per-check coop3 kernel first differs
from the oracle -- per code, batch and iteration count: differing soft values,
the first differing (codeword, variable), the variable's kind (info / parity)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as O  # noqa: E402
from test_gpu_coop3_r23 import _llr, _run  # noqa: E402
from ldpcgputegra_amd import default_params, load_table  # noqa: E402

for code, ebn0 in (("dvbs2_r8_9", 4.3), ("dvbs2_r9_10", 4.4), ("dvbs2shape_r5_6", 3.4)):
    t = load_table(code)
    for batch, iters in ((1, 1), (1, 2), (1, 3), (16, 1), (16, 3), (37, 1), (37, 2), (37, 10)):
        llr = _llr(code, batch, ebn0, 11 + batch)
        eh, es, _ = O.decode_i8(t, llr, iters, return_soft=True, threads=O.host_threads())
        h, s, _, _ = _run(code, llr, iters, default_params())
        d = np.argwhere(s != es)
        msg = "%s b%d it%d: %d soft diffs" % (code, batch, iters, len(d))
        if len(d):
            cws = sorted(set(d[:, 0].tolist()))
            msg += ", codewords %s, first (cw %d, var %d %s) got %d want %d, vars %s" % (
                cws[:12], d[0][0], d[0][1], "info" if d[0][1] < t.k_info else "parity", s[d[0][0], d[0][1]],
                es[d[0][0], d[0][1]], sorted(set(d[:, 1].tolist()))[:10])
        print(msg, flush=True)
