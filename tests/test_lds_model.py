"""The LDS kernel's decomposition (csrc/lds.hip), modelled in numpy: the
layered schedule cut into layers -- maximal runs of consecutive same-group
checks sharing no variable -- with every check of a layer evaluated at once
(vectorised, as the kernel's lanes do), reproduces the oracle's check-serial
float decode bit-exactly, and the layer count agrees with the C planner
(ldpc_code_layer_info).  CPU-only check of the commutation argument."""
import numpy as np
import pytest

import oracle as O
from ldpcgputegra_amd import Code, channel, load_table


def layers_of(t):
    """Python restatement of lds_plan (csrc/lds.hip)."""
    checks = list(t.checks())
    out, i = [], 0
    while i < len(checks):
        g = checks[i][0]
        seen, j = set(), i
        while j < len(checks) and checks[j][0] == g:
            vs = set(int(v) for v in checks[j][1])
            if vs & seen:
                break
            seen |= vs
            j += 1
        out.append((i, j))
        i = j
    return out, checks


def decode_layers_f32(t, llr, iters):
    """Float min-sum (beta 0) over the layer plan, whole layers at a time."""
    layers, checks = layers_of(t)
    V = llr.astype(np.float32).copy()                     # [B, N]
    msg = [np.zeros((llr.shape[0], len(vs)), np.float32) for _, vs in checks]
    idx = [np.asarray(vs, dtype=np.int64) for _, vs in checks]
    for _ in range(iters):
        for a, b in layers:
            d = len(idx[a])
            vi = np.stack([idx[c] for c in range(a, b)])            # [L, d]
            m = np.stack([msg[c] for c in range(a, b)], axis=1)      # [B, L, d]
            c = V[:, vi] - m                                         # all checks of the layer read first
            ac = np.abs(c)
            sign = ((c < 0).sum(axis=2) + d) & 1                     # parity incl. the odd-degree flip
            min1 = ac.min(axis=2)
            srt = np.sort(ac, axis=2)
            min2 = srt[:, :, 1]
            r = np.where(ac == min1[:, :, None], min2[:, :, None], min1[:, :, None])
            neg = (sign[:, :, None] ^ (c < 0)).astype(bool)
            new = np.where(neg, -r, r).astype(np.float32)
            V[:, vi] = (c + new).astype(np.float32)                  # disjoint variables: no write conflicts
            for k, cc in enumerate(range(a, b)):
                msg[cc] = new[:, k, :]
    return (V > 0).astype(np.uint8), V


@pytest.mark.parametrize("code", ["648x324", "576x288", "1944x972"])
def test_layer_plan_matches_c_planner(code):
    t = load_table(code)
    layers, _ = layers_of(t)
    info = Code(code).layer_info()
    assert info["n_layers"] == len(layers)
    assert info["max_width"] == max(b - a for a, b in layers)


@pytest.mark.parametrize("code,ebn0", [("648x324", 1.0), ("648x324", 2.5), ("576x288", 2.0)])
def test_layer_parallel_float_model_matches_oracle(code, ebn0):
    t = load_table(code)
    rng = np.random.default_rng(13)
    sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
    llr = (-1.0 + sigma * rng.standard_normal((6, t.n))).astype(np.float32)
    hard, soft = decode_layers_f32(t, llr, 10)
    eh, es, _ = O.decode_f32(t, llr, 10, O.OMS, 0.0)
    assert np.array_equal(soft, es)
    assert np.array_equal(hard, eh)
