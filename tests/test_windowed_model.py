"""The windowed kernel's decomposition (pre / serial chain / post, two-window
V read-ahead, compressed per-check messages), modelled in numpy, reproduces
the oracle bit-exactly.  CPU-only check of the algebra the HIP kernel uses."""
import numpy as np
import pytest
import windowed_model as WM

import oracle as O
from ldpcgputegra_amd import channel, load_table


@pytest.mark.parametrize("code,ebn0", [("dvbs2_r1_2", 0.8), ("dvbs2_r1_2", 1.5), ("dvbs2_r2_3", 2.0)])
def test_windowed_model_matches_oracle(code, ebn0):
    t = load_table(code)
    sigma = channel.sigma_from_ebn0(ebn0, t.k_info / t.n)
    llr = channel.awgn_i8_host(t.n, 3, seed=17, table=channel.i8_table(sigma))
    hard, soft = WM.decode(t, llr, 3)
    eh, es, _ = O.decode_i8(t, llr, 3, return_soft=True)
    assert np.array_equal(soft, es)
    assert np.array_equal(hard, eh)
