"""The native BER/FER sweep driver (ldpcgputegra_amd/bin/ldpc_sim, the
caller side of the boundary modelled on code/x86/main_p.cpp:404-656): one
report line + one JSON line per SNR point."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIM = os.path.join(ROOT, "ldpcgputegra_amd", "bin", "ldpc_sim")


def run(args, timeout=120):
    return subprocess.run([SIM] + args, capture_output=True, text=True, timeout=timeout)


def points(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_sim_without_gpu_fails_cleanly(gpu_available):
    if gpu_available:
        pytest.skip("GPU present")
    r = run(["-code", "576x288", "-min", "1", "-max", "1", "-iter", "2"])
    assert r.returncode != 0
    assert "GPU" in r.stderr or "device" in r.stderr


@pytest.mark.gpu
def test_sim_sweep_648_float_free_int8():
    r = run(["-code", "648x324", "-min", "1.0", "-max", "3.0", "-pas", "1.0", "-iter", "20", "-fer", "50",
             "-frames", "8192", "-batch", "1024"])
    assert r.returncode == 0, r.stderr
    pts = points(r.stdout)
    assert [round(p["ebn0"], 2) for p in pts] == [1.0, 2.0, 3.0]
    for p in pts:
        assert 0 <= p["frame_errors"] <= p["frames"]
        assert p["bit_errors"] >= p["frame_errors"]
    ber = [p["bit_errors"] / p["frames"] for p in pts]
    assert ber[0] > ber[1] >= ber[2] and ber[0] > 0     # the waterfall


@pytest.mark.gpu
def test_sim_dvbs2_random_codewords_early_termination():
    r = run(["-code", "dvbs2_r1_2", "-min", "1.3", "-max", "1.3", "-iter", "50", "-fer", "10", "-frames", "4096",
             "-batch", "4096", "-encoder", "-et"])
    assert r.returncode == 0, r.stderr
    (p,) = points(r.stdout)
    assert p["frames"] >= 4096
    assert p["frame_errors"] <= 4                      # far past the r1/2 waterfall at 1.3 dB
