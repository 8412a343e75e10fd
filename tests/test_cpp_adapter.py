"""include/ldpc_mi355x.hpp compiles as a drop-in for the reference's decoder
construction and runs (on a GPU box: decodes; here: documented EDEVICE)."""
import os
import subprocess

import pytest
from conftest import ROOT

EXE = os.path.join(ROOT, "build", "adapter_example")


def build():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    lib = os.path.join(ROOT, "ldpcgputegra_amd")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "adapter_example.cpp"), "-L", lib,
                           "-lldpc_mi355x", "-Wl,-rpath," + lib, "-o", EXE])


def run():
    return subprocess.run([EXE, os.path.join(ROOT, "ldpcgputegra_amd", "codes", "576x288.ldpc")],
                          capture_output=True, text=True, timeout=300)


def test_adapter_builds_and_reports_no_device(gpu_available):
    build()
    if gpu_available:
        pytest.skip("GPU present: covered by the gpu-marked test")
    r = run()
    assert r.returncode == 3, r.stdout + r.stderr


@pytest.mark.gpu
def test_adapter_decodes_on_gpu():
    build()
    r = run()
    assert r.returncode == 0, r.stdout + r.stderr
