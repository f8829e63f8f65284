"""The C ABI from a plain-C host (examples/c_host.c, built with gcc by
p2pdl_amd/csrc/Makefile): FedAvg, FedAvg with torch's GPU division and the
median, each bit-exact against the same op sequences written in C -- the
boundary a cgo / JNI / N-API binding would use, with no Python in the path."""
import os
import subprocess

import pytest

EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "c_host")


def test_c_host_is_built_against_the_library():
    assert os.path.exists(EXE), "run __graft_entry__.build() (make -C p2pdl_amd/csrc)"
    out = subprocess.check_output(["ldd", EXE], text=True)
    assert "libp2pdl_hip.so" in out and "not found" not in out.split("libp2pdl_hip.so")[1].splitlines()[0]


@pytest.mark.gpu
def test_c_host_results_bit_exact(cuda):
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("bit-exact") == 3, r.stdout
