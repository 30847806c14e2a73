"""Runs the C++ adapter parity program (tests/cpp/adapter_test.cpp, built by
__graft_entry__.build()) on the GPU: orbfe::ORBextractor / orbfe::ORBmatcher from
include/orbfe_orbslam.hpp against the oracle, bit-exact."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
BIN = os.path.join(os.path.dirname(__file__), "cpp", "build", "adapter_test")


def test_cpp_adapter_parity():
    assert os.path.exists(BIN), "run __graft_entry__.build() first"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "ADAPTER PASS" in r.stdout, r.stdout + r.stderr
    assert "LATENCY" in r.stdout  # the C++ caller's single-frame latency (tools/bench_rows.py row)
    assert "BOW_LATENCY" in r.stdout  # SearchByBoW from C++: GPU and the one-thread CPU port
