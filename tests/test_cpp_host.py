"""Runs the C++ adapter parity suite (tests/cpp/test_dcrt.cpp) on the GPU.
The suite mirrors UnitTestTransform / UnitTestNTT / UnitTestMubintvec /
UnitTestDCRTElements through upmem--openfhe_amd/host/ofhe_dcrt.hpp."""
import os
import subprocess

import pytest
from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cpp_adapter_suite():
    d = os.path.join(ROOT, "tests", "cpp")
    subprocess.run(["make", "-s", "-C", d], check=True)
    r = subprocess.run([os.path.join(d, "test_dcrt_bin")], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout
