"""Shared pytest setup: markers, import paths, golden fixtures."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "upmem--openfhe_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built backend")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def O():
    import oracle

    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def hip():
    """The product backend on cuda:0.  Fails (does not skip) when the GPU or
    the built library is missing: -m gpu runs on an MI355X box."""
    import torch

    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    import ofhe_hip

    ofhe_hip.lib()
    ctx = ofhe_hip.Context(0)
    yield ofhe_hip, ctx
    torch.cuda.synchronize()
    ctx.close()
