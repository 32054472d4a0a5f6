"""CPU tests of the drop-in boundary: the C-ABI library loads and exports
every entry point include/ofhe_hip.h declares (no compute without a GPU)."""
import ctypes
import os
import re

import pytest
from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ofhe_hip.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ofhe_hip_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared()
    for must in ("ofhe_hip_ntt_fwd", "ofhe_hip_ntt_inv", "ofhe_hip_ntt_mul_intt", "ofhe_hip_modmul_vv",
                 "ofhe_hip_modadd_vv", "ofhe_hip_modsub_vv", "ofhe_hip_approx_switch_crt_basis",
                 "ofhe_hip_plan_create", "ofhe_hip_init"):
        assert must in names


def test_library_exports_every_symbol():
    import ofhe_hip

    if not os.path.exists(ofhe_hip.LIB_PATH):
        pytest.fail("libofhe_hip.so not built; run __graft_entry__.build()")
    L = ctypes.CDLL(ofhe_hip.LIB_PATH)
    missing = [n for n in declared() if not hasattr(L, n)]
    assert not missing, missing
    # the Python binding covers exactly the declared ABI
    assert sorted(ofhe_hip.EXPORTED_SYMBOLS) == declared()


def test_version_and_no_fallback():
    import ofhe_hip

    assert "gfx950" in ofhe_hip.version()
    # the product module must not reference the oracle
    src = open(os.path.join(ROOT, "upmem--openfhe_amd", "ofhe_hip.py")).read()
    assert "oracle" not in src.replace("oracle/", "")


def test_kernels_built_for_gfx950():
    import ofhe_hip

    blob = open(ofhe_hip.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
