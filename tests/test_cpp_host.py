"""Runs the C++ adapter parity suite (tests/cpp/test_dcrt.cpp) on the GPU.
The suite mirrors UnitTestTransform / UnitTestNTT / UnitTestMubintvec /
UnitTestDCRTElements through upmem--openfhe_amd/host/ofhe_dcrt.hpp."""
import os
import re
import subprocess

import pytest
from conftest import ROOT

gpu = pytest.mark.gpu


def _suite_names():
    """The sub-tests of tests/cpp/test_dcrt.cpp, read from its source (no
    binary needed to collect): one pytest item each, so a red sub-test names
    itself and does not hide the rest of the suite behind one item."""
    src = open(os.path.join(ROOT, "tests", "cpp", "test_dcrt.cpp")).read()
    return re.findall(r'^    TEST\("([^"]+)"', src, re.M)


@pytest.fixture(scope="module")
def cpp_bins():
    d = os.path.join(ROOT, "tests", "cpp")
    subprocess.run(["make", "-s", "-C", d], check=True)
    return d


def test_cpp_suite_listing_matches_source():
    """The registry the binary runs is the list collected here (CPU-side)."""
    names = _suite_names()
    assert len(names) == len(set(names)) >= 20


@gpu
@pytest.mark.parametrize("name", _suite_names())
def test_cpp_adapter(cpp_bins, name):
    r = subprocess.run([os.path.join(cpp_bins, "test_dcrt_bin"), "--only", name], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "1 tests, 0 failures" in r.stdout, r.stdout


def _read_chain(path):
    import numpy as np

    raw = open(path, "rb").read()
    out, off = [], 0
    while off < len(raw):
        n = int(np.frombuffer(raw, np.uint64, 1, off)[0])
        out.append(np.frombuffer(raw, np.uint64, n, off + 8).copy())
        off += 8 + 8 * n
    return out


@gpu
def test_cpp_device_resident_chain(tmp_path):
    """tests/cpp/chain.cpp strings SwitchFormat -> Times -> SwitchFormat ->
    scalar Plus/Minus -> ApproxModUp -> KeySwitchCore -> ApproxModDown together
    on device-resident DCRTPolyHip objects (no host round trip between steps)
    and dumps every intermediate; each is checked here against the oracle."""
    import numpy as np

    import keyswitch as K
    import oracle as O

    d = os.path.join(ROOT, "tests", "cpp")
    subprocess.run(["make", "-s", "-C", d], check=True)
    out = str(tmp_path / "chain.bin")
    r = subprocess.run([os.path.join(d, "chain_bin"), out, "5"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    v = _read_chain(out)
    log_n, B, sq, sp, dnum = (int(x) for x in v[0])
    q, p, rq, rp = ([int(x) for x in a] for a in v[1:5])
    n = 1 << log_n
    a, b = v[5].reshape(B, sq, n), v[6].reshape(B, sq, n)
    kb, ka = v[7].reshape(dnum, sq + sp, n), v[8].reshape(dnum, sq + sp, n)
    s1, s2 = [int(x) for x in v[9]], [int(x) for x in v[10]]
    Y, Z, Z2, U, K0, K1, D = v[11:18]
    tq = O.Tables(n, q, rq)
    y = O.eltwise("mul", O.ntt_fwd(a, tq), b, q)
    assert np.array_equal(Y.reshape(B, sq, n), y), "SwitchFormat -> Times"
    z = O.ntt_inv(y, tq)
    assert np.array_equal(Z.reshape(B, sq, n), z), "SwitchFormat back"
    assert np.array_equal(z, O.ntt_mul_intt(a, b, tq)), "the fused pipeline is the same op"
    z2 = O.sub_scalar(O.add_scalar_at(z, 0, s1, q), s2, q)
    assert np.array_equal(Z2.reshape(B, sq, n), z2), "Plus(Integer) in coefficient form, Minus(Integer)"
    u = K.approx_mod_up(z2, q, rq, p, rp, eval_form=False)
    assert np.array_equal(U.reshape(B, sq + sp, n), u), "ApproxModUp"
    kp = K.KeySwitchParams(n, q, rq, p, rp, dnum)
    r0, r1 = K.ks_core(kp, y, kb, ka)
    assert np.array_equal(K0.reshape(B, sq, n), r0), "KeySwitchCore ct0"
    assert np.array_equal(K1.reshape(B, sq, n), r1), "KeySwitchCore ct1"
    assert np.array_equal(D.reshape(B, sq, n), O.ntt_fwd(z2, tq)), "ApproxModDown(P * ApproxModUp(z2)) = z2"


@gpu
def test_cpp_openfhe_hooks(tmp_path):
    """The RUN_ON_HIP hook bodies (host/ofhe_openfhe_hooks.hpp) inside a test
    double of DCRTPolyImpl / KeySwitchHYBRID with the reference's accessor
    names (tests/cpp/mock_openfhe.hpp), with the gate forced to the device and
    to the CPU loop, each checked against the oracle (tests/cpp/test_hooks.cpp).
    The KeySwitchCore hook's device results (two levels, t = 0 and a BGV t)
    are dumped and checked here against oracle/keyswitch.py."""
    import numpy as np

    import keyswitch as K

    d = os.path.join(ROOT, "tests", "cpp")
    subprocess.run(["make", "-s", "-C", d], check=True)
    out = str(tmp_path / "ks.bin")
    r = subprocess.run([os.path.join(d, "test_hooks_bin"), out], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "hooks: 0 failures" in r.stdout
    v = _read_chain(out)
    log_n, sq, sp, dnum = (int(x) for x in v[0])
    n = 1 << log_n
    allq, allr = [int(x) for x in v[1]], [int(x) for x in v[2]]
    kb, ka = v[3].reshape(dnum, sq + sp, n), v[4].reshape(dnum, sq + sp, n)
    kp = K.KeySwitchParams(n, allq[:sq], allr[:sq], allq[sq:], allr[sq:], dnum)
    cases = v[5:]
    assert len(cases) == 4 * 4
    for i in range(0, len(cases), 4):
        l, t = (int(x) for x in cases[i])
        c = cases[i + 1].reshape(1, l, n)
        r0, r1 = K.ks_core(kp, c, kb, ka, t)
        assert np.array_equal(cases[i + 2].reshape(1, l, n), r0), f"KeySwitchCore hook ct0, l={l} t={t}"
        assert np.array_equal(cases[i + 3].reshape(1, l, n), r1), f"KeySwitchCore hook ct1, l={l} t={t}"
