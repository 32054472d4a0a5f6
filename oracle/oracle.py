"""ctypes wrapper of the CPU oracle (oracle/ofhe_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libofhe_oracle.so")

_u64 = ctypes.c_uint64
_u64p = ctypes.POINTER(ctypes.c_uint64)
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "oracle_msb": (ctypes.c_uint, [_u64]),
            "oracle_compute_mu": (_u64, [_u64]),
            "oracle_modmul_barrett": (_u64, [_u64, _u64, _u64, _u64]),
            "oracle_shoup_prep": (_u64, [_u64, _u64]),
            "oracle_modmul_shoup": (_u64, [_u64, _u64, _u64, _u64]),
            "oracle_modadd": (_u64, [_u64, _u64, _u64]),
            "oracle_modsub": (_u64, [_u64, _u64, _u64]),
            "oracle_modexp": (_u64, [_u64, _u64, _u64]),
            "oracle_modinv": (_u64, [_u64, _u64]),
            "oracle_is_prime": (ctypes.c_int, [_u64]),
            "oracle_first_prime": (_u64, [ctypes.c_uint, _u64]),
            "oracle_previous_prime": (_u64, [_u64, _u64]),
            "oracle_next_prime": (_u64, [_u64, _u64]),
            "oracle_root_of_unity": (_u64, [_u64, _u64]),
            "oracle_moduli_chain": (ctypes.c_int, [ctypes.c_uint, _u64, ctypes.c_uint, _u64p, _u64p]),
            "oracle_ntt_tables": (ctypes.c_int, [_u64, _u64, _u64, _u64p, _u64p, _u64p, _u64p, _u64p, _u64p]),
            "oracle_ntt_fwd": (None, [_u64p, _u64, _u64, _u64p, _u64p]),
            "oracle_ntt_inv": (None, [_u64p, _u64, _u64, _u64p, _u64p, _u64, _u64]),
            "oracle_vec_modmul": (None, [_u64p, _u64p, _u64p, _u64, _u64]),
            "oracle_vec_modadd": (None, [_u64p, _u64p, _u64p, _u64, _u64]),
            "oracle_vec_modsub": (None, [_u64p, _u64p, _u64p, _u64, _u64]),
            "oracle_vec_modmul_scalar": (None, [_u64p, _u64, _u64p, _u64, _u64]),
            "oracle_vec_modadd_scalar": (None, [_u64p, _u64, _u64p, _u64, _u64]),
            "oracle_vec_modsub_scalar": (None, [_u64p, _u64, _u64p, _u64, _u64]),
            "oracle_dcrt_ntt_fwd": (None, [_u64p, _u64, _u64, ctypes.c_uint, _u64p, _u64p, _u64p]),
            "oracle_dcrt_ntt_inv": (None, [_u64p, _u64, _u64, ctypes.c_uint, _u64p, _u64p, _u64p, _u64p, _u64p]),
            "oracle_dcrt_ntt_mul_intt": (None, [_u64p, _u64p, _u64p, _u64, _u64, ctypes.c_uint, _u64p, _u64p,
                                                _u64p, _u64p, _u64p, _u64p, _u64p]),
            "oracle_dcrt_eltwise": (None, [ctypes.c_int, _u64p, _u64p, _u64p, _u64, _u64, ctypes.c_uint, _u64p]),
            "oracle_approx_switch_crt_basis": (None, [_u64p, _u64p, _u64, ctypes.c_uint, ctypes.c_uint, _u64p,
                                                      _u64p, _u64p, _u64p, _u64p, _u64p, _u64p]),
            "oracle_base_conv_precompute": (None, [ctypes.c_uint, ctypes.c_uint, _u64p, _u64p, _u64p, _u64p,
                                                   _u64p, _u64p, _u64p]),
            "oracle_automorphism": (None, [_u64p, _u64p, _u64, ctypes.c_uint32, ctypes.c_int, _u64]),
            "oracle_splitmix64": (_u64, [_u64p]),
            "oracle_fill_uniform": (None, [_u64p, _u64, _u64, _u64p]),
            "oracle_fnv64": (_u64, [_u64p, _u64]),
            "oracle_num_threads": (ctypes.c_int, []),
            "oracle_set_threads": (None, [ctypes.c_int]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def P(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u64p)


def U(vals) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(vals, dtype=np.uint64))


# ---- scalar / number theory -------------------------------------------------
def first_prime(bits: int, m: int) -> int:
    return int(lib().oracle_first_prime(bits, m))


def previous_prime(q: int, m: int) -> int:
    return int(lib().oracle_previous_prime(q, m))


def next_prime(q: int, m: int) -> int:
    return int(lib().oracle_next_prime(q, m))


def root_of_unity(m: int, q: int) -> int:
    return int(lib().oracle_root_of_unity(m, q))


def moduli_chain(log_n: int, towers: int, bits: int = 60):
    """poly-benchmark modulus chain (poly-benchmark-16k.cpp:89-96) and minimal roots."""
    q = np.zeros(towers, dtype=np.uint64)
    r = np.zeros(towers, dtype=np.uint64)
    rc = lib().oracle_moduli_chain(bits, 2 << log_n, towers, P(q), P(r))
    assert rc == 0
    return [int(x) for x in q], [int(x) for x in r]


# ---- synthetic inputs ----------------------------------------------------------
def splitmix_fill(n: int, q: int, state: np.ndarray) -> np.ndarray:
    """n draws of splitmix64() % q continuing the stream in state (1-element uint64 array)."""
    out = np.empty(n, dtype=np.uint64)
    lib().oracle_fill_uniform(P(out), n, q, P(state))
    return out


def fnv64(x: np.ndarray) -> int:
    x = np.ascontiguousarray(x, dtype=np.uint64).reshape(-1)
    return int(lib().oracle_fnv64(P(x), x.size))


def uniform_dcrt(batch: int, towers: int, n: int, moduli, seed: int) -> np.ndarray:
    """[batch][towers][n] residues; tower t of batch b uses splitmix seed
    0x5EED ^ (b<<20) ^ (t<<8) ^ seed."""
    out = np.empty((batch, towers, n), dtype=np.uint64)
    for b in range(batch):
        for t in range(towers):
            st = U([0x5EED ^ (b << 20) ^ (t << 8) ^ seed])
            out[b, t] = splitmix_fill(n, moduli[t], st)
    return out


# ---- NTT ---------------------------------------------------------------------------
class Tables:
    def __init__(self, n: int, moduli, roots):
        self.n, self.towers = n, len(moduli)
        self.q = U(moduli)
        T = self.towers
        self.tab = np.zeros((T, n), np.uint64)
        self.tab_pre = np.zeros((T, n), np.uint64)
        self.itab = np.zeros((T, n), np.uint64)
        self.itab_pre = np.zeros((T, n), np.uint64)
        lg = n.bit_length() - 1
        self.coi = np.zeros((T, lg + 1), np.uint64)
        self.coi_pre = np.zeros((T, lg + 1), np.uint64)
        for t in range(T):
            rows = [self.tab[t], self.tab_pre[t], self.itab[t], self.itab_pre[t], self.coi[t], self.coi_pre[t]]
            ptrs = [r.ctypes.data_as(_u64p) for r in rows]
            assert lib().oracle_ntt_tables(n, int(moduli[t]), int(roots[t]), *ptrs) == 0
        # n^-1 = TableCOI[msb(n-1)] (transformnat-impl.h:661-665)
        self.ninv = U([self.coi[t, lg] for t in range(T)])
        self.ninv_pre = U([self.coi_pre[t, lg] for t in range(T)])


def ntt_fwd(x: np.ndarray, tb: Tables) -> np.ndarray:
    """[batch][towers][n] -> new array, forward NTT per tower."""
    y = np.ascontiguousarray(x, dtype=np.uint64).copy()
    B = y.shape[0]
    lib().oracle_dcrt_ntt_fwd(P(y), B, tb.n, tb.towers, P(tb.q), P(tb.tab), P(tb.tab_pre))
    return y


def ntt_inv(x: np.ndarray, tb: Tables) -> np.ndarray:
    y = np.ascontiguousarray(x, dtype=np.uint64).copy()
    B = y.shape[0]
    lib().oracle_dcrt_ntt_inv(P(y), B, tb.n, tb.towers, P(tb.q), P(tb.itab), P(tb.itab_pre), P(tb.ninv),
                              P(tb.ninv_pre))
    return y


def ntt_mul_intt(a: np.ndarray, b: np.ndarray, tb: Tables) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    c = np.empty_like(a)
    lib().oracle_dcrt_ntt_mul_intt(P(a), P(b), P(c), a.shape[0], tb.n, tb.towers, P(tb.q), P(tb.tab),
                                   P(tb.tab_pre), P(tb.itab), P(tb.itab_pre), P(tb.ninv), P(tb.ninv_pre))
    return c


def eltwise(op: str, a: np.ndarray, b: np.ndarray, moduli) -> np.ndarray:
    code = {"mul": 0, "add": 1, "sub": 2}[op]
    a = np.ascontiguousarray(a, dtype=np.uint64)
    b = np.ascontiguousarray(b, dtype=np.uint64)
    c = np.empty_like(a)
    q = U(moduli)
    lib().oracle_dcrt_eltwise(code, P(a), P(b), P(c), a.shape[0], a.shape[2], a.shape[1], P(q))
    return c


def _scalar(fn: str, a: np.ndarray, scalars, moduli) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    c = np.empty_like(a)
    f = getattr(lib(), fn)
    for bi in range(a.shape[0]):
        for t in range(a.shape[1]):
            f(P(a[bi, t]), int(scalars[t]), P(c[bi, t]), a.shape[2], int(moduli[t]))
    return c


def mul_scalar(a: np.ndarray, scalars, moduli) -> np.ndarray:
    """NativeVectorT::ModMul(const IntegerType&) per tower (mubintvecnat.cpp:310-332)."""
    return _scalar("oracle_vec_modmul_scalar", a, scalars, moduli)


def add_scalar(a: np.ndarray, scalars, moduli) -> np.ndarray:
    """NativeVectorT::ModAdd(const IntegerType&) per tower (mubintvecnat.cpp:198-219)."""
    return _scalar("oracle_vec_modadd_scalar", a, scalars, moduli)


def sub_scalar(a: np.ndarray, scalars, moduli) -> np.ndarray:
    """NativeVectorT::ModSub(const IntegerType&) per tower (mubintvecnat.cpp:267-288)."""
    return _scalar("oracle_vec_modsub_scalar", a, scalars, moduli)


def add_scalar_at(a: np.ndarray, index: int, scalars, moduli) -> np.ndarray:
    """NativeVectorT::ModAddAtIndex(index, s_t) per tower (mubintvecnat.cpp:221-231): NativeIntegerT::ModAddEq
    (ubintnat.h:726-737) on one word; Python big ints (small case)."""
    c = np.array(a, dtype=np.uint64, copy=True)
    for t in range(c.shape[1]):
        q = int(moduli[t])
        for bi in range(c.shape[0]):
            x, s = int(c[bi, t, index]), int(scalars[t])
            c[bi, t, index] = ((x % q) + (s % q)) % q
    return c


# ---- base conversion --------------------------------------------------------------
def base_conv_precompute(q, p):
    sq, sp = len(q), len(p)
    qa, pa = U(q), U(p)
    qhinv = np.zeros(sq, np.uint64)
    qhinv_pre = np.zeros(sq, np.uint64)
    qhmodp = np.zeros(sq * sp, np.uint64)
    mu_lo = np.zeros(sp, np.uint64)
    mu_hi = np.zeros(sp, np.uint64)
    lib().oracle_base_conv_precompute(sq, sp, P(qa), P(pa), P(qhinv), P(qhinv_pre), P(qhmodp), P(mu_lo),
                                      P(mu_hi))
    return dict(qhinv=qhinv, qhinv_pre=qhinv_pre, qhmodp=qhmodp, mu_lo=mu_lo, mu_hi=mu_hi)


def approx_switch_crt_basis(x: np.ndarray, q, p, pre) -> np.ndarray:
    """x: [size_q][n] -> [size_p][n]."""
    x = np.ascontiguousarray(x, dtype=np.uint64)
    sq, n = x.shape
    sp = len(p)
    out = np.empty((sp, n), np.uint64)
    lib().oracle_approx_switch_crt_basis(P(x), P(out), n, sq, sp, P(U(q)), P(U(p)), P(pre["qhinv"]),
                                         P(pre["qhinv_pre"]), P(pre["qhmodp"]), P(pre["mu_lo"]), P(pre["mu_hi"]))
    return out
