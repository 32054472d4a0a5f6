"""ctypes binding of the gfx950 RNS backend (C ABI: include/ofhe_hip.h).

Host-side mirror of the reference's offload interface for the hot path:

* ``Context``   ~ ``PimManager::getPim`` (src/core/include/pim/PimManager.h:23-29):
  one per device, allocation and host<->device copies.
* ``NTTPlan``   ~ ``ChineseRemainderTransformFTT<NativeVector>`` with its
  ``PreCompute`` tables (transformnat-impl.h:575-763) plus the
  ``NativeVectorT`` element-wise ops (mubintvecnat.cpp:245-367) over
  [batch][tower][N] device buffers.
* ``BaseConverter`` ~ ``DCRTPolyImpl::ApproxSwitchCRTBasis`` (dcrtpoly-impl.h:1034-1063).
* ``approx_mod_up`` / ``approx_mod_down`` ~ ``DCRTPolyImpl::ApproxModUp`` /
  ``ApproxModDown`` (dcrtpoly-impl.h:1085-1175).
* ``KeySwitch`` ~ ``KeySwitchHYBRID`` (pke/lib/keyswitch/keyswitch-hybrid.cpp:325-482)
  with the tables of ``CryptoParametersRNS::PrecomputeCRTTables``.
* ``switch_modulus`` / ``NTTPlan.automorphism`` ~ ``NativeVectorT::SwitchModulus``
  (mubintvecnat.cpp:111-136) / ``PolyImpl::AutomorphismTransform`` (poly-impl.h:312-365).

Errors raise ``MathError`` (the analogue of ``lbcrypto::math_error`` thrown by
``OPENFHE_THROW``).  Pointers are plain integers (e.g. ``torch.Tensor.data_ptr()``)
and streams are ``hipStream_t`` values as integers (``torch.cuda.Stream.cuda_stream``).

There is no CPU fallback: if ``lib/libofhe_hip.so`` is missing this module
raises on first use.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libofhe_hip.so")

_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


class MathError(RuntimeError):
    """Raised when a backend call returns a non-zero status (cf. lbcrypto::math_error)."""


_lib: Optional[ctypes.CDLL] = None

# name -> (restype, argtypes)
_SIGS = {
    "ofhe_hip_last_error": (ctypes.c_char_p, []),
    "ofhe_hip_version": (ctypes.c_char_p, []),
    "ofhe_hip_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "ofhe_hip_init": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_vp)]),
    "ofhe_hip_finalize": (ctypes.c_int, [_vp]),
    "ofhe_hip_alloc": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "ofhe_hip_free": (ctypes.c_int, [_vp, _vp]),
    "ofhe_hip_alloc_async": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp), _vp]),
    "ofhe_hip_free_async": (ctypes.c_int, [_vp, _vp, _vp]),
    "ofhe_hip_host_alloc": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.POINTER(_vp)]),
    "ofhe_hip_host_free": (ctypes.c_int, [_vp, _vp]),
    "ofhe_hip_zero": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, _vp]),
    "ofhe_hip_copy_to_device": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ofhe_hip_copy_to_host": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ofhe_hip_copy_device": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "ofhe_hip_sync": (ctypes.c_int, [_vp, _vp]),
    "ofhe_hip_event_create": (ctypes.c_int, [_vp, ctypes.POINTER(_vp)]),
    "ofhe_hip_event_record": (ctypes.c_int, [_vp, _vp]),
    "ofhe_hip_event_sync": (ctypes.c_int, [_vp]),
    "ofhe_hip_event_destroy": (ctypes.c_int, [_vp]),
    "ofhe_hip_trim": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "ofhe_hip_plan_create": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p,
                                            ctypes.POINTER(_vp)]),
    "ofhe_hip_plan_destroy": (ctypes.c_int, [_vp]),
    "ofhe_hip_plan_tune": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32]),
    "ofhe_hip_plan_create_ex": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p,
                                               _vp, ctypes.POINTER(_vp)]),
    "ofhe_hip_plan_tables": (ctypes.c_int, [_vp, _u64p, _u64p, _u64p, _u64p, _u64p]),
    "ofhe_hip_ntt_fwd": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_ntt_inv": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modmul_vv": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modadd_vv": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modsub_vv": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modmul_scalar": (ctypes.c_int, [_vp, _vp, _u64p, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modadd_scalar": (ctypes.c_int, [_vp, _vp, _u64p, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modsub_scalar": (ctypes.c_int, [_vp, _vp, _u64p, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_modadd_scalar_at": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _u64p, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_fill_uniform": (ctypes.c_int, [_vp, _vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, _vp]),
    "ofhe_hip_ntt_mul_intt": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_ntt_mul_intt_stage": (ctypes.c_int, [_vp, ctypes.c_int, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_bconv_create": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                             _u64p, _u64p, _u64p, _u64p, ctypes.POINTER(_vp)]),
    "ofhe_hip_bconv_create_ex": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                _u64p, _u64p, _u64p, _u64p, _vp, ctypes.POINTER(_vp)]),
    "ofhe_hip_bconv_destroy": (ctypes.c_int, [_vp]),
    "ofhe_hip_approx_switch_crt_basis": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_ntt_fwd_range": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint32, _vp]),
    "ofhe_hip_ntt_inv_range": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64,
                                              ctypes.c_uint64, ctypes.c_uint32, _vp]),
    "ofhe_hip_approx_mod_up": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_int, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_approx_mod_down": (ctypes.c_int, [_vp, _vp, _vp, _u64p, ctypes.c_uint64, _vp, _vp,
                                                ctypes.c_uint32, _vp]),
    "ofhe_hip_ks_create": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p, ctypes.c_uint32,
                                          _u64p, _u64p, ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "ofhe_hip_ks_create_ex": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, _u64p, _u64p,
                                             ctypes.c_uint32, _u64p, _u64p, ctypes.c_uint32, _vp,
                                             ctypes.POINTER(_vp)]),
    "ofhe_hip_ks_destroy": (ctypes.c_int, [_vp]),
    "ofhe_hip_ks_digits": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                          ctypes.POINTER(ctypes.c_uint32)]),
    "ofhe_hip_ks_precompute": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_ks_fast_core_ext": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32,
                                                 _vp]),
    "ofhe_hip_ks_mod_down": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                            _vp]),
    "ofhe_hip_ks_core": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint64,
                                        ctypes.c_uint32, _vp]),
    "ofhe_hip_switch_modulus": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                               _vp]),
    "ofhe_hip_automorphism": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_int, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_drop_last_and_scale": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                                    ctypes.c_int, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_mod_reduce": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, ctypes.c_uint64, _vp, ctypes.c_uint64,
                                           ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_bv_precompute": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_bv_core": (ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                        ctypes.c_uint32, _vp]),
    "ofhe_hip_eval_mult_core": (ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]),
    "ofhe_hip_comm_unique_id": (ctypes.c_int, [_vp]),
    "ofhe_hip_comm_init": (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.POINTER(_vp)]),
    "ofhe_hip_comm_destroy": (ctypes.c_int, [_vp]),
    "ofhe_hip_bcast_evalkey": (ctypes.c_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_int, _vp]),
}

COMM_ID_BYTES = 128  # OFHE_COMM_ID_BYTES

EXPORTED_SYMBOLS = tuple(_SIGS)


def lib() -> ctypes.CDLL:
    """Load (once) and return the backend library; raise if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MathError(
                f"HIP backend not built: {LIB_PATH} is missing "
                "(run __graft_entry__.build() or make -C upmem--openfhe_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def _check(rc: int) -> None:
    if rc != 0:
        msg = lib().ofhe_hip_last_error().decode(errors="replace")
        raise MathError(f"ofhe_hip error {rc}: {msg}")


def _arr(vals: Sequence[int]):
    return (ctypes.c_uint64 * len(vals))(*[int(v) for v in vals])


def version() -> str:
    return lib().ofhe_hip_version().decode()


def device_count() -> int:
    n = ctypes.c_int(0)
    _check(lib().ofhe_hip_device_count(ctypes.byref(n)))
    return n.value


# Kernel-choice options of include/ofhe_hip.h (ofhe_plan_options,
# ofhe_bconv_options, ofhe_ks_options).  Zero = the library's defaults; every
# setting gives the same results (tests reach every kernel through them).
SPLIT_AUTO, SPLIT_COLS, SPLIT_8_8, SPLIT_9_8, SPLIT_8_9 = range(5)
BCONV_KERNEL_AUTO, BCONV_KERNEL_LIMB, BCONV_KERNEL_WIDE = range(3)


class PlanOptions(ctypes.Structure):
    _fields_ = [("split", ctypes.c_uint32), ("generic_moduli", ctypes.c_uint32)]


class BconvOptions(ctypes.Structure):
    _fields_ = [("kernel", ctypes.c_uint32), ("separate_cols", ctypes.c_uint32)]


class KsOptions(ctypes.Structure):
    _fields_ = [("plan", PlanOptions), ("separate_cols", ctypes.c_uint32), ("separate_icol", ctypes.c_uint32),
                ("chunk", ctypes.c_uint32), ("single_stream", ctypes.c_uint32)]


def _opt_ptr(o):
    return None if o is None else ctypes.cast(ctypes.byref(o), _vp)


class Context:
    """Per-device context (PimManager analogue)."""

    def __init__(self, device: int = 0):
        h = _vp()
        _check(lib().ofhe_hip_init(int(device), ctypes.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        if self._h is None:
            raise MathError("context finalized")
        return self._h

    def close(self) -> None:
        if self._h is not None:
            _check(lib().ofhe_hip_finalize(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def alloc(self, nbytes: int) -> int:
        p = _vp()
        _check(lib().ofhe_hip_alloc(self.handle, int(nbytes), ctypes.byref(p)))
        return p.value

    def free(self, ptr: int) -> None:
        _check(lib().ofhe_hip_free(self.handle, _vp(ptr)))

    def alloc_async(self, nbytes: int, stream: int = 0) -> int:
        p = _vp()
        _check(lib().ofhe_hip_alloc_async(self.handle, int(nbytes), ctypes.byref(p), _vp(stream or None)))
        return p.value

    def free_async(self, ptr: int, stream: int = 0) -> None:
        _check(lib().ofhe_hip_free_async(self.handle, _vp(ptr), _vp(stream or None)))

    def host_alloc(self, nbytes: int) -> int:
        """Pinned host memory (staging for host-buffer integrations)."""
        p = _vp()
        _check(lib().ofhe_hip_host_alloc(self.handle, int(nbytes), ctypes.byref(p)))
        return p.value

    def host_free(self, ptr: int) -> None:
        _check(lib().ofhe_hip_host_free(self.handle, _vp(ptr)))

    def zero(self, dst: int, nbytes: int, stream: int = 0) -> None:
        _check(lib().ofhe_hip_zero(self.handle, _vp(dst), int(nbytes), _vp(stream or None)))

    def copy_to_device(self, dst: int, src: int, nbytes: int, stream: int = 0) -> None:
        _check(lib().ofhe_hip_copy_to_device(self.handle, _vp(dst), _vp(src), int(nbytes), _vp(stream or None)))

    def copy_to_host(self, dst: int, src: int, nbytes: int, stream: int = 0) -> None:
        _check(lib().ofhe_hip_copy_to_host(self.handle, _vp(dst), _vp(src), int(nbytes), _vp(stream or None)))

    def copy_device(self, dst: int, src: int, nbytes: int, stream: int = 0) -> None:
        _check(lib().ofhe_hip_copy_device(self.handle, _vp(dst), _vp(src), int(nbytes), _vp(stream or None)))

    def sync(self, stream: int = 0) -> None:
        _check(lib().ofhe_hip_sync(self.handle, _vp(stream or None)))

    def trim(self, keep_bytes: int = 0) -> None:
        """Give the context's cached stream-ordered memory back to the device."""
        _check(lib().ofhe_hip_trim(self.handle, keep_bytes))


class NTTPlan:
    """Device-resident NTT tables for N = 2**log_n and one modulus per tower.

    Data buffers are [batch][towers][N] uint64 residues in device memory.
    """

    def __init__(self, ctx: Context, log_n: int, moduli: Sequence[int], roots: Sequence[int],
                 split: int = SPLIT_AUTO, generic_moduli: bool = False):
        if len(moduli) != len(roots):
            raise MathError("moduli and roots differ in length")
        self.ctx = ctx
        self.log_n = int(log_n)
        self.n = 1 << self.log_n
        self.moduli = [int(q) for q in moduli]
        self.roots = [int(r) for r in roots]
        self.towers = len(self.moduli)
        h = _vp()
        o = PlanOptions(int(split), 1 if generic_moduli else 0)
        _check(lib().ofhe_hip_plan_create_ex(ctx.handle, self.log_n, self.towers, _arr(self.moduli),
                                             _arr(self.roots), _opt_ptr(o), ctypes.byref(h)))
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise MathError("plan destroyed")
        return self._h

    def close(self) -> None:
        if self._h is not None:
            _check(lib().ofhe_hip_plan_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tune(self, chunk_batch: int = 0, streams: int = 1) -> None:
        """Chunking / stream knob of ntt_mul_intt (speed only; results are identical)."""
        _check(lib().ofhe_hip_plan_tune(self.handle, int(chunk_batch), int(streams)))

    def tables(self):
        """Host copies of (Table, TableP, TableI, TableIP, ninv) as flat lists."""
        tn = self.towers * self.n
        a, b, c, d = (ctypes.c_uint64 * tn)(), (ctypes.c_uint64 * tn)(), (ctypes.c_uint64 * tn)(), (ctypes.c_uint64 * tn)()
        e = (ctypes.c_uint64 * self.towers)()
        _check(lib().ofhe_hip_plan_tables(self.handle, a, b, c, d, e))
        return list(a), list(b), list(c), list(d), list(e)

    # --- transforms (ChineseRemainderTransformFTT) ---
    def forward(self, data: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ntt_fwd(self.handle, _vp(data), int(batch), _vp(stream or None)))

    def inverse(self, data: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ntt_inv(self.handle, _vp(data), int(batch), _vp(stream or None)))

    # --- NativeVectorT element-wise (vector, vector) ---
    def mod_mul(self, a: int, b: int, c: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_modmul_vv(self.handle, _vp(a), _vp(b), _vp(c), int(batch), _vp(stream or None)))

    def mod_add(self, a: int, b: int, c: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_modadd_vv(self.handle, _vp(a), _vp(b), _vp(c), int(batch), _vp(stream or None)))

    def mod_sub(self, a: int, b: int, c: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_modsub_vv(self.handle, _vp(a), _vp(b), _vp(c), int(batch), _vp(stream or None)))

    def mod_mul_scalar(self, a: int, scalars: Sequence[int], c: int, batch: int = 1, stream: int = 0) -> None:
        if len(scalars) != self.towers:
            raise MathError("one scalar per tower required")
        _check(lib().ofhe_hip_modmul_scalar(self.handle, _vp(a), _arr(scalars), _vp(c), int(batch),
                                            _vp(stream or None)))

    def mod_add_scalar(self, a: int, scalars: Sequence[int], c: int, batch: int = 1, stream: int = 0) -> None:
        """NativeVectorT::ModAdd(const IntegerType&) per tower (mubintvecnat.cpp:198-219)."""
        if len(scalars) != self.towers:
            raise MathError("one scalar per tower required")
        _check(lib().ofhe_hip_modadd_scalar(self.handle, _vp(a), _arr(scalars), _vp(c), int(batch),
                                            _vp(stream or None)))

    def mod_sub_scalar(self, a: int, scalars: Sequence[int], c: int, batch: int = 1, stream: int = 0) -> None:
        """NativeVectorT::ModSub(const IntegerType&) per tower (mubintvecnat.cpp:267-288)."""
        if len(scalars) != self.towers:
            raise MathError("one scalar per tower required")
        _check(lib().ofhe_hip_modsub_scalar(self.handle, _vp(a), _arr(scalars), _vp(c), int(batch),
                                            _vp(stream or None)))

    def mod_add_scalar_at(self, a: int, index: int, scalars: Sequence[int], c: int, batch: int = 1,
                          stream: int = 0) -> None:
        """NativeVectorT::ModAddAtIndex(index, s_t) per tower (mubintvecnat.cpp:221-231); only word
        `index` of each (batch, tower) of c is written."""
        if len(scalars) != self.towers:
            raise MathError("one scalar per tower required")
        _check(lib().ofhe_hip_modadd_scalar_at(self.handle, _vp(a), int(index), _arr(scalars), _vp(c), int(batch),
                                               _vp(stream or None)))

    def fill_uniform(self, dst: int, batch: int, seed: int, batch_offset: int = 0, stream: int = 0) -> None:
        """Synthetic residues: splitmix64 streams seeded 0x5EED ^ (b<<20) ^ (t<<8) ^ seed, mod q_t."""
        _check(lib().ofhe_hip_fill_uniform(self.handle, _vp(dst), int(batch), int(batch_offset), int(seed),
                                           _vp(stream or None)))

    # --- tower-range transforms on strided data ---
    def forward_range(self, t0: int, count: int, src: int, dst: int, src_stride: int, dst_stride: int,
                      batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ntt_fwd_range(self.handle, int(t0), int(count), _vp(src), _vp(dst), int(src_stride),
                                            int(dst_stride), int(batch), _vp(stream or None)))

    def inverse_range(self, t0: int, count: int, src: int, dst: int, src_stride: int, dst_stride: int,
                      batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ntt_inv_range(self.handle, int(t0), int(count), _vp(src), _vp(dst), int(src_stride),
                                            int(dst_stride), int(batch), _vp(stream or None)))

    def automorphism(self, k: int, eval_form: bool, src: int, dst: int, batch: int = 1, stream: int = 0) -> None:
        """PolyImpl::AutomorphismTransform(k) on every (batch, tower); dst must not alias src."""
        _check(lib().ofhe_hip_automorphism(self.handle, int(k), 1 if eval_form else 0, _vp(src), _vp(dst),
                                           int(batch), _vp(stream or None)))

    # --- rescaling (DCRTPolyImpl::DropLastElementAndScale / ModReduce) ---
    def drop_last_and_scale(self, towers: int, x: int, x_stride: int, out: int, out_stride: int, eval_form: bool,
                            ql_ql_inv_modql_divql_modq, ql_inv_modq, batch: int = 1, stream: int = 0) -> None:
        """dcrtpoly-impl.h:746-768 on [batch][towers] -> [batch][towers - 1] (out may be x with equal strides; other overlap is rejected)."""
        c, a = list(ql_ql_inv_modql_divql_modq), list(ql_inv_modq)
        if len(c) < towers - 1 or len(a) < towers - 1:
            raise MathError("need towers - 1 constants")
        _check(lib().ofhe_hip_drop_last_and_scale(self.handle, int(towers), _vp(x), int(x_stride), _vp(out),
                                                  int(out_stride), 1 if eval_form else 0, _arr(c), _arr(a), int(batch),
                                                  _vp(stream or None)))

    def mod_reduce(self, towers: int, x: int, x_stride: int, out: int, out_stride: int, eval_form: bool, t: int,
                   neg_t_inv_modq: int, ql_inv_modq, batch: int = 1, stream: int = 0) -> None:
        """dcrtpoly-impl.h:792-812 on [batch][towers] -> [batch][towers - 1] (out may be x with equal strides; other overlap is rejected)."""
        a = list(ql_inv_modq)
        if len(a) < towers - 1:
            raise MathError("need towers - 1 constants")
        _check(lib().ofhe_hip_mod_reduce(self.handle, int(towers), _vp(x), int(x_stride), _vp(out), int(out_stride),
                                         1 if eval_form else 0, int(t), int(neg_t_inv_modq), _arr(a), int(batch),
                                         _vp(stream or None)))

    # --- BV key switching, digitSize = 0 (keyswitch-bv.cpp:302-340) ---
    def bv_precompute(self, towers: int, c: int, digits: int, batch: int = 1, stream: int = 0) -> None:
        """CRTDecompose(0) of c [batch][towers][N] (evaluation form) -> digits [batch][towers][towers][N]."""
        _check(lib().ofhe_hip_bv_precompute(self.handle, int(towers), _vp(c), _vp(digits), int(batch),
                                            _vp(stream or None)))

    def bv_core(self, towers: int, digits: int, key_b: int, key_a: int, key_towers: int, out0: int, out1: int,
                batch: int = 1, stream: int = 0) -> None:
        """EvalFastKeySwitchCore: out0 = sum_i kb[i] d_i, out1 = sum_i ka[i] d_i."""
        _check(lib().ofhe_hip_bv_core(self.handle, int(towers), _vp(digits), _vp(key_b), _vp(key_a), int(key_towers),
                                      _vp(out0), _vp(out1), int(batch), _vp(stream or None)))

    # --- LeveledSHEBase::EvalMultCore, 2 x 2 elements (base-leveledshe.cpp:667-672) ---
    def eval_mult_core(self, c0: int, c1: int, d0: int, d1: int, out0: int, out1: int, out2: int, batch: int = 1,
                       stream: int = 0) -> None:
        _check(lib().ofhe_hip_eval_mult_core(self.handle, _vp(c0), _vp(c1), _vp(d0), _vp(d1), _vp(out0), _vp(out1),
                                             _vp(out2), int(batch), _vp(stream or None)))

    # --- the metric pipeline ---
    def ntt_mul_intt(self, a: int, b: int, c: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ntt_mul_intt(self.handle, _vp(a), _vp(b), _vp(c), int(batch), _vp(stream or None)))


    def ntt_mul_intt_stage(self, stage: int, a: int, b: int, c: int, batch: int = 1, stream: int = 0) -> None:
        """One kernel of ntt_mul_intt (0: forward columns, 1: fused block pass, 2: inverse columns)."""
        _check(lib().ofhe_hip_ntt_mul_intt_stage(self.handle, int(stage), _vp(a), _vp(b), _vp(c), int(batch),
                                                 _vp(stream or None)))


class BaseConverter:
    """ApproxSwitchCRTBasis from basis Q (size_q towers) to basis P (size_p towers)."""

    def __init__(self, ctx: Context, log_n: int, q: Sequence[int], p: Sequence[int],
                 qhat_inv_modq: Sequence[int], qhat_modp: Sequence[int], kernel: int = BCONV_KERNEL_AUTO,
                 separate_cols: bool = False):
        self.ctx = ctx
        self.log_n = int(log_n)
        self.size_q, self.size_p = len(q), len(p)
        if len(qhat_inv_modq) != self.size_q or len(qhat_modp) != self.size_q * self.size_p:
            raise MathError("precomputation sizes do not match the bases")
        h = _vp()
        o = BconvOptions(int(kernel), 1 if separate_cols else 0)
        _check(lib().ofhe_hip_bconv_create_ex(ctx.handle, self.log_n, self.size_q, self.size_p, _arr(q), _arr(p),
                                              _arr(qhat_inv_modq), _arr(qhat_modp), _opt_ptr(o), ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h is not None:
            _check(lib().ofhe_hip_bconv_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def switch(self, x: int, out: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_approx_switch_crt_basis(self._h, _vp(x), _vp(out), int(batch), _vp(stream or None)))


def switch_modulus(ctx: Context, src: int, dst: int, n: int, old_q: int, new_q: int, stream: int = 0) -> None:
    """NativeVectorT::SwitchModulus on n words of device memory."""
    _check(lib().ofhe_hip_switch_modulus(ctx.handle, _vp(src), _vp(dst), int(n), int(old_q), int(new_q),
                                         _vp(stream or None)))


def approx_mod_up(plan_q: NTTPlan, plan_p: NTTPlan, q_to_p: BaseConverter, eval_form: bool, x: int, out: int,
                  batch: int = 1, stream: int = 0) -> None:
    """ApproxModUp: x [batch][Q][N] -> out [batch][Q+P][N] (evaluation form)."""
    _check(lib().ofhe_hip_approx_mod_up(plan_q.handle, plan_p.handle, q_to_p._h, 1 if eval_form else 0, _vp(x),
                                        _vp(out), int(batch), _vp(stream or None)))


def approx_mod_down(plan_q: NTTPlan, plan_p: NTTPlan, p_to_q: BaseConverter, p_inv_modq: Sequence[int], t: int,
                    x: int, out: int, batch: int = 1, stream: int = 0) -> None:
    """ApproxModDown: x [batch][Q+P][N] -> out [batch][Q][N] (evaluation form)."""
    if len(p_inv_modq) != plan_q.towers:
        raise MathError("p_inv_modq needs one entry per Q tower")
    _check(lib().ofhe_hip_approx_mod_down(plan_q.handle, plan_p.handle, p_to_q._h, _arr(p_inv_modq), int(t),
                                          _vp(x), _vp(out), int(batch), _vp(stream or None)))


class KeySwitch:
    """HYBRID key switching for ring 2**log_n, ciphertext moduli q (with roots
    rq), special moduli p (roots rp) and num_part_q digits."""

    def __init__(self, ctx: Context, log_n: int, q: Sequence[int], rq: Sequence[int], p: Sequence[int],
                 rp: Sequence[int], num_part_q: int, options: "KsOptions" = None):
        self.ctx = ctx
        self.log_n, self.n = int(log_n), 1 << int(log_n)
        self.q, self.p = [int(v) for v in q], [int(v) for v in p]
        self.size_q, self.size_p = len(self.q), len(self.p)
        self.num_part_q = int(num_part_q)
        h = _vp()
        self.options = options
        _check(lib().ofhe_hip_ks_create_ex(ctx.handle, self.log_n, self.size_q, _arr(q), _arr(rq), self.size_p,
                                           _arr(p), _arr(rp), self.num_part_q, _opt_ptr(options), ctypes.byref(h)))
        self._h = h

    def close(self) -> None:
        if self._h is not None:
            _check(lib().ofhe_hip_ks_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def digits(self, size_ql: int):
        """(alpha, beta) at level size_ql."""
        a, b = ctypes.c_uint32(0), ctypes.c_uint32(0)
        _check(lib().ofhe_hip_ks_digits(self._h, int(size_ql), ctypes.byref(a), ctypes.byref(b)))
        return a.value, b.value

    def precompute(self, size_ql: int, c: int, digits: int, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ks_precompute(self._h, int(size_ql), _vp(c), _vp(digits), int(batch),
                                            _vp(stream or None)))

    def fast_core_ext(self, size_ql: int, digits: int, key_b: int, key_a: int, ct0: int, ct1: int,
                      batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ks_fast_core_ext(self._h, int(size_ql), _vp(digits), _vp(key_b), _vp(key_a),
                                               _vp(ct0), _vp(ct1), int(batch), _vp(stream or None)))

    def mod_down(self, size_ql: int, x: int, out: int, t: int = 0, batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ks_mod_down(self._h, int(size_ql), _vp(x), _vp(out), int(t), int(batch),
                                          _vp(stream or None)))

    def core(self, size_ql: int, c: int, key_b: int, key_a: int, out0: int, out1: int, t: int = 0,
             batch: int = 1, stream: int = 0) -> None:
        _check(lib().ofhe_hip_ks_core(self._h, int(size_ql), _vp(c), _vp(key_b), _vp(key_a), _vp(out0),
                                      _vp(out1), int(t), int(batch), _vp(stream or None)))


def comm_unique_id() -> bytes:
    """Rank 0's RCCL unique id (OFHE_COMM_ID_BYTES), to be sent to the others."""
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    _check(lib().ofhe_hip_comm_unique_id(buf))
    return buf.raw


class Comm:
    """RCCL communicator of this process's device (ofhe_hip_comm_init).
    Collective: every rank constructs it with the same id."""

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise MathError(f"unique id must be {COMM_ID_BYTES} bytes")
        h = _vp()
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _check(lib().ofhe_hip_comm_init(ctx.handle, int(nranks), int(rank), buf, ctypes.byref(h)))
        self._h, self._ctx, self.nranks, self.rank = h, ctx, nranks, rank

    def bcast_evalkey(self, key_ptr: int, words: int, root: int = 0, stream: int = 0) -> None:
        """In-place broadcast of `words` u64 of device memory from `root`."""
        if self._h is None:
            raise MathError("communicator destroyed")
        _check(lib().ofhe_hip_bcast_evalkey(self._h, _vp(key_ptr or None), int(words), int(root),
                                            _vp(stream or None)))

    def close(self) -> None:
        if self._h is not None:
            _check(lib().ofhe_hip_comm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
