"""CPU ORACLE loader -- TEST INFRASTRUCTURE ONLY.

Loads oracle/build/libntt_oracle.so (a C restatement of the reference
NTT.cu, see ntt_oracle.h for the file:line map) and adds two independent
numpy definitions (O(n^2) transform and schoolbook negacyclic product).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libntt_oracle.so")

PARAM_SETS = {"ref": 0, "p-I": 1, "p-III": 2, "p-III-4096": 3, "p-III-8192": 4}

_u32p = ctypes.POINTER(ctypes.c_uint32)
_lib = None


def build() -> str:
    """Compile the oracle with its own Makefile (gcc, no reference sources)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)

        class Params(ctypes.Structure):
            _fields_ = [(k, ctypes.c_uint32) for k in
                        ("n", "logn", "q", "psi", "omega", "omega_inv", "n_inv")]

        L.Params = Params
        L.oracle_params_get.argtypes = [ctypes.c_int, ctypes.POINTER(Params)]
        L.oracle_bitrev.restype = ctypes.c_uint32
        L.oracle_bitrev.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_tables.argtypes = [ctypes.c_int] + [_u32p] * 5
        L.oracle_barrett_red_ref.restype = ctypes.c_uint32
        L.oracle_barrett_red_ref.argtypes = [ctypes.c_uint64]
        for nm in ("oracle_radix2NTT", "oracle_radix2INTT", "oracle_radix2NTTGS", "oracle_radix2INTTGS"):
            getattr(L, nm).argtypes = [_u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_bit_reverse_copy.argtypes = [_u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        for nm in ("oracle_poly_ntt", "oracle_poly_invntt", "oracle_poly_invntt_ct"):
            getattr(L, nm).argtypes = [_u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_poly_mul.argtypes = [_u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_pointwise.argtypes = [_u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_ntt_direct.argtypes = [_u32p, _u32p, ctypes.c_int]
        L.oracle_schoolbook_negacyclic.argtypes = [_u32p, _u32p, _u32p, ctypes.c_int]
        L.oracle_gpu_ct_gs_polymul.argtypes = [_u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_gpu_ct_ct_polymul.argtypes = [_u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_int]
        L.oracle_fill_uniform.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64]
        for nm in ("oracle_nussbaumer", "oracle_naive_negacyclic"):
            getattr(L, nm).argtypes = [_u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]
        L.oracle_m32_canon.restype = ctypes.c_uint32
        L.oracle_m32_canon.argtypes = [ctypes.c_uint32]
        L.oracle_time_op.restype = ctypes.c_double
        L.oracle_time_op.argtypes = [ctypes.c_int, _u32p, _u32p, _u32p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int]
        L.oracle_time_fwd_inv.restype = ctypes.c_double
        L.oracle_time_fwd_inv.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        _lib = L
    return _lib


def _ps(param_set) -> int:
    return PARAM_SETS[param_set] if isinstance(param_set, str) else int(param_set)


def _ptr(a: np.ndarray):
    assert a.dtype == np.uint32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u32p)


def params(param_set) -> dict:
    L = lib()
    p = L.Params()
    if L.oracle_params_get(_ps(param_set), ctypes.byref(p)) != 0:
        raise ValueError(f"bad param set {param_set}")
    return {k: getattr(p, k) for k, _ in p._fields_}


def tables(param_set) -> dict:
    n = params(param_set)["n"]
    out = {k: np.zeros(n, np.uint32) for k in ("bitrev_tbl", "Phi", "invPhi", "tf0", "ti0")}
    lib().oracle_tables(_ps(param_set), *(_ptr(out[k]) for k in ("bitrev_tbl", "Phi", "invPhi", "tf0", "ti0")))
    return out


def _batched(x: np.ndarray, n: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.uint32).copy()
    assert x.size % n == 0
    return x


def poly_ntt(x, param_set):
    n = params(param_set)["n"]
    y = _batched(x, n)
    lib().oracle_poly_ntt(_ptr(y), y.size // n, _ps(param_set))
    return y.reshape(np.shape(x))


def poly_invntt(X, param_set):
    n = params(param_set)["n"]
    y = _batched(X, n)
    lib().oracle_poly_invntt(_ptr(y), y.size // n, _ps(param_set))
    return y.reshape(np.shape(X))


def poly_invntt_ct(X, param_set):
    n = params(param_set)["n"]
    y = _batched(X, n)
    lib().oracle_poly_invntt_ct(_ptr(y), y.size // n, _ps(param_set))
    return y.reshape(np.shape(X))


def bit_reverse_copy(x, param_set):
    """bit_reverse_copy (NTT.cu:81-91) restated in C: out[t] = in[brv(t)]"""
    n = params(param_set)["n"]
    x = _batched(x, n)
    y = np.zeros_like(x)
    lib().oracle_bit_reverse_copy(_ptr(x), _ptr(y), x.size // n, _ps(param_set))
    return y


def poly_mul(a, b, param_set):
    n = params(param_set)["n"]
    a = _batched(a, n)
    b = _batched(b, n)
    c = np.zeros_like(a)
    lib().oracle_poly_mul(_ptr(c), _ptr(a), _ptr(b), a.size // n, _ps(param_set))
    return c


def pointwise(a, b, param_set):
    a = np.ascontiguousarray(a, np.uint32)
    b = np.ascontiguousarray(b, np.uint32)
    c = np.zeros_like(a)
    lib().oracle_pointwise(_ptr(c), _ptr(a), _ptr(b), a.size, _ps(param_set))
    return c


def gpu_ct_gs_polymul(x, y, param_set):
    n = params(param_set)["n"]
    x = _batched(x, n)
    y = _batched(y, n)
    z = np.zeros_like(x)
    lib().oracle_gpu_ct_gs_polymul(_ptr(x), _ptr(y), _ptr(z), x.size // n, _ps(param_set))
    return z


def gpu_ct_ct_polymul(x, y, param_set):
    n = params(param_set)["n"]
    x = _batched(x, n)
    y = _batched(y, n)
    z = np.zeros_like(x)
    lib().oracle_gpu_ct_ct_polymul(_ptr(x), _ptr(y), _ptr(z), x.size // n, _ps(param_set))
    return z


def ntt_direct_c(x, param_set):
    n = params(param_set)["n"]
    x = np.ascontiguousarray(x, np.uint32)
    X = np.zeros(n, np.uint32)
    lib().oracle_ntt_direct(_ptr(x), _ptr(X), _ps(param_set))
    return X


def fill_uniform(batch: int, param_set, seed: int, first_poly: int = 0) -> np.ndarray:
    n = params(param_set)["n"]
    x = np.zeros(batch * n, np.uint32)
    lib().oracle_fill_uniform(_ptr(x), batch, _ps(param_set), seed & (2**64 - 1), first_poly)
    return x.reshape(batch, n)


def time_fwd_inv(x: np.ndarray, param_set, threads: int = 1, reps: int = 1) -> float:
    n = params(param_set)["n"]
    y = _batched(x, n)
    return lib().oracle_time_fwd_inv(_ptr(y), y.size // n, _ps(param_set), threads, reps)


TIME_OPS = {"fwdinv": 0, "fwd": 1, "inv": 2, "polymul": 3, "nussbaumer_m32": 4, "nussbaumer_q": 5}


def time_op(op: str, x: np.ndarray, param_set, threads: int = 1, reps: int = 1, y: np.ndarray = None) -> float:
    """Wall seconds of `reps` passes of the reference's serial CPU path `op`
    (oracle_time_op) over the polys of x (and y for the products), split
    across `threads` pthreads, on copies (the inputs are not modified)."""
    n = params(param_set)["n"]
    xa = _batched(x, n)
    ya = za = None
    if op in ("polymul", "nussbaumer_m32", "nussbaumer_q"):
        ya = _batched(y, n)
        za = np.zeros_like(xa)
    t = lib().oracle_time_op(TIME_OPS[op], _ptr(xa), _ptr(ya) if ya is not None else None,
                             _ptr(za) if za is not None else None, xa.size // n, _ps(param_set), threads, reps)
    if t < 0:
        raise ValueError(f"oracle_time_op({op}) failed")
    return t


M32 = 0xFFFFFFFF   # the reference's Nussbaumer ring Z/(2^32-1) (NTT.cu:102-134)


def _ring_q(ring, n):
    """ring: "m32" (mod 2^32-1) or a param-set name / q (mod q)."""
    if ring == "m32":
        return 0
    if isinstance(ring, str):
        return params(ring)["q"]
    return int(ring)


def nussbaumer(x, y, n: int, ring="m32") -> np.ndarray:
    """nussbaumer_fft (NTT.cu:167-277) restated, m=32, r=n/32, batched.

    ring "m32": the reference's ones'-complement ring, op for op (so
    0xFFFFFFFF can appear as a second zero; compare via m32_canon)."""
    x = _batched(x, n)
    y = _batched(y, n)
    z = np.zeros_like(x)
    rc = lib().oracle_nussbaumer(_ptr(z), _ptr(x), _ptr(y), x.size // n, n, _ring_q(ring, n))
    assert rc == 0
    return z.reshape(-1, n)


def naive_negacyclic(x, y, n: int, ring="m32") -> np.ndarray:
    """naive (NTT.cu:147-165) at full length n, batched."""
    x = _batched(x, n)
    y = _batched(y, n)
    z = np.zeros_like(x)
    rc = lib().oracle_naive_negacyclic(_ptr(z), _ptr(x), _ptr(y), x.size // n, n, _ring_q(ring, n))
    assert rc == 0
    return z.reshape(-1, n)


def m32_canon(a) -> np.ndarray:
    """canonical residue mod 2^32-1 (normalize, NTT.cu:125): 0xFFFFFFFF -> 0"""
    a = np.asarray(a, np.uint32)
    return np.where(a == np.uint32(M32), np.uint32(0), a)


# ---------------- independent numpy definitions ----------------

def ntt_direct_np(x: np.ndarray, param_set) -> np.ndarray:
    """X[k] = sum_i x_i psi^{(2k+1) i} mod q  (O(n^2), vectorised; SURVEY 8 FWD)."""
    p = params(param_set)
    n, q, psi = p["n"], p["q"], p["psi"]
    pw = np.zeros(2 * n, np.uint64)
    acc = 1
    for e in range(2 * n):
        pw[e] = acc
        acc = acc * psi % q
    k = np.arange(n, dtype=np.uint64)[:, None]
    i = np.arange(n, dtype=np.uint64)[None, :]
    M = pw[((2 * k + 1) * i) % (2 * n)]
    xs = np.asarray(x, np.uint64).reshape(-1, n)
    out = np.empty(xs.shape, np.uint32)
    for r in range(xs.shape[0]):
        out[r] = (((M * xs[r][None, :]) % q).sum(axis=1) % q).astype(np.uint32)
    return out.reshape(np.shape(x))


def schoolbook_m32_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """a*b mod (x^n + 1, 2^32-1), one polynomial, exact Python-integer convolution."""
    a = [int(v) for v in np.asarray(a, np.uint32)]
    b = np.asarray(b, np.uint32).astype(object)
    n = len(a)
    full = np.convolve(np.array(a, dtype=object), b)
    c = full[:n].copy()
    c[: n - 1] -= full[n:]
    return np.array([int(v) % M32 for v in c], dtype=np.uint32)


def schoolbook_np(a: np.ndarray, b: np.ndarray, param_set) -> np.ndarray:
    """a*b mod (x^n + 1, q), one polynomial, numpy."""
    p = params(param_set)
    n, q = p["n"], p["q"]
    a = np.asarray(a, np.uint64)
    b = np.asarray(b, np.uint64)
    c = np.zeros(n, np.uint64)
    for i in range(n):
        ai = int(a[i])
        if ai == 0:
            continue
        prod = (ai * b) % q
        c[i:] = (c[i:] + prod[: n - i]) % q
        if i:
            c[:i] = (c[:i] + (q - prod[n - i:])) % q
    return c.astype(np.uint32)
