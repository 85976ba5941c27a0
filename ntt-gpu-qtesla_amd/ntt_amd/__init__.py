"""ntt_amd -- Python host binding of the MI355X batched negacyclic NTT engine.

Thin ctypes layer over the C ABI in include/qtesla_ntt.h (libqtesla_ntt.so,
built in-tree for gfx950).  PyTorch is used only as plumbing: device memory
(int32 tensors carry the uint32 coefficient bit patterns), the current HIP
stream and torch.distributed.  There is no CPU fallback: if the HIP library
is missing every call raises.

Names and argument meaning follow the reference's GPU pipeline
(benlwk/ntt-gpu-qTESLA NTT.cu):
  poly_ntt      -- bit_reverse_copy_tbl_Phi_gpu + radix2NTT_gpu0/1 (NTT.cu:2388-2400)
  poly_invntt   -- GS_radix2INTT_gpu0/2 + bit_reverse_copy_tbl_invPhi_gpu (:2415-2425)
  poly_mul      -- the whole CT-GS poly-mul driver (test_NTT_CT_GS_nega_gpu, :2358)
  poly_pointwise -- pointwise_mult (:1155-1160)
  poly_mul_nussbaumer -- nussbaumer_fft (:167-277), batched, n = 1024 / 2048
  poly_ntt_bitrev / poly_invntt_bitrev -- the CT-CT ordering: bit-reversed
                   NTT domain (radix2INTT_gpu0/1/2 on bit-reversed input, :2240-2249)

Every torch wrapper runs on its tensors' device (all operands must share
one) and, by default, on that device's current stream.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.environ.get("NTT_AMD_LIB") or os.path.join(ROOT_DIR, "lib", "libqtesla_ntt.so")
HEADER_PATH = os.path.join(os.path.dirname(ROOT_DIR), "include", "qtesla_ntt.h")

PARAM_SETS = {"ref": 0, "p-I": 1, "p-III": 2, "p-III-4096": 3, "p-III-8192": 4}

NTT_OK = 0
NTT_ERR_PARAM = -1
NTT_ERR_NULL = -2
NTT_ERR_ALIGN = -3
NTT_ERR_HIP = -4
NTT_ERR_SIZE = -5
NTT_ERR_ALIAS = -6

RINGS = {"q": 0, "m32": 1}   # NTT_RING_Q, NTT_RING_M32


class NTTError(RuntimeError):
    def __init__(self, code: int, where: str):
        self.code = code
        msg = lib().ntt_strerror(code).decode()
        if code == NTT_ERR_HIP:
            msg += f" (hipError {lib().ntt_last_hip_error()})"
        super().__init__(f"{where}: {msg} [{code}]")


_lib = None
_u32p = ctypes.POINTER(ctypes.c_uint32)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t


def lib():
    """Load libqtesla_ntt.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"HIP library {LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
        # One HIP runtime per process: torch ships its own libamdhip64, loaded
        # into the global scope when torch is imported.  Importing it first
        # makes this library's hip* references bind to that same runtime; a
        # second runtime initialised after torch's finds no device
        # (hipErrorNoDevice from the host-buffer context, measured).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.ntt_param_info.argtypes = [ctypes.c_int] + [_u32p] * 6
        L.ntt_get_tables.argtypes = [ctypes.c_int] + [_u32p] * 5
        for nm in ("poly_ntt", "poly_invntt"):
            getattr(L, nm).argtypes = [_vp, _vp, _sz, ctypes.c_int, _vp]
        for nm in ("poly_ntt_oop", "poly_invntt_oop", "poly_bitrev_copy", "poly_ntt_bitrev", "poly_invntt_bitrev"):
            getattr(L, nm).argtypes = [_vp, _vp, _sz, ctypes.c_int, _vp]
        for nm in ("poly_mul", "poly_mul_ntt", "poly_pointwise"):
            getattr(L, nm).argtypes = [_vp, _vp, _vp, _sz, ctypes.c_int, _vp]
        L.poly_mul_nussbaumer.argtypes = [_vp, _vp, _vp, _sz, ctypes.c_int, ctypes.c_int, _vp]
        L.ntt_fill_uniform.argtypes = [_vp, _sz, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, _vp]
        L.ntt_last_hip_error.restype = ctypes.c_int
        L.ntt_strerror.restype = ctypes.c_char_p
        L.ntt_strerror.argtypes = [ctypes.c_int]
        L.ntt_build_info.argtypes = [ctypes.c_char_p, _sz]
        L.ntt_sync_expiries.argtypes = [_u32p]
        L.ntt_small_batch_max.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_sz)]
        L.ntt_small_batch_radix.argtypes = [ctypes.c_int, ctypes.c_int, _sz, ctypes.POINTER(ctypes.c_int)]
        L.ntt_host_ctx_create.argtypes = [ctypes.POINTER(_vp), ctypes.c_int, _sz, ctypes.c_int]
        L.ntt_host_ctx_destroy.argtypes = [_vp]
        for nm in ("poly_ntt_host", "poly_invntt_host"):
            getattr(L, nm).argtypes = [_vp, _vp, _vp, _sz]
        L.poly_mul_host.argtypes = [_vp, _vp, _vp, _vp, _sz]
        L.ntt_host_alloc.argtypes = [_sz]
        L.ntt_host_alloc.restype = _vp
        L.ntt_host_free.argtypes = [_vp]
        _lib = L
    return _lib


def _ps(param_set) -> int:
    return PARAM_SETS[param_set] if isinstance(param_set, str) else int(param_set)


def _check(rc: int, where: str):
    if rc != NTT_OK:
        raise NTTError(rc, where)


_PARAM_CACHE: dict = {}
_N_CACHE: dict = {}


def _n(param_set) -> int:
    """n of a parameter set, cached (the per-call wrappers' fast path)."""
    n = _N_CACHE.get(param_set)
    if n is None:
        n = _N_CACHE[param_set] = param_info(param_set)["n"]
    return n


def param_info(param_set) -> dict:
    """n, q, psi, omega, omega^-1, n^-1 of a parameter set (immutable: cached,
    so that the per-call wrappers cost no extra library call)."""
    ps = _ps(param_set)
    info = _PARAM_CACHE.get(ps)
    if info is None:
        vals = [ctypes.c_uint32() for _ in range(6)]
        _check(lib().ntt_param_info(ps, *[ctypes.byref(v) for v in vals]), "ntt_param_info")
        info = _PARAM_CACHE[ps] = dict(zip(("n", "q", "psi", "omega", "omega_inv", "n_inv"), (v.value for v in vals)))
    return dict(info)


def tables(param_set) -> dict:
    n = _n(param_set)
    names = ("bitrev_tbl", "Phi", "invPhi", "tf0", "ti0")
    out = {k: np.zeros(n, np.uint32) for k in names}
    _check(lib().ntt_get_tables(_ps(param_set), *(out[k].ctypes.data_as(_u32p) for k in names)), "ntt_get_tables")
    return out


def sync_expiries() -> int:
    """Expired bounded waits of the n = 4096 / 8192 kernels on the current
    device (0 unless a per-polynomial barrier broke; see qtesla_ntt.h)."""
    v = ctypes.c_uint32()
    _check(lib().ntt_sync_expiries(ctypes.byref(v)), "ntt_sync_expiries")
    return v.value


# entry points of the small-batch switch (NTT_OP_* in qtesla_ntt.h)
SWITCH_OPS = {"fwd": 0, "inv": 1, "fwd_br": 2, "inv_br": 3, "mul": 4, "mul_ntt": 5, "fwd_oop": 6, "inv_oop": 7}


def small_batch_max(param_set, op: str) -> int:
    """Largest batch for which entry point `op` (a SWITCH_OPS key) runs the
    small-batch kernels, one polynomial per workgroup (0: never)."""
    v = _sz()
    _check(lib().ntt_small_batch_max(_ps(param_set), SWITCH_OPS[op], ctypes.byref(v)), "ntt_small_batch_max")
    return v.value


def small_batch_radix(param_set, op: str, batch: int) -> int:
    """Radix of the one-polynomial-per-workgroup kernel entry point `op`
    runs at `batch` polynomials (4 / 8 / 16), 0 for the batch kernels."""
    v = ctypes.c_int()
    _check(lib().ntt_small_batch_radix(_ps(param_set), SWITCH_OPS[op], batch, ctypes.byref(v)), "ntt_small_batch_radix")
    return v.value


def build_info() -> str:
    buf = ctypes.create_string_buffer(1024)
    lib().ntt_build_info(buf, 1024)
    return buf.value.decode()


def build_hash() -> str:
    """Hash of the library sources the loaded .so was built from ("src=" field)."""
    info = build_info()
    return info.rsplit("src=", 1)[1].strip() if "src=" in info else "unknown"


# ---------------------------------------------------------------- raw API
# device pointers as ints, stream as int (hipStream_t) or None

def raw_poly_ntt(ptr: int, batch: int, param_set, stream=None):
    _check(lib().poly_ntt(ptr, None, batch, _ps(param_set), stream), "poly_ntt")


def raw_poly_invntt(ptr: int, batch: int, param_set, stream=None):
    _check(lib().poly_invntt(ptr, None, batch, _ps(param_set), stream), "poly_invntt")


def raw_poly_mul(c: int, a: int, b: int, batch: int, param_set, stream=None):
    _check(lib().poly_mul(c, a, b, batch, _ps(param_set), stream), "poly_mul")


# ------------------------------------------------------------- torch API

_TORCH = None
_INT_DTYPES = ()


def _torch():
    """torch, imported on first use (this module also serves torch-free
    ctypes callers) and then cached: the per-call wrappers below run once per
    polynomial in the signing loop's small calls."""
    global _TORCH, _INT_DTYPES
    if _TORCH is None:
        import torch
        _INT_DTYPES = (torch.int32, getattr(torch, "uint32", torch.int32))
        _TORCH = torch
    return _TORCH


def _device_of(*tensors):
    """The one device all operands live on (ValueError otherwise)."""
    if len(tensors) == 1 and getattr(tensors[0], "is_cuda", False):
        return tensors[0].device
    dev = None
    for t in tensors:
        if not getattr(t, "is_cuda", False):
            raise ValueError("ntt_amd operates on device tensors only (no CPU fallback)")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"operands on different devices: {dev} and {t.device}")
    return dev


def _stream(stream, device=None):
    if stream is None:
        torch = _torch()
        if isinstance(device, torch.device) and device.index is not None:
            return _current_raw_stream(device.index)
        return torch.cuda.current_stream(device).cuda_stream
    return getattr(stream, "cuda_stream", stream)


def _batch(t, n: int) -> int:
    _torch()
    if not t.is_cuda:
        raise ValueError("ntt_amd operates on device tensors only (no CPU fallback)")
    if t.dtype not in _INT_DTYPES:
        raise TypeError(f"expected int32/uint32 storage, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous (poly-major [batch][n])")
    numel = t.numel()
    if numel % n:
        raise ValueError(f"numel {numel} is not a multiple of n={n}")
    return numel // n


def _run(where: str, tensors, stream, call):
    """Check the operands, make their device current and call `call(stream)`."""
    dev = _device_of(*tensors)
    torch = _TORCH or _torch()
    if torch.cuda.current_device() == dev.index:   # already current: no device switch
        _check(call(_stream(stream, dev)), where)
        return
    with torch.cuda.device(dev):
        _check(call(_stream(stream, dev)), where)


def _same_batch(n: int, first, *others) -> int:
    b = _batch(first, n)
    for o in others:
        if _batch(o, n) != b:
            raise ValueError("batch mismatch")
    return b


def _inplace(name: str, t, param_set, stream):
    """The in-place transforms' call path, the signing loop's one-polynomial
    calls (config 1): the same checks as _batch / _run with fewer
    interpreter steps -- the device as an int (no torch.device object), no
    closure, the ctypes function looked up once -- 5.3 -> ~4 us per call
    against 3.25 us for a bare ctypes call (tools/call_overhead.py)."""
    n = _N_CACHE.get(param_set)
    if n is None:
        n = _n(param_set)
    torch = _TORCH or _torch()
    if not t.is_cuda or t.dtype not in _INT_DTYPES or not t.is_contiguous():
        _batch(t, n)   # raises the specific error
    numel = t.numel()
    if numel % n:
        _batch(t, n)
    fn = _FN.get(name)
    if fn is None:
        fn = _FN[name] = getattr(lib(), name)
    ps = PARAM_SETS[param_set] if isinstance(param_set, str) else int(param_set)
    dev = t.get_device()
    if torch.cuda.current_device() == dev:
        s = _current_raw_stream(dev) if stream is None else getattr(stream, "cuda_stream", stream)
        rc = fn(t.data_ptr(), None, numel // n, ps, s)
    else:
        with torch.cuda.device(dev):
            s = _current_raw_stream(dev) if stream is None else getattr(stream, "cuda_stream", stream)
            rc = fn(t.data_ptr(), None, numel // n, ps, s)
    if rc != NTT_OK:
        raise NTTError(rc, name)
    return t


_FN: dict = {}


def _current_raw_stream(dev: int):
    """The device's current stream handle as an int: torch's raw accessor
    where this torch build has it (no Stream object: ~1.4 us less per call,
    tools/call_overhead.py), else the public current_stream()."""
    raw = getattr(_TORCH._C, "_cuda_getCurrentRawStream", None)
    if raw is not None:
        return raw(dev)
    return _TORCH.cuda.current_stream(dev).cuda_stream


def poly_ntt(t, param_set, stream=None):
    """In-place forward negacyclic NTT of a [batch, n] device tensor."""
    return _inplace("poly_ntt", t, param_set, stream)


def poly_invntt(t, param_set, stream=None):
    """In-place inverse negacyclic NTT (includes n^-1 and psi^-i)."""
    return _inplace("poly_invntt", t, param_set, stream)


def _oop(name, out, inp, param_set, stream):
    n = _n(param_set)
    b = _same_batch(n, inp, out)
    fn = getattr(lib(), name)
    _run(name, (out, inp), stream, lambda s: fn(out.data_ptr(), inp.data_ptr(), b, _ps(param_set), s))
    return out


def poly_ntt_oop(out, inp, param_set, stream=None):
    return _oop("poly_ntt_oop", out, inp, param_set, stream)


def poly_invntt_oop(out, inp, param_set, stream=None):
    return _oop("poly_invntt_oop", out, inp, param_set, stream)


def poly_ntt_bitrev(out, inp, param_set, stream=None):
    """Forward NTT with bit-reversed output order: out[b, t] = X[b, brv(t)]."""
    return _oop("poly_ntt_bitrev", out, inp, param_set, stream)


def poly_invntt_bitrev(out, inp, param_set, stream=None):
    """Inverse NTT of a bit-reversed-order input (inp[b, t] = X[b, brv(t)])."""
    return _oop("poly_invntt_bitrev", out, inp, param_set, stream)


def poly_bitrev_copy(out, inp, param_set, stream=None):
    """out[b, t] = inp[b, brv(t)] (bit_reverse_copy_tbl_gpu); out may be inp."""
    return _oop("poly_bitrev_copy", out, inp, param_set, stream)


def _mul(name, c, a, b, param_set, stream, *extra):
    n = _n(param_set)
    nb = _same_batch(n, a, b, c)
    fn = getattr(lib(), name)
    _run(name, (c, a, b), stream,
         lambda s: fn(c.data_ptr(), a.data_ptr(), b.data_ptr(), nb, _ps(param_set), *extra, s))
    return c


def poly_mul(c, a, b, param_set, stream=None):
    """c = a*b mod (x^n + 1, q), fused single launch."""
    return _mul("poly_mul", c, a, b, param_set, stream)


def poly_mul_ntt(c, a, bhat, param_set, stream=None):
    """c = a*b mod (x^n + 1, q) with bhat = poly_ntt(b) given (NTT domain)."""
    return _mul("poly_mul_ntt", c, a, bhat, param_set, stream)


def poly_mul_nussbaumer(c, a, b, param_set, ring="q", stream=None):
    """c = a*b mod x^n + 1 by the Nussbaumer algorithm (nussbaumer_fft, NTT.cu:167-277).

    ring "q": mod param_set's q (equals poly_mul); ring "m32": mod 2^32 - 1,
    the reference's ring.  Buffers must be 16-byte aligned."""
    r = RINGS[ring] if isinstance(ring, str) else int(ring)
    return _mul("poly_mul_nussbaumer", c, a, b, param_set, stream, r)


def poly_pointwise(c, a, b, param_set, stream=None):
    return _mul("poly_pointwise", c, a, b, param_set, stream)


def fill_uniform(t, param_set, seed: int, first_poly: int = 0, stream=None):
    """Device-side counter-based uniform coefficients in [0, q)."""
    n = _n(param_set)
    b = _batch(t, n)
    _run("ntt_fill_uniform", (t,), stream,
         lambda s: lib().ntt_fill_uniform(t.data_ptr(), b, _ps(param_set), seed & (2**64 - 1), first_poly, s))
    return t


def to_numpy_u32(t) -> np.ndarray:
    return t.detach().cpu().numpy().view(np.uint32)


def from_numpy_u32(a: np.ndarray, device="cuda"):
    torch = _torch()
    return torch.from_numpy(np.ascontiguousarray(a, np.uint32).view(np.int32)).to(device)


# ------------------------------------------------------- host-buffer API
# Host -> host operation pipelined over HIP streams (include/qtesla_ntt.h,
# "host-buffer (streamed) operation"; the reference's PCIe-inclusive driver
# body NTT.cu:2384-2428).  Arrays are numpy uint32, C-contiguous [batch, n].

class HostContext:
    """Owns the device / pinned staging buffers of ntt_host_ctx_create."""

    def __init__(self, param_set, chunk_polys: int = 0, nslots: int = 0):
        self.param_set = param_set
        self.n = _n(param_set)
        h = _vp()
        _check(lib().ntt_host_ctx_create(ctypes.byref(h), _ps(param_set), chunk_polys, nslots),
               "ntt_host_ctx_create")
        self._h = h

    def close(self):
        if self._h is not None and self._h.value:
            _check(lib().ntt_host_ctx_destroy(self._h), "ntt_host_ctx_destroy")
        self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _arr(self, x, name):
        if not isinstance(x, np.ndarray) or x.dtype != np.uint32 or not x.flags["C_CONTIGUOUS"]:
            raise TypeError(f"{name}: expected a C-contiguous numpy uint32 array")
        if x.size % self.n:
            raise ValueError(f"{name}: size {x.size} is not a multiple of n={self.n}")
        return x.size // self.n

    def ntt(self, out, inp):
        b = self._arr(inp, "inp")
        if self._arr(out, "out") != b:
            raise ValueError("out/in batch mismatch")
        _check(lib().poly_ntt_host(self._h, out.ctypes.data, inp.ctypes.data, b), "poly_ntt_host")
        return out

    def invntt(self, out, inp):
        b = self._arr(inp, "inp")
        if self._arr(out, "out") != b:
            raise ValueError("out/in batch mismatch")
        _check(lib().poly_invntt_host(self._h, out.ctypes.data, inp.ctypes.data, b), "poly_invntt_host")
        return out

    def mul(self, c, a, b):
        nb = self._arr(a, "a")
        if self._arr(b, "b") != nb or self._arr(c, "c") != nb:
            raise ValueError("batch mismatch")
        _check(lib().poly_mul_host(self._h, c.ctypes.data, a.ctypes.data, b.ctypes.data, nb), "poly_mul_host")
        return c


def host_empty(count: int) -> np.ndarray:
    """A numpy uint32 array of `count` words in pinned host memory (ntt_host_alloc).

    The memory is freed when the last array viewing it is garbage-collected
    (the ctypes buffer below is the numpy base of every view)."""
    words = max(int(count), 1)
    ptr = lib().ntt_host_alloc(words * 4)
    if not ptr:
        raise MemoryError("ntt_host_alloc failed")

    def _free(self):
        if getattr(self, "_ptr", None):
            lib().ntt_host_free(self._ptr)
            self._ptr = None

    buf_t = type("PinnedU32", (ctypes.c_uint32 * words,), {"__del__": _free})
    buf = buf_t.from_address(ptr)
    buf._ptr = ptr
    return np.frombuffer(buf, dtype=np.uint32, count=int(count))
