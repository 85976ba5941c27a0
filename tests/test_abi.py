"""The C-ABI library loads, exports every symbol include/qtesla_ntt.h declares,
and validates arguments before touching the GPU (no compute calls here)."""
import re

import pytest


def header_functions(ntt):
    src = open(ntt.HEADER_PATH).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(\w+)\s*\(", src, flags=re.M)))


def test_exports_every_declared_symbol(ntt):
    fns = header_functions(ntt)
    assert {"poly_ntt", "poly_invntt", "poly_mul", "poly_pointwise", "ntt_get_tables"} <= set(fns)
    L = ntt.lib()
    for f in fns:
        assert hasattr(L, f), f"{f} declared in qtesla_ntt.h but not exported"


def test_header_param_sets_match_library(ntt):
    """Every NTT_PARAM_* the header defines names a set the library knows, with
    the n its comment states (param sets 3 / 4: the n = 4096 / 8192 transforms)."""
    src = open(ntt.HEADER_PATH).read()
    defs = re.findall(r"#define NTT_PARAM_(\w+) (\d+)\s*/\*\s*n = (\d+), q = (\d+)", src)
    assert len(defs) == len(ntt.PARAM_SETS), defs
    by_id = {v: k for k, v in ntt.PARAM_SETS.items()}
    for _, ps, n, q in defs:
        info = ntt.param_info(by_id[int(ps)])
        assert (info["n"], info["q"]) == (int(n), int(q))


def test_error_codes_before_any_gpu_work(ntt):
    L = ntt.lib()
    fake = 0x10000  # never dereferenced: validation fails first
    assert L.poly_ntt(fake, None, 1, 5, None) == ntt.NTT_ERR_PARAM
    assert L.poly_mul_nussbaumer(fake, fake, fake, 1, 3, 0, None) == ntt.NTT_ERR_PARAM   # no Nussbaumer split at n > 2048
    assert L.poly_mul(fake + 8, fake, fake + 0x100000, 1, 3, None) == ntt.NTT_ERR_ALIAS   # n = 4096 product: checked
    assert L.poly_ntt(None, None, 1, 0, None) == ntt.NTT_ERR_NULL
    assert L.poly_ntt(fake + 2, None, 1, 0, None) == ntt.NTT_ERR_ALIGN
    assert L.poly_ntt(None, None, 0, 0, None) == ntt.NTT_OK      # empty batch is a no-op
    assert L.poly_invntt(fake, None, 1, -1, None) == ntt.NTT_ERR_PARAM
    assert L.poly_ntt_oop(fake, fake + 4, 2, 0, None) == ntt.NTT_ERR_ALIAS   # partial overlap
    assert L.poly_mul(fake, None, fake, 1, 2, None) == ntt.NTT_ERR_NULL
    assert L.poly_mul(fake + 8, fake, fake + 0x100000, 1, 2, None) == ntt.NTT_ERR_ALIAS
    assert L.poly_pointwise(fake + 4, fake, fake + 0x100000, 1, 2, None) == ntt.NTT_ERR_ALIGN
    assert L.ntt_fill_uniform(None, 1, 1, 0, 0, None) == ntt.NTT_ERR_NULL
    assert L.poly_ntt(fake, None, 1 << 31, 2, None) == ntt.NTT_ERR_SIZE
    assert L.poly_ntt_bitrev(fake, fake + 4, 2, 0, None) == ntt.NTT_ERR_ALIAS
    assert L.poly_invntt_bitrev(None, fake, 1, 2, None) == ntt.NTT_ERR_NULL
    for code in (0, -1, -2, -3, -4, -5, -6):
        assert L.ntt_strerror(code)
    with pytest.raises(KeyError):
        ntt.param_info("p-II")


def test_param_info(ntt):
    assert ntt.param_info("ref")["q"] == 8404993
    assert ntt.param_info("p-I")["q"] == 343576577 and ntt.param_info("p-I")["n"] == 1024
    assert ntt.param_info("p-III")["q"] == 856145921 and ntt.param_info("p-III")["n"] == 2048
    assert ntt.param_info("p-III-4096")["n"] == 4096 and ntt.param_info("p-III-8192")["n"] == 8192
    assert ntt.param_info("p-III-8192")["q"] == 856145921
    assert "gfx950" in ntt.build_info()
    h = ntt.build_hash()
    assert len(h) == 16 and all(c in "0123456789abcdef" for c in h), h


def test_cpu_tensor_rejected(ntt):
    torch = pytest.importorskip("torch")
    with pytest.raises(ValueError):
        ntt.poly_ntt(torch.zeros(2048, dtype=torch.int32), "p-III")


def test_host_ctx_validation_without_gpu(ntt):
    import ctypes
    L = ntt.lib()
    h = ctypes.c_void_p()
    assert L.ntt_host_ctx_create(None, 0, 0, 0) == ntt.NTT_ERR_NULL
    assert L.ntt_host_ctx_create(ctypes.byref(h), 5, 0, 0) == ntt.NTT_ERR_PARAM
    assert L.ntt_host_ctx_create(ctypes.byref(h), 0, 0, 9) == ntt.NTT_ERR_SIZE
    assert L.ntt_host_ctx_destroy(None) == ntt.NTT_ERR_NULL
    assert L.poly_mul_host(None, None, None, None, 1) == ntt.NTT_ERR_NULL
