"""Host-buffer (streamed) operation, SURVEY.md §8(f) row 4: host -> host
poly_ntt / poly_invntt / poly_mul pipelined over HIP streams
(ntt-gpu-qtesla_amd/csrc/host_stream.cpp), bit-exact vs the CPU oracle.

Covers pageable (numpy) and pinned (ntt_host_alloc) buffers, batches that are
not multiples of the chunk, fewer chunks than streams, in-place calls, the
empty batch and argument errors.  The reference's equivalent is its
PCIe-inclusive driver body (NTT.cu:2384-2428).
"""
import numpy as np
import pytest

from conftest import PARAM_SETS

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("pinned", [False, True])
def test_host_mul_and_transforms(ntt, oracle, dev, ps, pinned):
    n = ntt.param_info(ps)["n"]
    batch = 37   # chunk 8 x 3 streams: 5 chunks, ragged last one, slots reused
    a = oracle.fill_uniform(batch, ps, 0x5EED0101, 0)
    b = oracle.fill_uniform(batch, ps, 0x5EED0102, 0)

    def buf(src=None):
        if pinned:
            x = ntt.host_empty(batch * n).reshape(batch, n)
        else:
            x = np.empty((batch, n), np.uint32)
        if src is not None:
            x[...] = src
        return x

    with ntt.HostContext(ps, chunk_polys=8, nslots=3) as ctx:
        c = buf()
        ctx.mul(c, buf(a), buf(b))
        assert np.array_equal(c, oracle.poly_mul(a, b, ps))
        X = buf()
        ctx.ntt(X, buf(a))
        assert np.array_equal(X, oracle.poly_ntt(a, ps))
        x = buf()
        ctx.invntt(x, X)
        assert np.array_equal(x, a)
        # in place
        t = buf(a)
        ctx.ntt(t, t)
        assert np.array_equal(t, X)
        ctx.invntt(t, t)
        assert np.array_equal(t, a)


def test_host_mixed_pinned_pageable_and_default_ctx(ntt, oracle, dev):
    ps = "p-III"
    n = 2048
    batch = 5     # one chunk with the default chunk size, fewer chunks than streams
    a = oracle.fill_uniform(batch, ps, 7, 0)
    b = oracle.fill_uniform(batch, ps, 8, 0)
    pa = ntt.host_empty(batch * n).reshape(batch, n)
    pa[...] = a
    with ntt.HostContext(ps) as ctx:
        c = np.zeros((batch, n), np.uint32)
        ctx.mul(c, pa, b)   # pinned a, pageable b -> staged path
        assert np.array_equal(c, oracle.poly_mul(a, b, ps))
        pc = ntt.host_empty(batch * n).reshape(batch, n)
        ctx.mul(pc, pa, pa)   # all pinned
        assert np.array_equal(pc, oracle.poly_mul(a, a, ps))


def test_host_errors(ntt, dev):
    L = ntt.lib()
    with ntt.HostContext("p-I", chunk_polys=4, nslots=2) as ctx:
        h = ctx._h
        z = np.zeros(1024, np.uint32)
        assert L.poly_ntt_host(h, z.ctypes.data, z.ctypes.data, 0) == ntt.NTT_OK
        assert L.poly_ntt_host(h, None, z.ctypes.data, 1) == ntt.NTT_ERR_NULL
        assert L.poly_mul_host(h, z.ctypes.data, z.ctypes.data, None, 1) == ntt.NTT_ERR_NULL
        assert L.poly_ntt_host(h, z.ctypes.data + 2, z.ctypes.data, 1) == ntt.NTT_ERR_ALIGN
        with pytest.raises(ValueError):
            ctx.ntt(np.zeros(1000, np.uint32), np.zeros(1000, np.uint32))
    assert L.poly_ntt_host(None, None, None, 1) == ntt.NTT_ERR_NULL
    with pytest.raises(ntt.NTTError):
        ntt.HostContext(7)
    with pytest.raises(ntt.NTTError):
        ntt.HostContext("p-I", nslots=9)
