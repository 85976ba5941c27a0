"""GPU parity of the batched Nussbaumer product (poly_mul_nussbaumer) -- config 5.

Oracle: oracle/nussbaumer_oracle.c, the reference's nussbaumer_fft
(NTT.cu:167-277) restated op for op and generalised to n = 2048, pinned by
the all-ones KAT of test_nussbaumer (NTT.cu:1987-2005), the full-length
`naive` (NTT.cu:147-165) and a big-integer schoolbook (tests/test_oracle_nussbaumer.py).
Ring Z/(2^32-1) results are compared as canonical residues (the reference
may print 0xFFFFFFFF for zero); ring Z/q must equal poly_mul bit for bit.
"""
import os

import numpy as np
import pytest
import torch

from conftest import PARAM_SETS

pytestmark = pytest.mark.gpu
M32 = 0xFFFFFFFF


def _dev(ntt, a, dev):
    return ntt.from_numpy_u32(np.ascontiguousarray(a, np.uint32), dev)


def _n(ps):
    return 2048 if ps == "p-III" else 1024


def _rand_words(rng, shape):
    x = rng.integers(0, 1 << 32, shape, dtype=np.uint64).astype(np.uint32)
    x.reshape(-1)[::97] = M32          # the second zero of Z/(2^32-1)
    x.reshape(-1)[1::101] = 0
    return x


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 2, 3, 37])
def test_m32_random_vs_oracle(ntt, oracle, dev, ps, batch):
    n = _n(ps)
    rng = np.random.default_rng(1000 + batch + n)
    x, y = _rand_words(rng, (batch, n)), _rand_words(rng, (batch, n))
    c = torch.empty(batch * n, dtype=torch.int32, device=dev)
    ntt.poly_mul_nussbaumer(c, _dev(ntt, x, dev), _dev(ntt, y, dev), ps, "m32")
    got = ntt.to_numpy_u32(c).reshape(batch, n)
    assert np.array_equal(got, oracle.m32_canon(oracle.nussbaumer(x, y, n, "m32")))


# Z/(2^32-1) runs several units per workgroup with the next unit's words
# loaded during the current one (csrc/nussbaumer.hip, NUS_PPW_M32): batches
# of more than 2 units per pair slot (512 slots on 256 CUs) take that path,
# including partial last workgroups, a half-valid last n = 1024 unit (odd
# batch) and the in-place form (c == a; the prefetch reads the NEXT unit's a
# before this unit's stores, which never touch it)
@pytest.mark.parametrize("ps,batch", [("p-III", 1537), ("p-III", 4099), ("p-I", 3075), ("ref", 2049)])
def test_m32_multi_unit_workgroups(ntt, oracle, dev, ps, batch):
    n = _n(ps)
    rng = np.random.default_rng(2000 + batch + n)
    x, y = _rand_words(rng, (batch, n)), _rand_words(rng, (batch, n))
    c = torch.empty(batch * n, dtype=torch.int32, device=dev)
    ntt.poly_mul_nussbaumer(c, _dev(ntt, x, dev), _dev(ntt, y, dev), ps, "m32")
    got = ntt.to_numpy_u32(c).reshape(batch, n)
    assert np.array_equal(got, oracle.m32_canon(oracle.nussbaumer(x, y, n, "m32")))
    da = _dev(ntt, x, dev)
    ntt.poly_mul_nussbaumer(da, da, _dev(ntt, y, dev), ps, "m32")   # in place
    assert np.array_equal(ntt.to_numpy_u32(da).reshape(batch, n), got)


@pytest.mark.parametrize("n", [1024, 2048])
def test_m32_reference_kat(ntt, dev, n):
    """test_nussbaumer (NTT.cu:1987-2005): all-ones operands -> z[k] = 2k + 2 - n mod 2^32-1"""
    ps = "p-III" if n == 2048 else "ref"
    ones = np.ones((3, n), np.uint32)
    c = torch.empty(3 * n, dtype=torch.int32, device=dev)
    ntt.poly_mul_nussbaumer(c, _dev(ntt, ones, dev), _dev(ntt, ones, dev), ps, "m32")
    kat = np.array([(2 * k + 2 - n) % M32 for k in range(n)], np.uint32)
    got = ntt.to_numpy_u32(c).reshape(3, n)
    assert all(np.array_equal(g, kat) for g in got)


@pytest.mark.parametrize("ps", PARAM_SETS)
@pytest.mark.parametrize("batch", [1, 3, 64])
def test_q_ring_equals_poly_mul(ntt, oracle, dev, ps, batch):
    n, q = _n(ps), ntt.param_info(ps)["q"]
    rng = np.random.default_rng(7 * batch + n)
    a = rng.integers(0, q, (batch, n)).astype(np.uint32)
    b = rng.integers(0, q, (batch, n)).astype(np.uint32)
    da, db = _dev(ntt, a, dev), _dev(ntt, b, dev)
    c = torch.empty_like(da)
    ntt.poly_mul_nussbaumer(c, da, db, ps, "q")
    ref = oracle.poly_mul(a, b, ps).reshape(batch, n)
    assert np.array_equal(ntt.to_numpy_u32(c).reshape(batch, n), ref)
    c2 = torch.empty_like(da)
    ntt.poly_mul(c2, da, db, ps)
    assert torch.equal(c, c2)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_q_ring_edge_and_lazy_inputs(ntt, oracle, dev, ps):
    """operands at 0, q-1 and (tolerated) [q, 2q) values"""
    n, q = _n(ps), ntt.param_info(ps)["q"]
    rng = np.random.default_rng(5)
    a = np.stack([np.zeros(n), np.full(n, q - 1), rng.integers(0, q, n), np.full(n, q - 1)]).astype(np.uint32)
    b = np.stack([rng.integers(0, q, n), np.full(n, q - 1), np.full(n, q - 1), rng.integers(0, q, n)]).astype(np.uint32)
    lazy_a = a + np.uint32(q) * (rng.integers(0, 2, a.shape).astype(np.uint32))
    lazy_b = b + np.uint32(q) * (rng.integers(0, 2, b.shape).astype(np.uint32))
    c = torch.empty(a.size, dtype=torch.int32, device=dev)
    ntt.poly_mul_nussbaumer(c, _dev(ntt, lazy_a, dev), _dev(ntt, lazy_b, dev), ps, "q")
    assert np.array_equal(ntt.to_numpy_u32(c).reshape(a.shape), oracle.poly_mul(a, b, ps).reshape(a.shape))


@pytest.mark.parametrize("ring", ["q", "m32"])
def test_in_place_aliasing(ntt, oracle, dev, ring):
    ps, n = "p-III", 2048
    rng = np.random.default_rng(11)
    hi = ntt.param_info(ps)["q"] if ring == "q" else 1 << 32
    a = rng.integers(0, hi, (5, n), dtype=np.uint64).astype(np.uint32)
    b = rng.integers(0, hi, (5, n), dtype=np.uint64).astype(np.uint32)
    da, db = _dev(ntt, a, dev), _dev(ntt, b, dev)
    ntt.poly_mul_nussbaumer(da, da, db, ps, ring)       # c == a
    want = oracle.nussbaumer(a, b, n, ring if ring == "m32" else ps)
    if ring == "m32":
        want = oracle.m32_canon(want)
    assert np.array_equal(ntt.to_numpy_u32(da).reshape(5, n), want)


def test_golden_fixtures(ntt, dev):
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "vectors_nussbaumer.npz"))
    for n, ps in ((1024, "ref"), (2048, "p-III")):
        x, y, z = g[f"x{n}"], g[f"y{n}"], g[f"z{n}"]
        c = torch.empty(x.size, dtype=torch.int32, device=dev)
        ntt.poly_mul_nussbaumer(c, _dev(ntt, x, dev), _dev(ntt, y, dev), ps, "m32")
        assert np.array_equal(ntt.to_numpy_u32(c).reshape(z.shape), z)


def test_errors(ntt, dev):
    L = ntt.lib()
    t = torch.zeros(2048 * 2, dtype=torch.int32, device=dev)
    p = t.data_ptr()
    assert L.poly_mul_nussbaumer(p, p, p, 1, 2, 7, None) == ntt.NTT_ERR_PARAM
    assert L.poly_mul_nussbaumer(p + 4, p, p, 1, 2, 0, None) == ntt.NTT_ERR_ALIGN
    assert L.poly_mul_nussbaumer(p + 16, p, p, 1, 2, 0, None) == ntt.NTT_ERR_ALIAS
    assert L.poly_mul_nussbaumer(p, p, p, 0, 2, 0, None) == ntt.NTT_OK


@pytest.mark.slow
@pytest.mark.parametrize("ps,batch", [("p-III", 1 << 20), ("p-I", 1 << 16)])
def test_full_batch_q_equals_poly_mul(ntt, oracle, dev, ps, batch):
    """BASELINE config 5 size: the Nussbaumer product equals the NTT product
    on every polynomial; a sample is checked against the oracle."""
    n = _n(ps)
    a = torch.empty(batch * n, dtype=torch.int32, device=dev)
    b = torch.empty_like(a)
    ntt.fill_uniform(a, ps, 91, 0)
    ntt.fill_uniform(b, ps, 92, 0)
    c1 = torch.empty_like(a)
    c2 = torch.empty_like(a)
    ntt.poly_mul_nussbaumer(c1, a, b, ps, "q")
    ntt.poly_mul(c2, a, b, ps)
    assert torch.equal(c1, c2)
    idx = [0, batch // 3, batch - 1]
    ah = ntt.to_numpy_u32(a).reshape(batch, n)[idx]
    bh = ntt.to_numpy_u32(b).reshape(batch, n)[idx]
    assert np.array_equal(ntt.to_numpy_u32(c1).reshape(batch, n)[idx], oracle.poly_mul(ah, bh, ps).reshape(3, n))
