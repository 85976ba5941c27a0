"""CPU: the Nussbaumer oracle and the lane-level model of the GPU kernel.

1. oracle/nussbaumer_oracle.c (nussbaumer_fft, NTT.cu:167-277, generalised to
   n = 2048) is pinned by the reference's own test input (test_nussbaumer,
   NTT.cu:1987-2005: all-ones -> z[k] = 2k+2-n), by its full-length `naive`
   (NTT.cu:147-165), by an exact big-integer schoolbook and, mod q, by the
   NTT poly-mul oracle.
2. tests/nussbaumer_model.py replays the kernel's data movement (lane
   rotations, swizzled LDS transpose, blocked inner level, deferred 2^-L)
   and must reproduce the oracle.
3. The kernel's LDS swizzle is a bijection and bank-conflict free under the
   gfx950 lane-group model used in tests/test_lds_layout.py.
"""
import os

import numpy as np
import pytest

from nussbaumer_model import M32, Ring, Wave, lds_off

G_B128_READ = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
               [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
G_B128_READ += [[l + 32 for l in g] for g in G_B128_READ]


@pytest.mark.parametrize("n", [1024, 2048])
def test_reference_kat(oracle, n):
    ones = np.ones((1, n), np.uint32)
    z = oracle.m32_canon(oracle.nussbaumer(ones, ones, n, "m32"))[0]
    assert np.array_equal(z, np.array([(2 * k + 2 - n) % M32 for k in range(n)], np.uint32))


@pytest.mark.parametrize("n", [1024, 2048])
def test_matches_naive_and_bigint_schoolbook(oracle, n):
    rng = np.random.default_rng(n)
    x = rng.integers(0, 1 << 32, (2, n), dtype=np.uint64).astype(np.uint32)
    y = rng.integers(0, 1 << 32, (2, n), dtype=np.uint64).astype(np.uint32)
    x[0, :5] = M32
    z = oracle.m32_canon(oracle.nussbaumer(x, y, n, "m32"))
    assert np.array_equal(z, oracle.m32_canon(oracle.naive_negacyclic(x, y, n, "m32")))
    assert np.array_equal(z[0], oracle.schoolbook_m32_np(x[0], y[0]))


@pytest.mark.parametrize("ps", ["ref", "p-I", "p-III"])
def test_mod_q_matches_ntt_poly_mul(oracle, ps):
    n, q = oracle.params(ps)["n"], oracle.params(ps)["q"]
    rng = np.random.default_rng(3)
    a = rng.integers(0, q, (3, n)).astype(np.uint32)
    b = rng.integers(0, q, (3, n)).astype(np.uint32)
    assert np.array_equal(oracle.nussbaumer(a, b, n, ps), oracle.poly_mul(a, b, ps).reshape(3, n))
    assert np.array_equal(oracle.naive_negacyclic(a, b, n, ps)[0], oracle.schoolbook_np(a[0], b[0], ps))


def test_golden_fixture_reproduced(oracle):
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "vectors_nussbaumer.npz"))
    for n in (1024, 2048):
        z = oracle.m32_canon(oracle.nussbaumer(g[f"x{n}"], g[f"y{n}"], n, "m32"))
        assert np.array_equal(z, g[f"z{n}"])


@pytest.mark.parametrize("n", [1024, 2048])
@pytest.mark.parametrize("ring", ["m32", "q"])
def test_kernel_model_matches_oracle(oracle, n, ring):
    ps = "p-III" if n == 2048 else "p-I"
    mod = M32 if ring == "m32" else oracle.params(ps)["q"]
    H = 64 // (n // 32)
    rng = np.random.default_rng(17)
    x = rng.integers(0, mod, (H, n), dtype=np.uint64)
    y = rng.integers(0, mod, (H, n), dtype=np.uint64)
    z = Wave(n, Ring(mod)).run(x, y).astype(np.uint32)
    want = oracle.nussbaumer(x.astype(np.uint32), y.astype(np.uint32), n, "m32" if ring == "m32" else ps)
    if ring == "m32":
        want = oracle.m32_canon(want)
    assert np.array_equal(z, want)


@pytest.mark.parametrize("R", [32, 64])
def test_lds_swizzle_bijective_and_conflict_free(R):
    H = 64 // R
    offs = {lds_off(h, k, a, R) for h in range(H) for k in range(64) for a in range(R)}
    assert offs == set(range(H * 64 * R))
    for h in range(H):
        # outer side: ds_write/read_b32, two 32-lane groups, bank = dword % 32
        for k in range(64):
            for g in (range(32), range(32, 64)):
                lanes = [l for l in g if l // R == h]
                if lanes:
                    banks = [lds_off(h, k, l % R, R) % 32 for l in lanes]
                    assert len(set(banks)) == len(banks)
        # inner side: lane k reads / writes 16-B chunk c of row (h, k)
        for c in range(R // 4):
            addr = [lds_off(h, k, 4 * c, R) for k in range(64)]
            assert all(a % 4 == 0 for a in addr)
            for g in G_B128_READ:   # ds_read_b128: 16-lane groups, slot = (dword/4) % 16
                assert len({(addr[l] // 4) % 16 for l in g}) == 16
            for g0 in range(0, 64, 8):   # ds_write_b128: 8-lane groups, slot = (dword/4) % 8
                assert len({(addr[l] // 4) % 8 for l in range(g0, g0 + 8)}) == 8
