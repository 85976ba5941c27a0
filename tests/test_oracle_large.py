"""The oracle at n = 4096 / 8192 (p-III's prime; SURVEY.md 8f row 3, larger n).

No qTESLA set and no reference output exists at these sizes (the reference is
hard-wired to n = 1024), so the restated loops (NTT.cu:1201-1222, 1241-1266,
1473-1494 generalised to logn) are pinned by the O(n^2) definition after
NTT_precom (NTT.cu:560-570), the round-trip identity on the reference's
operand pattern (NTT.cu:10-15, 1557-1565) and the all-ones poly-mul KAT
(NTT.cu:2360, 2433-2438); the restated GPU kernel sequences of both drivers
must agree too.
"""
import numpy as np
import pytest

from conftest import LARGE_SETS


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_params(oracle, ps):
    p = oracle.params(ps)
    n, q, psi = p["n"], p["q"], p["psi"]
    assert q == 856145921 and n in (4096, 8192)
    assert (q - 1) % (2 * n) == 0
    assert pow(psi, n, q) == q - 1                      # order exactly 2n
    assert p["n_inv"] * n % q == 1


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_fwd_equals_direct_definition(oracle, ps):
    x = oracle.fill_uniform(1, ps, 4242, 0)
    assert np.array_equal(oracle.poly_ntt(x, ps)[0], oracle.ntt_direct_c(x[0], ps))


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_large_roundtrip_and_kat(oracle, ps):
    p = oracle.params(ps)
    n, q = p["n"], p["q"]
    pat = np.zeros(n, np.uint32)
    pat[: n // 2] = n // 2 - np.arange(n // 2)
    X = oracle.poly_ntt(pat, ps)
    assert np.array_equal(oracle.poly_invntt(X, ps), pat)
    assert np.array_equal(oracle.poly_invntt_ct(X, ps), pat)
    ones = np.ones((1, n), np.uint32)
    want = ((2 * np.arange(n) + 2 - n) % q).astype(np.uint32)
    for z in (oracle.poly_mul(ones, ones, ps), oracle.gpu_ct_gs_polymul(ones, ones, ps),
              oracle.gpu_ct_ct_polymul(ones, ones, ps)):
        assert np.array_equal(z[0], want)


def test_large_polymul_schoolbook(oracle):
    ps = "p-III-4096"
    a = oracle.fill_uniform(1, ps, 5, 0)
    b = oracle.fill_uniform(1, ps, 6, 0)
    assert np.array_equal(oracle.poly_mul(a, b, ps)[0], oracle.schoolbook_np(a[0], b[0], ps))


@pytest.mark.parametrize("n", [4096, 8192])
@pytest.mark.parametrize("direction", ["fwd", "inv"])
def test_subtree_twiddles_factor(n, direction):
    """ntt_large.hpp's shared sub-tree table: for sub-block B of the n-point
    transform and every stage b of its 2048-point sub-transform, the twiddle
    psi^(+-brv_L(2^(10-b) (G + B) + m)) equals c_{B,b} times sub-block 0's,
    with one constant per (B, b) for all m (the kernels scale by products of
    these constants instead of holding G lane tables)."""
    q = 856145921
    L = n.bit_length() - 1
    G = n // 2048
    psi = pow(3, (q - 1) // (2 * n), q)
    root = psi if direction == "fwd" else pow(psi, q - 2, q)

    def brv(k, bits):
        return int(format(k, f"0{bits}b")[::-1], 2)

    for B in range(G):
        for b in range(11):
            ratios = set()
            for m in range(0, 1 << (10 - b), max(1, (1 << (10 - b)) // 64)):
                kB = (1 << (10 - b)) * (G + B) + m
                k0 = (1 << (10 - b)) * G + m
                ratios.add(pow(root, brv(kB, L), q) * pow(pow(root, brv(k0, L), q), q - 2, q) % q)
            assert len(ratios) == 1, (B, b)
