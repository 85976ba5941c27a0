"""Pin the CPU oracle (tests-only restatement of NTT.cu) before trusting it.

The reference could not be compiled or run here, so the pins
are: constants.h table hashes (test_tables.py), the reference's round-trip
identity (NTT.cu:1557-1565) on its fixed operand pattern (NTT.cu:10-15), the
all-ones poly-mul KAT of its GPU drivers (NTT.cu:2360, 2433-2438), and
independent O(n^2) / schoolbook definitions.
"""
import os

import numpy as np
import pytest

from conftest import PARAM_SETS

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_oracle_matches_golden(oracle, ps):
    g = np.load(os.path.join(GOLD, f"vectors_{ps}.npz"))
    p = oracle.params(ps)
    assert list(g["params"]) == [p["n"], p["q"], p["psi"], p["n_inv"]]
    assert np.array_equal(oracle.fill_uniform(g["x"].shape[0], ps, {"ref": 0x5EED0001, "p-I": 0x5EED0002,
                                                                       "p-III": 0x5EED0003}[ps], 0), g["x"])
    assert np.array_equal(oracle.poly_ntt(g["x"], ps), g["X"])
    assert np.array_equal(oracle.poly_invntt(g["Xin"], ps), g["xinv"])
    assert np.array_equal(oracle.poly_mul(g["x"], g["y"], ps), g["c"])
    assert np.array_equal(oracle.poly_ntt(g["pattern"], ps), g["pattern_X"])


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_fwd_equals_direct_definition(oracle, ps):
    x = oracle.fill_uniform(2, ps, 31337, 0)
    X = oracle.poly_ntt(x, ps)
    for r in range(2):
        assert np.array_equal(X[r], oracle.ntt_direct_np(x[r], ps))
    assert np.array_equal(X[0], oracle.ntt_direct_c(x[0], ps))


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_roundtrip_reference_pattern(oracle, ps):
    n = oracle.params(ps)["n"]
    pat = np.zeros(n, np.uint32)
    pat[: n // 2] = n // 2 - np.arange(n // 2)          # init_operand, RANDOM=0
    X = oracle.poly_ntt(pat, ps)
    assert np.array_equal(oracle.poly_invntt(X, ps), pat)      # GS inverse (CT-GS driver)
    assert np.array_equal(oracle.poly_invntt_ct(X, ps), pat)   # CT inverse (CT-CT driver)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_all_ones_kat_all_pipelines(oracle, ps):
    p = oracle.params(ps)
    n, q = p["n"], p["q"]
    ones = np.ones((2, n), np.uint32)
    want = ((2 * np.arange(n) + 2 - n) % q).astype(np.uint32)
    for z in (oracle.poly_mul(ones, ones, ps), oracle.gpu_ct_gs_polymul(ones, ones, ps),
              oracle.gpu_ct_ct_polymul(ones, ones, ps)):
        assert np.array_equal(z[0], want) and np.array_equal(z[1], want)
    if ps == "ref":   # the values the reference's DEBUG dump would show
        assert (int(want[0]), int(want[1]), int(want[-1])) == (8403971, 8403973, 1024)


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_polymul_schoolbook_and_gpu_order(oracle, ps):
    a = oracle.fill_uniform(2, ps, 5, 0)
    b = oracle.fill_uniform(2, ps, 6, 0)
    c = oracle.poly_mul(a, b, ps)
    assert np.array_equal(c[1], oracle.schoolbook_np(a[1], b[1], ps))
    assert np.array_equal(oracle.gpu_ct_gs_polymul(a, b, ps), c)
    assert np.array_equal(oracle.gpu_ct_ct_polymul(a, b, ps), c)


def test_barrett_red_ref_is_exact_on_products(oracle):
    """barrett_red (NTT.cu:379-452) returns x mod P for products of canonical values."""
    P = 8404993
    rng = np.random.default_rng(0)
    L = oracle.lib()
    a = rng.integers(0, P, 20000, dtype=np.uint64)
    b = rng.integers(0, P, 20000, dtype=np.uint64)
    for x, y in zip(a, b):
        v = int(x) * int(y)
        assert L.oracle_barrett_red_ref(v) == v % P
    for v in (0, 1, P - 1, (P - 1) ** 2, P * (P - 1)):
        r = L.oracle_barrett_red_ref(v)
        assert r == v % P or (v % P == 0 and v and r == P)   # `while (res > P)` quirk (NTT.cu:446)


def test_bitrev_matches_reference_rule(oracle):
    L = oracle.lib()
    for bits in (10, 11):
        for j in (0, 1, 2, 3, 511, 512, 1023, (1 << bits) - 1):
            assert L.oracle_bitrev(j, bits) == int(format(j, f"0{bits}b")[::-1], 2)


def test_oracle_under_sanitizers(oracle, tmp_path):
    """Host-only ASan/UBSan build of the oracle self-test (sanitizers on host code)."""
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("gcc missing")
    here = os.path.dirname(oracle.__file__)
    exe = tmp_path / "oracle_asan"
    r = subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                        "-std=c11", "-D_POSIX_C_SOURCE=200809L", "-o", str(exe),
                        os.path.join(here, "oracle_selftest.c"), os.path.join(here, "ntt_oracle.c"),
                        os.path.join(here, "nussbaumer_oracle.c"), "-lpthread"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300,
                       env={**os.environ, "ASAN_OPTIONS": "detect_leaks=1", "UBSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0, r.stdout + r.stderr
    assert "oracle selftest ok" in r.stdout
