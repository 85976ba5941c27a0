"""Product tables (ntt_get_tables, host-side) vs the reference's constants.h.

tests/golden/constants_h.json holds sha256 digests of the constants.h tables
(parsed as text by tests/golden/make_golden.py); no table contents are copied.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import PARAM_SETS

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, "<u4").tobytes()).hexdigest()


@pytest.fixture(scope="module")
def consts():
    with open(os.path.join(GOLD, "constants_h.json")) as f:
        return json.load(f)


def test_ref_tables_bit_identical_to_constants_h(ntt, consts):
    t = ntt.tables("ref")
    assert sha(t["bitrev_tbl"]) == consts["bitrev_tbl"]["sha256"] == consts["bitrev_tbl_gpu"]["sha256"]
    assert sha(t["Phi"]) == consts["Phi"]["sha256"] == consts["Phi_gpu"]["sha256"]
    assert sha(t["invPhi"]) == consts["invPhi"]["sha256"] == consts["invPhi_gpu"]["sha256"]
    assert sha(t["tf0"]) == consts["tf0_gpu"]["sha256"]
    assert sha(t["ti0"]) == consts["ti0_gpu"]["sha256"]
    assert all(consts[k]["len"] == 1024 for k in consts if not k.startswith("_"))


def test_ref_params_match_main_cu(ntt, consts):
    p = ntt.param_info("ref")
    r, h = consts["_main_cu_roots"], consts["_main_cuh"]
    assert (p["n"], p["q"]) == (h["NTTSIZE"], h["P"])
    assert (p["omega"], p["omega_inv"], p["n_inv"]) == (r["fg0"], r["ig0"], r["Ni"])
    assert h["MIU"] == (1 << 48) // h["P"]          # Barrett constant of main.cuh:20


@pytest.mark.parametrize("ps", PARAM_SETS)
def test_tables_match_oracle_and_rules(ntt, oracle, ps):
    t, o = ntt.tables(ps), oracle.tables(ps)
    for k in t:
        assert np.array_equal(t[k], o[k]), k
    p = ntt.param_info(ps)
    n, q, psi = p["n"], p["q"], p["psi"]
    assert pow(psi, n, q) == q - 1                  # primitive 2n-th root
    assert int(t["Phi"][1]) == psi and int(t["tf0"][1]) == psi * psi % q
    assert int(t["invPhi"][0]) == pow(n, q - 2, q)
    i = 777 % n
    assert int(t["tf0"][i]) * int(t["ti0"][i]) % q == 1
    assert int(t["Phi"][i]) * int(t["invPhi"][i]) % q == p["n_inv"]


def test_psi_choice_documented(ntt):
    # p-I / p-III use psi = 3^((q-1)/2n), 3 the smallest primitive root
    for ps in ("p-I", "p-III"):
        p = ntt.param_info(ps)
        assert p["psi"] == pow(3, (p["q"] - 1) // (2 * p["n"]), p["q"])
    assert ntt.param_info("ref")["psi"] == 2083362
