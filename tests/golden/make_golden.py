"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (it reads /root/reference, which does not exist
on the GPU box):  python tests/golden/make_golden.py

1. constants_h.json -- parses /root/reference/constants.h AS TEXT and records,
   per table, its length and the sha256 of its little-endian uint32 bytes
   (no table contents are copied), plus the root constants of main.cu:25-27.
   The reference could not be compiled or run here, so these
   hashes are what pins the table-construction rules.
2. vectors_<set>.npz -- seeded inputs and the oracle's FWD / INV / MUL
   outputs, each cross-checked in this script against the independent
   O(n^2) definition and the schoolbook negacyclic product before writing.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

REF = "/root/reference"
SEEDS = {"ref": 0x5EED0001, "p-I": 0x5EED0002, "p-III": 0x5EED0003}
NPOLY = 2


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, "<u4").tobytes()).hexdigest()


def parse_constants_h() -> dict:
    txt = open(os.path.join(REF, "constants.h"), "rb").read().decode().replace("\r", "")
    out = {}
    for m in re.finditer(r"(?:__constant__\s+)?uint32_t\s+(\w+)\s*\[\s*NTTSIZE\s*\]\s*=\s*\{([^}]*)\}", txt):
        name, body = m.group(1), m.group(2)
        vals = np.array([int(v) for v in body.replace("\n", " ").split(",") if v.strip()], np.uint64)
        assert vals.max() < 2**32
        out[name] = {"len": int(vals.size), "sha256": sha(vals.astype(np.uint32))}
    main = open(os.path.join(REF, "main.cu"), "rb").read().decode().replace("\r", "")
    m = re.search(r"NTTSIZE == 1024\)\s*\{\s*fg0 = (\d+); ig0 = (\d+); Ni = (\d+); nfg0 = (\d+); nig0 = (\d+);", main)
    out["_main_cu_roots"] = dict(zip(["fg0", "ig0", "Ni", "nfg0", "nig0"], map(int, m.groups())))
    mh = open(os.path.join(REF, "main.cuh"), "rb").read().decode().replace("\r", "")
    out["_main_cuh"] = {
        "P": int(re.search(r"#define P\s+(\d+)", mh).group(1)),
        "NTTSIZE": int(re.search(r"#define NTTSIZE (\d+)", mh).group(1)),
        "MIU": int(re.search(r"#define MIU\s+(\d+)", mh).group(1)),
    }
    return out


def make_vectors(ps: str) -> dict:
    p = O.params(ps)
    n, q = p["n"], p["q"]
    x = O.fill_uniform(NPOLY, ps, SEEDS[ps], 0)
    y = O.fill_uniform(NPOLY, ps, SEEDS[ps] ^ 0xFFFF, 0)
    X = O.poly_ntt(x, ps)
    Xin = O.fill_uniform(NPOLY, ps, SEEDS[ps] ^ 0xABCD, 0)   # arbitrary frequency-domain input
    xinv = O.poly_invntt(Xin, ps)
    c = O.poly_mul(x, y, ps)
    # reference fixed operand pattern init_operand (NTT.cu:10-15): x[i]=n/2-i, i<n/2
    pat = np.zeros(n, np.uint32)
    pat[: n // 2] = n // 2 - np.arange(n // 2)
    pat_X = O.poly_ntt(pat, ps)
    for r in range(NPOLY):
        assert np.array_equal(X[r], O.ntt_direct_np(x[r], ps))
        assert np.array_equal(O.poly_ntt(xinv[r], ps), Xin[r])
        assert np.array_equal(c[r], O.schoolbook_np(x[r], y[r], ps))
    assert np.array_equal(O.poly_invntt(pat_X, ps), pat)
    return dict(x=x, y=y, X=X, Xin=Xin, xinv=xinv, c=c, pattern=pat, pattern_X=pat_X,
                params=np.array([n, q, p["psi"], p["n_inv"]], np.uint64))


def make_nussbaumer() -> dict:
    """mod 2^32-1 operands over the full word range (0 and 0xFFFFFFFF included),
    nussbaumer_fft restated (NTT.cu:167-277), canonical residues; each checked
    against an exact big-integer schoolbook."""
    rng = np.random.default_rng(0x4E55)
    out = {}
    for n in (1024, 2048):
        x = rng.integers(0, 1 << 32, (2, n), dtype=np.uint64).astype(np.uint32)
        y = rng.integers(0, 1 << 32, (2, n), dtype=np.uint64).astype(np.uint32)
        x[0, :8] = O.M32
        y[1, -8:] = 0
        z = O.m32_canon(O.nussbaumer(x, y, n, "m32"))
        for r in range(2):
            assert np.array_equal(z[r], O.schoolbook_m32_np(x[r], y[r]))
        out.update({f"x{n}": x, f"y{n}": y, f"z{n}": z})
    return out


def main():
    os.makedirs(HERE, exist_ok=True)
    if os.path.isdir(REF):
        ch = parse_constants_h()
        with open(os.path.join(HERE, "constants_h.json"), "w") as f:
            json.dump(ch, f, indent=1, sort_keys=True)
        print("wrote constants_h.json:", sorted(ch))
    for ps in ("ref", "p-I", "p-III"):
        v = make_vectors(ps)
        np.savez(os.path.join(HERE, f"vectors_{ps}.npz"), **v)
        print("wrote", f"vectors_{ps}.npz")
    np.savez(os.path.join(HERE, "vectors_nussbaumer.npz"), **make_nussbaumer())
    print("wrote vectors_nussbaumer.npz")


if __name__ == "__main__":
    main()
