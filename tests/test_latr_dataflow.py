"""CPU model of the radix-2^RB workgroup-per-polynomial transforms of
ntt-gpu-qtesla_amd/csrc/ntt_latr.hpp (one polynomial per workgroup of n/2^RB
threads, 2^RB coefficients per thread, RB = 3 and 4): the pass groups tile
every position exactly once, every padded LDS exchange is a bijection inside
one buffer with conflict-free reads (one 2-way exchange, see below) and at
most 2-way writes in the 32-lane bank groups of ds_read_b32 / ds_write_b32
(MI355X_MICROARCH.md §LDS), the twiddles of a stage sit at consecutive
indices, and the dataflow -- the kernel's passes, twiddle indices, exchanges
and orders run with exact arithmetic mod q -- equals the oracle's forward and
inverse (natural and bit-reversed order) for n = 1024 (ref, p-I), 2048
(p-III), 4096 and 8192."""
import numpy as np
import pytest

from test_lat_dataflow import _tables, brv


def pad_of(L, RB, inv, x):
    """latr_pad(L, RB, inv, x) of ntt_latr.hpp: (C1, C2)."""
    if RB == 3:
        np_ = (L + 2) // 3
        if x == np_ - 1:
            return (1, 1) if inv else (1, 0)
        tab = {10: ((4, 2, 1), (0, 4, 2)), 11: ((0, 4, 3), (0, 2, 2)), 12: ((0, 4, 3), (0, 2, 2)),
               13: ((0, 4, 2, 1), (0, 0, 4, 2))}
        return (tab[L][1 if inv else 0][x], 0)
    tab = {10: ((2, 1, 0), (1, 2, 1)), 11: ((2, 1, 1), (1, 2, 1)), 12: ((2, 1, 1), (0, 2, 1)),
           13: ((0, 2, 1, 1), (0, 1, 2, 1))}
    c2 = 1 if inv and ((L == 12 and x == 2) or (L == 13 and x == 3)) else 0
    return (tab[L][1 if inv else 0][x], c2)


def phys(p, pd):
    return p + pd[0] * (p >> 5) + pd[1] * (p >> 10)


class GeoR:
    """LatRGeo<L, RB> of ntt_latr.hpp."""

    def __init__(self, L, RB):
        self.L, self.RB, self.N = L, RB, 1 << L
        self.NE = 1 << RB
        self.T, self.NP = self.N // self.NE, (L + RB - 1) // RB
        self.BUF = max(phys(self.N - 1, pad_of(L, RB, inv, x)) + 1 for x in range(self.NP) for inv in (0, 1))

    def sh(self, j): return self.L - 1 - self.RB * j
    def sl(self, j): return max(self.sh(j) - (self.RB - 1), 0)
    def g0(self, j): return self.sh(j) - (self.RB - 1) if self.sh(j) >= self.RB - 1 else 0
    def has(self, j, i): return self.sl(j) <= self.g0(j) + i <= self.sh(j)

    def pos(self, j, t, e):
        g0 = self.g0(j)
        return ((t >> g0) << (g0 + self.RB)) | (e << g0) | (t & ((1 << g0) - 1))

    def exchanges(self, inv):
        """(name, pad, write map, read map) of every exchange of one direction,
        maps (t, e) -> position"""
        L, T, NP, NE, RB = self.L, self.T, self.NP, self.NE, self.RB
        out = []
        if not inv:
            for x in range(NP - 1):
                out.append((f"x{x}", pad_of(L, RB, 0, x), lambda t, e, j=x: self.pos(j, t, e),
                            lambda t, e, j=x: self.pos(j + 1, t, e)))
            out.append(("brv", pad_of(L, RB, 0, NP - 1), lambda t, e: brv(NE * t + e, L), lambda t, e: t + T * e))
        else:
            out.append(("brv", pad_of(L, RB, 1, NP - 1), lambda t, e: brv(t + T * e, L), lambda t, e: NE * t + e))
            for j in range(NP - 1, 0, -1):
                out.append((f"x{j - 1}", pad_of(L, RB, 1, j - 1), lambda t, e, j=j: self.pos(j, t, e),
                            lambda t, e, j=j: self.pos(j - 1, t, e)))
        return out


PARAMS = [("ref", 10), ("p-I", 10), ("p-III", 11), ("p-III-4096", 12), ("p-III-8192", 13)]


def conflict(addrs):
    """largest number of distinct words on one bank (word mod 32) within a
    32-lane group of a 64-lane b32 access"""
    worst = 1
    for g in (addrs[:32], addrs[32:]):
        banks = {}
        for a in g:
            banks.setdefault(a % 32, set()).add(a)
        worst = max(worst, max(len(v) for v in banks.values()))
    return worst


@pytest.mark.parametrize("RB", [3, 4])
@pytest.mark.parametrize("L", [10, 11, 12, 13])
def test_groups_tile_pads_and_banks(L, RB):
    G = GeoR(L, RB)
    NE = G.NE
    assert G.T <= 1024
    for j in range(G.NP):
        ps = [G.pos(j, t, e) for t in range(G.T) for e in range(NE)]
        assert sorted(ps) == list(range(G.N)), j
        assert any(G.has(j, i) for i in range(RB))
    assert all(G.pos(0, t, e) == t + G.T * e for t in range(G.T) for e in range(NE))
    assert all(G.pos(G.NP - 1, t, e) == NE * t + e for t in range(G.T) for e in range(NE))
    # every stage is run once, high to low within a pass
    stages = [G.g0(j) + i for j in range(G.NP) for i in range(RB - 1, -1, -1) if G.has(j, i)]
    assert stages == list(range(L - 1, -1, -1))
    # the kernel's LDS (double-buffered at RB = 3) fits next to 7 more workgroups
    assert (2 if RB == 3 else 1) * G.BUF * 4 * (8 if RB == 3 else 16) <= 160 * 1024 or L > 11
    for inv in (0, 1):
        for name, pd, wmap, rmap in G.exchanges(inv):
            wa = {phys(wmap(t, e), pd) for t in range(G.T) for e in range(NE)}
            assert len(wa) == G.N and max(wa) < G.BUF, name
            # linear split used by the kernel: phys(base | E) = phys(base) + phys(E)
            for t in range(0, G.T, max(1, G.T // 37)):
                for e in range(NE):
                    p = wmap(t, e)
                    assert phys(p, pd) == phys(wmap(t, 0), pd) + phys(p ^ wmap(t, 0), pd), (name, t, e)
            for wave in range(max(1, G.T // 64)):
                for e in range(NE):
                    lanes = range(64 * wave, min(64 * wave + 64, G.T))
                    w = [phys(wmap(t, e), pd) for t in lanes]
                    r = [phys(rmap(t, e), pd) for t in lanes]
                    # reads 1-way but for the radix-8 inverse's pass 3 -> 2
                    # exchange at L = 11 / 12 (2-way); writes at most 2-way
                    # (free for ds_write_b32)
                    two = RB == 3 and inv and L in (11, 12) and name == "x2"
                    assert conflict(r) <= (2 if two else 1), (L, RB, inv, name, "read", e)
                    assert conflict(w) <= 2, (L, RB, inv, name, "write", e)
    # a stage on group bit i: twiddle index k0 + (e >> (i+1)), consecutive
    for j in range(G.NP):
        for i in range(RB):
            if not G.has(j, i):
                continue
            b = G.g0(j) + i
            for t in range(0, G.T, max(1, G.T // 29)):
                k0 = (1 << (L - 1 - b)) + (G.pos(j, t, 0) >> (b + 1))
                for e in range(NE):
                    if not e & (1 << i):
                        assert (1 << (L - 1 - b)) + (G.pos(j, t, e) >> (b + 1)) == k0 + (e >> (i + 1))


def _xchg(G, v, pd, wmap, rmap):
    buf = {}
    for t in range(G.T):
        for e in range(G.NE):
            buf[phys(wmap(t, e), pd)] = v[t][e]
    return [[buf[phys(rmap(t, e), pd)] for e in range(G.NE)] for t in range(G.T)]


def latr_forward(x, q, L, RB, tw, br=False):
    """k_ntt_latr<PS, false, BR, RB>: returns the stored words."""
    G = GeoR(L, RB)
    NE = G.NE
    v = [[int(x[t + G.T * e]) for e in range(NE)] for t in range(G.T)]
    ex = G.exchanges(0)
    for j in range(G.NP):
        for i in range(RB - 1, -1, -1):
            if not G.has(j, i):
                continue
            b = G.g0(j) + i
            for t in range(G.T):
                V = v[t]
                k0 = (1 << (L - 1 - b)) + (G.pos(j, t, 0) >> (b + 1))
                for e in range(NE):
                    if e & (1 << i):
                        continue
                    w = tw[k0 + (e >> (i + 1))]
                    f = e | (1 << i)
                    tt = w * V[f] % q
                    V[e], V[f] = (V[e] + tt) % q, (V[e] - tt) % q
        if j + 1 < G.NP:
            _, pd, wm, rm = ex[j]
            v = _xchg(G, v, pd, wm, rm)
    out = np.zeros(G.N, np.int64)
    if br:
        for t in range(G.T):
            for e in range(NE):
                out[NE * t + e] = v[t][e]
        return out
    _, pd, wm, rm = ex[-1]
    v = _xchg(G, v, pd, wm, rm)
    for t in range(G.T):
        for e in range(NE):
            out[t + G.T * e] = v[t][e]
    return out


def latr_inverse(X, q, L, RB, itw, ninv, br=False):
    """k_ntt_latr<PS, true, BR, RB>: X natural (or bit-reversed when br)."""
    G = GeoR(L, RB)
    NE = G.NE
    ex = G.exchanges(1)
    if br:
        v = [[int(X[NE * t + e]) for e in range(NE)] for t in range(G.T)]
    else:
        v = [[int(X[t + G.T * e]) for e in range(NE)] for t in range(G.T)]
        _, pd, wm, rm = ex[0]
        v = _xchg(G, v, pd, wm, rm)
    k = 1
    for j in range(G.NP - 1, -1, -1):
        for i in range(RB):
            if not G.has(j, i) or (j == 0 and i == RB - 1):
                continue
            b = G.g0(j) + i
            for t in range(G.T):
                V = v[t]
                k0 = (1 << (L - 1 - b)) + (G.pos(j, t, 0) >> (b + 1))
                for e in range(NE):
                    if e & (1 << i):
                        continue
                    w = itw[k0 + (e >> (i + 1))]
                    f = e | (1 << i)
                    V[e], V[f] = (V[e] + V[f]) % q, (V[e] - V[f]) * w % q
        if j > 0:
            _, pd, wm, rm = ex[k]
            k += 1
            v = _xchg(G, v, pd, wm, rm)
    out = np.zeros(G.N, np.int64)
    c1 = ninv * itw[1] % q
    h = NE // 2
    for t in range(G.T):
        V = v[t]
        for e in range(h):
            out[t + G.T * e] = (V[e] + V[e + h]) * ninv % q
            out[t + G.T * (e + h)] = (V[e] - V[e + h]) * c1 % q
    return out


@pytest.mark.parametrize("RB", [3, 4])
@pytest.mark.parametrize("param,L", PARAMS)
def test_latr_dataflow_matches_oracle(oracle, param, L, RB):
    q, n, Lq, tw, itw = _tables(oracle, param)
    assert Lq == L
    x = oracle.fill_uniform(1, param, 13, 0)[0]
    want = oracle.poly_ntt(x[None, :], param)[0].astype(np.int64)
    X = latr_forward(x, q, L, RB, tw)
    assert np.array_equal(X, want)
    Xb = latr_forward(x, q, L, RB, tw, br=True)
    assert np.array_equal(Xb, want[[brv(t, L) for t in range(n)]])
    ninv = pow(n, q - 2, q)
    assert np.array_equal(latr_inverse(X, q, L, RB, itw, ninv), x.astype(np.int64))
    assert np.array_equal(latr_inverse(Xb, q, L, RB, itw, ninv, br=True), x.astype(np.int64))
    y = oracle.fill_uniform(1, param, 14, 0)[0]
    assert np.array_equal(latr_inverse(y, q, L, RB, itw, ninv),
                          oracle.poly_invntt(y[None, :], param)[0].astype(np.int64))
