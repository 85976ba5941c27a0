"""CPU model of the small-batch (latency) transforms of
ntt-gpu-qtesla_amd/csrc/ntt_lat.hpp (one polynomial per workgroup of n/4
threads, 4 coefficients per thread): the pass groups tile every position
exactly once, the padded LDS exchange addresses stay inside one buffer, and
the dataflow -- the kernel's passes, twiddle indices and exchanges run with
exact arithmetic mod q -- equals the oracle's forward and inverse for n = 1024
(ref, p-I), 2048 (p-III) and 4096 / 8192, in natural and bit-reversed order."""
import numpy as np
import pytest


def brv(x, bits):
    return int(format(x, f"0{bits}b")[::-1], 2)


class Geo:
    """LatGeo<L> of ntt_lat.hpp."""

    def __init__(self, L):
        # T here counts groups (GN of the kernel); the kernel's threads take
        # R = GN / 1024 groups each at n = 8192, which changes no position
        self.L, self.N, self.T, self.NP = L, 1 << L, 1 << (L - 2), (L + 1) // 2
        self.BUF = self.pad(self.N - 1) + 1
        self.R = max(1, self.T // 1024)

    @staticmethod
    def pad(x):
        return x + (x >> 5)

    def hb(self, j): return self.L - 1 - 2 * j
    def lb(self, j): return self.L - 2 - 2 * j
    def gh(self, j): return 1 if self.lb(j) < 0 else self.hb(j)
    def gl(self, j): return 0 if self.lb(j) < 0 else self.lb(j)

    def base(self, j, t):
        gl, gh = self.gl(j), self.gh(j)
        return ((t >> gl) << (gh + 1)) | (t & ((1 << gl) - 1))

    def pos(self, j, t, e):
        return self.base(j, t) + ((e >> 1) << self.gh(j)) + ((e & 1) << self.gl(j))


PARAMS = [("ref", 10), ("p-I", 10), ("p-III", 11), ("p-III-4096", 12), ("p-III-8192", 13)]


@pytest.mark.parametrize("L", [10, 11, 12, 13])
def test_groups_tile_and_pad(L):
    G = Geo(L)
    for j in range(G.NP):
        ps = [G.pos(j, t, e) for t in range(G.T) for e in range(4)]
        assert sorted(ps) == list(range(G.N)), j
        if j == 0:   # the coalesced natural-order groups t + T e
            assert all(G.pos(0, t, e) == t + G.T * e for t in range(G.T) for e in range(4))
    pads = {G.pad(p) for p in range(G.N)}
    assert len(pads) == G.N and max(pads) < G.BUF
    assert G.T // G.R <= 1024                  # threads per workgroup
    # stage-lb twiddle pairs: the second pair's index is the first's + 1
    for j in range(G.NP):
        for t in range(G.T):
            b0 = G.base(j, t)
            k0 = (1 << (L - 1 - G.gl(j))) + (b0 >> (G.gl(j) + 1))
            k1 = (1 << (L - 1 - G.gl(j))) + ((b0 + (1 << G.gh(j))) >> (G.gl(j) + 1))
            assert k1 == k0 + 1


def _tables(oracle, param):
    p = oracle.params(param)
    q, n, L = p["q"], p["n"], p["n"].bit_length() - 1
    psi = p["psi"]
    ipsi = pow(psi, q - 2, q)
    tw = [pow(psi, brv(k, L), q) for k in range(n)]
    itw = [pow(ipsi, brv(k, L), q) for k in range(n)]
    return q, n, L, tw, itw


def lat_forward(x, q, L, tw, br=False):
    """k_ntt_lat<PS, false, BR>: returns the stored words."""
    G = Geo(L)
    v = [[int(x[t + G.T * e]) for e in range(4)] for t in range(G.T)]

    def bf(V, i, j, w):
        tt = w * V[j] % q
        V[i], V[j] = (V[i] + tt) % q, (V[i] - tt) % q

    for j in range(G.NP):
        for t in range(G.T):
            V, b0 = v[t], G.base(j, t)
            if G.lb(j) >= 0:
                w = tw[(1 << (L - 1 - G.hb(j))) + (b0 >> (G.hb(j) + 1))]
                bf(V, 0, 2, w)
                bf(V, 1, 3, w)
            kb = (1 << (L - 1 - G.gl(j))) + (b0 >> (G.gl(j) + 1))
            bf(V, 0, 1, tw[kb])
            bf(V, 2, 3, tw[kb + 1])
        if j + 1 < G.NP:   # exchange through one padded buffer
            buf = {}
            for t in range(G.T):
                for e in range(4):
                    buf[G.pad(G.pos(j, t, e))] = v[t][e]
            v = [[buf[G.pad(G.pos(j + 1, t, e))] for e in range(4)] for t in range(G.T)]
    out = np.zeros(G.N, np.int64)
    for t in range(G.T):
        for e in range(4):
            p = G.pos(G.NP - 1, t, e)
            out[p if br else brv(p, L)] = v[t][e]
    return out


def lat_inverse(X, q, L, itw, ninv, br=False):
    """k_ntt_lat<PS, true, BR>: X natural (or bit-reversed when br)."""
    G = Geo(L)
    A = [int(X[p]) if br else int(X[brv(p, L)]) for p in range(G.N)]   # A[pos] = X[brv(pos)]
    v = [[A[G.pos(G.NP - 1, t, e)] for e in range(4)] for t in range(G.T)]

    def gs(V, i, j, w):
        V[i], V[j] = (V[i] + V[j]) % q, (V[i] - V[j]) * w % q

    for j in range(G.NP - 1, -1, -1):
        for t in range(G.T):
            V, b0 = v[t], G.base(j, t)
            kb = (1 << (L - 1 - G.gl(j))) + (b0 >> (G.gl(j) + 1))
            gs(V, 0, 1, itw[kb])
            gs(V, 2, 3, itw[kb + 1])
            if j > 0 and G.lb(j) >= 0:
                w = itw[(1 << (L - 1 - G.hb(j))) + (b0 >> (G.hb(j) + 1))]
                gs(V, 0, 2, w)
                gs(V, 1, 3, w)
        if j > 0:
            buf = {}
            for t in range(G.T):
                for e in range(4):
                    buf[G.pad(G.pos(j, t, e))] = v[t][e]
            v = [[buf[G.pad(G.pos(j - 1, t, e))] for e in range(4)] for t in range(G.T)]
    # stage L-1 (k = 1) with n^-1: (x + y) n^-1, (x - y) n^-1 psi^-brv(1)
    out = np.zeros(G.N, np.int64)
    c1 = ninv * itw[1] % q
    for t in range(G.T):
        x0, x1, y0, y1 = v[t]
        out[t] = (x0 + y0) * ninv % q
        out[t + G.T] = (x1 + y1) * ninv % q
        out[t + 2 * G.T] = (x0 - y0) * c1 % q
        out[t + 3 * G.T] = (x1 - y1) * c1 % q
    return out


@pytest.mark.parametrize("param,L", PARAMS)
def test_lat_dataflow_matches_oracle(oracle, param, L):
    q, n, Lq, tw, itw = _tables(oracle, param)
    assert Lq == L
    x = oracle.fill_uniform(1, param, 11, 0)[0]
    want = oracle.poly_ntt(x[None, :], param)[0].astype(np.int64)
    X = lat_forward(x, q, L, tw)
    assert np.array_equal(X, want)
    Xb = lat_forward(x, q, L, tw, br=True)
    assert np.array_equal(Xb, want[[brv(t, L) for t in range(n)]])
    ninv = pow(n, q - 2, q)
    assert np.array_equal(lat_inverse(X, q, L, itw, ninv), x.astype(np.int64))
    assert np.array_equal(lat_inverse(Xb, q, L, itw, ninv, br=True), x.astype(np.int64))


@pytest.mark.parametrize("param,L", PARAMS[:4])   # the product kernels stop at n = 4096
def test_lat_product_dataflow(oracle, param, L):
    """k_poly_mul_lat: both forwards left in the CT's bit-reversed group
    order, the pointwise product there (the kernel's Montgomery 2^-32 is undone
    by the inverse's n^-1 2^32), the inverse from that order; BHAT reads the
    natural-order b-hat at the bit-reversed positions."""
    q, n, _, tw, itw = _tables(oracle, param)
    a = oracle.fill_uniform(1, param, 21, 0)[0]
    b = oracle.fill_uniform(1, param, 22, 0)[0]
    ninv = pow(n, q - 2, q)
    A = lat_forward(a, q, L, tw, br=True)
    B = lat_forward(b, q, L, tw, br=True)
    c = lat_inverse(A * B % q, q, L, itw, ninv, br=True)
    want = oracle.poly_mul(a[None, :], b[None, :], param)[0].astype(np.int64)
    assert np.array_equal(c, want)
    bhat = oracle.poly_ntt(b[None, :], param)[0].astype(np.int64)   # natural order
    Bh = bhat[[brv(p, L) for p in range(n)]]
    assert np.array_equal(lat_inverse(A * Bh % q, q, L, itw, ninv, br=True), want)
