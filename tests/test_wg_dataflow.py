"""CPU model of the workgroup-per-polynomial n = 2048 transforms
(ntt-gpu-qtesla_amd/tools/ntt_wg.hpp, tools-only diag library -- DESIGN.md §7a): the
six pass layouts and five LDS exchange maps are bijective, every register's
address is a fixed offset from one per-thread base (the offsets the kernel
hard-codes), every access is bank-conflict-free per half-wave, and the
dataflow run exactly (mod q) equals the oracle's forward and inverse."""
import numpy as np


def b(p, i):
    return (p >> i) & 1


def posA(w, l, e): return (e << 9) | (w << 6) | l
def posB(w, l, e): return ((w >> 2) << 10) | (((w >> 1) & 1) << 9) | ((e >> 1) << 8) | ((e & 1) << 7) | ((w & 1) << 6) | l
def posC(w, l, e): return (w << 8) | ((l >> 5) << 7) | ((e >> 1) << 6) | ((e & 1) << 5) | (l & 31)
def posD(w, l, e): return (w << 8) | ((l >> 3) << 5) | ((e >> 1) << 4) | ((e & 1) << 3) | (l & 7)
def posE(w, l, e): return (w << 8) | ((l >> 1) << 3) | ((e >> 1) << 2) | ((e & 1) << 1) | (l & 1)


def posF(w, l, e):
    p = e | (b(w, 2) << 2) | (b(w, 1) << 3) | (b(w, 0) << 4)
    for i in range(6):
        p |= b(l, 5 - i) << (5 + i)
    return p


def x12(p): return p
def x3(p): return (p >> 5) * 40 + (p & 31)
def x4(p): return ((((p >> 7) << 2) | ((p >> 3) & 3)) * 34) + ((((p >> 5) & 3) << 3) | (p & 7))


def x5(p):
    return (b(p, 7) | b(p, 8) << 1 | b(p, 9) << 2 | b(p, 10) << 3 | b(p, 1) << 4 | b(p, 2) << 5) * 34 + \
           (b(p, 6) | b(p, 0) << 1 | b(p, 3) << 2 | b(p, 4) << 3 | b(p, 5) << 4)


LAY = [None, posA, posB, posC, posD, posE, posF]
XM = {1: x12, 2: x12, 3: x3, 4: x4, 5: x5}
# WgOff<X>::W / ::R of ntt_wg.hpp
OFF = {1: ([0, 512, 1024, 1536], [0, 128, 256, 384]), 2: ([0, 128, 256, 384], [0, 32, 64, 96]),
       3: ([0, 40, 80, 120], [0, 8, 16, 24]), 4: ([0, 34, 68, 102], [0, 2, 4, 6]),
       5: ([0, 544, 1088, 1632], [0, 2, 544, 546])}
PASSBITS = {1: (10, 9), 2: (8, 7), 3: (6, 5), 4: (4, 3), 5: (2, 1), 6: (1, 0)}


def brv(k, n=11):
    return int(format(k, f"0{n}b")[::-1], 2)


def test_layouts_and_exchanges():
    for f in LAY[1:]:
        assert len({f(w, l, e) for w in range(8) for l in range(64) for e in range(4)}) == 2048
    for X in range(1, 6):
        a = XM[X]
        addrs = {a(p) for p in range(2048)}
        assert len(addrs) == 2048 and max(addrs) < 2560          # WGP_BUF
        for side, lay in ((0, LAY[X]), (1, LAY[X + 1])):
            for w in range(8):
                for l in range(64):
                    base = a(lay(w, l, 0))
                    assert [a(lay(w, l, e)) - base for e in range(4)] == OFF[X][side]
            for w in range(8):
                for h in range(2):
                    for e in range(4):
                        banks = {a(lay(w, 32 * h + i, e)) % 32 for i in range(32)}
                        assert len(banks) == 32, (X, side, w, h, e)
    # bit-reversed side of pass F: X[1024 e0 + 512 e1 + 64 w + l]
    assert all(brv(posF(w, l, e)) == 1024 * (e & 1) + 512 * (e >> 1) + 64 * w + l
               for w in range(8) for l in range(64) for e in range(4))


def test_dataflow_matches_oracle(oracle):
    q = 856145921
    psi = pow(3, (q - 1) // 4096, q)
    ipsi = pow(psi, q - 2, q)
    tw = [pow(psi, brv(k), q) for k in range(2048)]
    itw = [pow(ipsi, brv(k), q) for k in range(2048)]

    def kidx(pos0, bit):
        return (1 << (10 - bit)) + (pos0 >> (bit + 1))

    def xchg(v, X, src, dst):
        a, buf = XM[X], {}
        for t in range(512):
            for e in range(4):
                buf[a(src(t >> 6, t & 63, e))] = v[t][e]
        return [[buf[a(dst(t >> 6, t & 63, e))] for e in range(4)] for t in range(512)]

    x = oracle.fill_uniform(1, "p-III", 5, 0)[0].astype(np.int64)
    v = [[int(x[t + 512 * e]) for e in range(4)] for t in range(512)]
    for P in range(1, 7):   # forward: CT, high stage first
        pa, pb = PASSBITS[P]
        for t in range(512):
            pos0, V = LAY[P](t >> 6, t & 63, 0), v[t]
            if P < 6:
                w = tw[kidx(pos0, pa)]
                for i, j in ((0, 2), (1, 3)):
                    tt = w * V[j] % q
                    V[i], V[j] = (V[i] + tt) % q, (V[i] - tt) % q
            for e1, (i, j) in enumerate(((0, 1), (2, 3))):
                tt = tw[kidx(pos0 | (e1 << pa), pb)] * V[j] % q
                V[i], V[j] = (V[i] + tt) % q, (V[i] - tt) % q
        if P < 6:
            v = xchg(v, P, LAY[P], LAY[P + 1])
    X = np.zeros(2048, np.int64)
    for t in range(512):
        for e in range(4):
            X[1024 * (e & 1) + 512 * (e >> 1) + t] = v[t][e]
    want = oracle.poly_ntt(x.astype(np.uint32)[None, :], "p-III")[0].astype(np.int64)
    assert np.array_equal(X, want)

    v = [[int(X[1024 * (e & 1) + 512 * (e >> 1) + t]) for e in range(4)] for t in range(512)]
    for P in range(6, 0, -1):   # inverse: GS, low stage first
        pa, pb = PASSBITS[P]
        for t in range(512):
            pos0, V = LAY[P](t >> 6, t & 63, 0), v[t]
            for e1, (i, j) in enumerate(((0, 1), (2, 3))):
                s, d = (V[i] + V[j]) % q, (V[i] - V[j]) * itw[kidx(pos0 | (e1 << pa), pb)] % q
                V[i], V[j] = s, d
            if P < 6:
                w = itw[kidx(pos0, pa)]
                for i, j in ((0, 2), (1, 3)):
                    s, d = (V[i] + V[j]) % q, (V[i] - V[j]) * w % q
                    V[i], V[j] = s, d
        if P > 1:
            v = xchg(v, P - 1, LAY[P], LAY[P - 1])
    ninv = pow(2048, q - 2, q)
    back = np.array([v[t][e] * ninv % q for e in range(4) for t in range(512)], np.int64)
    assert np.array_equal(back, x)
