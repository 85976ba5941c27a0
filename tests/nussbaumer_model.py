"""Lane-level numpy model of the gfx950 Nussbaumer kernel (csrc/nussbaumer.hip).

Mirrors the kernel's data movement exactly -- registers are arrays over the
64 lanes of one wave, ds_bpermute is a gather over lanes, the LDS transpose
uses the kernel's swizzle -- so the index math (rotation amounts, block
decomposition of the inner transform, deferred 2^-L scaling, recombination)
is checked on the CPU before it runs on the GPU.  The arithmetic itself is
plain modular arithmetic (mod 2^32-1 or mod q) on Python-int-safe uint64.

Algorithm (restating NTT.cu:167-277 with m = 32, r = n/32, recursively):
  outer  : 64 sub-polynomials of length R = n/32 (R = 64: one product per
           wave; R = 32: two products per wave, one per 32-lane half);
           lane a holds coefficient a of every sub-polynomial k (register k).
  inner  : after the transpose lane k holds sub-polynomial k and multiplies
           X_k * Y_k mod (y^R + 1) by a second Nussbaumer level, m' = R/8,
           r' = 8, computed as two independent blocks of m' points each.
"""
from __future__ import annotations

import numpy as np

M32 = (1 << 32) - 1


def brv(x: int, bits: int) -> int:
    return int(format(x, f"0{bits}b")[::-1], 2) if bits else 0


class Ring:
    def __init__(self, mod: int):
        self.m = mod

    def add(self, a, b):
        return (a + b) % self.m

    def sub(self, a, b):
        return (a + self.m - b) % self.m

    def neg(self, a):
        return (self.m - a) % self.m

    def negm(self, a, mask):
        return np.where(mask, self.neg(a), a)

    def mul(self, a, b):
        a = np.asarray(a, dtype=object)
        b = np.asarray(b, dtype=object)
        return np.asarray((a * b) % self.m, dtype=np.uint64)

    def scale(self, a, L: int):
        """a * 2^-L (M32: rotate right by L)"""
        inv = pow(2, -L, self.m)
        return self.mul(a, np.full_like(a, inv))


def swz(k: int, R: int) -> int:
    return (k & 15) if R == 64 else (((k >> 1) ^ ((k & 1) << 2)) & 7)


def lds_off(h: int, k: int, a: int, R: int) -> int:
    """word offset of coefficient a of row (h, k) in the wave-private buffer"""
    return (h * 64 + k) * R + ((((a >> 2) ^ swz(k, R)) << 2) | (a & 3))


class Wave:
    def __init__(self, n: int, ring: Ring):
        self.n = n
        self.R = n // 32
        self.H = 64 // self.R
        self.SC = self.R // 32            # outer rotation scale
        self.MI = self.R // 8             # inner m'
        self.LMI = self.MI.bit_length() - 1
        self.SCI = 8 // self.MI           # inner rotation scale
        self.L = 6 + self.LMI + 1         # deferred 2^-L
        self.ring = ring
        self.lane = np.arange(64)
        self.a = self.lane & (self.R - 1)
        self.h = self.lane // self.R

    # ---- outer layout helpers: v is a [64] lane array
    def rot_fwd(self, v, sr):
        if sr == 0:
            return v
        d = self.a - sr
        src = (d & (self.R - 1)) + self.h * self.R
        return self.ring.negm(v[src], d < 0)

    def rot_inv(self, v, sr):
        if sr == 0:
            return v
        d = self.a + sr - self.R
        src = ((self.a + sr) & (self.R - 1)) + self.h * self.R
        return self.ring.negm(v[src], d >= 0)

    def outer_forward(self, X):
        rg = self.ring
        for j in range(4, -1, -1):
            for i in range(1 << (5 - j)):
                sr = self.SC * (brv(i, 5 - j) << j)
                for t in range(1 << j):
                    I = (i << (j + 1)) + t
                    L = I + (1 << j)
                    T = self.rot_fwd(X[L], sr)
                    X[L] = rg.sub(X[I], T)
                    X[I] = rg.add(X[I], T)

    def outer_inverse(self, Z):
        rg = self.ring
        for j in range(6):
            for i in range(1 << (5 - j)):
                sr = 0 if j == 5 else self.SC * (brv(i, 5 - j) << j)
                for t in range(1 << j):
                    A = (i << (j + 1)) + t
                    B = A + (1 << j)
                    T = rg.sub(Z[A], Z[B])
                    Z[A] = rg.add(Z[A], Z[B])
                    Z[B] = self.rot_inv(T, sr)

    # ---- inner: per-lane registers, U is [MI][8][64 lanes]
    def rot8(self, u, sr, inverse=False):
        """compile-time register rotation of one length-8 sub-polynomial"""
        out = [None] * 8
        for a in range(8):
            if not inverse:
                out[a] = u[a - sr] if a >= sr else self.ring.neg(u[8 + a - sr])
            else:
                out[a] = u[a + sr] if a < 8 - sr else self.ring.neg(u[a + sr - 8])
        return out

    def inner_block_forward(self, U, bl):
        rg = self.ring
        for j in range(self.LMI - 1, -1, -1):
            cnt = 1 << (self.LMI - 1 - j)
            for i in range(bl * cnt, (bl + 1) * cnt):
                sr = self.SCI * (brv(i, self.LMI - j) << j)
                for t in range(1 << j):
                    I = (i << (j + 1)) + t - bl * self.MI
                    L = I + (1 << j)
                    T = self.rot8(U[L], sr)
                    U[L] = [rg.sub(U[I][c], T[c]) for c in range(8)]
                    U[I] = [rg.add(U[I][c], T[c]) for c in range(8)]

    def inner_block_inverse(self, Z, bl):
        rg = self.ring
        for j in range(self.LMI):
            cnt = 1 << (self.LMI - 1 - j)
            for i in range(bl * cnt, (bl + 1) * cnt):
                sr = self.SCI * (brv(i, self.LMI - j) << j)
                for t in range(1 << j):
                    A = (i << (j + 1)) + t - bl * self.MI
                    B = A + (1 << j)
                    T = [rg.sub(Z[A][c], Z[B][c]) for c in range(8)]
                    Z[A] = [rg.add(Z[A][c], Z[B][c]) for c in range(8)]
                    Z[B] = self.rot8(T, sr, inverse=True)

    def mul8(self, u, v):
        rg = self.ring
        z = []
        for c in range(8):
            acc = 0
            for j in range(8):
                w = v[c - j] if j <= c else rg.neg(v[8 + c - j])
                acc = (acc + np.asarray(rg.mul(u[j], w), dtype=object)) % rg.m
            z.append(np.asarray(acc, dtype=np.uint64))
        return z

    def inner(self, xrow, yrow):
        """xrow, yrow: [R][64 lanes] -> W [R][64 lanes] = X_k * Y_k * 2^(LMI+1)"""
        rg, MI = self.ring, self.MI
        Zb = []
        for bl in range(2):
            U = [[xrow[MI * jj + ii] for jj in range(8)] for ii in range(MI)]
            V = [[yrow[MI * jj + ii] for jj in range(8)] for ii in range(MI)]
            self.inner_block_forward(U, bl)
            self.inner_block_forward(V, bl)
            Z = [self.mul8(U[i], V[i]) for i in range(MI)]
            self.inner_block_inverse(Z, bl)
            Zb.append(Z)
        Z = Zb[0] + Zb[1]
        for t in range(MI):
            T = [rg.sub(Z[t][c], Z[t + MI][c]) for c in range(8)]
            Z[t] = [rg.add(Z[t][c], Z[t + MI][c]) for c in range(8)]
            Z[t + MI] = T
        W = [None] * self.R
        for ii in range(MI):
            W[ii] = rg.sub(Z[ii][0], Z[MI + ii][7])
            for jj in range(1, 8):
                W[MI * jj + ii] = rg.add(Z[ii][jj], Z[MI + ii][jj - 1])
        return W

    # ---- whole wave: polys x, y of shape [H][n]
    def run(self, x, y):
        rg, R, H = self.ring, self.R, self.H
        X = [None] * 64
        Y = [None] * 64
        for i in range(32):   # lane (h, a) loads x[h][32a + i]
            X[i] = rg.scale(np.array([x[self.h[l]][32 * self.a[l] + i] for l in range(64)], np.uint64), self.L)
            Y[i] = np.array([y[self.h[l]][32 * self.a[l] + i] for l in range(64)], np.uint64) % rg.m
            X[i + 32] = X[i].copy()
            Y[i + 32] = Y[i].copy()
        self.outer_forward(X)
        self.outer_forward(Y)
        lds = {}
        for name, src in (("x", X), ("y", Y)):
            buf = np.zeros(H * 64 * R, np.uint64)
            for k in range(64):
                for l in range(64):
                    buf[lds_off(self.h[l], k, self.a[l], R)] = src[k][l]
            lds[name] = buf
        out = np.zeros(H * 64 * R, np.uint64)
        for h in range(H):   # inner layout: lane k = sub-polynomial k of product h
            rows = {nm: [np.array([lds[nm][lds_off(h, k, c, R)] for k in range(64)], np.uint64) for c in range(R)]
                    for nm in ("x", "y")}
            W = self.inner(rows["x"], rows["y"])
            for c in range(R):
                for k in range(64):
                    out[lds_off(h, k, c, R)] = W[c][k]
        Z = [np.array([out[lds_off(self.h[l], k, self.a[l], R)] for l in range(64)], np.uint64) for k in range(64)]
        self.outer_inverse(Z)
        z = np.zeros((H, self.n), np.uint64)
        for i in range(32):
            v = rg.add(Z[i], self.rot_fwd(Z[32 + i], 1))
            for l in range(64):
                z[self.h[l]][32 * self.a[l] + i] = v[l]
        return z
