"""CPU model of the wave-per-polynomial n = 4096 / 8192 transforms
(ntt-gpu-qtesla_amd/csrc/ntt_big.hpp): one wave owns a whole
polynomial, R = n/64 registers per lane.  The model follows the kernel's
register layouts, permlane32 swap, chunked LDS transposes (addresses, b32 /
b128 bank groups), twiddle indexing of the uniform, bit-5 and lane tables,
and the store / load address maps, with exact arithmetic mod q, and must equal
the oracle's transforms (oracle/, the restatement of NTT.cu's serial loops).

Layouts (L = log2 n, M = L - 6 register bits, H = R/2, NC = L - 11 chunk bits):
  A   (load / pass 1)  lane = pos 0..5, register j = pos 6..L-1
  A'' (after the bit-5 stage, swap of lane bit 5 with register bit M-1)
      lane = pos 0..4 + pos L-1 (bit 5), register j: bits 0..M-2 = pos 6..L-2,
      bit M-1 = pos 5
  chunk c = (pos 5, .., pos 5+NC-1): registers j(c, t) = (c >> 1) + 2^(NC-1) t + H (c & 1)
  B   (pass 2 / store) per chunk: lane l' with l' bit i = pos L-1-i, register j' = pos 0..4
"""
import numpy as np
import pytest

from conftest import LARGE_SETS
from test_lds_layout import G_B128_READ, G_B128_WRITE, G_B32, Lane, brv, worst_conflict, xm_of


def geometry(n):
    L = n.bit_length() - 1
    M = L - 6
    return L, M, 1 << M, 1 << (M - 1), L - 11


def chunk_reg(c, t, H, NC):
    return (c >> 1) + (1 << (NC - 1)) * t + H * (c & 1)


def a2_pos(lane, j, L, M):
    """position held by register j of `lane` in layout A''"""
    return (lane & 31) + 32 * (j >> (M - 1)) + 64 * (j & ((1 << (M - 1)) - 1)) + (lane >> 5) * (1 << (L - 1))


def w_addr(lane, t):
    """chunk transpose, A'' side (b32): P = (l & 31) + 32 t + 1024 (l >> 5), swizzled"""
    h = lane >> 5
    return ((lane & 31) ^ (h << 4) ^ xm_of(t)) + 32 * (t ^ ((t >> 2) & 1)) + 1024 * h


def chunk_P(lane, t):
    return (lane & 31) + 32 * t + 1024 * (lane >> 5)


def b_pos(lane, jp, c, L, NC):
    """position held by register j' of `lane` in chunk c's layout B"""
    u = brv(lane, 6)      # pos 5+NC .. L-1
    return jp + 32 * c + (u << (5 + NC))


def store_addr(lane, jp, c, L, NC):
    return (brv(jp, 5) << (L - 5)) + (brv(c, NC) << 6) + lane


def tables(oracle, ps):
    p = oracle.params(ps)
    n, q, psi = p["n"], p["q"], p["psi"]
    L = n.bit_length() - 1
    pw = [1] * (2 * n)
    for i in range(1, 2 * n):
        pw[i] = pw[i - 1] * psi % q
    fwd = [pw[brv(k, L)] for k in range(n)]
    inv = [pow(pw[brv(k, L)], q - 2, q) for k in range(n)]
    return p, fwd, inv


def lane_k(b, c, lane, m, L, NC):
    """twiddle index of the pass-2 lane table (stage on pos bit b, chunk c)"""
    return (1 << (L - 1 - b)) + ((c + (brv(lane, 6) << NC)) << (4 - b)) + m


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_layout_maps(oracle, ps):
    n = oracle.params(ps)["n"]
    L, M, R, H, NC = geometry(n)
    # A'' covers every position once; chunk registers are disjoint
    assert sorted(a2_pos(l, j, L, M) for l in range(64) for j in range(R)) == list(range(n))
    regs = sorted(chunk_reg(c, t, H, NC) for c in range(1 << NC) for t in range(32))
    assert regs == list(range(R))
    for c in range(1 << NC):
        # the transposition moves exactly chunk c's positions
        src = {a2_pos(l, chunk_reg(c, t, H, NC), L, M) for l in range(64) for t in range(32)}
        dst = {b_pos(l, jp, c, L, NC) for l in range(64) for jp in range(32)}
        assert src == dst
        mem = {}
        for l in range(64):
            for t in range(32):
                P = chunk_P(l, t)
                pos = a2_pos(l, chunk_reg(c, t, H, NC), L, M)
                # chunk-local P = (pos 0..4) + 32 (pos 5+NC .. L-1)
                assert P == (pos & 31) + 32 * (pos >> (5 + NC))
                mem[w_addr(l, t)] = pos
        assert len(mem) == 2048
        for l in range(64):
            Lb = Lane(l, 11)     # the n = 2048 read side: rbase / rxm of Lp = brv6(lane)
            for cc in range(8):
                a = Lb.rbase + ((4 * cc) ^ Lb.rxm)
                for i in range(4):
                    assert mem[a + i] == b_pos(l, 4 * cc + i, c, L, NC)
        # the natural index of every B position is its store address
        for l in range(64):
            for jp in range(32):
                assert brv(b_pos(l, jp, c, L, NC), L) == store_addr(l, jp, c, L, NC)


def test_chunk_transpose_banks():
    for t in range(32):
        a = [w_addr(l, t) for l in range(64)]
        assert worst_conflict(a, G_B32, lambda d: d % 32, 1) == 1
    lanes = [Lane(l, 11) for l in range(64)]
    for cc in range(8):
        a = [lanes[l].rbase + ((4 * cc) ^ lanes[l].rxm) for l in range(64)]
        assert worst_conflict(a, G_B128_READ, lambda d: (d // 4) % 16, 1) == 1
        assert worst_conflict(a, G_B128_WRITE, lambda d: (d // 4) % 8, 1) == 1


def swap32(dst, src):
    """v_permlane32_swap: upper 32 lanes of dst <-> lower 32 lanes of src"""
    nd = np.concatenate([dst[:32], src[:32]])
    ns = np.concatenate([dst[32:], src[32:]])
    return nd, ns


def model_fwd(x, oracle, ps):
    p, fwd, _ = tables(oracle, ps)
    n, q = p["n"], p["q"]
    L, M, R, H, NC = geometry(n)
    lanes = np.arange(64)
    r = [np.array([int(x[l + 64 * j]) for l in range(64)], dtype=object) for j in range(R)]
    for s in range(M):                       # pass 1: uniform twiddles
        hh = 1 << (M - 1 - s)
        for j in range(R):
            if j & hh == 0:
                w = fwd[(1 << s) + (j >> (M - s))]
                t = r[j + hh] * w % q
                r[j], r[j + hh] = (r[j] + t) % q, (r[j] - t) % q
    for m in range(H):                       # bit-5 stage: swap, then lane-half twiddles
        r[m], r[m + H] = swap32(r[m], r[m + H])
        w = np.array([fwd[(1 << M) + m + H * (l >> 5)] for l in lanes], dtype=object)
        t = r[m + H] * w % q
        r[m], r[m + H] = (r[m] + t) % q, (r[m] - t) % q
    for l in range(64):
        for j in range(R):
            pass
    out = np.zeros(n, np.uint64)
    for c in range(1 << NC):
        # chunk transpose through the swizzled buffer
        buf = {}
        for t in range(32):
            j = chunk_reg(c, t, H, NC)
            for l in range(64):
                buf[w_addr(l, t)] = r[j][l]
        rb = []
        for jp in range(32):
            v = []
            for l in range(64):
                Lb = Lane(l, 11)
                v.append(buf[Lb.rbase + ((4 * (jp >> 2)) ^ Lb.rxm) + (jp & 3)])
            rb.append(np.array(v, dtype=object))
        for b in range(4, -1, -1):          # pass 2: lane table of chunk c
            hh = 1 << b
            for jp in range(32):
                if jp & hh == 0:
                    m = jp >> (b + 1)
                    w = np.array([fwd[lane_k(b, c, l, m, L, NC)] for l in lanes], dtype=object)
                    t = rb[jp + hh] * w % q
                    rb[jp], rb[jp + hh] = (rb[jp] + t) % q, (rb[jp] - t) % q
        for jp in range(32):
            for l in range(64):
                out[store_addr(l, jp, c, L, NC)] = rb[jp][l]
    return out.astype(np.uint32)


def model_inv(X, oracle, ps):
    p, _, inv = tables(oracle, ps)
    n, q = p["n"], p["q"]
    L, M, R, H, NC = geometry(n)
    lanes = np.arange(64)
    r = [None] * R
    for c in range(1 << NC):
        rb = [np.array([int(X[store_addr(l, jp, c, L, NC)]) for l in range(64)], dtype=object) for jp in range(32)]
        for b in range(5):                   # GS pass 2
            hh = 1 << b
            for jp in range(32):
                if jp & hh == 0:
                    m = jp >> (b + 1)
                    w = np.array([inv[lane_k(b, c, l, m, L, NC)] for l in lanes], dtype=object)
                    xx, yy = rb[jp], rb[jp + hh]
                    rb[jp], rb[jp + hh] = (xx + yy) % q, (xx - yy) * w % q
        buf = {}
        for jp in range(32):
            for l in range(64):
                Lb = Lane(l, 11)
                buf[Lb.rbase + ((4 * (jp >> 2)) ^ Lb.rxm) + (jp & 3)] = rb[jp][l]
        for t in range(32):
            r[chunk_reg(c, t, H, NC)] = np.array([buf[w_addr(l, t)] for l in range(64)], dtype=object)
    for m in range(H):                       # bit-5 stage GS, then swap back
        w = np.array([inv[(1 << M) + m + H * (l >> 5)] for l in lanes], dtype=object)
        xx, yy = r[m], r[m + H]
        r[m], r[m + H] = (xx + yy) % q, (xx - yy) * w % q
        r[m], r[m + H] = swap32(r[m], r[m + H])
    for s in range(M - 1, -1, -1):           # pass 1 GS, low register bit first
        hh = 1 << (M - 1 - s)
        for j in range(R):
            if j & hh == 0:
                w = inv[(1 << s) + (j >> (M - s))]
                xx, yy = r[j], r[j + hh]
                r[j], r[j + hh] = (xx + yy) % q, (xx - yy) * w % q
    ninv = p["n_inv"]
    out = np.zeros(n, np.uint64)
    for j in range(R):
        for l in range(64):
            out[l + 64 * j] = r[j][l] * ninv % q
    return out.astype(np.uint32)


@pytest.mark.parametrize("ps", LARGE_SETS)
def test_model_equals_oracle(oracle, ps):
    x = oracle.fill_uniform(1, ps, 0xB16 + len(ps), 0)[0]
    X = model_fwd(x, oracle, ps)
    assert np.array_equal(X, oracle.poly_ntt(x[None], ps)[0])
    assert np.array_equal(model_inv(X, oracle, ps), x)
    assert np.array_equal(model_inv(x, oracle, ps), oracle.poly_invntt(x[None], ps)[0])
