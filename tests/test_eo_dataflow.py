"""CPU model of the even/odd n = 8192 transforms (ntt-gpu-qtesla_amd/csrc/ntt_eo.hpp,
DESIGN.md §9): a pair of waves per polynomial, wave parity `par` runs the
n = 4096 transform of x[2i + par] (the validated ntt_big.hpp path, modelled
in test_big_dataflow.py; here the oracle's n = 4096 transform stands in for
it), then the pair exchanges half of every chunk through the two waves' LDS
buffers and each wave runs 16 of the final radix-2 butterflies.  The model
follows the kernel's index maps (the B-layout natural index boff(c, j') +
lane, the exchange rows, the buffer-resource byte offsets, the split twiddle
lambda_l mu of EO_TWJIT) with exact arithmetic mod q and must equal the
oracle's n = 8192 transforms.
"""
import numpy as np
import pytest

from test_lds_layout import brv

N, HN = 8192, 4096


def boff(c, jp):
    """Big<3>::boff: natural index of B-layout register j' of chunk c, lane 0"""
    return (brv(jp, 5) << 7) + (c << 6)


def k_of(par, c, i, lane):
    """natural k of the combine butterfly that wave `par` runs for register i of chunk c"""
    return boff(c, i) + 128 * par + lane


def test_psi_squares(oracle):
    p3, p4 = oracle.params("p-III-4096"), oracle.params("p-III-8192")
    assert p3["q"] == p4["q"]
    assert p4["psi"] ** 2 % p4["q"] == p3["psi"]      # psi_8192^2 = psi_4096 (static_assert in EO)


def test_index_maps():
    # each wave's half: j' = i + 16 par is boff(c, i) + 128 par (brv5 puts bit 4 at bit 0)
    for c in range(2):
        for i in range(16):
            assert boff(c, i + 16) == boff(c, i) + 128
    # the pair's combine butterflies cover k in [0, 4096) exactly once
    ks = sorted(k_of(par, c, i, l) for par in range(2) for c in range(2) for i in range(16) for l in range(64))
    assert ks == list(range(HN))
    # buffer-resource byte offsets stay inside the 32 KiB polynomial / twiddle table
    assert max(4 * (k + HN) for k in ks) < 4 * N
    assert max(8 * k for k in ks) < 8 * HN
    # stride-2 parity loads / stores: lo = 2 lane + par, soffset 512 J, J < 64 registers
    pos = sorted(2 * lane + par + 128 * j for par in range(2) for lane in range(64) for j in range(64))
    assert pos == list(range(N))


def exchange_fwd(A, B):
    """forward exchange: the even wave's buffer holds A, the odd wave's B (rows j',
    lane-contiguous); wave par reads rows 16 par + i of both -> (A, B) at k_of(par, c, i, lane)"""
    out = {}
    for c in range(2):
        abuf = {(jp, l): A[boff(c, jp) + l] for jp in range(32) for l in range(64)}
        bbuf = {(jp, l): B[boff(c, jp) + l] for jp in range(32) for l in range(64)}
        for par in range(2):
            for i in range(16):
                for l in range(64):
                    out[k_of(par, c, i, l)] = (abuf[(16 * par + i, l)], bbuf[(16 * par + i, l)])
    return out


def exchange_inv(A2, B2):
    """inverse exchange: wave par writes its A to its own buffer's row i and B to row
    16 + i; wave par then reads row 16 par + i of the even and of the odd wave's
    buffer into its registers i and 16 + i -> every j' of its own parity"""
    got = {0: np.zeros(HN, dtype=object), 1: np.zeros(HN, dtype=object)}
    for c in range(2):
        buf = {par: {} for par in range(2)}
        for par in range(2):
            for i in range(16):
                for l in range(64):
                    k = k_of(par, c, i, l)
                    buf[par][(i, l)] = A2[k]
                    buf[par][(16 + i, l)] = B2[k]
        for par in range(2):
            for i in range(16):
                for l in range(64):
                    got[par][boff(c, i) + l] = buf[0][(16 * par + i, l)]        # register i
                    got[par][boff(c, 16 + i) + l] = buf[1][(16 * par + i, l)]   # register 16 + i
    return got


@pytest.mark.parametrize("jit", [False, True])
def test_forward_model(oracle, jit):
    q, psi = oracle.params("p-III-8192")["q"], oracle.params("p-III-8192")["psi"]
    x = oracle.fill_uniform(2, "p-III-8192", seed=11)
    for xs in x:
        A = [int(v) for v in oracle.poly_ntt(xs[0::2].copy(), "p-III-4096")]
        B = [int(v) for v in oracle.poly_ntt(xs[1::2].copy(), "p-III-4096")]
        X = np.zeros(N, dtype=np.int64)
        for k, (a, b) in exchange_fwd(A, B).items():
            if jit:   # lambda_l = psi^(2 l), mu = psi^(2 k0 + 1), k0 = k - l
                l = k % 64
                w = pow(psi, 2 * l, q) * pow(psi, 2 * (k - l) + 1, q) % q
            else:     # g_eotw[0][k] = the n = 8192 table's entry 4096 + brv12(k)
                w = pow(psi, brv(HN + brv(k, 12), 13), q)
                assert w == pow(psi, 2 * k + 1, q)
            t = b * w % q
            X[k], X[k + HN] = (a + t) % q, (a - t) % q
        assert np.array_equal(X, oracle.poly_ntt(xs.copy(), "p-III-8192").astype(np.int64))


def test_inverse_model(oracle):
    p = oracle.params("p-III-8192")
    q, psi = p["q"], p["psi"]
    X = oracle.fill_uniform(2, "p-III-8192", seed=12)
    inv2 = pow(2, q - 2, q)
    for Xs in X:
        Xs = [int(v) for v in Xs]
        A2, B2 = [0] * HN, [0] * HN
        for k in range(HN):
            winv = pow(pow(psi, 2 * k + 1, q), q - 2, q)
            A2[k] = (Xs[k] + Xs[k + HN]) % q
            B2[k] = (Xs[k] - Xs[k + HN]) * winv % q
        got = exchange_inv(A2, B2)
        assert list(got[0]) == A2 and list(got[1]) == B2
        # the n = 4096 inverse with n_8192^-1 in its last stage: the combine's 1/2 folded in
        x = np.zeros(N, dtype=np.int64)
        for par in range(2):
            half = oracle.poly_invntt(np.array(got[par], dtype=np.uint32), "p-III-4096").astype(object)
            x[par::2] = [int(v) * inv2 % q for v in half]
        assert np.array_equal(x, oracle.poly_invntt(np.array(Xs, dtype=np.uint32), "p-III-8192").astype(np.int64))
