"""CPU model of the device arithmetic of csrc/ntt_device.hpp, instruction by
instruction with 32-bit wrap-around (Python ints masked to 32 / 64 bits):
the lazy CT butterfly, the typed "lazy-bias" CT butterfly of poly_mul
(ct_bfly_t: S-form values in (-2q, 2q), signed Shoup quotients with centred
twiddles), the signed Shoup product and BaseMul's zeta-split residue
products.  Checks congruence mod q and the output ranges the kernels rely on,
over edge values and random samples, for every prime.  The GPU parity tests
check the kernels themselves; this pins the bounds the static_asserts and
comments state."""
import random

import pytest

PRIMES = {"ref": 8404993, "p-I": 343576577, "p-III": 856145921}
M32 = (1 << 32) - 1
M64 = (1 << 64) - 1


def s32(x):
    x &= M32
    return x - (1 << 32) if x >> 31 else x


def shoup(w, q):
    return (w << 32) // q


def centred(w, q):
    """csigned_tw (pset.hpp): ws in (-q/2, q/2], wps = floor(ws 2^32 / q)."""
    ws = w if w <= q // 2 else w - q
    return ws, (ws << 32) // q   # Python // floors, as the device constant does


def madlo32(a, b, c):
    return (a * b + c) & M32


def umulhi(a, b):
    return ((a & M32) * (b & M32)) >> 32


def sq_quot(y, wps):
    """e = floor((d * wps - 2^31) / 2^32), d and wps signed (v_mad_i64_i32)."""
    return ((s32(y) * s32(wps) - (1 << 31)) >> 32) & M32


def ct_bfly_t(x, y, w, q, red, xs, ys, yos):
    """ntt_device.hpp ct_bfly_t with the twiddle w in [0, q): returns (x', y')
    as 32-bit words.  Unsigned y: (2^32 - w, w'); signed y: (-ws, ws')."""
    if not red:
        a = x
    elif xs:
        a = min(x, (x + 2 * q) & M32)
    else:
        a = min(x, (x - 2 * q) & M32)
    if ys:
        ws, wps = centred(w, q)
        qe = sq_quot(y, wps & M32)
        tn = madlo32(qe, q, (y * ((-ws) & M32)) & M32)
    else:
        qe = umulhi(y, shoup(w, q))
        tn = madlo32(qe, q, (y * ((-w) & M32)) & M32)
    xo = (a - tn) & M32
    yo = (a + tn) & M32 if yos else (a + tn + 2 * q) & M32
    return xo, yo


def value(word, s):
    """the integer a word stands for: S form is signed"""
    return s32(word) if s else word


def samples(q, s, rng, k=400):
    """edge and random words of a U ([0, 4q)) or S ((-2q, 2q)) operand"""
    if s:
        edge = [0, 1, -1, q - 1, -(q - 1), q, -q, 2 * q - 1, -(2 * q - 1)]
        rnd = [rng.randrange(-2 * q + 1, 2 * q) for _ in range(k)]
    else:
        edge = [0, 1, q - 1, q, 2 * q - 1, 2 * q, 4 * q - 1]
        rnd = [rng.randrange(0, 4 * q) for _ in range(k)]
    return [v & M32 for v in edge + rnd]


@pytest.mark.parametrize("name", list(PRIMES))
@pytest.mark.parametrize("xs,ys,yos", [(False, False, False), (False, False, True), (True, True, True),
                                       (True, True, False), (True, False, True), (True, False, False)])
def test_typed_ct_butterfly(name, xs, ys, yos):
    q = PRIMES[name]
    rng = random.Random(hash((name, xs, ys, yos)) & 0xFFFF)
    ws = [0, 1, q - 1, q // 2, q // 2 + 1] + [rng.randrange(q) for _ in range(40)]
    for w in ws:
        for x, y in zip(samples(q, xs, rng), samples(q, ys, rng)):
            xo, yo = ct_bfly_t(x, y, w, q, True, xs, ys, yos)
            X, Y = value(x, xs), value(y, ys)
            assert 0 <= xo < 4 * q
            assert (xo - (X + w * Y)) % q == 0
            Yv = value(yo, yos)
            assert ((-2 * q < Yv < 2 * q) if yos else (0 <= Yv < 4 * q))
            assert (Yv - (X - w * Y)) % q == 0


@pytest.mark.parametrize("name", list(PRIMES))
def test_canonical_stage0_and_s_canon(name):
    """stage 0 of fwd_pass1_lz: canonical inputs, no reduction, S output; and
    BaseMul::canon: (-2q, 2q) -> [0, q) by
    min(x, x + 2q) then one conditional subtraction of q"""
    q = PRIMES[name]
    rng = random.Random(7)
    for _ in range(2000):
        x, y, w = rng.randrange(q), rng.randrange(q), rng.randrange(q)
        xo, yo = ct_bfly_t(x, y, w, q, False, False, False, True)
        assert 0 <= xo < 4 * q and -2 * q < s32(yo) < 2 * q
        a = min(yo, (yo + 2 * q) & M32)
        c = min(a, (a - q) & M32)
        assert c == (x - w * y) % q


@pytest.mark.parametrize("name", list(PRIMES))
def test_signed_shoup_range(name):
    """sshoup_mul: |d| < 2^31, centred twiddle -> d ws - e q in (0, 2q)"""
    q = PRIMES[name]
    rng = random.Random(3)
    for _ in range(3000):
        d = rng.randrange(-(1 << 31) + 1, 1 << 31)
        w = rng.randrange(q)
        ws, wps = centred(w, q)
        e = sq_quot(d & M32, wps & M32)
        t = ((d & M32) * (ws & M32) - e * q) & M32
        assert 0 < t < 2 * q
        assert (t - d * w) % q == 0


def fwd_signed_table(q, psi, logn):
    """FwdSignedTw<P>: (-ws mod 2^32, wps) of psi^brv(k), k < 32"""
    out = []
    for k in range(32):
        e = int(format(k, f"0{logn}b")[::-1], 2)
        ws, wps = centred(pow(psi, e, q), q)
        out.append(((-ws) & M32, wps & M32))
    return out


def test_fwd_signed_table_is_the_fwd_table_centred(ntt):
    """the compile-time signed pass-1 twiddles name the same psi^brv(k) as the
    library's tables (ntt_get_tables Phi[i] = psi^i)"""
    for name in ("ref", "p-I", "p-III"):
        info = ntt.param_info(name)
        q, n = info["q"], info["n"]
        phi = ntt.tables(name)["Phi"]
        logn = n.bit_length() - 1
        tab = fwd_signed_table(q, info["psi"], logn)
        for k in range(2, 32):
            w = int(phi[int(format(k, f"0{logn}b")[::-1], 2)])
            ws, wps = centred(w, q)
            assert tab[k] == ((-ws) & M32, wps & M32)


def redc(c, q, qneg):
    m = (c * qneg) & M32
    return ((m * q + c) >> 32)


@pytest.mark.parametrize("name", list(PRIMES))
def test_zeta_split_residue_product(name):
    """BaseMul::run_zsplit: c_k = L_k + zR * REDC(H_k) fits 64 bits, its REDC
    lands in [0, 2q) after one conditional subtraction, and equals the
    product mod x^8 - zeta times 2^-32"""
    q = PRIMES[name]
    qinv = pow(q, -1, 1 << 32)
    qneg = (-qinv) & M32
    R = (1 << 32) % q
    rinv = pow(R, -1, q)
    rng = random.Random(11)
    cases = [([q - 1] * 8, [q - 1] * 8, q - 1)] + \
        [([rng.randrange(q) for _ in range(8)], [rng.randrange(q) for _ in range(8)], rng.randrange(q))
         for _ in range(300)]
    for a, b, zeta in cases:
        # device: one negated Shoup product of R by the pair's twiddle w, then
        # the two-candidate min for the +w and the -w residue -> [0, q]
        w = zeta
        tn = madlo32(umulhi(R, shoup(w, q)), q, (R * ((-w) & M32)) & M32)
        for sign in (1, -1):
            if sign == 1:
                zr = min((-tn) & M32, ((-q) - tn) & M32)
            else:
                zr = min((tn + q) & M32, (tn + 2 * q) & M32)
            z = w if sign == 1 else q - w   # the residue's zeta
            assert 0 <= zr <= q and (zr - z * R) % q == 0
            for k in range(8):
                L = sum(a[i] * b[k - i] for i in range(k + 1))
                c = L
                if k < 7:
                    H = sum(a[i] * b[k + 8 - i] for i in range(k + 1, 8))
                    assert H + M32 * q <= M64
                    c += zr * redc(H, q, qneg)
                assert c + M32 * q <= M64, "REDC input fits 64 bits"
                r = redc(c, q, qneg)
                assert r < 4 * q
                r = min(r, (r - 2 * q) & M32)
                assert 0 <= r < 2 * q
                want = (L + z * sum(a[i] * b[k + 8 - i] for i in range(k + 1, 8))) * rinv % q
                assert r % q == want


@pytest.mark.parametrize("name", list(PRIMES))
def test_half_canonical_residue_product_and_wide_first_stage(name):
    """BaseMul::AH, the half-canonical a (p-III, where the z-split output
    needs its csub anyway):
    a in [0, 2q), b canonical -> c_k < 16 q^2 fits 64 bits with the REDC's
    m q; the REDC output after one csub lies below 2.19 q (p-III), and the
    inverse's first GS stage (inv_pass2 WIDE0) maps such x, y to
    (x + y) mod 2q by a three-candidate min, with |x - y| < 2^31"""
    q = PRIMES[name]
    qneg = (-pow(q, -1, 1 << 32)) & M32
    R = (1 << 32) % q
    rinv = pow(R, -1, q)
    rng = random.Random(5)
    cases = [([2 * q - 1] * 8, [q - 1] * 8, q - 1)] + \
        [([rng.randrange(2 * q) for _ in range(8)], [rng.randrange(q) for _ in range(8)], rng.randrange(q))
         for _ in range(300)]
    outs = []
    for a, b, z in cases:
        zr = z * R % q
        for k in range(8):
            L = sum(a[i] * b[k - i] for i in range(k + 1))
            H = sum(a[i] * b[k + 8 - i] for i in range(k + 1, 8))
            c = L + (zr * redc(H, q, qneg) if k < 7 else 0)
            assert c < 16 * q * q and c + M32 * q <= M64
            r = redc(c, q, qneg)
            assert r < 16 * q * q / 2 ** 32 + q
            r = min(r, (r - 2 * q) & M32)
            assert (r - (L + z * H) * rinv) % q == 0
            outs.append(r)
    wh = max(16 * q * q / 2 ** 32 + q - 2 * q, 2 * q)
    assert max(outs) < wh and wh < 3 * q and wh < 2 ** 31
    for _ in range(2000):
        x, y = rng.choice(outs), rng.choice(outs)
        sm = (x + y) & M32
        xo = min(sm, (sm - 2 * q) & M32, (sm - 4 * q) & M32)
        assert xo == (x + y) % (2 * q)
        assert abs(x - y) < 2 ** 31
