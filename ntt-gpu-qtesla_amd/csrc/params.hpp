// params.hpp -- parameter sets and twiddle-table construction (host side).
//
// Product code (not the oracle).  Implements the constants.h table rules of
// the reference:
//   Phi[i]    = psi^i                      constants.h:11-13
//   invPhi[i] = n^-1 * psi^-i              constants.h:19-22 ("combined N-1 and invPhi")
//   tf0[i]    = omega^i,  omega = psi^2    constants.h:29-31, main.cu:119-125 (fg0 = 2893)
//   ti0[i]    = omega^-i                   constants.h:33-35, main.cu:127-130
//   bitrev_tbl[i] = logn-bit reversal      constants.h:3-5, NTT.cu:61-79
// and derives the kernels' merged-twist twiddles with Shoup companions:
//   fwd[k] = psi^{brv(k)},  inv[k] = psi^{-brv(k)},  w' = floor(w * 2^32 / q).
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace qntt {

constexpr int NPARAM_SETS = 5;

struct ParamSet {
    int id;
    uint32_t n, logn, q, psi;
    const char *name;
};

// psi for p-I / p-III: 3^((q-1)/2n) with 3 the smallest primitive root of
// both primes (DESIGN.md "psi choice"); the ref set keeps constants.h's Phi[1].
inline uint32_t powmod(uint64_t b, uint64_t e, uint32_t q)
{
    uint64_t r = 1 % q;
    b %= q;
    while (e) {
        if (e & 1) r = r * b % q;
        b = b * b % q;
        e >>= 1;
    }
    return (uint32_t)r;
}
inline uint32_t invmod(uint32_t a, uint32_t q) { return powmod(a, q - 2, q); }

inline const ParamSet *param_set(int id)
{
    // 3, 4: p-III's prime at n = 4096 / 8192 (q - 1 = 2^14 * 52255 admits
    // negacyclic transforms up to n = 8192), for the multi-wave four-step
    // kernels (ntt_large.hpp)
    static const ParamSet sets[NPARAM_SETS] = {
        {0, 1024, 10, 8404993u, 2083362u, "ref(qTESLA-III-speed r1)"},
        {1, 1024, 10, 343576577u, powmod(3, (343576577u - 1) / 2048, 343576577u), "qTESLA-p-I"},
        {2, 2048, 11, 856145921u, powmod(3, (856145921u - 1) / 4096, 856145921u), "qTESLA-p-III"},
        {3, 4096, 12, 856145921u, powmod(3, (856145921u - 1) / 8192, 856145921u), "p-III-q n=4096"},
        {4, 8192, 13, 856145921u, powmod(3, (856145921u - 1) / 16384, 856145921u), "p-III-q n=8192"},
    };
    return (id >= 0 && id < NPARAM_SETS) ? &sets[id] : nullptr;
}

inline uint32_t bitrev(uint32_t j, uint32_t bits)
{
    return bits ? (__builtin_bitreverse32(j) >> (32 - bits)) : 0;
}

inline uint32_t shoup(uint32_t w, uint32_t q) { return (uint32_t)(((uint64_t)w << 32) / q); }

struct Tables {
    // constants.h-equivalent tables
    std::vector<uint32_t> bitrev_tbl, Phi, invPhi, tf0, ti0;
    // kernel twiddles, interleaved (w, w') pairs, index k in [0, n)
    std::vector<uint32_t> fwd, inv;
    // scaling constants (w, w') pairs:
    //   [0] n^-1, [1] n^-1 * inv[1], [2] n^-1 * 2^32, [3] n^-1 * inv[1] * 2^32,
    //   [4] 2^32 mod q (Montgomery fix-up for the stand-alone pointwise)
    uint32_t scale[10];
    uint32_t qinv_neg;   // -q^-1 mod 2^32 (Montgomery)
    uint32_t omega, omega_inv, n_inv;
};

inline void make_tables(const ParamSet &p, Tables &t)
{
    const uint32_t n = p.n, q = p.q;
    const uint32_t psi_inv = invmod(p.psi, q);
    t.omega = (uint32_t)((uint64_t)p.psi * p.psi % q);
    t.omega_inv = invmod(t.omega, q);
    t.n_inv = invmod(n, q);
    t.bitrev_tbl.resize(n); t.Phi.resize(n); t.invPhi.resize(n); t.tf0.resize(n); t.ti0.resize(n);
    std::vector<uint32_t> ppow(n), ipow(n);
    uint64_t a = 1, b = 1, w = 1, wi = 1, ip = t.n_inv;
    for (uint32_t i = 0; i < n; i++) {
        t.bitrev_tbl[i] = bitrev(i, p.logn);
        ppow[i] = (uint32_t)a;
        ipow[i] = (uint32_t)b;
        t.Phi[i] = (uint32_t)a;
        t.invPhi[i] = (uint32_t)ip;
        t.tf0[i] = (uint32_t)w;
        t.ti0[i] = (uint32_t)wi;
        a = a * p.psi % q;
        b = b * psi_inv % q;
        ip = ip * psi_inv % q;
        w = w * t.omega % q;
        wi = wi * t.omega_inv % q;
    }
    t.fwd.resize(2 * n);
    t.inv.resize(2 * n);
    for (uint32_t k = 0; k < n; k++) {
        uint32_t fw = ppow[bitrev(k, p.logn)], iw = ipow[bitrev(k, p.logn)];
        t.fwd[2 * k] = fw;
        t.fwd[2 * k + 1] = shoup(fw, q);
        t.inv[2 * k] = iw;
        t.inv[2 * k + 1] = shoup(iw, q);
    }
    const uint32_t R = (uint32_t)((1ull << 32) % q);
    const uint32_t c1 = (uint32_t)((uint64_t)t.n_inv * t.inv[2] % q);
    const uint32_t v[5] = {t.n_inv, c1, (uint32_t)((uint64_t)t.n_inv * R % q), (uint32_t)((uint64_t)c1 * R % q), R};
    for (int i = 0; i < 5; i++) {
        t.scale[2 * i] = v[i];
        t.scale[2 * i + 1] = shoup(v[i], q);
    }
    uint32_t inv = q;                                  // Newton: q*inv = 1 mod 2^32
    for (int i = 0; i < 5; i++) inv *= 2u - q * inv;
    t.qinv_neg = 0u - inv;
}

}  // namespace qntt
