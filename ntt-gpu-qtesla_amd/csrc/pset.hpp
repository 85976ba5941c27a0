// pset.hpp -- compile-time parameter sets shared by the gfx950 kernels.
#pragma once
#include <cstdint>

namespace qntt {

// ------------------------------------------------------------------------
// compile-time parameter sets
// ------------------------------------------------------------------------
constexpr uint32_t cpow(uint64_t b, uint64_t e, uint64_t q)
{
    uint64_t r = 1;
    b %= q;
    while (e) {
        if (e & 1) r = r * b % q;
        b = b * b % q;
        e >>= 1;
    }
    return (uint32_t)r;
}
constexpr uint32_t cshoup(uint32_t w, uint32_t q) { return (uint32_t)(((uint64_t)w << 32) / q); }
// Centred twiddle for the signed Shoup product (sshoup_mul): ws = w or w - q,
// whichever lies in (-q/2, q/2], and wps = floor(ws 2^32 / q), both as the
// bit patterns of signed 32-bit values.
struct TwPair { uint32_t x, y; };
constexpr TwPair csigned_tw(uint32_t w, uint32_t q)
{
    const int64_t ws = w <= q / 2 ? (int64_t)w : (int64_t)w - (int64_t)q;
    const int64_t num = ws * ((int64_t)1 << 32);
    const int64_t wps = num >= 0 ? num / (int64_t)q : -((-num + (int64_t)q - 1) / (int64_t)q);
    return {(uint32_t)(int32_t)ws, (uint32_t)(int32_t)wps};
}
constexpr uint32_t cqinv_neg(uint32_t q)
{
    uint32_t inv = q;
    for (int i = 0; i < 5; i++) inv *= 2u - q * inv;
    return 0u - inv;
}

template <uint32_t Q_, int LOGN_, uint32_t PSI_>
struct PSet {
    static constexpr uint32_t Q = Q_;
    static constexpr int LOGN = LOGN_;
    static constexpr uint32_t N = 1u << LOGN_;
    static constexpr uint32_t Q2 = 2 * Q_;
    static constexpr uint32_t PSI = PSI_;
    static constexpr uint32_t QNEG = cqinv_neg(Q_);
    static constexpr uint32_t NINV = cpow(N, Q_ - 2, Q_);
    static constexpr uint32_t PSI_INV = cpow(PSI_, Q_ - 2, Q_);
    // inv twiddle of k = 1 is psi^-brv(1) = psi^-(n/2)
    static constexpr uint32_t C1 = (uint32_t)((uint64_t)NINV * cpow(PSI_INV, N / 2, Q_) % Q_);
    static constexpr uint32_t R = (uint32_t)((1ull << 32) % Q_);
    static constexpr uint32_t NINV_R = (uint32_t)((uint64_t)NINV * R % Q_);
    static constexpr uint32_t C1_R = (uint32_t)((uint64_t)C1 * R % Q_);
    // poly_mul's inverse runs LOGR stages short (residues mod x^(2^LOGR) -
    // zeta, see BaseMul): its final scaling is (n / 2^LOGR)^-1
    template <int LOGR> static constexpr uint32_t ninv_r() { return (uint32_t)((1ull << LOGR) * NINV_R % Q_); }
    template <int LOGR> static constexpr uint32_t c1_r() { return (uint32_t)((1ull << LOGR) * C1_R % Q_); }
};
using PS0 = PSet<8404993u, 10, 2083362u>;
using PS1 = PSet<343576577u, 10, cpow(3, (343576577u - 1) / 2048, 343576577u)>;
using PS2 = PSet<856145921u, 11, cpow(3, (856145921u - 1) / 4096, 856145921u)>;
using PS3 = PSet<856145921u, 12, cpow(3, (856145921u - 1) / 8192, 856145921u)>;
using PS4 = PSet<856145921u, 13, cpow(3, (856145921u - 1) / 16384, 856145921u)>;
static_assert(4ull * PS2::Q < (1ull << 32), "lazy bounds need 4q < 2^32");

template <int PS> struct PSel;
template <> struct PSel<0> { using T = PS0; };
template <> struct PSel<1> { using T = PS1; };
template <> struct PSel<2> { using T = PS2; };
template <> struct PSel<3> { using T = PS3; };
template <> struct PSel<4> { using T = PS4; };

}  // namespace qntt
