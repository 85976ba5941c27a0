// nussbaumer.hip -- gfx950 batched Nussbaumer negacyclic product (SURVEY.md 8f,
// config 5): c = a * b mod (x^n + 1) over Z/(2^32-1) (the reference's ring,
// nussbaumer_fft NTT.cu:167-277) or over Z/q (the qTESLA ring; then the result
// equals poly_mul's bit for bit).  No roots of unity in the coefficient ring:
// every "twiddle" is a negacyclic rotation of an inner polynomial.
//
// Geometry (one wave = one n=2048 product, or two n=1024 products):
//   outer level  (m = 32, as NTT.cu:193-201): 64 sub-polynomials of length
//                R = n/32 in Z[y]/(y^R+1).  Lane a (a < R; R = 32 -> one product
//                per 32-lane half) holds coefficient a of every sub-polynomial,
//                register k holds sub-polynomial k.  Butterfly twiddles y^sr are
//                lane rotations: one ds_bpermute + a per-lane sign fix.
//   transpose    wave-private 32 KiB LDS, XOR-swizzled (conflict-free b32 on one
//                side, b128 on the other; tests/test_nussbaumer_model.py).
//   inner level  lane k owns sub-polynomial k of X and Y and multiplies them
//                mod y^R+1 with a second Nussbaumer level (m' = R/8, r' = 8)
//                entirely in registers: rotations are compile-time register
//                renames, 2m' length-8 schoolbook products.  The 2m' points
//                split into two independent blocks after the implicit first
//                stage, which bounds the register peak at 3R values.
//   deferred     the reference halves after every inverse butterfly (moddiv2,
//   scaling      NTT.cu:255-258); here all 2^-L is applied once to `a` on load:
//                a 32-bit rotate in Z/(2^32-1) (2^32 == 1), a Shoup multiply
//                by 2^(32-L) mod q in Z/q (the 2^32 cancels the Montgomery REDC
//                of the inner products).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/qtesla_ntt.h"
#include "ntt_internal.h"
#include "pset.hpp"

namespace qntt {
namespace {

constexpr int NUS_WG = 256;                     // 4 waves, one per SIMD
constexpr int NUS_WAVES = NUS_WG / 64;
constexpr int NUS_WAVE_WORDS = 8192;            // X and Y: 64 rows x R x H = 4096 words each
constexpr int NUS_PPW_MAX = 16;

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

__host__ __device__ constexpr int cbrv(int x, int bits)
{
    int r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
    return r;
}

__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }

// LDS operations of one wave complete in issue order, so the wave-private
// transposes need no s_barrier; this only keeps the compiler from moving
// accesses across the phase boundaries
__device__ __forceinline__ void wave_lds_fence() { asm volatile("" ::: "memory"); }

__device__ __forceinline__ uint32_t bperm(uint32_t byte_addr, uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)byte_addr, (int)v);
}

// ------------------------------------------------------------------------
// geometry of one product
// ------------------------------------------------------------------------
template <uint32_t N>
struct Geo {
    static constexpr int R = (int)N / 32;         // outer inner-length: 64 or 32
    static constexpr int H = 64 / R;              // products per wave
    static constexpr int SC = R / 32;             // outer rotation scale r/m
    static constexpr int MI = R / 8;              // inner m'
    static constexpr int LMI = MI == 8 ? 3 : 2;   // log2 m'
    static constexpr int SCI = 8 / MI;            // inner rotation scale r'/m'
    static constexpr int L = 6 + LMI + 1;         // total deferred 2^-L
    static_assert(N == 1024 || N == 2048, "n = 1024 or 2048");
};

// swizzle of row k (16-byte chunk XOR), see file header
template <int R>
__host__ __device__ constexpr uint32_t swz(uint32_t k)
{
    return R == 64 ? (k & 15u) : (((k >> 1) ^ ((k & 1u) << 2)) & 7u);
}

// ------------------------------------------------------------------------
// rings
// ------------------------------------------------------------------------
template <int RING, class P> struct Ring;

// Z/(2^32-1): ones'-complement arithmetic (NTT.cu:102-134).  Values are any
// 32-bit word; 0xFFFFFFFF is a second zero, mapped to 0 on output.
template <class P>
struct Ring<NTT_RING_M32, P> {
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b)
    {
        uint32_t t;
        const bool c = __builtin_add_overflow(a, b, &t);
        return t + (uint32_t)c;
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b)
    {
        uint32_t t;
        const bool c = __builtin_sub_overflow(a, b, &t);
        return t - (uint32_t)c;
    }
    static __device__ __forceinline__ uint32_t negm(uint32_t a, uint32_t m) { return a ^ m; }
    template <int L>
    static __device__ __forceinline__ uint32_t in_a(uint32_t x) { return __builtin_rotateright32(x, L); }
    static __device__ __forceinline__ uint32_t in_b(uint32_t x) { return x; }
    static __device__ __forceinline__ uint32_t out(uint32_t x) { return x == 0xFFFFFFFFu ? 0u : x; }
    // negacyclic length-8 product; the 64-bit accumulator is folded after every
    // multiply-add (2^32 == 1) so it stays below 2^33 and never overflows
    static __device__ __forceinline__ void mul8(uint32_t (&z)[8], const uint32_t (&u)[8], const uint32_t (&v)[8])
    {
        uint32_t vn[8];
#pragma unroll
        for (int j = 1; j < 8; ++j) vn[j] = ~v[j];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t w = j <= c ? v[c - j] : vn[8 + c - j];
                acc = (uint64_t)u[j] * w + acc;
                if (j < 7) acc = (acc & 0xFFFFFFFFull) + (acc >> 32);
            }
            z[c] = add((uint32_t)acc, (uint32_t)(acc >> 32));
        }
    }
};

// Z/q: values kept in [0, q] (q itself is a second zero), canonical on output.
template <class P>
struct Ring<NTT_RING_Q, P> {
    static constexpr uint32_t Q = P::Q;
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b)
    {
        const uint32_t s = a + b;
        return umin32(s, s - Q);
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b)
    {
        const uint32_t d = a + Q - b;
        return umin32(d, d - Q);
    }
    static __device__ __forceinline__ uint32_t negm(uint32_t a, uint32_t m) { return (m & (Q - a)) | (~m & a); }
    template <int L>
    static __device__ __forceinline__ uint32_t in_a(uint32_t x)
    {
        // x * 2^(32-L) mod q (Shoup), [0, 2q) -> [0, q)
        constexpr uint32_t S = (uint32_t)((uint64_t)cpow(2, 32 - L, Q) % Q);
        constexpr uint32_t SP = cshoup(S, Q);
        const uint32_t t = (uint32_t)((uint64_t)__umulhi(x, SP) * (0u - Q) + x * S);
        return umin32(t, t - Q);
    }
    static __device__ __forceinline__ uint32_t in_b(uint32_t x) { return umin32(x, x - Q); }   // x < 2q
    static __device__ __forceinline__ uint32_t out(uint32_t x) { return umin32(x, x - Q); }
    // sum of 8 products <= 8 q^2 < 2^63, then one Montgomery REDC (x 2^-32)
    static __device__ __forceinline__ void mul8(uint32_t (&z)[8], const uint32_t (&u)[8], const uint32_t (&v)[8])
    {
        static_assert((unsigned __int128)8 * Q * Q + (((unsigned __int128)Q) << 32) < ((unsigned __int128)1 << 64),
                      "REDC input must fit 64 bits");
        constexpr uint64_t TMAX = (uint64_t)(((unsigned __int128)8 * Q * Q) >> 32) + Q + 1;   // REDC output bound
        static_assert(TMAX <= 3ull * Q, "at most two conditional subtractions");
        uint32_t vn[8];
#pragma unroll
        for (int j = 1; j < 8; ++j) vn[j] = Q - v[j];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            uint64_t acc = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += (uint64_t)u[j] * (j <= c ? v[c - j] : vn[8 + c - j]);
            const uint32_t m = (uint32_t)acc * P::QNEG;
            uint32_t t = (uint32_t)(((uint64_t)m * Q + acc) >> 32);
            if constexpr (TMAX > 2ull * Q) t = umin32(t, t - 2 * Q);
            z[c] = umin32(t, t - Q);
        }
    }
};

// ------------------------------------------------------------------------
// outer level (lane = coefficient, register = sub-polynomial)
// ------------------------------------------------------------------------
// forward, NTT.cu:203-244 with sr scaled by r/m; X and Y share the lane
// addresses of each (stage, i) group
template <class RG, class G>
__device__ __forceinline__ void outer_fwd(uint32_t (&X)[64], uint32_t (&Y)[64], uint32_t a4, uint32_t hb4)
{
    static_for<0, 5>([&](auto JJ) {
        constexpr int j = 4 - decltype(JJ)::value;
        static_for<0, (1 << (5 - j))>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = G::SC * (cbrv(i, 5 - j) << j);
            uint32_t addr = 0, mask = 0;
            if constexpr (sr != 0) {
                const int d = (int)a4 - 4 * sr;   // source lane a - sr; wraps (negated) when a < sr
                addr = ((uint32_t)d & (4u * G::R - 1)) | hb4;
                mask = (uint32_t)(d >> 31);
            }
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int I = (i << (j + 1)) + decltype(TT)::value, L = I + (1 << j);
                uint32_t tx = X[L], ty = Y[L];
                if constexpr (sr != 0) {
                    tx = RG::negm(bperm(addr, tx), mask);
                    ty = RG::negm(bperm(addr, ty), mask);
                }
                X[L] = RG::sub(X[I], tx);
                X[I] = RG::add(X[I], tx);
                Y[L] = RG::sub(Y[I], ty);
                Y[I] = RG::add(Y[I], ty);
            });
        });
    });
}

// inverse, NTT.cu:248-270 without the per-stage halving (deferred)
template <class RG, class G>
__device__ __forceinline__ void outer_inv(uint32_t (&Z)[64], uint32_t a4, uint32_t hb4)
{
    static_for<0, 6>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        static_for<0, (1 << (5 - j))>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = j == 5 ? 0 : G::SC * (cbrv(i, 5 - j) << j);
            uint32_t addr = 0, mask = 0;
            if constexpr (sr != 0) {
                const int s = (int)a4 + 4 * sr;   // source lane a + sr; wraps (negated) when a + sr >= R
                addr = ((uint32_t)s & (4u * G::R - 1)) | hb4;
                mask = ~(uint32_t)((s - 4 * G::R) >> 31);
            }
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int A = (i << (j + 1)) + decltype(TT)::value, B = A + (1 << j);
                const uint32_t t = RG::sub(Z[A], Z[B]);
                Z[A] = RG::add(Z[A], Z[B]);
                Z[B] = sr != 0 ? RG::negm(bperm(addr, t), mask) : t;
            });
        });
    });
}

// ------------------------------------------------------------------------
// inner level (lane = sub-polynomial; U[i'][j'] = coefficient MI*j' + i')
// ------------------------------------------------------------------------
template <class RG, class G, int BL>
__device__ __forceinline__ void inner_fwd_block(uint32_t (&U)[G::MI][8])
{
    static_for<0, G::LMI>([&](auto JJ) {
        constexpr int j = G::LMI - 1 - decltype(JJ)::value;
        constexpr int cnt = 1 << (G::LMI - 1 - j);
        static_for<BL * cnt, (BL + 1) * cnt>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = G::SCI * (cbrv(i, G::LMI - j) << j);
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int I = (i << (j + 1)) + decltype(TT)::value - BL * G::MI, L = I + (1 << j);
                uint32_t nl[8], ni[8];
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    if (a >= sr) {   // T[a] = U[L][a - sr]
                        nl[a] = RG::sub(U[I][a], U[L][a - sr]);
                        ni[a] = RG::add(U[I][a], U[L][a - sr]);
                    } else {         // T[a] = -U[L][8 + a - sr]
                        nl[a] = RG::add(U[I][a], U[L][8 + a - sr]);
                        ni[a] = RG::sub(U[I][a], U[L][8 + a - sr]);
                    }
                }
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    U[L][a] = nl[a];
                    U[I][a] = ni[a];
                }
            });
        });
    });
}

template <class RG, class G, int BL>
__device__ __forceinline__ void inner_inv_block(uint32_t (&Z)[G::MI][8])
{
    static_for<0, G::LMI>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        constexpr int cnt = 1 << (G::LMI - 1 - j);
        static_for<BL * cnt, (BL + 1) * cnt>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = G::SCI * (cbrv(i, G::LMI - j) << j);
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int A = (i << (j + 1)) + decltype(TT)::value - BL * G::MI, B = A + (1 << j);
                uint32_t na[8], nb[8];
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    na[a] = RG::add(Z[A][a], Z[B][a]);
                    // Z[B][a] = (Z[A]-Z[B])[a+sr], negated when it wraps
                    nb[a] = a < 8 - sr ? RG::sub(Z[A][a + sr], Z[B][a + sr])
                                       : RG::sub(Z[B][a + sr - 8], Z[A][a + sr - 8]);
                }
#pragma unroll
                for (int a = 0; a < 8; ++a) {
                    Z[A][a] = na[a];
                    Z[B][a] = nb[a];
                }
            });
        });
    });
}

// one inner block: rows -> forward block BL of X and Y -> 8-point products ->
// inverse stages inside the block
template <class RG, class G, int BL>
__device__ __forceinline__ void inner_block(uint32_t (&Z)[G::MI][8], const uint32_t *xrow, const uint32_t *yrow,
                                            uint32_t sw)
{
    uint32_t U[G::MI][8], V[G::MI][8];
#pragma unroll
    for (int ch = 0; ch < G::R / 4; ++ch) {
        const uint4 x = *(const uint4 *)(xrow + (((uint32_t)ch ^ sw) << 2));
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) U[(4 * ch + e) % G::MI][(4 * ch + e) / G::MI] = xs[e];
    }
    inner_fwd_block<RG, G, BL>(U);
#pragma unroll
    for (int ch = 0; ch < G::R / 4; ++ch) {
        const uint4 y = *(const uint4 *)(yrow + (((uint32_t)ch ^ sw) << 2));
        const uint32_t ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) V[(4 * ch + e) % G::MI][(4 * ch + e) / G::MI] = ys[e];
    }
    inner_fwd_block<RG, G, BL>(V);
#pragma unroll
    for (int i = 0; i < G::MI; ++i) RG::mul8(Z[i], U[i], V[i]);
    inner_inv_block<RG, G, BL>(Z);
}

// lane k: W = X_k * Y_k * 2^(LMI+1) mod (y^R + 1), written back over the X row
template <class RG, class G>
__device__ __forceinline__ void inner_product(uint32_t *xrow, const uint32_t *yrow, uint32_t sw)
{
    uint32_t Z0[G::MI][8], Z1[G::MI][8];
    inner_block<RG, G, 0>(Z0, xrow, yrow, sw);
    inner_block<RG, G, 1>(Z1, xrow, yrow, sw);
    uint32_t W[G::R];
#pragma unroll
    for (int t = 0; t < G::MI; ++t) {   // last inverse stage (j = LMI, sr = 0) + recombination
#pragma unroll
        for (int a = 0; a < 8; ++a) {
            const uint32_t s = RG::add(Z0[t][a], Z1[t][a]), d = RG::sub(Z0[t][a], Z1[t][a]);
            Z0[t][a] = s;
            Z1[t][a] = d;
        }
    }
#pragma unroll
    for (int i = 0; i < G::MI; ++i) {
        W[i] = RG::sub(Z0[i][0], Z1[i][7]);
#pragma unroll
        for (int j = 1; j < 8; ++j) W[G::MI * j + i] = RG::add(Z0[i][j], Z1[i][j - 1]);
    }
    wave_lds_fence();
#pragma unroll
    for (int ch = 0; ch < G::R / 4; ++ch)
        *(uint4 *)(xrow + (((uint32_t)ch ^ sw) << 2)) = make_uint4(W[4 * ch], W[4 * ch + 1], W[4 * ch + 2], W[4 * ch + 3]);
}

template <int PS, int RING>
__global__ __launch_bounds__(NUS_WG, 1) void k_nussbaumer(const uint32_t *a, const uint32_t *b, uint32_t *c,
                                                         uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using G = Geo<P::N>;
    using RG = Ring<RING, P>;
    constexpr int R = G::R, H = G::H;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NUS_WAVES * NUS_WAVE_WORDS];

    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    uint32_t *const wl = lds + wave * NUS_WAVE_WORDS;
    const uint32_t ca = lane & (R - 1), h = lane / R;        // outer layout
    const uint32_t a4 = ca * 4, hb4 = h * R * 4;
    const uint32_t nunits = (npoly + H - 1) / H;

    uint32_t u = blockIdx.x * (NUS_WAVES * ppw) + wave;
#pragma unroll 1
    for (uint32_t it = 0; it < ppw; ++it, u += NUS_WAVES) {
        if (u >= nunits) break;
        const uint32_t poly = u * H + h;
        const bool valid = poly < npoly;
        const size_t off = (size_t)poly * P::N + 32u * ca;

        uint32_t X[64], Y[64];
#pragma unroll
        for (int q4 = 0; q4 < 8; ++q4) {
            uint4 x = make_uint4(0, 0, 0, 0), y = make_uint4(0, 0, 0, 0);
            if (valid) {
                x = *(const uint4 *)(a + off + 4 * q4);
                y = *(const uint4 *)(b + off + 4 * q4);
            }
            X[4 * q4 + 0] = RG::template in_a<G::L>(x.x);
            X[4 * q4 + 1] = RG::template in_a<G::L>(x.y);
            X[4 * q4 + 2] = RG::template in_a<G::L>(x.z);
            X[4 * q4 + 3] = RG::template in_a<G::L>(x.w);
            Y[4 * q4 + 0] = RG::in_b(y.x);
            Y[4 * q4 + 1] = RG::in_b(y.y);
            Y[4 * q4 + 2] = RG::in_b(y.z);
            Y[4 * q4 + 3] = RG::in_b(y.w);
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) {   // implicit first stage: X1[i + 32] = X1[i] (NTT.cu:196-200)
            X[k + 32] = X[k];
            Y[k + 32] = Y[k];
        }
        outer_fwd<RG, G>(X, Y, a4, hb4);

        // transpose: row (h, k) of X at wl[(h*64 + k)*R ...], Y at +4096
        wave_lds_fence();
#pragma unroll
        for (int k = 0; k < 64; ++k) {
            const uint32_t o = (h * 64 + k) * R + (ca ^ (swz<R>(k) << 2));
            wl[o] = X[k];
            wl[4096 + o] = Y[k];
        }
        wave_lds_fence();
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
            uint32_t *xrow = wl + (hh * 64 + lane) * R;
            inner_product<RG, G>(xrow, xrow + 4096, swz<R>(lane));
        }
        wave_lds_fence();
        uint32_t Z[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) Z[k] = wl[(h * 64 + k) * R + (ca ^ (swz<R>(k) << 2))];
        wave_lds_fence();
        outer_inv<RG, G>(Z, a4, hb4);

        // recombination (NTT.cu:272-277): c[32a + i] = Z_i[a] + Z_{32+i}[a-1], wrapping negated
        const uint32_t d1 = a4 - 4, addr1 = (d1 & (4u * R - 1)) | hb4, mask1 = (uint32_t)((int)d1 >> 31);
        uint32_t o[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) o[i] = RG::out(RG::add(Z[i], RG::negm(bperm(addr1, Z[32 + i]), mask1)));
        if (valid) {   // both halves of a lane group share validity, so bpermute sources are valid lanes
#pragma unroll
            for (int q4 = 0; q4 < 8; ++q4)
                *(uint4 *)(c + off + 4 * q4) = make_uint4(o[4 * q4], o[4 * q4 + 1], o[4 * q4 + 2], o[4 * q4 + 3]);
        }
    }
}

}  // namespace

int nussbaumer_launch(int ps, int ring, const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch, void *stream,
                      int cus)
{
    const size_t per_wave = ps == 2 ? 1 : 2;
    const size_t units = (batch + per_wave - 1) / per_wave;
    size_t ppw = units / ((size_t)NUS_WAVES * (size_t)cus * 4);
    ppw = ppw < 1 ? 1 : (ppw > NUS_PPW_MAX ? NUS_PPW_MAX : ppw);
    const dim3 grid((uint32_t)((units + NUS_WAVES * ppw - 1) / (NUS_WAVES * ppw)));
    hipStream_t s = (hipStream_t)stream;
    const uint32_t nb = (uint32_t)batch, pw = (uint32_t)ppw;
#define QNTT_NUS(PSV, RV)                                                                                   \
    if (ps == PSV && ring == RV) {                                                                          \
        hipLaunchKernelGGL((k_nussbaumer<PSV, RV>), grid, dim3(NUS_WG), 0, s, a, b, c, nb, pw);             \
        return (int)hipGetLastError();                                                                      \
    }
    QNTT_NUS(0, NTT_RING_Q)
    QNTT_NUS(1, NTT_RING_Q)
    QNTT_NUS(2, NTT_RING_Q)
    QNTT_NUS(1, NTT_RING_M32)   // Z/(2^32-1) does not depend on q: ps 0 and 1 share n = 1024
    if (ps == 0 && ring == NTT_RING_M32) return nussbaumer_launch(1, ring, a, b, c, batch, stream, cus);
    QNTT_NUS(2, NTT_RING_M32)
#undef QNTT_NUS
    return (int)hipErrorInvalidValue;
}

}  // namespace qntt
