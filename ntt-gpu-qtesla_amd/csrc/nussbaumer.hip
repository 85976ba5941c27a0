// nussbaumer.hip -- gfx950 batched Nussbaumer negacyclic product (SURVEY.md 8f,
// config 5): c = a * b mod (x^n + 1) over Z/(2^32-1) (the reference's ring,
// nussbaumer_fft NTT.cu:167-277) or over Z/q (the qTESLA ring; then the result
// equals poly_mul's bit for bit).  No roots of unity in the coefficient ring:
// every "twiddle" is a negacyclic rotation of an inner polynomial.
//
// Geometry: a PAIR of waves computes one n=2048 product (or two n=1024
// products, one per 32-lane half); wave w of the pair owns half w of the
// work at every level, so a lane never holds more than one half:
//   outer level  (m = 32, as NTT.cu:193-201): 64 sub-polynomials of length
//                R = n/32 in Z[y]/(y^R+1).  Lane a holds coefficient a of every
//                sub-polynomial; wave w holds sub-polynomials 32w..32w+31 in
//                registers.  The implicit first stage copies sub-polynomial k
//                to k+32, so both waves start from the same 32 input words and
//                the forward stages j = 4..0 never cross halves.  Butterfly
//                twiddles y^sr are lane rotations: ds_bpermute + a sign fix.
//   transposes   the pair's 32 KiB of LDS holds the X and Y matrices
//                (XOR-swizzled rows, conflict-free b32 on one side, b128 on
//                the other); each wave writes its half of both.
//   inner level  lane k of wave w multiplies block w of X_k * Y_k mod y^R+1:
//                a second Nussbaumer level (m' = R/8, r' = 8) in registers
//                whose 2m' points split into two independent blocks after the
//                implicit first stage; rotations are compile-time register
//                renames, m' length-8 schoolbook products per block.  The two
//                blocks meet again through LDS (last inner stage and the
//                recombination of the halves, read back in the outer layout).
//   outer inverse stages j = 0..4 per half; stage 5 and the final
//                recombination (NTT.cu:272-277) exchange half a sub-polynomial
//                set through LDS, each wave storing half of the output words.
//   16 KiB of LDS and <= 256 VGPRs per wave -> 8 waves (2 per SIMD) per CU,
//   one pair per workgroup (the LDS allocation is padded to hold it there).
//   deferred     the reference halves after every inverse butterfly (moddiv2,
//   scaling      NTT.cu:255-258); here all 2^-L is applied once: a 32-bit
//                rotate of `a` on load in Z/(2^32-1) (2^32 == 1); in Z/q a
//                signed Shoup multiply of the n OUTPUTS by 2^(32-L) mod q (the
//                2^32 cancels the Montgomery REDC of the inner products), which
//                also replaces the output's reduction.
//
// Z/q arithmetic is signed and lazy: values are int32 residues congruent mod q
// with a compile-time magnitude bound; an add or sub is ONE instruction, and a
// centred Barrett reduction (two instructions, |r| < ~q/2) runs on a whole
// stage only where the bound would otherwise pass 2^31 (bounds tracked at
// compile time in units of q/1024, see Ring<NTT_RING_Q> and Schedule).  The
// inner products accumulate signed 64-bit (v_mad_i64_i32) and end in a signed
// Montgomery REDC.  Z/(2^32-1) keeps the reference's ones'-complement words.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "../../include/qtesla_ntt.h"
#include "ntt_internal.h"
#include "pset.hpp"

namespace qntt {
namespace {

#ifndef NUS_WG_CFG
#define NUS_WG_CFG 128   // one pair per workgroup: its barriers wait for the partner only
#endif
#ifndef NUS_OCC_CFG
#define NUS_OCC_CFG 2
#endif
#ifndef NUS_WG_PER_CU
#define NUS_WG_PER_CU 4
#endif
// one pair per workgroup (32 KiB LDS), 4 workgroups per CU: 2 waves per SIMD;
// 4 pairs per 512-thread workgroup measured 1.29x slower (every barrier then
// waits for all 8 waves, profiles/r02/ab_nussbaumer_wg.log).  The allocation is
// padded to 40 KiB so that a fifth workgroup never joins a CU: the kernels
// under 168 VGPRs (n <= 1024) would otherwise run 5 per CU, measured 6 % slower
// (ref 7.10 -> 6.73 ms, p-I mod q 8.16 -> 7.66, mod 2^32-1 10.77 -> 10.44 at
// 4 per CU; 3 per CU is slower again, profiles/r05/ab/ab_nus_lds_*.log).
// Against the round-5 f06b3ab8 build (170 VGPRs at p-I mod q, so already 4 per
// CU there): ref 7.11 -> 6.76 ms, p-I mod 2^32-1 11.11 -> 10.59, n = 2048
// unchanged (ab_nus_lds40_*.log)
constexpr int NUS_WG = NUS_WG_CFG;
constexpr int NUS_WAVES = NUS_WG / 64;
constexpr int NUS_PAIRS = NUS_WAVES / 2;
constexpr int NUS_MAT_WORDS = 4096;             // one 64-row x R x H matrix (16 KiB)
constexpr int NUS_PAIR_WORDS = 2 * NUS_MAT_WORDS;
constexpr int NUS_CU_LDS_WORDS = 160 * 1024 / 4;
// n = 2048 needs > 168 VGPRs, which caps it at 2 waves per SIMD anyway; padding
// it too makes the compiler schedule for that occupancy and spill a VGPR
template <int N> constexpr int nus_lds_words()
{
    return (N < 2048 && NUS_PAIRS * NUS_PAIR_WORDS < NUS_CU_LDS_WORDS / NUS_WG_PER_CU) ? NUS_CU_LDS_WORDS / NUS_WG_PER_CU
                                                                                      : NUS_PAIRS * NUS_PAIR_WORDS;
}
// units per workgroup, per ring.  Z/q: one (no table prologue to amortise;
// 2 % faster than 16 without the prefetch, profiles/r02/s4/ab_nussbaumer_ppw.log,
// and the prefetch does not pay there: p-III 17.68 -> 17.82 ms at 16,
// profiles/r05/ab/ab_nus_v2_p3.log).  Z/(2^32-1) at n = 2048: 16 with the next
// unit's loads prefetched, 21.89 -> 21.47 ms (profiles/r05/ab/ab_nus_v2_p3.log);
// at n = 1024 it does not pay (11.10 -> 11.17 ms, ab_nus_v2_p1.log) and costs
// SGPR spills, so n = 1024 keeps one unit per workgroup
#ifndef NUS_PPW_Q
#define NUS_PPW_Q 1
#endif
#ifndef NUS_PPW_M32
#define NUS_PPW_M32 16
#endif
template <int PS, int RING> constexpr int nus_ppw_max()
{
    return (RING == NTT_RING_M32 && PSel<PS>::T::N == 2048) ? NUS_PPW_M32 : NUS_PPW_Q;
}

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

// Phase stamps, diagnostic builds only (-DNUS_STAMPS, tools/nus_stamps.py):
// s_memtime at the phase boundaries of a unit, after `dep` is computed,
// written by lane 0 of each wave of the first NUS_STAMP_WGS workgroups with
// a vector store (the last unit of a workgroup wins).  In the product build
// NUS_STAMP expands to nothing.
#ifdef NUS_STAMPS
constexpr int NUS_STAMP_N = 16;
constexpr int NUS_STAMP_WGS = 8192;
__device__ unsigned long long g_nus_stamps[NUS_STAMP_WGS * 2][NUS_STAMP_N];
__device__ __forceinline__ void nus_stamp(int k, uint32_t dep)
{
    asm volatile("" ::"v"(dep));
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (blockIdx.x < (uint32_t)NUS_STAMP_WGS && (threadIdx.x & 63) == 0)
        g_nus_stamps[blockIdx.x * 2 + ((threadIdx.x >> 6) & 1)][k] = t;
}
#define NUS_STAMP(k, dep) nus_stamp(k, dep)
#else
#define NUS_STAMP(k, dep) ((void)0)
#endif

// LDS hand-offs between the two waves of a pair: a workgroup barrier (the
// workgroup is one pair; with several pairs per workgroup every pair runs the
// same sequence, so all waves meet there)
__device__ __forceinline__ void pair_sync() { __syncthreads(); }

// keeps the compiler from hoisting the next LDS reads above this point (the
// register peak of the inner level is the operand rows in flight)
__device__ __forceinline__ void lds_order_fence() { asm volatile("" ::: "memory"); }

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
// Both rings carry 32-bit words.  Bounds (Z/q only) are magnitudes in units
// of q/1024, rounded up: RB after red(), IN after in_a / in_b, HR the largest
// bound that stays below 2^31.  An add/sub of two values of bound B gives 2B.
template <int RING, class P> struct Ring;

// Z/(2^32-1): ones'-complement arithmetic (NTT.cu:102-134).  Values are any
// 32-bit word; 0xFFFFFFFF is a second zero, mapped to 0 on output.  Closed
// under add/sub: no reductions (all bounds 0).
template <class P>
struct Ring<NTT_RING_M32, P> {
    static constexpr int RB = 0, IN = 0, HR = 1 << 20;
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b)
    {
        // 33-bit sum in a 64-bit VALU add (no carry in an SGPR pair), then
        // the end-around carry: lo + hi cannot wrap (hi = 1 -> lo <= 2^32 - 2)
        const uint64_t t = (uint64_t)a + b;
        return (uint32_t)t + (uint32_t)(t >> 32);
    }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b)
    {
        uint32_t t;
        const bool c = __builtin_sub_overflow(a, b, &t);
        return t - (uint32_t)c;
    }
    static __device__ __forceinline__ uint32_t negm(uint32_t a, uint32_t m) { return a ^ m; }
    static __device__ __forceinline__ uint32_t red(uint32_t a) { return a; }
    template <int L>
    static __device__ __forceinline__ uint32_t in_a(uint32_t x) { return __builtin_rotateright32(x, L); }
    static __device__ __forceinline__ uint32_t in_b(uint32_t x) { return x; }
    template <int B>
    static __device__ __forceinline__ uint32_t out(uint32_t x) { return x == 0xFFFFFFFFu ? 0u : x; }
    // the deferred 2^-L is a rotate here: applied to a on load
    template <int L>
    static __device__ __forceinline__ uint32_t in_x(uint32_t x) { return in_a<L>(x); }
    template <int L, int B>
    static __device__ __forceinline__ uint32_t out_s(uint32_t x) { return out<B>(x); }
    static constexpr bool mul_ok(int, int) { return true; }
    static constexpr int mul_out(int, int) { return 0; }
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

// Z/q, signed lazy residues (file header).  red() is a centred Barrett with
// MB = round(2^32 / q): e = round(a MB / 2^32) (one v_mad_i64_i32 with the
// rounding constant), r = a - e q (one v_mad_u64_u32);
// |a/q - a MB/2^32| < EPS for |a| < 2^31, so |r| < (1/2 + EPS) q.
template <class P>
struct Ring<NTT_RING_Q, P> {
    static constexpr uint32_t Q = P::Q;
    static constexpr int64_t MB = ((1ll << 32) + Q / 2) / Q;
    static constexpr double EPS =
        2147483648.0 * (double)((1ll << 32) > MB * Q ? (1ll << 32) - MB * Q : MB * Q - (1ll << 32)) /
        ((double)Q * 4294967296.0);
    static constexpr int RB = (int)((0.5 + EPS) * 1024.0) + 2;
    static constexpr int IN = 1024;                                   // |x - q| <= q
    static constexpr int HR = (int)(2147483647.0 / (double)Q * 1024.0) - 1;
    static_assert(2 * RB <= HR, "a reduced value must survive one add/sub");

    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
    static __device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return a - b; }
    static __device__ __forceinline__ uint32_t negm(uint32_t a, uint32_t m) { return (a ^ m) - m; }
    static __device__ __forceinline__ uint32_t red(uint32_t a)
    {
        const uint32_t e = (uint32_t)(((int64_t)(int32_t)a * MB + 0x80000000ll) >> 32);
        return (uint32_t)((uint64_t)e * (0u - Q) + a);
    }
    template <int L>
    static __device__ __forceinline__ uint32_t in_a(uint32_t x)
    {
        // x * 2^(32-L) mod q (Shoup), x < 2q -> [0, 2q) -> centred [-q, q)
        constexpr uint32_t S = (uint32_t)((uint64_t)cpow(2, 32 - L, Q) % Q);
        constexpr uint32_t SP = cshoup(S, Q);
        const uint32_t t = (uint32_t)((uint64_t)__umulhi(x, SP) * (0u - Q) + x * S);
        return t - Q;
    }
    static __device__ __forceinline__ uint32_t in_b(uint32_t x) { return x - Q; }   // x < 2q
    // canonical [0, q) from a value of bound B
    template <int B>
    static __device__ __forceinline__ uint32_t out(uint32_t x)
    {
        if constexpr (B > RB) x = red(x);
        return umin32(x, x + Q);   // (-q, q) -> [0, q)
    }
    // a enters like b; the deferred 2^-L (times the 2^32 that cancels the
    // inner REDCs) is applied to the n outputs instead of the n inputs of a:
    // a signed Shoup product by S = 2^(32-L) mod q (any int32 x, centred
    // twiddle, quotient estimate minus one: result in (0, 2q)) that also
    // replaces the output's reduction, then one conditional subtraction
    template <int L>
    static __device__ __forceinline__ uint32_t in_x(uint32_t x) { return in_b(x); }
    template <int L, int B>
    static __device__ __forceinline__ uint32_t out_s(uint32_t x)
    {
        constexpr uint32_t S = (uint32_t)((uint64_t)cpow(2, 32 - L, Q) % Q);
        constexpr TwPair C = csigned_tw(S, Q);
        const uint32_t e = (uint32_t)(((int64_t)(int32_t)x * (int32_t)C.y - 0x80000000ll) >> 32);
        const uint32_t t = (uint32_t)((uint64_t)e * (0u - Q) + x * C.x);
        return umin32(t, t - Q);
    }
    // products of bounds Bu, Bv: 8 terms must fit a signed 64-bit accumulator
    static constexpr bool mul_ok(int bu, int bv)
    {
        return 8.0 * (bu / 1024.0) * (bv / 1024.0) * (double)Q * (double)Q < 9.2e18;
    }
    // REDC output bound: |acc| / 2^32 + q/2
    static constexpr int mul_out(int bu, int bv)
    {
        return (int)((8.0 * (bu / 1024.0) * (bv / 1024.0) * (double)Q / 4294967296.0 + 0.5) * 1024.0) + 2;
    }
    // negacyclic length-8 product, signed 64-bit sums, one signed Montgomery
    // REDC per output (x 2^-32): m = acc * q^-1 mod 2^32, (acc - m q) / 2^32
    static __device__ __forceinline__ void mul8(uint32_t (&z)[8], const uint32_t (&u)[8], const uint32_t (&v)[8])
    {
        uint32_t vn[8];
#pragma unroll
        for (int j = 1; j < 8; ++j) vn[j] = 0u - v[j];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            int64_t acc = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += (int64_t)(int32_t)u[j] * (int32_t)(j <= c ? v[c - j] : vn[8 + c - j]);
            const uint32_t m = (uint32_t)acc * (0u - P::QNEG);   // q^-1 mod 2^32
            z[c] = (uint32_t)(acc >> 32) - (uint32_t)__mulhi((int)m, (int)Q);
        }
    }
};

// Bound bookkeeping of a transform stage: inputs of bound b are reduced
// first when one add/sub would pass HR.
template <class RG> constexpr bool stage_red(int b) { return 2 * b > RG::HR; }
template <class RG> constexpr int stage_out(int b) { return 2 * (stage_red<RG>(b) ? RG::RB : b); }
template <class RG> constexpr int stages_out(int b, int s) { return s == 0 ? b : stages_out<RG>(stage_out<RG>(b), s - 1); }
template <class RG> constexpr int reduced_if(bool c, int b) { return c ? RG::RB : b; }

template <class RG, int NREG>
__device__ __forceinline__ void red_all(uint32_t (&v)[NREG])
{
#pragma unroll
    for (int k = 0; k < NREG; ++k) v[k] = RG::red(v[k]);
}

// ------------------------------------------------------------------------
// outer level (lane = coefficient, register = sub-polynomial of half W)
// ------------------------------------------------------------------------
// forward, NTT.cu:203-244 with sr scaled by r/m, stages j = 4..0 restricted to
// the groups of half W (register k = sub-polynomial 32W + k); X and Y share
// the lane addresses of each (stage, i) group.  Inputs of bound B0.
template <class RG, class G, int B0, int W>
__device__ __forceinline__ void outer_fwd_half(uint32_t (&X)[32], uint32_t (&Y)[32], uint32_t a4, uint32_t hb4)
{
    static_for<0, 5>([&](auto JJ) {
        constexpr int s = decltype(JJ)::value, j = 4 - s;
        if constexpr (stage_red<RG>(stages_out<RG>(B0, s))) {
            red_all<RG>(X);
            red_all<RG>(Y);
        }
        constexpr int gh = 1 << (4 - j);   // groups per half
        static_for<W * gh, (W + 1) * gh>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = G::SC * (cbrv(i, 5 - j) << j);
            uint32_t addr = 0, mask = 0;
            if constexpr (sr != 0) {
                const int d = (int)a4 - 4 * sr;   // source lane a - sr; wraps (negated) when a < sr
                addr = ((uint32_t)d & (4u * G::R - 1)) | hb4;
                mask = (uint32_t)(d >> 31);
            }
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int I = (i << (j + 1)) + decltype(TT)::value - 32 * W, L = I + (1 << j);
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

// inverse, NTT.cu:248-270 without the per-stage halving (deferred), stages
// j = 0..4 of half W (stage 5 crosses the halves: see the kernel).  Inputs of
// bound B0.
template <class RG, class G, int B0, int W>
__device__ __forceinline__ void outer_inv_half(uint32_t (&Z)[32], uint32_t a4, uint32_t hb4)
{
    static_for<0, 5>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        if constexpr (stage_red<RG>(stages_out<RG>(B0, j))) red_all<RG>(Z);
        constexpr int gh = 1 << (4 - j);
        static_for<W * gh, (W + 1) * gh>([&](auto II) {
            constexpr int i = decltype(II)::value;
            constexpr int sr = G::SC * (cbrv(i, 5 - j) << j);
            uint32_t addr = 0, mask = 0;
            if constexpr (sr != 0) {
                const int s = (int)a4 + 4 * sr;   // source lane a + sr; wraps (negated) when a + sr >= R
                addr = ((uint32_t)s & (4u * G::R - 1)) | hb4;
                mask = ~(uint32_t)((s - 4 * G::R) >> 31);
            }
            static_for<0, (1 << j)>([&](auto TT) {
                constexpr int A = (i << (j + 1)) + decltype(TT)::value - 32 * W, B = A + (1 << j);
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
template <class RG, class G, int BL, int B0>
__device__ __forceinline__ void inner_fwd_block(uint32_t (&U)[G::MI][8])
{
    static_for<0, G::LMI>([&](auto JJ) {
        constexpr int s = decltype(JJ)::value, j = G::LMI - 1 - s;
        if constexpr (stage_red<RG>(stages_out<RG>(B0, s)))
            static_for<0, G::MI>([&](auto K) { red_all<RG>(U[decltype(K)::value]); });
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

template <class RG, class G, int BL, int B0>
__device__ __forceinline__ void inner_inv_block(uint32_t (&Z)[G::MI][8])
{
    static_for<0, G::LMI>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        if constexpr (stage_red<RG>(stages_out<RG>(B0, j)))
            static_for<0, G::MI>([&](auto K) { red_all<RG>(Z[decltype(K)::value]); });
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

// Bounds through the inner level for rows of bound BR: the forward's output,
// a reduction if the products' accumulator needs it, the REDC output and the
// inverse's output.
template <class RG, class G, int BR> struct InnerBounds {
    static constexpr int FWD = stages_out<RG>(BR, G::LMI);
    static constexpr bool MRED = !RG::mul_ok(FWD, FWD);
    static constexpr int MIN = reduced_if<RG>(MRED, FWD);
    static_assert(RG::mul_ok(MIN, MIN), "inner products must fit the accumulator");
    static constexpr int PROD = RG::mul_out(MIN, MIN);
    static constexpr int INV = stages_out<RG>(PROD, G::LMI);
};

template <class G>
__device__ __forceinline__ void read_row(uint32_t (&U)[G::MI][8], const uint32_t *row, uint32_t sw)
{
#pragma unroll
    for (int ch = 0; ch < G::R / 4; ++ch) {
        const uint4 x = *(const uint4 *)(row + (((uint32_t)ch ^ sw) << 2));
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) U[(4 * ch + e) % G::MI][(4 * ch + e) / G::MI] = xs[e];
    }
}

// block BL of one row product: rows of X and Y from LDS -> forward block BL
// of both -> m' 8-point products -> inverse stages inside the block
template <class RG, class G, int BL, int BR>
__device__ __forceinline__ void inner_block(uint32_t (&Z)[G::MI][8], const uint32_t *xrow, const uint32_t *yrow,
                                            uint32_t sw)
{
    using IB = InnerBounds<RG, G, BR>;
    uint32_t U[G::MI][8], V[G::MI][8];
    read_row<G>(U, xrow, sw);
    inner_fwd_block<RG, G, BL, BR>(U);
    lds_order_fence();
    read_row<G>(V, yrow, sw);
    inner_fwd_block<RG, G, BL, BR>(V);
    if constexpr (IB::MRED) {
        static_for<0, G::MI>([&](auto K) {
            red_all<RG>(U[decltype(K)::value]);
            red_all<RG>(V[decltype(K)::value]);
        });
    }
#pragma unroll
    for (int i = 0; i < G::MI; ++i) RG::mul8(Z[i], U[i], V[i]);
    inner_inv_block<RG, G, BL, IB::PROD>(Z);
}

// Bounds of the last inner stage (s = Z0 + Z1, d = Z0 - Z1) and of the
// recombination W[c] = s[c] + d[c - m'] (negated when it wraps).
template <class RG, class G, int BR> struct RowOutBounds {
    static constexpr int INV = InnerBounds<RG, G, BR>::INV;
    static constexpr bool R1 = stage_red<RG>(INV);
    static constexpr int REC = stage_out<RG>(INV);
    static constexpr bool R2 = stage_red<RG>(REC);
    static constexpr int W = stage_out<RG>(REC);
};

// Whole-product bound schedule (units of q/1024; 0 everywhere for Z/(2^32-1)).
template <class RG> struct Schedule {
    static constexpr int OFWD = stages_out<RG>(RG::IN, 5);   // after the outer forward
    // rows enter the inner level reduced when the forward left them above RB
    static constexpr bool ROWRED = OFWD > RG::RB;
    static constexpr int ROW = reduced_if<RG>(ROWRED, OFWD);
};

// offset of coefficient a of row (h, k) inside a matrix
template <int R>
__device__ __forceinline__ uint32_t mat_off(uint32_t h, int k, uint32_t a)
{
    return (h * 64 + k) * R + (a ^ (swz<R>(k) << 2));
}

// The 32 input words of a lane for unit u (raw, before in_x / in_b): lane
// a of half h holds words 32 a .. 32 a + 31 of product u H + h.  Loads are
// unconditional: an idle half-wave (odd n=1024 batch) reads the unit's
// first product and never stores; both waves of the pair load the same
// words (the implicit first stage copies sub-polynomial k to k + 32).
template <int PS>
__device__ __forceinline__ void nus_load(const uint32_t *a, const uint32_t *b, uint32_t npoly, uint32_t u,
                                         uint32_t (&X)[32], uint32_t (&Y)[32])
{
    using P = typename PSel<PS>::T;
    using G = Geo<P::N>;
    uint32_t lane = threadIdx.x & 63u;
    asm volatile("" : "+v"(lane));
    const uint32_t ca = lane & (G::R - 1), h = lane / G::R;
    const uint32_t poly = u * G::H + h;
    const size_t loff = (size_t)(poly < npoly ? poly : u * G::H) * P::N + 32u * ca;
#pragma unroll
    for (int q4 = 0; q4 < 8; ++q4) {
        const uint4 x = *(const uint4 *)(a + loff + 4 * q4);
        const uint4 y = *(const uint4 *)(b + loff + 4 * q4);
        X[4 * q4 + 0] = x.x;
        X[4 * q4 + 1] = x.y;
        X[4 * q4 + 2] = x.z;
        X[4 * q4 + 3] = x.w;
        Y[4 * q4 + 0] = y.x;
        Y[4 * q4 + 1] = y.y;
        Y[4 * q4 + 2] = y.z;
        Y[4 * q4 + 3] = y.w;
    }
}

// One unit (one n=2048 product or two n=1024 products) by wave W of a pair.
// X / Y: this unit's raw input words (nus_load).  The next unit (u_next,
// npoly_next) is loaded into X / Y while this one runs -- issued once the
// inner level's results are in LDS (the register peak is past), so its HBM
// latency hides behind the recombination, the outer inverse and the stores
// instead of stalling the next unit's start (PF: the launch runs several units
// per workgroup).  The load is unconditional (a workgroup's last unit reloads
// itself, unused): a branch around it would end in a join that waits for the
// loads on the spot.  `last`: the workgroup's last unit skips the final
// barrier (it only frees the exchange area for a next unit).
template <int PS, int RING, int W, bool PF>
__device__ __forceinline__ void nus_unit(const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t npoly, uint32_t u,
                                         uint32_t *pl, uint32_t (&X)[32], uint32_t (&Y)[32], uint32_t u_next,
                                         uint32_t npoly_next, bool last)
{
    using P = typename PSel<PS>::T;
    using G = Geo<P::N>;
    using RG = Ring<RING, P>;
    using SCH = Schedule<RG>;
    using OB = RowOutBounds<RG, G, SCH::ROW>;
    constexpr int R = G::R, H = G::H, MI = G::MI;
    uint32_t *const xm = pl, *const ym = pl + NUS_MAT_WORDS;

    // lane, opaque per unit: the ~30 per-group rotation addresses and masks and
    // the ~30 swizzled LDS offsets derived from it are recomputed (1-3 VALU
    // each) instead of being hoisted out of the unit loop into registers
    // (they would spill to scratch)
    uint32_t lane = threadIdx.x & 63u;
    asm volatile("" : "+v"(lane));
    const uint32_t ca = lane & (R - 1), h = lane / R;   // outer layout
    const uint32_t a4 = ca * 4, hb4 = h * R * 4;
    const uint32_t poly = u * H + h;
    const bool valid = poly < npoly;
    NUS_STAMP(0, lane);

    {
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            X[k] = RG::template in_x<G::L>(X[k]);
            Y[k] = RG::in_b(Y[k]);
        }
        NUS_STAMP(1, X[31] ^ Y[31]);
        outer_fwd_half<RG, G, RG::IN, W>(X, Y, a4, hb4);
        if constexpr (SCH::ROWRED) {
            red_all<RG>(X);
            red_all<RG>(Y);
        }
        // this half's rows of both matrices
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            xm[mat_off<R>(h, 32 * W + k, ca)] = X[k];
            ym[mat_off<R>(h, 32 * W + k, ca)] = Y[k];
        }
        NUS_STAMP(2, X[31] ^ Y[31]);
    }
    pair_sync();
    NUS_STAMP(3, lane);

    // block W of every row product: lane = sub-polynomial (row), all H products
    uint32_t Zb[H][MI][8];
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
        inner_block<RG, G, W, SCH::ROW>(Zb[hh], xm + (hh * 64 + lane) * R, ym + (hh * 64 + lane) * R, swz<R>(lane));
    NUS_STAMP(4, Zb[H - 1][MI - 1][7] ^ Zb[0][0][0]);
    pair_sync();   // both waves are done reading the matrices
    NUS_STAMP(5, lane);
    uint32_t *const zm = W == 0 ? xm : ym;   // block W's results, same row layout
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
        uint32_t *row = zm + (hh * 64 + lane) * R;
#pragma unroll
        for (int ch = 0; ch < R / 4; ++ch) {
            const int c0 = 4 * ch;
            *(uint4 *)(row + (((uint32_t)ch ^ swz<R>(lane)) << 2)) =
                make_uint4(Zb[hh][(c0 + 0) % MI][(c0 + 0) / MI], Zb[hh][(c0 + 1) % MI][(c0 + 1) / MI],
                           Zb[hh][(c0 + 2) % MI][(c0 + 2) / MI], Zb[hh][(c0 + 3) % MI][(c0 + 3) / MI]);
        }
    }
    if constexpr (PF) nus_load<PS>(a, b, npoly_next, u_next, X, Y);   // the next unit's words (see above)
    NUS_STAMP(6, lane);
    pair_sync();
    NUS_STAMP(7, lane);

    // back in the outer layout for this half: the last inner stage of the two
    // blocks (s, d) and the recombination W[a] = s[a] + d[a - m'], negated
    // when it wraps (a < m')
    uint32_t Z[32];
    {
        const uint32_t ap = (ca - MI) & (R - 1);
        const uint32_t wmask = ca < (uint32_t)MI ? 0xFFFFFFFFu : 0u;
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const int kk = 32 * W + k;
            uint32_t z0 = xm[mat_off<R>(h, kk, ca)], z1 = ym[mat_off<R>(h, kk, ca)];
            uint32_t p0 = xm[mat_off<R>(h, kk, ap)], p1 = ym[mat_off<R>(h, kk, ap)];
            if constexpr (OB::R1) {
                z0 = RG::red(z0);
                z1 = RG::red(z1);
                p0 = RG::red(p0);
                p1 = RG::red(p1);
            }
            uint32_t s = RG::add(z0, z1), d = RG::sub(p0, p1);
            if constexpr (OB::R2) {
                s = RG::red(s);
                d = RG::red(d);
            }
            Z[k] = RG::add(s, RG::negm(d, wmask));
        }
    }
    NUS_STAMP(8, Z[31] ^ Z[0]);
    outer_inv_half<RG, G, OB::W, W>(Z, a4, hb4);
    constexpr int B5 = stages_out<RG>(OB::W, 5);
    NUS_STAMP(9, Z[31] ^ Z[0]);
    pair_sync();   // both waves are done reading the block results

    // stage 5 (sr = 0) pairs sub-polynomials i and i + 32 across the halves,
    // then c[32a + i] = Z'_i[a] + Z'_{32+i}[a-1] (NTT.cu:272-277); wave W
    // finishes i in [16W, 16W + 16) with the other wave's registers 16W..16W+15
    {
        uint32_t *xo = pl + W * 1024;   // what the other wave needs
#pragma unroll
        for (int k = 0; k < 16; ++k) xo[k * 64 + lane] = Z[16 * (1 - W) + k];
    }
    NUS_STAMP(10, lane);
    pair_sync();
    NUS_STAMP(11, lane);
    const uint32_t *xi = pl + (1 - W) * 1024;
    const uint32_t d1 = a4 - 4, addr1 = (d1 & (4u * R - 1)) | hb4, mask1 = (uint32_t)((int)d1 >> 31);
    constexpr bool FR5 = stage_red<RG>(B5);
    constexpr int BA = stage_out<RG>(B5);
    constexpr bool FRO = stage_red<RG>(BA);
    uint32_t o[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
        const int i = 16 * W + t;   // output column
        // sub-polynomial i (half 0) and i + 32 (half 1)
        uint32_t zl = W == 0 ? Z[i] : xi[t * 64 + lane];
        uint32_t zh = W == 0 ? xi[t * 64 + lane] : Z[i];
        if constexpr (FR5) {
            zl = RG::red(zl);
            zh = RG::red(zh);
        }
        uint32_t A = RG::add(zl, zh), B = RG::sub(zl, zh);
        if constexpr (FRO) {
            A = RG::red(A);
            B = RG::red(B);
        }
        o[t] = RG::template out_s<G::L, stage_out<RG>(BA)>(RG::add(A, RG::negm(bperm(addr1, B), mask1)));
    }
    if (valid) {   // both halves of a lane group share validity, so bpermute sources are valid lanes
        uint32_t *dst = c + (size_t)poly * P::N + 32u * ca + 16 * W;
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4)
            *(uint4 *)(dst + 4 * q4) = make_uint4(o[4 * q4], o[4 * q4 + 1], o[4 * q4 + 2], o[4 * q4 + 3]);
    }
    NUS_STAMP(12, o[15] ^ o[0]);
    // the exchange area is free for the next unit (wave-uniform, pair-uniform);
    // a one-unit-per-workgroup kernel (!PF) never has a next unit
    if constexpr (PF) {
        if (!last) pair_sync();
    }
    NUS_STAMP(13, lane);
}

template <int PS, int RING>
__global__ __launch_bounds__(NUS_WG, NUS_OCC_CFG) void k_nussbaumer(const uint32_t *a, const uint32_t *b, uint32_t *c,
                                                                   uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    constexpr int H = Geo<P::N>::H;
    __shared__ __attribute__((aligned(16))) uint32_t lds[nus_lds_words<P::N>()];
    const uint32_t wave = threadIdx.x >> 6, pair = wave >> 1;
    uint32_t *const pl = lds + pair * NUS_PAIR_WORDS;
    const uint32_t nunits = (npoly + H - 1) / H;
    constexpr bool PF = nus_ppw_max<PS, RING>() > 1;   // several units per workgroup: prefetch the next
    if constexpr (!PF) ppw = 1;   // the host's cap for these kernels (nussbaumer_launch); no final barrier below
    // every pair of the workgroup runs the same number of units (idle pairs
    // past the batch still meet the barriers)
    uint32_t u = blockIdx.x * (NUS_PAIRS * ppw) + pair;
    const uint32_t first = blockIdx.x * (NUS_PAIRS * ppw);
    if (first >= nunits) return;   // whole workgroup idle (uniform)
    const uint32_t wg_units = min((uint32_t)(NUS_PAIRS * ppw), nunits - first);
    const uint32_t steps = (wg_units + NUS_PAIRS - 1) / NUS_PAIRS;
    // a pair past the batch recomputes the workgroup's first unit and stores nothing
    auto unit_of = [&](uint32_t v) { return v < nunits ? v : first; };
    auto np_of = [&](uint32_t v) { return v < nunits ? npoly : 0u; };
    uint32_t X[32], Y[32];
#pragma unroll 1
    for (uint32_t it = 0; it < steps; ++it, u += NUS_PAIRS) {
        if (!PF || it == 0) nus_load<PS>(a, b, np_of(u), unit_of(u), X, Y);
        const bool last = it + 1 == steps;
        const uint32_t v = last ? u : u + NUS_PAIRS;   // (the last unit reloads itself, unused)
        const uint32_t un = unit_of(v), npn = np_of(v);
        if ((wave & 1) == 0) nus_unit<PS, RING, 0, PF>(a, b, c, np_of(u), unit_of(u), pl, X, Y, un, npn, last);
        else nus_unit<PS, RING, 1, PF>(a, b, c, np_of(u), unit_of(u), pl, X, Y, un, npn, last);
    }
}

}  // namespace

#ifdef NUS_STAMPS
extern "C" int nus_debug_stamps(unsigned long long *host, size_t count)
{
    const size_t n = sizeof(g_nus_stamps) / sizeof(unsigned long long);
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_nus_stamps), (count < n ? count : n) * 8, 0,
                                    hipMemcpyDeviceToHost);
}
#endif

int nussbaumer_launch(int ps, int ring, const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch, void *stream,
                      int cus)
{
    const size_t per_unit = ps == 2 ? 1 : 2;
    const size_t units = (batch + per_unit - 1) / per_unit;
    size_t ppw = units / ((size_t)NUS_PAIRS * (size_t)cus * 2);
    const size_t pmax = (size_t)((ring == NTT_RING_M32 && ps == 2) ? nus_ppw_max<2, NTT_RING_M32>() : nus_ppw_max<0, NTT_RING_Q>());
    ppw = ppw < 1 ? 1 : (ppw > pmax ? pmax : ppw);
    const dim3 grid((uint32_t)((units + NUS_PAIRS * ppw - 1) / (NUS_PAIRS * ppw)));
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
