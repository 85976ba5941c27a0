// ntt_kernels.hip -- CDNA4 (gfx950) kernels for the batched negacyclic NTT.
//
// Replaces the reference's 10-34 per-stage launches per batch (NTT.cu:2388-2425)
// with one persistent launch per operation.  Geometry (DESIGN.md "kernels"):
//
//   * one wave owns one n=2048 polynomial, or two n=1024 polynomials (one per
//     32-lane half); every lane holds 32 coefficients in VGPRs;
//   * pass 1: register layout pos = Lp + S*j (S = 64 or 32, j = 0..31); the
//     five stages on pos bits [LOGN-5, LOGN-1] are in-register radix-2
//     butterflies with wave-uniform twiddles (scalar loads from __constant__);
//   * n = 2048 only: the stage on pos bit 5 pairs lanes l and l^32 and runs on
//     v_permlane32_swap (no LDS);
//   * one wave-private LDS transpose (conflict-free XOR swizzle, 32 x ds_write_b32
//     + 8 x ds_read_b128 per lane, no s_barrier) to layout pos = 32*Lp + j;
//   * pass 2: the five stages on pos bits [0,4] in registers with per-lane
//     twiddles held in VGPRs for the whole persistent loop;
//   * forward output is bit-reversed in registers; it is written in natural
//     order directly: for fixed j the 64 lanes cover one contiguous 256-B chunk.
//
// Arithmetic: Harvey lazy butterflies with Shoup (precomputed-quotient
// Barrett) multiplication, q < 2^30 so 4q < 2^32:
//   CT: x in [0,4q) -> x' = x mod 2q;  t = y*w mod q in [0,2q);
//       (x'+t, x'-t+2q) in [0,4q)^2
//   GS: (x+y reduced to [0,2q), (x-y+2q)*w in [0,2q))
// Outputs are reduced to canonical [0,q) before they are stored.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>

#include "../../include/qtesla_ntt.h"
#include "params.hpp"
#include "pset.hpp"
#include "ntt_internal.h"

namespace qntt {


// twiddles (w, w'), index k in [0, n): fwd = psi^brv(k), inv = psi^-brv(k)
__constant__ uint2 c_fwd0[1024];
__constant__ uint2 c_inv0[1024];
__constant__ uint2 c_fwd1[1024];
__constant__ uint2 c_inv1[1024];
__constant__ uint2 c_fwd2[2048];
__constant__ uint2 c_inv2[2048];

template <int PS, bool INV>
__device__ __forceinline__ uint2 twd(uint32_t k)
{
    if constexpr (PS == 0) return INV ? c_inv0[k] : c_fwd0[k];
    else if constexpr (PS == 1) return INV ? c_inv1[k] : c_fwd1[k];
    else return INV ? c_inv2[k] : c_fwd2[k];
}

// ------------------------------------------------------------------------
// modular arithmetic
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// NTT_FAKE_MUL (diagnostic builds only, results are wrong): every mul-class
// instruction is replaced 1:1 by a cheap VALU op with the same dependences,
// to price the 32-bit multiplies inside the real kernels.
#ifndef NTT_FAKE_MUL
#define NTT_FAKE_MUL 0
#endif
// NTT_FAKE_TW (diagnostic builds only): twiddles are compile-time constants
// instead of table loads, to price the twiddle fetches.
#ifndef NTT_FAKE_TW
#define NTT_FAKE_TW 0
#endif
__device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b)
{
#if NTT_FAKE_MUL
    uint32_t r;
    asm volatile("v_xor_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return __umulhi(a, b);
#endif
}
__device__ __forceinline__ uint32_t mullo32(uint32_t a, uint32_t b)
{
#if NTT_FAKE_MUL
    uint32_t r;
    asm volatile("v_or_b32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return a * b;
#endif
}
// low word of a*b + c
__device__ __forceinline__ uint32_t madlo32(uint32_t a, uint32_t b, uint32_t c)
{
#if NTT_FAKE_MUL
    uint32_t r;
    asm volatile("v_add3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return (uint32_t)((uint64_t)a * b + c);
#endif
}

template <uint32_t Q>
__device__ __forceinline__ uint32_t shoup_mul(uint32_t a, uint32_t w, uint32_t wp)
{
    // a < 2^32, w < q, wp = floor(w 2^32 / q)  ->  result == a*w mod q, in [0, 2q)
    const uint32_t qe = mulhi32(a, wp);
    return madlo32(qe, 0u - Q, mullo32(a, w));
}

// Forward twiddles are stored NEGATED on the device (wn = 2^32 - w, Shoup
// companion wp of w): the multiply-add then yields -t directly, so both outputs
// cost one instruction each (v_sub, v_add3):  x' = a + t,  y' = a - t + 2q.
template <uint32_t Q, bool REDUCE = true>
__device__ __forceinline__ void ct_bfly(uint32_t &x, uint32_t &y, uint32_t wn, uint32_t wp)
{
    const uint32_t a = REDUCE ? umin(x, x - 2 * Q) : x;        // [0,4q) -> [0,2q)
    const uint32_t qe = mulhi32(y, wp);
    const uint32_t tn = madlo32(qe, Q, mullo32(y, wn));   // -t, t in [0,2q)
    x = a - tn;
    y = a + tn + 2 * Q;
}

// Signed Shoup product: d is read as a signed 32-bit value with |d| < 2^31,
// the twiddle is stored centred, ws in (-q/2, q/2], with wps = floor(ws 2^32 / q)
// (a signed 32-bit value).  |d ws / q - d wps / 2^32| < 1/2, so with the
// rounded quotient minus one, e = floor((d wps - 2^31) / 2^32),
//   d ws - e q  lies in (0, 2q)  and is congruent to d * ws.
// Three mul-class instructions (v_mad_i64_i32, v_mul_lo_u32, v_mad_u64_u32),
// like shoup_mul, but d = x - y needs no +2q bias.
template <uint32_t Q>
__device__ __forceinline__ uint32_t sshoup_mul(uint32_t d, uint32_t ws, uint32_t wps)
{
    const uint32_t e = (uint32_t)(((int64_t)(int32_t)d * (int32_t)wps - 0x80000000ll) >> 32);
    return madlo32(e, 0u - Q, mullo32(d, ws));
}

// GS butterfly, inputs in [0,2q): x' = (x+y) mod 2q, y' = (x-y) w in [0,2q).
// 7 VALU: v_add, v_sub, v_min, v_sub, then the three of sshoup_mul.
template <uint32_t Q>
__device__ __forceinline__ void gs_bfly(uint32_t &x, uint32_t &y, uint32_t ws, uint32_t wps)
{
    uint32_t s = x + y;                          // [0,4q)
    s = umin(s, s - 2 * Q);
    const uint32_t d = x - y;                    // (-2q, 2q) as a signed value
    x = s;
    y = sshoup_mul<Q>(d, ws, wps);
}

// Montgomery product, a,b in [0,2q): returns a*b*2^-32 mod q in [0,2q)
template <class P>
__device__ __forceinline__ uint32_t mont_mul(uint32_t a, uint32_t b)
{
    const uint32_t lo = a * b;
    const uint32_t hi = __umulhi(a, b);
    const uint32_t m = lo * P::QNEG;
    return hi + __umulhi(m, P::Q) + (lo != 0u ? 1u : 0u);
}

// XOR swizzle of the wave-private transpose buffer (hi = pos >> 5):
//   phys(pos) = pos ^ (pos8 << 2) ^ (pos9 << 3) ^ ((pos7 ^ pos10) << 4) ^ (pos7 << 5)
// Bijective; conflict-free for ds_write_b32 / ds_read_b32 in the pass-1
// layouts and ds_read_b128 / ds_write_b128 in the bit-reversed pass-2
// layout (tests/test_lds_layout.py, gfx950 lane-group bank model).
__host__ __device__ constexpr uint32_t xm_of(uint32_t hi)   // XOR on pos bits 2..4
{
    return (((hi >> 3) & 1) << 2) | (((hi >> 4) & 1) << 3) | ((((hi >> 2) ^ (hi >> 5)) & 1) << 4);
}

// ------------------------------------------------------------------------
// per-lane geometry
// ------------------------------------------------------------------------
template <class P>
struct Lane {
    static constexpr bool BIG = (P::LOGN == 11);  // one poly per wave
    static constexpr uint32_t S = BIG ? 64 : 32;  // pass-1 stride
    uint32_t lane, h, Lp;
    uint32_t wlo, woff;   // pass-1 LDS write/read (b32) address parts
    uint32_t rbase, rxm;  // pass-2 LDS read/write (b128) address parts
    uint32_t brl;         // lane index within its poly: pass-1 column, and bitrev(Lp)

    __device__ __forceinline__ Lane()
    {
        lane = threadIdx.x & 63;
        h = lane >> 5;
        // pass-2 row of this lane: Lp = bitrev(lane).  Then the bit-reversed
        // side of each transform (forward store, inverse load) addresses
        // brv5(j) * S + brv(Lp) = brv5(j) * S + lane: lane-contiguous 128/256-B runs.
        Lp = BIG ? (__builtin_bitreverse32(lane) >> 26) : (__builtin_bitreverse32(lane & 31) >> 27);
        wlo = lane & 31;
        woff = BIG ? 64 * h : 1024 * h;
        rxm = xm_of(Lp);
        rbase = 32 * (Lp ^ ((Lp >> 2) & 1)) + (BIG ? 0u : 1024 * h);
        brl = BIG ? lane : (lane & 31);
    }
};

// pos>>5 of register j in the pass-1 layout (n=2048: after the bit-5 swap)
template <class P>
__host__ __device__ constexpr uint32_t hi_of(int j)
{
    return P::LOGN == 11 ? (uint32_t)((j & 1) + 4 * (j >> 1)) : (uint32_t)j;
}

template <class P>
__device__ __forceinline__ uint32_t p1_addr(const Lane<P> &L, int j)
{
    const uint32_t hj = hi_of<P>(j);   // the lane part of hi (n = 2048: 2h) enters neither XOR term
    return (L.wlo ^ xm_of(hj)) + 32 * (hj ^ ((hj >> 2) & 1)) + L.woff;
}

__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// In-kernel phase stamp (diagnostic variants V >= 4 only): s_memtime with its
// lgkmcnt wait in one statement, fenced against scheduling.
#define NTT_STAMP(var)                                                                  \
    do {                                                                                \
        __builtin_amdgcn_sched_barrier(0);                                              \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");     \
        __builtin_amdgcn_sched_barrier(0);                                              \
    } while (0)

// A wave-uniform zero the compiler cannot see through.  Adding it to the
// index of a uniform twiddle load keeps that load an s_load inside the
// persistent loop instead of letting LICM hoist all ~126 twiddle words into
// registers (which cost 2-3 waves/SIMD of occupancy).
__device__ __forceinline__ uint32_t opaque_zero()
{
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

// pass-1 layout (registers, post-swap for n=2048) -> pass-2 layout
template <class P>
__device__ __forceinline__ void lds_p1_to_p2(uint32_t (&r)[32], uint32_t *buf, const Lane<P> &L)
{
#pragma unroll
    for (int j = 0; j < 32; ++j) buf[p1_addr<P>(L, j)] = r[j];
    compiler_fence();
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const uint4 v = *reinterpret_cast<const uint4 *>(buf + L.rbase + ((4u * c) ^ L.rxm));
        r[4 * c + 0] = v.x;
        r[4 * c + 1] = v.y;
        r[4 * c + 2] = v.z;
        r[4 * c + 3] = v.w;
    }
    compiler_fence();
}

// pass-2 layout -> pass-1 layout (n=2048: the post-swap arrangement)
template <class P>
__device__ __forceinline__ void lds_p2_to_p1(uint32_t (&r)[32], uint32_t *buf, const Lane<P> &L)
{
#pragma unroll
    for (int c = 0; c < 8; ++c)
        *reinterpret_cast<uint4 *>(buf + L.rbase + ((4u * c) ^ L.rxm)) =
            make_uint4(r[4 * c + 0], r[4 * c + 1], r[4 * c + 2], r[4 * c + 3]);
    compiler_fence();
#pragma unroll
    for (int j = 0; j < 32; ++j) r[j] = buf[p1_addr<P>(L, j)];
    compiler_fence();
}

constexpr int XPOSE_WORDS = 2048;   // per-wave transpose buffer (8 KiB)
template <class P>
__device__ __forceinline__ void xpose_p1_to_p2(uint32_t (&r)[32], uint32_t *buf, const Lane<P> &L)
{
    lds_p1_to_p2<P>(r, buf, L);
}
template <class P>
__device__ __forceinline__ void xpose_p2_to_p1(uint32_t (&r)[32], uint32_t *buf, const Lane<P> &L)
{
    lds_p2_to_p1<P>(r, buf, L);
}

// ------------------------------------------------------------------------
// transform passes
// ------------------------------------------------------------------------
// Table base + an opaque wave-uniform zero: every uniform twiddle read below
// becomes an s_load_dwordx{2,8,16} with an immediate offset, re-issued per
// persistent-loop iteration instead of ~126 hoisted words pinning registers.
template <int PS, bool INV>
__device__ __forceinline__ const uint2 *tw_base()
{
    const uint32_t z = opaque_zero();
    if constexpr (PS == 0) return (INV ? c_inv0 : c_fwd0) + z;
    else if constexpr (PS == 1) return (INV ? c_inv1 : c_fwd1) + z;
    else return (INV ? c_inv2 : c_fwd2) + z;
}

// forward pass 1: CT stages on pos bits LOGN-1 .. LOGN-5 (j bits 4..0),
// twiddle index k = 2^s + (j >> (5-s)) -- wave-uniform.
template <int PS, class P>
__device__ __forceinline__ void fwd_pass1(uint32_t (&r)[32], uint32_t h, const uint2 *sw)
{
    const uint2 *tw = tw_base<PS, false>();
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int hh = 16 >> s;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const uint2 w = NTT_FAKE_TW ? make_uint2(0u - 12345u * (j + 1), 777u * (j + 3)) : tw[(1u << s) + (uint32_t)(j >> (5 - s))];
                if (s == 0) ct_bfly<P::Q, false>(r[j], r[j + hh], w.x, w.y);   // inputs < 2q
                else ct_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
            }
        }
    }
    if constexpr (P::LOGN == 11) {
        // pos bit 5 pairs lanes l, l^32: exchange halves, butterfly, keep the
        // swapped arrangement (p1_addr accounts for it)
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const auto pr = __builtin_amdgcn_permlane32_swap(r[2 * m], r[2 * m + 1], false, false);
            r[2 * m] = pr[0];
            r[2 * m + 1] = pr[1];
            const uint2 w = NTT_FAKE_TW ? make_uint2(0u - 5u * (m + 1), 99u * (m + 1)) : sw[2 * m + h];    // k = 32 + 2m + h
            ct_bfly<P::Q>(r[2 * m], r[2 * m + 1], w.x, w.y);
        }
    }
}

// Per-lane pass-2 twiddles live in a per-workgroup LDS table, lane-major
// (entry e, lane t) so a ds_read_b64 by 64 lanes is conflict-free:
//   e = 2^(4-b) - 1 + m for stage bit b,  k = 2^(LOGN-1-b) + (Lp << (4-b)) + m
constexpr int TW2_ENTRIES = 31;
constexpr int TW2_WORDS = TW2_ENTRIES * 64 * 2 + 64;   // 15.5 KiB + the 32-entry bit-5 table

__host__ __device__ constexpr int tw2_b(int e) { return e < 1 ? 4 : e < 3 ? 3 : e < 7 ? 2 : e < 15 ? 1 : 0; }

// Host-built images of the per-workgroup LDS twiddle table (lane-major
// pass-2 entries + the 32-entry bit-5 table), one per (param set, direction):
// the workgroup prologue is then one coalesced 16 KiB copy with one wait.
constexpr int TW2_VEC4 = TW2_WORDS / 4;   // 1008 uint4
__device__ uint4 g_tw2img[3][2][TW2_VEC4];

template <int PS, bool INV, int NT>
__device__ __forceinline__ void fill_tw2(uint2 *tab)
{
    const uint4 *src = g_tw2img[PS][INV ? 1 : 0];
    uint4 *dst = reinterpret_cast<uint4 *>(tab);
    constexpr int ITER = (TW2_VEC4 + NT - 1) / NT;
    uint4 v[ITER];
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
        const int i = threadIdx.x + k * NT;
        if (i < TW2_VEC4) v[k] = src[i];
    }
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
        const int i = threadIdx.x + k * NT;
        if (i < TW2_VEC4) dst[i] = v[k];
    }
}

template <class P>
__device__ __forceinline__ void fwd_pass2(uint32_t (&r)[32], const uint2 *tab, uint32_t lane)
{
#pragma unroll
    for (int b = 4; b >= 0; --b) {
        const int hh = 1 << b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const int e = (1 << (4 - b)) - 1 + (j >> (b + 1));
                const uint2 w = NTT_FAKE_TW ? make_uint2(0u - 31u * (e + 1), 1234u * (e + 1)) : tab[e * 64 + lane];
                ct_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
            }
        }
    }
}

template <class P>
__device__ __forceinline__ void inv_pass2(uint32_t (&r)[32], const uint2 *tab, uint32_t lane)
{
#pragma unroll
    for (int b = 0; b <= 4; ++b) {
        const int hh = 1 << b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const int e = (1 << (4 - b)) - 1 + (j >> (b + 1));
                const uint2 w = tab[e * 64 + lane];
                gs_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
            }
        }
    }
}

// inverse pass 1: (n=2048) GS on pos bit 5 + swap back, then GS stages on pos
// bits LOGN-5 .. LOGN-1 (j bits 0..4); the last one carries the n^-1 scaling
// (times S0 / S1 constants), output canonical.
struct NoEmit {
    __device__ __forceinline__ void operator()(int, uint32_t) const {}
};

// `emit(j, v)` is called with each final canonical output as soon as it is
// computed (the inverse kernel stores from there, so its 32 stores interleave
// with the last stage instead of queueing behind it as one tail).
template <int PS, class P, uint32_t S0, uint32_t S1, class Emit = NoEmit>
__device__ __forceinline__ void inv_pass1(uint32_t (&r)[32], uint32_t h, const uint2 *sw, const Emit &emit = Emit())
{
    const uint2 *tw = tw_base<PS, true>();
    if constexpr (P::LOGN == 11) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const uint2 w = sw[2 * m + h];
            gs_bfly<P::Q>(r[2 * m], r[2 * m + 1], w.x, w.y);
            const auto pr = __builtin_amdgcn_permlane32_swap(r[2 * m], r[2 * m + 1], false, false);
            r[2 * m] = pr[0];
            r[2 * m + 1] = pr[1];
        }
    }
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) {
        const int hh = 1 << jb;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const uint2 w = tw[(16u >> jb) + (uint32_t)(j >> (jb + 1))];
                gs_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
            }
        }
    }
    constexpr uint32_t S0P = cshoup(S0, P::Q);
    constexpr TwPair S1S = csigned_tw(S1, P::Q);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = r[j], y = r[j + 16];
        const uint32_t s = x + y;              // [0,4q)
        const uint32_t d = x - y;              // (-2q, 2q), signed
        uint32_t a = shoup_mul<P::Q>(s, S0, S0P);
        uint32_t b = sshoup_mul<P::Q>(d, S1S.x, S1S.y);
        r[j] = umin(a, a - P::Q);
        r[j + 16] = umin(b, b - P::Q);
        emit(j, r[j]);
        emit(j + 16, r[j + 16]);
    }
}

__device__ __forceinline__ constexpr uint32_t brv5(int j)
{
    return (uint32_t)(((j & 1) << 4) | ((j & 2) << 2) | (j & 4) | ((j & 8) >> 2) | ((j & 16) >> 4));
}

// ------------------------------------------------------------------------
// kernels
// ------------------------------------------------------------------------
// Workgroup = WGX waves, each with a private 8 KiB transpose buffer; the
// lane-twiddle tables are shared by the workgroup.
#ifndef NTT_WG
#define NTT_WG 512          // fwd / inv: 8 waves, 64 + 15.5 KiB LDS -> 2 WG/CU
#endif
// poly_mul workgroup per parameter set: n=2048 runs 16 waves (128 + 31.5 KiB
// LDS, 1 WG/CU, <=128 VGPRs -> 4 waves/SIMD, 6 spilled VGPRs: -1..-2 % time);
// n=1024 keeps 8 waves at <=256 VGPRs (2 waves/SIMD; at 128 VGPRs it spills 60
// and loses 37 %), profiles/r01/ab_poly_mul_wg.json
#ifndef MUL_WG
#define MUL_WG 512
#endif
#ifndef MUL_WG_BIG
#define MUL_WG_BIG 1024
#endif
#ifndef NTT_WAVES_PER_SIMD
#define NTT_WAVES_PER_SIMD 4
#endif
#ifndef MUL_WAVES_PER_SIMD
#define MUL_WAVES_PER_SIMD 2
#endif
#ifndef MUL_WAVES_PER_SIMD_BIG
#define MUL_WAVES_PER_SIMD_BIG 4
#endif
template <int PS> constexpr int mul_wg() { return PSel<PS>::T::LOGN == 11 ? MUL_WG_BIG : MUL_WG; }
template <int PS> constexpr int mul_occ() { return PSel<PS>::T::LOGN == 11 ? MUL_WAVES_PER_SIMD_BIG : MUL_WAVES_PER_SIMD; }
constexpr int WG = 256;             // elementwise kernels

// Work distribution: workgroup b owns the contiguous unit range
// [b*WAVES*PPW, (b+1)*WAVES*PPW); at step i its waves take consecutive units
// b*WAVES*PPW + i*WAVES + wave.  Workgroups are dispatched in order, so the
// units in flight chip-wide form a sliding contiguous window of HBM: measured
// 5.9 TB/s for this access shape vs 5.4 TB/s for a persistent grid-stride
// loop (tools/copy_bw.hip, profiles/r01/copybw.log).
// units per wave: chosen per launch by launch_for (up to NTT_PPW_MAX) so that
// large batches amortise the workgroup prologue and small ones fill the chip
#ifndef NTT_PPW_MAX
#define NTT_PPW_MAX 16
#endif
// The first unit's global loads are issued before the workgroup prologue
// (`prologue` = the LDS twiddle-table fill + barrier), so the fill latency
// hides under the first unit's HBM latency.
template <int WAVES, class Prologue, class Load, class Process>
__device__ __forceinline__ void chunk_loop(uint32_t nunits, uint32_t ppw, Prologue &prologue, Load &load,
                                           Process &process)
{
    uint32_t r[32];
    uint32_t u = blockIdx.x * (WAVES * ppw) + (threadIdx.x >> 6);
    if (u < nunits) load(r, u);
    prologue();   // every wave reaches the barrier inside
    if (u >= nunits) return;
    process(r, u);
#pragma unroll 1
    for (uint32_t i = 1; i < ppw; ++i) {
        u += WAVES;
        if (u >= nunits) break;
        load(r, u);
        process(r, u);
    }
}

// ------------------------------------------------------------------------
// LDS-DMA prefetch (NTT_DMA=1): the next unit's 8 KiB streams HBM -> LDS by
// global_load_lds_dwordx4 into the wave's transpose buffer -- free from the
// transpose read until the next unit's first ds_read -- while the current
// unit's pass 2 and stores run.  No extra VGPRs (a register prefetch would
// need 32 and cost a wave per SIMD), so HBM latency hides at the same
// occupancy.  The DMA is inline asm (hipcc would otherwise wait vmcnt(0) --
// i.e. for the previous unit's stores too -- before the buffer's ds_reads):
// its completion is counted by hand.  vmcnt counts loads, stores and LDS-DMA
// together in issue order (MI355X_MICROARCH.md), and exactly 32 stores follow
// each DMA, so `s_waitcnt vmcnt(32)` retires precisely the DMA.
// Bit-exact but measured neutral on p-III (fwd +-0 %, inv +1.7 %, interleaved
// A/B, profiles/r01/ab_ntstore_dma.json): the memory side of this access shape
// is not latency-bound at 4 waves/SIMD (tools/copy_bw.hip "occ" modes), so the
// option stays off.
// ------------------------------------------------------------------------
#ifndef NTT_DMA
#define NTT_DMA 0
#endif

// one 1 KiB piece: lane l's 16 B from gsrc -> LDS byte address lds + 16 l
__device__ __forceinline__ void dma16(const uint32_t *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(gsrc), "s"(lds)
                 : "memory");
}

// LDS byte address of a wave-uniform __shared__ pointer
__device__ __forceinline__ uint32_t lds_addr(const uint32_t *p)
{
    return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)p);
}

// Unit u (2048 consecutive words: one n=2048 poly or two n=1024 polys) ->
// the wave's buffer in natural order.  `pieces` = 8, or 4 when the unit's
// second n=1024 poly lies past the batch.
__device__ __forceinline__ void dma_unit(const uint32_t *unit, uint32_t lds, uint32_t lane, int pieces)
{
    const uint32_t *src = unit + 4 * lane;
#pragma unroll
    for (int c = 0; c < 8; ++c)
        if (c < pieces) dma16(src + 256 * c, lds + 1024 * c);
}

// Output stores of the transforms; NTT_NT_STORE=1 marks them nontemporal
// (streamed once, never re-read by the kernel).
#ifndef NTT_NT_STORE
#define NTT_NT_STORE 1
#endif
// NTT_INV_EMIT=1: the inverse stores each output from inside its last stage
#ifndef NTT_INV_EMIT
#define NTT_INV_EMIT 1
#endif
__device__ __forceinline__ void st_out(uint32_t *p, uint32_t v)
{
    if constexpr (NTT_NT_STORE) __builtin_nontemporal_store(v, p);
    else *p = v;
}
// Input loads of the transforms and products; NTT_NT_LOAD=1 marks them
// nontemporal (read once): with nt stores, in place -4.5 % fwd / -2.1 % inv,
// out of place -3.6 % / -1.0 % (profiles/r01/ab_nt_load.json).
#ifndef NTT_NT_LOAD
#define NTT_NT_LOAD 1
#endif
__device__ __forceinline__ uint32_t ld_in(const uint32_t *p)
{
    if constexpr (NTT_NT_LOAD) return __builtin_nontemporal_load(p);
    else return *p;
}

__device__ __forceinline__ void wait_vm(void) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_vm32(void) { asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); }
__device__ __forceinline__ void wait_lgkm(void) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Work loop with the DMA prefetch: `read(r)` takes the unit from the buffer
// into registers, `front(r, u)` runs up to and including the transpose (after
// which the buffer is free), `back(r, u)` runs the rest and issues exactly 32
// stores per lane.
template <int WAVES, class Prologue, class Read, class Front, class Back>
__device__ __forceinline__ void chunk_loop_dma(const uint32_t *in, uint32_t npoly, uint32_t nunits, uint32_t ppw,
                                               uint32_t lds, uint32_t lane, bool half_units, Prologue &prologue,
                                               Read &read, Front &front, Back &back)
{
    auto pieces = [&](uint32_t u) { return (half_units && 2 * u + 1 >= npoly) ? 4 : 8; };
    uint32_t u = blockIdx.x * (WAVES * ppw) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (u < nunits) dma_unit(in + (size_t)u * 2048, lds, lane, pieces(u));
    prologue();   // every wave reaches the barrier inside
    if (u >= nunits) return;
    wait_vm();
    uint32_t r[32];
#pragma unroll 1
    for (uint32_t i = 0;; ++i) {
        read(r);
        front(r, u);
        wait_lgkm();   // the transpose's reads are done: the buffer is free
        const uint32_t un = u + WAVES;
        const bool more = i + 1 < ppw && un < nunits;
        if (more) dma_unit(in + (size_t)un * 2048, lds, lane, pieces(un));
        back(r, u);
        if (!more) break;
        u = un;
        wait_vm32();   // all but the 32 stores issued after the DMA
    }
}

// NTT_PRIO=1: one s_setprio 1 for the second-dispatched half of each
// workgroup (waves 4-7), the static form of MI355X_MICROARCH.md "Two waves
// per SIMD" item 4.  Measured: fwd -0.6 %, inv +2.2 % (profiles/r01/ab_prio.json), off.
#ifndef NTT_PRIO
#define NTT_PRIO 0
#endif
__device__ __forceinline__ void younger_half_priority(int wg)
{
    if constexpr (NTT_PRIO)
        if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= (unsigned)(wg / 2)) __builtin_amdgcn_s_setprio(1);
}

// V (diagnostic variants, reached only through ntt_debug_variant): 0 = full,
// 1 = global load + store only, 2 = compute only (no global memory),
// 3 = load + LDS transpose + store (no arithmetic)
//
// Persistent loop, software-pipelined over two register sets: the 32 loads of
// the wave's next polynomial are in flight while the current one is
// transformed, so HBM latency hides under the VALU work of the same wave.
template <int PS, int V = 0>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_ntt_fwd(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    constexpr uint32_t PPW = LT::BIG ? 1 : 2;
    constexpr int WAVES = NTT_WG / 64;
    __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES * XPOSE_WORDS + TW2_WORDS];
    uint2 *tw2 = reinterpret_cast<uint2 *>(lds + WAVES * XPOSE_WORDS);
    younger_half_priority(NTT_WG);
    auto prologue = [&]() {
        fill_tw2<PS, false, NTT_WG>(tw2);
        __syncthreads();
    };
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + PPW - 1) / PPW;

    auto load = [&](uint32_t (&r)[32], uint32_t u) {
        // per-lane base pointer + compile-time offsets (offsets fold into the
        // instructions' immediate field instead of 32 address registers)
        const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
        const bool valid = LT::BIG || poly < npoly;
        const uint32_t *src = in + (size_t)poly * P::N + L.brl;   // pass-1 layout: natural lane index
#pragma unroll
        for (int j = 0; j < 32; ++j) r[j] = (V == 2 || V == 5) ? L.lane * (j + u) : (valid ? ld_in(src + LT::S * j) : 0u);
    };
    // V 4/5: V 0/2 with per-phase s_memtime stamps accumulated per wave
    // V 6: no arithmetic, raw words -- the bit-reversal copy (poly_bitrev_copy)
    constexpr bool STAMPS = V == 4 || V == 5;
    constexpr bool ALU = V == 0 || V == 2 || V == 4 || V == 5;
    unsigned long long acc[6] = {0, 0, 0, 0, 0, 0}, ts[7];
    // canonical output, bit-reversed registers -> natural order: brv5(j)*S + lane
    auto store = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
        if (LT::BIG || poly < npoly) {
            uint32_t *dst = out + (size_t)poly * P::N + L.brl;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                uint32_t x = r[j];
                if constexpr (V != 6) {
                    x = umin(x, x - P::Q2);
                    x = umin(x, x - P::Q);
                }
                if constexpr (V == 2 || V == 5) asm volatile("" ::"v"(x));
                else st_out(dst + brv5(j) * LT::S, x);
            }
        }
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        if constexpr (STAMPS) NTT_STAMP(ts[0]);
        if constexpr (ALU) fwd_pass1<PS, P>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
        if constexpr (V == 6 && LT::BIG) {   // the pass-1 lane-half exchange alone (p1_addr expects it)
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const auto pr = __builtin_amdgcn_permlane32_swap(r[2 * m], r[2 * m + 1], false, false);
                r[2 * m] = pr[0];
                r[2 * m + 1] = pr[1];
            }
        }
        if constexpr (STAMPS) NTT_STAMP(ts[1]);
        if constexpr (V != 1) xpose_p1_to_p2<P>(r, buf, L);
        if constexpr (STAMPS) NTT_STAMP(ts[2]);
        if constexpr (ALU) fwd_pass2<P>(r, tw2 + opaque_zero(), L.lane);
        if constexpr (STAMPS) NTT_STAMP(ts[3]);
        store(r, u);
        if constexpr (STAMPS) {
            NTT_STAMP(ts[4]);
            for (int i = 0; i < 4; i++) acc[i] += ts[i + 1] - ts[i];
        }
    };
    if constexpr (NTT_DMA && V == 0) {
        const uint32_t *nb = buf + (LT::BIG ? 0u : 1024u * L.h) + L.brl;   // natural image, pass-1 layout
        auto read = [&](uint32_t (&r)[32]) {
#pragma unroll
            for (int j = 0; j < 32; ++j) r[j] = nb[LT::S * j];
        };
        auto front = [&](uint32_t (&r)[32], uint32_t) {
            fwd_pass1<PS, P>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
            xpose_p1_to_p2<P>(r, buf, L);
        };
        auto back = [&](uint32_t (&r)[32], uint32_t u) {
            fwd_pass2<P>(r, tw2 + opaque_zero(), L.lane);
            store(r, u);
        };
        chunk_loop_dma<WAVES>(in, npoly, nunits, ppw, lds_addr(buf), L.lane, !LT::BIG, prologue, read, front, back);
        return;
    }
    unsigned long long t_begin = 0, t_end = 0;
    if constexpr (STAMPS) NTT_STAMP(t_begin);
    chunk_loop<WAVES>(nunits, ppw, prologue, load, process);
    if constexpr (STAMPS) {
        NTT_STAMP(t_end);
        if (L.lane == 0) {   // diagnostic build: stamps go to the (garbage) output buffer
            unsigned long long *o = reinterpret_cast<unsigned long long *>(out) + (blockIdx.x * WAVES + (threadIdx.x >> 6)) * 8;
            for (int k = 0; k < 4; k++) o[k] = acc[k];
            o[4] = t_end - t_begin;
        }
    }
}

template <int PS, int V = 0>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_ntt_inv(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    constexpr uint32_t PPW = LT::BIG ? 1 : 2;
    constexpr int WAVES = NTT_WG / 64;
    __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES * XPOSE_WORDS + TW2_WORDS];
    uint2 *tw2 = reinterpret_cast<uint2 *>(lds + WAVES * XPOSE_WORDS);
    younger_half_priority(NTT_WG);
    auto prologue = [&]() {
        fill_tw2<PS, true, NTT_WG>(tw2);
        __syncthreads();
    };
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + PPW - 1) / PPW;

    auto load = [&](uint32_t (&r)[32], uint32_t u) {
        // natural-order input; pass-2 position 32*Lp + j holds X[brv(pos)]
        const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
        const bool valid = LT::BIG || poly < npoly;
        const uint32_t *src = in + (size_t)poly * P::N + L.brl;
#pragma unroll
        for (int j = 0; j < 32; ++j) r[j] = V == 2 ? L.lane * (j + u) : (valid ? ld_in(src + brv5(j) * LT::S) : 0u);
    };
    auto store = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
        if (LT::BIG || poly < npoly) {
            uint32_t *dst = out + (size_t)poly * P::N + L.brl;   // pass-1 layout: natural lane index
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                if constexpr (V == 2) asm volatile("" ::"v"(r[j]));
                else st_out(dst + LT::S * j, r[j]);
            }
        }
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        // inputs < 2q by contract: they feed the GS butterflies directly
        if constexpr (V == 0 || V == 2) inv_pass2<P>(r, tw2 + opaque_zero(), L.lane);
        if constexpr (V != 1) xpose_p2_to_p1<P>(r, buf, L);
        if constexpr (V == 0 && NTT_INV_EMIT) {
            const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
            uint32_t *dst = out + (size_t)poly * P::N + L.brl;
            const bool valid = LT::BIG || poly < npoly;
            auto emit = [&](int j, uint32_t v) {
                if (valid) st_out(dst + LT::S * j, v);
            };
            inv_pass1<PS, P, P::NINV, P::C1>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero(), emit);
            return;
        }
        if constexpr (V == 0 || V == 2) inv_pass1<PS, P, P::NINV, P::C1>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
        store(r, u);
    };
    if constexpr (NTT_DMA && V == 0) {
        const uint32_t *nb = buf + (LT::BIG ? 0u : 1024u * L.h) + L.brl;   // natural image, pass-2 (bit-reversed) layout
        auto read = [&](uint32_t (&r)[32]) {
#pragma unroll
            for (int j = 0; j < 32; ++j) r[j] = nb[LT::S * brv5(j)];
        };
        auto front = [&](uint32_t (&r)[32], uint32_t) {
            inv_pass2<P>(r, tw2 + opaque_zero(), L.lane);
            xpose_p2_to_p1<P>(r, buf, L);
        };
        auto back = [&](uint32_t (&r)[32], uint32_t u) {
            inv_pass1<PS, P, P::NINV, P::C1>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
            store(r, u);
        };
        chunk_loop_dma<WAVES>(in, npoly, nunits, ppw, lds_addr(buf), L.lane, !LT::BIG, prologue, read, front, back);
        return;
    }
    chunk_loop<WAVES>(nunits, ppw, prologue, load, process);
}

// fused c = a*b mod (x^n+1): FWD(a), FWD(b), Montgomery pointwise (the 2^-32
// is folded into the inverse's final n^-1 scaling), INV -- one HBM read of a
// and b, one write of c.  BHAT: b is given already transformed (natural-order
// output of poly_ntt), so only a is transformed -- two transforms of work per
// product instead of three (poly_mul_ntt).
template <int PS, bool BHAT = false>
__global__ __launch_bounds__(mul_wg<PS>(), mul_occ<PS>()) void k_poly_mul(const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    constexpr uint32_t PPW = LT::BIG ? 1 : 2;
    constexpr int WG_ = mul_wg<PS>();
    constexpr int WAVES = WG_ / 64;
    __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES * XPOSE_WORDS + 2 * TW2_WORDS];
    uint2 *ftw2 = reinterpret_cast<uint2 *>(lds + WAVES * XPOSE_WORDS);
    uint2 *itw2 = ftw2 + TW2_WORDS / 2;
    fill_tw2<PS, false, WG_>(ftw2);
    fill_tw2<PS, true, WG_>(itw2);
    __syncthreads();
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;

    const uint32_t nunits = (npoly + PPW - 1) / PPW;
    uint32_t u = blockIdx.x * (WAVES * ppw) + (threadIdx.x >> 6);
#pragma unroll 1
    for (uint32_t it = 0; it < ppw; ++it, u += WAVES) {   // dispatch-ordered chunk (see chunk_loop)
        if (u >= nunits) break;
        const uint32_t poly = u * PPW + (LT::BIG ? 0u : L.h);
        const bool valid = poly < npoly;
        const size_t off = (size_t)poly * P::N + L.brl;   // pass-1 layout: natural lane index
        const uint32_t *pa = a + off, *pb = b + off;
        // a first, then b: the transpose's memory fences keep b's loads below
        // a's transform, so only ~64 coefficients are live at the peak
        uint32_t ra[32], rb[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) ra[j] = valid ? ld_in(pa + LT::S * j) : 0u;
        fwd_pass1<PS, P>(ra, L.h, ftw2 + TW2_ENTRIES * 64 + opaque_zero());
        xpose_p1_to_p2<P>(ra, buf, L);
        fwd_pass2<P>(ra, ftw2 + opaque_zero(), L.lane);
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            ra[j] = umin(ra[j], ra[j] - P::Q2);
            // b-hat is in natural order: register j of the pass-2 layout holds
            // index brv5(j)*S + lane (the forward's store mapping)
            rb[j] = valid ? ld_in(pb + LT::S * (BHAT ? brv5(j) : (uint32_t)j)) : 0u;
        }
        if constexpr (!BHAT) {
            fwd_pass1<PS, P>(rb, L.h, ftw2 + TW2_ENTRIES * 64 + opaque_zero());
            xpose_p1_to_p2<P>(rb, buf, L);
            fwd_pass2<P>(rb, ftw2 + opaque_zero(), L.lane);
        }
#pragma unroll
        for (int j = 0; j < 32; ++j) ra[j] = mont_mul<P>(ra[j], umin(rb[j], rb[j] - P::Q2));   // b-hat < 2q
        inv_pass2<P>(ra, itw2 + opaque_zero(), L.lane);
        xpose_p2_to_p1<P>(ra, buf, L);
        uint32_t *pc = c + off;
        auto emit = [&](int j, uint32_t v) {   // stores interleaved with the last stage (see k_ntt_inv)
            if (valid) st_out(pc + LT::S * j, v);
        };
        inv_pass1<PS, P, P::NINV_R, P::C1_R>(ra, L.h, itw2 + TW2_ENTRIES * 64 + opaque_zero(), emit);
    }
}

// c = a.*b mod q over `count` coefficients (count % 4 == 0): Montgomery then
// Shoup by 2^32 mod q to undo the 2^-32.
template <int PS>
__global__ __launch_bounds__(WG) void k_pointwise(const uint4 *a, const uint4 *b, uint4 *c, size_t count4)
{
    using P = typename PSel<PS>::T;
    constexpr uint32_t RP = cshoup(P::R, P::Q);
    for (size_t i = (size_t)blockIdx.x * WG + threadIdx.x; i < count4; i += (size_t)gridDim.x * WG) {
        const uint4 x = a[i], y = b[i];
        uint32_t v[4] = {x.x, x.y, x.z, x.w}, w[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t m = mont_mul<P>(umin(v[k], v[k] - P::Q2), umin(w[k], w[k] - P::Q2));
            m = shoup_mul<P::Q>(m, P::R, RP);
            v[k] = umin(m, m - P::Q);
        }
        c[i] = make_uint4(v[0], v[1], v[2], v[3]);
    }
}

// Diagnostic copy kernels (ntt_debug_variant op 2): one poly per wave,
// persistent grid like the transforms; dword (the transforms' access shape)
// vs dwordx4 accesses, to price access width against the HBM roofline.
template <int W>
__global__ __launch_bounds__(512) void k_copy_diag(const uint32_t *in, uint32_t *out, uint32_t npoly)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * 8;
    for (uint32_t u = blockIdx.x * 8 + (threadIdx.x >> 6); u < npoly; u += nw) {
        if constexpr (W == 4) {
            const uint4 *s4 = reinterpret_cast<const uint4 *>(in + (size_t)u * 2048) + lane;
            uint4 *d4 = reinterpret_cast<uint4 *>(out + (size_t)u * 2048) + lane;
            uint4 v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = s4[64 * j];
#pragma unroll
            for (int j = 0; j < 8; ++j) d4[64 * j] = v[j];
        } else {
            const uint32_t *s1 = in + (size_t)u * 2048 + lane;
            uint32_t *d1 = out + (size_t)u * 2048 + lane;
            uint32_t v[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s1[64 * j];
#pragma unroll
            for (int j = 0; j < 32; ++j) d1[64 * j] = v[j];
        }
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(WG) void k_fill_uniform(uint32_t *x, size_t count, uint32_t q, uint64_t seed, uint64_t first)
{
    for (size_t i = (size_t)blockIdx.x * WG + threadIdx.x; i < count; i += (size_t)gridDim.x * WG) {
        const uint64_t r = splitmix64(seed + (first + i + 1) * 0x9E3779B97F4A7C15ULL);
        x[i] = (uint32_t)(((r >> 32) * (uint64_t)q) >> 32);
    }
}

// ------------------------------------------------------------------------
// host side: table upload, launch configuration, C ABI
// ------------------------------------------------------------------------
namespace {

thread_local int t_last_hip = 0;

constexpr int kMaxDev = 64;
std::once_flag g_tab_once[kMaxDev];
int g_tab_status[kMaxDev];
std::once_flag g_cpu_tables_once;
Tables g_cpu_tables[3];

const Tables &cpu_tables(int ps)
{
    std::call_once(g_cpu_tables_once, [] {
        for (int i = 0; i < 3; i++) make_tables(*param_set(i), g_cpu_tables[i]);
    });
    return g_cpu_tables[ps];
}

int upload_tables(int dev)
{
    struct Sym { const void *sym; int ps; bool inv; };
    const Sym syms[6] = {{HIP_SYMBOL(c_fwd0), 0, false}, {HIP_SYMBOL(c_inv0), 0, true},
                         {HIP_SYMBOL(c_fwd1), 1, false}, {HIP_SYMBOL(c_inv1), 1, true},
                         {HIP_SYMBOL(c_fwd2), 2, false}, {HIP_SYMBOL(c_inv2), 2, true}};
    for (const auto &s : syms) {
        const Tables &t = cpu_tables(s.ps);
        std::vector<uint32_t> v = s.inv ? t.inv : t.fwd;
        for (size_t k = 0; k < v.size(); k += 2) {
            if (s.inv) {   // device inverse table holds the centred (ws, ws'): see sshoup_mul
                const TwPair c = csigned_tw(v[k], param_set(s.ps)->q);
                v[k] = c.x;
                v[k + 1] = c.y;
            } else {       // device forward table holds (2^32 - w, w'): see ct_bfly
                v[k] = 0u - v[k];
            }
        }
        hipError_t e = hipMemcpyToSymbol(s.sym, v.data(), v.size() * 4, 0, hipMemcpyHostToDevice);
        if (e != hipSuccess) { t_last_hip = (int)e; return NTT_ERR_HIP; }
    }
    // LDS twiddle-table images (see fill_tw2), in the device conventions
    static std::vector<uint32_t> img[3][2];
    static std::once_flag img_once;
    std::call_once(img_once, [] {
        for (int ps = 0; ps < 3; ps++)
            for (int inv = 0; inv < 2; inv++) {
                const ParamSet &p = *param_set(ps);
                const Tables &t = cpu_tables(ps);
                const std::vector<uint32_t> &tw = inv ? t.inv : t.fwd;
                std::vector<uint32_t> &o = img[ps][inv];
                o.assign(TW2_WORDS, 0);
                auto put = [&](int slot, uint32_t k) {
                    if (inv) {   // inverse stored centred (sshoup_mul)
                        const TwPair c = csigned_tw(tw[2 * k], p.q);
                        o[2 * slot] = c.x;
                        o[2 * slot + 1] = c.y;
                    } else {     // forward stored negated (ct_bfly)
                        o[2 * slot] = 0u - tw[2 * k];
                        o[2 * slot + 1] = tw[2 * k + 1];
                    }
                };
                for (int e = 0; e < TW2_ENTRIES; e++) {
                    const int b = e < 1 ? 4 : e < 3 ? 3 : e < 7 ? 2 : e < 15 ? 1 : 0;
                    const uint32_t m = e - ((1u << (4 - b)) - 1);
                    for (uint32_t lane = 0; lane < 64; lane++) {   // Lp = bitrev(lane), see Lane
                        const uint32_t Lp = p.logn == 11 ? bitrev(lane, 6) : bitrev(lane & 31, 5);
                        put(e * 64 + lane, (1u << (p.logn - 1 - b)) + (Lp << (4 - b)) + m);
                    }
                }
                for (int i = 0; i < 32; i++) put(TW2_ENTRIES * 64 + i, 32u + i);   // bit-5 stage: k = 32 + 2m + h
            }
    });
    for (int ps = 0; ps < 3; ps++)
        for (int inv = 0; inv < 2; inv++) {
            hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_tw2img), img[ps][inv].data(), TW2_WORDS * 4,
                                             (size_t)(ps * 2 + inv) * TW2_WORDS * 4, hipMemcpyHostToDevice);
            if (e != hipSuccess) { t_last_hip = (int)e; return NTT_ERR_HIP; }
        }
    (void)dev;
    return NTT_OK;
}

int ensure_device_tables()
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) { t_last_hip = (int)e; return NTT_ERR_HIP; }
    if (dev < 0 || dev >= kMaxDev) return NTT_ERR_HIP;
    std::call_once(g_tab_once[dev], [dev] { g_tab_status[dev] = upload_tables(dev); });
    return g_tab_status[dev];
}

struct DevInfo { int cus = 0; int occ[3][3] = {}; };
DevInfo g_dev[kMaxDev];
std::once_flag g_dev_once[kMaxDev];

template <class K>
int blocks_per_cu(K kernel, int wg)
{
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, wg, 0) != hipSuccess || nb < 1) nb = 1;
    return nb;
}

const DevInfo &dev_info()
{
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::call_once(g_dev_once[dev], [dev] {
        DevInfo &d = g_dev[dev];
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) == hipSuccess) d.cus = prop.multiProcessorCount;
        if (d.cus <= 0) d.cus = 256;
        d.occ[0][0] = blocks_per_cu(k_ntt_fwd<0>, NTT_WG);
        d.occ[0][1] = blocks_per_cu(k_ntt_fwd<1>, NTT_WG);
        d.occ[0][2] = blocks_per_cu(k_ntt_fwd<2>, NTT_WG);
        d.occ[1][0] = blocks_per_cu(k_ntt_inv<0>, NTT_WG);
        d.occ[1][1] = blocks_per_cu(k_ntt_inv<1>, NTT_WG);
        d.occ[1][2] = blocks_per_cu(k_ntt_inv<2>, NTT_WG);
        d.occ[2][0] = blocks_per_cu(k_poly_mul<0, false>, mul_wg<0>());
        d.occ[2][1] = blocks_per_cu(k_poly_mul<1, false>, mul_wg<1>());
        d.occ[2][2] = blocks_per_cu(k_poly_mul<2, false>, mul_wg<2>());
    });
    return g_dev[dev];
}

// Launch shape: one workgroup per `ppw * waves` consecutive work units.  ppw
// grows with the batch (amortising the 16 KiB LDS-table prologue) but never
// beyond what keeps >= 4 workgroups per CU in flight.
#ifndef NTT_MIN_WG_PER_CU
#define NTT_MIN_WG_PER_CU 2   // 4 and 8 measured 2-5 % slower on a 65 536-poly n=1024 launch, equal at 2^20 (profiles/r01/ab_launch_shape.json)
#endif
struct Launch { uint32_t grid, ppw; };
Launch launch_for(int op, int ps, size_t npoly)
{
    const size_t upw = param_set(ps)->logn == 11 ? 1 : 2;
    const size_t units = (npoly + upw - 1) / upw;
    const size_t waves = (size_t)(op == 2 ? (param_set(ps)->logn == 11 ? MUL_WG_BIG : MUL_WG) : NTT_WG) / 64;
    const size_t min_groups = (size_t)dev_info().cus * NTT_MIN_WG_PER_CU;
    size_t ppw = units / (waves * min_groups);
    ppw = ppw < 1 ? 1 : (ppw > NTT_PPW_MAX ? NTT_PPW_MAX : ppw);
    return {(uint32_t)((units + waves * ppw - 1) / (waves * ppw)), (uint32_t)ppw};
}

int check_common(int ps, const void *p, size_t batch)
{
    if (!param_set(ps)) return NTT_ERR_PARAM;
    if (batch == 0) return NTT_OK;
    if (!p) return NTT_ERR_NULL;
    if (((uintptr_t)p) & 3u) return NTT_ERR_ALIGN;
    if (batch > (size_t)0xFFFFFFFFu / 2) return NTT_ERR_SIZE;
    return NTT_OK;
}

bool partial_overlap(const void *x, const void *y, size_t bytes)
{
    const uintptr_t a = (uintptr_t)x, b = (uintptr_t)y;
    if (a == b) return false;
    return a < b + bytes && b < a + bytes;
}

int finish_launch()
{
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) { t_last_hip = (int)e; return NTT_ERR_HIP; }
    return NTT_OK;
}

template <template <int> class Launcher, class... Args>
int dispatch(int ps, Args... args)
{
    switch (ps) {
    case 0: return Launcher<0>::run(args...);
    case 1: return Launcher<1>::run(args...);
    case 2: return Launcher<2>::run(args...);
    default: return NTT_ERR_PARAM;
    }
}

template <int PS> struct LFwd {
    static int run(const uint32_t *in, uint32_t *out, size_t batch, hipStream_t s)
    {
        const Launch l = launch_for(0, PS, batch);
        hipLaunchKernelGGL(k_ntt_fwd<PS>, dim3(l.grid), dim3(NTT_WG), 0, s, in, out, (uint32_t)batch, l.ppw);
        return finish_launch();
    }
};
// out[t] = in[brv(t)] per polynomial: the forward kernel's load -> LDS
// transpose -> store path with no arithmetic (V = 6).  Natural-order load,
// pass-2 register j of lane l holds pos 32*brv6(l) + j, stored at
// brv(pos) = brv5(j)*S + l: both sides lane-contiguous 256-B runs.
template <int PS> struct LBitrev {
    static int run(const uint32_t *in, uint32_t *out, size_t batch, hipStream_t s)
    {
        const Launch l = launch_for(0, PS, batch);
        hipLaunchKernelGGL((k_ntt_fwd<PS, 6>), dim3(l.grid), dim3(NTT_WG), 0, s, in, out, (uint32_t)batch, l.ppw);
        return finish_launch();
    }
};
template <int PS> struct LInv {
    static int run(const uint32_t *in, uint32_t *out, size_t batch, hipStream_t s)
    {
        const Launch l = launch_for(1, PS, batch);
        hipLaunchKernelGGL(k_ntt_inv<PS>, dim3(l.grid), dim3(NTT_WG), 0, s, in, out, (uint32_t)batch, l.ppw);
        return finish_launch();
    }
};
template <int PS> struct LMul {
    static int run(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch, hipStream_t s, bool bhat)
    {
        const Launch l = launch_for(2, PS, batch);
        if (bhat) hipLaunchKernelGGL((k_poly_mul<PS, true>), dim3(l.grid), dim3(mul_wg<PS>()), 0, s, a, b, c, (uint32_t)batch, l.ppw);
        else hipLaunchKernelGGL((k_poly_mul<PS, false>), dim3(l.grid), dim3(mul_wg<PS>()), 0, s, a, b, c, (uint32_t)batch, l.ppw);
        return finish_launch();
    }
};
template <int PS> struct LPw {
    static int run(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t count4, hipStream_t s)
    {
        const DevInfo &d = dev_info();
        size_t g = (count4 + WG - 1) / WG, cap = (size_t)d.cus * 8;
        hipLaunchKernelGGL(k_pointwise<PS>, dim3((uint32_t)(g < cap ? g : cap)), dim3(WG), 0, s,
                           (const uint4 *)a, (const uint4 *)b, (uint4 *)c, count4);
        return finish_launch();
    }
};

int transform(bool inverse, uint32_t *out, const uint32_t *in, size_t batch, int ps, void *stream)
{
    int rc = check_common(ps, in, batch);
    if (rc == NTT_OK && batch) rc = check_common(ps, out, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    const size_t bytes = batch * param_set(ps)->n * 4;
    if (partial_overlap(in, out, bytes)) return NTT_ERR_ALIAS;
    if ((rc = ensure_device_tables()) != NTT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    return inverse ? dispatch<LInv>(ps, in, out, batch, s) : dispatch<LFwd>(ps, in, out, batch, s);
}

}  // namespace

void set_last_hip(int e) { t_last_hip = e; }

}  // namespace qntt

// ==========================================================================
// C ABI (include/qtesla_ntt.h)
// ==========================================================================
using namespace qntt;

extern "C" {

int ntt_param_info(int ps, uint32_t *n, uint32_t *q, uint32_t *psi, uint32_t *omega,
                   uint32_t *omega_inv, uint32_t *n_inv)
{
    const ParamSet *p = param_set(ps);
    if (!p) return NTT_ERR_PARAM;
    const Tables &t = cpu_tables(ps);
    if (n) *n = p->n;
    if (q) *q = p->q;
    if (psi) *psi = p->psi;
    if (omega) *omega = t.omega;
    if (omega_inv) *omega_inv = t.omega_inv;
    if (n_inv) *n_inv = t.n_inv;
    return NTT_OK;
}

int ntt_get_tables(int ps, uint32_t *bitrev_tbl, uint32_t *Phi, uint32_t *invPhi, uint32_t *tf0, uint32_t *ti0)
{
    const ParamSet *p = param_set(ps);
    if (!p) return NTT_ERR_PARAM;
    const Tables &t = cpu_tables(ps);
    const size_t b = (size_t)p->n * 4;
    if (bitrev_tbl) memcpy(bitrev_tbl, t.bitrev_tbl.data(), b);
    if (Phi) memcpy(Phi, t.Phi.data(), b);
    if (invPhi) memcpy(invPhi, t.invPhi.data(), b);
    if (tf0) memcpy(tf0, t.tf0.data(), b);
    if (ti0) memcpy(ti0, t.ti0.data(), b);
    return NTT_OK;
}

int poly_ntt(uint32_t *d_poly, const uint32_t *twiddleFactor, size_t batch, int ps, void *stream)
{
    (void)twiddleFactor;  // dead parameter, as in the reference kernels
    return transform(false, d_poly, d_poly, batch, ps, stream);
}

int poly_invntt(uint32_t *d_poly, const uint32_t *twiddleFactor, size_t batch, int ps, void *stream)
{
    (void)twiddleFactor;
    return transform(true, d_poly, d_poly, batch, ps, stream);
}

int poly_bitrev_copy(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    int rc = check_common(ps, d_in, batch);
    if (rc == NTT_OK && batch) rc = check_common(ps, d_out, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    if (partial_overlap(d_in, d_out, batch * param_set(ps)->n * 4)) return NTT_ERR_ALIAS;
    if ((rc = ensure_device_tables()) != NTT_OK) return rc;
    return dispatch<LBitrev>(ps, d_in, d_out, batch, (hipStream_t)stream);
}

int poly_ntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(false, d_out, d_in, batch, ps, stream);
}

int poly_invntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(true, d_out, d_in, batch, ps, stream);
}

static int mul_common(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b, size_t batch, int ps, void *stream,
                      bool bhat)
{
    int rc;
    if ((rc = check_common(ps, d_a, batch)) != NTT_OK || batch == 0) return rc;
    if ((rc = check_common(ps, d_b, batch)) != NTT_OK) return rc;
    if ((rc = check_common(ps, d_c, batch)) != NTT_OK) return rc;
    const size_t bytes = batch * param_set(ps)->n * 4;
    if (partial_overlap(d_a, d_c, bytes) || partial_overlap(d_b, d_c, bytes)) return NTT_ERR_ALIAS;
    if ((rc = ensure_device_tables()) != NTT_OK) return rc;
    return dispatch<LMul>(ps, d_a, d_b, d_c, batch, (hipStream_t)stream, bhat);
}

int poly_mul(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b, size_t batch, int ps, void *stream)
{
    return mul_common(d_c, d_a, d_b, batch, ps, stream, false);
}

int poly_mul_ntt(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_bhat, size_t batch, int ps, void *stream)
{
    return mul_common(d_c, d_a, d_bhat, batch, ps, stream, true);
}

int poly_mul_nussbaumer(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b, size_t batch, int ps, int ring,
                        void *stream)
{
    int rc;
    if ((rc = check_common(ps, d_a, batch)) != NTT_OK) return rc;
    if (ring != NTT_RING_Q && ring != NTT_RING_M32) return NTT_ERR_PARAM;
    if (batch == 0) return NTT_OK;
    if ((rc = check_common(ps, d_b, batch)) != NTT_OK) return rc;
    if ((rc = check_common(ps, d_c, batch)) != NTT_OK) return rc;
    if ((((uintptr_t)d_a) | ((uintptr_t)d_b) | ((uintptr_t)d_c)) & 15u) return NTT_ERR_ALIGN;
    const size_t bytes = batch * param_set(ps)->n * 4;
    if (partial_overlap(d_a, d_c, bytes) || partial_overlap(d_b, d_c, bytes)) return NTT_ERR_ALIAS;
    const int e = nussbaumer_launch(ps, ring, d_a, d_b, d_c, batch, stream, dev_info().cus);
    if (e != (int)hipSuccess) { t_last_hip = e; return NTT_ERR_HIP; }
    return NTT_OK;
}

int poly_pointwise(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b, size_t batch, int ps, void *stream)
{
    int rc;
    if ((rc = check_common(ps, d_a, batch)) != NTT_OK || batch == 0) return rc;
    if ((rc = check_common(ps, d_b, batch)) != NTT_OK) return rc;
    if ((rc = check_common(ps, d_c, batch)) != NTT_OK) return rc;
    if ((((uintptr_t)d_a) | ((uintptr_t)d_b) | ((uintptr_t)d_c)) & 15u) return NTT_ERR_ALIGN;
    const size_t count = batch * param_set(ps)->n;
    if (partial_overlap(d_a, d_c, count * 4) || partial_overlap(d_b, d_c, count * 4)) return NTT_ERR_ALIAS;
    return dispatch<LPw>(ps, d_a, d_b, d_c, count / 4, (hipStream_t)stream);
}

int ntt_fill_uniform(uint32_t *d_poly, size_t batch, int ps, uint64_t seed, uint64_t first_poly, void *stream)
{
    int rc = check_common(ps, d_poly, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    const ParamSet *p = param_set(ps);
    const size_t count = batch * p->n;
    const DevInfo &d = dev_info();
    size_t g = (count + WG - 1) / WG, cap = (size_t)d.cus * 16;
    hipLaunchKernelGGL(k_fill_uniform, dim3((uint32_t)(g < cap ? g : cap)), dim3(WG), 0, (hipStream_t)stream,
                       d_poly, count, p->q, seed, first_poly * p->n);
    return finish_launch();
}

int ntt_last_hip_error(void) { return t_last_hip; }

// Diagnostic entry point (csrc/ntt_internal.h, not part of the public ABI):
// launches kernel variant `variant` of op 0 = forward / 1 = inverse with the
// production grid, for bottleneck attribution (tools/variants.py).
int ntt_debug_variant(int op, int variant, uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    int rc = check_common(ps, d_in, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    if ((rc = ensure_device_tables()) != NTT_OK) return rc;
    hipStream_t s = (hipStream_t)stream;
    if (op == 2) {   // copies of n = 2048 polys, 2 workgroups of 8 waves per CU
        const uint32_t g2 = (uint32_t)dev_info().cus * 2;
        if (variant == 0) hipLaunchKernelGGL((k_copy_diag<1>), dim3(g2), dim3(512), 0, s, d_in, d_out, (uint32_t)batch);
        else hipLaunchKernelGGL((k_copy_diag<4>), dim3(g2), dim3(512), 0, s, d_in, d_out, (uint32_t)batch);
        return finish_launch();
    }
    const Launch l = launch_for(op, ps, batch);
    const uint32_t g = l.grid, nb = (uint32_t)batch, pw = l.ppw;
#define QNTT_VAR(PSV)                                                                                   \
    if (ps == PSV) {                                                                                    \
        switch (op * 16 + variant) {                                                                     \
        case 0: hipLaunchKernelGGL((k_ntt_fwd<PSV, 0>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 1: hipLaunchKernelGGL((k_ntt_fwd<PSV, 1>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 2: hipLaunchKernelGGL((k_ntt_fwd<PSV, 2>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 3: hipLaunchKernelGGL((k_ntt_fwd<PSV, 3>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 4: hipLaunchKernelGGL((k_ntt_fwd<PSV, 4>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 5: hipLaunchKernelGGL((k_ntt_fwd<PSV, 5>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 16: hipLaunchKernelGGL((k_ntt_inv<PSV, 0>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 17: hipLaunchKernelGGL((k_ntt_inv<PSV, 1>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 18: hipLaunchKernelGGL((k_ntt_inv<PSV, 2>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        case 19: hipLaunchKernelGGL((k_ntt_inv<PSV, 3>), dim3(g), dim3(NTT_WG), 0, s, d_in, d_out, nb, pw); break; \
        default: return NTT_ERR_PARAM;                                                                  \
        }                                                                                               \
        return finish_launch();                                                                         \
    }
    QNTT_VAR(0)
    QNTT_VAR(1)
    QNTT_VAR(2)
#undef QNTT_VAR
    return NTT_ERR_PARAM;
}

const char *ntt_strerror(int code)
{
    switch (code) {
    case NTT_OK: return "ok";
    case NTT_ERR_PARAM: return "unknown param_set";
    case NTT_ERR_NULL: return "NULL device pointer";
    case NTT_ERR_ALIGN: return "misaligned device pointer";
    case NTT_ERR_HIP: return "HIP runtime error";
    case NTT_ERR_SIZE: return "batch too large";
    case NTT_ERR_ALIAS: return "partially overlapping buffers";
    default: return "unknown error";
    }
}

int ntt_build_info(char *buf, size_t len)
{
    const char *s = "qtesla_ntt gfx950: 1 launch/op, wave-per-poly (n=2048) / half-wave-per-poly (n=1024), "
                    "32 coeff/lane, LDS XOR-swizzled transpose, permlane32 bit-5 stage, Shoup/Harvey lazy butterflies";
    if (!buf || !len) return (int)strlen(s);
    snprintf(buf, len, "%s", s);
    return (int)strlen(s);
}

}  // extern "C"
