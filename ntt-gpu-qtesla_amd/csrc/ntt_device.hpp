// ntt_device.hpp -- gfx950 (CDNA4) device code of the batched negacyclic NTT:
// arithmetic, register/LDS geometry, transform passes and the kernel templates.
// Included by exactly one translation unit per shared object (csrc/ntt_kernels.hip
// for the product library, tools/ntt_diag.hip for the diagnostic one).
//
// Replaces the reference's 10-34 per-stage launches per batch (NTT.cu:2388-2425)
// with one launch per operation.  Geometry:
//
//   * one wave owns one n=2048 polynomial, or two n=1024 polynomials (one per
//     32-lane half); every lane holds 32 coefficients in VGPRs;
//   * pass 1: register layout pos = lane + S*j (S = 64 or 32, j = 0..31); the
//     five stages on pos bits [LOGN-5, LOGN-1] are in-register radix-2
//     butterflies with wave-uniform twiddles (scalar loads from __constant__);
//   * n = 2048 only: the stage on pos bit 5 pairs lanes l and l^32 and runs on
//     v_permlane32_swap (no LDS);
//   * one wave-private LDS transpose (conflict-free XOR swizzle, 32 x ds_write_b32
//     + 8 x ds_read_b128 per lane, no s_barrier) to layout pos = 32*Lp + j;
//   * pass 2: the five stages on pos bits [0,4] in registers with per-lane
//     twiddles read from the workgroup's LDS table;
//   * the forward's output is bit-reversed in registers and is written in
//     natural order directly: for fixed j the lanes cover one contiguous run.
//
// Arithmetic: Harvey lazy butterflies with Shoup (precomputed-quotient
// Barrett) multiplication, q < 2^30 so 4q < 2^32:
//   CT: x in [0,4q) -> x' = x mod 2q;  t = y*w mod q in [0,2q);
//       (x'+t, x'-t+2q) in [0,4q)^2                             (7 VALU)
//   GS: (x+y reduced to [0,2q), (x-y)*w by a signed Shoup product in [0,2q))
//                                                               (7 VALU)
// Outputs are reduced to canonical [0,q) before they are stored.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "pset.hpp"

namespace qntt {

// twiddles (w, w'), index k in [0, n): fwd = psi^brv(k) stored negated,
// inv = psi^-brv(k) stored centred (see ct_bfly / sshoup_mul)
__constant__ uint2 c_fwd0[1024];
__constant__ uint2 c_inv0[1024];
__constant__ uint2 c_fwd1[1024];
__constant__ uint2 c_inv1[1024];
__constant__ uint2 c_fwd2[2048];
__constant__ uint2 c_inv2[2048];

// ------------------------------------------------------------------------
// modular arithmetic (NTT.cu:379-470 barrett_red/_addModP/_subModP, restated)
// ------------------------------------------------------------------------
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return a < b ? a : b; }

// Conditional subtraction x >= C ? x - C : x, the lazy reductions (hipcc:
// v_sub_u32 + v_min_u32).  A v_sub_co_u32 + v_cndmask_b32 form issues faster
// in isolation (50 vs 36 lanes/clk/CU per pair, profiles/r02/valu_rates.log)
// but its SGPR-mask hazards cost the same in the kernels: fwd / inv / poly_mul
// unchanged within noise (profiles/r02/ab_csub.log).
template <uint32_t C>
__device__ __forceinline__ uint32_t csub(uint32_t x)
{
    return umin(x, x - C);
}

// low word of a*b + c (one v_mad_u64_u32)
__device__ __forceinline__ uint32_t madlo32(uint32_t a, uint32_t b, uint32_t c)
{
    return (uint32_t)((uint64_t)a * b + c);
}

template <uint32_t Q>
__device__ __forceinline__ uint32_t shoup_mul(uint32_t a, uint32_t w, uint32_t wp)
{
    // a < 2^32, w < q, wp = floor(w 2^32 / q)  ->  result == a*w mod q, in [0, 2q)
    const uint32_t qe = __umulhi(a, wp);
    return madlo32(qe, 0u - Q, a * w);
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
    return madlo32(e, 0u - Q, d * ws);
}

// Forward twiddles are stored NEGATED on the device (wn = 2^32 - w, Shoup
// companion wp of w): the multiply-add then yields -t directly, so both outputs
// cost one instruction each (v_sub, v_add3):  x' = a + t,  y' = a - t + 2q.
template <uint32_t Q, bool REDUCE = true>
__device__ __forceinline__ void ct_bfly(uint32_t &x, uint32_t &y, uint32_t wn, uint32_t wp)
{
    const uint32_t a = REDUCE ? csub<2 * Q>(x) : x;   // [0,4q) -> [0,2q)
    const uint32_t qe = __umulhi(y, wp);
    const uint32_t tn = madlo32(qe, Q, y * wn);           // -t, t in [0,2q)
    x = a - tn;
    y = a + tn + 2 * Q;
}

// GS butterfly, inputs in [0,2q): x' = (x+y) mod 2q, y' = (x-y) w in [0,2q).
// 7 VALU: v_add, v_sub, v_min, v_sub, then the three of sshoup_mul.
template <uint32_t Q>
__device__ __forceinline__ void gs_bfly(uint32_t &x, uint32_t &y, uint32_t ws, uint32_t wps)
{
    const uint32_t s = csub<2 * Q>(x + y);   // [0,4q) -> [0,2q)
    const uint32_t d = x - y;                 // (-2q, 2q) as a signed value
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

// [0,4q) -> canonical [0,q)
template <class P>
__device__ __forceinline__ uint32_t canon4(uint32_t x)
{
    return csub<P::Q>(csub<P::Q2>(x));
}

// ------------------------------------------------------------------------
// per-lane geometry and the wave-private LDS transpose
// ------------------------------------------------------------------------
// XOR swizzle of the transpose buffer (hi = pos >> 5):
//   phys(pos) = pos ^ (pos8 << 2) ^ (pos9 << 3) ^ ((pos7 ^ pos10) << 4) ^ (pos7 << 5)
// Bijective; conflict-free for ds_write_b32 / ds_read_b32 in the pass-1
// layouts and ds_read_b128 / ds_write_b128 in the bit-reversed pass-2
// layout (tests/test_lds_layout.py, gfx950 lane-group bank model).
__host__ __device__ constexpr uint32_t xm_of(uint32_t hi)   // XOR on pos bits 2..4
{
    return (((hi >> 3) & 1) << 2) | (((hi >> 4) & 1) << 3) | ((((hi >> 2) ^ (hi >> 5)) & 1) << 4);
}

template <class P>
struct Lane {
    static constexpr bool BIG = (P::LOGN == 11);   // one poly per wave
    static constexpr uint32_t S = BIG ? 64 : 32;   // pass-1 stride
    static constexpr uint32_t UPW = BIG ? 1 : 2;   // polys per wave unit
    uint32_t lane, h, Lp;
    uint32_t wlo, woff;    // pass-1 LDS write/read (b32) address parts
    uint32_t rbase, rxm;   // pass-2 LDS read/write (b128) address parts
    uint32_t brl;          // lane index within its poly: pass-1 column, and bitrev(Lp)

    __device__ __forceinline__ Lane() : Lane(threadIdx.x & 63) {}
    // from a lane index the compiler cannot see through (opaque_lane): the
    // derived LDS addresses are recomputed where they are used instead of
    // being kept live across a whole work unit
    __device__ __forceinline__ explicit Lane(uint32_t lane_)
    {
        lane = lane_;
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
    // word offset of this lane's pass-1 column relative to the first word of
    // unit u (a wave-uniform base, u * UPW * N): stores, and loads with the
    // odd-batch rule of load_poly
    __device__ __forceinline__ uint32_t col() const { return BIG ? brl : h * P::N + brl; }
    __device__ __forceinline__ uint32_t col_load(uint32_t u, uint32_t npoly) const
    {
        return BIG ? brl : ((u * UPW + h < npoly) ? h * P::N : 0u) + brl;
    }
    __device__ __forceinline__ static size_t unit_base(uint32_t u) { return (size_t)u * (UPW * P::N); }
    // index of this lane's polynomial in wave unit u
    __device__ __forceinline__ uint32_t poly(uint32_t u) const { return u * UPW + (BIG ? 0u : h); }
    // the polynomial this lane loads from: its own, or for the second half of
    // the batch's last n=1024 unit when the batch is odd, the unit's first
    // (valid) one -- loads stay unconditional (no exec masking and no selects
    // per load, which cost ~900 v_mov_b64 per unit in the plain loop); the
    // results of such lanes are never stored
    __device__ __forceinline__ uint32_t load_poly(uint32_t u, uint32_t npoly) const
    {
        const uint32_t p = poly(u);
        return (BIG || p < npoly) ? p : u * UPW;
    }
};

// pos>>5 of register j in the pass-1 layout (n=2048: after the bit-5 swap)
template <class P>
__host__ __device__ constexpr uint32_t hi_of(int j)
{
    return P::LOGN == 11 ? (uint32_t)((j & 1) + 4 * (j >> 1)) : (uint32_t)j;
}

// Word offset, relative to the lane's `brl` column of its polynomial, of
// register j in the pass-1 arrangement that the transposes use (n = 2048: the
// post-swap arrangement pos = l5 + 32 e + 64 h + 128 m for j = 2m + e, i.e.
// two 128-B runs per instruction; n = 1024: pos = l5 + 32 j).
template <class P>
__host__ __device__ constexpr uint32_t p1s_off(int j)
{
    return P::LOGN == 11 ? (uint32_t)(32 * (j & 1) + 128 * (j >> 1)) : (uint32_t)(32 * j);
}

template <class P>
__device__ __forceinline__ uint32_t p1_addr(const Lane<P> &L, int j)
{
    const uint32_t hj = hi_of<P>(j);   // the lane part of hi (n = 2048: 2h) enters neither XOR term
    return (L.wlo ^ xm_of(hj)) + 32 * (hj ^ ((hj >> 2) & 1)) + L.woff;
}

// LDS operations of one wave complete in issue order, so the wave-private
// transposes need no s_barrier; this only keeps the compiler from moving
// accesses across the phase boundaries.
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// A wave-uniform zero the compiler cannot see through.  Adding it to the
// index of a uniform twiddle load keeps that load an s_load inside the
// work loop instead of letting LICM hoist all ~126 twiddle words into
// registers (which cost 2-3 waves/SIMD of occupancy).
__device__ __forceinline__ uint32_t opaque_zero()
{
    uint32_t z = 0;
    asm volatile("" : "+s"(z));
    return z;
}

__device__ __forceinline__ uint32_t opaque_lane()
{
    uint32_t l = threadIdx.x & 63;
    asm volatile("" : "+v"(l));
    return l;
}

// wave index within the workgroup, as a scalar (wave-uniform) value: unit
// indices and per-unit base addresses derived from it stay in SGPRs, so the
// global accesses take the saddr + 32-bit lane offset form
__device__ __forceinline__ uint32_t wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

constexpr int XPOSE_WORDS = 2048;   // per-wave transpose buffer (8 KiB)

// pass-1 arrangement (registers, post-swap for n=2048) -> pass-2 layout
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

// pass-2 layout -> pass-1 arrangement (n=2048: the post-swap arrangement)
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

__device__ __forceinline__ constexpr uint32_t brv5(int j)
{
    return (uint32_t)(((j & 1) << 4) | ((j & 2) << 2) | (j & 4) | ((j & 8) >> 2) | ((j & 16) >> 4));
}

// ------------------------------------------------------------------------
// twiddle access
// ------------------------------------------------------------------------
// Table base + an opaque wave-uniform zero: every uniform twiddle read below
// becomes an s_load_dwordx{2,8,16} with an immediate offset, re-issued per
// work unit instead of ~126 hoisted words pinning registers.
template <int PS, bool INV>
__device__ __forceinline__ const uint2 *tw_base()
{
    const uint32_t z = opaque_zero();
    if constexpr (PS == 0) return (INV ? c_inv0 : c_fwd0) + z;
    else if constexpr (PS == 1) return (INV ? c_inv1 : c_fwd1) + z;
    else return (INV ? c_inv2 : c_fwd2) + z;
}

// Per-lane pass-2 twiddles live in a per-workgroup LDS table, lane-major
// (entry e, lane t) so a ds_read_b64 by 64 lanes is conflict-free:
//   e = 2^(4-b) - 1 + m for stage bit b,  k = 2^(LOGN-1-b) + (Lp << (4-b)) + m
constexpr int TW2_ENTRIES = 31;
constexpr int TW2_WORDS = TW2_ENTRIES * 64 * 2 + 64;   // 15.5 KiB + the 32-entry bit-5 table
constexpr int TW2_VEC4 = TW2_WORDS / 4;                // 1008 uint4
// lanes per table entry: n = 1024 runs two polynomials per wave, one per
// 32-lane half, whose lane twiddles are equal -- its table holds 32 lanes
// (7.75 KiB: half the workgroup prologue, config 2's HBM traffic 1.04x ->
// see DESIGN.md §7) and lane l reads entry column l & 31 (lanes l, l + 32
// share an address: a broadcast, still conflict-free)
template <class P> constexpr uint32_t tw2_lanes() { return P::LOGN == 11 ? 64u : 32u; }
template <class P> constexpr int tw2_vec4() { return P::LOGN == 11 ? TW2_VEC4 : TW2_ENTRIES * 32 * 2 / 4; }
template <class P> __device__ __forceinline__ uint32_t tw2_idx(int e, uint32_t lane)
{
    return (uint32_t)e * tw2_lanes<P>() + (lane & (tw2_lanes<P>() - 1u));
}

// Host-built images of the per-workgroup LDS twiddle table (lane-major
// pass-2 entries + the 32-entry bit-5 table), one per (param set, direction):
// the workgroup prologue is then one coalesced 16 KiB copy with one wait.
__device__ uint4 g_tw2img[3][2][TW2_VEC4];

template <int PS, bool INV, int NT>
__device__ __forceinline__ void fill_tw2(uint2 *tab)
{
    constexpr int V4 = tw2_vec4<typename PSel<PS>::T>();
    const uint4 *src = g_tw2img[PS][INV ? 1 : 0];
    uint4 *dst = reinterpret_cast<uint4 *>(tab);
    constexpr int ITER = (V4 + NT - 1) / NT;
    uint4 v[ITER];   // loads unconditional (clamped index): a conditionally set array went to scratch memory
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
        const int i = threadIdx.x + k * NT;
        v[k] = src[i < V4 ? i : V4 - 1];
    }
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
        const int i = threadIdx.x + k * NT;
        if (i < V4) dst[i] = v[k];
    }
}

// ------------------------------------------------------------------------
// transform passes
// ------------------------------------------------------------------------
// forward pass 1: CT stages on pos bits LOGN-1 .. LOGN-5 (j bits 4..0),
// twiddle index k = 2^s + (j >> (5-s)) -- wave-uniform.
// `tw` = the uniform twiddles k < 32 (wave-uniform pointer), `sw` = the
// 32-entry bit-5 table in LDS.  RED0: inputs in [0,4q) (stage 0 reduces too);
// otherwise inputs < 2q.
// USW: `sw` is a wave-uniform (__constant__) bit-5 table; the lane-half
// twiddle is selected per lane from the two scalar-loaded candidates
template <bool USW>
__device__ __forceinline__ uint2 bit5_tw(const uint2 *sw, int m, uint32_t h)
{
    if constexpr (USW) {
        const uint2 w0 = sw[2 * m], w1 = sw[2 * m + 1];
        return make_uint2(h ? w1.x : w0.x, h ? w1.y : w0.y);
    } else {
        return sw[2 * m + h];
    }
}

template <class P, bool RED0 = false, bool USW = false>
__device__ __forceinline__ void fwd_pass1_tw(uint32_t (&r)[32], uint32_t h, const uint2 *tw, const uint2 *sw)
{
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int hh = 16 >> s;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const uint2 w = tw[(1u << s) + (uint32_t)(j >> (5 - s))];
                if (s == 0 && !RED0) ct_bfly<P::Q, false>(r[j], r[j + hh], w.x, w.y);   // inputs < 2q
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
            const uint2 w = bit5_tw<USW>(sw, m, h);   // k = 32 + 2m + h
            ct_bfly<P::Q>(r[2 * m], r[2 * m + 1], w.x, w.y);
        }
    }
}

template <int PS, class P>
__device__ __forceinline__ void fwd_pass1(uint32_t (&r)[32], uint32_t h, const uint2 *sw)
{
    fwd_pass1_tw<P>(r, h, tw_base<PS, false>(), sw);
}

// ---- typed forward for poly_mul --------------------------------------------
// Inside the fused product the forward's outputs never leave the kernel, so a
// butterfly may skip the +2q bias of y' = a - t + 2q when the value's next
// consumer tolerates a signed value in (-2q, 2q) ("S" type; "U" = [0, 4q)):
// a reduction (min(x, x + 2q) instead of min(x, x - 2q)), BaseMul's
// canonicalisation, or a multiply by a signed Shoup product with a centred
// twiddle.  That turns the v_add3 of y' into a v_add.  Which registers are S
// is fixed at compile time by the stage structure (register j after pass-1
// stage s <= 3 is S iff it was the y output).  Pass 1's S-typed multiplies
// use the centred twiddles below (compile-time literals, k < 32); pass 2's
// lane twiddles exist unsigned only, so there a y' is left S only when its
// consumer is an x input or BaseMul.  With the loop-invariant transpose
// addresses it pays for: -1.4 % (p-III) / -2.2 % (p-I); alone +1.5 % / +0.9 %
// (profiles/r03/ab_polymul_*.log).  In poly_ntt (HBM-bound) it was -0.6 %
// p-III, 0 p-I (profiles/r03/ab_fwd_lazybias.log) and is not used there.
__host__ __device__ constexpr uint32_t cbrv32(uint32_t x, int bits)
{
    uint32_t r = 0;
    for (int i = 0; i < bits; i++) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
// (-ws mod 2^32, wps) of forward twiddle k < 32, ws = psi^brv(k) centred
template <class P>
struct FwdSignedTw {
    uint32_t wn[32], wp[32];
    constexpr FwdSignedTw() : wn(), wp()
    {
        for (uint32_t k = 0; k < 32; k++) {
            const TwPair c = csigned_tw(cpow(P::PSI, cbrv32(k, P::LOGN), P::Q), P::Q);
            wn[k] = 0u - c.x;
            wp[k] = c.y;
        }
    }
};

// CT butterfly with typed operands: XS / YS = x / y in S form, YOS = leave
// y' in S form (no +2q); RED = reduce x (off for canonical inputs).  y in S
// form takes the signed Shoup quotient (centred twiddle (wsn, wps)).
template <uint32_t Q, bool RED, bool XS, bool YS, bool YOS>
__device__ __forceinline__ void ct_bfly_t(uint32_t &x, uint32_t &y, uint32_t wn, uint32_t wp)
{
    const uint32_t a = !RED ? x : XS ? umin(x, x + 2 * Q) : csub<2 * Q>(x);   // [0, 2q)
    uint32_t qe;
    if constexpr (YS) qe = (uint32_t)(((int64_t)(int32_t)y * (int32_t)wp - 0x80000000ll) >> 32);
    else qe = __umulhi(y, wp);
    const uint32_t tn = madlo32(qe, Q, y * wn);   // -t, t in [0, 2q)
    x = a - tn;
    y = YOS ? a + tn : a + tn + 2 * Q;
}

template <class P>
__device__ __forceinline__ void fwd_pass1_lz(uint32_t (&r)[32], uint32_t h, const uint2 *tw, const uint2 *sw)
{
    constexpr FwdSignedTw<P> ST{};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int hh = 16 >> s;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const uint32_t k = (1u << s) + (uint32_t)(j >> (5 - s));
                // both inputs were outputs of the same kind of the previous stage
                const bool ts = s > 0 && (j & (2 * hh)) != 0;
                if (s == 0) {
                    const uint2 w = tw[k];
                    ct_bfly_t<P::Q, false, false, false, true>(r[j], r[j + hh], w.x, w.y);   // canonical inputs
                } else if (ts) {
                    if (s < 4) ct_bfly_t<P::Q, true, true, true, true>(r[j], r[j + hh], ST.wn[k], ST.wp[k]);
                    else ct_bfly_t<P::Q, true, true, true, false>(r[j], r[j + hh], ST.wn[k], ST.wp[k]);
                } else {
                    const uint2 w = tw[k];
                    if (s < 4) ct_bfly_t<P::Q, true, false, false, true>(r[j], r[j + hh], w.x, w.y);
                    else ct_bfly_t<P::Q, true, false, false, false>(r[j], r[j + hh], w.x, w.y);   // U into the swap / transpose
                }
            }
        }
    }
    if constexpr (P::LOGN == 11) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const auto pr = __builtin_amdgcn_permlane32_swap(r[2 * m], r[2 * m + 1], false, false);
            r[2 * m] = pr[0];
            r[2 * m + 1] = pr[1];
            const uint2 w = sw[2 * m + h];
            ct_bfly<P::Q>(r[2 * m], r[2 * m + 1], w.x, w.y);
        }
    }
}

// pass 2 down to pos bit BMIN (U inputs from the transpose).  A y' stays S
// when its consumer is an x input of the next stage or (last stage) BaseMul;
// so after the last stage register j is S iff j & 2^BMIN.
template <class P, int BMIN>
__device__ __forceinline__ void fwd_pass2_lz(uint32_t (&r)[32], const uint2 *tab, uint32_t lane)
{
#pragma unroll
    for (int b = 4; b >= BMIN; --b) {
        const int hh = 1 << b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const int e = (1 << (4 - b)) - 1 + (j >> (b + 1));
                const uint2 w = tab[tw2_idx<P>(e, lane)];
                const bool xs = b < 4 && (j & (2 * hh)) != 0;          // x came out S from stage b+1
                const bool yos = b == BMIN || ((j + hh) & (hh >> 1)) == 0;
                if (xs) {
                    if (yos) ct_bfly_t<P::Q, true, true, false, true>(r[j], r[j + hh], w.x, w.y);
                    else ct_bfly_t<P::Q, true, true, false, false>(r[j], r[j + hh], w.x, w.y);
                } else {
                    if (yos) ct_bfly_t<P::Q, true, false, false, true>(r[j], r[j + hh], w.x, w.y);
                    else ct_bfly_t<P::Q, true, false, false, false>(r[j], r[j + hh], w.x, w.y);
                }
            }
        }
    }
}

// BMIN > 0 stops short: the stages on pos bits BMIN-1..0 are left out
// (poly_mul's incomplete transform, BaseMul)
template <class P, int BMIN = 0>
__device__ __forceinline__ void fwd_pass2(uint32_t (&r)[32], const uint2 *tab, uint32_t lane)
{
#pragma unroll
    for (int b = 4; b >= BMIN; --b) {
        const int hh = 1 << b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const int e = (1 << (4 - b)) - 1 + (j >> (b + 1));
                const uint2 w = tab[tw2_idx<P>(e, lane)];
                ct_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
            }
        }
    }
}

// WIDE0: the first stage's inputs lie in [0, 3q) with |x - y| < 2^31
// (poly_mul's BaseMul with a half-canonical first operand, p-III:
// [0, 2.19q)): x' = (x + y) mod 2q by a three-candidate min (v_min3)
template <class P, int BMIN = 0, bool WIDE0 = false>
__device__ __forceinline__ void inv_pass2(uint32_t (&r)[32], const uint2 *tab, uint32_t lane)
{
#pragma unroll
    for (int b = BMIN; b <= 4; ++b) {
        const int hh = 1 << b;
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if ((j & hh) == 0) {
                const int e = (1 << (4 - b)) - 1 + (j >> (b + 1));
                const uint2 w = tab[tw2_idx<P>(e, lane)];
                if (WIDE0 && b == BMIN) {
                    const uint32_t x = r[j], y = r[j + hh], sm = x + y;   // [0, 6q)
                    r[j] = umin(umin(sm, sm - P::Q2), sm - 2 * P::Q2);
                    r[j + hh] = sshoup_mul<P::Q>(x - y, w.x, w.y);
                } else {
                    gs_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
                }
            }
        }
    }
}

// Products in the incomplete NTT domain of poly_mul.  After the forward's
// stages down to pos bit LOGR, register group g = j >> LOGR of a lane holds
// the residue of its polynomial mod x^D - zeta, D = 2^LOGR (coefficient i in
// register D g + i), zeta = +w for g even and -w for g odd, w = psi^brv(k) the
// twiddle of the stage on pos bit LOGR (LDS entry 2^(4-LOGR) - 1 + (g >> 1)).
// Per residue: a, b canonical, b~_i = zeta b_i (negated Shoup product,
// two-candidate min, in [0, q]), the D sums of D products in 64 bits
// (< D q^2) and one Montgomery REDC each, (c + m q) / 2^32 with
// m = -c q^-1 mod 2^32 (one v_mad_u64_u32), times 2^-32 (folded into the
// final scaling with (n/D)^-1); outputs above 2q get one conditional
// subtraction.  Replaces LOGR stages of each forward and of the inverse and
// the pointwise product.
template <class P, int LOGR>
struct BaseMul {
    static constexpr int D = 1 << LOGR;
    static_assert(D >= 2, "the zeta-split residue products need D >= 2");
    static constexpr double QD = P::Q;
    static constexpr int E0 = (1 << (4 - LOGR)) - 1;   // LDS entry of the stage on pos bit LOGR

    // zeta-split form: c_k = L_k + zeta R * REDC(H_k), L_k / H_k the
    // sums of the D products without / with the wrap (a, b canonical, H_k
    // < (D-1) q^2), zeta R = zeta 2^32 mod q in [0, q] per residue PAIR (the
    // +w / -w residues share w).  Per residue that is 7 x (REDC + one 64-bit
    // multiply-add) instead of 7 b~ products (Shoup + two-candidate min):
    // p-III 8.19 -> 8.04 ms, p-I 3.65 -> 3.58 ms (profiles/r03/ab_polymul_zsplit_lz.log).
    // Bound: c_k < (k+1) q^2 + q ((D-1-k) q^2 / 2^32 + q) <= (D + q/2^32) q^2.
    static constexpr double CZ = (D + QD / 4294967296.0) * QD * QD;
    static_assert(CZ + 4294967296.0 * QD < 18446744073709551616.0, "zeta-split REDC input fits 64 bits");
    static_assert(CZ / 4294967296.0 + QD < 4.0 * QD, "zeta-split: one conditional subtraction reaches [0, 2q)");
    static constexpr bool OUT_CSUB_Z = CZ / 4294967296.0 + QD >= 2.0 * QD;
    // Half-canonical a: a only reduced to [0, 2q) (one conditional subtraction
    // instead of two), b canonical: c_k < 2 D q^2 (the k = D-1 sum; the others
    // stay below (2D - 1 + 2q/2^32) q^2).  The REDC output may then pass 4q
    // (p-III: 4.19q): one conditional subtraction leaves it below WH = 2.19q and
    // the inverse's first stage takes such inputs (inv_pass2 WIDE0).
    static constexpr double CZH = 2.0 * D * QD * QD;
    static_assert(CZH + 4294967296.0 * QD < 18446744073709551616.0, "half-canonical REDC input fits 64 bits");
    static constexpr double OUTH = CZH / 4294967296.0 + QD;
    static constexpr double WH = OUTH >= 2.0 * QD ? OUTH - 2.0 * QD : OUTH;   // after the csub
    static_assert(!OUT_CSUB_Z || (WH < 3.0 * QD && WH < 2147483648.0 && 2.0 * WH < 4294967296.0),
                  "first inverse stage: x + y < 6q fits 32 bits, |x - y| < 2^31");
    static constexpr bool OUT_CSUB_H = OUTH >= 2.0 * QD;
    // only where the z-split output already needs its conditional subtraction
    // (p-III, -1.3 %, profiles/r03/ab_polymul_ahalf.log); elsewhere the
    // half-canonical a would move one csub to the output
    static constexpr bool AH = OUT_CSUB_Z;
    static constexpr bool WIDE = AH && OUTH >= 4.0 * QD;   // inverse's first stage in WIDE0 form

    static __device__ __forceinline__ uint32_t redc(uint64_t c)
    {
        const uint32_t m = (uint32_t)c * P::QNEG;
        return (uint32_t)(((uint64_t)m * P::Q + c) >> 32);
    }

    // [0,4q) (U) or (-2q,2q) (S, typed forward) -> canonical [0,q)
    // (s is a compile-time constant once the residue loop is unrolled)
    static __device__ __forceinline__ uint32_t canon(bool s, uint32_t x)
    {
        return s ? csub<P::Q>(umin(x, x + P::Q2)) : canon4<P>(x);
    }
    // the same to [0, 2q) only
    static __device__ __forceinline__ uint32_t half(bool s, uint32_t x)
    {
        return s ? umin(x, x + P::Q2) : csub<P::Q2>(x);
    }

    // ODD_S: the odd residues (registers with bit LOGR set) hold S-form values
    template <bool ODD_S>
    static __device__ __forceinline__ void run_zsplit(uint32_t (&ra)[32], const uint32_t (&rb)[32], const uint2 *tab,
                                                      uint32_t lane)
    {
#pragma unroll
        for (int gp = 0; gp < 16 / D; ++gp) {
            const uint2 w = tab[tw2_idx<P>(E0 + gp, lane)];   // (-w mod 2^32, w')
            // -(w R mod q) in (-2q, 0] (negated Shoup product of the constant R)
            const uint32_t tn = madlo32(__umulhi(P::R, w.y), P::Q, P::R * w.x);
            const uint32_t zr[2] = {umin(0u - tn, (0u - P::Q) - tn),   // +w: w R mod q in [0, q]
                                    umin(tn + P::Q, tn + P::Q2)};      // -w
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const int g = 2 * gp + e;
                uint32_t z = zr[e];
                asm volatile("" : "+v"(z));   // one residue at a time (no interleaving of the pair: it spills)
                uint32_t a[D], b[D];
#pragma unroll
                for (int i = 0; i < D; ++i) {
                    a[i] = AH ? half(ODD_S && (g & 1), ra[D * g + i]) : canon(ODD_S && (g & 1), ra[D * g + i]);
                    b[i] = canon(ODD_S && (g & 1), rb[D * g + i]);
                }
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    uint64_t c = 0;
#pragma unroll
                    for (int i = 0; i <= k; ++i) c += (uint64_t)a[i] * b[k - i];
                    if (k < D - 1) {
                        uint64_t hs = 0;
#pragma unroll
                        for (int i = k + 1; i < D; ++i) hs += (uint64_t)a[i] * b[k + D - i];
                        c += (uint64_t)z * redc(hs);
                    }
                    const uint32_t r = redc(c);
                    ra[D * g + k] = (AH ? OUT_CSUB_H : OUT_CSUB_Z) ? csub<P::Q2>(r) : r;
                }
            }
        }
    }

    template <bool ODD_S = false>
    static __device__ __forceinline__ void run(uint32_t (&ra)[32], const uint32_t (&rb)[32], const uint2 *tab, uint32_t lane)
    {
        run_zsplit<ODD_S>(ra, rb, tab, lane);
    }
};

struct NoEmit {
    __device__ __forceinline__ void operator()(int, uint32_t) const {}
};

// inverse pass 1 without its last stage: (n=2048) GS on pos bit 5 + swap
// back, then the GS stages on pos bits LOGN-5 .. LOGN-2 (j bits 0..3); `tw` =
// the uniform twiddles k < 32.
template <class P, bool USW = false>
__device__ __forceinline__ void inv_pass1_head(uint32_t (&r)[32], uint32_t h, const uint2 *tw, const uint2 *sw)
{
    if constexpr (P::LOGN == 11) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const uint2 w = bit5_tw<USW>(sw, m, h);
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
}

// The last GS stage (pos bit LOGN-1, j bits 4): x' = (x+y) s0, y' = (x-y) s1
// with s0 = (s0w, s0p) a Shoup pair and s1 = (s1w, s1p) a centred signed
// pair (the stage's twiddle times the scaling), outputs in [0,2q), canonical
// when CANON.  `emit(j, v)` is called with each final output as soon as it is
// computed (the kernels store from there, so the 32 stores interleave with
// the last stage instead of queueing behind it as one tail).
template <class P, bool CANON, class Emit = NoEmit>
__device__ __forceinline__ void inv_last_stage(uint32_t (&r)[32], uint32_t s0w, uint32_t s0p, uint32_t s1w, uint32_t s1p,
                                               const Emit &emit = Emit())
{
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = r[j], y = r[j + 16];
        const uint32_t s = x + y;   // [0,4q)
        const uint32_t d = x - y;   // (-2q, 2q), signed
        const uint32_t a = shoup_mul<P::Q>(s, s0w, s0p);
        const uint32_t b = sshoup_mul<P::Q>(d, s1w, s1p);
        r[j] = CANON ? csub<P::Q>(a) : a;
        r[j + 16] = CANON ? csub<P::Q>(b) : b;
        emit(j, r[j]);
        emit(j + 16, r[j + 16]);
    }
}

// inverse pass 1: the head, then the last stage with the n^-1 scaling (times
// the S0 / S1 constants), output canonical.
template <int PS, class P, uint32_t S0, uint32_t S1, class Emit = NoEmit>
__device__ __forceinline__ void inv_pass1(uint32_t (&r)[32], uint32_t h, const uint2 *sw, const Emit &emit = Emit())
{
    inv_pass1_head<P>(r, h, tw_base<PS, true>(), sw);
    constexpr uint32_t S0P = cshoup(S0, P::Q);
    constexpr TwPair S1S = csigned_tw(S1, P::Q);
    inv_last_stage<P, true>(r, S0, S0P, S1S.x, S1S.y, emit);
}

// ------------------------------------------------------------------------
// global memory access
// ------------------------------------------------------------------------
// Output stores are nontemporal (streamed once, never re-read by the kernel);
// input loads too (read once): with nt stores, in place -4.5 % fwd / -2.1 %
// inv (profiles/r01/ab_nt_load.json, ab_ntstore_dma.json).
__device__ __forceinline__ void st_out(uint32_t *p, uint32_t v) { __builtin_nontemporal_store(v, p); }
__device__ __forceinline__ uint32_t ld_in(const uint32_t *p) { return __builtin_nontemporal_load(p); }

// The 32 words of a lane in a unit, at compile-time offsets from one base
// pointer (the offsets fold into the instructions' immediate field).
template <class Off>
__device__ __forceinline__ void load32(uint32_t (&r)[32], const uint32_t *src, Off off)
{
#pragma unroll
    for (int j = 0; j < 32; ++j) r[j] = ld_in(src + off(j));
}

// ------------------------------------------------------------------------
// work distribution
// ------------------------------------------------------------------------
// Workgroup b owns the contiguous unit range [b*WAVES*PPW, (b+1)*WAVES*PPW);
// at step i its waves take consecutive units b*WAVES*PPW + i*WAVES + wave.
// Workgroups are dispatched in order, so the units in flight chip-wide form a
// sliding contiguous window of HBM: measured 5.9 TB/s for this access shape
// vs 5.4 TB/s for a persistent grid-stride loop (profiles/r01/copybw.log).
// The first unit's global loads are issued before the workgroup prologue
// (`prologue` = the LDS twiddle-table fill + barrier), so the fill latency
// hides under the first unit's HBM latency.
template <int WAVES, class Prologue, class Load, class Process>
__device__ __forceinline__ void chunk_loop(uint32_t nunits, uint32_t ppw, Prologue &prologue, Load &load,
                                           Process &process)
{
    uint32_t r[32];
    uint32_t u = blockIdx.x * (WAVES * ppw) + wave_id();
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
// kernels
// ------------------------------------------------------------------------
// Workgroup = NTT_WG/64 waves, each with a private 8 KiB transpose buffer;
// the lane-twiddle table is shared by the workgroup.
#ifndef NTT_WG
#define NTT_WG 512   // fwd / inv: 8 waves, 64 + 15.75 KiB LDS -> 2 WG/CU
#endif
// poly_mul workgroup: 16 waves (128 + 31.5 KiB LDS, 1 WG/CU) at <= 128 VGPRs
// -> 4 waves/SIMD for both n.  n=1024 ran 8 waves at 2 waves/SIMD before the
// incomplete-domain product and the per-transpose address recomputation
// (fresh lanes) brought it under 128 VGPRs: 4 waves/SIMD is 4 % faster there
// (poly_mul_ntt 8 %), profiles/r02/ab_polymul_incomplete.log
// poly_mul's residue degree 2^MUL_LOGR: 8 (3 stages of each transform
// replaced by 8x8 products) is 3 % faster than 4 on p-III and 6 % on p-I; 16
// spills (profiles/r02/ab_polymul_incomplete.log)
constexpr int MUL_LOGR = 3;
#ifndef MUL_WG
#define MUL_WG 1024
#endif
#ifndef NTT_WAVES_PER_SIMD
#define NTT_WAVES_PER_SIMD 4
#endif
#ifndef MUL_WAVES_PER_SIMD
#define MUL_WAVES_PER_SIMD 4
#endif
// Compact tables: poly_mul (not poly_mul_ntt) reads only lane-table entries
// 0..2 (pass 2 stops at pos bit 3; BaseMul's zeta are entries 1, 2) and the
// bit-5 pairs, so its workgroup keeps just those (compact tables: 3.5 KiB for
// both directions instead of 31.5) and runs as two 8-wave workgroups per CU
// (same 4 waves/SIMD): the CU no longer drains to start the next workgroup.
// p-III 7.69 -> 7.35 ms, p-I 3.46 -> 3.25 ms per 2^20 (profiles/r04/r/)
template <int PS, bool BHAT> constexpr bool mul_compact() { return !BHAT; }
template <int PS, bool BHAT = false> constexpr int mul_wg() { return mul_compact<PS, BHAT>() ? 512 : MUL_WG; }
template <int PS> constexpr int mul_occ() { return MUL_WAVES_PER_SIMD; }
// lane-table entries a compact table keeps: the stages on pos bits 4 .. LOGR
// read entries 0 .. 2^(5-LOGR) - 2, BaseMul's zeta the last 2^(4-LOGR) of them
constexpr int MUL_CENT = (1 << (5 - MUL_LOGR)) - 1;
// compact table image: entries 0..MUL_CENT-1 (L lanes each), then the 32 bit-5 pairs
template <class P> constexpr int mul_ctab_words() { return MUL_CENT * (int)tw2_lanes<P>() * 2 + 64; }
template <int PS> constexpr int mul_logr() { return MUL_LOGR; }
constexpr int WG = 256;   // elementwise kernels
constexpr int NTT_WAVES = NTT_WG / 64;
constexpr int NTT_LDS_WORDS = NTT_WAVES * XPOSE_WORDS + TW2_WORDS;

// Ordering of the transforms' natural-order boundary (BR = bit-reversed):
//   forward: natural input; output natural (BR=false) or out[t] = X[brv(t)] (BR=true)
//   inverse: input natural (BR=false) or in[t] = X[brv(t)] (BR=true); output natural
template <int PS, bool BR>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_ntt_fwd(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NTT_LDS_WORDS];
    uint2 *tw2 = reinterpret_cast<uint2 *>(lds + NTT_WAVES * XPOSE_WORDS);
    auto prologue = [&]() {
        fill_tw2<PS, false, NTT_WG>(tw2);
        __syncthreads();
    };
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + LT::UPW - 1) / LT::UPW;

    auto load = [&](uint32_t (&r)[32], uint32_t u) {   // pass-1 layout: natural lane index
        load32(r, in + LT::unit_base(u) + L.col_load(u, npoly), [](int j) { return LT::S * j; });
    };
    // canonical output: BR=false from the bit-reversed pass-2 registers to
    // natural order, brv5(j)*S + lane; BR=true from the pass-1 arrangement
    auto store = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t poly = L.poly(u);
        if (LT::BIG || poly < npoly) {
            uint32_t *dst = out + LT::unit_base(u) + L.col();
            if constexpr (BR) dst += LT::BIG ? 32 * L.h : 0u;   // brl + 32 h = l5 + 64 h (p1s_off)
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                st_out(dst + (BR ? p1s_off<P>(j) : brv5(j) * LT::S), canon4<P>(r[j]));
            }
        }
    };
    auto front = [&](uint32_t (&r)[32], uint32_t) {
        fwd_pass1<PS, P>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
        lds_p1_to_p2<P>(r, buf, L);
        if constexpr (BR) {
            fwd_pass2<P>(r, tw2 + opaque_zero(), L.lane);
            lds_p2_to_p1<P>(r, buf, L);
        }
    };
    auto back = [&](uint32_t (&r)[32], uint32_t u) {
        if constexpr (!BR) fwd_pass2<P>(r, tw2 + opaque_zero(), L.lane);
        store(r, u);
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        front(r, u);
        back(r, u);
    };
    chunk_loop<NTT_WAVES>(nunits, ppw, prologue, load, process);
}

template <int PS, bool BR>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_ntt_inv(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NTT_LDS_WORDS];
    uint2 *tw2 = reinterpret_cast<uint2 *>(lds + NTT_WAVES * XPOSE_WORDS);
    auto prologue = [&]() {
        fill_tw2<PS, true, NTT_WG>(tw2);
        __syncthreads();
    };
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + LT::UPW - 1) / LT::UPW;

    // BR=false: natural-order input; pass-2 position 32*Lp + j holds X[brv(pos)]
    // BR=true:  bit-reversed input read in the pass-1 arrangement, transposed below
    auto load = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t *src = in + LT::unit_base(u) + L.col_load(u, npoly);
        if constexpr (BR) src += LT::BIG ? 32 * L.h : 0u;   // brl + 32 h = l5 + 64 h (p1s_off)
        load32(r, src, [](int j) { return BR ? p1s_off<P>(j) : brv5(j) * LT::S; });
    };
    auto front = [&](uint32_t (&r)[32], uint32_t) {
        if constexpr (BR) lds_p1_to_p2<P>(r, buf, L);
        inv_pass2<P>(r, tw2 + opaque_zero(), L.lane);
        lds_p2_to_p1<P>(r, buf, L);
    };
    auto back = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t poly = L.poly(u);
        uint32_t *dst = out + LT::unit_base(u) + L.col();   // pass-1 layout: natural lane index
        const bool valid = LT::BIG || poly < npoly;
        auto emit = [&](int j, uint32_t v) {
            if (valid) st_out(dst + LT::S * j, v);
        };
        inv_pass1<PS, P, P::NINV, P::C1>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero(), emit);
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        front(r, u);
        back(r, u);
    };
    chunk_loop<NTT_WAVES>(nunits, ppw, prologue, load, process);
}

// out[t] = in[brv(t)] per polynomial, any 32-bit words: the pass-1
// arrangement load -> LDS transpose -> the forward's bit-reversed store
// mapping (pass-2 register j of lane l holds word 32*Lp + j, stored at
// brv5(j)*S + l); both sides are 128/256-B runs, no arithmetic.
template <int PS>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_bitrev(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NTT_WAVES * XPOSE_WORDS];
    auto prologue = [] {};
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + LT::UPW - 1) / LT::UPW;
    auto load = [&](uint32_t (&r)[32], uint32_t u) {
        load32(r, in + LT::unit_base(u) + L.col_load(u, npoly) + (LT::BIG ? 32 * L.h : 0u),
               [](int j) { return p1s_off<P>(j); });
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        lds_p1_to_p2<P>(r, buf, L);
        const uint32_t poly = L.poly(u);
        if (LT::BIG || poly < npoly) {
            uint32_t *dst = out + LT::unit_base(u) + L.col();
#pragma unroll
            for (int j = 0; j < 32; ++j) st_out(dst + brv5(j) * LT::S, r[j]);
        }
    };
    chunk_loop<NTT_WAVES>(nunits, ppw, prologue, load, process);
}


// fused c = a*b mod (x^n+1): FWD(a), FWD(b) down to residues mod x^8 -+ zeta,
// their products (BaseMul; the 2^-32 of its REDC and the (n/8)^-1 are folded
// into the inverse's final scaling), INV from those residues -- one HBM read
// of a and b, one write of c.  The internal domain never leaves the kernel,
// so it need not be poly_ntt's.  BHAT: b is given already transformed
// (natural-order output of poly_ntt, the full domain), so a is transformed
// completely and multiplied pointwise (Montgomery) -- two transforms of work
// per product instead of three (poly_mul_ntt).  a, b and c may alias (no
// __restrict__): every lane loads its words before it stores any.
// VAR (tools/ntt_diag.hip only, bottleneck attribution): 1 = global loads
// and stores only (no arithmetic, no LDS), 2 = arithmetic + LDS only
// (register-made inputs, outputs kept live, nothing stored).
// compact copy of a direction's image (mul_compact)
template <int PS, bool INV, int NT>
__device__ __forceinline__ void fill_tw2_compact(uint2 *tab)
{
    using P = typename PSel<PS>::T;
    constexpr int LV = MUL_CENT * (int)tw2_lanes<P>() * 2 / 4, CV = mul_ctab_words<P>() / 4;
    const uint4 *src = g_tw2img[PS][INV ? 1 : 0];
    uint4 *dst = reinterpret_cast<uint4 *>(tab);
    for (int i = threadIdx.x; i < CV; i += NT) dst[i] = src[i < LV ? i : TW2_ENTRIES * 64 * 2 / 4 + (i - LV)];
}

template <int PS, bool BHAT, int VAR = 0>
__global__ __launch_bounds__((mul_wg<PS, BHAT>()), mul_occ<PS>()) void k_poly_mul(const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    constexpr bool CMP = mul_compact<PS, BHAT>();
    static_assert(MUL_CENT >= (1 << (5 - mul_logr<PS>())) - 1, "the compact table holds every lane entry pass 2 reads");
    constexpr int WG_ = mul_wg<PS, BHAT>();
    constexpr int WAVES = WG_ / 64;
    constexpr int TABW = CMP ? mul_ctab_words<P>() : TW2_WORDS;   // words per direction
    constexpr int SWO = CMP ? MUL_CENT * (int)tw2_lanes<P>() : TW2_ENTRIES * 64;   // bit-5 pairs' offset (pairs)
    __shared__ __attribute__((aligned(16))) uint32_t lds[WAVES * XPOSE_WORDS + 2 * TABW];
    uint2 *ftw2 = reinterpret_cast<uint2 *>(lds + WAVES * XPOSE_WORDS);
    uint2 *itw2 = ftw2 + TABW / 2;
    if constexpr (CMP) {
        fill_tw2_compact<PS, false, WG_>(ftw2);
        fill_tw2_compact<PS, true, WG_>(itw2);
    } else {
        fill_tw2<PS, false, WG_>(ftw2);
        fill_tw2<PS, true, WG_>(itw2);
    }
    __syncthreads();
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;

    const uint32_t nunits = (npoly + LT::UPW - 1) / LT::UPW;
    uint32_t u = blockIdx.x * (WAVES * ppw) + wave_id();
#pragma unroll 1
    for (uint32_t it = 0; it < ppw; ++it, u += WAVES) {   // dispatch-ordered chunk (see chunk_loop)
        if (u >= nunits) break;
        const uint32_t poly = L.poly(u);
        const bool valid = poly < npoly;
        const size_t ubase = LT::unit_base(u);
        // pass-1 layout: natural lane index.  Opaque per unit, so the lane
        // offsets are not folded into loop-invariant 64-bit addresses (which
        // pin VGPRs): the accesses keep the scalar base + 32-bit offset form
        uint32_t off = L.col(), loff = L.col_load(u, npoly);
        if constexpr (!BHAT) asm volatile("" : "+v"(off), "+v"(loff));
        // a first, then b: the transpose's memory fences keep b's loads below
        // a's transform, so only ~64 coefficients are live at the peak
        uint32_t ra[32], rb[32];
        if constexpr (VAR == 2) {
#pragma unroll
            for (int j = 0; j < 32; ++j) ra[j] = (u + (uint32_t)j * 0x01000193u + L.lane) & 0x1FFFFFFFu;   // < q
        } else {
            load32(ra, a + ubase + loff, [](int j) { return LT::S * j; });
        }
        if constexpr (VAR == 1) {
            load32(rb, b + ubase + loff, [](int j) { return LT::S * j; });
            uint32_t *pc = c + ubase + off;
#pragma unroll
            for (int j = 0; j < 32; ++j)
                if (valid) st_out(pc + LT::S * j, ra[j] + rb[j]);
            continue;
        }
        constexpr bool LZ = !BHAT;   // typed forwards (fwd_pass1_lz)
        if constexpr (LZ) fwd_pass1_lz<P>(ra, L.h, tw_base<PS, false>(), ftw2 + SWO + opaque_zero());
        else fwd_pass1<PS, P>(ra, L.h, ftw2 + SWO + opaque_zero());
        // loop-invariant transpose addresses (poly_mul: affordable once the
        // typed forwards took the p-III kernel from 126 to 96 VGPRs, 121 with
        // the hoisted addresses, no spills); the b-hat product keeps them at
        // n = 2048 and recomputes them from an opaque lane at n = 1024 (32-lane
        // twiddle table; hoisted: 22 spilled VGPRs)
        constexpr bool HOIST = BHAT ? P::LOGN == 11 : true;
        lds_p1_to_p2<P>(ra, buf, HOIST ? L : LT(opaque_lane()));
        if constexpr (LZ) fwd_pass2_lz<P, mul_logr<PS>()>(ra, ftw2 + opaque_zero(), L.lane);
        else fwd_pass2<P, BHAT ? 0 : mul_logr<PS>()>(ra, ftw2 + opaque_zero(), L.lane);
        // b-hat is in natural order: register j of the pass-2 layout holds
        // index brv5(j)*S + lane (the forward's store mapping)
        if constexpr (VAR == 2) {
#pragma unroll
            for (int j = 0; j < 32; ++j) rb[j] = (u + (uint32_t)j * 0x00FF0101u + L.lane) & 0x1FFFFFFFu;
        } else {
            load32(rb, b + ubase + loff, [](int j) { return LT::S * (BHAT ? brv5(j) : (uint32_t)j); });
        }
        uint32_t *pc = c + ubase + off;
        auto emit = [&](int j, uint32_t v) {   // stores interleaved with the last stage (see inv_pass1)
            if constexpr (VAR == 2) asm volatile("" ::"v"(v));
            else if (valid) st_out(pc + LT::S * j, v);
        };
        if constexpr (!BHAT) {
            // incomplete domain: both forwards stop above pos bit LOGR-1,
            // products mod x^(2^LOGR) -+ zeta, the inverse starts at pos bit
            // LOGR (BaseMul)
            if constexpr (LZ) fwd_pass1_lz<P>(rb, L.h, tw_base<PS, false>(), ftw2 + SWO + opaque_zero());
            else fwd_pass1<PS, P>(rb, L.h, ftw2 + SWO + opaque_zero());
            lds_p1_to_p2<P>(rb, buf, L);
            if constexpr (LZ) fwd_pass2_lz<P, mul_logr<PS>()>(rb, ftw2 + opaque_zero(), L.lane);
            else fwd_pass2<P, mul_logr<PS>()>(rb, ftw2 + opaque_zero(), L.lane);
            BaseMul<P, mul_logr<PS>()>::template run<LZ>(ra, rb, ftw2 + opaque_zero(), L.lane);
            inv_pass2<P, mul_logr<PS>(), BaseMul<P, mul_logr<PS>()>::WIDE>(ra, itw2 + opaque_zero(), L.lane);
            lds_p2_to_p1<P>(ra, buf, L);
            inv_pass1<PS, P, P::template ninv_r<mul_logr<PS>()>(), P::template c1_r<mul_logr<PS>()>()>(ra, L.h, itw2 + SWO + opaque_zero(), emit);
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) ra[j] = mont_mul<P>(csub<P::Q2>(ra[j]), csub<P::Q2>(rb[j]));   // b-hat < 2q
            inv_pass2<P>(ra, itw2 + opaque_zero(), L.lane);
            lds_p2_to_p1<P>(ra, buf, HOIST ? L : LT(opaque_lane()));
            inv_pass1<PS, P, P::NINV_R, P::C1_R>(ra, L.h, itw2 + SWO + opaque_zero(), emit);
        }
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
            uint32_t m = mont_mul<P>(csub<P::Q2>(v[k]), csub<P::Q2>(w[k]));
            m = shoup_mul<P::Q>(m, P::R, RP);
            v[k] = csub<P::Q>(m);
        }
        c[i] = make_uint4(v[0], v[1], v[2], v[3]);
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

}  // namespace qntt
