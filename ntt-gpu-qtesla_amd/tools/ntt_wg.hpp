// ntt_wg.hpp -- gfx950 n = 2048 transforms with one polynomial per 512-thread
// workgroup (round 3 experiment; measured slower than the
// wave-per-polynomial kernels, so it lives in the tools-only diag library:
// ntt_diag.hip op 4).  Included after ntt_device.hpp (it owns the twiddle
// tables c_fwd2 / c_inv2).
//
// Why this shape: measured on MI355X (profiles/r03/), an in-place stream in
// which every wave moves ONE 1 KiB piece (4 dwords per lane) runs at the
// flat-copy rate, 2.9 ms per 2 x 8 GiB, while one 8 KiB polynomial per wave
// (the wave-per-polynomial kernels of ntt_device.hpp) cannot go below
// 3.1-3.3 ms however the waves, workgroups, cache policies or store order
// are arranged: the store side of a wave that writes 8 KiB streams at
// 5.5-5.8 TB/s against 6.9 TB/s for 1 KiB (profiles/r03/rw_bw_*.log).
// So the 8 KiB of a polynomial are spread over the 8 waves of a workgroup:
// thread t holds 4 coefficients, loaded and stored as 4 lane-contiguous
// 256-B runs per wave (1 KiB per wave and direction).
//
// Dataflow (pos bits p10..p0; wave w = (w2, w1, w0), lane l = (l5..l0),
// register e = (e1, e0), v[e] with e = 2 e1 + e0):
//   pass A: e = (p10, p9)  w = (p8, p7, p6)   l = (p5..p0)                 stages 10, 9
//   pass B: e = (p8, p7)   w = (p10, p9, p6)  l = (p5..p0)                 stages 8, 7
//   pass C: e = (p6, p5)   w = (p10, p9, p8)  l = (p7, p4..p0)             stages 6, 5
//   pass D: e = (p4, p3)   w = (p10, p9, p8)  l = (p7, p6, p5, p2, p1, p0) stages 4, 3
//   pass E: e = (p2, p1)   w = (p10, p9, p8)  l = (p7..p3, p0)             stages 2, 1
//   pass F: e = (p1, p0)   w = (p2, p3, p4)   l = (p5, p6, ..., p10)       stage 0
// CT with psi^brv twiddles leaves X[k] at pos = brv11(k); pass F is laid out
// so that brv11(pos) = 1024 e0 + 512 e1 + 64 w + l: the forward stores, and
// the inverse loads, lane-contiguous 256-B runs at a per-register offset.
// The inverse runs F..A with GS butterflies, low stage first.  The twiddle of
// the stage on bit b is psi^(+-brv(k)), k = 2^(10-b) + (pos >> (b+1)): in
// passes A and B it is wave-uniform (scalar loads), in C..F it depends on the
// lane -- 11 (w, w') pairs per thread, the same for every polynomial, so the
// persistent workgroups load them once into VGPRs.  No LDS twiddle table.
//
// Between passes: 5 LDS exchanges, each one barrier (double-buffered by
// parity), every access conflict-free (32 distinct banks per half-wave for
// every register on both sides) and every register's address a compile-time
// offset from one per-thread base (padded row layouts instead of XOR
// swizzles): tests/test_lds_layout.py checks both properties and
// tests/test_wg_dataflow.py runs the dataflow exactly against the oracle.
//
// Workgroups are persistent (grid = resident workgroups), polynomial
// p = blockIdx + i gridDim, the next polynomial's 4 words prefetched into
// registers while the current one is transformed.
#pragma once
#include "../csrc/ntt_device.hpp"

namespace qntt {

// Diagnostic switches (tools/ab.py builds, never set in the product):
// WGP_DIAG 1 = no butterflies, 2 = no LDS exchanges, 3 = neither (memory only),
// 4 = no global memory (register-made inputs, stores behind an opaque false)
#ifndef WGP_DIAG
#define WGP_DIAG 0
#endif
// polynomials in flight per persistent workgroup beyond the current one
#ifndef WGP_PF
#define WGP_PF 2
#endif

constexpr int WGP_T = 512;         // threads per workgroup = one polynomial
constexpr int WGP_BUF = 2560;      // words per exchange buffer (largest address 2551)

// ---- pass layouts: pos of register 0 of thread (w, l) ----------------------
__host__ __device__ constexpr uint32_t wg_posA(uint32_t w, uint32_t l) { return (w << 6) | l; }
__host__ __device__ constexpr uint32_t wg_posB(uint32_t w, uint32_t l)
{
    return ((w >> 2) << 10) | (((w >> 1) & 1) << 9) | ((w & 1) << 6) | l;
}
__host__ __device__ constexpr uint32_t wg_posC(uint32_t w, uint32_t l) { return (w << 8) | ((l >> 5) << 7) | (l & 31); }
__host__ __device__ constexpr uint32_t wg_posD(uint32_t w, uint32_t l) { return (w << 8) | ((l >> 3) << 5) | (l & 7); }
__host__ __device__ constexpr uint32_t wg_posE(uint32_t w, uint32_t l) { return (w << 8) | ((l >> 1) << 3) | (l & 1); }
__host__ __device__ constexpr uint32_t wg_posF(uint32_t w, uint32_t l)
{
    // w = (p2, p3, p4), l = (p5, ..., p10): bit-reversed into pos bits 2..10
    return ((w >> 2) & 1) << 2 | ((w >> 1) & 1) << 3 | (w & 1) << 4 | (((l >> 5) & 1) << 5) | (((l >> 4) & 1) << 6) |
           (((l >> 3) & 1) << 7) | (((l >> 2) & 1) << 8) | (((l >> 1) & 1) << 9) | ((l & 1) << 10);
}

// ---- exchange address maps (bijective, pos -> LDS word) ---------------------
__host__ __device__ constexpr uint32_t wg_x12(uint32_t p) { return p; }
__host__ __device__ constexpr uint32_t wg_x3(uint32_t p) { return (p >> 5) * 40 + (p & 31); }
__host__ __device__ constexpr uint32_t wg_x4(uint32_t p)
{
    return ((((p >> 7) << 2) | ((p >> 3) & 3)) * 34) + ((((p >> 5) & 3) << 3) | (p & 7));
}
__host__ __device__ constexpr uint32_t wg_bit(uint32_t p, int i) { return (p >> i) & 1u; }
__host__ __device__ constexpr uint32_t wg_x5(uint32_t p)
{
    // columns: the writer's half-wave bits (p6 at stride 1), rows: p7..p10
    // (the reader's half-wave) then the writer's registers p1, p2; row stride 34
    return (wg_bit(p, 7) | wg_bit(p, 8) << 1 | wg_bit(p, 9) << 2 | wg_bit(p, 10) << 3 | wg_bit(p, 1) << 4 | wg_bit(p, 2) << 5) * 34 +
           (wg_bit(p, 6) | wg_bit(p, 0) << 1 | wg_bit(p, 3) << 2 | wg_bit(p, 4) << 3 | wg_bit(p, 5) << 4);
}

// register offsets (words) of exchange X on its earlier-pass side (W) and
// later-pass side (R), index e = 2 e1 + e0
template <int X> struct WgOff;
template <> struct WgOff<1> {
    static constexpr uint32_t W[4] = {0, 512, 1024, 1536}, R[4] = {0, 128, 256, 384};
};
template <> struct WgOff<2> {
    static constexpr uint32_t W[4] = {0, 128, 256, 384}, R[4] = {0, 32, 64, 96};
};
template <> struct WgOff<3> {
    static constexpr uint32_t W[4] = {0, 40, 80, 120}, R[4] = {0, 8, 16, 24};
};
template <> struct WgOff<4> {
    static constexpr uint32_t W[4] = {0, 34, 68, 102}, R[4] = {0, 2, 4, 6};
};
template <> struct WgOff<5> {
    static constexpr uint32_t W[4] = {0, 544, 1088, 1632}, R[4] = {0, 2, 544, 546};
};

// Per-thread constants: the 10 exchange bases and the lane-dependent
// twiddles of passes C..F (forward: negated (2^32 - w, w'); inverse: centred
// signed pairs), loaded once per workgroup.
struct WgThread {
    uint32_t wb[6], rb[6];   // [X] for X = 1..5
    uint2 tC6, tC5[2], tD4, tD3[2], tE2, tE1[2], tF0[2];
};

template <bool INV>
__device__ __forceinline__ void wg_setup(WgThread &T, uint32_t w, uint32_t l, const uint2 *tw)
{
    T.wb[1] = wg_x12(wg_posA(w, l));
    T.rb[1] = wg_x12(wg_posB(w, l));
    T.wb[2] = wg_x12(wg_posB(w, l));
    T.rb[2] = wg_x12(wg_posC(w, l));
    T.wb[3] = wg_x3(wg_posC(w, l));
    T.rb[3] = wg_x3(wg_posD(w, l));
    T.wb[4] = wg_x4(wg_posD(w, l));
    T.rb[4] = wg_x4(wg_posE(w, l));
    T.wb[5] = wg_x5(wg_posE(w, l));
    T.rb[5] = wg_x5(wg_posF(w, l));
    // stage on bit b of a pass with registers (pa, pb): k = 2^(10-b) + (pos >> (b+1)),
    // pos = the pass layout's pos of register 0 (+ e1 for the stage on pb)
    const uint32_t c = wg_posC(w, l), d = wg_posD(w, l), e = wg_posE(w, l), f = wg_posF(w, l);
    T.tC6 = tw[16 + (c >> 7)];
    T.tC5[0] = tw[32 + (c >> 6)];
    T.tC5[1] = tw[32 + (c >> 6) + 1];
    T.tD4 = tw[64 + (d >> 5)];
    T.tD3[0] = tw[128 + (d >> 4)];
    T.tD3[1] = tw[128 + (d >> 4) + 1];
    T.tE2 = tw[256 + (e >> 3)];
    T.tE1[0] = tw[512 + (e >> 2)];
    T.tE1[1] = tw[512 + (e >> 2) + 1];
    T.tF0[0] = tw[1024 + (f >> 1)];
    T.tF0[1] = tw[1024 + (f >> 1) + 1];
}

// exchange X: the forward writes its earlier-pass layout and reads the later
// one; the inverse the reverse.  One barrier: the buffer of the next exchange
// is the other one, whose last readers all passed this barrier.
template <int X, bool INV>
__device__ __forceinline__ void wg_xchg(uint32_t (&v)[4], uint32_t *buf, const WgThread &T)
{
    if constexpr (WGP_DIAG == 2 || WGP_DIAG == 3) return;
    const uint32_t wbase = INV ? T.rb[X] : T.wb[X], rbase = INV ? T.wb[X] : T.rb[X];
#pragma unroll
    for (int e = 0; e < 4; ++e) buf[wbase + (INV ? WgOff<X>::R[e] : WgOff<X>::W[e])] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = buf[rbase + (INV ? WgOff<X>::W[e] : WgOff<X>::R[e])];
}

// forward radix-4 pass, registers (pa, pb) = (e1, e0): stage pa with one
// twiddle, then stage pb with one twiddle per e1.  Inputs of the x operands
// in [0, 4q) (RED) -- or < 2q for the first stage -- outputs in [0, 4q).
template <class P, bool RED = true>
__device__ __forceinline__ void wg_ct4(uint32_t (&v)[4], uint2 ta, uint2 tb0, uint2 tb1)
{
    if constexpr (WGP_DIAG == 1 || WGP_DIAG == 3) return;
    ct_bfly<P::Q, RED>(v[0], v[2], ta.x, ta.y);
    ct_bfly<P::Q, RED>(v[1], v[3], ta.x, ta.y);
    ct_bfly<P::Q>(v[0], v[1], tb0.x, tb0.y);
    ct_bfly<P::Q>(v[2], v[3], tb1.x, tb1.y);
}

// inverse radix-4 pass: stage pb (per e1 twiddle) first, then stage pa
template <class P>
__device__ __forceinline__ void wg_gs4(uint32_t (&v)[4], uint2 ta, uint2 tb0, uint2 tb1)
{
    if constexpr (WGP_DIAG == 1 || WGP_DIAG == 3) return;
    gs_bfly<P::Q>(v[0], v[1], tb0.x, tb0.y);
    gs_bfly<P::Q>(v[2], v[3], tb1.x, tb1.y);
    gs_bfly<P::Q>(v[0], v[2], ta.x, ta.y);
    gs_bfly<P::Q>(v[1], v[3], ta.x, ta.y);
}

// wave-uniform twiddle of index k (a scalar load through an opaque zero, so
// the per-wave values are not hoisted into VGPRs)
template <bool INV>
__device__ __forceinline__ uint2 wg_utw(uint32_t k)
{
    return tw_base<2, INV>()[k];
}

// Forward transform of v (pass-A layout) in place; on return v holds the
// pass-F layout, outputs canonical.  `parity` selects the first buffer.
template <class P>
__device__ __forceinline__ void wg_fwd(uint32_t (&v)[4], uint32_t *lds, uint32_t parity, const WgThread &T, uint32_t w)
{
    uint32_t *b0 = lds + parity * WGP_BUF, *b1 = lds + (parity ^ 1) * WGP_BUF;
    // A: stage 10 (k = 1, inputs < 2q: no reduction), stage 9 (k = 2 + p10)
    wg_ct4<P, false>(v, wg_utw<false>(1), wg_utw<false>(2), wg_utw<false>(3));
    wg_xchg<1, false>(v, b0, T);
    // B: wave = (p10, p9, p6): stage 8 k = 4 + (p10 p9), stage 7 k = 8 + (p10 p9 p8)
    {
        const uint32_t hb = w >> 1;
        wg_ct4<P>(v, wg_utw<false>(4 + hb), wg_utw<false>(8 + 2 * hb), wg_utw<false>(9 + 2 * hb));
    }
    wg_xchg<2, false>(v, b1, T);
    wg_ct4<P>(v, T.tC6, T.tC5[0], T.tC5[1]);
    wg_xchg<3, false>(v, b0, T);
    wg_ct4<P>(v, T.tD4, T.tD3[0], T.tD3[1]);
    wg_xchg<4, false>(v, b1, T);
    wg_ct4<P>(v, T.tE2, T.tE1[0], T.tE1[1]);
    wg_xchg<5, false>(v, b0, T);
    ct_bfly<P::Q>(v[0], v[1], T.tF0[0].x, T.tF0[0].y);
    ct_bfly<P::Q>(v[2], v[3], T.tF0[1].x, T.tF0[1].y);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = canon4<P>(v[e]);
}

// Inverse transform of v (pass-F layout) in place; on return v holds the
// pass-A layout, outputs canonical (n^-1 psi^-i folded into the last stage).
template <class P>
__device__ __forceinline__ void wg_inv(uint32_t (&v)[4], uint32_t *lds, uint32_t parity, const WgThread &T, uint32_t w)
{
    uint32_t *b0 = lds + parity * WGP_BUF, *b1 = lds + (parity ^ 1) * WGP_BUF;
    gs_bfly<P::Q>(v[0], v[1], T.tF0[0].x, T.tF0[0].y);
    gs_bfly<P::Q>(v[2], v[3], T.tF0[1].x, T.tF0[1].y);
    wg_xchg<5, true>(v, b0, T);
    wg_gs4<P>(v, T.tE2, T.tE1[0], T.tE1[1]);
    wg_xchg<4, true>(v, b1, T);
    wg_gs4<P>(v, T.tD4, T.tD3[0], T.tD3[1]);
    wg_xchg<3, true>(v, b0, T);
    wg_gs4<P>(v, T.tC6, T.tC5[0], T.tC5[1]);
    wg_xchg<2, true>(v, b1, T);
    {
        const uint32_t hb = w >> 1;
        wg_gs4<P>(v, wg_utw<true>(4 + hb), wg_utw<true>(8 + 2 * hb), wg_utw<true>(9 + 2 * hb));
    }
    wg_xchg<1, true>(v, b0, T);
    // A: stage 9 (k = 2 + p10), then stage 10 with the n^-1 scaling
    {
        const uint2 t2 = wg_utw<true>(2), t3 = wg_utw<true>(3);
        gs_bfly<P::Q>(v[0], v[1], t2.x, t2.y);
        gs_bfly<P::Q>(v[2], v[3], t3.x, t3.y);
    }
    constexpr uint32_t S0P = cshoup(P::NINV, P::Q);
    constexpr TwPair S1S = csigned_tw(P::C1, P::Q);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const uint32_t x = v[j], y = v[j + 2];
        v[j] = csub<P::Q>(shoup_mul<P::Q>(x + y, P::NINV, S0P));
        v[j + 2] = csub<P::Q>(sshoup_mul<P::Q>(x - y, S1S.x, S1S.y));
    }
}

#ifndef WGP_WAVES_PER_SIMD
#define WGP_WAVES_PER_SIMD 8   // 4 workgroups (polynomials) per CU
#endif

// PERSIST: one persistent workgroup transforms polynomials blockIdx.x +
// i gridDim.x (grid = resident workgroups), per-thread twiddles loaded once
// from the __constant__ tables into VGPRs, the next polynomial prefetched.
// !PERSIST: one polynomial per workgroup (grid = batch), the twiddle table
// copied into LDS (16 KiB) while the polynomial's loads are in flight.
template <int PS, bool INV, bool PERSIST>
__global__ __launch_bounds__(WGP_T, WGP_WAVES_PER_SIMD) void k_wg_xform(const uint32_t *in, uint32_t *out, uint32_t npoly)
{
    using P = typename PSel<PS>::T;
    static_assert(P::N == 2048, "workgroup-per-polynomial kernels are n = 2048");
    __shared__ __attribute__((aligned(16))) uint32_t lds[2 * WGP_BUF + (PERSIST ? 0 : 4096)];
    const uint32_t t = threadIdx.x, w = wave_id(), l = t & 63;
    uint32_t p = blockIdx.x;
    if (p >= npoly) return;   // whole workgroup
    // natural side (forward load, inverse store): pos = t + 512 e;
    // bit-reversed side (forward store, inverse load): X[1024 e0 + 512 e1 + t]
    constexpr uint32_t NAT[4] = {0, 512, 1024, 1536}, BRV[4] = {0, 1024, 512, 1536};
    auto load = [&](uint32_t (&v)[4], uint32_t q) {
        const uint32_t *s = in + (size_t)q * 2048 + t;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            if constexpr (WGP_DIAG == 4) v[e] = (t + 7 * e + q) % P::Q;
            else v[e] = ld_in(s + (INV ? BRV[e] : NAT[e]));
        }
    };
    auto store = [&](const uint32_t (&v)[4], uint32_t q) {
        uint32_t *d = out + (size_t)q * 2048 + t;
        if constexpr (WGP_DIAG == 4) {
            if (opaque_zero() != 7u) return;
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) st_out(d + (INV ? NAT[e] : BRV[e]), v[e]);
    };
    WgThread T;
    uint32_t v[4];
    if constexpr (!PERSIST) {
        // table loads first: vmcnt retires in order, so the table can be
        // written to LDS while the polynomial's loads are still in flight
        const uint4 *src = reinterpret_cast<const uint4 *>(INV ? c_inv2 : c_fwd2);
        uint4 *tab4 = reinterpret_cast<uint4 *>(lds + 2 * WGP_BUF);
        const uint4 a = src[t], b = src[t + 512];
        load(v, p);
        tab4[t] = a;
        tab4[t + 512] = b;
        __syncthreads();
        wg_setup<INV>(T, w, l, reinterpret_cast<const uint2 *>(lds + 2 * WGP_BUF));
        if constexpr (INV) wg_inv<P>(v, lds, 0, T, w);
        else wg_fwd<P>(v, lds, 0, T, w);
        store(v, p);
    } else {
        load(v, p);
        wg_setup<INV>(T, w, l, INV ? c_inv2 : c_fwd2);
        // ring of WGP_PF prefetched polynomials: pf[i] holds p + (i+1) G
        uint32_t pf[WGP_PF][4];
        const uint32_t G = gridDim.x;
#pragma unroll
        for (int i = 0; i < WGP_PF; ++i)
            if (p + (i + 1) * G < npoly) load(pf[i], p + (i + 1) * G);
        uint32_t parity = 0;
        for (;;) {
            const uint32_t pn = p + (WGP_PF + 1) * G;   // the one to request now
            uint32_t nv[4];
            if (pn < npoly) load(nv, pn);
            if constexpr (INV) wg_inv<P>(v, lds, parity, T, w);
            else wg_fwd<P>(v, lds, parity, T, w);
            store(v, p);
            p += G;
            if (p >= npoly) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                v[e] = pf[0][e];
#pragma unroll
                for (int i = 0; i + 1 < WGP_PF; ++i) pf[i][e] = pf[i + 1][e];
                pf[WGP_PF - 1][e] = nv[e];
            }
            parity ^= 1;   // 5 exchanges per polynomial: the next one starts on the other buffer
        }
    }
}

}  // namespace qntt
