// ntt_lat.hpp -- gfx950 small-batch (latency) transforms for n = 1024 ..
// 8192 and products for n <= 4096: one polynomial per workgroup of n/4
// threads (n/8 at n = 8192), 4 coefficients per thread and radix-4 group.
//
// Why: the qTESLA signing loop transforms one polynomial per call (BASELINE
// config 1), and the batch kernels of ntt_device.hpp give a polynomial to one
// wave (half a wave at n = 1024): ~1 500 VALU in one wave, which a lone wave
// issues at one instruction per ~4 cycles (MI355X_MICROARCH.md, 'vector-
// instruction ISSUE cost'), behind a 15.75 KiB LDS table fill and barrier.
// Here the same butterflies are spread over n/4 lanes (4 or 8 waves, one or
// two per SIMD), so a thread runs ~L/2 radix-4 groups (~80 VALU) and the
// critical path is the global loads, L/2 LDS exchanges and the stores.
//
// Dataflow (L = log2 n, T = n/4 threads, thread t, pos bits p_{L-1}..p_0):
//   pass j = 0 .. NP-1 runs CT stages hb = L-1-2j and lb = hb-1 on the group
//   base(t) + {0, 2^lb, 2^hb, 2^hb + 2^lb}, base(t) = t with two zero bits
//   inserted at lb, hb (pass 0: base = t, so the group is t + {0,T,2T,3T}, the
//   coalesced natural-order loads).  For odd L the last pass is the lone stage
//   on bit 0, over the group 4t + {0,1,2,3}.  Stage b's twiddle index is
//   k = 2^(L-1-b) + (pos >> (b+1)), psi^brv(k) (the batch kernels' tables
//   c_fwd*/c_inv*, NTT.cu:2216-2260's CT with merged twist), so stage hb uses
//   one twiddle per group and stage lb two (k and k+1).
//   Between passes the group values go through LDS (double-buffered, one
//   barrier per exchange, addresses padded by one word per 32 so the strided
//   late passes stay conflict-free); the forward's last exchange is the
//   bit-reversal to natural order, the inverse's first the reverse.
//   The inverse runs the passes backwards with GS butterflies (stage lb, then
//   hb), the last stage scaled by n^-1 (and psi^-brv(1)) like the batch
//   kernels; every twiddle is loaded from the __constant__ table up front,
//   while the polynomial's own loads are in flight.
// BR = true: the forward leaves X in bit-reversed order (out[t] = X[brv(t)],
// poly_ntt_bitrev) and the inverse takes that order (poly_invntt_bitrev):
// the reordering exchange is skipped.
#pragma once
#include "ntt_big.hpp"   // sfor

namespace qntt {

// The small-batch switch (entry points of include/qtesla_ntt.h NTT_OP_*):
// up to two tiers of one-polynomial-per-workgroup kernels per (parameter
// set, entry point) before the batch kernels take over -- tier 0 for batches
// up to max0 with radix rb0, tier 1 up to max1 with radix rb1 (rb = 2: the
// radix-4 kernels of this file, 3 / 4: the radix-8 / radix-16 ones of
// ntt_latr.hpp; the products have radix-4 kernels only).  Round 6 set them
// from sweeps that time every family against the batch kernels in one
// process from 64 polynomials to the BASELINE batches (tools/switch_sweep.py,
// profiles/r06/sweep/, profiles/r06/latr/) and the per-launch latency of
// batches 1-256 (tools/latency.py, profiles/r06/latr/latsmall_*.log): each max
// is the last measured batch at which that family beat the batch kernels.
// The one-polynomial-per-workgroup kernels keep the memory system's fast
// regime (short-lived workgroups) but pay their twiddles per
// polynomial; at the BASELINE batches the batch kernels stay ahead (p-III
// forward at 2^20: 3.23 ms against 3.38 / 3.50 ms radix-8 / 16, 4.77 radix-4),
// except at n = 1024 where radix-16 (one wave per polynomial) runs level.
// LAT_FWD / LAT_INV: in place (poly_ntt / poly_invntt, or the _oop calls
// with d_out == d_in); LAT_FWD_OOP / LAT_INV_OOP: distinct buffers.  The
// families rank differently in place: the batch kernels run 2-3 % slower in
// place than out of place, the one-polynomial-per-workgroup kernels the same
// (one process: p-I forward at 2^20 1.686 / 1.649 ms against radix-16 1.593 /
// 1.600, profiles/r06/latr/floorio_*.log; the in-place and out-of-place
// sweeps, switch_sweep_inplace.json / switch_sweep_latr.json, ran on two
// boxes), so at n = 1024 the radix-16 kernel takes every in-place batch above
// its first tier
enum LatOp { LAT_FWD, LAT_INV, LAT_FWD_BR, LAT_INV_BR, LAT_MUL, LAT_MUL_NTT, LAT_FWD_OOP, LAT_INV_OOP, LAT_NOPS };
struct LatTier {
    int rb0;
    size_t max0;
    int rb1;
    size_t max1;
};
// A/B builds only (tools/switch_sweep.py): NTT_LAT_FORCE 0 sends every batch
// to the batch kernels, 1 every batch to the radix-4 kernels where they exist
#ifdef NTT_LAT_FORCE
constexpr LatTier lat_tier(int ps, int op)
{
    return NTT_LAT_FORCE == 0 || (ps == 4 && (op == LAT_MUL || op == LAT_MUL_NTT)) ? LatTier{2, 0, 2, 0}
                                                                                    : LatTier{2, ~(size_t)0, 2, 0};
}
#else
constexpr size_t kAll = 0x7FFFFFFF;   // every batch the ABI accepts
constexpr LatTier kLatTier[5][LAT_NOPS] = {
    // fwd (in place)         inv (in place)         fwd_br               inv_br                mul              mul_ntt          fwd_oop                inv_oop
    {{2, 1024, 4, kAll}, {2, 1024, 4, kAll}, {2, 1024, 3, 4096}, {2, 1024, 3, 32768}, {2, 2816, 0, 0}, {2, 5120, 0, 0}, {2, 1024, 4, 262144}, {2, 1024, 4, 262144}},  // ref
    {{2, 1024, 4, kAll}, {2, 1024, 4, kAll}, {2, 1024, 3, 4096}, {2, 1024, 3, 32768}, {2, 2816, 0, 0}, {2, 5120, 0, 0}, {2, 1024, 4, 262144}, {2, 1024, 4, 262144}},  // p-I
    {{3, 131072, 0, 0}, {3, 65536, 0, 0}, {3, 2048, 0, 0}, {3, 2048, 0, 0}, {2, 1280, 0, 0}, {2, 1792, 0, 0}, {3, 65536, 0, 0}, {3, 32768, 0, 0}},                  // p-III
    {{4, 16384, 0, 0}, {4, 16384, 0, 0}, {3, 2048, 0, 0}, {3, 16384, 0, 0}, {2, 512, 0, 0}, {2, 512, 0, 0}, {4, 16384, 0, 0}, {3, 32768, 0, 0}},                     // n = 4096
    {{4, 32768, 0, 0}, {4, 32768, 0, 0}, {4, 1024, 0, 0}, {3, 16384, 0, 0}, {2, 0, 0, 0}, {2, 0, 0, 0}, {4, 32768, 0, 0}, {4, 32768, 0, 0}},                         // n = 8192
};
constexpr LatTier lat_tier(int ps, int op) { return kLatTier[ps][op]; }
#endif
// the largest batch any small-batch tier takes (0: none)
constexpr size_t lat_max_batch(int ps, int op)
{
    const LatTier t = lat_tier(ps, op);
    return t.max1 > t.max0 ? t.max1 : t.max0;
}
// radix bits of the small-batch kernel for `batch` (0: the batch kernels)
constexpr int lat_radix(int ps, int op, size_t batch)
{
    const LatTier t = lat_tier(ps, op);
    return batch <= t.max0 ? t.rb0 : batch <= t.max1 ? t.rb1 : 0;
}

// full n-point twiddle tables of the n = 4096 / 8192 sets for the latency
// kernels (the batch kernels there read per-chunk images), [fwd / inv][k],
// same pairs as c_fwd* / c_inv* (dev_const_table)
__device__ uint2 g_lattw3[2][4096];
__device__ uint2 g_lattw4[2][8192];

template <int PS, bool INV>
__device__ __forceinline__ const uint2 *lat_tw()
{
    if constexpr (PS == 0) return INV ? c_inv0 : c_fwd0;
    else if constexpr (PS == 1) return INV ? c_inv1 : c_fwd1;
    else if constexpr (PS == 2) return INV ? c_inv2 : c_fwd2;
    else if constexpr (PS == 3) return g_lattw3[INV ? 1 : 0];
    else return g_lattw4[INV ? 1 : 0];
}

__host__ __device__ constexpr uint32_t lat_pad(uint32_t x) { return x + (x >> 5); }

// n/4 radix-4 groups per pass; a workgroup has at most 1024 threads, so at
// n = 8192 each thread takes R = 2 groups, g = t and t + T
template <int L>
struct LatGeo {
    static constexpr int N = 1 << L;
    static constexpr int GN = N / 4;                 // groups per pass
    static constexpr int R = GN > 1024 ? GN / 1024 : 1;
    static constexpr int T = GN / R;                 // threads
    static constexpr int NP = (L + 1) / 2;           // passes (the last one radix-2 when L is odd)
    static constexpr int BUF = lat_pad(N - 1) + 1;   // words per exchange buffer
    // high / low stage bit of pass j (lb < 0: the lone stage on bit 0)
    static constexpr int hb(int j) { return L - 1 - 2 * j; }
    static constexpr int lb(int j) { return L - 2 - 2 * j; }
    // group layout bits of pass j: (gh, gl) = (hb, lb), or (1, 0) for the lone stage
    static constexpr int gh(int j) { return lb(j) < 0 ? 1 : hb(j); }
    static constexpr int gl(int j) { return lb(j) < 0 ? 0 : lb(j); }
    // base of group g in pass j: g with zero bits inserted at gl and gh = gl + 1
    static __host__ __device__ constexpr uint32_t base(int j, uint32_t g)
    {
        return ((g >> gl(j)) << (gh(j) + 1)) | (g & ((1u << gl(j)) - 1u));
    }
    // position of register e = 2 e1 + e0 of the group
    static __host__ __device__ constexpr uint32_t pos(int j, uint32_t g, int e)
    {
        return base(j, g) + ((uint32_t)(e >> 1) << gh(j)) + ((uint32_t)(e & 1) << gl(j));
    }
};

__host__ __device__ constexpr uint32_t lat_brv(uint32_t x, int bits)
{
    uint32_t r = 0;
    for (int i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}

// Every pass's twiddles of one direction for group g (3 per radix-4 pass, 2
// for the lone stage), loaded up front so that their latency overlaps the
// polynomial's own loads.
template <int PS, bool INV>
struct LatTw {
    using G = LatGeo<PSel<PS>::T::LOGN>;
    static constexpr int L = PSel<PS>::T::LOGN, NP = G::NP;
    uint2 ta[NP], tb[NP][2];
    __device__ __forceinline__ void load(uint32_t g)
    {
        const uint2 *tw = lat_tw<PS, INV>();
        sfor<NP>([&](auto JJ) {
            constexpr int j = decltype(JJ)::value;
            const uint32_t b0 = G::base(j, g);
            if constexpr (G::lb(j) >= 0) ta[j] = tw[(1u << (L - 1 - G::hb(j))) + (b0 >> (G::hb(j) + 1))];
            else ta[j] = make_uint2(0u, 0u);
            const uint32_t kb = (1u << (L - 1 - G::gl(j))) + (b0 >> (G::gl(j) + 1));
            tb[j][0] = tw[kb];
            tb[j][1] = tw[kb + 1];
        });
    }
};

// A thread's groups are slots s = o R + r: operand o (a polynomial with its
// own exchange buffer), group g = t + r T.
template <class G>
__device__ __forceinline__ uint32_t lat_group(uint32_t t, int s)
{
    return t + (uint32_t)(s % G::R) * G::T;
}

// LDS exchange number x (buffer x & 1 of 2 x NB x BUF words, NB >= the
// operands in v, fixed per kernel; consecutive exchanges alternate, so one
// barrier each suffices): slot s's register e goes out at position wmap(g, e)
// of its operand's buffer and comes back from rmap(g, e).
template <class G, int NB, int NS, class WMap, class RMap>
__device__ __forceinline__ void lat_xchg(uint32_t (&v)[NS][4], uint32_t *lds, uint32_t t, int x, WMap wmap, RMap rmap)
{
    static_assert(NS <= NB * G::R, "exchange buffer too small");
    uint32_t *buf = lds + (x & 1) * NB * G::BUF;
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e) buf[(s / G::R) * G::BUF + lat_pad(wmap(lat_group<G>(t, s), e))] = v[s][e];
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[s][e] = buf[(s / G::R) * G::BUF + lat_pad(rmap(lat_group<G>(t, s), e))];
}

// Forward CT passes of every slot (natural-order groups of pass 0 in, the
// last pass's groups out: position pos holds X[brv(pos)], values in [0, 4q)).
// Exchanges 0 .. NP-2.  w[r]: the twiddles of group r.
template <int PS, int NB, int NS>
__device__ __forceinline__ void lat_fwd(uint32_t (&v)[NS][4], const LatTw<PS, false> (&w)[LatGeo<PSel<PS>::T::LOGN>::R],
                                        uint32_t *lds, uint32_t t)
{
    using P = typename PSel<PS>::T;
    using G = LatGeo<P::LOGN>;
    constexpr int NP = G::NP;
    sfor<NP>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const LatTw<PS, false> &W = w[s % G::R];
            if constexpr (G::lb(j) >= 0) {
                // stage hb; the first pass's inputs are the caller's (< 2q): no reduction
                ct_bfly<P::Q, (j > 0)>(v[s][0], v[s][2], W.ta[j].x, W.ta[j].y);
                ct_bfly<P::Q, (j > 0)>(v[s][1], v[s][3], W.ta[j].x, W.ta[j].y);
            }
            ct_bfly<P::Q>(v[s][0], v[s][1], W.tb[j][0].x, W.tb[j][0].y);
            ct_bfly<P::Q>(v[s][2], v[s][3], W.tb[j][1].x, W.tb[j][1].y);
        }
        if constexpr (j + 1 < NP)
            lat_xchg<G, NB>(v, lds, t, j, [&](uint32_t g, int e) { return G::pos(j, g, e); },
                            [&](uint32_t g, int e) { return G::pos(j + 1, g, e); });
    });
}

// Inverse GS passes of one operand (R slots) from the last pass's groups
// (inputs in [0, 2q)) to the natural-order groups g + GN e, the last stage
// scaled by S0 (x + y) and S1 (x - y); canonical outputs.  Exchanges x0 + 1 ..
// x0 + NP - 1.
template <int PS, int NB, uint32_t S0, uint32_t S1>
__device__ __forceinline__ void lat_inv(uint32_t (&v)[LatGeo<PSel<PS>::T::LOGN>::R][4],
                                        const LatTw<PS, true> (&w)[LatGeo<PSel<PS>::T::LOGN>::R], uint32_t *lds,
                                        uint32_t t, int x0)
{
    using P = typename PSel<PS>::T;
    using G = LatGeo<P::LOGN>;
    constexpr int NP = G::NP;
    sfor<NP>([&](auto JJ) {
        constexpr int j = NP - 1 - decltype(JJ)::value;
#pragma unroll
        for (int r = 0; r < G::R; ++r) {
            uint32_t(&u)[4] = v[r];
            gs_bfly<P::Q>(u[0], u[1], w[r].tb[j][0].x, w[r].tb[j][0].y);
            gs_bfly<P::Q>(u[2], u[3], w[r].tb[j][1].x, w[r].tb[j][1].y);
            if constexpr (j > 0 && G::lb(j) >= 0) {
                gs_bfly<P::Q>(u[0], u[2], w[r].ta[j].x, w[r].ta[j].y);
                gs_bfly<P::Q>(u[1], u[3], w[r].ta[j].x, w[r].ta[j].y);
            }
        }
        if constexpr (j > 0)
            lat_xchg<G, NB>(v, lds, t, x0 + NP - j, [&](uint32_t g, int e) { return G::pos(j, g, e); },
                            [&](uint32_t g, int e) { return G::pos(j - 1, g, e); });
    });
    // stage L-1 (k = 1) with the scaling folded in (inv_last_stage)
    constexpr uint32_t S0P = cshoup(S0, P::Q);
    constexpr TwPair S1S = csigned_tw(S1, P::Q);
#pragma unroll
    for (int r = 0; r < G::R; ++r)
#pragma unroll
        for (int e = 0; e < 2; ++e) {
            const uint32_t x = v[r][e], y = v[r][e + 2];
            v[r][e] = csub<P::Q>(shoup_mul<P::Q>(x + y, S0, S0P));
            v[r][e + 2] = csub<P::Q>(sshoup_mul<P::Q>(x - y, S1S.x, S1S.y));
        }
}

template <int PS, bool INV>
__device__ __forceinline__ void lat_tws(LatTw<PS, INV> (&w)[LatGeo<PSel<PS>::T::LOGN>::R], uint32_t t)
{
    using G = LatGeo<PSel<PS>::T::LOGN>;
#pragma unroll
    for (int r = 0; r < G::R; ++r) w[r].load(t + (uint32_t)r * G::T);
}

template <int PS, bool INV, bool BR>
__global__ __launch_bounds__(LatGeo<PSel<PS>::T::LOGN>::T) void k_ntt_lat(const uint32_t *in, uint32_t *out)
{
    using P = typename PSel<PS>::T;
    constexpr int L = P::LOGN;
    using G = LatGeo<L>;
    constexpr int GN = G::GN, NP = G::NP, R = G::R;
    // n = 8192: 2 x 8448 words = 66 KiB, above the 64 KiB of earlier CDNA
    // generations; gfx950 gives a workgroup up to 160 KiB
    static_assert(2 * G::BUF * 4 <= 160 * 1024, "LDS per workgroup (gfx950: 160 KiB)");
    __shared__ uint32_t lds[2 * G::BUF];
    const uint32_t t = threadIdx.x;
    const uint32_t *src = in + (size_t)blockIdx.x * P::N;
    uint32_t *dst = out + (size_t)blockIdx.x * P::N;

    // the polynomial's words: natural order g + GN e (the inverse's
    // bit-reversed-order input: the last forward pass's groups)
    uint32_t v[R][4];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const uint32_t g = t + (uint32_t)r * G::T;
            v[r][e] = ld_in(src + (INV && BR ? G::pos(NP - 1, g, e) : g + GN * e));
        }
    LatTw<PS, INV> w[R];
    lat_tws<PS, INV>(w, t);
    if constexpr (!INV) {
        lat_fwd<PS, 1>(v, w, lds, t);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int e = 0; e < 4; ++e) v[r][e] = canon4<P>(v[r][e]);
        if constexpr (BR) {
            // bit-reversed order is the CT's own: position pos holds X[brv(pos)]
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e) st_out(dst + G::pos(NP - 1, t + (uint32_t)r * G::T, e), v[r][e]);
        } else {
            lat_xchg<G, 1>(v, lds, t, NP - 1, [&](uint32_t g, int e) { return lat_brv(G::pos(NP - 1, g, e), L); },
                           [&](uint32_t g, int e) { return g + GN * e; });
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int e = 0; e < 4; ++e) st_out(dst + t + (uint32_t)r * G::T + GN * e, v[r][e]);
        }
    } else {
        // A[pos] = X[brv(pos)]: a natural-order input reaches the last forward
        // pass's groups through LDS (exchange 0)
        if constexpr (!BR)
            lat_xchg<G, 1>(v, lds, t, 0, [&](uint32_t g, int e) { return lat_brv(g + GN * e, L); },
                           [&](uint32_t g, int e) { return G::pos(NP - 1, g, e); });
        lat_inv<PS, 1, P::NINV, P::C1>(v, w, lds, t, 0);
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int e = 0; e < 4; ++e) st_out(dst + t + (uint32_t)r * G::T + GN * e, v[r][e]);
    }
}

// Small-batch products c = a b mod (x^n + 1, q), one product per workgroup:
// both forwards in the same passes (shared twiddles and barriers), the
// pointwise Montgomery product in the forward's own bit-reversed group layout
// (no reordering exchange either side), the inverse with n^-1 2^32 (the
// Montgomery factor).  BHAT (poly_mul_ntt): b is already transformed, natural
// order, so each thread reads the words of its bit-reversed positions.
// n <= 4096 (one group per thread: both directions' twiddles stay in VGPRs).
template <int PS, bool BHAT>
__global__ __launch_bounds__(LatGeo<PSel<PS>::T::LOGN>::T) void k_poly_mul_lat(const uint32_t *a, const uint32_t *b, uint32_t *c)
{
    using P = typename PSel<PS>::T;
    constexpr int L = P::LOGN;
    using G = LatGeo<L>;
    static_assert(G::R == 1, "latency products: n <= 4096");
    constexpr int GN = G::GN, NP = G::NP, NF = BHAT ? 1 : 2;
    // n = 4096 poly_mul (NF = 2): 4 x 4224 words = 66 KiB (gfx950: up to 160 KiB)
    static_assert(2 * NF * G::BUF * 4 <= 160 * 1024, "LDS per workgroup (gfx950: 160 KiB)");
    __shared__ uint32_t lds[2 * NF * G::BUF];
    const uint32_t t = threadIdx.x;
    const size_t off = (size_t)blockIdx.x * P::N;
    uint32_t v[NF][4], bh[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        v[0][e] = ld_in(a + off + t + GN * e);
        if constexpr (BHAT) bh[e] = ld_in(b + off + lat_brv(G::pos(NP - 1, t, e), L));
        else v[NF - 1][e] = ld_in(b + off + t + GN * e);
    }
    LatTw<PS, false> fw[1];
    LatTw<PS, true> iw[1];
    lat_tws<PS, false>(fw, t);
    lat_tws<PS, true>(iw, t);
    lat_fwd<PS, NF>(v, fw, lds, t);
    uint32_t z[1][4];
#pragma unroll
    for (int e = 0; e < 4; ++e)   // a-hat, b-hat < 4q -> [0, 2q); b-hat from memory < q
        z[0][e] = mont_mul<P>(csub<P::Q2>(v[0][e]), BHAT ? bh[e] : csub<P::Q2>(v[NF - 1][e]));
    // the forward's last exchange was NP - 2: the inverse's first is NP - 1
    lat_inv<PS, NF, P::NINV_R, P::C1_R>(z, iw, lds, t, NP - 2);
#pragma unroll
    for (int e = 0; e < 4; ++e) st_out(c + off + t + GN * e, z[0][e]);
}

}  // namespace qntt
