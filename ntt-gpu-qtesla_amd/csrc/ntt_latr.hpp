// ntt_latr.hpp -- gfx950 transforms with one polynomial per workgroup of
// n / 2^RB threads, 2^RB coefficients per thread and radix-2^RB passes
// (RB = 3: n = 2048 -> 256 threads, 4 waves, each wave loading and storing
// 2 KiB of the polynomial; RB = 4: 128 threads, 2 waves, 4 KiB).
//
// Why: the batch kernels (ntt_device.hpp) give a polynomial to one wave that
// stays resident over 16 of them, and that access pattern's memory-only floor
// is 3.23 ms per 2^20 n = 2048 transforms (0.66 of the HBM peak); the same
// loads, LDS exchanges and stores with one polynomial per short-lived
// workgroup run 2.84 ms (0.75; tools/latr_floor.py, profiles/r06/lat8/), and
// any workgroup that takes two or more polynomials in turn -- even two
// consecutive ones, the next one's loads in flight -- loses that (3.36-3.56
// ms).  The radix-4 latency kernels (ntt_lat.hpp, 1 KiB per wave) spend 6 LDS
// exchanges and barriers per polynomial and run 4.8 ms at 2^20; radix-8
// passes halve the exchanges (L = 11: passes of 3, 3, 3, 2 stages).
//
// Dataflow (L = log2 n, NE = 2^RB words per thread, T = n / NE threads):
//   pass j works on the group of NE positions pos(j, t, e), e = 0..NE-1, that
//   differ in the RB contiguous bits g0(j) .. g0(j)+RB-1 (the group bits), the
//   thread index filling the other L-RB bits in order:
//     full pass:  group bits = its RB stage bits sh .. sh-RB+1 (sh = L-1-RB j)
//     last pass with fewer stages: group bits RB-1 .. 0
//   pass 0's group is t + T e: the coalesced natural-order loads; the last
//   pass's NE t + e.  Stage b (group bit i = b - g0) pairs e with e ^ 2^i; its
//   twiddle is psi^brv(k), k = 2^(L-1-b) + (pos >> (b+1)) (the batch kernels'
//   c_fwd / c_inv tables, NTT.cu:2216-2260's CT with the merged twist), so a
//   stage on group bit i uses 2^(RB-1-i) twiddles per thread at consecutive k.
//   Between passes the NE values go through LDS (RB = 3: double-buffered, one
//   barrier per exchange; RB = 4: one buffer, a second barrier before the next
//   exchange's writes) at offsets linear in e from one per-pass base: word
//   pos + C1 (pos >> 5) + C2 (pos >> 10), the pad multipliers chosen per
//   exchange and direction for the fewest LDS cycles in the 32-lane bank
//   groups (latr_pad; tests/test_latr_dataflow.py checks every exchange).
//   The forward ends with the bit-reversal exchange to natural order (BR:
//   stores the last pass's positions directly); the inverse starts with the
//   reverse one and runs the passes backwards with GS butterflies, the last
//   stage scaled by n^-1 (and psi^-brv(1)).
#pragma once
#include "ntt_lat.hpp"

namespace qntt {

// pad multipliers (C1, C2) of the LDS word pos + C1 (pos >> 5) + C2 (pos >> 10)
// for exchange x: x < NP-1 between passes x and x+1 (forward: written in pass
// x's layout, read in x+1's; inverse the other way round), x = NP-1 the
// bit-reversal exchange (forward: last pass -> natural order; inverse:
// natural order -> last pass).  Found by search over the exchanges' 32-lane
// bank groups (64 banks of 4 B; ds_read_b32 / ds_write_b32 bank = word mod 32)
// for the fewest LDS cycles (a 2-way ds_write_b32 conflict is free, a 4-way
// one doubles it; a 2-way ds_read_b32 doubles it): RB = 3: every read 1-way
// except the inverse's pass 3 -> 2 exchange at n = 2048 / 4096 (2-way); RB =
// 4: every read 1-way; every write at most 2-way.
struct LatPad {
    int c1, c2;
};
constexpr LatPad latr_pad(int L, int RB, bool inv, int x)
{
    if (RB == 3) {
        const int np = (L + 2) / 3;
        if (x == np - 1) return inv ? LatPad{1, 1} : LatPad{1, 0};
        constexpr int F10[] = {4, 2, 1}, I10[] = {0, 4, 2}, F11[] = {0, 4, 3}, I11[] = {0, 2, 2}, F13[] = {0, 4, 2, 1},
                      I13[] = {0, 0, 4, 2};
        const int c = L == 10 ? (inv ? I10 : F10)[x] : L <= 12 ? (inv ? I11 : F11)[x] : (inv ? I13 : F13)[x];
        return LatPad{c, 0};
    }
    // RB = 4 (x = NP-1 the bit-reversal exchange)
    constexpr int F10[] = {2, 1, 0}, I10[] = {1, 2, 1}, F11[] = {2, 1, 1}, I11[] = {1, 2, 1}, I12[] = {0, 2, 1},
                  F13[] = {0, 2, 1, 1}, I13[] = {0, 1, 2, 1};
    if (L == 10) return LatPad{(inv ? I10 : F10)[x], 0};
    if (L == 11) return LatPad{(inv ? I11 : F11)[x], 0};
    if (L == 12) return inv ? LatPad{I12[x], x == 2 ? 1 : 0} : LatPad{F11[x], 0};
    return inv ? LatPad{I13[x], x == 3 ? 1 : 0} : LatPad{F13[x], 0};
}
__host__ __device__ constexpr uint32_t latr_phys(uint32_t pos, LatPad p)
{
    return pos + (uint32_t)p.c1 * (pos >> 5) + (uint32_t)p.c2 * (pos >> 10);
}

#ifndef LATR_JIT_TW
#define LATR_JIT_TW 0   // A/B: load each pass's twiddles after the previous pass's butterflies
#endif

template <int L_, int RB_>
struct LatRGeo {
    static constexpr int L = L_, RB = RB_;
    static constexpr int N = 1 << L;
    static constexpr int NE = 1 << RB;                    // words per thread
    static constexpr int T = N / NE;                      // threads = groups per pass
    static constexpr int NP = (L + RB - 1) / RB;          // passes
    static constexpr bool DB = RB == 3;                   // double-buffered exchanges
    static constexpr int sh(int j) { return L - 1 - RB * j; }                             // highest stage bit of pass j
    static constexpr int sl(int j) { return sh(j) - (RB - 1) > 0 ? sh(j) - (RB - 1) : 0; }  // lowest stage bit
    static constexpr int g0(int j) { return sh(j) >= RB - 1 ? sh(j) - (RB - 1) : 0; }      // lowest group bit
    static constexpr bool has(int j, int i) { return g0(j) + i >= sl(j) && g0(j) + i <= sh(j); }
    // position of register e of thread t in pass j: e inserted at bits g0 .. g0+RB-1
    static __host__ __device__ constexpr uint32_t pos(int j, uint32_t t, int e)
    {
        return ((t >> g0(j)) << (g0(j) + RB)) | ((uint32_t)e << g0(j)) | (t & ((1u << g0(j)) - 1u));
    }
    // words per exchange buffer: the largest padded extent of any exchange
    static constexpr uint32_t buf_words()
    {
        uint32_t m = 0;
        for (int x = 0; x < NP; ++x)
            for (int inv = 0; inv < 2; ++inv) {
                const uint32_t w = latr_phys((uint32_t)N - 1, latr_pad(L, RB, inv, x)) + 1;
                m = w > m ? w : m;
            }
        return m;
    }
    static constexpr uint32_t BUF = buf_words();
    static constexpr uint32_t LDS_WORDS = (DB ? 2 : 1) * BUF;
};

// Every pass's twiddles of one direction for thread t: w[j][slot(i, m)] is
// stage g0(j) + i's twiddle for the e with e >> (i+1) == m.
template <int PS, bool INV, int RB>
struct LatRTw {
    static constexpr int L = PSel<PS>::T::LOGN;
    using G = LatRGeo<L, RB>;
    static constexpr int NS = (1 << RB) - 1;   // twiddles per full pass
    uint2 w[G::NP][NS];
    static constexpr int slot(int i, int m) { return (1 << (RB - 1 - i)) - 1 + m; }
    // (A pass's twiddle indices depend on the thread through t >> g0(j) only:
    // wave-uniform for g0 >= 6, two values per wave for g0 = 5.  Loading
    // those as scalars, selected per lane by v_cndmask, measured no faster:
    // p-III radix-8 fwd / inv 3.60 / 3.74 -> 3.66 / 3.72 ms per 2^20, p-I
    // 1.67 / 1.66 -> 1.74 / 1.71 (profiles/r06/latr/ab9/); the compiler turns
    // the uniform pass-0 indices into scalar loads by itself.)
    // pass j's twiddles; `anchor` (0) is an opaque value the caller derives
    // from the data, so the loads cannot be hoisted above that point
    template <int j>
    __device__ __forceinline__ void load_pass(uint32_t t, uint32_t anchor = 0)
    {
        const uint2 *tw = lat_tw<PS, INV>() + anchor;
        const uint32_t p0 = G::pos(j, t, 0);
        sfor<RB>([&](auto II) {
            constexpr int i = decltype(II)::value;
            if constexpr (G::has(j, i)) {
                constexpr int b = G::g0(j) + i;
                const uint32_t k0 = (1u << (L - 1 - b)) + (p0 >> (b + 1));
                sfor<(1 << (RB - 1 - i))>([&](auto MM) {
                    constexpr int m = decltype(MM)::value;
                    w[j][slot(i, m)] = tw[k0 + m];
                });
            }
        });
    }
    __device__ __forceinline__ void load(uint32_t t)
    {
        sfor<G::NP>([&](auto JJ) { load_pass<decltype(JJ)::value>(t); });
    }
};

// LDS exchange number x: register e goes out at word wbase + woff(e) and
// comes back from rbase + roff(e).  Double-buffered (G::DB): buffer x & 1,
// consecutive exchanges alternate, one barrier each; single buffer: a
// barrier before the writes of every exchange but the first.
template <class G, int NE, class WOff, class ROff>
__device__ __forceinline__ void latr_xchg(uint32_t (&v)[NE], uint32_t *lds, int x, uint32_t wbase, WOff woff,
                                          uint32_t rbase, ROff roff)
{
    uint32_t *buf = lds + (G::DB && (x & 1) ? G::BUF : 0);
    if (!G::DB && x > 0) __syncthreads();
#pragma unroll
    for (int e = 0; e < NE; ++e) buf[wbase + woff(e)] = v[e];
    __syncthreads();
#pragma unroll
    for (int e = 0; e < NE; ++e) v[e] = buf[rbase + roff(e)];
}

// forward CT passes (natural-order groups of pass 0 in; the last pass's
// groups out, position pos holding X[brv(pos)], values in [0, 4q));
// exchanges 0 .. NP-2
// JIT: pass j+1's twiddles are loaded after pass j's butterflies (in flight
// during the exchange), so only one pass's twiddles are live at a time;
// otherwise the caller has loaded every pass's up front.
template <class V>
__device__ __forceinline__ uint32_t latr_anchor(const V &v)
{
    uint32_t a = 0;
    asm volatile("" : "+v"(a) : "v"(v[0]), "v"(v[sizeof(V) / sizeof(v[0]) - 1]));
    return a;
}

template <int PS, int RB, bool ARITH = true, bool JIT = false>
__device__ __forceinline__ void latr_fwd(uint32_t (&v)[1 << RB], LatRTw<PS, false, RB> &W, uint32_t *lds, uint32_t t)
{
    using P = typename PSel<PS>::T;
    using G = LatRGeo<P::LOGN, RB>;
    constexpr int NE = G::NE;
    sfor<G::NP>([&](auto JJ) {
        constexpr int j = decltype(JJ)::value;
        sfor<RB>([&](auto II) {
            constexpr int i = RB - 1 - decltype(II)::value;   // high stage first
            if constexpr (ARITH && G::has(j, i)) {
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    if (e & (1 << i)) continue;
                    const uint2 w = W.w[j][LatRTw<PS, false, RB>::slot(i, e >> (i + 1))];
                    // the very first stage's inputs are the caller's (< 2q): no reduction
                    ct_bfly<P::Q, !(j == 0 && i == RB - 1)>(v[e], v[e | (1 << i)], w.x, w.y);
                }
            }
        });
        if constexpr (ARITH && JIT && j + 1 < G::NP) W.template load_pass<j + 1>(t, latr_anchor(v));
        if constexpr (j + 1 < G::NP) {
            constexpr LatPad pd = latr_pad(G::L, RB, false, j);
            latr_xchg<G>(v, lds, j, latr_phys(G::pos(j, t, 0), pd),
                         [&](int e) { return latr_phys((uint32_t)e << G::g0(j), pd); },
                         latr_phys(G::pos(j + 1, t, 0), pd), [&](int e) { return latr_phys((uint32_t)e << G::g0(j + 1), pd); });
        }
    });
}

// inverse GS passes from the last pass's groups (inputs in [0, 2q)) to pass
// 0's natural-order groups, the last stage scaled by S0 (x + y) and S1
// (x - y); canonical outputs.  Exchanges x0 + 1 .. x0 + NP - 1.
template <int PS, int RB, uint32_t S0, uint32_t S1, bool ARITH = true, bool JIT = false>
__device__ __forceinline__ void latr_inv(uint32_t (&v)[1 << RB], LatRTw<PS, true, RB> &W, uint32_t *lds, uint32_t t,
                                         int x0)
{
    using P = typename PSel<PS>::T;
    using G = LatRGeo<P::LOGN, RB>;
    constexpr int NE = G::NE;
    sfor<G::NP>([&](auto JJ) {
        constexpr int j = G::NP - 1 - decltype(JJ)::value;
        sfor<RB>([&](auto II) {
            constexpr int i = decltype(II)::value;   // low stage first
            if constexpr (ARITH && G::has(j, i) && !(j == 0 && i == RB - 1)) {
#pragma unroll
                for (int e = 0; e < NE; ++e) {
                    if (e & (1 << i)) continue;
                    const uint2 w = W.w[j][LatRTw<PS, true, RB>::slot(i, e >> (i + 1))];
                    gs_bfly<P::Q>(v[e], v[e | (1 << i)], w.x, w.y);
                }
            }
        });
        if constexpr (ARITH && JIT && j > 0) W.template load_pass<j - 1>(t, latr_anchor(v));
        if constexpr (j > 0) {
            constexpr LatPad pd = latr_pad(G::L, RB, true, j - 1);
            latr_xchg<G>(v, lds, x0 + G::NP - j, latr_phys(G::pos(j, t, 0), pd),
                         [&](int e) { return latr_phys((uint32_t)e << G::g0(j), pd); },
                         latr_phys(G::pos(j - 1, t, 0), pd), [&](int e) { return latr_phys((uint32_t)e << G::g0(j - 1), pd); });
        }
    });
    if constexpr (!ARITH) return;
    // stage L-1 (k = 1, group bit RB-1 of pass 0) with the scaling folded in
    constexpr uint32_t S0P = cshoup(S0, P::Q);
    constexpr TwPair S1S = csigned_tw(S1, P::Q);
#pragma unroll
    for (int e = 0; e < NE / 2; ++e) {
        const uint32_t x = v[e], y = v[e + NE / 2];
        v[e] = csub<P::Q>(shoup_mul<P::Q>(x + y, S0, S0P));
        v[e + NE / 2] = csub<P::Q>(sshoup_mul<P::Q>(x - y, S1S.x, S1S.y));
    }
}

// VAR 0: the transform.  Diagnostic variants (tools/ntt_diag.hip only):
// VAR 1 the same loads, LDS exchanges, barriers and stores without twiddles
// or arithmetic (the access pattern's own floor, bench.py
// roofline.pattern_floor_ms); VAR 2 arithmetic, twiddle loads and LDS
// exchanges only (no global data traffic); VAR 3 VAR 1 plus the twiddle loads.
template <int PS, bool INV, bool BR, int RB, int VAR = 0>
__global__ __launch_bounds__((LatRGeo<PSel<PS>::T::LOGN, RB>::T)) void k_ntt_latr(const uint32_t *in, uint32_t *out)
{
    using P = typename PSel<PS>::T;
    constexpr int L = P::LOGN;
    using G = LatRGeo<L, RB>;
    constexpr uint32_t T = G::T;
    constexpr int NE = G::NE, NP = G::NP;
    constexpr bool ARITH = VAR == 0 || VAR == 2;
    // n = 8192 radix-8: 2 x 9216 words = 72 KiB (gfx950: up to 160 KiB per workgroup)
    static_assert(G::LDS_WORDS * 4 <= 160 * 1024, "LDS per workgroup (gfx950: 160 KiB)");
    __shared__ uint32_t lds[G::LDS_WORDS];
    const uint32_t t = threadIdx.x;
    const uint32_t poly = blockIdx.x;
    const uint32_t *src = in + (size_t)poly * P::N;
    uint32_t *dst = out + (size_t)poly * P::N;
    auto store = [&](uint32_t *p, uint32_t x) __attribute__((always_inline)) {
        if constexpr (VAR == 2) asm volatile("" ::"v"(x));
        else st_out(p, x);
    };
    // natural order t + T e (the inverse's bit-reversed-order input: the last
    // forward pass's positions NE t + e)
    uint32_t v[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        if constexpr (VAR == 2) v[e] = (t * NE + e + poly) & 0xFFFFu;   // no global traffic: synthetic words
        else v[e] = ld_in(src + (INV && BR ? NE * t + e : t + T * e));
    }
    LatRTw<PS, INV, RB> W;
    constexpr bool JIT = LATR_JIT_TW;
    if constexpr (ARITH && JIT) W.template load_pass<INV ? NP - 1 : 0>(t);
    else if constexpr (ARITH || VAR == 3) W.load(t);
    if constexpr (VAR == 3)
#pragma unroll
        for (int j = 0; j < NP; ++j)
#pragma unroll
            for (int i = 0; i < LatRTw<PS, INV, RB>::NS; ++i) v[i % NE] ^= W.w[j][i].x ^ W.w[j][i].y;
    if constexpr (!INV) {
        latr_fwd<PS, RB, ARITH, JIT>(v, W, lds, t);
        if constexpr (ARITH)
#pragma unroll
            for (int e = 0; e < NE; ++e) v[e] = canon4<P>(v[e]);
        if constexpr (BR) {
#pragma unroll
            for (int e = 0; e < NE; ++e) store(dst + NE * t + e, v[e]);
        } else {
            // position NE t + e holds X[brv(NE t + e)]: to natural order
            // through LDS, brv(NE t + e) = brv_{L-RB}(t) + brv_RB(e) 2^(L-RB)
            constexpr LatPad pd = latr_pad(L, RB, false, NP - 1);
            const uint32_t bt = __builtin_bitreverse32(t) >> (32 - (L - RB));
            latr_xchg<G>(v, lds, NP - 1, latr_phys(bt, pd),
                         [&](int e) { return latr_phys(lat_brv(e, RB) << (L - RB), pd); }, latr_phys(t, pd),
                         [&](int e) { return latr_phys(T * e, pd); });
#pragma unroll
            for (int e = 0; e < NE; ++e) store(dst + t + T * e, v[e]);
        }
    } else {
        if constexpr (!BR) {
            // A[pos] = X[brv(pos)]: natural-order input to the last forward
            // pass's positions NE t + e through LDS (exchange 0),
            // brv(t + T e) = brv_L(t) + brv_RB(e)
            constexpr LatPad pd = latr_pad(L, RB, true, NP - 1);
            const uint32_t bt = __builtin_bitreverse32(t) >> (32 - L);
            latr_xchg<G>(v, lds, 0, latr_phys(bt, pd), [&](int e) { return latr_phys(lat_brv(e, RB), pd); },
                         latr_phys(NE * t, pd), [&](int e) { return latr_phys(e, pd); });
        }
        latr_inv<PS, RB, P::NINV, P::C1, ARITH, JIT>(v, W, lds, t, BR ? -1 : 0);
#pragma unroll
        for (int e = 0; e < NE; ++e) store(dst + t + T * e, v[e]);
    }
}

}  // namespace qntt
