// ntt_big.hpp -- gfx950 n = 4096 / 8192 transforms with ONE WAVE PER
// POLYNOMIAL (param sets 3 / 4, p-III's prime; SURVEY.md 8f row 3, larger n;
// the reference's alternatives for other sizes are its Stockham kernels,
// NTT.cu:1085-1153 / 1268-1337).  Included by ntt_kernels.hip after
// ntt_large.hpp.
//
// The n = 2048 kernels' geometry, widened: every lane holds R = n/64
// coefficients in VGPRs (64 / 128), so a polynomial never leaves its wave --
// no cross-wave exchange, no slot barrier, no sub-tree scaling.  With
// L = log2 n, M = L - 6 register bits, H = R/2, NC = L - 11 chunk bits
// (tests/test_big_dataflow.py models every map below against the oracle):
//   A   load / pass 1: lane = pos 0..5, register j = pos 6..L-1.  The M CT
//       stages on pos L-1 .. 6 run in registers with wave-uniform twiddles
//       (scalar loads, k < R).
//   bit-5 stage: v_permlane32_swap of registers j, j + H exchanges lane bit 5
//       (pos 5) with register bit M-1 (pos L-1); the butterfly's twiddle
//       depends on the lane half (LDS table of R pairs).  Layout A'': lane =
//       pos 0..4 + pos L-1, register j: bits 0..M-2 = pos 6..L-2, bit M-1 =
//       pos 5.
//   chunks: c = (pos 5 .. 5+NC-1) selects 32 registers j(c, t) =
//       (c >> 1) + 2^(NC-1) t + H (c & 1); each chunk is transposed through the
//       wave's private 8 KiB LDS buffer (b32 writes, the n = 2048 kernels'
//       b128 read side and XOR swizzle, conflict-free both ways) into
//   B   pass 2 / store: lane l with bit i = pos L-1-i, register j' = pos 0..4:
//       the five CT stages on pos 4..0 with per-lane twiddles (the chunk's
//       lane-major LDS table), then natural index brv_L(pos) =
//       brv5(j') 2^(L-5) + brv_NC(c) 64 + l: every store is a lane-contiguous
//       256-B run, chunk by chunk (the stores of chunk c overlap chunk c+1's
//       transpose and arithmetic).
// The inverse runs the mirror image (B loads, GS pass 2 and transposes per
// chunk, the GS bit-5 stage and swap back, the GS stages on pos 6..L-1, the
// last one scaled by n^-1, A stores).
//
// LDS: one workgroup per CU -- WAVES 8 KiB transpose buffers plus the
// direction's table image (31 x 2^NC lane entries + R bit-5 pairs):
//   n = 4096: 16 waves x 8 KiB + 31.75 KiB (4 waves per SIMD, <= 128 VGPRs)
//   n = 8192: BIG_WAVES_8192 x 8 KiB + 63 KiB
#pragma once
#include <utility>

#include "ntt_large.hpp"

namespace qntt {

// Compile-time loop: f(integral_constant<int, 0>) ... f(<N-1>).  The n = 8192
// bodies (128 registers, ~10k instructions) pass LLVM's pragma-unroll
// threshold, and a partly rolled loop indexes the register array at run time
// (scratch memory, ~7x slower, measured); this expansion cannot fail.
template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F &&f, std::integer_sequence<int, I...>)
{
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F &&f)
{
    sfor_impl(f, std::make_integer_sequence<int, N>{});
}

#ifndef BIG_WAVES_8192
#define BIG_WAVES_8192 8   // n = 8192: 128 data VGPRs (217 / 205 in all): 8 waves = 2 per SIMD
#endif

constexpr int BIG_RMAX = 128;
constexpr int BIG_IMG_VEC4_MAX = (TW2_ENTRIES * 64 * 4 + BIG_RMAX) * 2 / 4;   // n = 8192 image, uint4

// wave-uniform pass-1 twiddles k < R, [set][fwd/inv][k] (device conventions)
__constant__ uint2 c_bigtw[LARGE_NPS][2][BIG_RMAX];
// per-workgroup LDS images: lane table [c][e][lane] (e as TW2_ENTRIES), then
// the R bit-5 pairs, [set][fwd/inv]
__device__ uint4 g_bigimg[LARGE_NPS][2][BIG_IMG_VEC4_MAX];

template <int PS, int WV = 0, bool CMP = false>
struct Big {
    using PL = typename PSel<PS>::T;   // the n-point set
    using P = PS2;                     // same prime; butterflies only use Q
    static_assert(PL::Q == P::Q, "large-n sets use p-III's prime");
    static constexpr int L = PL::LOGN;
    static constexpr int M = L - 6;
    static constexpr int R = 1 << M;
    static constexpr int H = R / 2;
    static constexpr int NC = L - 11;
    static constexpr int CH = 1 << NC;
    static constexpr int IDX = PS - LARGE_PS0;
    static constexpr int WAVES = WV ? WV : L == 12 ? 16 : BIG_WAVES_8192;
    static constexpr int NT = WAVES * 64;
    static constexpr int OCC = (WAVES + 3) / 4;                   // waves per SIMD
    static constexpr int LANE_PAIRS = TW2_ENTRIES * 64 * CH;      // lane table
    static constexpr int IMG_WORDS = 2 * (LANE_PAIRS + R);         // + bit-5 table
    static constexpr int IMG_VEC4 = IMG_WORDS / 4;
    static constexpr int LDS_WORDS = WAVES * XPOSE_WORDS + IMG_WORDS;
    // CMP (the products' incomplete domain): per chunk only lane entries
    // 0 .. MUL_CENT-1, then the bit-5 pairs -- TS pairs per chunk, the bit-5
    // pairs at SWO, TAB_WORDS per direction
    static constexpr bool CMP_ = CMP;
    static constexpr int TS = CMP ? MUL_CENT * 64 : TW2_ENTRIES * 64;
    static constexpr int SWO = CMP ? CH * TS : LANE_PAIRS;
    static constexpr int TAB_WORDS = CMP ? 2 * (CH * TS + R) : IMG_WORDS;
    static_assert(IMG_VEC4 <= BIG_IMG_VEC4_MAX, "image size");
    static_assert(LDS_WORDS * 4 <= 160 * 1024, "one workgroup per CU");
    // register of transposition row t of chunk c (layout A'')
    static __host__ __device__ constexpr int creg(int c, int t) { return (c >> 1) + (1 << (NC - 1)) * t + H * (c & 1); }
    // word offset of A'' register j from the lane's base (l & 31) + 2^(L-1) (l >> 5):
    // pos 6..L-2 = register bits 0..M-2, pos 5 = register bit M-1
    static __host__ __device__ constexpr uint32_t aoff(int j) { return ((uint32_t)(j & (H - 1)) << 6) | ((uint32_t)(j >> (M - 1)) << 5); }
    // word offset of B register j' of chunk c from the lane's natural-order base
    static __host__ __device__ constexpr uint32_t boff(int c, int jp)
    {
        return (brv5(jp) << (L - 5)) + ((NC == 2 ? (((c & 1) << 1) | (c >> 1)) : c) << 6);
    }
};

// A'' -> LDS address of transposition row t (b32, conflict-free per 32-lane
// group): the chunk-local position P = (l & 31) + 32 t + 1024 h through the
// n = 2048 swizzle (tests/test_big_dataflow.py::w_addr)
__device__ __forceinline__ uint32_t big_waddr(uint32_t wb, int t)
{
    return (wb ^ xm_of((uint32_t)t)) + 32u * ((uint32_t)t ^ (((uint32_t)t >> 2) & 1u));
}
__device__ __forceinline__ uint32_t big_wbase(uint32_t lane)
{
    const uint32_t h = lane >> 5;
    return ((lane & 31u) ^ (h << 4)) + 1024u * h;
}

// Buffer-resource access (scalar base, one 32-bit VGPR offset, the constant
// part of each offset in an SGPR, `bytes` the bound: accesses past it are
// dropped / read 0; POL: cache policy, 2 = nontemporal).  A region wider than
// the 8 KiB immediate range takes one 64-bit VGPR base per 8 KiB as global
// addresses (ntt_eo.hpp: held across its loop, they spilled).  The one-wave
// n = 8192 kernels measured no faster with them (4.27 / 4.33 against 4.24 /
// 4.27 ms per 2^18, profiles/r06/big8192), nor at 12 waves (4.75 / 5.54 ms:
// 168 VGPRs leave 32 / 171 spilled), so they keep global addresses.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base, uint32_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), (short)0, (int)bytes, 0x00020000);
}
template <int POL = 2>
__device__ __forceinline__ void buf_st(uint32_t v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
    __builtin_amdgcn_raw_buffer_store_b32(v, r, voff, soff, POL);
}
template <int POL = 2>
__device__ __forceinline__ uint32_t buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
    return __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, POL);
}
__device__ __forceinline__ uint2 buf_ld2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff)
{
    const auto x = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return make_uint2(x[0], x[1]);
}

// the R words of a lane at compile-time offsets from one base pointer
template <int NR, class Off>
__device__ __forceinline__ void load32n(uint32_t (&r)[NR], const uint32_t *src, Off off)
{
    sfor<NR>([&](auto J) { r[J] = ld_in(src + off(J)); });
}

// chunk_loop with R registers: workgroup b owns polynomials [b WAVES ppw,
// (b+1) WAVES ppw), its waves take consecutive ones (dispatch-ordered), the
// first polynomial's loads are issued before the table prologue.  The kernels'
// `load` / `process` lambdas are always_inline: the n = 8192 bodies are too
// large for the inliner's heuristics, and an outlined body takes the register
// array by reference (in scratch memory)
template <class BG, class Prologue, class Load, class Process>
__device__ __forceinline__ void big_loop(uint32_t npoly, uint32_t ppw, Prologue &prologue, Load &load, Process &process)
{
    uint32_t r[BG::R];
    uint32_t u = blockIdx.x * (BG::WAVES * ppw) + wave_id();
    if (u < npoly) load(r, u);
    prologue();   // every wave reaches the barrier inside
    if (u >= npoly) return;
    process(r, u);
#pragma unroll 1
    for (uint32_t i = 1; i < ppw; ++i) {
        u += BG::WAVES;
        if (u >= npoly) break;
        load(r, u);
        process(r, u);
    }
}

template <class BG, bool INV>
__device__ __forceinline__ void fill_big_tw(uint32_t *tab)
{
    const uint4 *src = g_bigimg[BG::IDX][INV ? 1 : 0];
    uint4 *dst = reinterpret_cast<uint4 *>(tab);
    if constexpr (BG::TS != TW2_ENTRIES * 64) {   // gather the compact image
        constexpr int CV = BG::TS * 2 / 4, SV = TW2_ENTRIES * 64 * 2 / 4;
        for (int i = threadIdx.x; i < BG::TAB_WORDS / 4; i += BG::NT)
            dst[i] = src[i < BG::CH * CV ? (i / CV) * SV + i % CV : BG::LANE_PAIRS * 2 / 4 + (i - BG::CH * CV)];
        return;
    }
    for (int i = threadIdx.x; i < BG::IMG_VEC4; i += BG::NT) dst[i] = src[i];
}

template <class BG>
__device__ __forceinline__ const uint2 *big_tw(bool inv)
{
    return c_bigtw[BG::IDX][inv ? 1 : 0] + opaque_zero();
}

// forward pass 1: CT stages on pos L-1 .. 6 (register bits M-1 .. 0), twiddle
// k = 2^s + (j >> (M - s)), uniform; inputs < 2q (stage 0 unreduced)
template <class BG>
__device__ __forceinline__ void big_fwd_pass1(uint32_t (&r)[BG::R])
{
    constexpr int M = BG::M;
    sfor<M>([&](auto S) {
        constexpr int s = S, hh = 1 << (M - 1 - s);
        sfor<BG::R / 32>([&](auto B) {
            const uint2 *tw = big_tw<BG>(false);   // <= 16 pairs in SGPRs at a time
            sfor<32>([&](auto J) {
                constexpr int j = 32 * B + J;
                if constexpr ((j & hh) == 0) {
                    const uint2 w = tw[(1 << s) + (j >> (M - s))];
                    ct_bfly<BG::P::Q, (s > 0)>(r[j], r[j + hh], w.x, w.y);
                }
            });
        });
    });
}

// bit-5 stage (forward): swap lane bit 5 with register bit M-1, butterfly
// with twiddle k = 2^M + m + H h from the LDS table `sw`
template <class BG>
__device__ __forceinline__ void big_fwd_bit5(uint32_t (&r)[BG::R], const uint2 *sw, uint32_t h)
{
    sfor<BG::H>([&](auto Mi) {
        constexpr int m = Mi;
        const auto pr = __builtin_amdgcn_permlane32_swap(r[m], r[m + BG::H], false, false);
        r[m] = pr[0];
        r[m + BG::H] = pr[1];
        const uint2 w = sw[m + BG::H * h];
        ct_bfly<BG::P::Q>(r[m], r[m + BG::H], w.x, w.y);
    });
}

// Forward from layout A (registers r, inputs < 2q): pass 1, the bit-5 stage
// and, chunk by chunk, the transpose to layout B and the pass-2 stages on pos
// 4 .. BMIN (BMIN > 0 stops short, the products' incomplete domain);
// sink(C, v) takes chunk C's 32 B-layout registers, in [0, 4q).
template <class BG, int BMIN, class Sink>
__device__ __forceinline__ void big_fwd(uint32_t (&r)[BG::R], uint32_t *buf, const uint2 *tab, uint32_t h, uint32_t lane,
                                        Sink &&sink)
{
    using P = typename BG::P;
    big_fwd_pass1<BG>(r);
    big_fwd_bit5<BG>(r, tab + BG::SWO + opaque_zero(), h);
    sfor<BG::CH>([&](auto C) {
        constexpr int c = C;
        // transpose addresses recomputed per chunk from an opaque lane
        // (not 16 loop-invariant address VGPRs)
        const uint32_t wb = big_wbase(opaque_lane());
        const Lane<P> LB(opaque_lane());   // the n = 2048 b128 read side (Lp = brv6(lane))
        sfor<32>([&](auto T) { buf[big_waddr(wb, T)] = r[BG::creg(c, T)]; });
        compiler_fence();
        uint32_t v[32];
        sfor<8>([&](auto Q) {
            const uint4 x = *reinterpret_cast<const uint4 *>(buf + LB.rbase + ((4u * Q) ^ LB.rxm));
            v[4 * Q + 0] = x.x;
            v[4 * Q + 1] = x.y;
            v[4 * Q + 2] = x.z;
            v[4 * Q + 3] = x.w;
        });
        compiler_fence();
        fwd_pass2<P, BMIN>(v, tab + BG::TS * c + opaque_zero(), lane);
        sink(C, v);
    });
}

// Inverse to layout A, stored at dst (the polynomial's first word): chunk by
// chunk source(C, v) gives the 32 B-layout registers (inputs of the stage on
// pos BMIN, WIDE0: inv_pass2's wide first stage), GS pass 2 and the transpose
// back; then the GS bit-5 stage and swap, the GS stages on pos 6 .. L-2 and
// the last one scaled by S0 (x + y) and S1 (x - y), canonical.
// store(J, x) takes layout-A register J's canonical result (big_inv: at
// dpoly + 64 J + lane; ntt_eo.hpp: one parity of an n = 8192 polynomial).
template <class BG, int BMIN, bool WIDE0, uint32_t S0, uint32_t S1V, class Source, class Store>
__device__ __forceinline__ void big_inv_to(uint32_t (&r)[BG::R], uint32_t *buf, const uint2 *tab, uint32_t h, uint32_t lane,
                                           Source &&source, Store &&store)
{
    using P = typename BG::P;
    constexpr int M = BG::M, H = BG::H;
    sfor<BG::CH>([&](auto C) {
        constexpr int c = C;
        const uint32_t wb = big_wbase(opaque_lane());   // per chunk (see big_fwd)
        const Lane<P> LB(opaque_lane());
        uint32_t v[32];
        source(C, v);
        inv_pass2<P, BMIN, WIDE0>(v, tab + BG::TS * c + opaque_zero(), lane);
        sfor<8>([&](auto Q) {
            *reinterpret_cast<uint4 *>(buf + LB.rbase + ((4u * Q) ^ LB.rxm)) =
                make_uint4(v[4 * Q + 0], v[4 * Q + 1], v[4 * Q + 2], v[4 * Q + 3]);
        });
        compiler_fence();
        sfor<32>([&](auto T) { r[BG::creg(c, T)] = buf[big_waddr(wb, T)]; });
        compiler_fence();
    });
    // bit-5 stage: GS with the lane-half twiddle, then swap back
    const uint2 *sw = tab + BG::SWO + opaque_zero();
    sfor<H>([&](auto Mi) {
        constexpr int m = Mi;
        const uint2 w = sw[m + H * h];
        gs_bfly<P::Q>(r[m], r[m + H], w.x, w.y);
        const auto pr = __builtin_amdgcn_permlane32_swap(r[m], r[m + H], false, false);
        r[m] = pr[0];
        r[m + H] = pr[1];
    });
    // GS stages on pos 6 .. L-2 (register bits 0 .. M-2), uniform twiddles
    sfor<M - 1>([&](auto JB) {
        constexpr int jb = JB, hh = 1 << jb, s = M - 1 - jb;
        sfor<BG::R / 32>([&](auto B) {
            const uint2 *tw = big_tw<BG>(true);   // <= 16 pairs in SGPRs at a time
            sfor<32>([&](auto J) {
                constexpr int j = 32 * B + J;
                if constexpr ((j & hh) == 0) {
                    const uint2 w = tw[(1 << s) + (j >> (jb + 1))];
                    gs_bfly<P::Q>(r[j], r[j + hh], w.x, w.y);
                }
            });
        });
    });
    // last stage (pos L-1): x' = (x + y) S0, y' = (x - y) S1 (S1 = S0 psi^-brv(1))
    constexpr uint32_t S0P = cshoup(S0, P::Q);
    constexpr TwPair S1 = csigned_tw(S1V, P::Q);
    sfor<H>([&](auto J) {
        constexpr int j = J;
        const uint32_t x = r[j], y = r[j + H];
        store(J, csub<P::Q>(shoup_mul<P::Q>(x + y, S0, S0P)));
        store(std::integral_constant<int, j + H>{}, csub<P::Q>(sshoup_mul<P::Q>(x - y, S1.x, S1.y)));
    });
}
template <class BG, int BMIN, bool WIDE0, uint32_t S0, uint32_t S1V, class Source>
__device__ __forceinline__ void big_inv(uint32_t (&r)[BG::R], uint32_t *buf, const uint2 *tab, uint32_t h, uint32_t lane,
                                        Source &&source, uint32_t *dpoly)
{
    // layout A stores: lane-contiguous 256-B runs
    uint32_t lo = lane;
    asm volatile("" : "+v"(lo));
    uint32_t *const dst = dpoly + lo;
    big_inv_to<BG, BMIN, WIDE0, S0, S1V>(r, buf, tab, h, lane, source, [&](auto J, uint32_t x) __attribute__((always_inline)) {
        st_out(dst + 64u * (uint32_t)J, x);
    });
}

// register pins: the values are taken as redefined here, so the scheduler
// keeps the phases on either side apart (register pressure)
template <int NR>
__device__ __forceinline__ void pin(uint32_t (&r)[NR])
{
#pragma unroll
    for (int j = 0; j < NR; ++j) asm volatile("" : "+v"(r[j]));
}

// layout A loads: natural order, 256-B runs
template <class BG>
__device__ __forceinline__ void big_load_a(uint32_t (&r)[BG::R], const uint32_t *src, uint32_t lane)
{
    uint32_t lo = lane;
    asm volatile("" : "+v"(lo));
    load32n<BG::R>(r, src + lo, [](int j) { return 64u * (uint32_t)j; });
}

// layout B of every chunk (the forward's store order), in the chunk's register slots j(c, j')
template <class BG>
__device__ __forceinline__ void big_load_b(uint32_t (&r)[BG::R], const uint32_t *src, uint32_t lane)
{
    uint32_t lo = lane;
    asm volatile("" : "+v"(lo));
    sfor<BG::CH>([&](auto C) { sfor<32>([&](auto JP) { r[BG::creg(C, JP)] = ld_in(src + lo + BG::boff(C, JP)); }); });
}

// layout A'' words at their own positions: the bit-reversed NTT-domain order
// (position pos holds X[brv(pos)]), two 128-B runs per instruction
template <class BG>
__device__ __forceinline__ uint32_t big_a2_lane(uint32_t lane)
{
    uint32_t lo = (lane & 31u) + ((lane >> 5) << (BG::L - 1));
    asm volatile("" : "+v"(lo));
    return lo;
}

// Forward, natural-order input.  BR = false: natural-order output (layout B
// stores); BR = true (poly_ntt_bitrev): out[t] = X[brv(t)] in one launch --
// after pass 2 each chunk goes back through the wave's LDS buffer to layout
// A'' (the inverse's transpose) and is stored at its own positions.
template <int PS, bool BR>
__global__ __launch_bounds__(Big<PS>::NT, Big<PS>::OCC) void k_ntt_fwd_big(const uint32_t *in, uint32_t *out, uint32_t npoly,
                                                                        uint32_t ppw)
{
    using BG = Big<PS>;
    using P = typename BG::P;
    constexpr uint32_t N = BG::PL::N;
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::LDS_WORDS];
    uint32_t *const tabw = lds + BG::WAVES * XPOSE_WORDS;
    auto prologue = [&]() {
        fill_big_tw<BG, false>(tabw);
        __syncthreads();
    };
    const uint32_t lane = threadIdx.x & 63, h = lane >> 5;
    uint32_t *const buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint2 *const tab = reinterpret_cast<const uint2 *>(tabw);
    auto load = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) { big_load_a<BG>(r, in + (size_t)u * N, lane); };
    auto process = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        if constexpr (!BR) {
            uint32_t lo = lane;   // opaque per unit: scalar base + 32-bit lane offset stores
            asm volatile("" : "+v"(lo));
            uint32_t *const dst = out + (size_t)u * N + lo;
            // every store is a lane-contiguous 256-B run, chunk by chunk (the
            // stores of chunk c overlap chunk c+1's transpose and arithmetic)
            big_fwd<BG, 0>(r, buf, tab, h, lane, [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
                sfor<32>([&](auto JP) { st_out(dst + BG::boff(C, JP), canon4<P>(v[JP])); });
            });
        } else {
            uint32_t *const dst = out + (size_t)u * N + big_a2_lane<BG>(lane);
            big_fwd<BG, 0>(r, buf, tab, h, lane, [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
                constexpr int c = C;
                const uint32_t wb = big_wbase(opaque_lane());
                const Lane<P> LB(opaque_lane());
                sfor<8>([&](auto Q) {
                    *reinterpret_cast<uint4 *>(buf + LB.rbase + ((4u * Q) ^ LB.rxm)) =
                        make_uint4(canon4<P>(v[4 * Q + 0]), canon4<P>(v[4 * Q + 1]), canon4<P>(v[4 * Q + 2]),
                                   canon4<P>(v[4 * Q + 3]));
                });
                compiler_fence();
                sfor<32>([&](auto T) { st_out(dst + BG::aoff(BG::creg(c, T)), buf[big_waddr(wb, T)]); });
                compiler_fence();   // the next chunk's transpose rewrites buf
            });
        }
    };
    big_loop<BG>(npoly, ppw, prologue, load, process);
}

// Inverse, natural-order output.  BR = false: natural-order input (layout
// B loads); BR = true (poly_invntt_bitrev, input in[t] = X[brv(t)]): layout
// A'' loads from the words' own positions, each chunk transposed to layout B
// through the wave's LDS buffer (the forward's transpose) before GS pass 2.
template <int PS, bool BR>
__global__ __launch_bounds__(Big<PS>::NT, Big<PS>::OCC) void k_ntt_inv_big(const uint32_t *in, uint32_t *out, uint32_t npoly,
                                                                        uint32_t ppw)
{
    using BG = Big<PS>;
    constexpr uint32_t N = BG::PL::N;
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::LDS_WORDS];
    uint32_t *const tabw = lds + BG::WAVES * XPOSE_WORDS;
    auto prologue = [&]() {
        fill_big_tw<BG, true>(tabw);
        __syncthreads();
    };
    const uint32_t lane = threadIdx.x & 63, h = lane >> 5;
    uint32_t *const buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint2 *const tab = reinterpret_cast<const uint2 *>(tabw);
    auto load = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        if constexpr (!BR) {
            big_load_b<BG>(r, in + (size_t)u * N, lane);
        } else {
            load32n<BG::R>(r, in + (size_t)u * N + big_a2_lane<BG>(lane), [](int j) { return BG::aoff(j); });
        }
    };
    auto process = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        auto source = [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
                if constexpr (!BR) {
                    sfor<32>([&](auto JP) { v[JP] = r[BG::creg(C, JP)]; });
                } else {
                    constexpr int c = C;
                    const uint32_t wb = big_wbase(opaque_lane());
                    const Lane<typename BG::P> LB(opaque_lane());
                    sfor<32>([&](auto T) { buf[big_waddr(wb, T)] = r[BG::creg(c, T)]; });
                    compiler_fence();
                    sfor<8>([&](auto Q) {
                        const uint4 x = *reinterpret_cast<const uint4 *>(buf + LB.rbase + ((4u * Q) ^ LB.rxm));
                        v[4 * Q + 0] = x.x;
                        v[4 * Q + 1] = x.y;
                        v[4 * Q + 2] = x.z;
                        v[4 * Q + 3] = x.w;
                    });
                    compiler_fence();
                }
        };
        big_inv<BG, 0, false, BG::PL::NINV, BG::PL::C1>(r, buf, tab, h, lane, source, out + (size_t)u * N);
    };
    big_loop<BG>(npoly, ppw, prologue, load, process);
}

// Fused products with one wave per polynomial (n = 4096; n = 8192's operands
// do not fit one wave's registers and stay on k_poly_mul_large):
//   poly_mul (BHAT false): FWD(a) and FWD(b) down to residues mod x^8 -+ zeta
//     (big_fwd stopping at pos bit LOGR, layout B kept in registers), the
//     residue products chunk by chunk (BaseMul, the n = 2048 product's), and
//     the inverse from pos bit LOGR; (n/8)^-1 and the REDC's 2^32 in the last
//     stage's constants.
//   poly_mul_ntt (BHAT true): b-hat = poly_ntt(b) read in the forward's
//     store order (layout B), the complete FWD(a), one Montgomery product per
//     coefficient, the inverse with n^-1 2^32.
// a, b and c may alias: a wave loads its polynomial's a and b before it
// stores any c.  poly_mul_ntt: BIG_MUL_WAVES transpose buffers (8 KiB each)
// and both directions' tables (2 x 31.5 KiB) in LDS; poly_mul: 4 buffers and
// both compact tables (2 x 3.5 KiB), two workgroups per CU, so a CU never
// drains to its last wave at a workgroup boundary (4.45 -> 4.10 ms per 2^18,
// profiles/r04/u).  The register phases are pinned apart (pin), without which
// the scheduler interleaves a's forward with b's.  b-hat's loads are issued
// before a's forward (poly_mul_ntt 3.64 -> 3.55 ms), b's are not (poly_mul
// 4.24 -> 4.39 when they are, profiles/r04/g/ab_m4096.log).
// Measured per 2^18 products (profiles/r04/f/ab_m4096.log): poly_mul 5.75 ms
// (the multi-wave k_poly_mul_large) -> 4.82 (12 waves) -> 4.49 (8 waves);
// poly_mul_ntt 4.20 -> 3.90 -> 3.67.
#ifndef BIG_MUL_WAVES
#define BIG_MUL_WAVES 8   // 2 per SIMD, 0 spills (12 waves = 3 per SIMD: 27 VGPRs spilled, 7 % slower)
#endif
template <bool BHAT>
constexpr int big_mul_waves()
{
    return !BHAT ? 4 : BIG_MUL_WAVES;
}
template <int PS, bool BHAT>
using BigMul = Big<PS, big_mul_waves<BHAT>(), !BHAT>;
template <int PS, bool BHAT>
__global__ __launch_bounds__((BigMul<PS, BHAT>::NT), 2) void k_poly_mul_big(
    const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t npoly, uint32_t ppw)
{
    using BG = BigMul<PS, BHAT>;
    using P = typename BG::P;
    using PL = typename BG::PL;
    constexpr int LOGR = mul_logr<2>();   // p-III's prime: the n = 2048 product's residues
    using BM = BaseMul<P, LOGR>;
    static_assert(!BG::CMP_ || MUL_CENT >= (1 << (5 - LOGR)) - 1, "the compact table holds every lane entry pass 2 reads");
    constexpr uint32_t N = PL::N;
    static_assert(BG::WAVES * XPOSE_WORDS + 2 * BG::TAB_WORDS <= 160 * 256, "one workgroup per CU");
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::WAVES * XPOSE_WORDS + 2 * BG::TAB_WORDS];
    uint32_t *const tabfw = lds + BG::WAVES * XPOSE_WORDS, *const tabiw = tabfw + BG::TAB_WORDS;
    auto prologue = [&]() {
        fill_big_tw<BG, false>(tabfw);
        fill_big_tw<BG, true>(tabiw);
        __syncthreads();
    };
    const uint32_t lane = threadIdx.x & 63, h = lane >> 5;
    uint32_t *const buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint2 *const ftab = reinterpret_cast<const uint2 *>(tabfw);
    const uint2 *const itab = reinterpret_cast<const uint2 *>(tabiw);
    auto load = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) { big_load_a<BG>(r, a + (size_t)u * N, lane); };
    auto process = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        const size_t base = (size_t)u * N;
        auto keep = [&](uint32_t (&x)[BG::R]) __attribute__((always_inline)) {
            return [&x](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) { sfor<32>([&](auto JP) { x[BG::creg(C, JP)] = v[JP]; }); };
        };
        uint32_t rb[BG::R];
        if constexpr (!BHAT) {
            big_fwd<BG, LOGR>(r, buf, ftab, h, lane, keep(r));
            pin(r);   // phase boundary: nothing of b's forward moves above it
            big_load_a<BG>(rb, b + base, lane);   // 64 fewer live VGPRs through a's forward
            big_fwd<BG, LOGR>(rb, buf, ftab, h, lane, keep(rb));
            pin(rb);
            big_inv<BG, LOGR, BM::WIDE, PL::template ninv_r<LOGR>(), PL::template c1_r<LOGR>()>(
                r, buf, itab, h, lane,
                [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
                    constexpr int cc = C;
                    uint32_t vb[32];
                    sfor<32>([&](auto JP) {
                        v[JP] = r[BG::creg(cc, JP)];
                        vb[JP] = rb[BG::creg(cc, JP)];
                    });
                    BM::run(v, vb, ftab + BG::TS * cc + opaque_zero(), lane);
                },
                c + base);
        } else {
            big_load_b<BG>(rb, b + base, lane);   // b-hat in the forward's store order, before a's forward
            big_fwd<BG, 0>(r, buf, ftab, h, lane, keep(r));
            pin(r);
            big_inv<BG, 0, false, PL::NINV_R, PL::C1_R>(
                r, buf, itab, h, lane,
                [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
                    sfor<32>([&](auto JP) {
                        v[JP] = mont_mul<P>(csub<P::Q2>(r[BG::creg(C, JP)]), csub<P::Q2>(rb[BG::creg(C, JP)]));
                    });
                },
                c + base);
        }
    };
    big_loop<BG>(npoly, ppw, prologue, load, process);
}

}  // namespace qntt
