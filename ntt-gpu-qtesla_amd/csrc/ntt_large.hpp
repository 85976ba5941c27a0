// ntt_large.hpp -- gfx950 fused products for n = 4096 and n = 8192 (param
// sets 3 and 4, p-III's prime): the multi-wave four-step dataflow of SURVEY.md
// 8f row 3 (the reference's alternatives for other sizes are its Stockham
// kernels, NTT.cu:1085-1153 / 1268-1337, and CT2, :667-951).  The standalone
// n = 4096 / 8192 transforms run one wave per polynomial (ntt_big.hpp); a
// product holds two operands, which do not fit one wave's registers at
// n = 8192, so it keeps this split.  Included by ntt_kernels.hip after
// ntt_device.hpp (it owns the __constant__ symbols).
//
// One polynomial is split over G = n/2048 waves of a workgroup; wave B owns
// sub-block B (pos = 2048 B + p').  CT DIT with merged twist, stages on pos
// bits L-1 .. 0 (L = log2 n):
//   * the first g = log2 G stages (pos bits L-1 .. 11) pair sub-block B with
//     sub-block B ^ 2^(g-1-s): in registers from chunked loads plus one LDS
//     exchange (the in-register head; rounds 2-3 ran them as radix-2 stages
//     across waves, one LDS exchange round each, 6-8.5 % slower);
//   * sub-block B is then a 2048-point transform whose twiddles are its own
//     sub-tree of the n-point table, T_B[2^s + m] = psi^brv(2^s (2^g + B) + m):
//     the n = 2048 kernel's passes (register pass, permlane32 stage, LDS
//     transpose, register pass) with per-wave twiddle tables;
//   * the product is taken in that pass-2 layout (both forwards end there,
//     the inverse starts there), so no output all-to-all is needed;
//   * every exchange synchronises only the G waves of its polynomial (SlotSync).
#pragma once
#include "ntt_device.hpp"

namespace qntt {

constexpr int LARGE_PS0 = 3;    // first large-n param set
constexpr int LARGE_NPS = 2;    // n = 4096, 8192
constexpr int LARGE_GMAX = 4;   // waves per polynomial at n = 8192

// uniform pass-1 twiddles (k' < 32) of sub-tree B, [set][fwd/inv][B][k']
__constant__ uint2 c_subtw[LARGE_NPS][2][LARGE_GMAX][32];
// twiddles k = 1 .. G-1 of the cross-wave stages, [set][fwd/inv][k]
__constant__ uint2 c_cross[LARGE_NPS][2][4];
// last sub-tree inverse stage: n^-1 psi^-brv(2^g + B), centred signed pair,
// [set][plain / times 2^32 (the products' Montgomery factor)][B]
__constant__ uint2 c_lastinv[LARGE_NPS][3][LARGE_GMAX];
// bit-5 pairs of every sub-tree [set][fwd/inv][B][32] for kernels that keep
// them out of LDS (Large::BIT5U)
__constant__ uint2 c_bit5L[LARGE_NPS][2][LARGE_GMAX][32];
// LDS images (lane twiddles + bit-5 table) of T_B, [set][fwd/inv][B]; the
// kernels copy the lane twiddles of B = 0 only (shared, see c_fscale) and the
// 32-entry bit-5 table of every B
__device__ uint4 g_tw2imgL[LARGE_NPS][2][LARGE_GMAX][TW2_VEC4];
// Sub-tree twiddles share one table: for every stage b of the 2048-point
// sub-transform T_B[k'] = c_{B,b} T_0[k'] (one constant per (B, b);
// tests/test_oracle_large.py checks it for both sets and directions).  So the
// pass-2 stages (bits 4..0 of the sub-block position) run on T_0's lane
// table for every B once the forward has multiplied register j of the
// pass-2 layout (position 32 Lp + j) by F_B[j] = prod_{bit b of j} c_{B,b}
// (that factor is common to both inputs of every butterfly of the earlier
// stages, so it may enter anywhere before pass 2, and each pass-2 stage b
// then consumes exactly its c_{B,b}); the inverse multiplies by
// G_B[j] = prod_{bit b of j} c'_{B,b} after its pass-2 GS stages, which leave
// every value short of exactly that factor.  Shoup pairs (F, F'),
// [set][fwd/inv][B][j]; B = 0 is all ones and skipped.  Three of the four
// 15.75 KiB LDS images (n = 8192) are freed: 16 waves per workgroup instead of 12.
__constant__ uint2 c_fscale[LARGE_NPS][2][LARGE_GMAX][32];

constexpr int TW2_BIT5_VEC4 = TW2_ENTRIES * 64 * 2 / 4;   // uint4 offset of the bit-5 table in an image

// The fused products hold one operand's 32 transformed words through the
// other's transform, both directions' tables in LDS.  Two table forms:
//   INC (poly_mul, the incomplete domain: residues mod x^8 -+ zeta, the
//     n = 2048 product's BaseMul): pass 2 stops at pos bit 3, so a sub-tree's
//     lane table is only its first MUL_CENT entries (+ its bit-5 table) and
//     every B keeps its own (no shared table, no sub-tree scaling);
//   shared (poly_mul_ntt, b-hat in the full domain): the sub-trees share T_0's
//     lane table and scale by c_fscale (one 15.5 KiB image per direction
//     instead of four: 16 waves per workgroup instead of 12, transforms
//     4.94 / 4.75 -> 4.62 / 4.59 ms per 2^18 polys, profiles/r03/ab_l*_tab.log),
//     and take their bit-5 pairs from __constant__ memory (c_bit5L, a
//     per-lane select of two scalar-loaded candidates), which leaves room for
//     16 waves at 4 per SIMD (4.37 -> 4.19 ms per 2^17, profiles/r04/n).
template <int PS, int MULW, bool INC_>
struct Large {
    using PL = typename PSel<PS>::T;   // the n-point set
    using P = PS2;                     // 2048-point sub-transforms over the same prime
    static_assert(PL::Q == P::Q, "large-n sets use p-III's prime");
    static constexpr int G = (int)(PL::N / 2048);
    static constexpr int LOGG = G == 2 ? 1 : 2;
    static constexpr int WAVES = MULW;
    static constexpr bool INC = INC_;
    static constexpr int INC_ENTRIES = MUL_CENT;
    static_assert(!INC || INC_ENTRIES >= (1 << (5 - MUL_LOGR)) - 1, "the compact table holds every lane entry pass 2 reads");
    static constexpr int CTAB_WORDS = INC_ENTRIES * 64 * 2 + 64;   // compact per-B image
    static constexpr bool SHARED = !INC;
    static constexpr bool BIT5U = !INC;
    static constexpr int OCC = WAVES / 4;
    static constexpr int SLOTS = WAVES / G;   // polynomials per workgroup step
    static constexpr int NT = WAVES * 64;
    static constexpr int IDX = PS - LARGE_PS0;
    static constexpr int TAB_WORDS = INC ? G * CTAB_WORDS : TW2_BIT5_VEC4 * 4;
    static constexpr int NTAB = 2;   // forward table, then the inverse's
    static constexpr int LDS_WORDS = WAVES * XPOSE_WORDS + NTAB * TAB_WORDS + SLOTS + 1;   // + slot counters, poison word
};

// global-order offset of sub-block B's outputs: brv_g(B)
__host__ __device__ constexpr uint32_t brv_g(uint32_t b, int logg) { return logg == 1 ? b : (((b & 1u) << 1) | (b >> 1)); }

// Barrier among the G waves of one polynomial slot (the workgroup holds
// WAVES/G slots).  A workgroup-wide s_barrier would keep all 16 / 12 waves
// in lock step, so every wave of the CU would load, compute and store in the
// same phase; the slot barrier lets the slots drift apart.  Monotonic LDS
// counter per slot: each wave adds 1 (release) and waits (acquire) until
// the slot's G arrivals of this barrier are in.  Measured: n=4096 fwd 5.07
// -> 3.87 ms, n=8192 fwd 5.53 -> 4.71 ms against __syncthreads
// (profiles/r02/s4/large/ab_slotsync_*.log).  The wait is bounded (2^22
// short sleeps, ~0.1 s, far beyond any legitimate wait on partners resident
// on the same CU) so that a broken schedule could never hang the GPU.
//
// An expired wait must not pass silently (the wave would go on with a
// partner's buffer that is not written yet): it sets the workgroup's sticky
// LDS poison word before the wave touches any buffer again, and every wave
// re-reads that word after its last exchange read of a step and before the
// step's stores -- a poisoned workgroup writes the non-canonical sentinel
// 0xFFFFFFFF (>= q) for every remaining coefficient, so any range check on
// the output sees it without a device sync.  A wave whose read saw a
// partner's data of a later step reads the poison word after it, and LDS
// requests of one wave are served in order, so it sees the poison too.  The
// expiry is also counted on the device (ntt_sync_expiries; bench.py fails a
// run whose count is not 0).
#ifndef LARGE_SLOT_SYNC_SPIN
#define LARGE_SLOT_SYNC_SPIN (1u << 22)   // 0 in the test build lib/libqtesla_ntt_syncfail.so: every wait expires
#endif
constexpr uint32_t SYNC_SENTINEL = 0xFFFFFFFFu;
// count of slot-barrier waits that hit the bound (ntt_sync_expiries): 0 unless
// the schedule broke; a launch that adds to it wrote sentinels
__device__ unsigned int g_slot_sync_expired;
struct SlotSync {
    uint32_t *ctr;
    uint32_t *poison;   // the workgroup's sticky poison word
    uint32_t target;
    template <int G>
    __device__ __forceinline__ void wait()
    {
        target += G;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bool arrived = false;
        for (uint32_t spin = 0; spin < (uint32_t)LARGE_SLOT_SYNC_SPIN; ++spin) {
            if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) {
                arrived = true;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (!__builtin_amdgcn_readfirstlane((uint32_t)arrived)) {
            if ((threadIdx.x & 63) == 0) {
                __hip_atomic_store(poison, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                atomicAdd(&g_slot_sync_expired, 1u);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    // after the step's last exchange read: store sentinels from here on?
    __device__ __forceinline__ bool poisoned() const
    {
        return __builtin_amdgcn_readfirstlane(__hip_atomic_load(poison, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) != 0u;
    }
};

// ---- in-register head -------------------------------------------------------
// The g = log2 G stages on pos bits L-1 .. 11 run in registers instead of
// across waves: wave B loads chunk c's words
// 2048 c + (2048/G) B + p (p < 2048/G) at register (32/G) c + j'
// (p = 64 j' + l: G runs of 8/G KiB), so every radix-G group of a lane is
// registers j', 32/G + j', ...; the head's butterflies and twiddles are the
// cross stages' (c_cross).  One exchange then gives wave B its sub-block
// (register (32/G) B' + j' = sub-block word (2048/G) B' + 64 j' + l, the
// pass-1 layout): only the other waves' chunks move, (G-1)/G of the 32
// words, one LDS round trip and two slot barriers in place of the cross
// stages' g round trips of all 32 words and 2g barriers (session 2 of round 3:
// n = 8192 products -8.5 / -6.7 %, profiles/r03/ab_large_head_products.log).
template <class P, int G>
__device__ __forceinline__ void head_fwd(uint32_t (&r)[32], const uint2 *cross)
{
    const uint2 w1 = cross[1];
    if constexpr (G == 2) {
#pragma unroll
        for (int j = 0; j < 16; ++j) ct_bfly<P::Q, false>(r[j], r[16 + j], w1.x, w1.y);   // pos bit 11, inputs < 2q
    } else {
        const uint2 w2 = cross[2], w3 = cross[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // pos bit 12 (k = 1): chunks c, c + 2; inputs < 2q
            ct_bfly<P::Q, false>(r[j], r[16 + j], w1.x, w1.y);
            ct_bfly<P::Q, false>(r[8 + j], r[24 + j], w1.x, w1.y);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // pos bit 11 (k = 2, 3): chunks c, c + 1
            ct_bfly<P::Q>(r[j], r[8 + j], w2.x, w2.y);
            ct_bfly<P::Q>(r[16 + j], r[24 + j], w3.x, w3.y);
        }
    }
}
template <class P, int G>
__device__ __forceinline__ void head_inv(uint32_t (&r)[32], const uint2 *cross)
{
    const uint2 w1 = cross[1];
    if constexpr (G == 4) {
        const uint2 w2 = cross[2], w3 = cross[3];
#pragma unroll
        for (int j = 0; j < 8; ++j) {   // pos bit 11 (k = 2, 3)
            gs_bfly<P::Q>(r[j], r[8 + j], w2.x, w2.y);
            gs_bfly<P::Q>(r[16 + j], r[24 + j], w3.x, w3.y);
        }
    }
    constexpr int H = 16;   // pos bit L-1 (k = 1): chunks c, c + G/2
#pragma unroll
    for (int j = 0; j < H; ++j) gs_bfly<P::Q>(r[j], r[H + j], w1.x, w1.y);
}
// chunk c of wave B <-> chunk B of wave c among the slot's G waves (buffers
// [j][lane], conflict-free; chunk B stays in registers, it does not
// round-trip through LDS); the second wait frees
// the buffers for the next transpose / exchange
template <int G>
__device__ __forceinline__ void head_exchange(uint32_t (&r)[32], uint32_t *mine, const uint32_t *slot_bufs, uint32_t lane,
                                              uint32_t B, SlotSync &ss)
{
    constexpr int C = 32 / G;
#pragma unroll
    for (int c = 0; c < G; ++c)
        if ((uint32_t)c != B)
#pragma unroll
            for (int j = 0; j < C; ++j) mine[(C * c + j) * 64 + lane] = r[C * c + j];
    ss.wait<G>();
#pragma unroll
    for (int c = 0; c < G; ++c)
        if ((uint32_t)c != B) {
            const uint32_t *src = slot_bufs + c * XPOSE_WORDS + B * C * 64 + lane;
#pragma unroll
            for (int j = 0; j < C; ++j) r[C * c + j] = src[j * 64];
        }
    ss.wait<G>();
}

// Position of sub-block output k' in its wave's 8 KiB exchange buffer: the
// rotation by B 32/G words makes both sides conflict-free (ds_*_b32 runs as
// two 32-lane groups, bank = dword mod 32) -- the owner accesses consecutive
// k' per instruction, and 32 consecutive global words g = G k' + brv_g(B)
// hit banks (g / G) + B 32/G: 32 distinct (tests/test_lds_layout.py).
template <int G>
__device__ __forceinline__ uint32_t xch_pos(uint32_t kp, uint32_t B)
{
    return (kp + B * (32u / G)) & 2047u;
}

// The workgroup's twiddle tables of one direction into LDS at `tab`: per B
// the compact image (INC), else T_0's lane image (the bit-5 pairs come from
// __constant__ memory).
template <class LG, bool INV>
__device__ __forceinline__ void fill_large_tw(uint32_t *tab)
{
    uint4 *dst = reinterpret_cast<uint4 *>(tab);
    if constexpr (LG::INC) {   // per B: lane entries 0..2, then the bit-5 table
        constexpr int LV = LG::INC_ENTRIES * 64 * 2 / 4, CV = LG::CTAB_WORDS / 4;
        for (int i = threadIdx.x; i < LG::G * CV; i += LG::NT) {
            const int b = i / CV, o = i % CV;
            dst[i] = g_tw2imgL[LG::IDX][INV ? 1 : 0][b][o < LV ? o : TW2_BIT5_VEC4 + (o - LV)];
        }
        return;
    }
    for (int i = threadIdx.x; i < TW2_BIT5_VEC4; i += LG::NT) dst[i] = g_tw2imgL[LG::IDX][INV ? 1 : 0][0][i];
}

// register j of the pass-2 layout times F_B[j] / G_B[j] (Shoup, output in [0, 2q))
template <class P, class LG, bool INV>
__device__ __forceinline__ void subtree_scale(uint32_t (&r)[32], uint32_t B)
{
    if constexpr (!LG::SHARED) return;
    if (B == 0) return;   // wave-uniform
    const uint2 *f;
#pragma unroll
    for (int j = 0; j < 32; ++j) {
        if ((j & 7) == 0) f = c_fscale[LG::IDX][INV ? 1 : 0][B] + opaque_zero();   // 8 pairs in SGPRs at a time
        r[j] = shoup_mul<P::Q>(r[j], f[j].x, f[j].y);
    }
}

// Per-wave state of the large-n kernels: the wave's sub-block B and slot,
// its exchange buffer, the slot barrier and, per direction, the lane table
// (T_0's when SHARED, else T_B's compact image) and T_B's bit-5 table.
template <class LG>
struct LargeWave {
    using P = typename LG::P;
    using LT = Lane<P>;
    uint32_t *lds, *buf;
    uint32_t wave, B, slot;
    const uint2 *tw2[2], *bit5[2];
    SlotSync ss;
    LT L;
    // fills the tables of directions [D0, D1] and the counters (one __syncthreads)
    template <int D0, int D1>
    __device__ __forceinline__ void init(uint32_t *lds_)
    {
        lds = lds_;
        wave = wave_id();
        B = wave % LG::G;
        slot = wave / LG::G;
        buf = lds + wave * XPOSE_WORDS;
        uint32_t *tab = lds + LG::WAVES * XPOSE_WORDS;
        if constexpr (D0 == 0) table<0>(tab);
        if constexpr (D1 == 1) table<1>(tab + (D0 == 0 ? LG::TAB_WORDS : 0));
        uint32_t *const ctrs = tab + LG::NTAB * LG::TAB_WORDS;
        if (threadIdx.x <= (uint32_t)LG::SLOTS) ctrs[threadIdx.x] = 0;   // slot counters + poison word
        __syncthreads();
        ss = SlotSync{ctrs + slot, ctrs + LG::SLOTS, 0};
    }
    template <int D>
    __device__ __forceinline__ void table(uint32_t *t)
    {
        table_ptrs<D>(t);
        fill_large_tw<LG, D == 1>(t);
    }
    template <int D>
    __device__ __forceinline__ void table_ptrs(uint32_t *t)
    {
        if constexpr (LG::INC) {
            tw2[D] = reinterpret_cast<const uint2 *>(t + B * LG::CTAB_WORDS);
            bit5[D] = tw2[D] + LG::INC_ENTRIES * 64;
        } else {
            tw2[D] = reinterpret_cast<const uint2 *>(t);
            bit5[D] = c_bit5L[LG::IDX][D][B];
        }
    }
    // Re-derive the wave-uniform state from an opaque wave index at the top of
    // every step: otherwise every address, table pointer and branch mask
    // derived from it is hoisted out of the step loop and held for the whole
    // kernel (33 spilled SGPRs in the n = 8192 b-hat product)
    template <int D0, int D1>
    __device__ __forceinline__ void refresh()
    {
        uint32_t wv = wave_id();
        asm volatile("" : "+s"(wv));
        wave = wv;
        B = wv % LG::G;
        slot = wv / LG::G;
        buf = lds + wv * XPOSE_WORDS;
        uint32_t *tab = lds + LG::WAVES * XPOSE_WORDS;
        if constexpr (D0 == 0) table_ptrs<0>(tab);
        if constexpr (D1 == 1) table_ptrs<1>(tab + (D0 == 0 ? LG::TAB_WORDS : 0));
        uint32_t *const ctrs = tab + LG::NTAB * LG::TAB_WORDS;
        ss.ctr = ctrs + slot;
        ss.poison = ctrs + LG::SLOTS;
    }
    // forward of this wave's share (the head's chunked layout, see head_fwd,
    // inputs < 2q; the first g stages run in registers + one exchange) down
    // to the pass-2 layout: register j of lane l holds sub-block output
    // k' = brv5(j) 64 + l of global index G k' + brv_g(B), in [0,4q)
    template <int BMIN = 0>
    __device__ __forceinline__ void fwd(uint32_t (&r)[32])
    {
        constexpr int G = LG::G;
        head_fwd<P, G>(r, c_cross[LG::IDX][0]);
        head_exchange<G>(r, buf, lds + slot * G * XPOSE_WORDS, opaque_lane(), B, ss);
        fwd_pass1_tw<P, true, LG::BIT5U>(r, L.h, c_subtw[LG::IDX][0][B] + opaque_zero(), bit5[0] + opaque_zero());
        lds_p1_to_p2<P>(r, buf, LT(opaque_lane()));   // addresses recomputed (see inv)
        subtree_scale<P, LG, false>(r, B);             // T_B = c_{B,b} T_0 (c_fscale)
        fwd_pass2<P, BMIN>(r, tw2[0] + opaque_zero(), L.lane);
    }
    // contiguous words (global words [2048 B, 2048 B + 2048) at register j of
    // lane l = word 64 j + l) scattered to the owning waves, into the pass-2
    // layout (the buffers must be free).  Position of sub-block output k' in
    // its wave's buffer: xch_pos (conflict-free both ways)
    __device__ __forceinline__ void from_contiguous(uint32_t (&r)[32])
    {
        constexpr int G = LG::G;
        const uint32_t lane = opaque_lane();   // addresses recomputed per step, not hoisted into VGPRs
        {
            const uint32_t bt = brv_g(lane % G, LG::LOGG);   // owner of g (g = lane mod G)
            uint32_t *dst = lds + (slot * G + bt) * XPOSE_WORDS;
            const uint32_t k0 = 2048u / G * B + lane / G;
#pragma unroll
            for (int j = 0; j < 32; ++j) dst[xch_pos<G>(k0 + 64u / G * j, bt)] = r[j];
        }
        ss.template wait<G>();
#pragma unroll
        for (int j = 0; j < 32; ++j) r[j] = buf[xch_pos<G>(brv5(j) * 64 + lane, B)];
    }
    // inverse from the pass-2 layout (inputs < 2q) to this wave's share of
    // the natural order in the head's chunked layout (large_off), [0,2q),
    // scaled by n^-1 (RS: and by 2^32, undoing a Montgomery product's 2^-32)
    // RS 0: plain inverse; 1: also times 2^32 (undoes a Montgomery product's
    // 2^-32); 2: the incomplete-domain product's -- from pos bit BMIN (WIDE0:
    // BaseMul's wide outputs), scaled by (n/2^BMIN)^-1 2^32
    template <int RS, int BMIN = 0, bool WIDE0 = false>
    __device__ __forceinline__ void inv(uint32_t (&r)[32])
    {
        constexpr int G = LG::G;
        constexpr uint32_t NINV = RS == 2 ? LG::PL::template ninv_r<BMIN>() : RS ? LG::PL::NINV_R : LG::PL::NINV;
        constexpr uint32_t NINVP = cshoup(NINV, P::Q);
        inv_pass2<P, BMIN, WIDE0>(r, tw2[1] + opaque_zero(), L.lane);
        subtree_scale<P, LG, true>(r, B);   // the c'_{B,b} the shared table left out (c_fscale)
        // transpose addresses from an opaque lane: recomputed here instead of
        // 8 loop-invariant VGPRs (which spilled at the 128-VGPR budget)
        lds_p2_to_p1<P>(r, buf, LT(opaque_lane()));
        inv_pass1_head<P, LG::BIT5U>(r, L.h, c_subtw[LG::IDX][1][B] + opaque_zero(), bit5[1] + opaque_zero());
        const uint2 last = c_lastinv[LG::IDX][RS][B];
        inv_last_stage<P, false>(r, NINV, NINVP, last.x, last.y);   // [0,2q)
        head_exchange<G>(r, buf, lds + slot * G * XPOSE_WORDS, opaque_lane(), B, ss);   // the head's chunked layout
        head_inv<P, G>(r, c_cross[LG::IDX][1]);
    }
};

// Workgroup b owns polynomials [b SLOTS ppw, (b+1) SLOTS ppw); slot s of a
// step takes waves s G .. s G + G-1.  Every wave runs the workgroup's step
// count (the exchanges hold barriers): slots past the batch recompute the
// workgroup's first polynomial and store nothing.  step(base, valid): base =
// the wave's first global word (uniform); the steps add the lane offset as
// opaque_lane() at every load and store, so the accesses keep the scalar
// base + 32-bit offset form and no 64-bit lane address stays live (or is
// hoisted out of the loop into VGPRs).
template <class LG, class Step>
__device__ __forceinline__ void large_steps(const LargeWave<LG> &w, uint32_t first, uint32_t npoly, uint32_t ppw, Step &step)
{
    const uint32_t steps = (min((uint32_t)LG::SLOTS * ppw, npoly - first) + LG::SLOTS - 1) / LG::SLOTS;
#pragma unroll 1
    for (uint32_t it = 0; it < steps; ++it) {
        const uint32_t poly = first + it * LG::SLOTS + w.slot;
        const bool valid = poly < npoly;
        step((size_t)(valid ? poly : first) * LG::PL::N, valid);
    }
}

// Word offset of register j from a wave's first word in the head's chunks
// (chunk c = j / (32/G) at 2048 c); the wave's first word is (2048/G) B.
template <class LG>
__host__ __device__ constexpr uint32_t large_off(int j)
{
    return 2048u * (uint32_t)(j / (32 / LG::G)) + 64u * (uint32_t)(j % (32 / LG::G));
}
template <class LG>
__device__ __forceinline__ uint32_t large_first(uint32_t B)
{
    return B * (2048u / LG::G);
}

// the step's stores: a poisoned workgroup (expired slot barrier) writes sentinels
template <class LG, class F>
__device__ __forceinline__ void large_store(uint32_t *dst, const LargeWave<LG> &w, F val)
{
    const bool bad = w.ss.poisoned();
#pragma unroll
    for (int j = 0; j < 32; ++j) st_out(dst + large_off<LG>(j), bad ? SYNC_SENTINEL : val(j));
}

// Fused product c = a*b mod (x^n + 1) for n = 4096 / 8192: FWD(a) and FWD(b)
// (or b-hat = poly_ntt(b), natural order, brought to the pass-2 layout by the
// contiguous-load scatter: BHAT) meet in the pass-2 layout, where the
// pointwise Montgomery product is taken; the inverse starts from there (its
// n^-1 scaling carries the 2^32) -- the two forward exchanges and the
// inverse's scatter of a separate pipeline never happen, one HBM read of a
// and b, one write of c.  a, b and c may alias: the G waves of a slot load
// all of a and b before the slot barriers that precede any store.
// poly_mul (not poly_mul_ntt) in the incomplete domain (5.88 -> 4.72 ms per
// 2^17 products, profiles/r04/k)
template <int PS, bool BHAT>
constexpr bool mul_large_inc()
{
    return !BHAT;
}
#ifndef MUL_LARGE_INC_WAVES
#define MUL_LARGE_INC_WAVES 8   // two 8-wave workgroups per CU (78 KiB LDS each): no full-CU drain between workgroups
#endif
template <int PS, bool BHAT>
constexpr int mul_large_waves()
{
    // the incomplete domain's compact tables leave room for two 8-wave
    // workgroups per CU (4 waves per SIMD, 4.92 -> 4.55 ms per 2^20 products,
    // profiles/r04/s); the shared table without its bit-5 pairs for 16 waves
    return mul_large_inc<PS, BHAT>() ? MUL_LARGE_INC_WAVES : 16;
}
template <int PS, bool BHAT>
using LargeMul = Large<PS, mul_large_waves<PS, BHAT>(), mul_large_inc<PS, BHAT>()>;
template <int PS, bool BHAT>
__global__ __launch_bounds__((LargeMul<PS, BHAT>::NT), (LargeMul<PS, BHAT>::OCC))
void k_poly_mul_large(const uint32_t *a, const uint32_t *b, uint32_t *c, uint32_t npoly, uint32_t ppw)
{
    using LG = LargeMul<PS, BHAT>;
    using P = typename LG::P;
    // both operands' loads up front, except for the n = 8192 poly_mul (its
    // b loads follow a's forward: register pressure)
    constexpr bool PF = !(LG::G == 4 && !BHAT);
    __shared__ __attribute__((aligned(16))) uint32_t lds[LG::LDS_WORDS];
    const uint32_t first = blockIdx.x * (LG::SLOTS * ppw);
    if (first >= npoly) return;
    LargeWave<LG> w;
    w.template init<0, 1>(lds);
    auto step = [&](size_t pbase, bool valid) {
        w.template refresh<0, 1>();
        uint32_t ra[32], rb[32];
        // this wave's words: the forward's input layout (large_off), b-hat
        // contiguous (the scatter of from_contiguous)
        const size_t base = pbase + large_first<LG>(w.B), bbase = BHAT ? pbase + w.B * 2048u : base;
        auto boff = [](int j) { return BHAT ? 64u * (uint32_t)j : large_off<LG>(j); };
        // both operands' loads issued up front: b's latency hides behind a's
        // transform (its 32 words are live there either way, as a's are
        // through b's transform)
        load32(ra, a + base + opaque_lane(), [](int j) { return large_off<LG>(j); });
        if (PF) load32(rb, b + bbase + opaque_lane(), boff);
        constexpr int LOGR = LG::INC ? mul_logr<2>() : 0;
        using BM = BaseMul<P, mul_logr<2>()>;
        w.template fwd<LOGR>(ra);
#pragma unroll
        for (int j = 0; j < 32; ++j) asm volatile("" : "+v"(ra[j]));   // phase boundary (register pressure)
        if (!PF) load32(rb, b + bbase + opaque_lane(), boff);
        if constexpr (BHAT) {   // b-hat < 2q
            // the scatter writes the partners' buffers: their forward
            // transposes (lds_p1_to_p2 on their own buffers) must be done
            w.ss.template wait<LG::G>();
            w.from_contiguous(rb);
        }
        else w.template fwd<LOGR>(rb);
        if constexpr (LG::INC) {
            BM::run(ra, rb, w.tw2[0] + opaque_zero(), w.L.lane);
            w.template inv<2, LOGR, BM::WIDE>(ra);
        } else {
#pragma unroll
            for (int j = 0; j < 32; ++j) ra[j] = mont_mul<P>(csub<P::Q2>(ra[j]), csub<P::Q2>(rb[j]));
            w.template inv<1>(ra);
        }
        if (valid) large_store(c + base + opaque_lane(), w, [&](int j) { return csub<P::Q>(ra[j]); });
    };
    large_steps(w, first, npoly, ppw, step);
}

// out[t] = in[brv_L(t)] for n = 4096 / 8192 (L = log2 n), any 32-bit words:
// one 512-thread workgroup per polynomial, coalesced dword loads into LDS at
// swz(p) = p ^ ((p >> (L-5)) & 31), coalesced dword stores read from
// swz(brv(t)).  32 consecutive s (writes) share the XOR term and differ in
// the bank bits; 32 consecutive t (reads) differ only in bits L-1 .. L-5 of
// brv(t), which the XOR term moves into the bank bits: conflict-free both ways.
template <int PS>
__global__ __launch_bounds__(512) void k_bitrev_large(const uint32_t *in, uint32_t *out, uint32_t npoly)
{
    constexpr uint32_t N = PSel<PS>::T::N;
    constexpr int LOGN = PSel<PS>::T::LOGN;
    __shared__ uint32_t x[N];
    auto swz = [](uint32_t p) { return p ^ ((p >> (LOGN - 5)) & 31u); };
#pragma unroll 1
    for (uint32_t poly = blockIdx.x; poly < npoly; poly += gridDim.x) {   // in place: all loads before any store
        const size_t base = (size_t)poly * N;
        uint32_t v[N / 512];
#pragma unroll
        for (uint32_t k = 0; k < N / 512; ++k) v[k] = __builtin_nontemporal_load(in + base + 512 * k + threadIdx.x);
        __syncthreads();   // the previous polynomial's reads of x are done
#pragma unroll
        for (uint32_t k = 0; k < N / 512; ++k) x[swz(512 * k + threadIdx.x)] = v[k];
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < N / 512; ++k) {
            const uint32_t t = 512 * k + threadIdx.x;
            __builtin_nontemporal_store(x[swz(__builtin_bitreverse32(t) >> (32 - LOGN))], out + base + t);
        }
    }
}

}  // namespace qntt
