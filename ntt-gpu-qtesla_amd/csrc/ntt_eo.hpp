// ntt_eo.hpp -- EXPERIMENT (A/B builds with -DNTT_EO only; not in the
// product library): gfx950 n = 8192 transforms as two n = 4096 halves (param
// set 4 over p-III's prime), a PAIR of waves per polynomial, wave parity
// `par` taking the words x[2i + par].
//
// Idea: the one-wave-per-polynomial n = 8192 kernels (ntt_big.hpp) hold 128
// words per lane at 2 waves/SIMD (0.54 of the HBM peak); the n = 4096 ones,
// 64 words at 4 waves/SIMD, reach 0.60.  The forward CT stages on pos bits
// 12..1 never mix the parity classes and their twiddles psi_8192^brv13(k),
// k < 4096, are psi_4096^brv12(k) (psi_8192^2 = psi_4096 over the same
// prime), so (even/odd decomposition, tests/test_eo_dataflow.py)
//   A = NTT_4096(x[2i]),  B = NTT_4096(x[2i+1])   (natural order)
//   X[k] = A[k] + w_k B[k],  X[k + 4096] = A[k] - w_k B[k],  w_k = psi_8192^(2k+1).
// Each wave runs big_fwd<Big<3>> on its parity (stride-2 buffer loads); per
// chunk the pair exchanges its B-layout words through the two waves' LDS
// buffers and each wave runs 16 of the final butterflies (256-B stores of
// X[k], X[k + 4096]).  The inverse mirrors it (GS combine first, each wave
// half of it, then big_inv_to with n_8192^-1 in the last stage, stride-2
// stores).  16-wave workgroups, the n = 4096 kernels' LDS; the pair
// synchronises through LDS step counters (eo_signal / eo_wait), not
// workgroup barriers.
//
// Measured (profiles/r06/eo, p-III-8192, 2^18 polynomials in place, bit-exact
// against the product library): product 4.03-4.07 / 3.99 ms fwd / inv;
// workgroup barriers 5.22 / - ms; pair counters 5.14 / 4.94; + normal cache
// policy on the stride-2 accesses 4.92 / 4.17; + the split twiddle (EO_TWJIT)
// 4.58-4.64 / 4.03.  A timing-only variant with contiguous (wrong) loads
// still took 4.18 ms forward: the exchange, the pair's step waits and the
// combine cost more than 4 waves/SIMD recover, so the product keeps
// k_ntt_fwd_big<4> / k_ntt_inv_big<4>.
#pragma once
#include "ntt_big.hpp"

#ifdef NTT_EO
namespace qntt {

// w_k = psi_8192^(2k+1) (CT index 4096 + brv12(k)) for natural k < 4096,
// [fwd / inv][k] in the device conventions (dev_pair)
__device__ uint2 g_eotw[2][4096];
// EO_TWJIT: w_k = lambda_l mu with lambda_l = psi^(2 l) per lane (Shoup pair,
// [fwd / inv]) and mu = psi^(2 k0 + 1), k0 = k - l, wave-uniform (device
// convention, [fwd / inv][parity][chunk][I]): one more Shoup product per
// butterfly instead of a per-lane table load
#ifndef EO_TWJIT
#define EO_TWJIT 1   // the per-lane table loads instead: +0.28 / +0.14 ms per 2^18 fwd / inv (profiles/r06/eo)
#endif
__constant__ uint2 c_eolam[2][64];
__constant__ uint2 c_eomu[2][2][2][16];

struct EO {
    using BG = Big<3>;                    // the n = 4096 half: geometry, tables, registers
    using P = typename BG::P;
    using P8 = typename PSel<4>::T;
    static_assert(cpow(P8::PSI, 2, P8::Q) == PSel<3>::T::PSI, "psi_8192^2 = psi_4096");
    static constexpr uint32_t N = 8192, HN = 4096;
    static constexpr int NPAIR = BG::WAVES / 2;
    // the n = 4096 inverse's last-stage constants with n_8192^-1 (the
    // combine's factor 1/2 folded in): S0 = 8192^-1, S1 = S0 psi_4096^-brv12(1)
    static constexpr uint32_t S0 = P8::NINV;
    static constexpr uint32_t S1 = (uint32_t)((uint64_t)P8::NINV * cpow(PSel<3>::T::PSI_INV, 2048, P8::Q) % P8::Q);
    // natural index k of B-layout register j' of chunk c, lane l: boff(c, j') + l;
    // for j' = i + 16 h: boff(c, i) + 128 h (bit 4 of j' is bit 0 of brv5(j'))
    static_assert(BG::boff(0, 16) == BG::boff(0, 0) + 128 && BG::boff(1, 31) == BG::boff(1, 15) + 128, "own-half offset");
};

// The pair's exchange goes through the waves' LDS transpose buffers (rows
// of 64 lane-contiguous words, conflict-free), synchronised within the pair
// only: each wave counts its exchange steps in an LDS word (eo_signal) and
// waits for its partner's (eo_wait) -- a workgroup barrier would hold all 16
// waves in lock step (measured 29 % slower).  LDS operations of a wave
// complete in order, and the signal first waits for this wave's LDS writes
// (lgkmcnt 0).  The wait is bounded (~2^20 sleeps, tens of ms): a broken
// protocol gives wrong results, never a hung GPU.
__device__ __forceinline__ void eo_signal(uint32_t *flag, uint32_t v)
{
    compiler_fence();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0); vmcnt, expcnt unconstrained
    __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    compiler_fence();
}
__device__ __forceinline__ void eo_wait(const uint32_t *flag, uint32_t v)
{
    compiler_fence();
#pragma unroll 1
    for (uint32_t i = 0; i < (1u << 20); ++i) {
        const uint32_t f = __hip_atomic_load(const_cast<uint32_t *>(flag), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(f) >= v) break;
        __builtin_amdgcn_s_sleep(1);
    }
    compiler_fence();
}

// cache policy: 2 = nontemporal.  The stride-2 accesses (one parity of a
// polynomial) share every cache line with the partner wave
#ifndef EO_POL_S2
#define EO_POL_S2 0   // normal; 2 (nontemporal) costs +0.18 / +0.86 ms per 2^18 fwd / inv (profiles/r06/eo)
#endif
#ifndef EO_POL_C
#define EO_POL_C 2
#endif

__global__ __launch_bounds__(EO::BG::NT, EO::BG::OCC) void k_ntt_fwd_eo(const uint32_t *in, uint32_t *out, uint32_t npoly,
                                                                      uint32_t ppw)
{
    using BG = EO::BG;
    using P = EO::P;
    static_assert((BG::LDS_WORDS + BG::WAVES) * 4 <= 160 * 1024, "one workgroup per CU");
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::LDS_WORDS + BG::WAVES];
    uint32_t *const tabw = lds + BG::WAVES * XPOSE_WORDS;
    const uint2 *const tab = reinterpret_cast<const uint2 *>(tabw);
    const uint32_t lane = threadIdx.x & 63, h = lane >> 5;
    const uint32_t w = wave_id(), par = w & 1u;
    uint32_t *const buf = lds + w * XPOSE_WORDS;
    uint32_t *const abuf = lds + (w & ~1u) * XPOSE_WORDS, *const bbuf = abuf + XPOSE_WORDS;
    const uint32_t own = 1024u * par + lane;   // row 16 par, this lane
    uint32_t *const myflag = lds + BG::LDS_WORDS + w;
    const uint32_t *const pflag = lds + BG::LDS_WORDS + (w ^ 1u);
    *myflag = 0;
    uint32_t step = 0;   // exchange steps signalled so far (the pair's common count)
    uint32_t p = blockIdx.x * (EO::NPAIR * ppw) + (w >> 1);
    uint32_t r[BG::R];
    // this wave's parity, x[2 (64 j + lane) + par], zeros past the batch
    auto load = [&](uint32_t q) __attribute__((always_inline)) {
        uint32_t lo = 2u * lane + par;
        asm volatile("" : "+v"(lo));
        const auto src = buf_rsrc(in + (size_t)q * EO::N, q < npoly ? EO::N * 4u : 0u);
        sfor<BG::R>([&](auto J) { r[J] = buf_ld<EO_POL_S2>(src, 4u * lo, 4u * 128u * (uint32_t)J); });
    };
    load(p);
    fill_big_tw<BG, false>(tabw);
    __syncthreads();   // the only workgroup barrier: tables and flags ready
#pragma unroll 1
    for (uint32_t it = 0; it < ppw && p < npoly; ++it) {   // both waves of a pair agree on p
        big_fwd<BG, 0>(r, buf, tab, h, lane, [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
            constexpr int c = C;
            // this wave's half, j' = I + 16 par: natural k = boff(c, I) + 128 par + lane;
            // scalar bases + a 32-bit offset made opaque per chunk (not 64-bit
            // per-lane addresses held across the loop)
            uint32_t lo = 128u * par + lane;
            asm volatile("" : "+v"(lo));
            const auto dst = buf_rsrc(out + (size_t)p * EO::N, EO::N * 4u);
            const auto wt = buf_rsrc(g_eotw[0], 4096u * 8u);
            // the even wave's buffer gets A, the odd wave's B (every j')
            sfor<32>([&](auto J) { buf[64 * J + lane] = v[J]; });
            eo_signal(myflag, step + 1);
            eo_wait(pflag, step + 1);
            // this wave's half of the chunk: j' = I + 16 par, X = A +- w B
            uint32_t xa[16], xb[16];
            sfor<16>([&](auto I) {
                xa[I] = abuf[64 * I + own];
                xb[I] = bbuf[64 * I + own];
            });
            eo_signal(myflag, step + 2);   // done reading the partner's buffer
            sfor<16>([&](auto I) {
#if EO_TWJIT
                const uint2 lam = c_eolam[0][lane], mu = c_eomu[0][par][c][I];
                xb[I] = shoup_mul<P::Q>(xb[I], lam.x, lam.y);
                ct_bfly<P::Q>(xa[I], xb[I], mu.x, mu.y);
#else
                const uint2 tw = buf_ld2(wt, 8u * lo, 8u * BG::boff(c, I));
                ct_bfly<P::Q>(xa[I], xb[I], tw.x, tw.y);
#endif
                buf_st<EO_POL_C>(canon4<P>(xa[I]), dst, 4u * lo, 4u * BG::boff(c, I));
                buf_st<EO_POL_C>(canon4<P>(xb[I]), dst, 4u * lo, 4u * (BG::boff(c, I) + EO::HN));
            });
            eo_wait(pflag, step + 2);   // before the next transpose rewrites this wave's buffer
            step += 2;
        });
        p += EO::NPAIR;
        if (it + 1 < ppw && p < npoly) load(p);
    }
}

__global__ __launch_bounds__(EO::BG::NT, EO::BG::OCC) void k_ntt_inv_eo(const uint32_t *in, uint32_t *out, uint32_t npoly,
                                                                      uint32_t ppw)
{
    using BG = EO::BG;
    static_assert((BG::LDS_WORDS + BG::WAVES) * 4 <= 160 * 1024, "one workgroup per CU");
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::LDS_WORDS + BG::WAVES];
    uint32_t *const tabw = lds + BG::WAVES * XPOSE_WORDS;
    const uint2 *const tab = reinterpret_cast<const uint2 *>(tabw);
    const uint32_t lane = threadIdx.x & 63, h = lane >> 5;
    const uint32_t w = wave_id(), par = w & 1u;
    uint32_t *const buf = lds + w * XPOSE_WORDS;
    uint32_t *const abuf = lds + (w & ~1u) * XPOSE_WORDS, *const bbuf = abuf + XPOSE_WORDS;
    const uint32_t own = 1024u * par + lane;   // row 16 par, this lane
    uint32_t *const myflag = lds + BG::LDS_WORDS + w;
    const uint32_t *const pflag = lds + BG::LDS_WORDS + (w ^ 1u);
    *myflag = 0;
    uint32_t step = 0;   // exchange steps signalled so far (the pair's common count)
    uint32_t p = blockIdx.x * (EO::NPAIR * ppw) + (w >> 1);
    // staging: r[32c + i] = X[k], r[32c + 16 + i] = X[k + 4096] for this
    // wave's half of chunk c (k = boff(c, i + 16 par) + lane)
    uint32_t r[BG::R];
    auto load = [&](uint32_t q) __attribute__((always_inline)) {
        uint32_t lo = 128u * par + lane;
        asm volatile("" : "+v"(lo));
        const auto src = buf_rsrc(in + (size_t)q * EO::N, q < npoly ? EO::N * 4u : 0u);
        sfor<2>([&](auto C) {
            sfor<16>([&](auto I) {
                r[32 * C + I] = buf_ld<EO_POL_C>(src, 4u * lo, 4u * BG::boff(C, I));
                r[32 * C + 16 + I] = buf_ld<EO_POL_C>(src, 4u * lo, 4u * (BG::boff(C, I) + EO::HN));
            });
        });
    };
    load(p);
    fill_big_tw<BG, true>(tabw);
    __syncthreads();   // the only workgroup barrier
#pragma unroll 1
    for (uint32_t it = 0; it < ppw && p < npoly; ++it) {
        auto source = [&](auto C, uint32_t (&v)[32]) __attribute__((always_inline)) {
            constexpr int c = C;
            uint32_t lo = 128u * par + lane;   // natural k = boff(c, I) + lo (see the forward)
            asm volatile("" : "+v"(lo));
            const auto wt = buf_rsrc(g_eotw[1], 4096u * 8u);
            sfor<16>([&](auto I) {
                uint32_t a = r[32 * c + I], b = r[32 * c + 16 + I];
#if EO_TWJIT
                const uint2 lam = c_eolam[1][lane], mu = c_eomu[1][par][c][I];
                gs_bfly<EO::P::Q>(a, b, mu.x, mu.y);
                b = shoup_mul<EO::P::Q>(b, lam.x, lam.y);
#else
                const uint2 tw = buf_ld2(wt, 8u * lo, 8u * BG::boff(c, I));
                gs_bfly<EO::P::Q>(a, b, tw.x, tw.y);   // A = X[k] + X[k + 4096], B = (X[k] - X[k + 4096]) w^-1
#endif
                buf[64 * I + lane] = a;                 // own buffer: A rows 0..15, B rows 16..31
                buf[64 * (16 + I) + lane] = b;
            });
            eo_signal(myflag, step + 1);
            eo_wait(pflag, step + 1);
            // this wave's parity, every j': rows 16 par + I of the even wave's
            // buffer (j' < 16) and of the odd wave's (j' >= 16)
            sfor<16>([&](auto I) {
                v[I] = abuf[64 * I + own];
                v[16 + I] = bbuf[64 * I + own];
            });
            eo_signal(myflag, step + 2);
            eo_wait(pflag, step + 2);   // before the transpose rewrites this wave's buffer
            step += 2;
        };
        uint32_t lo = 2u * lane + par;   // x[2 (64 J + lane) + par]
        asm volatile("" : "+v"(lo));
        const auto dst = buf_rsrc(out + (size_t)p * EO::N, EO::N * 4u);
        big_inv_to<BG, 0, false, EO::S0, EO::S1>(r, buf, tab, h, lane, source, [&](auto J, uint32_t x) __attribute__((always_inline)) {
            buf_st<EO_POL_S2>(x, dst, 4u * lo, 4u * 128u * (uint32_t)J);
        });
        p += EO::NPAIR;
        if (it + 1 < ppw && p < npoly) load(p);
    }
}

}  // namespace qntt
#endif  // NTT_EO
