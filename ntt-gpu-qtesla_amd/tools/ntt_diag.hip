// ntt_diag.hip -- tools-only library (lib/libqtesla_ntt_diag.so, `make tools`)
// for bottleneck attribution of the transform kernels: the production kernels
// of csrc/ntt_device.hpp next to variants that keep one side of them only.
// Never linked into libqtesla_ntt.so; used by tools/variants.py.
//
//   variant 0  full kernel (k_ntt_fwd / k_ntt_inv, natural order)
//   variant 1  global load + store only (same addresses, grid and work loop)
//   variant 2  arithmetic + LDS transposes only (no global memory)
//   variant 3  load + LDS transpose(s) + store (no arithmetic)
//   op 2       plain copies of n=2048 polys, one per wave: dword (variant 0)
//              or dwordx4 (variant 1) accesses
//   op 3       k_poly_mul (d_out = in * in): variant 0 full, 1 global loads +
//              stores only, 2 arithmetic + LDS only (k_poly_mul's VAR)
//   op 4       the round-3 workgroup-per-polynomial n = 2048 transforms
//              (ntt_wg.hpp): variant 0 / 1 forward persistent /
//              one polynomial per workgroup, 2 / 3 the same inverses
//   op 5 / 6   the radix-8 / radix-16 workgroup-per-polynomial transforms
//              (csrc/ntt_latr.hpp, n <= 2048, one polynomial per workgroup):
//              variants 0-3 forward, 4-7 inverse: full, memory only (loads, LDS
//              exchanges and barriers, stores), arithmetic + twiddle loads +
//              LDS only (no global data traffic), memory only plus the twiddle
//              loads
//   op 7       the n = 4096 / 8192 one-wave-per-polynomial transforms
//              (csrc/ntt_big.hpp, param sets 3 / 4, natural order): variant 0
//              / 2 the forward / inverse kernels, 1 / 3 their memory-only
//              variants (the same launch shape, loads, per-chunk LDS
//              transposes and stores, no arithmetic)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

#include "../../include/qtesla_ntt.h"
#include "../csrc/dev_tables.hpp"
#include "../csrc/ntt_device.hpp"
#include "ntt_wg.hpp"
#include "../csrc/ntt_latr.hpp"

namespace qntt {
namespace {

// keeps a value live without storing it
__device__ __forceinline__ void sink(uint32_t v) { asm volatile("" ::"v"(v)); }

template <int PS, bool INV, int V>
__global__ __launch_bounds__(NTT_WG, NTT_WAVES_PER_SIMD) void k_variant(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    using P = typename PSel<PS>::T;
    using LT = Lane<P>;
    __shared__ __attribute__((aligned(16))) uint32_t lds[NTT_LDS_WORDS];
    uint2 *tw2 = reinterpret_cast<uint2 *>(lds + NTT_WAVES * XPOSE_WORDS);
    auto prologue = [&]() {
        fill_tw2<PS, INV, NTT_WG>(tw2);
        __syncthreads();
    };
    const LT L;
    uint32_t *buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    const uint32_t nunits = (npoly + LT::UPW - 1) / LT::UPW;
    auto load = [&](uint32_t (&r)[32], uint32_t u) {
        if constexpr (V == 2) {
#pragma unroll
            for (int j = 0; j < 32; ++j) r[j] = L.lane * (j + u);
        } else {
            load32(r, in + (size_t)L.load_poly(u, npoly) * P::N + L.brl,
                   [](int j) { return INV ? brv5(j) * LT::S : LT::S * j; });
        }
    };
    auto process = [&](uint32_t (&r)[32], uint32_t u) {
        const uint32_t poly = L.poly(u);
        if constexpr (!INV) {
            if constexpr (V == 2) fwd_pass1<PS, P>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
            if constexpr (V != 1) lds_p1_to_p2<P>(r, buf, L);
            if constexpr (V == 2) fwd_pass2<P>(r, tw2 + opaque_zero(), L.lane);
        } else {
            if constexpr (V == 2) inv_pass2<P>(r, tw2 + opaque_zero(), L.lane);
            if constexpr (V != 1) lds_p2_to_p1<P>(r, buf, L);
            if constexpr (V == 2) inv_pass1<PS, P, P::NINV, P::C1>(r, L.h, tw2 + TW2_ENTRIES * 64 + opaque_zero());
        }
        if (LT::BIG || poly < npoly) {
            uint32_t *dst = out + (size_t)poly * P::N + L.brl;
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                if constexpr (V == 2) sink(r[j]);
                else st_out(dst + (INV ? LT::S * j : brv5(j) * LT::S), r[j]);
            }
        }
    };
    chunk_loop<NTT_WAVES>(nunits, ppw, prologue, load, process);
}

// memory-only n = 4096 / 8192 transforms: k_ntt_fwd_big / k_ntt_inv_big's
// launch, table prologue, loads, chunk transposes and stores, without the
// butterflies, the bit-5 swap or the twiddle reads
template <int PS, bool INV>
__global__ __launch_bounds__(Big<PS>::NT, Big<PS>::OCC) void k_big_mem(const uint32_t *in, uint32_t *out, uint32_t npoly,
                                                                    uint32_t ppw)
{
    using BG = Big<PS>;
    using P = typename BG::P;
    constexpr uint32_t N = BG::PL::N;
    __shared__ __attribute__((aligned(16))) uint32_t lds[BG::LDS_WORDS];
    uint32_t *const tabw = lds + BG::WAVES * XPOSE_WORDS;
    auto prologue = [&]() {
        fill_big_tw<BG, INV>(tabw);
        __syncthreads();
    };
    const uint32_t lane = threadIdx.x & 63;
    uint32_t *const buf = lds + (threadIdx.x >> 6) * XPOSE_WORDS;
    auto load = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        if constexpr (!INV) big_load_a<BG>(r, in + (size_t)u * N, lane);
        else big_load_b<BG>(r, in + (size_t)u * N, lane);
    };
    auto process = [&](uint32_t (&r)[BG::R], uint32_t u) __attribute__((always_inline)) {
        uint32_t lo = lane;
        asm volatile("" : "+v"(lo));
        uint32_t *const dst = out + (size_t)u * N + lo;
        sfor<BG::CH>([&](auto C) {
            const uint32_t wb = big_wbase(opaque_lane());
            const Lane<P> LB(opaque_lane());
            if constexpr (!INV) {   // A'' rows -> b128 reads of layout B -> B-order stores
                sfor<32>([&](auto T) { buf[big_waddr(wb, T)] = r[BG::creg(C, T)]; });
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
                sfor<32>([&](auto JP) { st_out(dst + BG::boff(C, JP), v[JP]); });
            } else {   // layout B -> b128 writes -> A'' rows back into the registers
                sfor<8>([&](auto Q) {
                    *reinterpret_cast<uint4 *>(buf + LB.rbase + ((4u * Q) ^ LB.rxm)) =
                        make_uint4(r[BG::creg(C, 4 * Q + 0)], r[BG::creg(C, 4 * Q + 1)], r[BG::creg(C, 4 * Q + 2)],
                                   r[BG::creg(C, 4 * Q + 3)]);
                });
                compiler_fence();
                sfor<32>([&](auto T) { r[BG::creg(C, T)] = buf[big_waddr(wb, T)]; });
                compiler_fence();
            }
        });
        if constexpr (INV)   // layout A stores (lane-contiguous 256-B runs)
            sfor<BG::R>([&](auto J) { st_out(dst + 64u * (uint32_t)J, r[J]); });
    };
    big_loop<BG>(npoly, ppw, prologue, load, process);
}

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

std::once_flag g_once;
hipError_t g_upload = hipSuccess;
int g_cus = 256;

template <int PS>
int launch(int op, int variant, uint32_t *out, const uint32_t *in, uint32_t nb, hipStream_t s)
{
    using P = typename PSel<PS>::T;
    const uint32_t units = (nb + Lane<P>::UPW - 1) / Lane<P>::UPW;
    uint32_t ppw = units / (NTT_WAVES * 2 * g_cus);
    ppw = ppw < 1 ? 1 : (ppw > 16 ? 16 : ppw);
    const dim3 g((units + NTT_WAVES * ppw - 1) / (NTT_WAVES * ppw)), b(NTT_WG);
#define QNTT_V(INV, V) hipLaunchKernelGGL((k_variant<PS, INV, V>), g, b, 0, s, in, out, nb, ppw)
    switch (op * 16 + variant) {
    case 0: hipLaunchKernelGGL((k_ntt_fwd<PS, false>), g, b, 0, s, in, out, nb, ppw); break;
    case 1: QNTT_V(false, 1); break;
    case 2: QNTT_V(false, 2); break;
    case 3: QNTT_V(false, 3); break;
    case 16: hipLaunchKernelGGL((k_ntt_inv<PS, false>), g, b, 0, s, in, out, nb, ppw); break;
    case 48:
    case 49:
    case 50: {
        // the library's poly_mul launch shape (launch_for(OP_MUL)): 4 workgroups per CU
        constexpr int W = mul_wg<PS>() / 64;
        uint32_t mp = units / (W * 4 * g_cus);
        mp = mp < 1 ? 1 : (mp > 16 ? 16 : mp);
        const dim3 gm((units + W * mp - 1) / (W * mp)), bm(mul_wg<PS>());
        if (variant == 0) hipLaunchKernelGGL((k_poly_mul<PS, false, 0>), gm, bm, 0, s, in, in, out, nb, mp);
        else if (variant == 1) hipLaunchKernelGGL((k_poly_mul<PS, false, 1>), gm, bm, 0, s, in, in, out, nb, mp);
        else hipLaunchKernelGGL((k_poly_mul<PS, false, 2>), gm, bm, 0, s, in, in, out, nb, mp);
        break;
    }
    case 17: QNTT_V(true, 1); break;
    case 18: QNTT_V(true, 2); break;
    case 19: QNTT_V(true, 3); break;
    default: return NTT_ERR_PARAM;
    }
#undef QNTT_V
    return hipGetLastError() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
}

}  // namespace
}  // namespace qntt

using namespace qntt;

extern "C" int ntt_debug_variant(int op, int variant, uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps,
                                 void *stream)
{
    const ParamSet *p = param_set(ps);
    if (!p || (ps > 2) != (op == 7)) return NTT_ERR_PARAM;   // op 7: the n = 4096 / 8192 sets only
    if (batch == 0) return NTT_OK;
    if (!d_in || !d_out) return NTT_ERR_NULL;
    if ((((uintptr_t)d_in) | ((uintptr_t)d_out)) & 15u) return NTT_ERR_ALIGN;
    if (batch > 0x7FFFFFFF) return NTT_ERR_SIZE;
    const size_t bytes = batch * p->n * 4;
    const uintptr_t a = (uintptr_t)d_in, b = (uintptr_t)d_out;
    if (a != b && a < b + bytes && b < a + bytes) return NTT_ERR_ALIAS;
    std::call_once(g_once, [] {
        Tables tabs[NPARAM_SETS];
        for (int i = 0; i < NPARAM_SETS; i++) make_tables(*param_set(i), tabs[i]);
        g_upload = upload_device_tables(tabs);
        int dev = 0;
        hipDeviceProp_t prop;
        if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
            g_cus = prop.multiProcessorCount;
    });
    if (g_upload != hipSuccess) return NTT_ERR_HIP;
    hipStream_t s = (hipStream_t)stream;
    if (op == 2) {   // copies of n = 2048 polys, 2 workgroups of 8 waves per CU
        if (p->n != 2048) return NTT_ERR_PARAM;
        const dim3 g2((uint32_t)g_cus * 2);
        if (variant == 0) hipLaunchKernelGGL((k_copy_diag<1>), g2, dim3(512), 0, s, d_in, d_out, (uint32_t)batch);
        else hipLaunchKernelGGL((k_copy_diag<4>), g2, dim3(512), 0, s, d_in, d_out, (uint32_t)batch);
        return hipGetLastError() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
    if (op == 4) {   // workgroup-per-polynomial kernels (p-III only)
        if (ps != 2) return NTT_ERR_PARAM;
        const bool persist = !(variant & 1);
        int occ = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_wg_xform<2, false, true>, WGP_T, 0) !=
                hipSuccess || occ < 1)
            occ = 4;
        const size_t res = persist ? (size_t)g_cus * occ : batch;
        const dim3 g((uint32_t)(batch < res ? batch : res)), b(WGP_T);
        const uint32_t nb = (uint32_t)batch;
        switch (variant) {
        case 0: hipLaunchKernelGGL((k_wg_xform<2, false, true>), g, b, 0, s, d_in, d_out, nb); break;
        case 1: hipLaunchKernelGGL((k_wg_xform<2, false, false>), g, b, 0, s, d_in, d_out, nb); break;
        case 2: hipLaunchKernelGGL((k_wg_xform<2, true, true>), g, b, 0, s, d_in, d_out, nb); break;
        case 3: hipLaunchKernelGGL((k_wg_xform<2, true, false>), g, b, 0, s, d_in, d_out, nb); break;
        default: return NTT_ERR_PARAM;
        }
        return hipGetLastError() == hipSuccess ? NTT_OK : NTT_ERR_HIP;
    }
    if (op == 7) {   // n = 4096 / 8192: the library's launch shape (ntt_kernels.hip, LXform)
        auto run = [&](auto PSI) {
            constexpr int PS = decltype(PSI)::value;
            using BG = Big<PS>;
            size_t ppw = batch / ((size_t)BG::WAVES * g_cus * 2);
            ppw = ppw < 1 ? 1 : (ppw > 16 ? 16 : ppw);
            const dim3 g((uint32_t)((batch + BG::WAVES * ppw - 1) / (BG::WAVES * ppw))), b(BG::NT);
            const uint32_t nb = (uint32_t)batch, pw = (uint32_t)ppw;
            switch (variant) {
            case 0: hipLaunchKernelGGL((k_ntt_fwd_big<PS, false>), g, b, 0, s, d_in, d_out, nb, pw); break;
            case 1: hipLaunchKernelGGL((k_big_mem<PS, false>), g, b, 0, s, d_in, d_out, nb, pw); break;
            case 2: hipLaunchKernelGGL((k_ntt_inv_big<PS, false>), g, b, 0, s, d_in, d_out, nb, pw); break;
            case 3: hipLaunchKernelGGL((k_big_mem<PS, true>), g, b, 0, s, d_in, d_out, nb, pw); break;
            default: return (int)NTT_ERR_PARAM;
            }
            return hipGetLastError() == hipSuccess ? (int)NTT_OK : (int)NTT_ERR_HIP;
        };
        return ps == 3 ? run(std::integral_constant<int, 3>{}) : run(std::integral_constant<int, 4>{});
    }
    if (op == 5 || op == 6) {   // one polynomial per workgroup: the grid is the batch
        const dim3 g((uint32_t)batch);
        auto run = [&](auto PSI, auto RBI) {
            constexpr int PS = decltype(PSI)::value, RB = decltype(RBI)::value;
            const dim3 b(LatRGeo<PSel<PS>::T::LOGN, RB>::T);
            switch (variant) {
            case 0: hipLaunchKernelGGL((k_ntt_latr<PS, false, false, RB, 0>), g, b, 0, s, d_in, d_out); break;
            case 1: hipLaunchKernelGGL((k_ntt_latr<PS, false, false, RB, 1>), g, b, 0, s, d_in, d_out); break;
            case 2: hipLaunchKernelGGL((k_ntt_latr<PS, false, false, RB, 2>), g, b, 0, s, d_in, d_out); break;
            case 3: hipLaunchKernelGGL((k_ntt_latr<PS, false, false, RB, 3>), g, b, 0, s, d_in, d_out); break;
            case 4: hipLaunchKernelGGL((k_ntt_latr<PS, true, false, RB, 0>), g, b, 0, s, d_in, d_out); break;
            case 5: hipLaunchKernelGGL((k_ntt_latr<PS, true, false, RB, 1>), g, b, 0, s, d_in, d_out); break;
            case 6: hipLaunchKernelGGL((k_ntt_latr<PS, true, false, RB, 2>), g, b, 0, s, d_in, d_out); break;
            case 7: hipLaunchKernelGGL((k_ntt_latr<PS, true, false, RB, 3>), g, b, 0, s, d_in, d_out); break;
            default: return (int)NTT_ERR_PARAM;
            }
            return hipGetLastError() == hipSuccess ? (int)NTT_OK : (int)NTT_ERR_HIP;
        };
        using R3 = std::integral_constant<int, 3>;
        using R4 = std::integral_constant<int, 4>;
        switch (ps * 2 + (op == 6)) {
        case 0: return run(std::integral_constant<int, 0>{}, R3{});
        case 1: return run(std::integral_constant<int, 0>{}, R4{});
        case 2: return run(std::integral_constant<int, 1>{}, R3{});
        case 3: return run(std::integral_constant<int, 1>{}, R4{});
        case 4: return run(std::integral_constant<int, 2>{}, R3{});
        default: return run(std::integral_constant<int, 2>{}, R4{});
        }
    }
    if (op != 0 && op != 1 && op != 3) return NTT_ERR_PARAM;
    switch (ps) {
    case 0: return launch<0>(op, variant, d_out, d_in, (uint32_t)batch, s);
    case 1: return launch<1>(op, variant, d_out, d_in, (uint32_t)batch, s);
    case 2: return launch<2>(op, variant, d_out, d_in, (uint32_t)batch, s);
    default: return NTT_ERR_PARAM;
    }
}
