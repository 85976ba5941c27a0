// ntt_kernels.hip -- host side of the gfx950 batched negacyclic NTT library:
// per-device table upload, launch shapes, argument checks and the C ABI of
// include/qtesla_ntt.h.  The kernels themselves are in ntt_device.hpp.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>

#include "../../include/qtesla_ntt.h"
#include "dev_tables.hpp"
#include "ntt_device.hpp"
#include "ntt_large.hpp"
#include "ntt_big.hpp"
#include "ntt_eo.hpp"
#include "ntt_lat.hpp"
#include "ntt_latr.hpp"
#include "ntt_internal.h"
#include "params.hpp"
#include "pset.hpp"

#ifndef QNTT_SRC_HASH
#define QNTT_SRC_HASH "unknown"   // set by the Makefile: sha256 of the library sources
#endif
#define QNTT_STR2(x) #x
#define QNTT_STR(x) QNTT_STR2(x)

namespace qntt {
namespace {

thread_local int t_last_hip = 0;

int hip_err(hipError_t e)
{
    t_last_hip = (int)e;
    return NTT_ERR_HIP;
}

constexpr int kMaxDev = 64;

std::once_flag g_cpu_tables_once;
Tables g_cpu_tables[NPARAM_SETS];

const Tables &cpu_tables(int ps)
{
    std::call_once(g_cpu_tables_once, [] {
        for (int i = 0; i < NPARAM_SETS; i++) make_tables(*param_set(i), g_cpu_tables[i]);
    });
    return g_cpu_tables[ps];
}

// Per-device state: tables uploaded (retried after a failed attempt, e.g. a
// first call made while another stream was being captured) and the launch
// geometry of the device.  `ready` is published with release order once both
// are done, so every later call on that device -- from any host thread, on
// any stream -- takes the lock-free acquire-load path; only a device's first
// calls serialise on g_dev_mutex (a thread-per-GPU host never contends after
// its device's first call).
struct DevInfo {
    std::atomic<bool> ready{false};
    int cus = 256;
};
std::mutex g_dev_mutex;
DevInfo g_dev[kMaxDev];

// Current device, checked, with tables uploaded and geometry known.
int device_ready(DevInfo **out)
{
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_err(e);
    if (dev < 0 || dev >= kMaxDev) return hip_err(hipErrorInvalidDevice);
    DevInfo &d = g_dev[dev];
    if (!d.ready.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(g_dev_mutex);
        if (!d.ready.load(std::memory_order_relaxed)) {
            hipDeviceProp_t prop;
            if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) return hip_err(e);
            d.cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
            if ((e = upload_device_tables(&cpu_tables(0))) != hipSuccess) return hip_err(e);
            d.ready.store(true, std::memory_order_release);
        }
    }
    *out = &d;
    return NTT_OK;
}

// Launch shape: one workgroup per `ppw * waves` consecutive work units.  ppw
// grows with the batch (amortising the 16 KiB LDS-table prologue) but never
// beyond what keeps >= NTT_MIN_WG_PER_CU workgroups per CU in flight.
#ifndef NTT_MIN_WG_PER_CU
#define NTT_MIN_WG_PER_CU 4   // ppw 4 instead of 8 at 65 536 n=1024 polys: 3-4 % faster (profiles/r02/s4/ab_launch_ppw_p1_65536.log); 2^20 keeps ppw 16
#endif
#ifndef NTT_PPW_MAX
#define NTT_PPW_MAX 16
#endif
struct Launch {
    uint32_t grid, ppw;
};
enum Op { OP_XFORM, OP_MUL };
Launch launch_for(Op op, int ps, size_t npoly, const DevInfo &d, int wg = 0)
{
    const size_t upw = param_set(ps)->logn == 11 ? 1 : 2;
    const size_t units = (npoly + upw - 1) / upw;
    const size_t waves = (size_t)(wg ? wg : op == OP_MUL ? MUL_WG : NTT_WG) / 64;
    const size_t min_groups = (size_t)d.cus * NTT_MIN_WG_PER_CU;
    size_t ppw = units / (waves * min_groups);
    ppw = ppw < 1 ? 1 : (ppw > NTT_PPW_MAX ? NTT_PPW_MAX : ppw);
    Launch l;
    l.grid = (uint32_t)((units + waves * ppw - 1) / (waves * ppw));
    l.ppw = (uint32_t)ppw;
    return l;
}

int check_common(int ps, const void *p, size_t batch)
{
    if (!param_set(ps)) return NTT_ERR_PARAM;
    if (batch == 0) return NTT_OK;
    if (!p) return NTT_ERR_NULL;
    if (((uintptr_t)p) & 3u) return NTT_ERR_ALIGN;
    if (batch > (size_t)0x7FFFFFFF) return NTT_ERR_SIZE;
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
    if (e != hipSuccess) return hip_err(e);
    return NTT_OK;
}

template <template <int> class Launcher, class... Args>
int dispatch(int ps, Args &&...args)
{
    switch (ps) {
    case 0: return Launcher<0>::run(args...);
    case 1: return Launcher<1>::run(args...);
    case 2: return Launcher<2>::run(args...);
    case 3: return Launcher<3>::run(args...);
    case 4: return Launcher<4>::run(args...);
    default: return NTT_ERR_PARAM;
    }
}

// n = 4096 / 8192: polynomials per slot and step count, >= 2 workgroups per CU
template <class LG>
size_t large_ppw(size_t batch, const DevInfo &d)
{
    size_t ppw = batch / ((size_t)LG::SLOTS * d.cus * 2);
    return ppw < 1 ? 1 : (ppw > NTT_PPW_MAX ? NTT_PPW_MAX : ppw);
}

// transform kind: forward / inverse with natural or bit-reversed NTT-domain
// order, or the plain bit-reversal permutation
enum Xform { FWD, INV, FWD_BR, INV_BR, BITREV };
static_assert((int)FWD == (int)LAT_FWD && (int)INV == (int)LAT_INV && (int)FWD_BR == (int)LAT_FWD_BR &&
                  (int)INV_BR == (int)LAT_INV_BR,
              "switch table order");
static_assert(LAT_FWD == NTT_OP_FWD && LAT_INV == NTT_OP_INV && LAT_FWD_BR == NTT_OP_FWD_BR &&
                  LAT_INV_BR == NTT_OP_INV_BR && LAT_MUL == NTT_OP_MUL && LAT_MUL_NTT == NTT_OP_MUL_NTT &&
                  LAT_FWD_OOP == NTT_OP_FWD_OOP && LAT_INV_OOP == NTT_OP_INV_OOP,
              "ABI op codes");

template <int PS> struct LXform {
    template <int RB>
    static void launch_latr(Xform k, const uint32_t *in, uint32_t *out, size_t batch, hipStream_t s)
    {
        const dim3 g((uint32_t)batch), b(LatRGeo<PSel<PS>::T::LOGN, RB>::T);
        switch (k) {
        case FWD: hipLaunchKernelGGL((k_ntt_latr<PS, false, false, RB>), g, b, 0, s, in, out); break;
        case INV: hipLaunchKernelGGL((k_ntt_latr<PS, true, false, RB>), g, b, 0, s, in, out); break;
        case FWD_BR: hipLaunchKernelGGL((k_ntt_latr<PS, false, true, RB>), g, b, 0, s, in, out); break;
        case INV_BR: hipLaunchKernelGGL((k_ntt_latr<PS, true, true, RB>), g, b, 0, s, in, out); break;
        default: break;
        }
    }
    static int run(Xform k, const uint32_t *in, uint32_t *out, size_t batch, hipStream_t s, const DevInfo &d)
    {
#ifdef NTT_LATR_FORCE
        // A/B builds only: every transform on the radix-2^NTT_LATR_FORCE
        // workgroup-per-polynomial kernels (ntt_latr.hpp)
        if (k != BITREV) {
            launch_latr<NTT_LATR_FORCE>(k, in, out, batch, s);
            return finish_launch();
        }
#endif
        // FWD / INV: in place or out of place (LAT_FWD_OOP / LAT_INV_OOP)
        const int sop = (k == FWD || k == INV) && in != out ? (k == FWD ? LAT_FWD_OOP : LAT_INV_OOP) : (int)k;
        const int rb = k == BITREV ? 0 : lat_radix(PS, sop, batch);
        if (rb == 2) {
            // small batches: radix-4 passes, one polynomial per n/4-thread workgroup (ntt_lat.hpp)
            const dim3 g((uint32_t)batch), b(LatGeo<PSel<PS>::T::LOGN>::T);
            switch (k) {
            case FWD: hipLaunchKernelGGL((k_ntt_lat<PS, false, false>), g, b, 0, s, in, out); break;
            case INV: hipLaunchKernelGGL((k_ntt_lat<PS, true, false>), g, b, 0, s, in, out); break;
            case FWD_BR: hipLaunchKernelGGL((k_ntt_lat<PS, false, true>), g, b, 0, s, in, out); break;
            case INV_BR: hipLaunchKernelGGL((k_ntt_lat<PS, true, true>), g, b, 0, s, in, out); break;
            default: break;
            }
        } else if (rb == 3) {
            launch_latr<3>(k, in, out, batch, s);   // radix-8 passes, n/8 threads (ntt_latr.hpp)
        } else if (rb == 4) {
            launch_latr<4>(k, in, out, batch, s);   // radix-16 passes, n/16 threads
        } else if constexpr (PS >= LARGE_PS0) {
            // n = 4096 / 8192: one wave per polynomial (ntt_big.hpp); the
            // bit-reversed orders are one launch too (an extra LDS transpose per chunk)
            const uint32_t nb = (uint32_t)batch;
            const dim3 gb((uint32_t)(batch < (size_t)d.cus * 64 ? batch : (size_t)d.cus * 64)), bb(512);
            using BG = Big<PS>;
            size_t ppw = batch / ((size_t)BG::WAVES * d.cus * 2);
            ppw = ppw < 1 ? 1 : (ppw > NTT_PPW_MAX ? NTT_PPW_MAX : ppw);
            const dim3 g((uint32_t)((batch + BG::WAVES * ppw - 1) / (BG::WAVES * ppw))), b(BG::NT);
            const uint32_t pw = (uint32_t)ppw;
#ifdef NTT_EO
            if (PS == LARGE_PS0 + 1 && (k == FWD || k == INV)) {
                // n = 8192 as two n = 4096 halves, a pair of waves per polynomial (ntt_eo.hpp)
                size_t pe = batch / ((size_t)EO::NPAIR * d.cus * 2);
                pe = pe < 1 ? 1 : (pe > NTT_PPW_MAX ? NTT_PPW_MAX : pe);
                const dim3 ge((uint32_t)((batch + EO::NPAIR * pe - 1) / (EO::NPAIR * pe))), be(EO::BG::NT);
                if (k == FWD) hipLaunchKernelGGL(k_ntt_fwd_eo, ge, be, 0, s, in, out, nb, (uint32_t)pe);
                else hipLaunchKernelGGL(k_ntt_inv_eo, ge, be, 0, s, in, out, nb, (uint32_t)pe);
                return finish_launch();
            }
#endif
            switch (k) {
            case FWD: hipLaunchKernelGGL((k_ntt_fwd_big<PS, false>), g, b, 0, s, in, out, nb, pw); break;
            case INV: hipLaunchKernelGGL((k_ntt_inv_big<PS, false>), g, b, 0, s, in, out, nb, pw); break;
            case FWD_BR: hipLaunchKernelGGL((k_ntt_fwd_big<PS, true>), g, b, 0, s, in, out, nb, pw); break;
            case INV_BR: hipLaunchKernelGGL((k_ntt_inv_big<PS, true>), g, b, 0, s, in, out, nb, pw); break;
            case BITREV: hipLaunchKernelGGL(k_bitrev_large<PS>, gb, bb, 0, s, in, out, nb); break;
            }
        } else {
            const Launch l = launch_for(OP_XFORM, PS, batch, d);
            const dim3 g(l.grid), b(NTT_WG);
            const uint32_t nb = (uint32_t)batch;
            switch (k) {
            case FWD: hipLaunchKernelGGL((k_ntt_fwd<PS, false>), g, b, 0, s, in, out, nb, l.ppw); break;
            case INV: hipLaunchKernelGGL((k_ntt_inv<PS, false>), g, b, 0, s, in, out, nb, l.ppw); break;
            case FWD_BR: hipLaunchKernelGGL((k_ntt_fwd<PS, true>), g, b, 0, s, in, out, nb, l.ppw); break;
            case INV_BR: hipLaunchKernelGGL((k_ntt_inv<PS, true>), g, b, 0, s, in, out, nb, l.ppw); break;
            case BITREV: hipLaunchKernelGGL(k_bitrev<PS>, g, b, 0, s, in, out, nb, l.ppw); break;
            }
        }
        return finish_launch();
    }
};
template <int PS, bool BHAT>
void launch_mul_large(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch, hipStream_t s, const DevInfo &d)
{
    using LG = LargeMul<PS, BHAT>;
    const size_t ppw = large_ppw<LG>(batch, d);
    const dim3 g((uint32_t)((batch + LG::SLOTS * ppw - 1) / (LG::SLOTS * ppw))), blk(LG::NT);
    hipLaunchKernelGGL((k_poly_mul_large<PS, BHAT>), g, blk, 0, s, a, b, c, (uint32_t)batch, (uint32_t)ppw);
}
template <int PS> struct LMul {
    static int run(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch, hipStream_t s, bool bhat,
                   const DevInfo &d)
    {
        if constexpr (PSel<PS>::T::N <= 4096) {
            if (batch <= lat_max_batch(PS, bhat ? LAT_MUL_NTT : LAT_MUL)) {
                // small batches: one product per workgroup (ntt_lat.hpp)
                const dim3 g((uint32_t)batch), blk(LatGeo<PSel<PS>::T::LOGN>::T);
                if (bhat) hipLaunchKernelGGL((k_poly_mul_lat<PS, true>), g, blk, 0, s, a, b, c);
                else hipLaunchKernelGGL((k_poly_mul_lat<PS, false>), g, blk, 0, s, a, b, c);
                return finish_launch();
            }
        }
        if constexpr (PS >= LARGE_PS0 && PSel<PS>::T::N == 4096) {
            // one wave per product (ntt_big.hpp)
            const int waves = bhat ? big_mul_waves<true>() : big_mul_waves<false>();
            size_t ppw = batch / ((size_t)waves * d.cus * 2);
            ppw = ppw < 1 ? 1 : (ppw > NTT_PPW_MAX ? NTT_PPW_MAX : ppw);
            const dim3 g((uint32_t)((batch + waves * ppw - 1) / (waves * ppw))), blk(waves * 64);
            if (bhat) hipLaunchKernelGGL((k_poly_mul_big<PS, true>), g, blk, 0, s, a, b, c, (uint32_t)batch, (uint32_t)ppw);
            else hipLaunchKernelGGL((k_poly_mul_big<PS, false>), g, blk, 0, s, a, b, c, (uint32_t)batch, (uint32_t)ppw);
            return finish_launch();
        } else if constexpr (PS >= LARGE_PS0) {
            if (bhat) launch_mul_large<PS, true>(a, b, c, batch, s, d);
            else launch_mul_large<PS, false>(a, b, c, batch, s, d);
            return finish_launch();
        } else {
            if (bhat) {
                const Launch l = launch_for(OP_MUL, PS, batch, d, mul_wg<PS, true>());
                hipLaunchKernelGGL((k_poly_mul<PS, true>), dim3(l.grid), dim3(mul_wg<PS, true>()), 0, s, a, b, c, (uint32_t)batch, l.ppw);
            } else {
                const Launch l = launch_for(OP_MUL, PS, batch, d, mul_wg<PS, false>());
                hipLaunchKernelGGL((k_poly_mul<PS, false>), dim3(l.grid), dim3(mul_wg<PS, false>()), 0, s, a, b, c, (uint32_t)batch, l.ppw);
            }
            return finish_launch();
        }
    }
};
template <int PS> struct LPw {
    static int run(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t count4, hipStream_t s, const DevInfo &d)
    {
        size_t g = (count4 + WG - 1) / WG, cap = (size_t)d.cus * 8;
        hipLaunchKernelGGL(k_pointwise<PS>, dim3((uint32_t)(g < cap ? g : cap)), dim3(WG), 0, s,
                           (const uint4 *)a, (const uint4 *)b, (uint4 *)c, count4);
        return finish_launch();
    }
};

int transform(Xform k, uint32_t *out, const uint32_t *in, size_t batch, int ps, void *stream)
{
    int rc = check_common(ps, in, batch);
    if (rc == NTT_OK && batch) rc = check_common(ps, out, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    if (partial_overlap(in, out, batch * param_set(ps)->n * 4)) return NTT_ERR_ALIAS;
    DevInfo *d = nullptr;
    if ((rc = device_ready(&d)) != NTT_OK) return rc;
    return dispatch<LXform>(ps, k, in, out, batch, (hipStream_t)stream, *d);
}

int mul_common(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b, size_t batch, int ps, void *stream,
               bool bhat)
{
    int rc;
    if ((rc = check_common(ps, d_a, batch)) != NTT_OK || batch == 0) return rc;
    if ((rc = check_common(ps, d_b, batch)) != NTT_OK) return rc;
    if ((rc = check_common(ps, d_c, batch)) != NTT_OK) return rc;
    const size_t bytes = batch * param_set(ps)->n * 4;
    if (partial_overlap(d_a, d_c, bytes) || partial_overlap(d_b, d_c, bytes)) return NTT_ERR_ALIAS;
    DevInfo *d = nullptr;
    if ((rc = device_ready(&d)) != NTT_OK) return rc;
    return dispatch<LMul>(ps, d_a, d_b, d_c, batch, (hipStream_t)stream, bhat, *d);
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
    return transform(FWD, d_poly, d_poly, batch, ps, stream);
}

int poly_invntt(uint32_t *d_poly, const uint32_t *twiddleFactor, size_t batch, int ps, void *stream)
{
    (void)twiddleFactor;
    return transform(INV, d_poly, d_poly, batch, ps, stream);
}

int poly_ntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(FWD, d_out, d_in, batch, ps, stream);
}

int poly_invntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(INV, d_out, d_in, batch, ps, stream);
}

int poly_ntt_bitrev(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(FWD_BR, d_out, d_in, batch, ps, stream);
}

int poly_invntt_bitrev(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(INV_BR, d_out, d_in, batch, ps, stream);
}

int poly_bitrev_copy(uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream)
{
    return transform(BITREV, d_out, d_in, batch, ps, stream);
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
    if (param_set(ps)->n > 2048) return NTT_ERR_PARAM;   // Nussbaumer splits for n = 1024 / 2048
    if (batch == 0) return NTT_OK;
    if ((rc = check_common(ps, d_b, batch)) != NTT_OK) return rc;
    if ((rc = check_common(ps, d_c, batch)) != NTT_OK) return rc;
    if ((((uintptr_t)d_a) | ((uintptr_t)d_b) | ((uintptr_t)d_c)) & 15u) return NTT_ERR_ALIGN;
    const size_t bytes = batch * param_set(ps)->n * 4;
    if (partial_overlap(d_a, d_c, bytes) || partial_overlap(d_b, d_c, bytes)) return NTT_ERR_ALIAS;
    DevInfo *d = nullptr;
    if ((rc = device_ready(&d)) != NTT_OK) return rc;
    const int e = nussbaumer_launch(ps, ring, d_a, d_b, d_c, batch, stream, d->cus);
    if (e != (int)hipSuccess) return hip_err((hipError_t)e);
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
    DevInfo *d = nullptr;
    if ((rc = device_ready(&d)) != NTT_OK) return rc;
    return dispatch<LPw>(ps, d_a, d_b, d_c, count / 4, (hipStream_t)stream, *d);
}

int ntt_fill_uniform(uint32_t *d_poly, size_t batch, int ps, uint64_t seed, uint64_t first_poly, void *stream)
{
    int rc = check_common(ps, d_poly, batch);
    if (rc != NTT_OK || batch == 0) return rc;
    DevInfo *d = nullptr;
    if ((rc = device_ready(&d)) != NTT_OK) return rc;
    const ParamSet *p = param_set(ps);
    const size_t count = batch * p->n;
    size_t g = (count + WG - 1) / WG, cap = (size_t)d->cus * 16;
    hipLaunchKernelGGL(k_fill_uniform, dim3((uint32_t)(g < cap ? g : cap)), dim3(WG), 0, (hipStream_t)stream,
                       d_poly, count, p->q, seed, first_poly * p->n);
    return finish_launch();
}

int ntt_small_batch_max(int ps, int op, size_t *max_batch)
{
    if (!param_set(ps)) return NTT_ERR_PARAM;
    if (op < 0 || op >= LAT_NOPS) return NTT_ERR_PARAM;
    if (!max_batch) return NTT_ERR_NULL;
    *max_batch = lat_max_batch(ps, op);
    return NTT_OK;
}

int ntt_small_batch_radix(int ps, int op, size_t batch, int *radix)
{
    if (!param_set(ps)) return NTT_ERR_PARAM;
    if (op < 0 || op >= LAT_NOPS) return NTT_ERR_PARAM;
    if (!radix) return NTT_ERR_NULL;
    const int rb = lat_radix(ps, op, batch);
    *radix = rb ? 1 << rb : 0;
    return NTT_OK;
}

int ntt_last_hip_error(void) { return t_last_hip; }

int ntt_sync_expiries(uint32_t *count)
{
    if (!count) return NTT_ERR_NULL;
    const hipError_t e = hipMemcpyFromSymbol(count, HIP_SYMBOL(g_slot_sync_expired), sizeof(uint32_t), 0,
                                             hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        t_last_hip = (int)e;
        return NTT_ERR_HIP;
    }
    return NTT_OK;
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

// Build identity: the kernel design, the compiled launch configuration and a
// hash of the library sources ("src=<16 hex>"), so that committed counter
// summaries (profiles/pmc_summary.json) can be tied to the build they were
// measured on.
int ntt_build_info(char *buf, size_t len)
{
    static const char *s =
        "qtesla_ntt gfx950: 1 launch/op, wave-per-poly (n=2048) / half-wave-per-poly (n=1024), 32 coeff/lane, "
        "LDS XOR-swizzled transpose, permlane32 bit-5 stage, Shoup/Harvey lazy CT + signed-Shoup GS butterflies, "
        "dispatch-ordered unit chunks; small batches (per-(n, op) switch, ntt_small_batch_max) one poly per "
        "n/4-thread workgroup; wg=" QNTT_STR(NTT_WG)
        " mul_wg=" QNTT_STR(MUL_WG) " mul_compact=1 ppw<=" QNTT_STR(NTT_PPW_MAX)
        " min_wg/cu=" QNTT_STR(NTT_MIN_WG_PER_CU) "; src=" QNTT_SRC_HASH;
    const int n = (int)strlen(s);
    if (!buf || !len) return n;
    snprintf(buf, len, "%s", s);
    return n;
}

}  // extern "C"
