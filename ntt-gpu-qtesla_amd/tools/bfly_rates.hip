// bfly_rates.hip -- throughput of the butterflies in isolation (register-
// resident, 16 independent butterflies per stage, 256 CUs x 16 waves): the
// production unsigned lazy CT (ct_bfly) and GS (gs_bfly), and a signed CT
// candidate (sct_bfly below: t = y w by a signed Shoup product with a rounded
// companion, x' = x + t, y' = x - t; 5 VALU, + 2 where the x input needs a
// centred Barrett reduction).  Diagnostic only (tools), not in the library.
//
// Measured (profiles/r02/s4/bfly_rates.log): signed CT 2.05 ns per wave
// butterfly per CU without the reduction, 2.95 with it, unsigned CT 3.08,
// GS 2.95 -- yet a signed forward (reductions on 5 of 11 p-III stages) left
// k_ntt_fwd and k_poly_mul unchanged or 1-2 % slower (profiles/r02/s4/
// ab_signed_fwd_*.log): the transforms sit on the memory floor and poly_mul
// on occupancy, not on VALU issue.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../csrc/ntt_device.hpp"

using namespace qntt;
using P = PS2;

// the signed candidate (not in the library)
template <uint32_t Q>
__device__ __forceinline__ uint32_t sshoup_r(uint32_t y, uint32_t ws, uint32_t wps)
{
    const uint32_t e = (uint32_t)(((int64_t)(int32_t)y * (int32_t)wps + 0x80000000ll) >> 32);
    return madlo32(e, 0u - Q, y * ws);
}
template <bool RED>
__device__ __forceinline__ void sct_bfly(uint32_t &x, uint32_t &y, uint32_t ws, uint32_t wps)
{
    constexpr uint32_t MB = (uint32_t)(((1ull << 32) + P::Q / 2) / P::Q);   // round(2^32 / q)
    const uint32_t a = RED ? sshoup_r<P::Q>(x, 1u, MB) : x;
    const uint32_t t = sshoup_r<P::Q>(y, ws, wps);
    x = a + t;
    y = a - t;
}

// one "stage" = 16 butterflies on (j, j + 16), then 16 on (j, j + 8) ...
template <int KIND>
__device__ __forceinline__ void bf(uint32_t &x, uint32_t &y, uint32_t w0, uint32_t w1)
{
    if constexpr (KIND == 0) ct_bfly<P::Q>(x, y, w0, w1);
    else if constexpr (KIND == 1) sct_bfly<false>(x, y, w0, w1);
    else if constexpr (KIND == 2) sct_bfly<true>(x, y, w0, w1);
    else gs_bfly<P::Q>(x, y, w0, w1);
}

template <int KIND>
__global__ __launch_bounds__(256) void k_bfly(uint32_t *sink, const uint2 *tw, int iters)
{
    uint32_t r[32];
#pragma unroll
    for (int i = 0; i < 32; i++) r[i] = (threadIdx.x * 2654435761u + i) % P::Q;
    const uint2 t0 = tw[threadIdx.x & 7], t1 = tw[8 + (threadIdx.x & 7)];
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int s = 0; s < 4; s++) {
            const int hh = 16 >> s;
            const uint2 w = (s & 1) ? t1 : t0;
#pragma unroll
            for (int j = 0; j < 32; j++)
                if ((j & hh) == 0) bf<KIND>(r[j], r[j + hh], w.x, w.y);
        }
    }
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 32; i++) x ^= r[i];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

__global__ __launch_bounds__(256) void k_madi64(uint32_t *sink, const uint2 *tw, int iters)
{
    unsigned long long a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k;
    const uint32_t b = tw[0].x | 1;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_mad_i64_i32 %0, s[100:101], %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(b) : "s100", "s101");
    }
    uint32_t r = 0;
    for (int k = 0; k < 8; k++) r ^= (uint32_t)a[k];
    sink[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_madu64(uint32_t *sink, const uint2 *tw, int iters)
{
    unsigned long long a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k;
    const uint32_t b = tw[0].x | 1;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(b) : "s100", "s101");
    }
    uint32_t r = 0;
    for (int k = 0; k < 8; k++) r ^= (uint32_t)a[k];
    sink[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mulhi(uint32_t *sink, const uint2 *tw, int iters)
{
    uint32_t a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k;
    const uint32_t b = tw[0].x | 1;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
    }
    uint32_t r = 0;
    for (int k = 0; k < 8; k++) r ^= a[k];
    sink[blockIdx.x * 256 + threadIdx.x] = r;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 16, iters = 512;
    uint32_t *sink;
    uint2 *tw;
    hipMalloc(&sink, (size_t)blocks * 256 * 4);
    hipMalloc(&tw, 16 * sizeof(uint2));
    uint2 h[16];
    for (int i = 0; i < 16; i++) {
        const TwPair c = csigned_tw(12345u * (i + 3) % P::Q, P::Q);
        h[i] = make_uint2(c.x, c.y);
    }
    hipMemcpy(tw, h, sizeof h, hipMemcpyHostToDevice);
    struct K { const char *name; void (*fn)(uint32_t *, const uint2 *, int); double ops; };
    // butterflies per thread per iteration: 4 stages x 16
    const K ks[] = {{"ct_bfly (unsigned lazy, 7 VALU)", k_bfly<0>, 64.0},
                    {"sct_bfly no reduction (5 VALU)", k_bfly<1>, 64.0},
                    {"sct_bfly x reduced (7 VALU)", k_bfly<2>, 64.0},
                    {"gs_bfly (7 VALU)", k_bfly<3>, 64.0},
                    {"v_mad_i64_i32", k_madi64, 64.0},
                    {"v_mad_u64_u32", k_madu64, 64.0},
                    {"v_mul_hi_u32", k_mulhi, 64.0}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d", cus);
    for (const K &k : ks) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, sink, tw, 16);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, sink, tw, iters);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            best = ms < best ? ms : best;
        }
        const double per_s = (double)blocks * 256 * iters * k.ops / (best * 1e-3);
        printf(",\n \"%s\": {\"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"ns_per_wave_op_per_cu\": %.4f}", k.name, best, per_s,
               1e9 / (per_s / 64.0 / cus));
    }
    printf("}\n");
    hipFree(sink);
    hipFree(tw);
    return 0;
}
