// bfly_occupancy.hip -- SIMD cycles per CT butterfly (Shoup, lazy, negated
// twiddle: the production instruction sequence) as a function of waves per
// SIMD, with 16 independent butterflies per wave in flight.  Tells how much
// occupancy the transform kernels need to saturate VALU issue.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

constexpr unsigned Q = 856145921u;
__device__ __forceinline__ unsigned umin(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ void ct(unsigned &x, unsigned &y, unsigned wn, unsigned wp)
{
    const unsigned a = umin(x, x - 2 * Q);
    const unsigned qe = __umulhi(y, wp);
    const unsigned tn = (unsigned)((unsigned long long)qe * Q + (unsigned)(y * wn));
    x = a - tn;
    y = a + tn + 2 * Q;
}

template <int NB>   // independent butterflies per wave
__global__ __launch_bounds__(256) void k(unsigned long long *cyc, unsigned *sink, const uint2 *tw, int iters)
{
    unsigned r[2 * NB];
#pragma unroll
    for (int i = 0; i < 2 * NB; i++) r[i] = (threadIdx.x * 2654435761u + i) % Q;
    const uint2 w = tw[0], w2 = tw[1];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NB; i++) ct(r[i], r[i + NB], w.x, w.y);
#pragma unroll
        for (int i = 0; i < NB; i++) ct(r[2 * (i / 2) * 1 + (i & 1) + ((i / 2) & 1) * 0], r[(i + NB / 2) % (2 * NB)], w2.x, w2.y);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < 2 * NB; i++) x ^= r[i];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + threadIdx.x / 64] = t1 - t0;
}

int main()
{
    unsigned long long *cyc;
    unsigned *sink;
    uint2 *tw;
    (void)hipMalloc(&cyc, 256 * 8 * 4 * 8);
    (void)hipMalloc(&sink, 256 * 8 * 256 * 4);
    (void)hipMalloc(&tw, 16);
    uint2 h[2] = {{0u - 12345u, (unsigned)((12345ull << 32) / Q)}, {0u - 777u, (unsigned)((777ull << 32) / Q)}};
    (void)hipMemcpy(tw, h, 16, hipMemcpyHostToDevice);
    const int iters = 1000;
    printf("{");
    bool first = true;
    for (int w : {1, 2, 3, 4, 5, 6, 8}) {
        // w blocks of 4 waves per CU (one wave per SIMD each)
        hipLaunchKernelGGL(k<16>, dim3(256 * w), dim3(256), 0, 0, cyc, sink, tw, 10);
        hipLaunchKernelGGL(k<16>, dim3(256 * w), dim3(256), 0, 0, cyc, sink, tw, iters);
        (void)hipDeviceSynchronize();
        std::vector<unsigned long long> c(256 * 8 * 4);
        (void)hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
        double s = 0;
        for (int b = 0; b < 256 * w; b++)
            for (int v = 0; v < 4; v++) s += c[b * 4 + v];
        const double per_wave = s / (256.0 * 4 * w) / (iters * 32.0);   // cycles per butterfly per wave
        printf("%s\"waves_per_simd_%d\": {\"wave_cycles_per_bfly\": %.2f, \"simd_cycles_per_bfly\": %.2f}",
               first ? "" : ", ", w, per_wave, per_wave / w);
        first = false;
    }
    printf("}\n");
    return 0;
}
