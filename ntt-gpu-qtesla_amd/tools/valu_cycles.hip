// valu_cycles.hip -- cycles per wave-instruction of the integer VALU ops used
// by the NTT butterflies (gfx950), measured in-kernel with s_memtime over a
// loop of 16 independent accumulators per lane; W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int OP>
__global__ __launch_bounds__(1024) void k(unsigned long long *cyc, unsigned *sink, int iters)
{
    unsigned a[16], b = threadIdx.x | 1, c = threadIdx.x * 7 + 3;
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = threadIdx.x + i;
    unsigned long long a64[16];
#pragma unroll
    for (int i = 0; i < 16; i++) a64[i] = a[i];
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#define STEP(i)                                                                                   \
    if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));            \
    if constexpr (OP == 1) asm volatile("v_min_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));            \
    if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));         \
    if constexpr (OP == 3) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));         \
    if constexpr (OP == 4) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(a64[i]) : "v"(b), "v"(c) : "vcc"); \
    if constexpr (OP == 5) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c)); \
    if constexpr (OP == 6) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a[i]) : "v"(b));        \
    if constexpr (OP == 7) asm volatile("v_mul_lo_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b)); \
    if constexpr (OP == 8) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a[i]) : "v"(b));
        R16(STEP)
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned r = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) r ^= a[i] ^ (unsigned)a64[i];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + threadIdx.x / 64] = t1 - t0;
}

int main()
{
    const char *names[] = {"v_add_u32", "v_min_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mad_u64_u32", "v_add3_u32",
                           "v_mul_u32_u24", "mul_lo+add(pair)", "v_fma_f32"};
    void (*ks[])(unsigned long long *, unsigned *, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>};
    unsigned long long *cyc;
    unsigned *sink;
    (void)hipMalloc(&cyc, 256 * 16 * 8);
    (void)hipMalloc(&sink, 256 * 1024 * 4);
    const int iters = 2000;
    printf("{");
    for (int w : {1, 2, 4}) {   // waves per SIMD (block = 4*w waves, one block per CU)
        for (int o = 0; o < 9; o++) {
            hipLaunchKernelGGL(ks[o], dim3(256), dim3(256 * w), 0, 0, cyc, sink, 10);
            hipLaunchKernelGGL(ks[o], dim3(256), dim3(256 * w), 0, 0, cyc, sink, iters);
            (void)hipDeviceSynchronize();
            std::vector<unsigned long long> h(256 * 16);
            (void)hipMemcpy(h.data(), cyc, h.size() * 8, hipMemcpyDeviceToHost);
            double s = 0;
            int cnt = 0;
            for (int b = 0; b < 256; b++)
                for (int v = 0; v < 4 * w; v++) { s += h[b * 16 + v]; cnt++; }
            // per-wave cycles / instructions issued by that wave; x w waves share a SIMD
            double cpi_wave = s / cnt / (iters * 16.0 * (o == 7 ? 2 : 1));
            printf("%s\"w%d_%s\": {\"cycles_per_instr_per_wave\": %.2f, \"simd_cycles_per_instr\": %.2f}",
                   (w == 1 && o == 0) ? "" : ", ", w, names[o], cpi_wave, cpi_wave / w);
        }
    }
    printf("}\n");
    return 0;
}
