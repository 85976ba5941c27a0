// valu_rates.hip -- measures gfx950 VALU throughput of the integer ops the
// NTT butterflies use (chip-wide wave-instructions per second), to place the
// kernels against a VALU roofline next to the HBM one.
#include <hip/hip_runtime.h>
#include <cstdio>

#define OP_KERNEL(NAME, ASM)                                                              \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, unsigned seed, int iters)  \
    {                                                                                     \
        unsigned a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;          \
        unsigned a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = seed | 1;       \
        for (int i = 0; i < iters; i++) {                                                 \
            asm volatile(ASM : "+v"(a0) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a1) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a2) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a3) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a4) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a5) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a6) : "v"(b));                                        \
            asm volatile(ASM : "+v"(a7) : "v"(b));                                        \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;      \
    }

OP_KERNEL(k_add, "v_add_u32 %0, %0, %1")
OP_KERNEL(k_min, "v_min_u32 %0, %0, %1")
OP_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %0, %1")
OP_KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %0, %1")
OP_KERNEL(k_mul_u24, "v_mul_u32_u24 %0, %0, %1")
OP_KERNEL(k_mulhi_u24, "v_mul_hi_u32_u24 %0, %0, %1")
OP_KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %1")
OP_KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %0, %1, %1")
OP_KERNEL(k_fma_f32, "v_fma_f32 %0, %0, %1, %1")
OP_KERNEL(k_cndmask, "v_cndmask_b32 %0, %0, %1, vcc")
OP_KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %1")
OP_KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
OP_KERNEL(k_max, "v_max_u32 %0, %0, %1")
OP_KERNEL(k_med3, "v_med3_u32 %0, %0, %1, %1")
OP_KERNEL(k_and, "v_and_b32 %0, %0, %1")
OP_KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
OP_KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
OP_KERNEL(k_sub_e64, "v_sub_u32_e64 %0, %0, %1")
OP_KERNEL(k_mul_hi_i32, "v_mul_hi_i32 %0, %0, %1")
// two-instruction reductions x -> x mod 2q (the butterflies' lazy reduction),
// timed per pair
#define PAIR_KERNEL(NAME, ASM)                                                            \
    __global__ __launch_bounds__(256) void NAME(unsigned *out, unsigned seed, int iters)  \
    {                                                                                     \
        unsigned a[8], t;                                                                 \
        for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;                      \
        const unsigned b = seed | 1;                                                      \
        for (int i = 0; i < iters; i++) {                                                 \
            _Pragma("unroll") for (int k = 0; k < 8; k++)                                 \
                asm volatile(ASM : "+v"(a[k]), "=&v"(t) : "v"(b) : "vcc");                \
        }                                                                                 \
        out[blockIdx.x * 256 + threadIdx.x] = a[0] ^ a[1] ^ a[2] ^ a[3] ^ a[4] ^ a[5] ^ a[6] ^ a[7]; \
    }
PAIR_KERNEL(k_red_min, "v_sub_u32 %1, %0, %2\n\tv_min_u32 %0, %0, %1")
PAIR_KERNEL(k_red_cnd, "v_sub_co_u32 %1, vcc, %0, %2\n\tv_cndmask_b32 %0, %1, %0, vcc")

__global__ __launch_bounds__(256) void k_fma64(unsigned *out, unsigned seed, int iters)
{
    double a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k + seed;
    double b = 1.0000001 * seed;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a[k]) : "v"(b));
    }
    unsigned r = 0;
    for (int k = 0; k < 8; k++) r ^= (unsigned)a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_pk_add(unsigned *out, unsigned seed, int iters)
{
    unsigned long long a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k + seed;
    unsigned long long b = seed | 1;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(*(unsigned *)&a[k]) : "v"((unsigned)b));
    }
    unsigned r = 0;
    for (int k = 0; k < 8; k++) r ^= (unsigned)a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

__global__ __launch_bounds__(256) void k_mad64(unsigned *out, unsigned seed, int iters)
{
    unsigned long long a[8];
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k + seed;
    unsigned b = seed | 1;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_mad_u64_u32 %0, s[100:101], %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(b) : "s100", "s101");
    }
    unsigned r = 0;
    for (int k = 0; k < 8; k++) r ^= (unsigned)a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main()
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 16, iters = 4096;
    unsigned *out;
    hipMalloc(&out, blocks * 256 * 4);
    struct K { const char *name; void (*fn)(unsigned *, unsigned, int); };
    K ks[] = {{"v_sub_u32", k_sub}, {"v_max_u32", k_max}, {"v_med3_u32", k_med3}, {"v_and_b32", k_and},
              {"v_xor_b32", k_xor}, {"v_lshl_add_u32", k_lshl_add}, {"v_sub_u32_e64", k_sub_e64},
              {"v_mul_hi_i32", k_mul_hi_i32}, {"sub+min (per pair)", k_red_min}, {"sub_co+cndmask (per pair)", k_red_cnd},
              {"v_add_u32", k_add}, {"v_min_u32", k_min}, {"v_mul_lo_u32", k_mul_lo}, {"v_mul_hi_u32", k_mul_hi},
              {"v_mul_u32_u24", k_mul_u24}, {"v_mul_hi_u32_u24", k_mulhi_u24}, {"v_mad_u64_u32", k_mad64},
              {"v_add3_u32", k_add3}, {"v_mad_u32_u24", k_mad_u24}, {"v_fma_f32", k_fma_f32},
              {"v_cndmask_b32", k_cndmask}, {"v_perm_b32", k_perm}, {"v_fma_f64", k_fma64}, {"v_pk_add_u16", k_pk_add}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d", cus);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u, 64);
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        double lane_ops = (double)blocks * 256 * iters * 8;
        printf(",\n \"%s\": {\"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"lanes_per_clk_per_cu_at_2.4GHz\": %.2f}", k.name,
               ms, lane_ops / (ms * 1e-3), lane_ops / (ms * 1e-3) / 2.4e9 / cus);
    }
    printf("}\n");
    hipFree(out);
    return 0;
}
