// valu_cost.hip -- SIMD issue cost of every VALU opcode the hot kernels use
// (tools/asm_hist.py lists them), for the VALU roofline of bench.py
// (DESIGN.md §6): one kernel per opcode, 8 independent chains per lane,
// 8 waves per SIMD, ~2 ms per launch.  Run under
//   rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU -- ./bin/valu_cost
// and tools/valu_cost.py turns the counters into SIMD-cycles per
// wave-instruction at the clock the chip actually held (GRBM_GUI_ACTIVE / 8
// XCDs / kernel time), independent of the DVFS state.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define K32(NAME, ASM)                                                                    \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned *out, unsigned seed, int iters) \
    {                                                                                     \
        unsigned a[8];                                                                    \
        for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;                      \
        const unsigned b = seed | 1;                                                      \
        for (int i = 0; i < iters; i++) {                                                 \
            _Pragma("unroll") for (int u = 0; u < 4; u++)                                 \
            _Pragma("unroll") for (int k = 0; k < 8; k++)                                 \
                asm volatile(ASM : "+v"(a[k]) : "v"(b) : "vcc");                          \
        }                                                                                 \
        unsigned r = 0;                                                                   \
        for (int k = 0; k < 8; k++) r ^= a[k];                                            \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                          \
    }

#define K64(NAME, ASM)                                                                    \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned *out, unsigned seed, int iters) \
    {                                                                                     \
        unsigned long long a[8];                                                          \
        for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;                      \
        const unsigned b = seed | 1;                                                      \
        for (int i = 0; i < iters; i++) {                                                 \
            _Pragma("unroll") for (int u = 0; u < 4; u++)                                 \
            _Pragma("unroll") for (int k = 0; k < 8; k++)                                 \
                asm volatile(ASM : "+v"(a[k]) : "v"(b) : "vcc");          \
        }                                                                                 \
        unsigned r = 0;                                                                   \
        for (int k = 0; k < 8; k++) r ^= (unsigned)a[k] ^ (unsigned)(a[k] >> 32);         \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                          \
    }

K32(v_add_u32, "v_add_u32 %0, %0, %1")
K32(v_sub_u32, "v_sub_u32 %0, %0, %1")
K32(v_subrev_u32, "v_subrev_u32 %0, %0, %1")
K32(v_min_u32, "v_min_u32 %0, %0, %1")
K32(v_max_u32, "v_max_u32 %0, %0, %1")
K32(v_min3_u32, "v_min3_u32 %0, %0, %1, %1")
K32(v_med3_u32, "v_med3_u32 %0, %0, %1, %1")
K32(v_add3_u32, "v_add3_u32 %0, %0, %1, %1")
K32(v_xor_b32, "v_xor_b32 %0, %0, %1")
K32(v_and_b32, "v_and_b32 %0, %0, %1")
K32(v_or_b32, "v_or_b32 %0, %0, %1")
K32(v_mov_b32, "v_mov_b32 %0, %1")
K32(v_lshlrev_b32, "v_lshlrev_b32 %0, 1, %0")
K32(v_lshrrev_b32, "v_lshrrev_b32 %0, 1, %0")
K32(v_ashrrev_i32, "v_ashrrev_i32 %0, 1, %0")
K32(v_bitop3_b32, "v_bitop3_b32 %0, %0, %1, %1 bitop3:0x96")
K32(v_lshl_or_b32, "v_lshl_or_b32 %0, %0, 1, %1")
K32(v_lshl_add_u32, "v_lshl_add_u32 %0, %0, 1, %1")
K32(v_and_or_b32, "v_and_or_b32 %0, %0, %1, %1")
K32(v_mul_lo_u32, "v_mul_lo_u32 %0, %0, %1")
K32(v_mul_hi_u32, "v_mul_hi_u32 %0, %0, %1")
K32(v_mul_hi_i32, "v_mul_hi_i32 %0, %0, %1")
K32(v_mul_u32_u24, "v_mul_u32_u24 %0, %0, %1")
K32(v_cndmask_b32, "v_cndmask_b32 %0, %0, %1, vcc")
K32(v_add_co_u32, "v_add_co_u32 %0, vcc, %0, %1")
K32(v_addc_co_u32, "v_addc_co_u32 %0, vcc, %0, %1, vcc")
K32(v_cmp_lt_u32, "v_cmp_lt_u32 vcc, %0, %1")
K32(v_bfe_u32, "v_bfe_u32 %0, %0, 1, 7")
// round 5: every other opcode the product kernels emit (tools/asm_hist.py over
// `make asm`), so the VALU roofline's mean cost has no guessed term
K32(v_sub_co_u32, "v_sub_co_u32 %0, vcc, %0, %1")
K32(v_subrev_co_u32, "v_subrev_co_u32 %0, vcc, %0, %1")
K32(v_subb_co_u32, "v_subb_co_u32 %0, vcc, %0, %1, vcc")
K32(v_subbrev_co_u32, "v_subbrev_co_u32 %0, vcc, %0, %1, vcc")
K32(v_cmp_gt_u32, "v_cmp_gt_u32 vcc, %0, %1")
K32(v_cmp_ne_u32, "v_cmp_ne_u32 vcc, %0, %1")
K32(v_cmp_eq_u32, "v_cmp_eq_u32 vcc, %0, %1")
K32(v_cmp_le_u32, "v_cmp_le_u32 vcc, %0, %1")
K32(v_cmp_gt_u16, "v_cmp_gt_u16 vcc, %0, %1")
K32(v_not_b32, "v_not_b32 %0, %0")
K32(v_alignbit_b32, "v_alignbit_b32 %0, %0, %0, 1")
K32(v_bfrev_b32, "v_bfrev_b32 %0, %0")
K32(v_xad_u32, "v_xad_u32 %0, %0, %1, %1")
K32(v_or3_b32, "v_or3_b32 %0, %0, %1, %1")
K32(v_mad_u32_u24, "v_mad_u32_u24 %0, %0, %1, %1")
K32(v_mul_lo_u16, "v_mul_lo_u16 %0, %0, %1")
K32(v_sub_u16, "v_sub_u16 %0, %0, %1")
K32(v_mbcnt_lo_u32_b32, "v_mbcnt_lo_u32_b32 %0, %1, %0")
K32(v_mbcnt_hi_u32_b32, "v_mbcnt_hi_u32_b32 %0, %1, %0")
// v_readfirstlane_b32: VALU op with an SGPR destination, 8 independent ones
__global__ __launch_bounds__(256) void k_v_readfirstlane_b32(unsigned *out, unsigned seed, int iters)
{
    unsigned a[8], m[8];
    for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(m[k]) : "v"(a[k]));
    }
    unsigned r = 0;
    for (int k = 0; k < 8; k++) r ^= a[k] ^ m[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}
// v_cndmask with its condition in an SGPR pair that nothing in the loop
// writes (the K32 form above clobbers vcc in every asm statement)
#define KSEL(NAME, ASM)                                                                   \
    __global__ __launch_bounds__(256) void k_##NAME(unsigned *out, unsigned seed, int iters) \
    {                                                                                     \
        unsigned a[8];                                                                    \
        for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;                      \
        const unsigned b = seed | 1;                                                      \
        unsigned long long m;                                                             \
        asm volatile("v_cmp_gt_u32_e64 %0, %1, %2" : "=s"(m) : "v"(a[0]), "v"(b));         \
        for (int i = 0; i < iters; i++) {                                                 \
            _Pragma("unroll") for (int u = 0; u < 4; u++)                                 \
            _Pragma("unroll") for (int k = 0; k < 8; k++)                                 \
                asm volatile(ASM : "+v"(a[k]) : "v"(b), "s"(m));                          \
        }                                                                                 \
        unsigned r = 0;                                                                   \
        for (int k = 0; k < 8; k++) r ^= a[k];                                            \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                          \
    }
KSEL(v_cndmask_b32_sgpr, "v_cndmask_b32_e64 %0, %0, %1, %2")
KSEL(v_cndmask_b32_sgpr_neg, "v_cndmask_b32_e64 %0, %0, -%1, %2")

K64(v_mad_u64_u32, "v_mad_u64_u32 %0, vcc, %1, %1, %0")
K64(v_mad_i64_i32, "v_mad_i64_i32 %0, vcc, %1, %1, %0")
K64(v_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %0")
K64(v_lshlrev_b64, "v_lshlrev_b64 %0, 1, %0")
K64(v_mov_b64, "v_mov_b64 %0, %0")
K64(v_lshrrev_b64, "v_lshrrev_b64 %0, 1, %0")
K64(v_pk_mov_b32, "v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]")
K64(v_cmp_gt_u64, "v_cmp_gt_u64 vcc, %0, %0")
K64(v_cmp_le_u64, "v_cmp_le_u64 vcc, %0, %0")

__global__ __launch_bounds__(256) void k_v_permlane32_swap_b32(unsigned *out, unsigned seed, int iters)
{
    unsigned a[8];
    for (int k = 0; k < 8; k++) a[k] = (threadIdx.x ^ seed) + k;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int k = 0; k < 8; k += 2) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a[k]), "+v"(a[k + 1]));
    }
    unsigned r = 0;
    for (int k = 0; k < 8; k++) r ^= a[k];
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

typedef void (*Fn)(unsigned *, unsigned, int);
struct K {
    const char *name;
    Fn fn;
    int per_iter;   // wave-instructions of the op per loop iteration
};
#define E(N) {#N, k_##N, 32}

int main(int argc, char **argv)
{
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;   // 8 x 256 threads per CU = 8 waves per SIMD
    const int iters = argc > 1 ? atoi(argv[1]) : 4096;
    unsigned *out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    K ks[] = {E(v_add_u32), E(v_sub_u32), E(v_subrev_u32), E(v_min_u32), E(v_max_u32), E(v_min3_u32), E(v_med3_u32),
              E(v_add3_u32), E(v_xor_b32), E(v_and_b32), E(v_or_b32), E(v_mov_b32), E(v_lshlrev_b32),
              E(v_lshrrev_b32), E(v_ashrrev_i32), E(v_bitop3_b32), E(v_lshl_or_b32), E(v_lshl_add_u32),
              E(v_and_or_b32), E(v_mul_lo_u32), E(v_mul_hi_u32), E(v_mul_hi_i32), E(v_mul_u32_u24),
              E(v_cndmask_b32), E(v_cndmask_b32_sgpr), E(v_cndmask_b32_sgpr_neg), E(v_add_co_u32), E(v_addc_co_u32), E(v_cmp_lt_u32), E(v_bfe_u32),
              E(v_mad_u64_u32), E(v_mad_i64_i32), E(v_lshl_add_u64), E(v_lshlrev_b64), E(v_mov_b64),
              E(v_sub_co_u32), E(v_subrev_co_u32), E(v_subb_co_u32), E(v_subbrev_co_u32), E(v_cmp_gt_u32),
              E(v_cmp_ne_u32), E(v_cmp_eq_u32), E(v_cmp_le_u32), E(v_cmp_gt_u16), E(v_not_b32), E(v_alignbit_b32),
              E(v_bfrev_b32), E(v_xad_u32), E(v_or3_b32), E(v_mad_u32_u24), E(v_mul_lo_u16), E(v_sub_u16),
              E(v_mbcnt_lo_u32_b32), E(v_mbcnt_hi_u32_b32), E(v_readfirstlane_b32), E(v_lshrrev_b64), E(v_pk_mov_b32),
              E(v_cmp_gt_u64), E(v_cmp_le_u64),
              {"v_permlane32_swap_b32", k_v_permlane32_swap_b32, 16}};
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    printf("{\"cus\": %d, \"waves_per_simd\": 8, \"iters\": %d", cus, iters);
    for (auto &k : ks) {
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u, 64);   // warm
        hipEventRecord(e0);
        hipLaunchKernelGGL(k.fn, dim3(blocks), dim3(256), 0, 0, out, 7u, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double winstr = (double)blocks * 4 * iters * k.per_iter;   // 4 waves per block
        printf(",\n \"%s\": {\"ms\": %.4f, \"wave_instr\": %.6e, \"simd_cycles_per_instr_at_2.4GHz\": %.3f}", k.name, ms,
               winstr, ms * 1e-3 * 2.4e9 * 4 * cus / winstr);
    }
    printf("}\n");
    hipFree(out);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
