// wave_place.hip -- where the waves of a workgroup land (diagnostic for the
// Nussbaumer pair layout): every wave records its hardware id
// (HW_REG_HW_ID: wave slot, SIMD, CU, SE) and its XCC, for 128-thread
// (one pair) and 512-thread (four pairs) workgroups holding a Nussbaumer-sized
// LDS allocation, and the summary says how often wave w shares a SIMD with
// wave w ^ 1 (pair partner in the shipped layout) and with wave w ^ 4.
//   ./bin/wave_place
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

template <int WG, int LDSW>
__global__ __launch_bounds__(WG) void k_place(unsigned *out, unsigned spin)
{
    __shared__ unsigned lds[LDSW];
    const unsigned wave = threadIdx.x >> 6;
    lds[threadIdx.x] = threadIdx.x;
    // keep the wave resident a while so that the residency is the steady state's
    unsigned x = threadIdx.x;
    for (unsigned i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
    __syncthreads();
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID
    if ((threadIdx.x & 63) == 0) {
        unsigned *o = out + 4 * (blockIdx.x * (WG / 64) + wave);
        o[0] = hw;
        o[1] = xcc;
        o[2] = lds[(threadIdx.x + 1) % WG] + (x & 0);
        o[3] = blockIdx.x;
    }
}

template <int WG, int LDSW>
static void run(const char *name, unsigned nwg)
{
    const unsigned nw = nwg * (WG / 64);
    unsigned *d;
    CK(hipMalloc(&d, 16ull * nw));
    hipLaunchKernelGGL((k_place<WG, LDSW>), dim3(nwg), dim3(WG), 0, 0, d, 20000u);
    CK(hipDeviceSynchronize());
    std::vector<unsigned> h(4ull * nw);
    CK(hipMemcpy(h.data(), d, 16ull * nw, hipMemcpyDeviceToHost));
    CK(hipFree(d));
    auto simd = [&](unsigned w) { return (h[4 * w] >> 4) & 3; };
    auto cu = [&](unsigned w) { return ((h[4 * w] >> 8) & 15) | (((h[4 * w] >> 13) & 7) << 4) | ((h[4 * w + 1] & 15) << 8); };
    const unsigned per = WG / 64;
    std::map<unsigned, unsigned> simd_of_slot[8];
    unsigned same1 = 0, same4 = 0, n1 = 0, n4 = 0, samecu = 0;
    for (unsigned b = 0; b < nwg; ++b)
        for (unsigned w = 0; w < per; ++w) {
            const unsigned g = b * per + w;
            simd_of_slot[w][simd(g)]++;
            if (cu(g) == cu(b * per)) ++samecu;
            if ((w ^ 1) < per && w < (w ^ 1)) { ++n1; same1 += simd(g) == simd(b * per + (w ^ 1)); }
            if ((w ^ 4) < per && w < (w ^ 4)) { ++n4; same4 += simd(g) == simd(b * per + (w ^ 4)); }
        }
    printf("{\"wg\": \"%s\", \"workgroups\": %u, \"waves_same_cu_as_wave0\": %.4f", name, nwg, (double)samecu / nw);
    printf(", \"pair_w_w^1_same_simd\": %.4f", n1 ? (double)same1 / n1 : -1.0);
    printf(", \"pair_w_w^4_same_simd\": %.4f", n4 ? (double)same4 / n4 : -1.0);
    printf(", \"simd_hist_by_wave\": [");
    for (unsigned w = 0; w < per; ++w) {
        printf("%s[", w ? ", " : "");
        for (unsigned s = 0; s < 4; ++s) printf("%s%u", s ? ", " : "", simd_of_slot[w][s]);
        printf("]");
    }
    printf("]}\n");
}

int main()
{
    // 32 KiB per one-pair workgroup (5 per CU), 40 KiB (4 per CU), 4 pairs with 128 KiB
    run<128, 8192>("128x32KiB", 256 * 5 * 4);
    run<128, 10240>("128x40KiB", 256 * 4 * 4);
    run<512, 32768>("512x128KiB", 256 * 4);
    run<256, 16384>("256x64KiB", 256 * 2 * 4);
    return 0;
}
