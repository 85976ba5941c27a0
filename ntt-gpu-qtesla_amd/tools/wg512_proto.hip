// wg512_proto.hip -- round-3 prototype timing of a "workgroup per
// polynomial" transform for n = 2048: 512 threads x 4 coefficients, one
// dword load and store per coefficient (1 KiB per wave-instruction group, the
// access shape that streams at the flat-copy rate), 6 radix-4 / radix-2
// passes separated by 5 LDS exchanges (double-buffered, one barrier each),
// lazy CT butterflies with twiddles read from a per-workgroup LDS table.
// Not the exact arithmetic of the transform -- the same instruction mix, to
// decide the design before writing it.  Diagnostic tool, never in the product.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            exit(2);                                                                   \
        }                                                                              \
    } while (0)

constexpr uint32_t Q = 856145921u;

__device__ __forceinline__ void bfly(uint32_t &x, uint32_t &y, uint32_t wn, uint32_t wp)
{
    const uint32_t a = min(x, x - 2 * Q);
    const uint32_t qe = __umulhi(y, wp);
    const uint32_t tn = (uint32_t)((uint64_t)qe * Q + y * wn);
    x = a - tn;
    y = a + tn + 2 * Q;
}

// TWSRC 0: per-workgroup LDS table filled from global per polynomial;
//       1: table filled once (persistent); 2: no table (uniform twiddles only)
// MODE 0: one polynomial per workgroup; 1: persistent grid-stride with the
//         next polynomial's 4 words prefetched; 2: persistent, no compute
// PPWG: polynomials per workgroup (T = 512 PPWG threads)
template <int MODE, int TWSRC, int PPWG, bool COMPUTE>
__global__ __launch_bounds__(512 * PPWG) void k_proto(uint32_t *buf, uint32_t npoly, const uint4 *gtab, uint32_t w0, uint32_t w1)
{
    __shared__ __attribute__((aligned(16))) uint32_t tab[TWSRC == 2 ? 4 : 4096];   // 2048 (w, w') pairs
    __shared__ __attribute__((aligned(16))) uint32_t xb[PPWG][2][2048 + 64];
    const uint32_t tid = threadIdx.x, sub = tid >> 9, t = tid & 511;
    const uint32_t lane = t & 63, wv = t >> 6;
    // per-thread constant LDS addresses (write side: [e][t] rows; read side: a
    // transposing pattern with a per-pass rotation against bank conflicts)
    uint32_t ra[5];
#pragma unroll
    for (int x = 0; x < 5; ++x) ra[x] = ((t * (4u << x) + (t >> (6 - x))) & 511u) + ((t >> 7) & 3) * 0;
    auto fill = [&]() {
        if constexpr (TWSRC != 2) {
            const uint4 *s = gtab + tid;
            uint4 *d = reinterpret_cast<uint4 *>(tab) + tid;
#pragma unroll
            for (int i = 0; i < 2 / PPWG; ++i) d[512 * PPWG * i] = s[512 * PPWG * i];
        }
    };
    auto process = [&](uint32_t (&v)[4], uint32_t p) {
        if constexpr (COMPUTE) {
            bfly(v[0], v[2], w0, w1);
            bfly(v[1], v[3], w0, w1);
            bfly(v[0], v[1], w0 + 1, w1);
            bfly(v[2], v[3], w0 + 2, w1);
        }
        int b = 0;
#pragma unroll
        for (int x = 0; x < 5; ++x) {
            uint32_t *xw = xb[sub][b];
#pragma unroll
            for (int e = 0; e < 4; ++e) xw[t + 512 * e + (e << 4)] = v[e];
            __syncthreads();
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = xw[ra[x] + 512 * e + (e << 4)];
            b ^= 1;
            if constexpr (COMPUTE) {
                uint2 wa, wb, wc;
                if constexpr (TWSRC == 2) {
                    wa = make_uint2(w0 + x, w1);
                    wb = make_uint2(w0 + 2 * x, w1);
                    wc = make_uint2(w0 + 3 * x, w1);
                } else {
                    const uint2 *tw = reinterpret_cast<const uint2 *>(tab);
                    const uint32_t k = (t >> (5 - x)) + (1u << (2 * x + 1));
                    wa = tw[k & 2047];
                    wb = tw[(2 * k) & 2047];
                    wc = tw[(2 * k + 1) & 2047];
                }
                if (x < 4) {
                    bfly(v[0], v[2], wa.x, wa.y);
                    bfly(v[1], v[3], wa.x, wa.y);
                    bfly(v[0], v[1], wb.x, wb.y);
                    bfly(v[2], v[3], wc.x, wc.y);
                } else {
                    bfly(v[0], v[1], wb.x, wb.y);
                    bfly(v[2], v[3], wc.x, wc.y);
                }
            }
        }
        uint32_t *d = buf + (size_t)p * 2048 + t;
#pragma unroll
        for (int e = 0; e < 4; ++e) __builtin_nontemporal_store(COMPUTE ? min(v[e], v[e] - Q) : v[e], d + 512 * e);
    };
    auto load = [&](uint32_t (&v)[4], uint32_t p) {
        const uint32_t *s = buf + (size_t)p * 2048 + t;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = __builtin_nontemporal_load(s + 512 * e);
    };
    if constexpr (MODE == 0) {
        const uint32_t p = blockIdx.x * PPWG + sub;
        uint32_t v[4];
        if (p < npoly) load(v, p);
        if constexpr (TWSRC == 0) {
            fill();
            __syncthreads();
        }
        if (p < npoly) process(v, p);   // npoly is a multiple of PPWG here (barriers)
    } else {
        if constexpr (TWSRC != 2) {
            fill();
            __syncthreads();
        }
        uint32_t p = blockIdx.x * PPWG + sub;
        const uint32_t stride = gridDim.x * PPWG;
        if (p >= npoly) return;   // grid <= npoly / PPWG: never for whole workgroups
        uint32_t v[4], nv[4];
        load(v, p);
        for (;;) {
            const uint32_t pn = p + stride;
            const bool more = pn < npoly;
            if (more) load(nv, pn);
            process(v, p);
            if (!more) break;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = nv[e];
            p = pn;
        }
    }
}

__global__ void k_rand(uint32_t *x, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        x[i] = (uint32_t)((((z ^ (z >> 31)) >> 32) * (uint64_t)Q) >> 32);
    }
}

int main(int argc, char **argv)
{
    const uint32_t npoly = 1u << 20;
    const size_t nwords = (size_t)npoly * 2048;
    const size_t bytes = nwords * 4;
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    uint32_t *a;
    uint4 *gtab;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&gtab, 16384));
    {
        std::vector<uint32_t> h(4096);
        for (int i = 0; i < 2048; ++i) {
            const uint32_t w = (uint32_t)((1103515245ull * (i + 1)) % Q);
            h[2 * i] = 0u - w;
            h[2 * i + 1] = (uint32_t)(((uint64_t)w << 32) / Q);
        }
        CK(hipMemcpy(gtab, h.data(), 16384, hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, nwords);
    CK(hipDeviceSynchronize());
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::pair<std::string, std::function<void()>>> cases;
    char nm[160];
    const uint32_t w0 = 123456789u, w1 = 987654u;
#define PROTO(MODE, TWSRC, PPWG, COMP)                                                                          \
    {                                                                                                           \
        int occ = 0;                                                                                            \
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_proto<MODE, TWSRC, PPWG, COMP>, 512 * PPWG, 0)); \
        const uint32_t grid = MODE == 0 ? npoly / PPWG : (uint32_t)(occ * cus);                                 \
        snprintf(nm, sizeof nm, "proto mode=%d tw=%d ppwg=%d compute=%d (wg/cu=%d)", MODE, TWSRC, PPWG, COMP, occ); \
        cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_proto<MODE, TWSRC, PPWG, COMP>), dim3(grid), dim3(512 * PPWG), 0, 0, a, npoly, gtab, w0, w1); }); \
    }
    PROTO(0, 2, 1, false)
    PROTO(0, 2, 1, true)
    PROTO(0, 0, 1, false)
    PROTO(0, 0, 1, true)
    PROTO(0, 0, 2, true)
    PROTO(1, 1, 1, false)
    PROTO(1, 1, 1, true)
    PROTO(1, 2, 1, true)
    PROTO(1, 1, 2, true)

    for (auto &c : cases) c.second();
    CK(hipDeviceSynchronize());
    std::vector<std::vector<float>> tm(cases.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < cases.size(); ++i) {
            CK(hipEventRecord(e0, 0));
            cases[i].second();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            tm[i].push_back(ms);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    CK(hipGetLastError());
    for (size_t i = 0; i < cases.size(); ++i) {
        auto v = tm[i];
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-52s med %7.3f ms  min %7.3f ms  %6.0f GB/s\n", cases[i].first.c_str(), med, v[0], 2.0 * bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
