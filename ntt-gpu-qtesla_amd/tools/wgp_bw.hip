// wgp_bw.hip -- round-3 sweep of "T threads per n=2048 polynomial" shapes:
// how many threads share one polynomial (T = 512 / 256 / 128 / 64, i.e.
// C = 4 / 8 / 16 / 32 coefficients per lane), one polynomial per workgroup
// or persistent workgroups that prefetch the next polynomial into registers,
// with the LDS exchanges (one barrier each, double-buffered) and realistic
// lazy CT butterflies (7 VALU: v_sub/v_min, v_mul_hi, v_mul_lo, v_mad_u64,
// v_sub, v_add3 -- not foldable by the compiler) that a real kernel of that
// shape would run.  In place on 2^20 random polynomials (8 GiB).
// Diagnostic tool, never part of the product library.
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

__device__ __forceinline__ uint32_t ld(const uint32_t *p, bool nt) { return nt ? __builtin_nontemporal_load(p) : *p; }
__device__ __forceinline__ void st(uint32_t *p, uint32_t v, bool nt)
{
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// stages of one segment: radix-2 stages over the C registers (log2 C of them
// per segment, the last segment the rest of the 11), twiddles from `tw`
template <int C, int NS>
__device__ __forceinline__ void stages(uint32_t (&v)[C], const uint2 *tw)
{
    constexpr int LOGC = C == 4 ? 2 : C == 8 ? 3 : C == 16 ? 4 : 5;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int hh = C >> (1 + (s % LOGC));
#pragma unroll
        for (int j = 0; j < C; ++j)
            if ((j & hh) == 0) {
                const uint2 w = tw[(s * C + j) & 15];
                bfly(v[j], v[j + hh], w.x, w.y);
            }
    }
}

// MODE 0: one polynomial per workgroup (grid = npoly); per-lane twiddles
//         loaded from global memory (an L2-resident table) per polynomial.
// MODE 1: persistent, workgroup b owns polys [b ppw, (b+1) ppw), twiddles
//         loaded once, next polynomial prefetched into registers.
// MODE 2: persistent grid-stride, otherwise as MODE 1.
template <int T, int MODE, bool BF, bool NT>
__global__ __launch_bounds__(T) void k_wgp(uint32_t *buf, uint32_t npoly, uint32_t ppw, const uint2 *gtw)
{
    constexpr int C = 2048 / T;
    constexpr int XCH = T == 512 ? 5 : T == 256 ? 3 : T == 128 ? 2 : 1;
    constexpr int LOGC = C == 4 ? 2 : C == 8 ? 3 : C == 16 ? 4 : 5;
    __shared__ __attribute__((aligned(16))) uint32_t xb[T == 64 ? 1 : 2][2048];
    const uint32_t t = threadIdx.x;
    uint2 tw[16];
    auto load_tw = [&]() {
#pragma unroll
        for (int i = 0; i < 16; ++i) tw[i] = gtw[(t * 16 + i) & 4095];
    };
    auto load = [&](uint32_t (&v)[C], uint32_t p) {
        const uint32_t *s = buf + (size_t)p * 2048 + t;
#pragma unroll
        for (int e = 0; e < C; ++e) v[e] = ld(s + T * e, NT);
    };
    auto process = [&](uint32_t (&v)[C], uint32_t p) {
        int b = 0;
        if constexpr (BF) stages<C, LOGC>(v, tw);
#pragma unroll
        for (int x = 0; x < XCH; ++x) {
            uint32_t *xw = xb[T == 64 ? 0 : b];
            if (T == 64) {
                // one wave: the transposes need no barrier
#pragma unroll
                for (int e = 0; e < C; ++e) xw[t + T * e] = v[e];
                asm volatile("" ::: "memory");
#pragma unroll
                for (int e = 0; e < C; ++e) v[e] = xw[((t * C + e) + (t >> 1)) & 2047];
                asm volatile("" ::: "memory");
            } else {
#pragma unroll
                for (int e = 0; e < C; ++e) xw[t + T * e] = v[e];
                __syncthreads();
                const uint32_t r = (t * 37u) & (T - 1);
#pragma unroll
                for (int e = 0; e < C; ++e) v[e] = xw[r + T * e];
                b ^= 1;
            }
            if constexpr (BF) {
                constexpr int rest = 11 - LOGC;   // stages after the first segment
                if (x == XCH - 1) stages<C, rest - (XCH - 1) * LOGC>(v, tw);
                else stages<C, LOGC>(v, tw);
            }
        }
        uint32_t *d = buf + (size_t)p * 2048 + t;
#pragma unroll
        for (int e = 0; e < C; ++e) st(d + T * e, v[e], NT);
    };
    if constexpr (MODE == 0) {
        const uint32_t p = blockIdx.x;
        if (p >= npoly) return;
        uint32_t v[C];
        load(v, p);
        if constexpr (BF) load_tw();
        process(v, p);
    } else {
        if constexpr (BF) load_tw();
        uint32_t p = MODE == 1 ? blockIdx.x * ppw : blockIdx.x;
        const uint32_t end = MODE == 1 ? min(npoly, (blockIdx.x + 1) * ppw) : npoly;
        const uint32_t stride = MODE == 1 ? 1u : gridDim.x;
        if (p >= end) return;
        uint32_t v[C], nv[C];
        load(v, p);
        for (;;) {
            const uint32_t pn = p + stride;
            const bool more = pn < end;
            if (more) load(nv, pn);
            process(v, p);
            if (!more) break;
#pragma unroll
            for (int e = 0; e < C; ++e) v[e] = nv[e];
            p = pn;
            __syncthreads();   // the exchange buffers' last reads precede the next poly's writes
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

template <int W, int PER, bool NT>
__global__ __launch_bounds__(256) void k_flat(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * W * PER);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (size_t)(threadIdx.x & 63) * W;
    if constexpr (W == 4) {
        uint4 v = *reinterpret_cast<const uint4 *>(p);
        asm volatile("" ::: "memory");
        *reinterpret_cast<uint4 *>(p) = v;
    } else {
        uint32_t v[PER];
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = ld(p + 64 * i, NT);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < PER; ++i) st(p + 64 * i, v[i], NT);
    }
}

int main(int argc, char **argv)
{
    const uint32_t npoly = 1u << 20;
    const size_t nwords = (size_t)npoly * 2048;
    const size_t bytes = nwords * 4;
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const char *only = argc > 2 ? argv[2] : nullptr;
    uint32_t *a;
    uint2 *gtw;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&gtw, 4096 * sizeof(uint2)));
    {
        std::vector<uint2> h(4096);
        for (int i = 0; i < 4096; ++i) {
            const uint32_t w = (uint32_t)((1103515245ull * (i + 1)) % Q);
            h[i] = make_uint2(0u - w, (uint32_t)(((uint64_t)w << 32) / Q));
        }
        CK(hipMemcpy(gtw, h.data(), 4096 * sizeof(uint2), hipMemcpyHostToDevice));
    }
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, nwords);
    CK(hipDeviceSynchronize());
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::pair<std::string, std::function<void()>>> cases;
    auto add = [&](const std::string &name, std::function<void()> fn) {
        if (only && !strstr(name.c_str(), only)) return;
        cases.emplace_back(name, fn);
    };
    char nm[160];
#define WGP(T, MODE, BF, NT)                                                                                     \
    {                                                                                                            \
        int occ = 0;                                                                                             \
        CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void *)k_wgp<T, MODE, BF, NT>, T, 0));      \
        const uint32_t grid = MODE == 0 ? npoly : (uint32_t)(occ * cus);                                         \
        const uint32_t ppw = (npoly + grid - 1) / grid;                                                          \
        snprintf(nm, sizeof nm, "wgp T=%d mode=%d bf=%d nt=%d (wg/cu=%d)", T, MODE, BF, NT, occ);               \
        add(nm, [=] { hipLaunchKernelGGL((k_wgp<T, MODE, BF, NT>), dim3(grid), dim3(T), 0, 0, a, npoly, ppw, gtw); }); \
    }
#define WGP4(T)               \
    WGP(T, 0, false, false)   \
    WGP(T, 0, true, false)    \
    WGP(T, 0, true, true)     \
    WGP(T, 1, false, false)   \
    WGP(T, 1, true, false)    \
    WGP(T, 1, true, true)     \
    WGP(T, 2, true, false)
    WGP4(512)
    WGP4(256)
    WGP4(128)
    WGP4(64)
#define FLAT(W, PER, NT)                                                                                         \
    snprintf(nm, sizeof nm, "flat W=%d per=%d nt=%d", W, PER, NT);                                               \
    add(nm, [=] {                                                                                                \
        const unsigned grid = (unsigned)(nwords / (64 * W * PER) / 4);                                           \
        hipLaunchKernelGGL((k_flat<W, PER, NT>), dim3(grid), dim3(256), 0, 0, a, nwords);                       \
    });
    FLAT(4, 1, false)
    FLAT(1, 4, false)
    FLAT(1, 4, true)
    FLAT(1, 8, true)
    FLAT(1, 32, true)

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
        printf("%-48s med %7.3f ms  min %7.3f ms  %6.0f GB/s\n", cases[i].first.c_str(), med, v[0], 2.0 * bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
