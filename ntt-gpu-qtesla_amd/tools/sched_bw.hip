// sched_bw.hip -- memory-schedule sweep for the transform kernels' access
// shape (round 3): which way of walking 2^20 n=2048 polynomials (8 GiB, in
// place, random words) streams HBM fastest, with and without a synthetic
// per-unit VALU load between the loads and the stores.  Candidates:
//   burst  non-persistent grid, each wave copies one contiguous block of PER
//          wave-instructions of W dwords per lane (W=4 PER=1: the flat float4
//          copy; W=1 PER=32: one 8 KiB polynomial per wave)
//   chunk  the library's schedule: persistent 8-wave workgroups (80 KiB LDS
//          -> 2 per CU), workgroup b owns units [8 b ppw, 8 (b+1) ppw)
//   deq    persistent 8-wave workgroups (same LDS pin), every wave takes its
//          next unit from one of 8 ticket counters (blockIdx % 8) that hand
//          out 64 KiB groups in address order: the window of units in flight
//          stays as narrow as the dispatch-ordered grid's, the workgroup's
//          table prologue is paid once
//   wgpoly one 8 KiB polynomial per 512-thread workgroup, one dwordx4 per
//          lane in and out with an LDS transpose between (block-per-poly)
// plus the library's own poly_ntt / poly_invntt on the same buffer.
// Diagnostic tool, never part of the product library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/qtesla_ntt.h"

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(2);                                                               \
        }                                                                          \
    } while (0)

constexpr uint32_t NWORDS_POLY = 2048;

// synthetic per-unit VALU work on the 32 loaded words (ITER rounds of a
// multiply-add per word, data-dependent so the stores wait for it)
template <int ITER>
__device__ __forceinline__ void work32(uint32_t (&v)[32])
{
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = v[j] * 0x9E3779B1u + (uint32_t)k;
    }
}

template <bool NT>
__device__ __forceinline__ uint32_t ld(const uint32_t *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(uint32_t *p, uint32_t v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// ---- burst: non-persistent, per-wave contiguous blocks --------------------
template <int W, int PER, int WPB, bool NT, int ITER>
__global__ __launch_bounds__(64 * WPB) void k_burst(uint32_t *buf, size_t nwords)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63;
    const size_t wave = (size_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * W * PER);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (size_t)lane * W;
    constexpr int R = W * PER;
    uint32_t v[R < 32 ? 32 : R];
#pragma unroll
    for (int i = 0; i < PER; ++i)
#pragma unroll
        for (int e = 0; e < W; ++e) v[i * W + e] = 0;
    if constexpr (W == 4) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const uint4 x = *reinterpret_cast<const uint4 *>(p + i * 64 * W);
            v[4 * i] = x.x, v[4 * i + 1] = x.y, v[4 * i + 2] = x.z, v[4 * i + 3] = x.w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < PER; ++i) v[i] = ld<NT>(p + i * 64);
    }
    asm volatile("" ::: "memory");   // all loads issued before any store (the kernels' shape)
    if constexpr (R == 32) work32<ITER>(*reinterpret_cast<uint32_t(*)[32]>(v));
    if constexpr (W == 4) {
#pragma unroll
        for (int i = 0; i < PER; ++i)
            *reinterpret_cast<uint4 *>(p + i * 64 * W) = make_uint4(v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]);
    } else {
#pragma unroll
        for (int i = 0; i < PER; ++i) st<NT>(p + i * 64, v[i]);
    }
    if (nwords == 1) dyn[threadIdx.x] = v[0];   // never: keeps the dynamic LDS pin
}

// one 8 KiB unit per wave, dword accesses at stride 256 B (the transforms' shape)
template <bool NT, int ITER>
__device__ __forceinline__ void unit_copy(uint32_t *buf, uint32_t u, uint32_t lane)
{
    uint32_t *p = buf + (size_t)u * NWORDS_POLY + lane;
    uint32_t v[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = ld<NT>(p + 64 * j);
    asm volatile("" ::: "memory");   // all loads issued before any store (the kernels' shape)
    work32<ITER>(v);
#pragma unroll
    for (int j = 0; j < 32; ++j) st<NT>(p + 64 * j, v[j]);
}

// ---- chunk: the library's schedule ---------------------------------------
template <bool NT, int ITER, int WPB = 8>
__global__ __launch_bounds__(64 * WPB) void k_chunk(uint32_t *buf, uint32_t nunits, uint32_t ppw)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t u = blockIdx.x * WPB * ppw + w;
    for (uint32_t i = 0; i < ppw; ++i, u += WPB) {
        if (u >= nunits) break;
        unit_copy<NT, ITER>(buf, u, lane);
    }
    if (nunits == 0) dyn[threadIdx.x] = 0;
}

// chunk schedule, software-pipelined: unit i+1's loads are issued before unit
// i's stores (one vmcnt counts both on gfx9-family, so in the plain loop the
// first wait for unit i+1's data also waits for unit i's store acks)
template <bool NT, int ITER>
__global__ __launch_bounds__(512) void k_chunk_pipe(uint32_t *buf, uint32_t nunits, uint32_t ppw)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t u = blockIdx.x * 8 * ppw + w;
    if (u >= nunits) return;
    uint32_t cur[32], nxt[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) cur[j] = ld<NT>(buf + (size_t)u * NWORDS_POLY + lane + 64 * j);
    for (uint32_t i = 0; i < ppw; ++i, u += 8) {
        const bool more = i + 1 < ppw && u + 8 < nunits;
        if (more) {
#pragma unroll
            for (int j = 0; j < 32; ++j) nxt[j] = ld<NT>(buf + (size_t)(u + 8) * NWORDS_POLY + lane + 64 * j);
        }
        work32<ITER>(cur);
        uint32_t *p = buf + (size_t)u * NWORDS_POLY + lane;
#pragma unroll
        for (int j = 0; j < 32; ++j) st<NT>(p + 64 * j, cur[j]);
        if (!more) break;
#pragma unroll
        for (int j = 0; j < 32; ++j) cur[j] = nxt[j];
    }
    if (nunits == 0) dyn[threadIdx.x] = 0;
}

// ---- grid-stride persistent -----------------------------------------------
template <bool NT, int ITER>
__global__ __launch_bounds__(512) void k_stride(uint32_t *buf, uint32_t nunits)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint32_t u = blockIdx.x * 8 + w; u < nunits; u += gridDim.x * 8) unit_copy<NT, ITER>(buf, u, lane);
    if (nunits == 0) dyn[threadIdx.x] = 0;
}

// ---- deq: ticketed persistent ---------------------------------------------
// counter c (c = blockIdx % 8, 128 B apart) hands out tickets t = 0, 1, ...;
// ticket t of counter c is unit ((t >> 3) * 8 + c) * 8 + (t & 7): 64 KiB
// groups striped over the counters in address order.  Every unit is taken by
// exactly one wave; a wave leaves at its first ticket past the end (the
// tickets of one counter are monotonic, so all later ones are past it too).
template <bool NT, int ITER, int GROUP>
__global__ __launch_bounds__(512) void k_deq(uint32_t *buf, uint32_t nunits, uint32_t *ctr)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x & 7;
    uint32_t *my = ctr + 32 * c;
    auto unit_of = [&](uint32_t t) { return ((t / GROUP) * 8 + c) * GROUP + (t % GROUP); };
    auto grab = [&]() {
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(my, 1u);
        return __builtin_amdgcn_readfirstlane(t);
    };
    uint32_t t = grab();
    for (;;) {
        const uint32_t u = unit_of(t);
        if (u >= nunits) break;
        const uint32_t tn = grab();   // next ticket requested before this unit's work
        unit_copy<NT, ITER>(buf, u, lane);
        t = tn;
    }
    if (nunits == 0) dyn[threadIdx.x] = 0;
}


// ---- sync-stride: persistent grid-stride with bounded drift ----------------
// step i of workgroup b is unit i * G8 + 8 b + w (one contiguous window of the
// whole grid per step); after a step lane 0 of wave 0 adds 1 to the global
// count of finished workgroup-steps, and before step i a workgroup waits
// (bounded spin) until the grid has finished step i - K (count >= (i-K+1) G):
// the window in flight then spans at most K+1 steps of the grid
template <bool NT, int ITER, int K>
__global__ __launch_bounds__(512) void k_sync_stride(uint32_t *buf, uint32_t nunits, uint32_t *done)
{
    extern __shared__ uint32_t dyn[];
    const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t G = gridDim.x, G8 = G * 8;
    for (uint32_t i = 0;; ++i) {
        const uint32_t u = i * G8 + blockIdx.x * 8 + w;
        if (i * G8 >= nunits) break;
        if (i > K) {
            if (threadIdx.x == 0) {
                const uint32_t need = (i - K) * G;
                for (uint32_t spin = 0; spin < (1u << 20); ++spin) {
                    if (__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= need) break;
                    __builtin_amdgcn_s_sleep(2);
                }
            }
            __syncthreads();
        }
        if (u < nunits) unit_copy<NT, ITER>(buf, u, lane);
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (nunits == 0) dyn[threadIdx.x] = 0;
}

// ---- wgpoly: one polynomial per 512-thread workgroup ----------------------
template <int ITER>
__global__ __launch_bounds__(512) void k_wgpoly(uint32_t *buf, uint32_t nunits)
{
    __shared__ __attribute__((aligned(16))) uint32_t t[2048 + 64];
    const uint32_t u = blockIdx.x;
    if (u >= nunits) return;
    uint4 *p = reinterpret_cast<uint4 *>(buf + (size_t)u * NWORDS_POLY) + threadIdx.x;
    uint4 x = *p;
    asm volatile("" ::: "memory");
    // transpose-like exchange: thread i writes 4 words, reads 4 words of a rotated row
    const uint32_t i = threadIdx.x;
    t[4 * i + 0 + (i >> 4)] = x.x;
    t[4 * i + 1 + (i >> 4)] = x.y;
    t[4 * i + 2 + (i >> 4)] = x.z;
    t[4 * i + 3 + (i >> 4)] = x.w;
    __syncthreads();
    const uint32_t k = (i * 37u) & 511u;
    uint32_t v[4] = {t[4 * k + 0 + (k >> 4)], t[4 * k + 1 + (k >> 4)], t[4 * k + 2 + (k >> 4)], t[4 * k + 3 + (k >> 4)]};
#pragma unroll
    for (int r = 0; r < ITER * 8; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = v[j] * 0x9E3779B1u + (uint32_t)r;
    __syncthreads();
    t[4 * k + 0 + (k >> 4)] = v[0];
    t[4 * k + 1 + (k >> 4)] = v[1];
    t[4 * k + 2 + (k >> 4)] = v[2];
    t[4 * k + 3 + (k >> 4)] = v[3];
    __syncthreads();
    *p = make_uint4(t[4 * i + 0 + (i >> 4)], t[4 * i + 1 + (i >> 4)], t[4 * i + 2 + (i >> 4)], t[4 * i + 3 + (i >> 4)]);
}

__global__ void k_rand(uint32_t *x, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        x[i] = (uint32_t)((((z ^ (z >> 31)) >> 32) * 856145921ull) >> 32);
    }
}

int main(int argc, char **argv)
{
    const uint32_t npoly = 1u << 20;
    const size_t nwords = (size_t)npoly * NWORDS_POLY;
    const size_t bytes = nwords * 4;
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const char *only = argc > 2 ? argv[2] : nullptr;
    uint32_t *a, *ctr;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&ctr, 8 * 128));
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, nwords);
    CK(hipDeviceSynchronize());
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));

    struct Case {
        const char *name;
        std::function<void()> fn;
    };
    std::vector<std::pair<std::string, std::function<void()>>> cases;
    auto add = [&](const std::string &name, std::function<void()> fn) {
        if (only && !strstr(name.c_str(), only)) return;
        cases.emplace_back(name, fn);
    };
    const uint32_t LDS80 = 80 * 1024;
    char nm[160];
#define BURST(W, PER, WPB, NT, ITER, LDS)                                                                       \
    snprintf(nm, sizeof nm, "burst W=%d per=%d wpb=%d nt=%d iter=%d lds=%uK", W, PER, WPB, NT, ITER, (LDS) / 1024); \
    add(nm, [=] {                                                                                                \
        const size_t per_wave = (size_t)64 * W * PER;                                                            \
        const unsigned grid = (unsigned)((nwords / per_wave + WPB - 1) / WPB);                                   \
        hipLaunchKernelGGL((k_burst<W, PER, WPB, NT, ITER>), dim3(grid), dim3(64 * WPB), LDS, 0, a, nwords);    \
    });
    // flat copies: access width and per-wave burst length
#define CHUNK(NT, ITER, PPW)                                                                                     \
    snprintf(nm, sizeof nm, "chunk nt=%d iter=%d ppw=%d lds=80K", NT, ITER, PPW);                               \
    add(nm, [=] {                                                                                                \
        const uint32_t grid = (npoly + 8 * PPW - 1) / (8 * PPW);                                                 \
        hipLaunchKernelGGL((k_chunk<NT, ITER>), dim3(grid), dim3(512), LDS80, 0, a, npoly, (uint32_t)PPW);     \
    });
// the chunk schedule at other occupancies: WPB waves per workgroup, LDSK KiB
// pinned per workgroup (round 3, session 2: would smaller transpose buffers pay?)
#define CHUNKX(NT, ITER, PPW, WPB, LDSK)                                                                         \
    snprintf(nm, sizeof nm, "chunkx nt=%d iter=%d ppw=%d wpb=%d lds=%dK", NT, ITER, PPW, WPB, LDSK);            \
    add(nm, [=] {                                                                                                \
        const uint32_t grid = (npoly + WPB * PPW - 1) / (WPB * PPW);                                             \
        hipLaunchKernelGGL((k_chunk<NT, ITER, WPB>), dim3(grid), dim3(64 * WPB), (LDSK) * 1024, 0, a, npoly, (uint32_t)PPW); \
    });
#define STRIDE(NT, ITER)                                                                                         \
    snprintf(nm, sizeof nm, "stride nt=%d iter=%d lds=80K", NT, ITER);                                          \
    add(nm, [=] { hipLaunchKernelGGL((k_stride<NT, ITER>), dim3(2 * cus), dim3(512), LDS80, 0, a, npoly); });
#define DEQ(NT, ITER, G, WGPC)                                                                                   \
    snprintf(nm, sizeof nm, "deq nt=%d iter=%d group=%d wg/cu=%d", NT, ITER, G, WGPC);                          \
    add(nm, [=] {                                                                                                \
        CK(hipMemsetAsync(ctr, 0, 8 * 128, 0));                                                                  \
        hipLaunchKernelGGL((k_deq<NT, ITER, G>), dim3(WGPC * cus), dim3(512), (WGPC == 2 ? LDS80 : 40 * 1024), 0, a, npoly, ctr); \
    });
#define WGPOLY(ITER)                                                                                             \
    snprintf(nm, sizeof nm, "wgpoly iter=%d", ITER);                                                             \
    add(nm, [=] { hipLaunchKernelGGL((k_wgpoly<ITER>), dim3(npoly), dim3(512), 0, 0, a, npoly); });

#define SSTR(NT, ITER, K)                                                                                        \
    snprintf(nm, sizeof nm, "sync-stride nt=%d iter=%d K=%d lds=80K", NT, ITER, K);                            \
    add(nm, [=] {                                                                                                \
        CK(hipMemsetAsync(ctr, 0, 8 * 128, 0));                                                                  \
        hipLaunchKernelGGL((k_sync_stride<NT, ITER, K>), dim3(2 * cus), dim3(512), LDS80, 0, a, npoly, ctr);    \
    });
#define CHUNKP(NT, ITER, PPW)                                                                                    \
    snprintf(nm, sizeof nm, "chunk-pipe nt=%d iter=%d ppw=%d lds=80K", NT, ITER, PPW);                          \
    add(nm, [=] {                                                                                                \
        const uint32_t grid = (npoly + 8 * PPW - 1) / (8 * PPW);                                                 \
        hipLaunchKernelGGL((k_chunk_pipe<NT, ITER>), dim3(grid), dim3(512), LDS80, 0, a, npoly, (uint32_t)PPW); \
    });
    if (getenv("SCHED_PIPE")) {
        CHUNKP(true, 0, 16)
        CHUNKP(true, 0, 4)
        CHUNKP(true, 20, 16)
        CHUNKP(true, 40, 16)
        CHUNK(true, 20, 16)
        CHUNK(true, 40, 16)
    }
    if (getenv("SCHED_OCC")) {
        CHUNKX(true, 0, 16, 8, 80)
        CHUNKX(true, 0, 4, 8, 80)
        CHUNKX(true, 0, 16, 8, 48)
        CHUNKX(true, 0, 4, 8, 48)
        CHUNKX(true, 0, 16, 10, 56)
        CHUNKX(true, 0, 4, 10, 56)
        CHUNKX(true, 0, 16, 8, 40)
        CHUNKX(true, 0, 4, 8, 40)
        CHUNKX(true, 0, 16, 4, 32)
        CHUNKX(true, 20, 16, 8, 80)
        CHUNKX(true, 20, 16, 8, 48)
        CHUNKX(true, 20, 16, 10, 56)
        CHUNKX(true, 40, 16, 8, 80)
        CHUNKX(true, 40, 16, 8, 48)
        CHUNKX(true, 40, 16, 10, 56)
    } else {
    SSTR(true, 0, 1)
    SSTR(true, 0, 2)
    SSTR(true, 0, 4)
    SSTR(true, 0, 16)
    }
    CHUNK(true, 0, 16)
    CHUNK(true, 0, 4)
    STRIDE(true, 0)
    BURST(4, 1, 4, false, 0, 0)
    BURST(1, 32, 8, true, 0, 0)
    add("lib poly_ntt p-III", [=] {
        const int rc = poly_ntt(a, nullptr, npoly, NTT_PARAM_P_III, nullptr);
        if (rc) { fprintf(stderr, "poly_ntt rc=%d\n", rc); exit(3); }
    });
    add("lib poly_invntt p-III", [=] {
        const int rc = poly_invntt(a, nullptr, npoly, NTT_PARAM_P_III, nullptr);
        if (rc) { fprintf(stderr, "poly_invntt rc=%d\n", rc); exit(3); }
    });

    for (auto &c : cases) c.second();
    CK(hipDeviceSynchronize());
    std::vector<std::vector<float>> t(cases.size());
    for (int r = 0; r < rounds; ++r) {
        for (size_t i = 0; i < cases.size(); ++i) {
            CK(hipEventRecord(e0, 0));
            cases[i].second();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[i].push_back(ms);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    for (size_t i = 0; i < cases.size(); ++i) {
        auto v = t[i];
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-48s med %7.3f ms  min %7.3f ms  %6.0f GB/s\n", cases[i].first.c_str(), med, v[0], 2.0 * bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
