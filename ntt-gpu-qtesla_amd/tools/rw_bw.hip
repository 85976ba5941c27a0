// rw_bw.hip -- round-3 attribution of the "bytes per wave" effect seen in
// sched_bw / wgp_bw (one 8 KiB burst per wave streams ~11 % slower than
// 1 KiB per wave): read-only and write-only streams of 8 GiB with P
// wave-instructions per wave, and copies whose 32 loads per wave are issued in
// groups (each group waited for before the next is issued).  Non-persistent
// grids of 256-thread workgroups.  Diagnostic tool, never part of the product.
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

// read-only: P dword loads per lane (stride 256 B), xor-reduced; one store per
// wave into a small sink so nothing is optimised away
template <int P, bool NT>
__global__ __launch_bounds__(256) void k_read(const uint32_t *buf, size_t nwords, uint32_t *sink)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * P);
    if (base >= nwords) return;
    const uint32_t *p = buf + base + (threadIdx.x & 63);
    uint32_t v[P];
#pragma unroll
    for (int i = 0; i < P; ++i) v[i] = NT ? __builtin_nontemporal_load(p + 64 * i) : p[64 * i];
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < P; ++i) x ^= v[i];
    if (x == 0x12345678u) sink[threadIdx.x] = x;   // practically never
}

template <int P, bool NT>
__global__ __launch_bounds__(256) void k_write(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * P);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const uint32_t v = (uint32_t)(base + i) ^ threadIdx.x;
        if (NT) __builtin_nontemporal_store(v, p + 64 * i);
        else p[64 * i] = v;
    }
}

// copy of 32 dwords per lane, loads issued in groups of G, each group waited
// for (s_waitcnt vmcnt(0)) before the next group is issued
template <int G, bool NT>
__global__ __launch_bounds__(256) void k_copy_grouped(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * 32);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
    uint32_t v[32];
#pragma unroll
    for (int g = 0; g < 32 / G; ++g) {
#pragma unroll
        for (int i = 0; i < G; ++i) v[g * G + i] = NT ? __builtin_nontemporal_load(p + 64 * (g * G + i)) : p[64 * (g * G + i)];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        if (NT) __builtin_nontemporal_store(v[i], p + 64 * i);
        else p[64 * i] = v[i];
    }
}

// copy of 32 dwords per lane whose stores are issued in groups of G, each
// group drained before the next
template <int G, bool NT>
__global__ __launch_bounds__(256) void k_copy_stgrouped(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * 32);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = NT ? __builtin_nontemporal_load(p + 64 * i) : p[64 * i];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int g = 0; g < 32 / G; ++g) {
#pragma unroll
        for (int i = 0; i < G; ++i) {
            if (NT) __builtin_nontemporal_store(v[g * G + i], p + 64 * (g * G + i));
            else p[64 * (g * G + i)] = v[g * G + i];
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
}


// write-only, 32 dword stores per wave, chunks interleaved over the WPB waves
// of a workgroup: wave w stores 256-B chunk w + WPB i (i = 0..31) of the
// workgroup's 8 WPB KiB region, so consecutive waves write adjacent chunks
template <int WPB, bool NT>
__global__ __launch_bounds__(64 * WPB) void k_write_il(uint32_t *buf, size_t nwords)
{
    const size_t base = (size_t)blockIdx.x * (2048 * WPB);
    if (base >= nwords) return;
    const uint32_t w = threadIdx.x >> 6;
    uint32_t *p = buf + base + 64 * w + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        const uint32_t v = (uint32_t)(base + i) ^ threadIdx.x;
        if (NT) __builtin_nontemporal_store(v, p + 64 * WPB * i);
        else p[64 * WPB * i] = v;
    }
}

// write-only, 32 dword stores per wave in 8 groups of 4 separated by s_sleep(S)
template <int S, bool NT>
__global__ __launch_bounds__(256) void k_write_spread(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)2048;
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t v = (uint32_t)(base + g * 4 + i) ^ threadIdx.x;
            if (NT) __builtin_nontemporal_store(v, p + 64 * (4 * g + i));
            else p[64 * (4 * g + i)] = v;
        }
        __builtin_amdgcn_s_sleep(S);
    }
}

// write-only, 8 dwordx4 stores per wave (8 KiB)
__global__ __launch_bounds__(256) void k_write_x4(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)2048;
    if (base >= nwords) return;
    uint4 *p = reinterpret_cast<uint4 *>(buf + base) + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 8; ++i) p[64 * i] = make_uint4(i, threadIdx.x, (uint32_t)base, 7);
}

// copy, one 8 KiB polynomial per wave (nt loads), 8-wave workgroups, results
// through LDS: each wave writes its polynomial to its LDS buffer, barrier,
// then wave w stores 256-B chunks w + 8 i of the workgroup's 64 KiB block
// (adjacent chunks from consecutive waves), barrier before the buffers are
// reused.  PPW polynomials per wave (PPW = 1: non-persistent).  STNT: nt stores.
template <int PPW, bool STNT>
__global__ __launch_bounds__(512) void k_copy_lds_il(uint32_t *buf, uint32_t npoly)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[8 * 2048 + 4096];   // + 16 KiB: the tables' share
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (npoly == 0xFFFFFFFFu) lds[16384 + threadIdx.x] = 0;   // never
    for (uint32_t it = 0; it < PPW; ++it) {
        const uint32_t p0 = (blockIdx.x * PPW + it) * 8;   // first poly of the step
        if (p0 >= npoly) break;
        const uint32_t *s = buf + (size_t)(p0 + w) * 2048 + lane;
        uint32_t v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(s + 64 * j);
#pragma unroll
        for (int j = 0; j < 32; ++j) lds[w * 2048 + 64 * j + lane] = v[j];
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = lds[(w + 8 * i) * 64 + lane];
        uint32_t *d = buf + (size_t)p0 * 2048 + 64 * w + lane;
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            if (STNT) __builtin_nontemporal_store(v[i], d + 512 * i);
            else d[512 * i] = v[i];
        }
        __syncthreads();
    }
}

// baseline copy, one 8 KiB polynomial per wave, 8-wave workgroups, same LDS
// pin as k_copy_lds_il, nt loads, stores nt or not
template <int PPW, bool STNT>
__global__ __launch_bounds__(512) void k_copy_pw(uint32_t *buf, uint32_t npoly)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[8 * 2048 + 4096];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (npoly == 0xFFFFFFFFu) {
        lds[threadIdx.x] = 0;
        __syncthreads();
        buf[threadIdx.x] = lds[threadIdx.x ^ 1];
    }
    for (uint32_t it = 0; it < PPW; ++it) {
        const uint32_t p = (blockIdx.x * PPW + it) * 8 + w;
        if (p >= npoly) break;
        uint32_t *s = buf + (size_t)p * 2048 + lane;
        uint32_t v[32];
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = __builtin_nontemporal_load(s + 64 * j);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int j = 0; j < 32; ++j) {
            if (STNT) __builtin_nontemporal_store(v[j], s + 64 * j);
            else s[64 * j] = v[j];
        }
    }
}

// store with explicit cache-policy bits (gfx950 global_store_dword modifiers)
template <int POL>
__device__ __forceinline__ void st_pol(uint32_t *p, uint32_t v)
{
    if constexpr (POL == 0) asm volatile("global_store_dword %0, %1, off" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 1) asm volatile("global_store_dword %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 2) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 3) asm volatile("global_store_dword %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 4) asm volatile("global_store_dword %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    else if constexpr (POL == 5) asm volatile("global_store_dword %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
    else asm volatile("global_store_dword %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
}

template <int P, int POL>
__global__ __launch_bounds__(256) void k_write_pol(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * P);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < P; ++i) st_pol<POL>(p + 64 * i, (uint32_t)(base + i) ^ threadIdx.x);
}

// copy, one 8 KiB polynomial per wave (nt loads), non-persistent 4-wave
// workgroups, stores with policy POL
template <int POL>
__global__ __launch_bounds__(256) void k_copy_pol(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)2048;
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
    uint32_t v[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) v[i] = __builtin_nontemporal_load(p + 64 * i);
#pragma unroll
    for (int i = 0; i < 32; ++i) st_pol<POL>(p + 64 * i, v[i]);
}

// write-only with an LDS pin (dynamic) capping the waves per CU
template <int P>
__global__ __launch_bounds__(256) void k_write_occ(uint32_t *buf, size_t nwords)
{
    extern __shared__ uint32_t dyn[];
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(64 * P);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < P; ++i) p[64 * i] = (uint32_t)(base + i) ^ threadIdx.x;
    if (nwords == 1) dyn[threadIdx.x] = 0;
}

// write-only, 32 stores per wave, at most G outstanding per wave (s_waitcnt vmcnt(G-1) style throttle)
template <int G>
__global__ __launch_bounds__(256) void k_write_thr(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)2048;
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        p[64 * i] = (uint32_t)(base + i) ^ threadIdx.x;
        if (i >= G - 1) {
            if constexpr (G == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            else if constexpr (G == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
            else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
        }
    }
}

// write-only, 4 stores (1 KiB) per wave, 4-wave workgroups (4 KiB each):
// workgroup b (XCD x = b % 8 under round-robin dispatch, its k = b / 8-th)
// writes 4 KiB chunk c = (8 (k / M) + ((x + S) % 8)) M + k % M, i.e. the
// chunks of the 4M-KiB regions whose index is congruent to x + S mod 8
template <int M, int S>
__global__ __launch_bounds__(256) void k_write_map(uint32_t *buf, size_t nwords)
{
    const uint32_t b = blockIdx.x, x = b & 7, k = b >> 3;
    const size_t c = ((size_t)(8 * (k / M) + ((x + S) & 7))) * M + (k % M);
    const size_t base = c * 1024 + (threadIdx.x >> 6) * 256;
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[64 * i] = (uint32_t)(base + i) ^ threadIdx.x;
}

// the XCC each workgroup runs on
__global__ void k_xcc(uint32_t *out)
{
    uint32_t id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    if (threadIdx.x == 0) out[blockIdx.x] = id;
}

// persistent write-only: 4-wave workgroups (G = gridDim), each wave writes its
// 1 KiB piece of chunk b + i G (4 KiB per workgroup and step) -- the flat
// pattern in dispatch order, but long-lived waves; SLEEP s_sleep between steps
template <int SLEEP>
__global__ __launch_bounds__(256) void k_write_persist(uint32_t *buf, size_t nwords)
{
    const size_t nchunk = nwords / 1024;
    for (size_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        uint32_t *p = buf + c * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
        for (int i = 0; i < 4; ++i) p[64 * i] = (uint32_t)(c + i) ^ threadIdx.x;
        if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
}
template <int SLEEP>
__global__ __launch_bounds__(256) void k_copy_persist(uint32_t *buf, size_t nwords)
{
    const size_t nchunk = nwords / 1024;
    for (size_t c = blockIdx.x; c < nchunk; c += gridDim.x) {
        uint32_t *p = buf + c * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
        uint32_t v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = __builtin_nontemporal_load(p + 64 * i);
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < 4; ++i) __builtin_nontemporal_store(v[i] + 1, p + 64 * i);
        if (SLEEP) __builtin_amdgcn_s_sleep(SLEEP);
    }
}

// non-persistent write-only, each wave writes K 1-KiB pieces (its own
// consecutive K KiB), s_sleep(SLEEP) after each piece (and before exiting)
template <int K, int SLEEP>
__global__ __launch_bounds__(256) void k_write_life(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const size_t base = wave * (size_t)(256 * K);
    if (base >= nwords) return;
    uint32_t *p = buf + base + (threadIdx.x & 63);
#pragma unroll
    for (int k = 0; k < K; ++k) {
#pragma unroll
        for (int i = 0; i < 4; ++i) p[256 * k + 64 * i] = (uint32_t)(base + i) ^ threadIdx.x;
        for (int z = 0; z < SLEEP; ++z) __builtin_amdgcn_s_sleep(127);
    }
}

// persistent write-only with ticketed chunks: every workgroup (4 waves) takes
// 4 KiB chunks in address order from one of 8 counters (blockIdx % 8; the
// 8 counters interleave 4-KiB chunks round-robin), so the chunks in flight
// stay a narrow window however the workgroups drift
__global__ __launch_bounds__(256) void k_write_deq(uint32_t *buf, size_t nwords, uint32_t *ctr)
{
    __shared__ uint32_t tk;
    const uint32_t c = blockIdx.x & 7;
    const size_t nchunk = nwords / 1024;
    for (;;) {
        if (threadIdx.x == 0) tk = atomicAdd(ctr + 32 * c, 1u);
        __syncthreads();
        const size_t chunk = (size_t)tk * 8 + c;
        __syncthreads();
        if (chunk >= nchunk) break;
        uint32_t *p = buf + chunk * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
        for (int i = 0; i < 4; ++i) p[64 * i] = (uint32_t)(chunk + i) ^ threadIdx.x;
    }
}

// non-persistent write-only, 1 KiB per wave, 4-wave workgroups; workgroup b
// writes 4 KiB chunk (b % M) (nchunk / M) + b / M: M interleaved streams, so
// the workgroups in flight write M regions nchunk/M chunks apart
template <int M>
__global__ __launch_bounds__(256) void k_write_streams(uint32_t *buf, size_t nwords)
{
    const size_t nchunk = nwords / 1024, b = blockIdx.x;
    const size_t chunk = (b % M) * (nchunk / M) + b / M;
    uint32_t *p = buf + chunk * 1024 + (threadIdx.x >> 6) * 256 + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[64 * i] = (uint32_t)(chunk + i) ^ threadIdx.x;
}

// non-persistent write-only, 1 KiB per wave, the wave stays resident for
// SLEEP x 64 cycles after its stores
template <int SLEEP>
__global__ __launch_bounds__(256) void k_write_linger(uint32_t *buf, size_t nwords)
{
    const size_t wave = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t *p = buf + wave * 256 + (threadIdx.x & 63);
#pragma unroll
    for (int i = 0; i < 4; ++i) p[64 * i] = (uint32_t)(wave + i) ^ threadIdx.x;
    __builtin_amdgcn_s_sleep(SLEEP);
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
    const size_t nwords = (size_t)1 << 31;   // 8 GiB
    const size_t bytes = nwords * 4;
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    uint32_t *a, *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 4096));
    hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a, nwords);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<std::pair<std::string, std::function<void()>>> cases;
    std::vector<double> moved;
    char nm[160];
    auto grid = [&](int per) { return (unsigned)(nwords / (64 * per) / 4); };
#define RD(P, NT)                                                                                               \
    snprintf(nm, sizeof nm, "read  per=%d nt=%d", P, NT);                                                       \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_read<P, NT>), dim3(grid(P)), dim3(256), 0, 0, a, nwords, sink); }); \
    moved.push_back((double)bytes);
#define WR(P, NT)                                                                                               \
    snprintf(nm, sizeof nm, "write per=%d nt=%d", P, NT);                                                       \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write<P, NT>), dim3(grid(P)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);
#define CG(G, NT)                                                                                               \
    snprintf(nm, sizeof nm, "copy per=32 load groups of %d nt=%d", G, NT);                                       \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_copy_grouped<G, NT>), dim3(grid(32)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back(2.0 * bytes);
#define CS(G, NT)                                                                                               \
    snprintf(nm, sizeof nm, "copy per=32 store groups of %d nt=%d", G, NT);                                      \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_copy_stgrouped<G, NT>), dim3(grid(32)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back(2.0 * bytes);


#define WMAP(M, S)                                                                                              \
    snprintf(nm, sizeof nm, "write 1KiB/wave map region=%dKiB shift=%d", 4 * M, S);                              \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write_map<M, S>), dim3((unsigned)(nwords / 1024)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);

#define WPERS(MULT, SLEEP)                                                                                      \
    snprintf(nm, sizeof nm, "write persistent grid=%d x CUs sleep=%d", MULT, SLEEP);                            \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write_persist<SLEEP>), dim3(256 * MULT), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);
#define CPERS(MULT, SLEEP)                                                                                      \
    snprintf(nm, sizeof nm, "copy 1KiB/wave persistent grid=%d x CUs sleep=%d", MULT, SLEEP);                   \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_copy_persist<SLEEP>), dim3(256 * MULT), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back(2.0 * bytes);

#define WLIFE(K, SLEEP)                                                                                         \
    snprintf(nm, sizeof nm, "write non-persistent %d KiB/wave sleep=%dx127", K, SLEEP);                         \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write_life<K, SLEEP>), dim3((unsigned)(nwords / (256 * K) / 4)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);

#define WSTR(M)                                                                                                 \
    snprintf(nm, sizeof nm, "write 1KiB/wave %d interleaved streams", M);                                        \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write_streams<M>), dim3((unsigned)(nwords / 1024)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);
#define WLING(S)                                                                                                \
    snprintf(nm, sizeof nm, "write 1KiB/wave then s_sleep(%d)", S);                                              \
    cases.emplace_back(nm, [=] { hipLaunchKernelGGL((k_write_linger<S>), dim3((unsigned)(nwords / 1024)), dim3(256), 0, 0, a, nwords); }); \
    moved.push_back((double)bytes);
    WMAP(1, 0)
    WSTR(1) WSTR(8) WSTR(64) WSTR(512) WSTR(4096)
    WLING(1) WLING(4) WLING(16) WLING(40)

    {
        uint32_t *xo;
        CK(hipMalloc(&xo, 64 * 4));
        hipLaunchKernelGGL(k_xcc, dim3(64), dim3(64), 0, 0, xo);
        uint32_t h[64];
        CK(hipMemcpy(h, xo, sizeof h, hipMemcpyDeviceToHost));
        printf("xcc of blocks 0..63:");
        for (int i = 0; i < 64; ++i) printf(" %u", h[i]);
        printf("\n");
    }
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
        printf("%-44s med %7.3f ms  min %7.3f ms  %6.0f GB/s\n", cases[i].first.c_str(), med, v[0], moved[i] / (med * 1e-3) / 1e9);
    }
    return 0;
}
