// copy_bw.hip -- HBM copy roofline on MI355X for the transform kernels'
// access shapes: 16 GiB moved (8 GiB read + 8 GiB write), per-wave 8 KiB
// "polys", varying access width, waves per CU, cache policy and grid style.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int W, bool NT, int WPB>   // W = dwords per lane per access, waves per block
__global__ __launch_bounds__(64 * WPB) void k_poly(const uint32_t *in, uint32_t *out, uint32_t npoly)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nw = gridDim.x * WPB;
    for (uint32_t u = blockIdx.x * WPB + (threadIdx.x >> 6); u < npoly; u += nw) {
        const uint32_t *s = in + (size_t)u * 2048;
        uint32_t *d = out + (size_t)u * 2048;
        if constexpr (W == 1) {
            uint32_t v[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = NT ? __builtin_nontemporal_load(s + lane + 64 * j) : s[lane + 64 * j];
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                if (NT) __builtin_nontemporal_store(v[j], d + lane + 64 * j);
                else d[lane + 64 * j] = v[j];
            }
        } else if constexpr (W == 2) {
            uint2 v[16];
            const uint2 *s2 = reinterpret_cast<const uint2 *>(s) + lane;
            uint2 *d2 = reinterpret_cast<uint2 *>(d) + lane;
#pragma unroll
            for (int j = 0; j < 16; ++j) v[j] = s2[64 * j];
#pragma unroll
            for (int j = 0; j < 16; ++j) d2[64 * j] = v[j];
        } else {
            uint4 v[8];
            const uint4 *s4 = reinterpret_cast<const uint4 *>(s) + lane;
            uint4 *d4 = reinterpret_cast<uint4 *>(d) + lane;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                if (NT) {
                    v[j].x = __builtin_nontemporal_load(&s4[64 * j].x);
                    v[j].y = __builtin_nontemporal_load(&s4[64 * j].y);
                    v[j].z = __builtin_nontemporal_load(&s4[64 * j].z);
                    v[j].w = __builtin_nontemporal_load(&s4[64 * j].w);
                } else v[j] = s4[64 * j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j) d4[64 * j] = v[j];
        }
    }
}

// non-persistent: block b, wave w handles polys (b*WPB + w) * PPW + i, i < PPW (contiguous per block)
template <int W, int WPB, int PPW>
__global__ __launch_bounds__(64 * WPB) void k_chunk(const uint32_t *in, uint32_t *out, uint32_t npoly)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t base = (blockIdx.x * WPB) * PPW;
    for (int i = 0; i < PPW; i++) {
        const uint32_t u = base + i * WPB + (threadIdx.x >> 6);   // consecutive waves -> consecutive polys
        if (u >= npoly) return;
        const uint32_t *s = in + (size_t)u * 2048;
        uint32_t *d = out + (size_t)u * 2048;
        if constexpr (W == 1) {
            uint32_t v[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s[lane + 64 * j];
#pragma unroll
            for (int j = 0; j < 32; ++j) d[lane + 64 * j] = v[j];
        } else {
            uint4 v[8];
            const uint4 *s4 = reinterpret_cast<const uint4 *>(s) + lane;
            uint4 *d4 = reinterpret_cast<uint4 *>(d) + lane;
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = s4[64 * j];
#pragma unroll
            for (int j = 0; j < 8; ++j) d4[64 * j] = v[j];
        }
    }
}

__global__ __launch_bounds__(256) void k_flat4(const uint4 *in, uint4 *out, size_t n4)
{
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) out[i] = in[i];
}

int main()
{
    const uint32_t npoly = 1u << 20;
    const size_t bytes = (size_t)npoly * 2048 * 4;
    uint32_t *a, *b;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&b, bytes);
    (void)hipMemset(a, 1, bytes);
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto run = [&](const char *name, auto launch) {
        launch();
        float best = 1e9;
        for (int r = 0; r < 5; r++) {
            (void)hipEventRecord(e0);
            launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("%-40s %7.3f ms  %6.0f GB/s\n", name, best, 2.0 * bytes / (best * 1e-3) / 1e9);
    };
#define POLY(W, NT, WPB, BPC)                                                                                  \
    run("poly W=" #W " nt=" #NT " waves/blk=" #WPB " blk/CU=" #BPC, [&] {                                     \
        hipLaunchKernelGGL((k_poly<W, NT, WPB>), dim3(cus * BPC), dim3(64 * WPB), 0, 0, a, b, npoly);          \
    })
    POLY(1, false, 8, 2);
    POLY(1, false, 8, 4);
    POLY(1, false, 16, 2);
    POLY(1, true, 8, 2);
    POLY(1, true, 8, 4);
    POLY(2, false, 8, 2);
    POLY(2, false, 8, 4);
    POLY(4, false, 8, 2);
    POLY(4, false, 8, 4);
    POLY(4, true, 8, 4);
    POLY(4, false, 4, 8);
#define CHUNK(W, WPB, PPW)                                                                                     \
    run("chunk W=" #W " waves/blk=" #WPB " polys/wave=" #PPW, [&] {                                             \
        hipLaunchKernelGGL((k_chunk<W, WPB, PPW>), dim3((npoly + WPB * PPW - 1) / (WPB * PPW)), dim3(64 * WPB), 0, 0, a, b, npoly); \
    })
    CHUNK(1, 8, 1);
    CHUNK(1, 16, 1);
    CHUNK(1, 8, 2);
    CHUNK(1, 8, 4);
    CHUNK(1, 16, 4);
    CHUNK(1, 8, 16);
    CHUNK(4, 8, 1);
    CHUNK(4, 8, 4);
    CHUNK(4, 16, 4);
    run("flat x4 grid=cus*8", [&] { hipLaunchKernelGGL(k_flat4, dim3(cus * 8), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    run("flat x4 grid=cus*32", [&] { hipLaunchKernelGGL(k_flat4, dim3(cus * 32), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    run("flat x4 grid=n/256", [&] { hipLaunchKernelGGL(k_flat4, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    return 0;
}
