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

// Occupancy-pinned chunked copies: 512-thread blocks whose static LDS (KB KiB)
// caps residency (80 KiB -> 2 blocks/CU = 4 waves/SIMD, the transforms'
// occupancy), each wave copying PPW consecutive-per-block n=2048 polys.
//  MODE 0: load 32 dwords -> store (the transforms' memory-only shape)
//  MODE 1: register double buffer (next poly's loads in flight during the store)
//  MODE 2: LDS-DMA 1 ahead into a wave buffer, ds_read -> store
//  MODE 3: LDS-DMA 2 ahead + register 1 ahead
__device__ __forceinline__ void cdma16(const uint32_t *gsrc, uint32_t lds)
{
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
template <int MODE, int KB>
__global__ __launch_bounds__(512) void k_occ(const uint32_t *in, uint32_t *out, uint32_t npoly, uint32_t ppw)
{
    __shared__ __attribute__((aligned(16))) uint32_t lds[KB * 256];
    const uint32_t lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint32_t *buf = lds + w * 2048;
    if (npoly == 0xFFFFFFFFu) {   // never true: keeps the LDS allocation (residency cap) in every mode
        lds[threadIdx.x * (KB / 2)] = threadIdx.x;
        __syncthreads();
        out[threadIdx.x] = lds[(threadIdx.x + 1) % (KB * 256)];
    }
    const uint32_t la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)buf);
    uint32_t u = blockIdx.x * 8 * ppw + w;
    const uint32_t end = min(npoly, (blockIdx.x + 1) * 8 * ppw);
    if (u >= end) return;
    if constexpr (MODE == 11 || MODE == 12) {
        // workgroup-cooperative: the 8 waves DMA the block's 8 consecutive polys (64 KiB) as one
        // contiguous sweep (piece p = w + 8c goes to poly p/8's buffer), barrier, then
        // 11: each wave stores its own poly from LDS with dword stores (the transforms' store shape)
        // 12: cooperative sweep of x4 stores (wave w stores pieces w + 8c), barrier before reuse
        const uint32_t base_la = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) uint32_t *)lds);
        for (uint32_t g = blockIdx.x * 8 * ppw; g < end; g += 8) {   // g = first poly of this step
            const uint32_t *s = in + (size_t)g * 2048 + 4 * lane;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const uint32_t p = w + 8 * c;   // piece index in the 64 KiB step
                cdma16(s + 256 * p, base_la + 1024 * p);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            if constexpr (MODE == 11) {
                uint32_t v[32];
#pragma unroll
                for (int j = 0; j < 32; ++j) v[j] = buf[lane + 64 * j];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                uint32_t *d = out + (size_t)(g + w) * 2048 + lane;
#pragma unroll
                for (int j = 0; j < 32; ++j) d[64 * j] = v[j];
            } else {
                uint4 v[8];
                const uint4 *b4 = reinterpret_cast<const uint4 *>(lds) + lane;
#pragma unroll
                for (int c = 0; c < 8; ++c) v[c] = b4[64 * (w + 8 * c)];
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                uint4 *d = reinterpret_cast<uint4 *>(out + (size_t)g * 2048) + lane;
#pragma unroll
                for (int c = 0; c < 8; ++c) d[64 * (w + 8 * c)] = v[c];
            }
        }
    } else if constexpr (MODE == 9) {   // dword copy, chunk order rotated per wave (rot = u mod 32)
        for (; u < end; u += 8) {
            const uint32_t rot = u & 31;
            uint32_t v[32];
            const uint32_t *s = in + (size_t)u * 2048 + lane;
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s[64 * ((j + rot) & 31)];
#pragma unroll
            for (int j = 0; j < 32; ++j) d[64 * ((j + rot) & 31)] = v[j];
        }
    } else if constexpr (MODE == 10) {   // x4 DMA in + x4 out via LDS, piece order rotated per wave (rot = u mod 8)
        for (; u < end; u += 8) {
            const uint32_t rot = u & 7;
            const uint32_t *s = in + (size_t)u * 2048 + 4 * lane;
            for (int c = 0; c < 8; ++c) {
                const uint32_t cc = (c + rot) & 7;
                cdma16(s + 256 * cc, la + 1024 * cc);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            uint4 *d = reinterpret_cast<uint4 *>(out + (size_t)u * 2048) + lane;
            const uint4 *b4 = reinterpret_cast<const uint4 *>(buf) + lane;
            uint4 w[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) w[c] = b4[64 * ((c + rot) & 7)];
#pragma unroll
            for (int c = 0; c < 8; ++c) d[64 * ((c + rot) & 7)] = w[c];
        }
    } else if constexpr (MODE == 7 || MODE == 8) {   // 7: dword loads, stores staged through LDS as dwordx4; 8: DMA x4 in, x4 out
        uint4 *b4 = reinterpret_cast<uint4 *>(buf) + lane;
        for (; u < end; u += 8) {
            uint4 *d = reinterpret_cast<uint4 *>(out + (size_t)u * 2048) + lane;
            if constexpr (MODE == 7) {
                uint32_t v[32];
                const uint32_t *s = in + (size_t)u * 2048 + lane;
#pragma unroll
                for (int j = 0; j < 32; ++j) v[j] = s[64 * j];
#pragma unroll
                for (int j = 0; j < 32; ++j) buf[lane + 64 * j] = v[j];
            } else {
                const uint32_t *s = in + (size_t)u * 2048 + 4 * lane;
                for (int c = 0; c < 8; ++c) cdma16(s + 256 * c, la + 1024 * c);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            uint4 w[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) w[c] = b4[64 * c];
#pragma unroll
            for (int c = 0; c < 8; ++c) d[64 * c] = w[c];
        }
    } else if constexpr (MODE >= 4) {   // 4: bit-reversed store order, 5: 16 KiB table prologue, 6: both
        if constexpr (MODE >= 5) {
            const uint4 *src = reinterpret_cast<const uint4 *>(in) + ((blockIdx.x * 7) & 1023);   // L2-resident
            uint4 *dst = reinterpret_cast<uint4 *>(lds + 16384);
            uint4 t0 = src[threadIdx.x], t1 = src[threadIdx.x + 512];
            dst[threadIdx.x] = t0;
            if (threadIdx.x < 496) dst[threadIdx.x + 512] = t1;
            __syncthreads();
        }
        for (; u < end; u += 8) {
            uint32_t v[32];
            const uint32_t *s = in + (size_t)u * 2048 + lane;
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s[64 * j];
            if constexpr (MODE >= 5) v[0] += lds[16384 + lane];
#pragma unroll
            for (int j = 0; j < 32; ++j) {
                const int jj = (MODE == 5) ? j : (((j & 1) << 4) | ((j & 2) << 2) | (j & 4) | ((j & 8) >> 2) | ((j & 16) >> 4));
                d[64 * jj] = v[j];
            }
        }
    } else if constexpr (MODE == 0) {
        for (; u < end; u += 8) {
            uint32_t v[32];
            const uint32_t *s = in + (size_t)u * 2048 + lane;
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s[64 * j];
#pragma unroll
            for (int j = 0; j < 32; ++j) d[64 * j] = v[j];
        }
    } else if constexpr (MODE == 1) {
        uint32_t v[32], nv[32];
        const uint32_t *s = in + (size_t)u * 2048 + lane;
#pragma unroll
        for (int j = 0; j < 32; ++j) v[j] = s[64 * j];
        for (; u < end; u += 8) {
            const bool more = u + 8 < end;
            if (more) {
                const uint32_t *sn = in + (size_t)(u + 8) * 2048 + lane;
#pragma unroll
                for (int j = 0; j < 32; ++j) nv[j] = sn[64 * j];
            }
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) d[64 * j] = v[j];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = nv[j];
        }
    } else if constexpr (MODE == 2) {
        const uint32_t *s = in + (size_t)u * 2048 + 4 * lane;
        for (int c = 0; c < 8; ++c) cdma16(s + 256 * c, la + 1024 * c);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        for (;;) {
            uint32_t v[32];
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = buf[lane + 64 * j];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            const bool more = u + 8 < end;
            if (more) {
                const uint32_t *sn = in + (size_t)(u + 8) * 2048 + 4 * lane;
                for (int c = 0; c < 8; ++c) cdma16(sn + 256 * c, la + 1024 * c);
            }
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) d[64 * j] = v[j];
            if (!more) break;
            u += 8;
            asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        }
    } else {
        // poly u in registers, u+8 in LDS (DMA), issue u+16 DMA after reading u+8 from LDS
        uint32_t v[32];
        {
            const uint32_t *s = in + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = s[64 * j];
        }
        if (u + 8 < end) {
            const uint32_t *s = in + (size_t)(u + 8) * 2048 + 4 * lane;
            for (int c = 0; c < 8; ++c) cdma16(s + 256 * c, la + 1024 * c);
        }
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");   // v landed (DMA may be in flight)
        for (;;) {
            uint32_t *d = out + (size_t)u * 2048 + lane;
#pragma unroll
            for (int j = 0; j < 32; ++j) d[64 * j] = v[j];
            if (u + 8 >= end) break;
            asm volatile("s_waitcnt vmcnt(32)" ::: "memory");   // DMA of u+8 done
#pragma unroll
            for (int j = 0; j < 32; ++j) v[j] = buf[lane + 64 * j];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            u += 8;
            if (u + 8 < end) {
                const uint32_t *sn = in + (size_t)(u + 8) * 2048 + 4 * lane;
                for (int c = 0; c < 8; ++c) cdma16(sn + 256 * c, la + 1024 * c);
            }
        }
    }
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
    const size_t bytes = (size_t)npoly * 2048 * 4;
    uint32_t *a, *b;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&b, bytes);
    (void)hipMemset(a, 1, bytes);
    if (argc > 1) {   // random data in [0, q) instead of a constant byte pattern
        hipLaunchKernelGGL(k_rand, dim3(4096), dim3(256), 0, 0, a, bytes / 4);
        (void)hipDeviceSynchronize();
    }
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
#define OCC(MODE, KB, PPW)                                                                                   \
    run("occ mode=" #MODE " lds=" #KB "KiB ppw=" #PPW, [&] {                                                  \
        hipLaunchKernelGGL((k_occ<MODE, KB>), dim3((npoly + 8 * PPW - 1) / (8 * PPW)), dim3(512), 0, 0, a, b, npoly, PPW); \
    })
    OCC(0, 80, 16);
    OCC(11, 80, 16);
    OCC(12, 80, 16);
    OCC(11, 80, 4);
    OCC(12, 80, 4);
    OCC(11, 64, 1);
    OCC(12, 64, 1);
    OCC(9, 80, 16);
    OCC(10, 80, 16);
    OCC(9, 80, 4);
    OCC(10, 80, 4);
    OCC(7, 80, 16);
    OCC(8, 80, 16);
    OCC(7, 80, 4);
    OCC(8, 80, 4);
    OCC(4, 80, 16);
    OCC(5, 80, 16);
    OCC(6, 80, 16);
    OCC(4, 80, 4);
    OCC(5, 80, 4);
    OCC(6, 80, 4);
    OCC(6, 80, 8);
    OCC(6, 80, 32);
    OCC(1, 80, 16);
    OCC(2, 80, 16);
    OCC(3, 80, 16);
    OCC(0, 64, 16);
    OCC(2, 64, 16);
    OCC(0, 40, 16);
    OCC(0, 80, 4);
    OCC(2, 80, 4);
    OCC(3, 80, 4);
    run("flat x4 grid=cus*8", [&] { hipLaunchKernelGGL(k_flat4, dim3(cus * 8), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    run("flat x4 grid=cus*32", [&] { hipLaunchKernelGGL(k_flat4, dim3(cus * 32), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    run("flat x4 grid=n/256", [&] { hipLaunchKernelGGL(k_flat4, dim3((unsigned)(bytes / 16 / 256)), dim3(256), 0, 0, (const uint4 *)a, (uint4 *)b, bytes / 16); });
    return 0;
}
