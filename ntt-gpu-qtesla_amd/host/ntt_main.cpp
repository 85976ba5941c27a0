// ntt_main.cpp -- C++ host driver over the C ABI (include/qtesla_ntt.h).
//
// Mirrors the reference's CLI and GPU test drivers (benlwk/ntt-gpu-qTESLA
// main.cu:12-230, NTT.cu:2008-2443) so the same experiments can be run on
// MI355X through the drop-in boundary:
//
//   -speedgpu 4   CT-CT negacyclic poly-mul   (test_NTT_CT_CT_nega_gpu, NTT.cu:2181)
//   -speedgpu 6   CT-GS negacyclic poly-mul   (test_NTT_CT_GS_nega_gpu, NTT.cu:2358)
//                 both as poly_ntt x2 + poly_pointwise + poly_invntt
//   -speedgpu 7   fused poly_mul (one launch per batch)
//   -speedgpu 8   speed suite: 5 x option 6 then 5 x option 7 (main.cu:213-225)
//   -speedgpu 9   forward+inverse transform throughput (BASELINE metric)
//   -speedgpu 10  fused poly-mul host -> host through the pipelined host-buffer
//                 context (ntt_host_ctx: H2D / kernel / D2H overlapped), the
//                 reference's PCIe-inclusive timing region (NTT.cu:2384-2428)
//   -speedgpu 11  Nussbaumer product on the GPU in the reference's ring
//                 Z/(2^32-1) (test_nussbaumer, NTT.cu:1987-2005; -speedcpu 6 there)
//   -speedgpu 12  per-call latency through the C ABI, the qTESLA signing loop's
//                 use (one small batch per call): poly_ntt, poly_invntt and
//                 poly_mul, each (a) called back to back (calls/s the host
//                 sustains, HIP events around R calls) and (b) synchronised
//                 after every call (the round trip a caller that consumes the
//                 result sees)
//   -param ref|p-I|p-III|p-III-4096|p-III-8192   parameter set (reference:
//                 compile-time QTESLA set; the n = 4096 / 8192 sets run every
//                 option but 11, whose Nussbaumer split is n <= 2048)
//   -batch B      polynomials per batch (reference: BATCH macro, main.cuh:7)
//   -r seed       random operands from the device generator (reference parses
//                 -r but never uses it, main.cu:89-91); default: all-ones
//                 operands as in NTT.cu:2360, checked against the KAT
//                 z[k] = 2k + 2 - n mod q
//   -pcie         include H2D/D2H copies in the timed region like the reference
//                 (NTT.cu:2384-2428); default times device-resident data
//   -debug        print the first/last coefficients of z (the DEBUG dump)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "qtesla_ntt.h"

#define HIP_OK(x)                                                                          \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)
#define NTT_CALL(x)                                                                        \
    do {                                                                                   \
        int rc_ = (x);                                                                     \
        if (rc_ != NTT_OK) {                                                               \
            fprintf(stderr, "%s failed: %s\n", #x, ntt_strerror(rc_));                     \
            exit(3);                                                                       \
        }                                                                                  \
    } while (0)

static void help_message()
{
    printf("usage: ntt_main -speedgpu {4,6,7,8,9,10,11,12} [-param ref|p-I|p-III|p-III-4096|p-III-8192] [-batch B] [-reps R] [-r seed] [-pcie] [-debug]\n");
}

struct Opts {
    int option = 6, ps = NTT_PARAM_REF, reps = 1;
    size_t batch = 2;
    bool random = false, pcie = false, debug = false;
    uint64_t seed = 0;
};

// Negacyclic poly-mul driver: inputs x, y (all ones or random), output z.
static double run_polymul(const Opts &o, bool fused, std::vector<uint32_t> &z, int *kat_ok)
{
    uint32_t n, q;
    NTT_CALL(ntt_param_info(o.ps, &n, &q, nullptr, nullptr, nullptr, nullptr));
    const size_t count = o.batch * n, bytes = count * 4;
    std::vector<uint32_t> x(count, 1), y(count, 1);
    uint32_t *d_x, *d_y, *d_z;
    HIP_OK(hipMalloc(&d_x, bytes));
    HIP_OK(hipMalloc(&d_y, bytes));
    HIP_OK(hipMalloc(&d_z, bytes));
    hipStream_t s;
    HIP_OK(hipStreamCreate(&s));
    if (o.random) {
        NTT_CALL(ntt_fill_uniform(d_x, o.batch, o.ps, o.seed, 0, s));
        NTT_CALL(ntt_fill_uniform(d_y, o.batch, o.ps, o.seed ^ 0xFFFF, 0, s));
        HIP_OK(hipMemcpyAsync(x.data(), d_x, bytes, hipMemcpyDeviceToHost, s));
        HIP_OK(hipMemcpyAsync(y.data(), d_y, bytes, hipMemcpyDeviceToHost, s));
        HIP_OK(hipStreamSynchronize(s));
    }
    auto body = [&]() {
        if (o.pcie) {
            HIP_OK(hipMemcpyAsync(d_x, x.data(), bytes, hipMemcpyHostToDevice, s));
            HIP_OK(hipMemcpyAsync(d_y, y.data(), bytes, hipMemcpyHostToDevice, s));
        }
        if (fused) {
            NTT_CALL(poly_mul(d_z, d_x, d_y, o.batch, o.ps, s));
        } else {
            // CT-GS composition; unlike bit_reverse_copy_tbl_Phi_gpu the inputs are
            // kept (out-of-place forward transforms into d_z / scratch)
            NTT_CALL(poly_ntt_oop(d_z, d_x, o.batch, o.ps, s));
            NTT_CALL(poly_ntt(d_y, nullptr, o.batch, o.ps, s));
            NTT_CALL(poly_pointwise(d_z, d_z, d_y, o.batch, o.ps, s));
            NTT_CALL(poly_invntt(d_z, nullptr, o.batch, o.ps, s));
        }
        if (o.pcie) HIP_OK(hipMemcpyAsync(z.data(), d_z, bytes, hipMemcpyDeviceToHost, s));
    };
    z.assign(count, 0);
    if (!o.pcie) {   // device-resident: restore y each rep in the composed path
        HIP_OK(hipMemcpyAsync(d_x, x.data(), bytes, hipMemcpyHostToDevice, s));
        HIP_OK(hipMemcpyAsync(d_y, y.data(), bytes, hipMemcpyHostToDevice, s));
    }
    body();  // warm-up (also uploads the twiddle tables)
    HIP_OK(hipStreamSynchronize(s));
    double ms = 0.0;
    for (int r = 0; r < o.reps; r++) {
        if (!o.pcie && !fused) HIP_OK(hipMemcpyAsync(d_y, y.data(), bytes, hipMemcpyHostToDevice, s));
        HIP_OK(hipStreamSynchronize(s));
        auto t0 = std::chrono::steady_clock::now();
        body();
        HIP_OK(hipStreamSynchronize(s));
        auto t1 = std::chrono::steady_clock::now();
        ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    if (!o.pcie) HIP_OK(hipMemcpy(z.data(), d_z, bytes, hipMemcpyDeviceToHost));
    *kat_ok = -1;
    if (!o.random) {
        *kat_ok = 1;
        for (size_t b = 0; b < o.batch && *kat_ok; b++)
            for (uint32_t k = 0; k < n; k++) {
                const uint32_t want = (uint32_t)((2ull * k + 2 + q - n) % q);
                if (z[b * n + k] != want) { *kat_ok = 0; break; }
            }
    }
    HIP_OK(hipFree(d_x));
    HIP_OK(hipFree(d_y));
    HIP_OK(hipFree(d_z));
    HIP_OK(hipStreamDestroy(s));
    return ms / o.reps;
}

static double run_fwdinv(const Opts &o, int *roundtrip_ok)
{
    uint32_t n;
    NTT_CALL(ntt_param_info(o.ps, &n, nullptr, nullptr, nullptr, nullptr, nullptr));
    const size_t bytes = o.batch * n * 4;
    uint32_t *d_x, *d_ref;
    HIP_OK(hipMalloc(&d_x, bytes));
    HIP_OK(hipMalloc(&d_ref, bytes));
    hipStream_t s;
    HIP_OK(hipStreamCreate(&s));
    NTT_CALL(ntt_fill_uniform(d_x, o.batch, o.ps, o.seed, 0, s));
    HIP_OK(hipMemcpyAsync(d_ref, d_x, bytes, hipMemcpyDeviceToDevice, s));
    NTT_CALL(poly_ntt(d_x, nullptr, o.batch, o.ps, s));
    NTT_CALL(poly_invntt(d_x, nullptr, o.batch, o.ps, s));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, s));
    for (int r = 0; r < o.reps; r++) {
        NTT_CALL(poly_ntt(d_x, nullptr, o.batch, o.ps, s));
        NTT_CALL(poly_invntt(d_x, nullptr, o.batch, o.ps, s));
    }
    HIP_OK(hipEventRecord(e1, s));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.f;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<uint32_t> a(o.batch * n), b(o.batch * n);
    HIP_OK(hipMemcpy(a.data(), d_x, bytes, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(b.data(), d_ref, bytes, hipMemcpyDeviceToHost));
    *roundtrip_ok = (a == b);
    HIP_OK(hipFree(d_x));
    HIP_OK(hipFree(d_ref));
    HIP_OK(hipEventDestroy(e0));
    HIP_OK(hipEventDestroy(e1));
    HIP_OK(hipStreamDestroy(s));
    return ms / o.reps;
}

// host -> host fused product through ntt_host_ctx; all-ones (KAT) or random operands
static double run_polymul_host(const Opts &o, int *kat_ok)
{
    uint32_t n, q;
    NTT_CALL(ntt_param_info(o.ps, &n, &q, nullptr, nullptr, nullptr, nullptr));
    const size_t count = o.batch * n, bytes = count * 4;
    uint32_t *x = (uint32_t *)ntt_host_alloc(bytes), *y = (uint32_t *)ntt_host_alloc(bytes),
             *z = (uint32_t *)ntt_host_alloc(bytes);
    if (!x || !y || !z) { fprintf(stderr, "ntt_host_alloc failed\n"); exit(2); }
    for (size_t i = 0; i < count; i++) x[i] = y[i] = 1;
    if (o.random) {
        uint32_t *d;
        HIP_OK(hipMalloc(&d, bytes));
        NTT_CALL(ntt_fill_uniform(d, o.batch, o.ps, o.seed, 0, nullptr));
        HIP_OK(hipMemcpy(x, d, bytes, hipMemcpyDeviceToHost));
        NTT_CALL(ntt_fill_uniform(d, o.batch, o.ps, o.seed ^ 0xFFFF, 0, nullptr));
        HIP_OK(hipMemcpy(y, d, bytes, hipMemcpyDeviceToHost));
        HIP_OK(hipFree(d));
    }
    ntt_host_ctx *ctx = nullptr;
    NTT_CALL(ntt_host_ctx_create(&ctx, o.ps, 0, 0));
    NTT_CALL(poly_mul_host(ctx, z, x, y, o.batch));   // warm-up
    double ms = 0.0;
    for (int r = 0; r < o.reps; r++) {
        auto t0 = std::chrono::steady_clock::now();
        NTT_CALL(poly_mul_host(ctx, z, x, y, o.batch));
        auto t1 = std::chrono::steady_clock::now();
        ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
    }
    *kat_ok = -1;
    if (!o.random) {
        *kat_ok = 1;
        for (size_t b = 0; b < o.batch && *kat_ok; b++)
            for (uint32_t k = 0; k < n; k++)
                if (z[b * n + k] != (uint32_t)((2ull * k + 2 + q - n) % q)) { *kat_ok = 0; break; }
    }
    NTT_CALL(ntt_host_ctx_destroy(ctx));
    ntt_host_free(x);
    ntt_host_free(y);
    ntt_host_free(z);
    return ms / o.reps;
}

// Nussbaumer mod 2^32-1 on the GPU, all-ones operands: z[k] = 2k + 2 - n mod 2^32-1
static double run_nussbaumer(const Opts &o, int *kat_ok)
{
    uint32_t n;
    NTT_CALL(ntt_param_info(o.ps, &n, nullptr, nullptr, nullptr, nullptr, nullptr));
    const size_t count = o.batch * n, bytes = count * 4;
    std::vector<uint32_t> x(count, 1), z(count, 0);
    uint32_t *d_x, *d_z;
    HIP_OK(hipMalloc(&d_x, bytes));
    HIP_OK(hipMalloc(&d_z, bytes));
    HIP_OK(hipMemcpy(d_x, x.data(), bytes, hipMemcpyHostToDevice));
    NTT_CALL(poly_mul_nussbaumer(d_z, d_x, d_x, o.batch, o.ps, NTT_RING_M32, nullptr));
    HIP_OK(hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < o.reps; r++) NTT_CALL(poly_mul_nussbaumer(d_z, d_x, d_x, o.batch, o.ps, NTT_RING_M32, nullptr));
    HIP_OK(hipDeviceSynchronize());
    auto t1 = std::chrono::steady_clock::now();
    HIP_OK(hipMemcpy(z.data(), d_z, bytes, hipMemcpyDeviceToHost));
    *kat_ok = 1;
    const uint64_t m = 0xFFFFFFFFull;
    for (size_t b = 0; b < o.batch && *kat_ok; b++)
        for (uint32_t k = 0; k < n; k++)
            if (z[b * n + k] != (uint32_t)((2ull * k + 2 + m - n) % m)) { *kat_ok = 0; break; }
    HIP_OK(hipFree(d_x));
    HIP_OK(hipFree(d_z));
    return std::chrono::duration<double, std::milli>(t1 - t0).count() / o.reps;
}

static void report_polymul(const Opts &o, const char *name, bool fused)
{
    std::vector<uint32_t> z;
    int kat = -1;
    const double ms = run_polymul(o, fused, z, &kat);
    printf("\n========================\n");
    printf("test_NTT_negacyclic %s GPU. Batch Size is %zu", name, o.batch);
    printf("\n========================\n");
    printf("Performance GPU %s GPU \n Time\t\t: % .4f ms. \nThroughput\t: %.2f Multiplications per second\n", name, ms,
           (double)o.batch / ms * 1000.0);
    if (kat >= 0) printf("all-ones KAT z[k] = 2k+2-n mod q: %s\n", kat ? "Identical." : "Incorrect result.");
    if (o.debug) {
        uint32_t n;
        ntt_param_info(o.ps, &n, nullptr, nullptr, nullptr, nullptr, nullptr);
        printf("z: ");
        for (uint32_t i = 0; i < 8 && i < n; i++) printf("%u ", z[i]);
        printf("... %u\n", z[n - 1]);
    }
}

// -speedgpu 12: per-call latency of the small-batch entry points.
static int run_latency(const Opts &o)
{
    uint32_t n;
    NTT_CALL(ntt_param_info(o.ps, &n, nullptr, nullptr, nullptr, nullptr, nullptr));
    const size_t bytes = o.batch * n * 4;
    uint32_t *d_x, *d_y, *d_z;
    HIP_OK(hipMalloc(&d_x, bytes));
    HIP_OK(hipMalloc(&d_y, bytes));
    HIP_OK(hipMalloc(&d_z, bytes));
    hipStream_t s;
    HIP_OK(hipStreamCreate(&s));
    NTT_CALL(ntt_fill_uniform(d_x, o.batch, o.ps, 1, 0, s));
    NTT_CALL(ntt_fill_uniform(d_y, o.batch, o.ps, 2, 0, s));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    const int calls = o.reps > 1 ? o.reps : 2000;
    struct Case {
        const char *name;
        int (*fn)(uint32_t *, uint32_t *, uint32_t *, size_t, int, hipStream_t);
    };
    const Case cases[] = {
        {"poly_ntt", [](uint32_t *x, uint32_t *, uint32_t *, size_t b, int ps, hipStream_t st) {
             return poly_ntt(x, nullptr, b, ps, st);
         }},
        {"poly_invntt", [](uint32_t *x, uint32_t *, uint32_t *, size_t b, int ps, hipStream_t st) {
             return poly_invntt(x, nullptr, b, ps, st);
         }},
        {"poly_mul", [](uint32_t *x, uint32_t *y, uint32_t *z, size_t b, int ps, hipStream_t st) {
             return poly_mul(z, x, y, b, ps, st);
         }},
    };
    for (const Case &c : cases) {
        for (int w = 0; w < 50; w++) NTT_CALL(c.fn(d_x, d_y, d_z, o.batch, o.ps, s));
        HIP_OK(hipStreamSynchronize(s));
        // (a) back to back
        auto t0 = std::chrono::steady_clock::now();
        HIP_OK(hipEventRecord(e0, s));
        for (int i = 0; i < calls; i++) NTT_CALL(c.fn(d_x, d_y, d_z, o.batch, o.ps, s));
        HIP_OK(hipEventRecord(e1, s));
        HIP_OK(hipEventSynchronize(e1));
        auto t1 = std::chrono::steady_clock::now();
        float gpu_ms = 0.f;
        HIP_OK(hipEventElapsedTime(&gpu_ms, e0, e1));
        const double wall_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / calls;
        // (b) synchronised after every call
        auto t2 = std::chrono::steady_clock::now();
        for (int i = 0; i < calls; i++) {
            NTT_CALL(c.fn(d_x, d_y, d_z, o.batch, o.ps, s));
            HIP_OK(hipStreamSynchronize(s));
        }
        auto t3 = std::chrono::steady_clock::now();
        const double rt_us = std::chrono::duration<double, std::micro>(t3 - t2).count() / calls;
        printf("{\"op\": \"%s\", \"n\": %u, \"batch\": %zu, \"calls\": %d, \"back_to_back_us\": %.3f, "
               "\"gpu_events_us\": %.3f, \"round_trip_us\": %.3f}\n",
               c.name, n, o.batch, calls, wall_us, gpu_ms * 1e3 / calls, rt_us);
    }
    HIP_OK(hipEventDestroy(e0));
    HIP_OK(hipEventDestroy(e1));
    HIP_OK(hipStreamDestroy(s));
    HIP_OK(hipFree(d_x));
    HIP_OK(hipFree(d_y));
    HIP_OK(hipFree(d_z));
    return 0;
}

int main(int argc, char **argv)
{
    Opts o;
    if (argc < 3) {
        help_message();
        return -1;
    }
    for (int i = 1; i < argc;) {
        std::string a = argv[i];
        auto next = [&](void) -> const char * {
            if (i + 1 >= argc) { help_message(); exit(-1); }
            return argv[i + 1];
        };
        if (a == "-speedgpu") { o.option = atoi(next()); i += 2; }
        else if (a == "-param") {
            std::string p = next();
            o.ps = p == "ref" ? NTT_PARAM_REF : p == "p-I" ? NTT_PARAM_P_I : p == "p-III" ? NTT_PARAM_P_III
                 : p == "p-III-4096" ? NTT_PARAM_N4096 : p == "p-III-8192" ? NTT_PARAM_N8192 : -1;
            i += 2;
        }
        else if (a == "-batch") { o.batch = strtoull(next(), nullptr, 10); i += 2; }
        else if (a == "-reps") { o.reps = atoi(next()); i += 2; }
        else if (a == "-r") { o.random = true; o.seed = strtoull(next(), nullptr, 0); i += 2; }
        else if (a == "-pcie") { o.pcie = true; i += 1; }
        else if (a == "-debug") { o.debug = true; i += 1; }
        else { help_message(); return -1; }
    }
    uint32_t n, q, psi;
    if (ntt_param_info(o.ps, &n, &q, &psi, nullptr, nullptr, nullptr) != NTT_OK) {
        fprintf(stderr, "unknown parameter set\n");
        return -1;
    }
    printf("NTT Parameters==> NTTSIZE: %u P: %u psi: %u batch: %zu\n", n, q, psi, o.batch);
    switch (o.option) {
    case 4: report_polymul(o, "CT-CT", false); break;
    case 6: report_polymul(o, "CT-GS", false); break;
    case 7: report_polymul(o, "fused", true); break;
    case 8:
        for (int i = 0; i < 5; i++) report_polymul(o, "CT-GS", false);
        for (int i = 0; i < 5; i++) report_polymul(o, "fused", true);
        break;
    case 9: {
        int ok = 0;
        const double ms = run_fwdinv(o, &ok);
        printf("fwd+inv n=%u: %.4f ms per batch of %zu -> %.3e pairs/s, %.1f GB/s algorithmic; round trip %s\n", n, ms,
               o.batch, o.batch / ms * 1e3, o.batch * 16.0 * n / ms / 1e6, ok ? "Identical." : "Incorrect result.");
        return ok ? 0 : 1;
    }
    case 10: {
        int kat = -1;
        const double ms = run_polymul_host(o, &kat);
        printf("\n========================\ntest_NTT_negacyclic fused host->host (pipelined PCIe). Batch Size is %zu"
               "\n========================\n", o.batch);
        printf("Performance GPU fused host->host \n Time\t\t: % .4f ms. \nThroughput\t: %.2f Multiplications per second\n",
               ms, (double)o.batch / ms * 1000.0);
        if (kat >= 0) printf("all-ones KAT z[k] = 2k+2-n mod q: %s\n", kat ? "Identical." : "Incorrect result.");
        return kat == 0 ? 1 : 0;
    }
    case 11: {
        int kat = 0;
        const double ms = run_nussbaumer(o, &kat);
        printf("\n========================\ntest_nussbaumer GPU (mod 2^32-1). Batch Size is %zu\n========================\n",
               o.batch);
        printf("Performance GPU Nussbaumer \n Time\t\t: % .4f ms. \nThroughput\t: %.2f Multiplications per second\n", ms,
               (double)o.batch / ms * 1000.0);
        printf("all-ones KAT z[k] = 2k+2-n mod 2^32-1: %s\n", kat ? "Identical." : "Incorrect result.");
        return kat ? 0 : 1;
    }
    case 12: return run_latency(o);
    default: help_message(); return -1;
    }
    return 0;
}
