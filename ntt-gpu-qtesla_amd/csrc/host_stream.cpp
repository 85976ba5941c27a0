// host_stream.cpp -- host-buffer ("streamed") operation of the engine,
// SURVEY.md §8(f) row 4.
//
// The reference times its GPU pipelines with the operands in host memory:
// cudaMemcpy H2D, the kernel sequence, cudaMemcpy D2H, all synchronous on the
// default stream (NTT.cu:2384-2428), so PCIe and the kernels never overlap.
// A qTESLA signing loop on the host needs exactly that host -> host
// operation.  This context pipelines it: the batch is cut into chunks that
// rotate over `nslots` buffer slots on three event-chained queues (H2D,
// kernels, D2H), so chunk i's D2H, chunk i+1's kernel and chunk i+2's H2D
// run at the same time (PCIe is full duplex), and the kernels are the same
// single-launch transforms as the device API.
//
// Host buffers that are pinned (hipHostMalloc / ntt_host_alloc / registered)
// are DMA'd directly.  Pageable buffers are staged through the context's
// pinned buffers with host memcpy, overlapped with the GPU work of the other
// streams; that path is host-memcpy bound.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/qtesla_ntt.h"
#include "ntt_internal.h"

struct ntt_host_ctx {
    int device = 0;
    int ps = 0;
    uint32_t n = 0;
    size_t chunk = 0;   // polynomials per chunk
    // three engines' queues: H2D copies, kernels, D2H copies
    hipStream_t s_in = nullptr, s_run = nullptr, s_out = nullptr;
    struct Slot {
        uint32_t *d_a = nullptr, *d_b = nullptr, *d_c = nullptr;   // device buffers, chunk*n words
        uint32_t *h_a = nullptr, *h_b = nullptr, *h_c = nullptr;   // pinned staging (pageable callers)
        hipEvent_t loaded = nullptr;    // H2D of the slot's chunk done (inputs free)
        hipEvent_t computed = nullptr;  // kernel done
        hipEvent_t stored = nullptr;    // D2H done (slot free)
        bool used = false;
        // pending staged output of the chunk last issued on this slot
        uint32_t *dst = nullptr;
        size_t words = 0;
    };
    std::vector<Slot> slots;
};

namespace {

int hip_fail(hipError_t e)
{
    qntt::set_last_hip((int)e);
    return NTT_ERR_HIP;
}

bool is_pinned(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();   // pageable memory: clear the sticky query error
        return false;
    }
    return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeManaged;
}

void release(ntt_host_ctx *c)
{
    for (hipStream_t s : {c->s_in, c->s_run, c->s_out})
        if (s) (void)hipStreamSynchronize(s);
    for (auto &s : c->slots) {
        (void)hipFree(s.d_a);
        (void)hipFree(s.d_b);
        (void)hipFree(s.d_c);
        (void)hipHostFree(s.h_a);
        (void)hipHostFree(s.h_b);
        (void)hipHostFree(s.h_c);
        for (hipEvent_t e : {s.loaded, s.computed, s.stored})
            if (e) (void)hipEventDestroy(e);
    }
    c->slots.clear();
    for (hipStream_t s : {c->s_in, c->s_run, c->s_out})
        if (s) (void)hipStreamDestroy(s);
    c->s_in = c->s_run = c->s_out = nullptr;
}

// flush a slot's staged output (if any) into the caller's buffer; its D2H
// must have completed
void drain_slot(ntt_host_ctx::Slot &s)
{
    if (s.dst) memcpy(s.dst, s.h_c, s.words * 4);
    s.dst = nullptr;
    s.words = 0;
}

// op: 0 = forward, 1 = inverse, 2 = poly_mul.
// Chunk i uses slot i % K.  The three queues are chained by events, so the
// H2D queue streams chunk after chunk while kernels and D2H copies of earlier
// chunks run; a slot is refilled only after its previous D2H (GPU-side wait).
// The host blocks only for pageable staging (input staging buffer free /
// staged output landed).
int run(ntt_host_ctx *c, int op, uint32_t *h_out, const uint32_t *h_a, const uint32_t *h_b, size_t batch)
{
    if (!c || c->slots.empty()) return NTT_ERR_NULL;
    if (batch == 0) return NTT_OK;
    if (!h_out || !h_a || (op == 2 && !h_b)) return NTT_ERR_NULL;
    if ((((uintptr_t)h_out) | ((uintptr_t)h_a) | ((uintptr_t)h_b)) & 3u) return NTT_ERR_ALIGN;
    if (batch > (size_t)0xFFFFFFFFu / 2) return NTT_ERR_SIZE;
    int prev = 0;
    hipError_t e = hipGetDevice(&prev);
    if (e != hipSuccess) return hip_fail(e);
    if (prev != c->device && (e = hipSetDevice(c->device)) != hipSuccess) return hip_fail(e);

    const bool pin_in = is_pinned(h_a) && (op != 2 || is_pinned(h_b));
    const bool pin_out = is_pinned(h_out);
    const size_t n = c->n, K = c->slots.size();
    int rc = NTT_OK;
    size_t i = 0;
    for (size_t first = 0; first < batch; first += c->chunk, ++i) {
        ntt_host_ctx::Slot &s = c->slots[i % K];
        const size_t polys = batch - first < c->chunk ? batch - first : c->chunk;
        const size_t words = polys * n, bytes = words * 4, off = first * n;
        const uint32_t *src_a = h_a + off, *src_b = op == 2 ? h_b + off : nullptr;
        if (s.used) {
            if (!pin_in && (e = hipEventSynchronize(s.loaded)) != hipSuccess) { rc = hip_fail(e); break; }
            if (s.dst) {
                if ((e = hipEventSynchronize(s.stored)) != hipSuccess) { rc = hip_fail(e); break; }
                drain_slot(s);
            }
            // the slot's previous D2H must be done before its buffers are overwritten
            if ((e = hipStreamWaitEvent(c->s_in, s.stored, 0)) != hipSuccess) { rc = hip_fail(e); break; }
        }
        if (!pin_in) {   // stage pageable input while the queues work on earlier chunks
            memcpy(s.h_a, src_a, bytes);
            src_a = s.h_a;
            if (op == 2) {
                memcpy(s.h_b, src_b, bytes);
                src_b = s.h_b;
            }
        }
        if ((e = hipMemcpyAsync(s.d_a, src_a, bytes, hipMemcpyHostToDevice, c->s_in)) != hipSuccess ||
            (op == 2 && (e = hipMemcpyAsync(s.d_b, src_b, bytes, hipMemcpyHostToDevice, c->s_in)) != hipSuccess) ||
            (e = hipEventRecord(s.loaded, c->s_in)) != hipSuccess ||
            (e = hipStreamWaitEvent(c->s_run, s.loaded, 0)) != hipSuccess) { rc = hip_fail(e); break; }
        s.used = true;
        if (op == 0) rc = poly_ntt_oop(s.d_c, s.d_a, polys, c->ps, c->s_run);
        else if (op == 1) rc = poly_invntt_oop(s.d_c, s.d_a, polys, c->ps, c->s_run);
        else rc = poly_mul(s.d_c, s.d_a, s.d_b, polys, c->ps, c->s_run);
        if (rc != NTT_OK) break;   // ntt_last_hip_error() already holds a HIP failure
        if ((e = hipEventRecord(s.computed, c->s_run)) != hipSuccess ||
            (e = hipStreamWaitEvent(c->s_out, s.computed, 0)) != hipSuccess) { rc = hip_fail(e); break; }
        uint32_t *dst = h_out + off;
        if ((e = hipMemcpyAsync(pin_out ? dst : s.h_c, s.d_c, bytes, hipMemcpyDeviceToHost, c->s_out)) != hipSuccess ||
            (e = hipEventRecord(s.stored, c->s_out)) != hipSuccess) { rc = hip_fail(e); break; }
        if (!pin_out) {
            s.dst = dst;
            s.words = words;
        }
    }
    // drain (also after an error, so no copy outlives the call)
    for (hipStream_t q : {c->s_in, c->s_run, c->s_out}) {
        e = hipStreamSynchronize(q);
        if (e != hipSuccess && rc == NTT_OK) rc = hip_fail(e);
    }
    for (auto &s : c->slots) {
        if (rc == NTT_OK) drain_slot(s);
        s.dst = nullptr;
        s.used = false;
    }
    if (prev != c->device) (void)hipSetDevice(prev);
    return rc;
}

}  // namespace

extern "C" {

int ntt_host_ctx_create(ntt_host_ctx **out, int param_set, size_t chunk_polys, int nslots)
{
    if (!out) return NTT_ERR_NULL;
    *out = nullptr;
    uint32_t n = 0;
    int rc = ntt_param_info(param_set, &n, nullptr, nullptr, nullptr, nullptr, nullptr);
    if (rc != NTT_OK) return rc;
    if (chunk_polys == 0) chunk_polys = 1u << 12;   // 32 MiB per buffer at n = 2048
    if (nslots <= 0) nslots = 3;
    if (nslots > 8 || chunk_polys > (size_t)0xFFFFFFFFu / 2) return NTT_ERR_SIZE;
    ntt_host_ctx *c = new (std::nothrow) ntt_host_ctx;
    if (!c) return NTT_ERR_SIZE;
    c->ps = param_set;
    c->n = n;
    c->chunk = chunk_polys;
    hipError_t e = hipGetDevice(&c->device);
    if (e != hipSuccess) {
        if (getenv("NTT_DEBUG")) fprintf(stderr, "ntt_host_ctx_create: hipGetDevice failed: %s\n", hipGetErrorString(e));
        delete c;
        return hip_fail(e);
    }
    const size_t bytes = chunk_polys * n * 4;
    int step = 0;
    auto fail = [&](hipError_t err) {
        if (getenv("NTT_DEBUG")) fprintf(stderr, "ntt_host_ctx_create: step %d failed: %s\n", step, hipGetErrorString(err));
        release(c);
        delete c;
        return hip_fail(err);
    };
    for (hipStream_t *q : {&c->s_in, &c->s_run, &c->s_out})
        if ((++step, e = hipStreamCreateWithFlags(q, hipStreamNonBlocking)) != hipSuccess) return fail(e);
    c->slots.resize(nslots);
    for (auto &s : c->slots) {
        for (uint32_t **d : {&s.d_a, &s.d_b, &s.d_c})
            if ((++step, e = hipMalloc(d, bytes)) != hipSuccess) return fail(e);
        for (uint32_t **h : {&s.h_a, &s.h_b, &s.h_c})
            if ((++step, e = hipHostMalloc(h, bytes)) != hipSuccess) return fail(e);
        for (hipEvent_t *ev : {&s.loaded, &s.computed, &s.stored})
            if ((++step, e = hipEventCreateWithFlags(ev, hipEventDisableTiming)) != hipSuccess) return fail(e);
    }
    *out = c;
    return NTT_OK;
}

int ntt_host_ctx_destroy(ntt_host_ctx *ctx)
{
    if (!ctx) return NTT_ERR_NULL;
    release(ctx);
    delete ctx;
    return NTT_OK;
}

int poly_ntt_host(ntt_host_ctx *ctx, uint32_t *h_out, const uint32_t *h_in, size_t batch)
{
    return run(ctx, 0, h_out, h_in, nullptr, batch);
}

int poly_invntt_host(ntt_host_ctx *ctx, uint32_t *h_out, const uint32_t *h_in, size_t batch)
{
    return run(ctx, 1, h_out, h_in, nullptr, batch);
}

int poly_mul_host(ntt_host_ctx *ctx, uint32_t *h_c, const uint32_t *h_a, const uint32_t *h_b, size_t batch)
{
    return run(ctx, 2, h_c, h_a, h_b, batch);
}

void *ntt_host_alloc(size_t bytes)
{
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes ? bytes : 1) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    return p;
}

void ntt_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

}  // extern "C"
