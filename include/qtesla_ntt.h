/*
 * qtesla_ntt.h -- C ABI of the MI355X (gfx950) batched negacyclic NTT engine.
 *
 * Drop-in boundary for the reference benlwk/ntt-gpu-qTESLA (NTT.cu).  The
 * reference has no library API: its "launch signature" is a family of
 * per-stage __global__ kernels launched <<<BATCH, T>>> by its test drivers
 * over caller-allocated, poly-major device buffers [BATCH][NTTSIZE] of
 * uint32 coefficients in [0,q).  Each entry point below replaces one whole
 * kernel sequence of those drivers (file:line cited per function) with one
 * launch of a hand-written CDNA4 kernel.
 *
 * Conventions (all entry points):
 *   - device pointers, poly-major [batch][n] uint32, coefficients in [0,q);
 *     the caller owns the memory, the library never allocates on the hot path;
 *   - `stream` is a hipStream_t (NULL = default stream); calls are
 *     asynchronous on that stream, reentrant across streams and devices;
 *   - return 0 on success, a negative NTT_ERR_* code otherwise (never abort);
 *   - `twiddleFactor` is accepted and ignored, exactly like the reference
 *     kernels' dead parameter (NTT.cu:1436 etc. read __constant__ tables).
 *   - inputs >= q are a contract violation (the reference silently returns
 *     non-congruent values for them).  This library tolerates inputs in
 *     [0, 2q): the output is then the exact canonical result for the input
 *     reduced mod q (DESIGN.md "lazy reduction bounds").  Outputs are
 *     always canonical, in [0, q).
 */
#ifndef QTESLA_NTT_H
#define QTESLA_NTT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- parameter sets ---------------------------------------------------- */
/* reference set: qTESLA-III-speed (round 1), main.cuh:13-21 + constants.h   */
#define NTT_PARAM_REF 0   /* n = 1024, q = 8404993,   psi = 2083362          */
#define NTT_PARAM_P_I 1   /* n = 1024, q = 343576577, psi = 3^((q-1)/2n)    */
#define NTT_PARAM_P_III 2 /* n = 2048, q = 856145921, psi = 3^((q-1)/2n)    */
/* Larger transforms over p-III's prime (q - 1 = 2^14 * 52255 admits
 * negacyclic n up to 8192), for the reference's n > 2048 dataflows (its
 * Stockham / CT2 kernels, NTT.cu:1085-1153, 1268-1337, 667-951): one wave
 * per polynomial (the n = 8192 products: a multi-wave four-step kernel).
 * For these sets every entry point is accepted except
 * poly_mul_nussbaumer (NTT_ERR_PARAM: its split is defined for n = 1024 /
 * 2048).  poly_mul / poly_mul_ntt are one fused launch; poly_bitrev_copy,
 * poly_ntt_bitrev and poly_invntt_bitrev are one launch each. */
#define NTT_PARAM_N4096 3 /* n = 4096, q = 856145921, psi = 3^((q-1)/2n)    */
#define NTT_PARAM_N8192 4 /* n = 8192, q = 856145921, psi = 3^((q-1)/2n)    */

/* ---- error codes ------------------------------------------------------- */
#define NTT_OK 0
#define NTT_ERR_PARAM (-1)   /* unknown param_set                              */
#define NTT_ERR_NULL (-2)    /* NULL device pointer with batch > 0             */
#define NTT_ERR_ALIGN (-3)   /* device pointer not 4-byte aligned (16-byte for  */
                             /* poly_pointwise and poly_mul_nussbaumer)        */
#define NTT_ERR_HIP (-4)     /* HIP runtime / launch error (ntt_last_hip_error)*/
#define NTT_ERR_SIZE (-5)    /* batch too large (at most 2^31 - 1 polynomials) */
#define NTT_ERR_ALIAS (-6)   /* forbidden partial overlap of in/out buffers    */

/* Parameter query: any out pointer may be NULL.
 * Replaces the compile-time macros P / NTTSIZE (main.cuh:14-16) and the root
 * constants fg0 / ig0 / Ni (main.cu:26). */
int ntt_param_info(int param_set, uint32_t *n, uint32_t *q, uint32_t *psi,
                   uint32_t *omega, uint32_t *omega_inv, uint32_t *n_inv);

/* Host copies of the constants.h-equivalent tables, n entries each (any
 * pointer may be NULL): bitrev_tbl (constants.h:3), Phi = psi^i (:11),
 * invPhi = n^-1 psi^-i (:19), tf0 = omega^i (:29), ti0 = omega^-i (:33).
 * For NTT_PARAM_REF they are bit-identical to constants.h. */
int ntt_get_tables(int param_set, uint32_t *bitrev_tbl, uint32_t *Phi,
                   uint32_t *invPhi, uint32_t *tf0, uint32_t *ti0);

/* Forward negacyclic NTT, in place, natural order in -> natural order out:
 *   X[k] = sum_i x_i psi^{(2k+1) i} mod q.
 * Replaces bit_reverse_copy_tbl_Phi_gpu + radix2NTT_gpu0 x5 + radix2NTT_gpu1 x5
 * (NTT.cu:2388-2400; kernels :502-509, :1436-1470) -- 12 launches -> 1. */
int poly_ntt(uint32_t *d_poly, const uint32_t *twiddleFactor, size_t batch,
             int param_set, void *stream);

/* Inverse negacyclic NTT, in place, natural -> natural (includes n^-1 and
 * psi^-i, i.e. invPhi):  x_i = n^-1 psi^-i sum_k X[k] omega^-ik.
 * Replaces GS_radix2INTT_gpu0 x5 + GS_radix2INTT_gpu2 x5 +
 * bit_reverse_copy_tbl_invPhi_gpu (NTT.cu:2415-2425; kernels :1224-1240,
 * :1033-1056, :494-500) -- 11 launches -> 1. */
int poly_invntt(uint32_t *d_poly, const uint32_t *twiddleFactor, size_t batch,
                int param_set, void *stream);

/* Out-of-place variants (d_out may equal d_in; partial overlap rejected).
 * Unlike bit_reverse_copy_tbl_Phi_gpu (NTT.cu:506) the input is never
 * clobbered when d_out != d_in. */
int poly_ntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch,
                 int param_set, void *stream);
int poly_invntt_oop(uint32_t *d_out, const uint32_t *d_in, size_t batch,
                    int param_set, void *stream);

/* Transforms with the NTT domain in bit-reversed order (out of place; d_out
 * may equal d_in, partial overlap rejected), for callers that keep the
 * reference's CT-CT ordering:
 *   poly_ntt_bitrev:    out[t] = X[brv(t)]  (= poly_ntt then poly_bitrev_copy)
 *   poly_invntt_bitrev: input in[t] = X[brv(t)], natural-order output; this
 *     is the CT inverse on bit-reversed input radix2INTT_gpu0 x5 + gpu1 x4 +
 *     gpu2 with its x invPhi (NTT.cu:2240-2249, kernels :1374-1433) -- 10
 *     launches -> 1; poly_bitrev_copy then poly_invntt_bitrev = poly_invntt.
 * Each costs one more LDS transpose per polynomial than the natural-order
 * transform (the bit-reversed side is not lane-contiguous in the pass-2
 * register layout). */
int poly_ntt_bitrev(uint32_t *d_out, const uint32_t *d_in, size_t batch,
                    int param_set, void *stream);
int poly_invntt_bitrev(uint32_t *d_out, const uint32_t *d_in, size_t batch,
                       int param_set, void *stream);

/* Bit-reversal permutation, out[b*n + t] = in[b*n + brv(t)] (log2 n bits),
 * any 32-bit words.  Replaces bit_reverse_copy_tbl_gpu (NTT.cu:487-492), used
 * by the CT-CT pipeline (:2239) to feed radix2INTT with bit-reversed input.
 * d_out may equal d_in (in place); partial overlap is rejected. */
int poly_bitrev_copy(uint32_t *d_out, const uint32_t *d_in, size_t batch,
                     int param_set, void *stream);

/* Fused negacyclic product c = a * b mod (x^n + 1, q), natural order.
 * Replaces the whole CT-GS pipeline of test_NTT_CT_GS_nega_gpu
 * (NTT.cu:2388-2425, 34 launches) and CT-CT (NTT.cu:2213-2249) with one
 * launch; d_c may alias d_a or d_b. */
int poly_mul(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b,
             size_t batch, int param_set, void *stream);

/* Fused product with the second operand already in the NTT domain:
 *   c = a * b mod (x^n + 1, q)  where  d_bhat = poly_ntt(b)  (natural order,
 *   this library's psi, entries < 2q).
 * qTESLA samples its public polynomial directly in the NTT domain; this is
 * the CT-GS driver (NTT.cu:2388-2425) with the second forward transform
 * (:2402-2411) dropped: two transforms of work per product instead of three.
 * d_c may alias d_a or d_bhat. */
int poly_mul_ntt(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_bhat,
                 size_t batch, int param_set, void *stream);

/* Nussbaumer negacyclic product (the paper's alternate algorithm): the
 * reference's single-polynomial CPU routine nussbaumer_fft (NTT.cu:167-277,
 * driver test_nussbaumer :1987-2005), batched on the GPU and extended from
 * n = 1024 to n = param_set's n (1024 or 2048; split m = 32, r = n/32).
 *   ring NTT_RING_M32: coefficients mod 2^32 - 1, the reference's ring
 *                      (NTT.cu:102-134); any 32-bit input, 0xFFFFFFFF is
 *                      read as zero, outputs canonical in [0, 2^32 - 1).
 *   ring NTT_RING_Q:   coefficients mod param_set's q, inputs < 2q, outputs
 *                      canonical -- bit-identical to poly_mul.
 * d_c may alias d_a or d_b.  All three pointers must be 16-byte aligned. */
#define NTT_RING_Q 0
#define NTT_RING_M32 1
int poly_mul_nussbaumer(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b,
                        size_t batch, int param_set, int ring, void *stream);

/* Pointwise product c[i] = a[i] * b[i] mod q over batch*n coefficients.
 * Replaces pointwise_mult (NTT.cu:1155-1160).  Inputs < 2q, canonical output;
 * all three pointers must be 16-byte aligned; d_c may alias d_a or d_b. */
int poly_pointwise(uint32_t *d_c, const uint32_t *d_a, const uint32_t *d_b,
                   size_t batch, int param_set, void *stream);

/* Device-side counter-based generator: coefficient i of poly p gets
 * splitmix64(seed + (idx+1)*0x9E3779B97F4A7C15) mapped to [0,q) by
 * multiply-high, idx = (first_poly + p) * n + i.  Lets benchmarks build
 * multi-GiB inputs on the device; any poly can be regenerated on the host. */
int ntt_fill_uniform(uint32_t *d_poly, size_t batch, int param_set,
                     uint64_t seed, uint64_t first_poly, void *stream);

/* ---- host-buffer (streamed) operation --------------------------------- */
/* The reference times its GPU pipelines host -> host: synchronous H2D, the
 * kernel sequence and D2H on the default stream (NTT.cu:2384-2428; SURVEY.md
 * §8(f) row 4).  A context pipelines that in chunks of `chunk_polys`
 * polynomials (0 -> 4096) over three event-chained HIP queues (H2D copies,
 * kernels, D2H copies) and `nslots` buffer slots (0 -> 3, at most 8):
 * chunk i's D2H, chunk i+1's kernel and chunk i+2's H2D overlap.  Each slot
 * owns 3 device and 3 pinned host buffers of chunk_polys*n words, on the
 * device that is current at creation.  Pinned host buffers (ntt_host_alloc,
 * hipHostMalloc, registered memory) are DMA'd directly; pageable ones are
 * staged through the slots' pinned buffers by host memcpy.  The calls are
 * synchronous: on return the outputs are in host memory.  h_out may equal
 * an input (in place); other overlaps are undefined.  A context serves one
 * host thread at a time. */
typedef struct ntt_host_ctx ntt_host_ctx;
int ntt_host_ctx_create(ntt_host_ctx **ctx, int param_set, size_t chunk_polys, int nslots);
int ntt_host_ctx_destroy(ntt_host_ctx *ctx);
/* host -> host forward / inverse transform (poly_ntt_oop / poly_invntt_oop) */
int poly_ntt_host(ntt_host_ctx *ctx, uint32_t *h_out, const uint32_t *h_in, size_t batch);
int poly_invntt_host(ntt_host_ctx *ctx, uint32_t *h_out, const uint32_t *h_in, size_t batch);
/* host -> host fused negacyclic product (poly_mul) */
int poly_mul_host(ntt_host_ctx *ctx, uint32_t *h_c, const uint32_t *h_a, const uint32_t *h_b, size_t batch);
/* pinned host memory for the calls above (NULL on failure) */
void *ntt_host_alloc(size_t bytes);
void ntt_host_free(void *p);

/* Last HIP error code seen by this thread (hipError_t as int), and a
 * static string for an NTT_ERR_* code. */
int ntt_last_hip_error(void);
const char *ntt_strerror(int code);

/* Diagnostic: on the current device, the number of bounded waits of the
 * n = 8192 fused products' per-polynomial barriers that expired since the
 * library was loaded (synchronises the device; every other kernel runs one
 * wave per polynomial and has none).  Always 0 unless the hardware schedule
 * broke the barrier; a launch that raised it produced invalid output. */
int ntt_sync_expiries(uint32_t *count);

/* Small-batch switch: writes to *max_batch the largest batch for which
 * entry point `op` (NTT_OP_*) of `param_set` runs the small-batch kernels
 * (one polynomial per workgroup; 0 = never); larger batches
 * run the batch kernels.  All give identical results; the thresholds are the
 * measured crossovers of their launch times, per (n, op).  The reference
 * has one launch shape for every batch (<<<BATCH, T>>>, NTT.cu:2216). */
#define NTT_OP_FWD 0     /* poly_ntt (in place; also poly_ntt_oop with d_out == d_in) */
#define NTT_OP_INV 1     /* poly_invntt (in place; also poly_invntt_oop, d_out == d_in) */
#define NTT_OP_FWD_BR 2  /* poly_ntt_bitrev                                           */
#define NTT_OP_INV_BR 3  /* poly_invntt_bitrev                                        */
#define NTT_OP_MUL 4     /* poly_mul                                                  */
#define NTT_OP_MUL_NTT 5 /* poly_mul_ntt                                              */
#define NTT_OP_FWD_OOP 6 /* poly_ntt_oop, distinct buffers                            */
#define NTT_OP_INV_OOP 7 /* poly_invntt_oop, distinct buffers                         */
int ntt_small_batch_max(int param_set, int op, size_t *max_batch);
/* Which kernel family entry point `op` of `param_set` runs at `batch`
 * polynomials: *radix = 4 / 8 / 16 for the one-polynomial-per-workgroup
 * kernels with radix-4 / 8 / 16 passes, 0 for the batch
 * kernels.  Diagnostic; every family gives identical results. */
int ntt_small_batch_radix(int param_set, int op, size_t batch, int *radix);

/* Library / kernel description for reports, ending in "src=<16 hex>" (a hash
 * of the library sources): writes at most len bytes, returns the length. */
int ntt_build_info(char *buf, size_t len);

#ifdef __cplusplus
}
#endif
#endif /* QTESLA_NTT_H */
