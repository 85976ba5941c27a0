/*
 * ntt_oracle.c -- CPU ORACLE (test infrastructure only; see ntt_oracle.h).
 *
 * A plain-C restatement of the reference's algorithm for the north-star path.
 * Every function cites the reference file:line it follows.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load this library,
 * always as the checker / CPU baseline, never as the measured product.
 */
#include "ntt_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* Parameter sets                                                      */
/* ------------------------------------------------------------------ */
static uint32_t powmod(uint32_t b, uint64_t e, uint32_t q)
{
    uint64_t r = 1 % q, x = b % q;
    while (e) {
        if (e & 1) r = r * x % q;
        x = x * x % q;
        e >>= 1;
    }
    return (uint32_t)r;
}
static uint32_t invmod(uint32_t a, uint32_t q) { return powmod(a, q - 2, q); } /* q prime */

int oracle_params_get(int ps, oracle_params *o)
{
    oracle_params p;
    memset(&p, 0, sizeof p);
    switch (ps) {
    case 0: /* qTESLA-III-speed round 1: main.cuh:13-21, psi = Phi[1] (constants.h:11-13) */
        p.n = 1024; p.logn = 10; p.q = 8404993u; p.psi = 2083362u; break;
    case 1: /* qTESLA-p-I: psi = 3^((q-1)/2n), 3 = smallest primitive root */
        p.n = 1024; p.logn = 10; p.q = 343576577u; p.psi = powmod(3, (343576577u - 1) / 2048, 343576577u); break;
    case 2: /* qTESLA-p-III */
        p.n = 2048; p.logn = 11; p.q = 856145921u; p.psi = powmod(3, (856145921u - 1) / 4096, 856145921u); break;
    case 3: /* p-III's prime at n = 4096 (larger n; not a qTESLA set) */
        p.n = 4096; p.logn = 12; p.q = 856145921u; p.psi = powmod(3, (856145921u - 1) / 8192, 856145921u); break;
    case 4: /* p-III's prime at n = 8192 (q - 1 = 2^14 * 52255) */
        p.n = 8192; p.logn = 13; p.q = 856145921u; p.psi = powmod(3, (856145921u - 1) / 16384, 856145921u); break;
    default:
        return -1;
    }
    p.omega = (uint32_t)((uint64_t)p.psi * p.psi % p.q);   /* fg0 = psi^2 (main.cu:26) */
    p.omega_inv = invmod(p.omega, p.q);                     /* ig0 */
    p.n_inv = invmod(p.n, p.q);                             /* Ni  */
    if (o) *o = p;
    return 0;
}

/* bitrev -- NTT.cu:61-79 (same result as the loop there). */
uint32_t oracle_bitrev(uint32_t j, uint32_t bits)
{
    uint32_t r = 0;
    for (uint32_t b = 0; b < bits; b++) r |= ((j >> b) & 1u) << (bits - 1 - b);
    return r;
}

/* constants.h:3-35 table rules; host precompute main.cu:119-133
 * (tf0[i] = fg0^i, ti0[i] = tf0[n-i]), Phi = psi^i,
 * invPhi = Ni * psi^-i ("combined N-1 and invPhi", constants.h:19). */
int oracle_tables(int ps, uint32_t *bitrev_tbl, uint32_t *Phi, uint32_t *invPhi,
                  uint32_t *tf0, uint32_t *ti0)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return -1;
    const uint32_t q = p.q, n = p.n;
    const uint32_t psi_inv = invmod(p.psi, q);
    uint64_t ph = 1, iph = p.n_inv, w = 1, wi = 1;
    for (uint32_t i = 0; i < n; i++) {
        if (bitrev_tbl) bitrev_tbl[i] = oracle_bitrev(i, p.logn);
        if (Phi) Phi[i] = (uint32_t)ph;
        if (invPhi) invPhi[i] = (uint32_t)iph;
        if (tf0) tf0[i] = (uint32_t)w;
        if (ti0) ti0[i] = (uint32_t)wi;
        ph = ph * p.psi % q;
        iph = iph * psi_inv % q;
        w = w * p.omega % q;
        wi = wi * p.omega_inv % q;
    }
    return 0;
}

/* barrett_red -- NTT.cu:379-452, live lines 385-388 and 446-451, with
 * MIU = floor(2^48/P) (main.cuh:20).  Shifts are specific to P=8404993. */
uint32_t oracle_barrett_red_ref(uint64_t ip)
{
    const uint32_t P = 8404993u, MIU = 33489019u;
    uint32_t q1 = (uint32_t)(ip >> 23);
    uint64_t q2 = (uint64_t)q1 * (uint64_t)MIU;
    uint32_t q3 = (uint32_t)(q2 >> 25);
    uint32_t res = (uint32_t)(ip - (uint64_t)q3 * (uint64_t)P);
    while (res > P) res = res - P;
    return res;
}

/* _addModP_cpu / _subModP_cpu -- NTT.cu:33-47 (device twins :454-470). */
static inline uint32_t addq(uint32_t a, uint32_t b, uint32_t q)
{
    uint64_t ans = a + b;              /* 32-bit add, safe for q < 2^31 */
    return (uint32_t)((ans >= q) ? ans - q : ans);
}
static inline uint32_t subq(uint32_t a, uint32_t b, uint32_t q)
{
    if (a < b) a += q;
    uint64_t ans = a - b;
    return (uint32_t)((ans >= q) ? ans - q : ans);
}
static inline uint32_t mulq(uint32_t a, uint32_t b, uint32_t q)
{
    return (uint32_t)((uint64_t)a * b % q);
}
/* the reduction the reference GPU kernels use: barrett_red for P, else exact */
static inline uint32_t redq(uint64_t x, uint32_t q)
{
    return (q == 8404993u) ? oracle_barrett_red_ref(x) : (uint32_t)(x % q);
}

/* bit_reverse_copy -- NTT.cu:81-91 (bitrev(j,10) generalised to logn) */
void oracle_bit_reverse_copy(const uint32_t *ip, uint32_t *op, size_t batch, int ps)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    for (size_t k = 0; k < batch; k++)
        for (uint32_t j = 0; j < p.n; j++)
            op[p.n * k + j] = ip[p.n * k + oracle_bitrev(j, p.logn)];
}

/* radix2NTT -- NTT.cu:1201-1222: CT DIT, bit-reversed in, natural out. */
void oracle_radix2NTT(uint32_t *ip, const uint32_t *tw, size_t batch, int ps)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    const uint32_t n = p.n, q = p.q;
    for (size_t b = 0; b < batch; b++) {
        uint32_t *a = ip + b * n;
        uint32_t k = n / 2;
        for (uint32_t l = 1; l < n; l = 2 * l) {
            for (uint32_t s = 0; s < n; s = s + 2 * l) {
                for (uint32_t j = 0; j < l; j++) {
                    uint32_t temp = mulq(a[j + l + s], tw[j * k], q);
                    uint32_t op1 = addq(a[j + s], temp, q);
                    uint32_t op2 = subq(a[j + s], temp, q);
                    a[j + l + s] = op2;
                    a[j + s] = op1;
                }
            }
            k = k >> 1;
        }
    }
}

/* radix2INTT -- NTT.cu:1473-1494 (identical loop, inverse twiddles). */
void oracle_radix2INTT(uint32_t *ip, const uint32_t *tw, size_t batch, int ps)
{
    oracle_radix2NTT(ip, tw, batch, ps);
}

/* radix2NTTGS -- NTT.cu:1058-1084: GS DIF, natural in, bit-reversed out. */
void oracle_radix2NTTGS(uint32_t *ip, const uint32_t *tw, size_t batch, int ps)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    const uint32_t n = p.n, q = p.q;
    for (size_t b = 0; b < batch; b++) {
        uint32_t *a = ip + b * n;
        for (uint32_t level = 0; level < p.logn; level++) {
            uint32_t m = n >> level, stride = 1u << level;
            for (uint32_t k = 0; k < n; k = k + m) {
                for (uint32_t j = 0; j < m / 2; j++) {
                    uint32_t op1 = addq(a[k + j], a[k + j + m / 2], q);
                    uint32_t op2 = subq(a[k + j], a[k + j + m / 2], q);
                    op2 = mulq(op2, tw[(j * stride) % n], q);
                    a[k + j] = op1;
                    a[k + j + m / 2] = op2;
                }
            }
        }
    }
}

/* radix2INTTGS -- NTT.cu:1241-1266 (identical loop, inverse twiddles). */
void oracle_radix2INTTGS(uint32_t *ip, const uint32_t *tw, size_t batch, int ps)
{
    oracle_radix2NTTGS(ip, tw, batch, ps);
}

typedef struct {
    oracle_params p;
    uint32_t *Phi, *invPhi, *tf0, *ti0;
} tabset;

static int tabset_make(int ps, tabset *t)
{
    if (oracle_params_get(ps, &t->p)) return -1;
    size_t n = t->p.n;
    t->Phi = (uint32_t *)malloc(4 * n);
    t->invPhi = (uint32_t *)malloc(4 * n);
    t->tf0 = (uint32_t *)malloc(4 * n);
    t->ti0 = (uint32_t *)malloc(4 * n);
    oracle_tables(ps, NULL, t->Phi, t->invPhi, t->tf0, t->ti0);
    return 0;
}
static void tabset_free(tabset *t)
{
    free(t->Phi); free(t->invPhi); free(t->tf0); free(t->ti0);
}

/* FWD: twist (NTT.cu:1914-1918) + bit_reverse_copy (:1923) + radix2NTT (:1925). */
static void poly_ntt_with(uint32_t *x, size_t batch, int ps, const tabset *t, uint32_t *tmp)
{
    const uint32_t n = t->p.n, q = t->p.q;
    for (size_t b = 0; b < batch; b++) {
        uint32_t *a = x + b * n;
        for (uint32_t i = 0; i < n; i++) tmp[i] = mulq(a[i], t->Phi[i], q);
        for (uint32_t i = 0; i < n; i++) a[i] = tmp[oracle_bitrev(i, t->p.logn)];
        oracle_radix2NTT(a, t->tf0, 1, ps);
    }
}

/* INV (GS): radix2INTTGS (natural in, bit-reversed out) then the fused
 * bit_reverse_copy + invPhi of bit_reverse_copy_tbl_invPhi_gpu (NTT.cu:494-500). */
static void poly_invntt_with(uint32_t *X, size_t batch, int ps, const tabset *t, uint32_t *tmp)
{
    const uint32_t n = t->p.n, q = t->p.q;
    for (size_t b = 0; b < batch; b++) {
        uint32_t *a = X + b * n;
        memcpy(tmp, a, 4 * (size_t)n);
        oracle_radix2INTTGS(tmp, t->ti0, 1, ps);
        for (uint32_t i = 0; i < n; i++) a[i] = mulq(tmp[oracle_bitrev(i, t->p.logn)], t->invPhi[i], q);
    }
}

void oracle_poly_ntt(uint32_t *x, size_t batch, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    uint32_t *tmp = (uint32_t *)malloc(4 * (size_t)t.p.n);
    poly_ntt_with(x, batch, ps, &t, tmp);
    free(tmp);
    tabset_free(&t);
}

void oracle_poly_invntt(uint32_t *X, size_t batch, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    uint32_t *tmp = (uint32_t *)malloc(4 * (size_t)t.p.n);
    poly_invntt_with(X, batch, ps, &t, tmp);
    free(tmp);
    tabset_free(&t);
}

/* INV (CT): bit_reverse_copy (NTT.cu:1934) + radix2INTT (:1935) + invPhi (:1943-1946). */
void oracle_poly_invntt_ct(uint32_t *X, size_t batch, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    const uint32_t n = t.p.n, q = t.p.q;
    uint32_t *tmp = (uint32_t *)malloc(4 * (size_t)n);
    for (size_t b = 0; b < batch; b++) {
        uint32_t *a = X + b * n;
        for (uint32_t i = 0; i < n; i++) tmp[i] = a[oracle_bitrev(i, t.p.logn)];
        oracle_radix2INTT(tmp, t.ti0, 1, ps);
        for (uint32_t i = 0; i < n; i++) a[i] = mulq(tmp[i], t.invPhi[i], q);
    }
    free(tmp);
    tabset_free(&t);
}

/* pointwise_mult -- NTT.cu:1155-1160 (host form :1931-1932, exact %). */
void oracle_pointwise(uint32_t *c, const uint32_t *a, const uint32_t *b, size_t count, int ps)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    for (size_t i = 0; i < count; i++) c[i] = mulq(a[i], b[i], p.q);
}

/* test_NTT_nega_CT composition (NTT.cu:1908-1946) with the GS inverse. */
void oracle_poly_mul(uint32_t *c, const uint32_t *a, const uint32_t *b, size_t batch, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    const size_t n = t.p.n;
    uint32_t *A = (uint32_t *)malloc(4 * n), *B = (uint32_t *)malloc(4 * n), *tmp = (uint32_t *)malloc(4 * n);
    for (size_t k = 0; k < batch; k++) {
        memcpy(A, a + k * n, 4 * n);
        memcpy(B, b + k * n, 4 * n);
        poly_ntt_with(A, 1, ps, &t, tmp);
        poly_ntt_with(B, 1, ps, &t, tmp);
        oracle_pointwise(A, A, B, n, ps);
        poly_invntt_with(A, 1, ps, &t, tmp);
        memcpy(c + k * n, A, 4 * n);
    }
    free(A); free(B); free(tmp);
    tabset_free(&t);
}

/* O(n^2) definition: NTT_precom (NTT.cu:560-570) applied to the Phi-twisted
 * input: X[k] = sum_i (x_i Phi[i]) tf0[(i*k) mod n] = sum_i x_i psi^{(2k+1)i}. */
void oracle_ntt_direct(const uint32_t *x, uint32_t *X, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    const uint32_t n = t.p.n, q = t.p.q;
    for (uint32_t k = 0; k < n; k++) {
        uint64_t acc = 0;
        for (uint32_t i = 0; i < n; i++) {
            uint32_t xt = mulq(x[i], t.Phi[i], q);
            acc = (acc + (uint64_t)xt * t.tf0[(uint32_t)(((uint64_t)i * k) % n)]) % q;
        }
        X[k] = (uint32_t)acc;
    }
    tabset_free(&t);
}

/* schoolbook a*b mod (x^n + 1, q) */
void oracle_schoolbook_negacyclic(const uint32_t *a, const uint32_t *b, uint32_t *c, int ps)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    const uint32_t n = p.n, q = p.q;
    uint64_t *acc = (uint64_t *)calloc(n, sizeof(uint64_t));
    for (uint32_t i = 0; i < n; i++) {
        for (uint32_t j = 0; j < n; j++) {
            uint64_t prod = (uint64_t)a[i] * b[j] % q;
            uint32_t k = i + j;
            if (k < n) acc[k] = (acc[k] + prod) % q;
            else acc[k - n] = (acc[k - n] + q - prod) % q;
        }
    }
    for (uint32_t k = 0; k < n; k++) c[k] = (uint32_t)acc[k];
    free(acc);
}

/* ---------- serial restatement of the reference GPU kernels ---------- */

/* bit_reverse_copy_tbl_Phi_gpu -- NTT.cu:502-509 (clobbers ip like :506) */
static void k_bitrev_phi(uint32_t *ip, uint32_t *op, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q;
    for (size_t b = 0; b < B; b++) {
        for (uint32_t tid = 0; tid < n; tid++)
            ip[n * b + tid] = redq((uint64_t)ip[n * b + tid] * t->Phi[tid], q);
        /* __syncthreads() */
        for (uint32_t tid = 0; tid < n; tid++)
            op[n * b + tid] = ip[n * b + oracle_bitrev(tid, t->p.logn)];
    }
}
/* bit_reverse_copy_tbl_gpu -- NTT.cu:487-492 */
static void k_bitrev(const uint32_t *ip, uint32_t *op, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n;
    for (size_t b = 0; b < B; b++)
        for (uint32_t tid = 0; tid < n; tid++)
            op[n * b + tid] = ip[n * b + oracle_bitrev(tid, t->p.logn)];
}
/* bit_reverse_copy_tbl_invPhi_gpu -- NTT.cu:494-500 */
static void k_bitrev_invphi(const uint32_t *ip, uint32_t *op, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q;
    for (size_t b = 0; b < B; b++)
        for (uint32_t tid = 0; tid < n; tid++) {
            op[n * b + tid] = ip[n * b + oracle_bitrev(tid, t->p.logn)];
            op[n * b + tid] = redq((uint64_t)op[n * b + tid] * t->invPhi[tid], q);
        }
}
/* radix2NTT_gpu0 / radix2INTT_gpu0 -- NTT.cu:1436-1452 / 1374-1390 */
static void k_ct_gpu0(uint32_t *ip, const uint32_t *tw, uint32_t stride, uint32_t lvl, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q, k = n >> lvl, threads = n / stride;
    for (size_t b = 0; b < B; b++)
        for (uint32_t th = 0; th < threads; th++) {
            uint32_t m = 0, tid = th * stride;
            for (uint32_t j = tid; j < tid + stride / 2; j++) {
                uint32_t temp = redq((uint64_t)ip[b * n + j + stride / 2] * tw[m * k], q);
                uint32_t op1 = addq(ip[b * n + j], temp, q);
                uint32_t op2 = subq(ip[b * n + j], temp, q);
                ip[b * n + j + stride / 2] = op2;
                ip[b * n + j] = op1;
                m++;
            }
        }
}
/* radix2NTT_gpu1 / radix2INTT_gpu1 -- NTT.cu:1454-1470 / 1392-1408 */
static void k_ct_gpu1(uint32_t *ip, const uint32_t *tw, uint32_t stride, uint32_t lvl, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q, k = n >> lvl;
    for (size_t b = 0; b < B; b++)
        for (uint32_t tid = 0; tid < stride; tid++)
            for (uint32_t s = 0; s < n; s = s + 2 * stride) {
                uint32_t temp = redq((uint64_t)ip[b * n + tid + stride + s] * tw[tid * k], q);
                uint32_t op1 = addq(ip[b * n + tid + s], temp, q);
                uint32_t op2 = subq(ip[b * n + tid + s], temp, q);
                ip[b * n + tid + stride + s] = op2;
                ip[b * n + tid + s] = op1;
            }
}
/* radix2INTT_gpu2 -- NTT.cu:1411-1433: last CT stage + invPhi fold */
static void k_ct_gpu2(uint32_t *ip, const uint32_t *tw, uint32_t stride, uint32_t lvl, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q;
    k_ct_gpu1(ip, tw, stride, lvl, B, t);
    for (size_t b = 0; b < B; b++)
        for (uint32_t i = 0; i < n; i++)
            ip[b * n + i] = redq((uint64_t)ip[b * n + i] * t->invPhi[i], q);
}
/* GS_radix2INTT_gpu0 -- NTT.cu:1224-1240 (uses % P, :1236) */
static void k_gs_gpu0(uint32_t *ip, uint32_t level, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q, m = n >> level, stride = 1u << level;
    for (size_t b = 0; b < B; b++)
        for (uint32_t tid = 0; tid < m / 2; tid++)
            for (uint32_t k = 0; k < n; k = k + m) {
                uint32_t op1 = addq(ip[b * n + k + tid], ip[b * n + k + tid + m / 2], q);
                uint32_t op2 = subq(ip[b * n + k + tid], ip[b * n + k + tid + m / 2], q);
                op2 = mulq(op2, t->ti0[(tid * stride) % n], q);
                ip[b * n + k + tid] = op1;
                ip[b * n + k + tid + m / 2] = op2;
            }
}
/* GS_radix2INTT_gpu2 -- NTT.cu:1033-1056 */
static void k_gs_gpu2(uint32_t *ip, uint32_t lvl, size_t B, const tabset *t)
{
    const uint32_t n = t->p.n, q = t->p.q, m = n >> lvl, stride = 1u << lvl, threads = n / m;
    for (size_t b = 0; b < B; b++)
        for (uint32_t th = 0; th < threads; th++) {
            uint32_t tid = th * m;
            for (uint32_t j = 0; j < m / 2; j++) {
                uint32_t op1 = addq(ip[b * n + tid + j], ip[b * n + tid + j + m / 2], q);
                uint32_t op2 = subq(ip[b * n + tid + j], ip[b * n + tid + j + m / 2], q);
                op2 = redq((uint64_t)op2 * t->ti0[j * stride], q);
                ip[b * n + tid + j] = op1;
                ip[b * n + tid + j + m / 2] = op2;
            }
        }
}
/* pointwise_mult -- NTT.cu:1155-1160 */
static void k_pointwise(const uint32_t *a, const uint32_t *b, uint32_t *c, size_t B, const tabset *t)
{
    for (size_t i = 0; i < B * t->p.n; i++) c[i] = redq((uint64_t)a[i] * b[i], t->p.q);
}

/* forward CT kernel sequence: NTT.cu:2391-2400 generalised to logn stages */
static void k_fwd_sequence(uint32_t *X, size_t B, const tabset *t)
{
    for (uint32_t lvl = 1; lvl <= 5; lvl++) k_ct_gpu0(X, t->tf0, 1u << lvl, lvl, B, t);
    for (uint32_t lvl = 6; lvl <= t->p.logn; lvl++) k_ct_gpu1(X, t->tf0, 1u << (lvl - 1), lvl, B, t);
}

void oracle_gpu_ct_gs_polymul(uint32_t *x, uint32_t *y, uint32_t *z, size_t B, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    size_t sz = 4 * B * t.p.n;
    uint32_t *X = (uint32_t *)malloc(sz), *Y = (uint32_t *)malloc(sz), *Z = (uint32_t *)malloc(sz);
    k_bitrev_phi(x, X, B, &t);                                    /* :2388 */
    k_bitrev_phi(y, Y, B, &t);                                    /* :2389 */
    k_fwd_sequence(X, B, &t);                                     /* :2391-2400 */
    k_fwd_sequence(Y, B, &t);                                     /* :2402-2411 */
    k_pointwise(X, Y, Z, B, &t);                                  /* :2413 */
    for (uint32_t lvl = 0; lvl <= 4; lvl++) k_gs_gpu0(Z, lvl, B, &t);            /* :2415-2419 */
    for (uint32_t lvl = 5; lvl < t.p.logn; lvl++) k_gs_gpu2(Z, lvl, B, &t);      /* :2420-2424 */
    k_bitrev_invphi(Z, z, B, &t);                                 /* :2425 (into d_x) */
    free(X); free(Y); free(Z);
    tabset_free(&t);
}

void oracle_gpu_ct_ct_polymul(uint32_t *x, uint32_t *y, uint32_t *z, size_t B, int ps)
{
    tabset t;
    if (tabset_make(ps, &t)) return;
    size_t sz = 4 * B * t.p.n;
    uint32_t *X = (uint32_t *)malloc(sz), *Y = (uint32_t *)malloc(sz), *zz = (uint32_t *)malloc(sz);
    k_bitrev_phi(x, X, B, &t);                                    /* :2213 */
    k_bitrev_phi(y, Y, B, &t);                                    /* :2214 */
    k_fwd_sequence(X, B, &t);                                     /* :2216-2225 */
    k_fwd_sequence(Y, B, &t);                                     /* :2227-2236 */
    k_pointwise(X, Y, zz, B, &t);                                 /* :2238 */
    k_bitrev(zz, z, B, &t);                                       /* :2239 */
    for (uint32_t lvl = 1; lvl <= 5; lvl++) k_ct_gpu0(z, t.ti0, 1u << lvl, lvl, B, &t);          /* :2240-2244 */
    for (uint32_t lvl = 6; lvl < t.p.logn; lvl++) k_ct_gpu1(z, t.ti0, 1u << (lvl - 1), lvl, B, &t); /* :2245-2248 */
    k_ct_gpu2(z, t.ti0, 1u << (t.p.logn - 1), t.p.logn, B, &t);  /* :2249 */
    free(X); free(Y); free(zz);
    tabset_free(&t);
}

/* ---------------------------- RNG ----------------------------------- */
static inline uint64_t splitmix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
void oracle_fill_uniform(uint32_t *x, size_t batch, int ps, uint64_t seed, uint64_t first_poly)
{
    oracle_params p;
    if (oracle_params_get(ps, &p)) return;
    for (size_t b = 0; b < batch; b++)
        for (uint32_t i = 0; i < p.n; i++) {
            uint64_t idx = (first_poly + b) * p.n + i;
            uint64_t r = splitmix64(seed + (idx + 1) * 0x9E3779B97F4A7C15ULL);
            x[b * p.n + i] = (uint32_t)(((r >> 32) * (uint64_t)p.q) >> 32);
        }
}

/* ----------------------- CPU baseline timing ------------------------ */
/* The reference's serial CPU paths restated above, timed over a batch split
 * across pthreads (CPU baseline of bench.py; never the product path):
 *   ORACLE_OP_FWDINV  FWD + INV (E4 test_NTT_nega_CT path, NTT.cu:1908-1946)
 *   ORACLE_OP_FWD     FWD only (twist + bit_reverse_copy + radix2NTT)
 *   ORACLE_OP_INV     INV only (radix2INTTGS + bitrev + invPhi)
 *   ORACLE_OP_POLYMUL FWD(a), FWD(b), pointwise, INV  (oracle_poly_mul)
 *   ORACLE_OP_NUS_M32 nussbaumer_fft (NTT.cu:167-277) mod 2^32-1
 *   ORACLE_OP_NUS_Q   the same algorithm mod q                              */
typedef struct {
    int op, ps, reps;
    uint32_t *x, *y, *z;
    size_t batch;
    const tabset *t;
} job;

static void *run_job(void *arg)
{
    job *j = (job *)arg;
    const uint32_t n = j->t->p.n;
    uint32_t *tmp = (uint32_t *)malloc(4 * (size_t)n);
    for (int r = 0; r < j->reps; r++) {
        switch (j->op) {
        case ORACLE_OP_FWDINV:
            poly_ntt_with(j->x, j->batch, j->ps, j->t, tmp);
            poly_invntt_with(j->x, j->batch, j->ps, j->t, tmp);
            break;
        case ORACLE_OP_FWD: poly_ntt_with(j->x, j->batch, j->ps, j->t, tmp); break;
        case ORACLE_OP_INV: poly_invntt_with(j->x, j->batch, j->ps, j->t, tmp); break;
        case ORACLE_OP_POLYMUL: oracle_poly_mul(j->z, j->x, j->y, j->batch, j->ps); break;
        case ORACLE_OP_NUS_M32: oracle_nussbaumer(j->z, j->x, j->y, j->batch, n, 0); break;
        case ORACLE_OP_NUS_Q: oracle_nussbaumer(j->z, j->x, j->y, j->batch, n, j->t->p.q); break;
        }
    }
    free(tmp);
    return NULL;
}

/* Times `reps` passes of `op` over `batch` polys (x, and y/z for the
 * products) split across `threads` pthreads.  Returns wall seconds
 * (CLOCK_MONOTONIC), or -1 on a bad argument. */
double oracle_time_op(int op, uint32_t *x, uint32_t *y, uint32_t *z, size_t batch, int ps, int threads, int reps)
{
    tabset t;
    if (op < ORACLE_OP_FWDINV || op > ORACLE_OP_NUS_Q) return -1.0;
    if (op >= ORACLE_OP_POLYMUL && (!y || !z)) return -1.0;
    if (tabset_make(ps, &t)) return -1.0;
    if (threads < 1) threads = 1;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * threads);
    job *jobs = (job *)malloc(sizeof(job) * threads);
    struct timespec a, b;
    clock_gettime(CLOCK_MONOTONIC, &a);
    size_t per = (batch + threads - 1) / threads, start = 0;
    int used = 0;
    for (int i = 0; i < threads && start < batch; i++) {
        size_t cnt = (start + per <= batch) ? per : batch - start;
        const size_t off = start * t.p.n;
        jobs[i] = (job){op, ps, reps, x + off, y ? y + off : NULL, z ? z + off : NULL, cnt, &t};
        pthread_create(&th[i], NULL, run_job, &jobs[i]);
        start += cnt;
        used++;
    }
    for (int i = 0; i < used; i++) pthread_join(th[i], NULL);
    clock_gettime(CLOCK_MONOTONIC, &b);
    free(th);
    free(jobs);
    tabset_free(&t);
    return (double)(b.tv_sec - a.tv_sec) + 1e-9 * (double)(b.tv_nsec - a.tv_nsec);
}

double oracle_time_fwd_inv(uint32_t *x, size_t batch, int ps, int threads, int reps)
{
    return oracle_time_op(ORACLE_OP_FWDINV, x, NULL, NULL, batch, ps, threads, reps);
}
