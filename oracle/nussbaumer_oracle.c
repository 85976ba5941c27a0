/*
 * nussbaumer_oracle.c -- CPU ORACLE for the Nussbaumer negacyclic product.
 *
 * TEST INFRASTRUCTURE ONLY (see ntt_oracle.h).  Restates the reference's
 * single-polynomial CPU routine nussbaumer_fft (NTT.cu:167-277) and its
 * schoolbook `naive` (NTT.cu:147-165) with:
 *
 *   - the reference's ring Z/(2^32-1) (ones'-complement macros NTT.cu:102-134:
 *     modadd / modsub / modmul / modmuladd / moddiv2 / neg), op for op, when
 *     q == 0;  or exact arithmetic mod q (the qTESLA ring) when q != 0;
 *   - the reference's 32 x 32 split (m = 32 outer points, inner length
 *     r = n/32) generalised from n = 1024 to n = 2048: the inner ring
 *     Z[y]/(y^r + 1) then holds y^(r/m) as the primitive 2m-th root, so every
 *     rotation amount `sr` of NTT.cu:209-212 / :249-252 is scaled by r/m
 *     (= 1 at n = 1024, i.e. exactly the reference).
 *
 * Parity pins: the all-ones known answer of test_nussbaumer (NTT.cu:1987-2005:
 * z[k] = 2k + 2 - n mod 2^32-1) and agreement with the full-length `naive`
 * and with an independent numpy big-integer schoolbook (tests/).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ntt_oracle.h"

/* ---- the reference's ring Z/(2^32-1), NTT.cu:102-134 ------------------- */
static uint32_t m32_add(uint32_t a, uint32_t b) { uint32_t t = a + b; return t + (t < a); }
static uint32_t m32_sub(uint32_t a, uint32_t b) { return (a - b) - (b > a); }
static uint32_t m32_muladd(uint32_t c, uint32_t a, uint32_t b)
{
    uint64_t T = (uint64_t)a * b + c;
    return m32_add((uint32_t)T, (uint32_t)(T >> 32));
}
static uint32_t m32_normalize(uint32_t a) { return a + (a == 0xFFFFFFFFu); }
static uint32_t m32_div2(uint32_t a) { return (uint32_t)(((uint64_t)a + (uint64_t)(uint32_t)(0u - (a & 1u))) >> 1); }
static uint32_t m32_moddiv2(uint32_t a) { return m32_div2(m32_normalize(a)); }
static uint32_t m32_neg(uint32_t a) { return m32_normalize(0xFFFFFFFFu - a); }

/* ---- ring dispatch: q == 0 -> Z/(2^32-1), else Z/q ---------------------- */
typedef struct { uint32_t q; } ring;
static uint32_t r_add(ring R, uint32_t a, uint32_t b)
{
    return R.q ? (uint32_t)(((uint64_t)a + b) % R.q) : m32_add(a, b);
}
static uint32_t r_sub(ring R, uint32_t a, uint32_t b)
{
    return R.q ? (uint32_t)(((uint64_t)a + R.q - b) % R.q) : m32_sub(a, b);
}
static uint32_t r_muladd(ring R, uint32_t c, uint32_t a, uint32_t b)
{
    return R.q ? (uint32_t)(((uint64_t)a * b + c) % R.q) : m32_muladd(c, a, b);
}
static uint32_t r_mul(ring R, uint32_t a, uint32_t b)   /* modmul (NTT.cu:111-115) = muladd with c = 0 */
{
    return r_muladd(R, 0, a, b);
}
static uint32_t r_div2(ring R, uint32_t a)
{
    if (!R.q) return m32_moddiv2(a);
    return (a & 1u) ? (uint32_t)(((uint64_t)a + R.q) >> 1) : a >> 1;
}
static uint32_t r_neg(ring R, uint32_t a) { return R.q ? (a ? R.q - a : 0) : m32_neg(a); }

/* reverse() (NTT.cu:139-145): 32-bit bit reversal */
static uint32_t reverse32(uint32_t x)
{
    x = ((x & 0xaaaaaaaau) >> 1) | ((x & 0x55555555u) << 1);
    x = ((x & 0xccccccccu) >> 2) | ((x & 0x33333333u) << 2);
    x = ((x & 0xf0f0f0f0u) >> 4) | ((x & 0x0f0f0f0fu) << 4);
    x = ((x & 0xff00ff00u) >> 8) | ((x & 0x00ff00ffu) << 8);
    return (x >> 16) | (x << 16);
}

/* naive (NTT.cu:147-165): negacyclic product of length n in the given ring,
 * same accumulation order (A over j <= i, B over the wrapped terms). */
static void naive_ring(ring R, uint32_t *z, const uint32_t *x, const uint32_t *y, unsigned n)
{
    for (unsigned i = 0; i < n; i++) {
        uint32_t B = 0, A = r_mul(R, x[0], y[i]);
        unsigned j, k;
        for (j = 1; j <= i; j++) A = r_muladd(R, A, x[j], y[i - j]);
        for (k = 1; j < n; j++, k++) B = r_muladd(R, B, x[j], y[n - k]);
        z[i] = r_sub(R, A, B);
    }
}

/* nussbaumer_fft (NTT.cu:167-277) with m = 32 and r = n / 32. */
static int nussbaumer_one(ring R, uint32_t *z, const uint32_t *x, const uint32_t *y, unsigned n)
{
    enum { M = 32, LM = 5, K = 2 * M };
    const unsigned r = n / M, sc = r / M;   /* sc: rotation scale, 1 at n = 1024 */
    uint32_t *X1 = malloc(sizeof(uint32_t) * K * r), *Y1 = malloc(sizeof(uint32_t) * K * r);
    uint32_t *Z1 = malloc(sizeof(uint32_t) * K * r), *T1 = malloc(sizeof(uint32_t) * r);
    if (!X1 || !Y1 || !Z1 || !T1) { free(X1); free(Y1); free(Z1); free(T1); return -1; }
#define AT(P, i, a) (P)[(size_t)(i) * r + (a)]

    for (unsigned i = 0; i < M; i++)       /* NTT.cu:193-201: X1[i][j] = x[32j+i], duplicated */
        for (unsigned j = 0; j < r; j++) {
            AT(X1, i, j) = AT(X1, i + M, j) = x[M * j + i];
            AT(Y1, i, j) = AT(Y1, i + M, j) = y[M * j + i];
        }

    for (int j = LM - 1; j >= 0; j--) {    /* forward, NTT.cu:203-244 */
        for (unsigned i = 0; i < (1u << (LM - j)); i++) {
            const uint32_t ssr = reverse32(i);
            for (unsigned t = 0; t < (1u << j); t++) {
                const unsigned sr = sc * ((ssr >> (32 - LM + j)) << j);
                const unsigned s = i << (j + 1), I = s + t, L = s + t + (1u << j);
                uint32_t *P[2] = {X1, Y1};
                for (int o = 0; o < 2; o++) {
                    for (unsigned a = sr; a < r; a++) T1[a] = AT(P[o], L, a - sr);
                    for (unsigned a = 0; a < sr; a++) T1[a] = r_neg(R, AT(P[o], L, r + a - sr));
                    for (unsigned a = 0; a < r; a++) {
                        AT(P[o], L, a) = r_sub(R, AT(P[o], I, a), T1[a]);
                        AT(P[o], I, a) = r_add(R, AT(P[o], I, a), T1[a]);
                    }
                }
            }
        }
    }

    for (unsigned i = 0; i < K; i++) naive_ring(R, &AT(Z1, i, 0), &AT(X1, i, 0), &AT(Y1, i, 0), r);

    for (int j = 0; j <= LM; j++) {        /* inverse, NTT.cu:248-270 */
        for (unsigned i = 0; i < (1u << (LM - j)); i++) {
            /* NTT.cu:251 shifts by 32 when j == LM (i == 0 there, sr = 0) */
            const uint32_t ssr = reverse32(i);
            const unsigned sr = j == LM ? 0 : sc * ((ssr >> (32 - LM + j)) << j);
            for (unsigned t = 0; t < (1u << j); t++) {
                const unsigned s = i << (j + 1), A = s + t, B = s + t + (1u << j);
                for (unsigned a = 0; a < r; a++) {
                    T1[a] = r_div2(R, r_sub(R, AT(Z1, A, a), AT(Z1, B, a)));
                    AT(Z1, A, a) = r_div2(R, r_add(R, AT(Z1, A, a), AT(Z1, B, a)));
                }
                for (unsigned a = 0; a < r - sr; a++) AT(Z1, B, a) = T1[a + sr];
                for (unsigned a = r - sr; a < r; a++) AT(Z1, B, a) = r_neg(R, T1[a - (r - sr)]);
            }
        }
    }

    for (unsigned i = 0; i < M; i++) {     /* NTT.cu:272-277 */
        z[i] = r_sub(R, AT(Z1, i, 0), AT(Z1, M + i, r - 1));
        for (unsigned j = 1; j < r; j++) z[M * j + i] = r_add(R, AT(Z1, i, j), AT(Z1, M + i, j - 1));
    }
#undef AT
    free(X1); free(Y1); free(Z1); free(T1);
    return 0;
}

int oracle_nussbaumer(uint32_t *z, const uint32_t *x, const uint32_t *y, size_t batch, uint32_t n, uint32_t q)
{
    if (n != 1024 && n != 2048) return -1;
    ring R = {q};
    for (size_t b = 0; b < batch; b++)
        if (nussbaumer_one(R, z + b * n, x + b * n, y + b * n, n)) return -1;
    return 0;
}

int oracle_naive_negacyclic(uint32_t *z, const uint32_t *x, const uint32_t *y, size_t batch, uint32_t n, uint32_t q)
{
    if (n == 0) return -1;
    ring R = {q};
    for (size_t b = 0; b < batch; b++) naive_ring(R, z + b * n, x + b * n, y + b * n, n);
    return 0;
}

uint32_t oracle_m32_canon(uint32_t a) { return m32_normalize(a); }
