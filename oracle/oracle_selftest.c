/* oracle_selftest.c -- TEST INFRASTRUCTURE: exercises every oracle entry
 * point once per parameter set so it can run under ASan/UBSan (host only). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ntt_oracle.h"

int main(void)
{
    for (int ps = 0; ps < 3; ps++) {
        oracle_params p;
        if (oracle_params_get(ps, &p)) return 1;
        const size_t n = p.n, B = 3;
        uint32_t *x = malloc(4 * n * B), *y = malloc(4 * n * B), *c = malloc(4 * n * B), *d = malloc(4 * n * B);
        uint32_t *t[5];
        for (int i = 0; i < 5; i++) t[i] = malloc(4 * n);
        oracle_tables(ps, t[0], t[1], t[2], t[3], t[4]);
        oracle_fill_uniform(x, B, ps, 1, 0);
        oracle_fill_uniform(y, B, ps, 2, 0);
        memcpy(d, x, 4 * n * B);
        oracle_poly_ntt(d, B, ps);
        oracle_poly_invntt(d, B, ps);
        if (memcmp(d, x, 4 * n * B)) { printf("roundtrip fail %d\n", ps); return 1; }
        oracle_poly_ntt(d, B, ps);
        oracle_poly_invntt_ct(d, B, ps);
        if (memcmp(d, x, 4 * n * B)) { printf("ct roundtrip fail %d\n", ps); return 1; }
        oracle_poly_mul(c, x, y, B, ps);
        oracle_schoolbook_negacyclic(x, y, d, ps);
        if (memcmp(c, d, 4 * n)) { printf("polymul fail %d\n", ps); return 1; }
        memcpy(d, x, 4 * n * B);
        uint32_t *yy = malloc(4 * n * B);
        memcpy(yy, y, 4 * n * B);
        uint32_t *z = malloc(4 * n * B);
        oracle_gpu_ct_gs_polymul(d, yy, z, B, ps);
        if (memcmp(c, z, 4 * n * B)) { printf("gpu ct-gs fail %d\n", ps); return 1; }
        memcpy(d, x, 4 * n * B);
        memcpy(yy, y, 4 * n * B);
        oracle_gpu_ct_ct_polymul(d, yy, z, B, ps);
        if (memcmp(c, z, 4 * n * B)) { printf("gpu ct-ct fail %d\n", ps); return 1; }
        oracle_ntt_direct(x, z, ps);
        memcpy(d, x, 4 * n);
        oracle_poly_ntt(d, 1, ps);
        if (memcmp(d, z, 4 * n)) { printf("direct fail %d\n", ps); return 1; }
        oracle_pointwise(z, x, y, n * B, ps);
        oracle_time_fwd_inv(x, B, ps, 2, 1);
        for (int op = ORACLE_OP_FWD; op <= ORACLE_OP_NUS_Q; op++) oracle_time_op(op, x, y, z, B, ps, 2, 1);
        free(x); free(y); free(c); free(d); free(yy); free(z);
        for (int i = 0; i < 5; i++) free(t[i]);
    }
    printf("oracle selftest ok\n");
    return 0;
}
