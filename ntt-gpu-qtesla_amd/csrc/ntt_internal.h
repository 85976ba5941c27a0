// ntt_internal.h -- diagnostic entry points (not part of include/qtesla_ntt.h).
#pragma once
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
/* op 0 = forward, 1 = inverse; variant 0 = full kernel, 1 = global load+store
 * only, 2 = arithmetic only (no global memory), 3 = load + LDS transpose + store. */
int ntt_debug_variant(int op, int variant, uint32_t *d_out, const uint32_t *d_in, size_t batch, int ps, void *stream);
#ifdef __cplusplus
}
namespace qntt {
/* csrc/nussbaumer.hip: launches the Nussbaumer kernel; returns a hipError_t */
/* csrc/ntt_kernels.hip: records a hipError_t for ntt_last_hip_error() */
void set_last_hip(int e);
int nussbaumer_launch(int ps, int ring, const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch,
                      void *stream, int cus);
}
#endif
