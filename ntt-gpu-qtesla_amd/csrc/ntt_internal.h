// ntt_internal.h -- internal interfaces between the library's translation
// units (not part of include/qtesla_ntt.h).
#pragma once
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
namespace qntt {
/* csrc/ntt_kernels.hip: records a hipError_t for ntt_last_hip_error() */
void set_last_hip(int e);
/* csrc/nussbaumer.hip: launches the Nussbaumer kernel; returns a hipError_t */
int nussbaumer_launch(int ps, int ring, const uint32_t *a, const uint32_t *b, uint32_t *c, size_t batch,
                      void *stream, int cus);
}  // namespace qntt
#endif
