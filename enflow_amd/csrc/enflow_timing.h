// Internal: launch-site hooks of the per-kernel event timer (enflow_timing.hip).
#ifndef ENFLOW_TIMING_INTERNAL_H
#define ENFLOW_TIMING_INTERNAL_H
#include <hip/hip_runtime.h>

__attribute__((visibility("hidden"))) int enflow_tm_begin(const char* name, hipStream_t st);
__attribute__((visibility("hidden"))) void enflow_tm_end(int slot, hipStream_t st);

// ENFLOW_TIMED("kernel name", stream, hipLaunchKernelGGL(...));
#define ENFLOW_TIMED(NAME, ST, ...)              \
  do {                                           \
    const int tm_slot_ = enflow_tm_begin(NAME, ST); \
    __VA_ARGS__;                                 \
    enflow_tm_end(tm_slot_, ST);                 \
  } while (0)

#endif
