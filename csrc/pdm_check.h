// PDM_CHECK: device-side bounds checks of the debug build (shared by common.h and xgmi.h).
#pragma once
#include <hip/hip_runtime.h>

// Debug build only (PDM_DEBUG_BOUNDS=1 python -m pytorch_distributed_mnist_amd.build):
// device-side index checks that print the failing site ("PDM_CHECK failed: ..."); compiled
// out otherwise.  They do not trap: a trap ends the kernel in a queue error on a shared GPU
// box, so the checked sites clamp (or stay inside their allocation) and the debug run's log
// is searched for the message instead (tools/gpu_r6_debug.sh).
#ifdef PDM_DEBUG_BOUNDS
#define PDM_CHECK(cond, what, v0, v1)                                                      \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      printf("PDM_CHECK failed: %s (%lld, %lld) block %d thread %d\n", what, (long long)(v0), \
             (long long)(v1), (int)blockIdx.x, (int)threadIdx.x);                           \
    }                                                                                      \
  } while (0)
#else
#define PDM_CHECK(cond, what, v0, v1) \
  do {                                \
  } while (0)
#endif
