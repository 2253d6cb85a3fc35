// fc1_fwd (kernel in cnn_fwd.hip) as its own translation unit, compiled with the max-ilp
// machine scheduler (build.py FILE_FLAGS): in-step 5.7 -> 5.3 us at B = 256.
#define PDM_FWD_TU 1
#include "cnn_fwd.hip"
