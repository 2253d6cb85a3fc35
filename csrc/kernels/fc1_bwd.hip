// fc1_bwd (kernels in cnn_bwd.hip) as its own translation unit, compiled with the
// max-ilp machine scheduler (build.py FILE_FLAGS): in-step 11.4 -> 10.8 us at B = 256.
#define PDM_FC1_BWD_TU 1
#include "cnn_bwd.hip"
