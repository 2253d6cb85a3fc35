// fc1_head (kernel in cnn_fwd.hip: fc1_fwd and the training head in one launch) as its own
// translation unit, compiled with the max-ilp machine scheduler as fc1_fwd is (build.py
// FILE_FLAGS).
#define PDM_FWD_TU 3
#include "cnn_fwd.hip"
