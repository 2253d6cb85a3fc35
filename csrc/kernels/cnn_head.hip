// cnn_head (kernel in cnn_fwd.hip) as its own translation unit, compiled with the
// iterative-ilp machine scheduler (build.py FILE_FLAGS).
#define PDM_FWD_TU 2
#include "cnn_fwd.hip"
