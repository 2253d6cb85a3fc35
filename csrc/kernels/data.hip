// Epoch materialisation: gather the rank's samples in DistributedSampler order into a
// contiguous uint8 buffer once per epoch (47 MB at 60k samples, one streaming pass).
// The step kernels then read their batch as rows [ctr*B, ctr*B + B) of that buffer:
// one dependent load (the step counter) instead of counter -> index -> random row.
//
// The index vector is read straight from the pinned host buffer the sampler thread filled
// (zero-copy over the host link, 240 KB once per epoch), and the launch also resets the
// step counters: an epoch boundary is this one kernel on the compute stream, with no
// copy-engine hand-off and no extra fill launches in front of the next step.
#include "common.h"
#include "kernels.h"

namespace {

__global__ __launch_bounds__(256) void gather_epoch_kernel(const uint8_t* __restrict__ images,
                                                           const int32_t* __restrict__ labels,
                                                           const int32_t* __restrict__ idx, int n,
                                                           int nimg, uint8_t* __restrict__ out_images,
                                                           int32_t* __restrict__ out_labels,
                                                           int64_t* __restrict__ ctr, int nctr,
                                                           int64_t* __restrict__ step,
                                                           int64_t step_value) {
  if (blockIdx.x == 0 && threadIdx.x < nctr) ctr[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && step != nullptr) *step = step_value;
  // 16 rows per workgroup pass; a grid smaller than the row count strides over the rest
  for (int row = blockIdx.x * 16 + (threadIdx.x >> 4); row < n; row += gridDim.x * 16) {
    const int src_u = idx[row];
    PDM_CHECK(src_u >= 0 && src_u < nimg, "gather_epoch index", src_u, nimg);
    const int src = min(max(src_u, 0), nimg - 1);   // (a bad host index reads a valid row)
    const uint4* s = reinterpret_cast<const uint4*>(images + (int64_t)src * 784);
    uint4* d = reinterpret_cast<uint4*>(out_images + (int64_t)row * 784);
    for (int c = threadIdx.x & 15; c < 49; c += 16) d[c] = s[c];
    if ((threadIdx.x & 15) == 0) out_labels[row] = labels[src];
  }
}

}  // namespace

void launch_gather_epoch(const uint8_t* images, const int32_t* labels, const int32_t* idx, int n,
                         int nimg, uint8_t* out_images, int32_t* out_labels, int64_t* ctr,
                         int nctr, int64_t* step, int64_t step_value, int max_wgs, hipStream_t st) {
  if (n <= 0 && nctr == 0 && step == nullptr) return;
  int grid = max((n + 15) / 16, 1);
  if (max_wgs > 0 && grid > max_wgs) grid = max_wgs;
  gather_epoch_kernel<<<grid, 256, 0, st>>>(images, labels, idx, n, nimg, out_images,
                                                             out_labels, ctr, nctr, step, step_value);
}
