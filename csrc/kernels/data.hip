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

// Rows per workgroup pass: the pass's sampler indices are read from the host buffer by one
// wave at once (one host-link round trip per 64 rows; one per 4 rows when every 16-lane
// group read its own index -- the kernel was host-latency-bound at ~28 us per epoch), and
// the 64 rows (50 KB) are copied with every thread's 13 loads in flight before its stores.
constexpr int GR = 64;
constexpr int G_CHUNKS = 784 / 16;                       // 49 16-B chunks per image
constexpr int G_PER = (GR * G_CHUNKS + 255) / 256;       // 13 chunks per thread

__global__ __launch_bounds__(256) void gather_epoch_kernel(const uint8_t* __restrict__ images,
                                                           const int32_t* __restrict__ labels,
                                                           const int32_t* __restrict__ idx, int n,
                                                           int nimg, uint8_t* __restrict__ out_images,
                                                           int32_t* __restrict__ out_labels,
                                                           int64_t* __restrict__ ctr, int nctr,
                                                           int64_t* __restrict__ step,
                                                           int64_t step_value) {
  __shared__ int sidx[GR];
  if (blockIdx.x == 0 && threadIdx.x < nctr) ctr[threadIdx.x] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0 && step != nullptr) *step = step_value;
  const int t = threadIdx.x;
  // a grid smaller than the row count strides over the rest (uniform trip count)
  for (int r0 = blockIdx.x * GR; r0 < n; r0 += gridDim.x * GR) {
    const int nr = min(GR, n - r0);
    if (t < nr) {
      const int src_u = idx[r0 + t];
      PDM_CHECK(src_u >= 0 && src_u < nimg, "gather_epoch index", src_u, nimg);
      const int src = min(max(src_u, 0), nimg - 1);   // (a bad host index reads a valid row)
      sidx[t] = src;
      out_labels[r0 + t] = labels[src];
    }
    __syncthreads();
    uint4 v[G_PER];
#pragma unroll
    for (int k = 0; k < G_PER; ++k) {   // clamped unconditional loads (stores are masked)
      const int q = min(t + 256 * k, nr * G_CHUNKS - 1), rr = q / G_CHUNKS, c = q - rr * G_CHUNKS;
      v[k] = reinterpret_cast<const uint4*>(images + (int64_t)sidx[rr] * 784)[c];
    }
    uint4* d = reinterpret_cast<uint4*>(out_images + (int64_t)r0 * 784);
#pragma unroll
    for (int k = 0; k < G_PER; ++k) {
      const int q = t + 256 * k;
      if (q < nr * G_CHUNKS) d[q] = v[k];
    }
    __syncthreads();   // sidx is rewritten by the next pass
  }
}

}  // namespace

void launch_gather_epoch(const uint8_t* images, const int32_t* labels, const int32_t* idx, int n,
                         int nimg, uint8_t* out_images, int32_t* out_labels, int64_t* ctr,
                         int nctr, int64_t* step, int64_t step_value, int max_wgs, hipStream_t st) {
  if (n <= 0 && nctr == 0 && step == nullptr) return;
  int grid = max((n + GR - 1) / GR, 1);
  if (max_wgs > 0 && grid > max_wgs) grid = max_wgs;
  gather_epoch_kernel<<<grid, 256, 0, st>>>(images, labels, idx, n, nimg, out_images,
                                                             out_labels, ctr, nctr, step, step_value);
}
