// Reference model (Net = Linear(784, 10), fp32) — fused train / eval kernels.
//
// Replaces, per step, the reference's DataLoader transform + H2D copy +
// addmm + log_softmax + nll_loss + their backward + argmax/eq/sum/.item()
// (reference multi_proc_single_gpu.py:83-95; SURVEY.md §2.5: ~20 launches and
// 2 blocking syncs per step) with two kernels:
//   lin_train : gather uint8 rows by the sampler index (device step counter),
//               normalise, logits, softmax-CE loss, dlogits, per-block partial
//               dW/db and metric sums -> one fp32 slab per block
//   lin_reduce: deterministic fixed-order sum of the slabs into the flat
//               gradient arena + fp64 metric accumulators; advances counters
// and evaluation is a single launch over the whole test set.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int K = LIN_K;        // 784
constexpr int N = LIN_N;        // 10
constexpr int ROWS = LIN_ROWS;  // rows per block (train)
constexpr int WPR = K / 4;      // 196 uint32 words per image

// Loads `nrows` images (gathered) into xs[ROWS][K] as normalised fp32; rows past
// nrows are zero.
__device__ __forceinline__ void load_rows(float (*xs)[K], const uint8_t* images, const int32_t* idx,
                                          int64_t base, int row0, int nrows, int rows_cap,
                                          bool gather, int64_t nrow = 0) {
  for (int i = threadIdx.x; i < rows_cap * WPR; i += blockDim.x) {
    const int r = i / WPR, w = i - r * WPR;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r < nrows) {
      // gather rows are clamped to the index buffer: a counter driven past the epoch
      // (misuse) reads a valid row instead of faulting
      const int64_t s = gather ? (int64_t)idx[min(base + row0 + r, nrow - 1)] : (int64_t)(row0 + r);
      const uint32_t word = reinterpret_cast<const uint32_t*>(images + s * K)[w];
      v.x = pdm_normalize(word & 0xff);
      v.y = pdm_normalize((word >> 8) & 0xff);
      v.z = pdm_normalize((word >> 16) & 0xff);
      v.w = pdm_normalize(word >> 24);
    }
    *reinterpret_cast<float4*>(&xs[r][4 * w]) = v;
  }
}

// One wave computes the 10 logits of row r (lane 0 holds them after the reduce).
__device__ __forceinline__ void row_logits(const float* xrow, const float* __restrict__ W,
                                           const float* __restrict__ bias, float (&lg)[N]) {
  const int lane = threadIdx.x & 63;
  float acc[N];
#pragma unroll
  for (int n = 0; n < N; ++n) acc[n] = 0.f;
  for (int k = lane; k < K; k += 64) {
    const float xv = xrow[k];
#pragma unroll
    for (int n = 0; n < N; ++n) acc[n] = fmaf(xv, W[n * K + k], acc[n]);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) lg[n] = wave_sum(acc[n]) + bias[n];
}

// log-softmax CE on one row's logits; returns loss, writes softmax probs, sets
// `correct` with torch.argmax tie-breaking (first maximal index).
__device__ __forceinline__ float row_xent(const float (&lg)[N], int y, float (&p)[N], int& correct) {
  float m = lg[0];
  int am = 0;
#pragma unroll
  for (int n = 1; n < N; ++n) {
    if (lg[n] > m) { m = lg[n]; am = n; }
  }
  float s = 0.f;
#pragma unroll
  for (int n = 0; n < N; ++n) { p[n] = expf(lg[n] - m); s += p[n]; }
  const float lse = m + logf(s);
  const float inv = 1.f / s;
#pragma unroll
  for (int n = 0; n < N; ++n) p[n] *= inv;
  correct = (am == y);
  float ly = lg[0];
#pragma unroll
  for (int n = 1; n < N; ++n) ly = (n == y) ? lg[n] : ly;
  return lse - ly;
}

__global__ __launch_bounds__(256) void lin_train_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ idx, int64_t nrow, const int64_t* __restrict__ ctr, int bfull,
    int B, const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ slab) {
  __shared__ float xs[ROWS][K];
  __shared__ float dl[ROWS][N];
  __shared__ float red[ROWS][2];
  const int row0 = blockIdx.x * ROWS;
  const int nrows = min(ROWS, B - row0);
  const int64_t base = (*ctr) * (int64_t)bfull;
  PDM_CHECK(base + row0 + nrows <= nrow, "lin_train sample row past the epoch", base + row0, nrow);
  load_rows(xs, images, idx, base, row0, nrows, ROWS, true, nrow);
  __syncthreads();

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const float invB = 1.f / (float)B;
  for (int r = wave; r < ROWS; r += 4) {
    float lg[N], p[N];
    row_logits(xs[r], W, bias, lg);
    if (lane == 0) {
      if (r < nrows) {
        const int y = labels[idx[min(base + row0 + r, nrow - 1)]];
        int correct;
        const float loss = row_xent(lg, y, p, correct);
#pragma unroll
        for (int n = 0; n < N; ++n) dl[r][n] = (p[n] - (n == y ? 1.f : 0.f)) * invB;
        red[r][0] = loss;
        red[r][1] = (float)correct;
      } else {
#pragma unroll
        for (int n = 0; n < N; ++n) dl[r][n] = 0.f;
        red[r][0] = 0.f;
        red[r][1] = 0.f;
      }
    }
  }
  __syncthreads();

  float* out = slab + (int64_t)blockIdx.x * LIN_SLAB;
  for (int e = threadIdx.x; e < N * K; e += blockDim.x) {
    const int n = e / K, k = e - n * K;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) s = fmaf(dl[r][n], xs[r][k], s);
    out[e] = s;
  }
  if (threadIdx.x < N) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) s += dl[r][threadIdx.x];
    out[N * K + threadIdx.x] = s;
  } else if (threadIdx.x == 64) {
    float l = 0.f, c = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) { l += red[r][0]; c += red[r][1]; }
    out[N * K + N] = l;
    out[N * K + N + 1] = c;
  }
}

__global__ __launch_bounds__(256) void lin_reduce_kernel(
    const float* __restrict__ slab, int nblk, float* __restrict__ gW, float* __restrict__ gb,
    double* __restrict__ metrics, int B, int64_t* c0, int64_t* c1, unsigned* c2) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < N * K + N + 2) {
    float s = 0.f;
    double sd = 0.0;
    for (int j = 0; j < nblk; ++j) {
      const float v = slab[(int64_t)j * LIN_SLAB + e];
      s += v;
      sd += (double)v;
    }
    if (e < N * K) gW[e] = s;
    else if (e < N * K + N) gb[e - N * K] = s;
    else if (e == N * K + N) { metrics[0] += sd; metrics[2] += (double)B; }
    else metrics[1] += sd;
  }
  pdm_bump_counters(c0, c1, c2);
}

__global__ __launch_bounds__(256) void lin_eval_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels, int n_total,
    const float* __restrict__ W, const float* __restrict__ bias, double* __restrict__ metrics) {
  constexpr int EROWS = 16;
  __shared__ float xs[EROWS][K];
  __shared__ float red[EROWS][2];
  const int row0 = blockIdx.x * EROWS;
  const int nrows = min(EROWS, n_total - row0);
  load_rows(xs, images, nullptr, 0, row0, nrows, EROWS, false);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int r = wave; r < EROWS; r += 4) {
    float lg[N], p[N];
    row_logits(xs[r], W, bias, lg);
    if (lane == 0) {
      float loss = 0.f;
      int correct = 0;
      if (r < nrows) loss = row_xent(lg, labels[row0 + r], p, correct);
      red[r][0] = loss;
      red[r][1] = (float)correct;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double l = 0.0, c = 0.0;
    for (int r = 0; r < EROWS; ++r) { l += red[r][0]; c += red[r][1]; }
    atomicAdd(&metrics[0], l);
    atomicAdd(&metrics[1], c);
    atomicAdd(&metrics[2], (double)nrows);
  }
}

}  // namespace

void launch_lin_train(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                      int64_t nrow, const int64_t* ctr, int bfull, int B, const float* W,
                      const float* b, float* slab, hipStream_t st) {
  const int nblk = (B + ROWS - 1) / ROWS;
  lin_train_kernel<<<nblk, 256, 0, st>>>(images, labels, idx, nrow, ctr, bfull, B, W, b, slab);
}

void launch_lin_reduce(const float* slab, int nblk, float* gW, float* gb, double* metrics, int B,
                       int64_t* c0, int64_t* c1, unsigned* c2, hipStream_t st) {
  const int n = N * K + N + 2;
  lin_reduce_kernel<<<(n + 255) / 256, 256, 0, st>>>(slab, nblk, gW, gb, metrics, B, c0, c1, c2);
}

void launch_lin_eval(const uint8_t* images, const int32_t* labels, int n_total, const float* W,
                     const float* b, double* metrics, hipStream_t st) {
  const int nblk = (n_total + 15) / 16;
  lin_eval_kernel<<<nblk, 256, 0, st>>>(images, labels, n_total, W, b, metrics);
}
