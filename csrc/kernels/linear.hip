// Reference model (Net = Linear(784, 10), fp32) — fused train / eval kernels.
//
// Replaces, per step, the reference's DataLoader transform + H2D copy +
// addmm + log_softmax + nll_loss + their backward + argmax/eq/sum/.item()
// (reference multi_proc_single_gpu.py:83-95; SURVEY.md §2.5: ~20 launches and
// 2 blocking syncs per step) with:
//   lin_train : LIN_ROWS rows per workgroup (epoch buffer or sampler gather),
//               normalise, logits, softmax-CE loss, dlogits, per-block partial
//               dW/db -> one fp32 slab per block; loss / correct into the fp64
//               train metrics; advances the optimizer-step counter
//   world size 1: the optimizer launch sums the slabs itself (optim.hip slab
//               segments) and advances the data-step counter
//   world size > 1: lin_reduce (fixed-order slab sum into the flat gradient
//               arena, data-step counter) -> bucket all-reduce -> optimizer
// and evaluation is a single launch over the whole test set.
//
// The step is latency-bound (B = 256 is 64 workgroups), so the kernel is built
// around the dependent-load chain: the weights go straight into registers as
// 16-B loads at entry, in flight together with the step counter -> image loads;
// a lane owns 4 consecutive features of every 256-feature chunk, so one LDS
// read of x feeds 40 FMAs.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int K = LIN_K;        // 784
constexpr int N = LIN_N;        // 10
constexpr int ROWS = LIN_ROWS;  // rows per block (train): 2, 4, 8 or 16
constexpr int NWV = ROWS < 4 ? ROWS : 4;     // waves per block
constexpr int RPW = ROWS / NWV;              // rows per wave
constexpr int THREADS = 64 * NWV;
static_assert(ROWS % NWV == 0 && RPW <= 4, "LIN_ROWS must be 1, 2, 4, 8, 12 or 16");
constexpr int K4 = K / 4;       // 196 float4 columns
constexpr int KJ = 4;           // 256-feature chunks per row (the last holds 16 features)
constexpr int Q16 = K / 16;     // 49 16-byte pieces per image row

// W[n][4 lane + 256 j .. +3] for every n, j (clamped past the row end: x is zero there)
__device__ __forceinline__ void load_w_regs(const float* __restrict__ W, float4 (&w)[N][KJ]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int k4 = min(lane + 64 * j, K4 - 1);
#pragma unroll
    for (int n = 0; n < N; ++n) w[n][j] = reinterpret_cast<const float4*>(W + n * K)[k4];
  }
}

// 16 uint8 pixels -> 16 normalised floats (lut = pdm_normalize table) at xrow[16 q ..]
__device__ __forceinline__ void put_pixels(float* xrow, int q, uint4 v, const float* lut) {
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    float4 f;
    f.x = lut[wd[c] & 0xff];
    f.y = lut[(wd[c] >> 8) & 0xff];
    f.z = lut[(wd[c] >> 16) & 0xff];
    f.w = lut[wd[c] >> 24];
    *reinterpret_cast<float4*>(xrow + 16 * q + 4 * c) = f;
  }
}

// One wave: the 10 logits of R rows (xs rows rows[0..R)), W in registers; every lane
// holds the results after the reduce.
template <int R>
__device__ __forceinline__ void wave_logits(const float (*xs)[K], const int (&rows)[R],
                                            const float4 (&w)[N][KJ],
                                            const float* __restrict__ bias, float (&lg)[R][N]) {
  const int lane = threadIdx.x & 63;
  float acc[R][N];
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int n = 0; n < N; ++n) acc[i][n] = 0.f;
#pragma unroll
  for (int j = 0; j < KJ; ++j) {
    const int k4 = lane + 64 * j;
    const bool on = k4 < K4;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
      if (on) x = reinterpret_cast<const float4*>(xs[rows[i]])[k4];
#pragma unroll
      for (int n = 0; n < N; ++n) {
        float a = acc[i][n];
        a = fmaf(x.x, w[n][j].x, a);
        a = fmaf(x.y, w[n][j].y, a);
        a = fmaf(x.z, w[n][j].z, a);
        a = fmaf(x.w, w[n][j].w, a);
        acc[i][n] = a;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i)
#pragma unroll
    for (int n = 0; n < N; ++n) lg[i][n] = wave_sum_dpp(acc[i][n]) + bias[n];
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

__global__ __launch_bounds__(THREADS) void lin_train_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels,
    const int32_t* __restrict__ idx, int64_t nrow, const int64_t* __restrict__ ctr, const StepRows sr,
    int B, const float* __restrict__ W, const float* __restrict__ bias, float* __restrict__ slab,
    double* __restrict__ metrics, int64_t* __restrict__ c1) {
  __shared__ __attribute__((aligned(16))) float xs[ROWS][K];
  __shared__ __attribute__((aligned(16))) float dl[ROWS][N];
  __shared__ float lut[256];
  __shared__ int lab[ROWS];
  __shared__ float red[ROWS][2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * ROWS;
  const int nrows = min(ROWS, B - row0);

  // 1. weights into registers: issued first, so they travel under the counter -> image chain
  float4 w[N][KJ];
  load_w_regs(W, w);
  // 2. the step's rows: counter -> (sampler index ->) 16-B image loads, labels
  const int64_t base = step_row(sr, nrow, *ctr, row0);
  PDM_CHECK(base + nrows <= nrow, "lin_train sample row past the epoch", base, nrow);
  // row -> sample (clamped: a counter driven past the epoch reads a valid row, not a fault)
  auto sample = [&](int r) -> int64_t {
    const int64_t i = min(base + r, nrow - 1);
    return idx ? (int64_t)idx[i] : i;
  };
  constexpr int NPIECE = ROWS * Q16;                 // 16-B pieces of the block's rows
  constexpr int PPT = (NPIECE + THREADS - 1) / THREADS;   // per thread
  uint4 px[PPT];
  int pr[PPT], pq[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int i = tid + THREADS * u;
    pr[u] = i / Q16;
    pq[u] = i - pr[u] * Q16;
    px[u] = make_uint4(0u, 0u, 0u, 0u);
    if (i < NPIECE && pr[u] < nrows)
      px[u] = reinterpret_cast<const uint4*>(images + sample(pr[u]) * K)[pq[u]];
  }
  if (tid < ROWS) lab[tid] = tid < nrows ? labels[sample(tid)] : 0;
  // normalisation table (built while the image is in flight)
#pragma unroll
  for (int i = tid; i < 256; i += THREADS) lut[i] = pdm_normalize((uint32_t)i);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PPT; ++u)
    if (tid + THREADS * u < NPIECE) put_pixels(xs[pr[u]], pq[u], px[u], lut);   // zeros past nrows
  __syncthreads();

  // 3. logits of rows wave + NWV i; lane i runs the CE of row wave + NWV i
  {
    int rows[RPW];
#pragma unroll
    for (int i = 0; i < RPW; ++i) rows[i] = wave + NWV * i;
    float lg[RPW][N];
    wave_logits<RPW>(xs, rows, w, bias, lg);
    if (lane < RPW) {
      const int r = wave + NWV * lane;
      float l[N], p[N];
#pragma unroll
      for (int n = 0; n < N; ++n) {
        l[n] = lg[0][n];
#pragma unroll
        for (int i = 1; i < RPW; ++i) l[n] = lane == i ? lg[i][n] : l[n];
      }
      const float invB = 1.f / (float)B;
      if (r < nrows) {
        const int y = lab[r];
        int correct;
        const float loss = row_xent(l, y, p, correct);
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

  // 4. partial dW = dl^T x (thread -> 4 consecutive features), db, metrics
  float* out = slab + (int64_t)blockIdx.x * LIN_SLAB;
  for (int c = tid; c < K4; c += THREADS) {
    float4 x[ROWS];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) x[r] = reinterpret_cast<const float4*>(xs[r])[c];
#pragma unroll
    for (int n = 0; n < N; ++n) {
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int r = 0; r < ROWS; ++r) {
        const float d = dl[r][n];
        s.x = fmaf(d, x[r].x, s.x);
        s.y = fmaf(d, x[r].y, s.y);
        s.z = fmaf(d, x[r].z, s.z);
        s.w = fmaf(d, x[r].w, s.w);
      }
      reinterpret_cast<float4*>(out + n * K)[c] = s;
    }
  }
  // db and the metrics on threads past the last dW column when there are any
  constexpr int TDB = THREADS > K4 + N ? K4 : THREADS - N - 1;
  if (tid >= TDB && tid < TDB + N) {
    const int n = tid - TDB;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) s += dl[r][n];
    out[N * K + n] = s;
  } else if (tid == TDB + N) {
    float l = 0.f, c = 0.f;
#pragma unroll
    for (int r = 0; r < ROWS; ++r) { l += red[r][0]; c += red[r][1]; }
    out[N * K + N] = l;
    out[N * K + N + 1] = c;
    // loss / correct go through the slab: the launch that sums the gradient slabs (the
    // optimizer at world size 1, lin_reduce otherwise) adds them to metrics[0..1] in a fixed
    // order; only the sample count is added here (one writer per step)
    if (metrics && blockIdx.x == 0) metrics[2] += (double)B;
  }
  // nothing in this launch reads the optimizer-step counter
  if (c1 && blockIdx.x == 0 && tid == 0) *c1 += 1;
}

// world size > 1: fixed-order slab sum into the gradient arena (then the all-reduce)
__global__ __launch_bounds__(256) void lin_reduce_kernel(
    const float* __restrict__ slab, int nblk, float* __restrict__ gW, float* __restrict__ gb,
    int64_t* c0, unsigned* c2, double* __restrict__ metrics) {
  if (metrics != nullptr && blockIdx.x == gridDim.x - 1) {   // the train-metrics workgroup
    pdm_slab_metrics(slab, nblk, N * K + N, LIN_SLAB, metrics);
    return;
  }
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < N * K + N) {
    float s = 0.f;
    for (int j0 = 0; j0 < nblk; j0 += 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slab[(int64_t)min(j0 + u, nblk - 1) * LIN_SLAB + e];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += (j0 + u < nblk) ? v[u] : 0.f;
    }
    if (e < N * K) gW[e] = s;
    else gb[e - N * K] = s;
  }
  pdm_bump_counters(c0, nullptr, c2);
}

__global__ __launch_bounds__(256) void lin_eval_kernel(
    const uint8_t* __restrict__ images, const int32_t* __restrict__ labels, int n_total,
    const float* __restrict__ W, const float* __restrict__ bias, double* __restrict__ metrics) {
  constexpr int EROWS = LIN_EVAL_ROWS;               // 16: 4 rows per wave
  __shared__ __attribute__((aligned(16))) float xs[EROWS][K];
  __shared__ float lut[256];
  __shared__ float red[EROWS][2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int row0 = blockIdx.x * EROWS;
  const int nrows = min(EROWS, n_total - row0);
  constexpr int NPIECE = EROWS * Q16;                // 784 pieces, 4 per thread at most
  uint4 px[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + 256 * u, r = i / Q16;
    px[u] = make_uint4(0u, 0u, 0u, 0u);
    if (i < NPIECE && r < nrows)
      px[u] = reinterpret_cast<const uint4*>(images + (int64_t)(row0 + r) * K)[i - r * Q16];
  }
  float4 w[N][KJ];
  load_w_regs(W, w);
  lut[tid] = pdm_normalize((uint32_t)tid);
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = tid + 256 * u, r = i / Q16;
    if (i < NPIECE) put_pixels(xs[r], i - r * Q16, px[u], lut);
  }
  __syncthreads();
  const int rows[4] = {wave, wave + 4, wave + 8, wave + 12};
  float lg[4][N];
  wave_logits<4>(xs, rows, w, bias, lg);
  if (lane < 4) {
    const int r = rows[lane];
    float l[N], p[N];
#pragma unroll
    for (int n = 0; n < N; ++n)
      l[n] = lane == 0 ? lg[0][n] : lane == 1 ? lg[1][n] : lane == 2 ? lg[2][n] : lg[3][n];
    float loss = 0.f;
    int correct = 0;
    if (r < nrows) loss = row_xent(l, labels[row0 + r], p, correct);
    red[r][0] = loss;
    red[r][1] = (float)correct;
  }
  __syncthreads();
  if (tid == 0) {
    double l = 0.0, c = 0.0;
    for (int r = 0; r < EROWS; ++r) { l += red[r][0]; c += red[r][1]; }
    atomicAdd(&metrics[0], l);
    atomicAdd(&metrics[1], c);
    atomicAdd(&metrics[2], (double)nrows);
  }
}

}  // namespace

void launch_lin_train(const uint8_t* images, const int32_t* labels, const int32_t* idx,
                      int64_t nrow, const int64_t* ctr, StepRows sr, int B, const float* W,
                      const float* b, float* slab, double* metrics, int64_t* c1, hipStream_t st) {
  const int nblk = (B + ROWS - 1) / ROWS;
  lin_train_kernel<<<nblk, THREADS, 0, st>>>(images, labels, idx, nrow, ctr, sr, B, W, b, slab,
                                         metrics, c1);
}

void launch_lin_reduce(const float* slab, int nblk, float* gW, float* gb, int64_t* c0,
                       unsigned* c2, double* metrics, hipStream_t st) {
  const int n = N * K + N;
  const int nb = (n + 255) / 256 + (metrics != nullptr ? 1 : 0);
  lin_reduce_kernel<<<nb, 256, 0, st>>>(slab, nblk, gW, gb, c0, c2, metrics);
}

void launch_lin_eval(const uint8_t* images, const int32_t* labels, int n_total, const float* W,
                     const float* b, double* metrics, hipStream_t st) {
  const int nblk = (n_total + LIN_EVAL_ROWS - 1) / LIN_EVAL_ROWS;
  lin_eval_kernel<<<nblk, 256, 0, st>>>(images, labels, n_total, W, b, metrics);
}
