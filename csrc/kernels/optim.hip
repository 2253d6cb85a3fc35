// Fused flat-arena optimizer step (Adam / SGD-momentum) — one launch per step.
//
// torch runs Adam on GPU as ~7 _foreach_* launches with the bias corrections
// computed on the host.  This kernel sweeps the whole flat
// parameter arena once:
//   * DDP's 1/world_size gradient average is folded in as `grad_scale`,
//   * lr (fp64) and the step count live in device memory (graph-capturable;
//     the step counter was already advanced by an earlier kernel of the step),
//   * the op order matches torch's single-tensor Adam/SGD
//     (lerp / mul+addcmul / sqrt / div / add / addcdiv),
//   * optionally the same pass writes bf16 compute copies of the updated
//     weights: `shadow` (same layout) and `shadow_t` (2-D transposed), which the
//     bf16 forward/backward kernels read as MFMA operands. Transposed segments
//     are processed as 32x64 tiles staged through LDS so both the fp32 sweep and
//     the transposed bf16 store stay coalesced.
#include "common.h"
#include "kernels.h"

namespace {

constexpr int CHUNK = 2048;  // elements per block for plain segments (256 thr x 8)
constexpr int TR = 32, TC = 64;

struct Hyper {
  float lr, step_size, bc2_sqrt, beta1, beta2, eps, wd, mom, damp;
  int first, nesterov;
};

template <int KIND>
__device__ __forceinline__ Hyper make_hyper(const OptArgs& a) {
  Hyper h;
  const double lr = *a.lr;
  const int64_t t = *a.step;
  h.lr = (float)lr;
  h.beta1 = a.beta1; h.beta2 = a.beta2; h.eps = a.eps; h.wd = a.wd;
  h.mom = a.momentum; h.damp = a.dampening; h.nesterov = a.nesterov;
  h.first = (t <= 1);
  if (KIND == OPT_ADAM) {
    // torch: bias_correction1 = 1 - beta1 ** step (python double), step_size = lr / bc1,
    //        bias_correction2_sqrt = (1 - beta2 ** step) ** 0.5
    const double bc1 = 1.0 - pow((double)a.beta1_d, (double)t);
    const double bc2 = 1.0 - pow((double)a.beta2_d, (double)t);
    h.step_size = (float)(lr / bc1);
    h.bc2_sqrt = (float)sqrt(bc2);
  } else {
    h.step_size = 0.f;
    h.bc2_sqrt = 1.f;
  }
  return h;
}

template <int KIND>
__device__ __forceinline__ float update(float p, float g, float& m, float& v, const Hyper& h,
                                        float gs) {
  g *= gs;
  if (h.wd != 0.f) g = fmaf(h.wd, p, g);  // grad.add(param, alpha=wd)
  if (KIND == OPT_ADAM) {
    const float w = 1.f - h.beta1;  // exp_avg.lerp_(grad, 1 - beta1)
    m = (w < 0.5f) ? m + w * (g - m) : g - (g - m) * (1.f - w);
    v = v * h.beta2 + (1.f - h.beta2) * g * g;  // mul_(beta2).addcmul_(g, g, 1 - beta2)
    const float denom = sqrtf(v) / h.bc2_sqrt + h.eps;
    return p + (-h.step_size) * (m / denom);  // addcdiv_(exp_avg, denom, -step_size)
  } else {
    float d = g;
    if (h.mom != 0.f) {
      m = h.first ? d : m * h.mom + (1.f - h.damp) * d;
      d = h.nesterov ? d + h.mom * m : m;
    }
    return p + (-h.lr) * d;
  }
}

template <int KIND>
__global__ __launch_bounds__(256) void optim_kernel(OptArgs a) {
  // locate segment
  int si = 0;
#pragma unroll 1
  for (int i = 1; i < a.nseg; ++i)
    if ((int)blockIdx.x >= a.seg[i].first_block) si = i;
  const OptSeg& s = a.seg[si];
  const int lb = blockIdx.x - s.first_block;
  const Hyper h = make_hyper<KIND>(a);
  float* __restrict__ P = a.p + s.offset;
  const float* __restrict__ G = a.g + s.offset;
  float* __restrict__ M = a.m + s.offset;
  float* __restrict__ V = (KIND == OPT_ADAM) ? a.v + s.offset : nullptr;
  const int64_t numel = (int64_t)s.rows * s.cols;

  if (s.shadow_t == nullptr) {
    // plain segment: 8 contiguous floats per thread (2 x float4)
    const int64_t e0 = (int64_t)lb * CHUNK + threadIdx.x * 8;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int64_t e = e0 + q * 4;
      if (e + 4 <= numel) {
        float4 p = *reinterpret_cast<float4*>(P + e);
        const float4 g = *reinterpret_cast<const float4*>(G + e);
        float4 m = *reinterpret_cast<float4*>(M + e);
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (KIND == OPT_ADAM) v = *reinterpret_cast<float4*>(V + e);
        p.x = update<KIND>(p.x, g.x, m.x, v.x, h, a.grad_scale);
        p.y = update<KIND>(p.y, g.y, m.y, v.y, h, a.grad_scale);
        p.z = update<KIND>(p.z, g.z, m.z, v.z, h, a.grad_scale);
        p.w = update<KIND>(p.w, g.w, m.w, v.w, h, a.grad_scale);
        *reinterpret_cast<float4*>(P + e) = p;
        *reinterpret_cast<float4*>(M + e) = m;
        if (KIND == OPT_ADAM) *reinterpret_cast<float4*>(V + e) = v;
        if (s.shadow) {
          bf16x4 hb = {to_bf16(p.x), to_bf16(p.y), to_bf16(p.z), to_bf16(p.w)};
          *reinterpret_cast<bf16x4*>(s.shadow + e) = hb;
        }
      } else {
        for (int64_t j = e; j < numel && j < e + 4; ++j) {
          float m = M[j], v = (KIND == OPT_ADAM) ? V[j] : 0.f;
          const float p = update<KIND>(P[j], G[j], m, v, h, a.grad_scale);
          P[j] = p;
          M[j] = m;
          if (KIND == OPT_ADAM) V[j] = v;
          if (s.shadow) s.shadow[j] = to_bf16(p);
        }
      }
    }
    return;
  }

  // transposed-shadow segment: tile of TR rows x TC cols
  __shared__ bf16 tile[TC][TR + 2];
  const int tiles_c = (s.cols + TC - 1) / TC;
  const int tr0 = (lb / tiles_c) * TR, tc0 = (lb % tiles_c) * TC;
  // thread -> (row r, cols c..c+7): 32 rows x 8 col-groups = 256 threads
  const int r = threadIdx.x >> 3, cg = (threadIdx.x & 7) * 8;
  const int row = tr0 + r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = tc0 + cg + j;
    if (row < s.rows && col < s.cols) {
      const int64_t e = (int64_t)row * s.cols + col;
      float m = M[e], v = (KIND == OPT_ADAM) ? V[e] : 0.f;
      const float p = update<KIND>(P[e], G[e], m, v, h, a.grad_scale);
      P[e] = p;
      M[e] = m;
      if (KIND == OPT_ADAM) V[e] = v;
      const bf16 hb = to_bf16(p);
      if (s.shadow) s.shadow[e] = hb;
      tile[cg + j][r] = hb;
    }
  }
  __syncthreads();
  // write transposed: shadow_t[col][row]; thread -> (col c, rows rr..rr+3)
  const int c = threadIdx.x >> 2, rr = (threadIdx.x & 3) * 8;
  const int col = tc0 + c;
  if (col < s.cols) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int rw = tr0 + rr + j;
      if (rw < s.rows) s.shadow_t[(int64_t)col * s.rows + rw] = tile[c][rr + j];
    }
  }
}

}  // namespace

int opt_blocks_for(const OptSeg& s) {
  if (s.shadow_t) return ((s.rows + TR - 1) / TR) * ((s.cols + TC - 1) / TC);
  const int64_t n = (int64_t)s.rows * s.cols;
  return (int)((n + CHUNK - 1) / CHUNK);
}

void launch_optim(int kind, OptArgs& a, hipStream_t st) {
  int total = 0;
  for (int i = 0; i < a.nseg; ++i) {
    a.seg[i].first_block = total;
    total += opt_blocks_for(a.seg[i]);
  }
  if (total == 0) return;
  if (kind == OPT_ADAM)
    optim_kernel<OPT_ADAM><<<total, 256, 0, st>>>(a);
  else
    optim_kernel<OPT_SGD><<<total, 256, 0, st>>>(a);
}
