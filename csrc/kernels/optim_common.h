// Optimizer math shared by the optimizer kernel (optim.hip) and the world-size-1 fc1 update
// fused into cnn_bwd (cnn_bwd.hip): torch's single-tensor Adam / SGD op order, fp32.
#pragma once
#include "../common.h"
#include "../kernels.h"

namespace optim_detail {

struct Hyper {
  float lr, step_size, bc2_sqrt, beta1, beta2, eps, wd, mom, damp;
  int first, nesterov;
};

// A: OptArgs or FcUpdate (the same hyper-parameter field names)
// lr / t: the device-resident learning rate and step count (*a.lr, *a.step), passed in so a
// caller can load them early and keep the memory round trip off its critical path
template <int KIND, class A>
__device__ __forceinline__ Hyper make_hyper(const A& a, double lr, int64_t t) {
  Hyper h;
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

template <int KIND, class A>
__device__ __forceinline__ Hyper make_hyper(const A& a) {
  return make_hyper<KIND>(a, *a.lr, *a.step);
}

template <int KIND>
__device__ __forceinline__ float update(float p, float g, float& m, float& v, const Hyper& h,
                                        float gs) {
  // torch rounds after every op (mul_, add_, addcmul_, ...): no FMA contraction, which
  // also keeps every code path of this kernel bit-identical
#pragma clang fp contract(off)
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


}  // namespace optim_detail
