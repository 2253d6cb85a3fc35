// Python bindings: validate torch tensors on the host, then launch on the
// current HIP stream (so calls compose with torch.cuda.graph capture).
// Every shape the kernels assume is checked here before any launch.
#include <c10/core/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include "kernels.h"

namespace py = pybind11;
void register_comm(py::module& m);

namespace {

hipStream_t cur_stream(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.get_device()).stream();
}

void need(const at::Tensor& t, at::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a HIP device tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void need_numel(const at::Tensor& t, int64_t n, const char* name) {
  TORCH_CHECK(t.numel() >= n, name, " has ", t.numel(), " elements, need >= ", n);
}

void need_aligned(const void* p, int bytes, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(p) % bytes == 0, name, " must be ", bytes,
              "-byte aligned");
}

template <typename T>
T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }

int64_t* opt_i64(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  need(*t, at::kLong, "counter");
  return ptr<int64_t>(*t);
}

// Common checks for the gathered-data inputs of a training step.
void check_data(const at::Tensor& images, const at::Tensor& labels, const at::Tensor& idx,
                const at::Tensor& ctr, int64_t bfull, int64_t B) {
  need(images, at::kByte, "images");
  need(labels, at::kInt, "labels");
  need(idx, at::kInt, "idx");
  need(ctr, at::kLong, "ctr");
  TORCH_CHECK(images.dim() == 2 && images.size(1) == 784, "images must be [N, 784]");
  TORCH_CHECK(labels.numel() == images.size(0), "labels must be [N]");
  TORCH_CHECK(B >= 1 && B <= bfull, "batch ", B, " must be in [1, ", bfull, "]");
  TORCH_CHECK(ctr.numel() >= 1, "ctr must hold at least one counter");
  need_aligned(images.data_ptr(), 4, "images");
  // The step counter lives on the device; the host keeps steps within the index
  // vector (TrainProgram only issues steps_per_epoch steps per upload), so the
  // kernels' reads idx[ctr*bfull + i] stay in range.
}

// ------------------------------------------------------------------ linear
void lin_train(at::Tensor images, at::Tensor labels, at::Tensor idx, at::Tensor ctr, int64_t bfull,
               int64_t B, at::Tensor W, at::Tensor b, at::Tensor slab) {
  c10::DeviceGuard g(images.device());
  check_data(images, labels, idx, ctr, bfull, B);
  need(W, at::kFloat, "W");
  need(b, at::kFloat, "b");
  need(slab, at::kFloat, "slab");
  TORCH_CHECK(W.numel() == LIN_N * LIN_K && b.numel() == LIN_N, "W/b must be [10,784]/[10]");
  const int64_t nblk = (B + LIN_ROWS - 1) / LIN_ROWS;
  need_numel(slab, nblk * LIN_SLAB, "slab");
  need_aligned(slab.data_ptr(), 16, "slab");
  launch_lin_train(images.data_ptr<uint8_t>(), labels.data_ptr<int32_t>(), idx.data_ptr<int32_t>(),
                   ctr.data_ptr<int64_t>(), (int)bfull, (int)B, W.data_ptr<float>(),
                   b.data_ptr<float>(), slab.data_ptr<float>(), cur_stream(images));
}

void lin_reduce(at::Tensor slab, int64_t B, at::Tensor gW, at::Tensor gb, at::Tensor metrics,
                c10::optional<at::Tensor> c0, c10::optional<at::Tensor> c1) {
  c10::DeviceGuard g(slab.device());
  need(slab, at::kFloat, "slab");
  need(gW, at::kFloat, "gW");
  need(gb, at::kFloat, "gb");
  need(metrics, at::kDouble, "metrics");
  const int64_t nblk = (B + LIN_ROWS - 1) / LIN_ROWS;
  need_numel(slab, nblk * LIN_SLAB, "slab");
  TORCH_CHECK(gW.numel() == LIN_N * LIN_K && gb.numel() == LIN_N, "bad grad views");
  need_numel(metrics, 3, "metrics");
  launch_lin_reduce(slab.data_ptr<float>(), (int)nblk, gW.data_ptr<float>(), gb.data_ptr<float>(),
                    metrics.data_ptr<double>(), (int)B, opt_i64(c0), opt_i64(c1),
                    cur_stream(slab));
}

void lin_eval(at::Tensor images, at::Tensor labels, at::Tensor W, at::Tensor b,
              at::Tensor metrics) {
  c10::DeviceGuard g(images.device());
  need(images, at::kByte, "images");
  need(labels, at::kInt, "labels");
  need(W, at::kFloat, "W");
  need(b, at::kFloat, "b");
  need(metrics, at::kDouble, "metrics");
  TORCH_CHECK(images.dim() == 2 && images.size(1) == 784, "images must be [N, 784]");
  TORCH_CHECK(labels.numel() == images.size(0), "labels must be [N]");
  TORCH_CHECK(W.numel() == LIN_N * LIN_K && b.numel() == LIN_N, "W/b must be [10,784]/[10]");
  need_numel(metrics, 3, "metrics");
  need_aligned(images.data_ptr(), 4, "images");
  if (images.size(0) == 0) return;
  launch_lin_eval(images.data_ptr<uint8_t>(), labels.data_ptr<int32_t>(), (int)images.size(0),
                  W.data_ptr<float>(), b.data_ptr<float>(), metrics.data_ptr<double>(),
                  cur_stream(images));
}

// ------------------------------------------------------------------ optimizer
// segs: list of (offset, rows, cols, shadow or None, shadow_t or None)
void optim_step(int64_t kind, at::Tensor p, at::Tensor g, at::Tensor m, c10::optional<at::Tensor> v,
                at::Tensor lr, at::Tensor step, double beta1, double beta2, double eps, double wd,
                double momentum, double dampening, bool nesterov, double grad_scale,
                std::vector<py::tuple> segs) {
  c10::DeviceGuard dg(p.device());
  need(p, at::kFloat, "params");
  need(g, at::kFloat, "grads");
  need(m, at::kFloat, "state m");
  need(lr, at::kDouble, "lr");
  need(step, at::kLong, "step");
  TORCH_CHECK(g.numel() == p.numel() && m.numel() == p.numel(), "arena size mismatch");
  TORCH_CHECK(kind == OPT_ADAM || kind == OPT_SGD, "bad optimizer kind");
  OptArgs a{};
  a.p = p.data_ptr<float>();
  a.g = g.data_ptr<float>();
  a.m = m.data_ptr<float>();
  a.v = nullptr;
  if (kind == OPT_ADAM) {
    TORCH_CHECK(v.has_value() && v->defined(), "adam needs exp_avg_sq");
    need(*v, at::kFloat, "state v");
    TORCH_CHECK(v->numel() == p.numel(), "arena size mismatch");
    a.v = v->data_ptr<float>();
  }
  a.lr = lr.data_ptr<double>();
  a.step = step.data_ptr<int64_t>();
  a.beta1_d = beta1;
  a.beta2_d = beta2;
  a.beta1 = (float)beta1;
  a.beta2 = (float)beta2;
  a.eps = (float)eps;
  a.wd = (float)wd;
  a.momentum = (float)momentum;
  a.dampening = (float)dampening;
  a.nesterov = nesterov ? 1 : 0;
  a.grad_scale = (float)grad_scale;
  TORCH_CHECK(!segs.empty() && segs.size() <= OPT_MAX_SEG, "1..8 optimizer segments");
  a.nseg = (int)segs.size();
  for (size_t i = 0; i < segs.size(); ++i) {
    const auto& t = segs[i];
    OptSeg& s = a.seg[i];
    s.offset = t[0].cast<int64_t>();
    s.rows = (int32_t)t[1].cast<int64_t>();
    s.cols = (int32_t)t[2].cast<int64_t>();
    TORCH_CHECK(s.offset >= 0 && s.rows >= 1 && s.cols >= 1 &&
                    s.offset + (int64_t)s.rows * s.cols <= p.numel(), "segment out of range");
    TORCH_CHECK(s.offset % 4 == 0, "segment offsets must be 16-byte aligned");
    s.shadow = nullptr;
    s.shadow_t = nullptr;
    if (!t[3].is_none()) {
      auto sh = t[3].cast<at::Tensor>();
      need(sh, at::kBFloat16, "shadow");
      TORCH_CHECK(sh.numel() == (int64_t)s.rows * s.cols, "shadow size mismatch");
      need_aligned(sh.data_ptr(), 8, "shadow");
      s.shadow = ptr<__bf16>(sh);
    }
    if (!t[4].is_none()) {
      auto sh = t[4].cast<at::Tensor>();
      need(sh, at::kBFloat16, "shadow_t");
      TORCH_CHECK(sh.numel() == (int64_t)s.rows * s.cols, "shadow_t size mismatch");
      s.shadow_t = ptr<__bf16>(sh);
    }
  }
  launch_optim((int)kind, a, cur_stream(p));
}

}  // namespace

PYBIND11_MODULE(_C, m) {
  m.doc() = "MI355X (gfx950) kernels + RCCL runtime for pytorch_distributed_mnist_amd";
  m.attr("LIN_ROWS") = LIN_ROWS;
  m.attr("LIN_SLAB") = LIN_SLAB;
  m.attr("OPT_ADAM") = OPT_ADAM;
  m.attr("OPT_SGD") = OPT_SGD;
  m.def("lin_train", &lin_train);
  m.def("lin_reduce", &lin_reduce);
  m.def("lin_eval", &lin_eval);
  m.def("optim_step", &optim_step);
  register_comm(m);
}
