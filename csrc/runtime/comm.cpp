// RCCL communicator + bucketed gradient reducer (C1/C2/C3 of SURVEY.md §2.2).
//
// RcclComm   — ncclCommInitRank from a unique id exchanged through the
//              rendezvous store (Python side), one dedicated non-blocking HIP
//              stream for communication, in-place all-reduce / broadcast /
//              all-gather that are ordered after the caller's current stream by
//              an event and make the caller's stream wait for completion.
// GradReducer — the DDP Reducer replacement: the flat gradient arena is cut into
//              contiguous buckets; bucket_ready(i) forks bucket i's ncclAllReduce
//              onto the comm stream behind an event recorded after the kernel
//              that produced it (so it overlaps the remaining backward kernels),
//              finalize() joins the comm stream back before the optimizer.
// Both only use stream/event primitives that hipStreamBeginCapture supports,
// so a whole step (kernels + collectives) is captured into one hipGraph.
//
// RCCL resolution: the extension links torch's bundled librccl.so (SONAME
// librccl.so.1), so the process has exactly one RCCL — the one torch loaded.
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include <string>
#include <vector>

namespace py = pybind11;

#define HIP_OK(x)                                                                         \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", #x);       \
  } while (0)
#define NCCL_OK(x)                                                                        \
  do {                                                                                    \
    ncclResult_t _r = (x);                                                                \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error ", ncclGetErrorString(_r), " at ", #x);    \
  } while (0)

static ncclDataType_t nccl_dtype(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kDouble: return ncclFloat64;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    default: TORCH_CHECK(false, "unsupported dtype for RCCL: ", t.scalar_type());
  }
}

static void check_dev(const at::Tensor& t, int device) {
  TORCH_CHECK(t.is_cuda(), "RCCL tensors must live on the HIP device");
  TORCH_CHECK(t.get_device() == device, "tensor on device ", t.get_device(),
              " but communicator is on ", device);
  TORCH_CHECK(t.is_contiguous(), "RCCL tensors must be contiguous");
}

py::bytes rccl_unique_id() {
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

class RcclComm {
 public:
  RcclComm(const std::string& uid, int rank, int nranks, int device)
      : rank_(rank), nranks_(nranks), device_(device) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad unique id size ", uid.size());
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    HIP_OK(hipSetDevice(device));
    NCCL_OK(ncclCommInitRank(&comm_, nranks, id, rank));
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    // highest priority: collectives should not queue behind compute kernels
    HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
    HIP_OK(hipEventCreateWithFlags(&ev_in_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&ev_out_, hipEventDisableTiming));
  }
  ~RcclComm() { destroy(); }

  void destroy() {
    if (comm_) {
      hipStreamSynchronize(stream_);
      ncclCommDestroy(comm_);
      comm_ = nullptr;
      hipEventDestroy(ev_in_);
      hipEventDestroy(ev_out_);
      hipStreamDestroy(stream_);
    }
  }

  hipStream_t caller() const { return c10::hip::getCurrentHIPStream(device_).stream(); }

  // caller stream -> comm stream
  void fork(hipStream_t cur) {
    HIP_OK(hipEventRecord(ev_in_, cur));
    HIP_OK(hipStreamWaitEvent(stream_, ev_in_, 0));
  }
  // comm stream -> caller stream
  void join(hipStream_t cur) {
    HIP_OK(hipEventRecord(ev_out_, stream_));
    HIP_OK(hipStreamWaitEvent(cur, ev_out_, 0));
  }

  void all_reduce_(at::Tensor t) {
    check_dev(t, device_);
    alive();
    hipStream_t cur = caller();
    fork(cur);
    NCCL_OK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), ncclSum, comm_,
                          stream_));
    join(cur);
  }

  void all_reduce_range(void* ptr, size_t count, ncclDataType_t dt) {
    NCCL_OK(ncclAllReduce(ptr, ptr, count, dt, ncclSum, comm_, stream_));
  }

  void broadcast_(at::Tensor t, int root) {
    check_dev(t, device_);
    alive();
    hipStream_t cur = caller();
    fork(cur);
    NCCL_OK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_,
                          stream_));
    join(cur);
  }

  at::Tensor all_gather(at::Tensor t) {
    check_dev(t, device_);
    alive();
    auto sizes = t.sizes().vec();
    sizes.insert(sizes.begin(), nranks_);
    at::Tensor out = at::empty(sizes, t.options());
    hipStream_t cur = caller();
    fork(cur);
    NCCL_OK(ncclAllGather(t.data_ptr(), out.data_ptr(), t.numel(), nccl_dtype(t), comm_, stream_));
    join(cur);
    return out;
  }

  void synchronize() { HIP_OK(hipStreamSynchronize(stream_)); }

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }

 private:
  void alive() const { TORCH_CHECK(comm_ != nullptr, "communicator destroyed"); }
  int rank_, nranks_, device_;
  ncclComm_t comm_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_in_ = nullptr, ev_out_ = nullptr;
};

class GradReducer {
 public:
  GradReducer(RcclComm& comm, at::Tensor grads, std::vector<int64_t> bounds)
      : comm_(comm), grads_(grads) {
    check_dev(grads, comm.device());
    TORCH_CHECK(grads.scalar_type() == at::kFloat, "gradient arena must be fp32");
    TORCH_CHECK(bounds.size() % 2 == 0 && !bounds.empty(), "bounds must be (start,end) pairs");
    for (size_t i = 0; i < bounds.size(); i += 2) {
      TORCH_CHECK(0 <= bounds[i] && bounds[i] < bounds[i + 1] && bounds[i + 1] <= grads.numel(),
                  "bucket out of range");
      starts_.push_back(bounds[i]);
      counts_.push_back(bounds[i + 1] - bounds[i]);
    }
    ready_.resize(starts_.size());
    for (auto& e : ready_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    reduced_.resize(starts_.size());
    for (auto& e : reduced_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  ~GradReducer() {
    for (auto& e : ready_) hipEventDestroy(e);
    for (auto& e : reduced_) hipEventDestroy(e);
    hipEventDestroy(done_);
  }

  void bucket_ready(int i) {
    TORCH_CHECK(i >= 0 && i < (int)starts_.size(), "bad bucket index");
    hipStream_t cur = comm_.caller();
    HIP_OK(hipEventRecord(ready_[i], cur));
    HIP_OK(hipStreamWaitEvent(comm_.stream(), ready_[i], 0));
    float* base = grads_.data_ptr<float>() + starts_[i];
    comm_.all_reduce_range(base, (size_t)counts_[i], ncclFloat32);
    HIP_OK(hipEventRecord(reduced_[i], comm_.stream()));
    pending_ = true;
  }

  // every bucket in one RCCL group (a single collective launch), ordered after the
  // caller's current stream
  void all_ready() {
    hipStream_t cur = comm_.caller();
    HIP_OK(hipEventRecord(ready_[0], cur));
    HIP_OK(hipStreamWaitEvent(comm_.stream(), ready_[0], 0));
    NCCL_OK(ncclGroupStart());
    for (size_t i = 0; i < starts_.size(); ++i)
      comm_.all_reduce_range(grads_.data_ptr<float>() + starts_[i], (size_t)counts_[i], ncclFloat32);
    NCCL_OK(ncclGroupEnd());
    for (auto& e : reduced_) HIP_OK(hipEventRecord(e, comm_.stream()));
    pending_ = true;
  }

  // make the caller's current stream wait for bucket i's all-reduce only (e.g. a side
  // stream running that bucket's optimizer while later backward kernels still run)
  void wait_bucket(int i) {
    TORCH_CHECK(i >= 0 && i < (int)starts_.size(), "bad bucket index");
    HIP_OK(hipStreamWaitEvent(comm_.caller(), reduced_[i], 0));
  }

  void finalize() {
    if (!pending_) return;
    hipStream_t cur = comm_.caller();
    HIP_OK(hipEventRecord(done_, comm_.stream()));
    HIP_OK(hipStreamWaitEvent(cur, done_, 0));
    pending_ = false;
  }

  int num_buckets() const { return (int)starts_.size(); }

 private:
  RcclComm& comm_;
  at::Tensor grads_;
  std::vector<int64_t> starts_, counts_;
  std::vector<hipEvent_t> ready_, reduced_;
  hipEvent_t done_ = nullptr;
  bool pending_ = false;
};

void register_comm(py::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId() as 128 bytes");
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int>(), py::arg("uid"), py::arg("rank"),
           py::arg("nranks"), py::arg("device"))
      .def("all_reduce_", &RcclComm::all_reduce_)
      .def("broadcast_", &RcclComm::broadcast_)
      .def("all_gather", &RcclComm::all_gather)
      .def("synchronize", &RcclComm::synchronize)
      .def("destroy", &RcclComm::destroy)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def_property_readonly("device", &RcclComm::device);
  py::class_<GradReducer>(m, "GradReducer")
      .def(py::init<RcclComm&, at::Tensor, std::vector<int64_t>>(), py::keep_alive<1, 2>())
      .def("bucket_ready", &GradReducer::bucket_ready)
      .def("finalize", &GradReducer::finalize)
      .def("wait_bucket", &GradReducer::wait_bucket)
      .def("all_ready", &GradReducer::all_ready)
      .def_property_readonly("num_buckets", &GradReducer::num_buckets);
}
