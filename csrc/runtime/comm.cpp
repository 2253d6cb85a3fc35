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
//
// Failure detection: the communicator is created NON-BLOCKING
// (ncclCommInitRankConfig, config.blocking = 0) and the host polls
// ncclCommGetAsyncError against a deadline (the app's --timeout), so a rank that
// never joins makes every other rank raise instead of hanging the node; the
// communicator is aborted (ncclCommAbort) on the way out.  Enqueue calls that
// report ncclInProgress are polled against the same deadline.  Device-side hangs of
// an enqueued collective are bounded at the host's sync points by
// parallel.comm.bounded_sync, which aborts the communicator (unblocking its
// kernels) once the deadline passes.
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
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

// Bring-up cancellation: a communicator init polled in settle() gives up at once when its
// cancel token is posted here (the Python side posts it from a watcher thread when another
// rank reports a failed bring-up through the rendezvous store), instead of waiting for
// peers that will never arrive until the full deadline.
static std::atomic<int64_t> g_cancelled_init{0};

void rccl_cancel_init(int64_t token) { g_cancelled_init.store(token); }

class RcclComm {
 public:
  RcclComm(const std::string& uid, int rank, int nranks, int device, double timeout_s,
           int64_t cancel_token = 0)
      : rank_(rank), nranks_(nranks), device_(device), timeout_s_(timeout_s),
        cancel_token_(cancel_token) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad unique id size ", uid.size());
    TORCH_CHECK(timeout_s > 0, "RCCL timeout must be positive");
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    HIP_OK(hipSetDevice(device));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;   // init returns at once; completion is polled against the deadline
    ncclResult_t r = ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) ncclCommAbort(comm_);
      comm_ = nullptr;
      TORCH_CHECK(false, "RCCL error ", ncclGetErrorString(r), " at ncclCommInitRankConfig (rank ",
                  rank, " of ", nranks, ")");
    }
    ncclResult_t st = settle("communicator init", /*cancellable=*/true);
    if (st != ncclSuccess) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      TORCH_CHECK(false, "RCCL communicator init failed on rank ", rank, " of ", nranks, ": ",
                  cancelled_ ? std::string("cancelled: another rank reported a failed bring-up")
                  : st == ncclInProgress ? "timed out after " + std::to_string(timeout_s) +
                                             " s waiting for the other ranks (a peer never joined "
                                             "or died during bring-up)"
                                       : std::string(ncclGetErrorString(st)));
    }
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
      // the comm stream drains within the deadline, or a collective is stuck on a peer that
      // never arrives: abort (its kernels exit on RCCL's abort flag) instead of hanging here
      if (!drain_stream()) {
        ncclCommAbort(comm_);
        comm_ = nullptr;
        release_stream();
        return;
      }
      // non-blocking communicator: finalize (flushes outstanding operations, in progress
      // until every peer has done the same) is polled against the deadline; a peer that
      // never finalizes gets the communicator aborted instead of a hang in destroy
      ncclResult_t r = ncclCommFinalize(comm_);
      if (r == ncclInProgress || r == ncclSuccess) r = settle("communicator finalize");
      if (r == ncclSuccess) {
        ncclCommDestroy(comm_);
      } else {
        ncclCommAbort(comm_);
      }
      comm_ = nullptr;
      release_stream();
    }
  }

  // Tear the communicator down without waiting for in-flight work: RCCL's abort flag
  // makes kernels that wait for a missing peer exit (used after a timeout).
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      release_stream();
    }
  }

  // Poll the communicator's async state until it leaves ncclInProgress or the deadline
  // passes; returns the final state (ncclInProgress = timed out).
  // Poll the comm stream against the deadline (hipStreamQuery, like settle()); false when it
  // is still busy at the deadline.
  bool drain_stream() {
    if (!stream_) return true;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; ++i) {
      hipError_t q = hipStreamQuery(stream_);
      if (q != hipErrorNotReady) return true;     // done (or an error: nothing left to wait on)
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s_) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(i < 100 ? 10 : 1000));
    }
  }

  ncclResult_t settle(const char* what, bool cancellable = false) {
    const auto t0 = std::chrono::steady_clock::now();
    ncclResult_t st = ncclInProgress;
    for (int i = 0;; ++i) {
      if (ncclCommGetAsyncError(comm_, &st) != ncclSuccess) return ncclInternalError;
      if (st != ncclInProgress) return st;
      if (cancellable && cancel_token_ != 0 && g_cancelled_init.load() == cancel_token_) {
        cancelled_ = true;
        return ncclInProgress;
      }
      const double el =
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s_) return ncclInProgress;
      std::this_thread::sleep_for(std::chrono::microseconds(i < 100 ? 10 : 1000));
    }
    (void)what;
  }

  // result of an enqueue call on the non-blocking communicator
  void enqueued(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) r = settle(what);
    if (r == ncclInProgress) {
      abort();
      TORCH_CHECK(false, "RCCL ", what, " timed out after ", timeout_s_, " s (rank ", rank_, " of ",
                  nranks_, "); communicator aborted");
    }
    TORCH_CHECK(r == ncclSuccess, "RCCL error ", ncclGetErrorString(r), " at ", what);
  }

  // ranks / device as the communicator itself reports them
  int comm_count() {
    alive();
    int n = 0;
    NCCL_OK(ncclCommCount(comm_, &n));
    return n;
  }
  int comm_user_rank() {
    alive();
    int r = -1;
    NCCL_OK(ncclCommUserRank(comm_, &r));
    return r;
  }
  // ncclSuccess (0) while healthy; an RCCL error code once something failed asynchronously
  int async_error() {
    if (!comm_) return (int)ncclInvalidUsage;
    ncclResult_t st = ncclSuccess;
    NCCL_OK(ncclCommGetAsyncError(comm_, &st));
    return (int)st;
  }
  double timeout_s() const { return timeout_s_; }

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
    enqueued(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), ncclSum, comm_,
                           stream_), "all-reduce");
    join(cur);
  }

  void all_reduce_range(void* ptr, size_t count, ncclDataType_t dt) {
    alive();
    enqueued(ncclAllReduce(ptr, ptr, count, dt, ncclSum, comm_, stream_), "bucket all-reduce");
  }

  // in place over [ptr, ptr + nranks * count): rank r's sum lands in its own slice
  // [ptr + r * count, ...); the other slices keep unspecified partial values
  void reduce_scatter_range(float* ptr, size_t count) {
    alive();
    enqueued(ncclReduceScatter(ptr, ptr + (size_t)rank_ * count, count, ncclFloat32, ncclSum, comm_,
                               stream_), "bucket reduce-scatter");
  }

  // in place over [ptr, ptr + nranks * count * elem): every rank's slice to every rank
  void all_gather_range(void* ptr, size_t count, ncclDataType_t dt, size_t elem) {
    alive();
    char* base = static_cast<char*>(ptr);
    enqueued(ncclAllGather(base + (size_t)rank_ * count * elem, base, count, dt, comm_, stream_),
             "shard all-gather");
  }

  void broadcast_(at::Tensor t, int root) {
    check_dev(t, device_);
    alive();
    hipStream_t cur = caller();
    fork(cur);
    enqueued(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), nccl_dtype(t), root, comm_,
                           stream_), "broadcast");
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
    enqueued(ncclAllGather(t.data_ptr(), out.data_ptr(), t.numel(), nccl_dtype(t), comm_, stream_),
             "all-gather");
    join(cur);
    return out;
  }

  void synchronize() { HIP_OK(hipStreamSynchronize(stream_)); }

  int rank() const { return rank_; }
  int size() const { return nranks_; }
  int device() const { return device_; }
  hipStream_t stream() const { return stream_; }

 private:
  void alive() const { TORCH_CHECK(comm_ != nullptr, "communicator destroyed or aborted"); }
  void release_stream() {
    if (ev_in_) hipEventDestroy(ev_in_);
    if (ev_out_) hipEventDestroy(ev_out_);
    if (stream_) hipStreamDestroy(stream_);
    ev_in_ = ev_out_ = nullptr;
    stream_ = nullptr;
  }
  int rank_, nranks_, device_;
  double timeout_s_;
  int64_t cancel_token_ = 0;
  bool cancelled_ = false;
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
    HIP_OK(hipEventCreateWithFlags(&gready_, hipEventDisableTiming));
    HIP_OK(hipEventCreateWithFlags(&gdone_, hipEventDisableTiming));
  }
  ~GradReducer() {
    for (auto& e : ready_) hipEventDestroy(e);
    for (auto& e : reduced_) hipEventDestroy(e);
    hipEventDestroy(done_);
    hipEventDestroy(gready_);
    hipEventDestroy(gdone_);
  }

  // Shard part of bucket i (ZeRO-1 style, optimizer-state sharding on one bucket): the
  // `nranks * count` floats at `start` are reduce-scattered (rank r receives the sum of
  // slice r only, which is all its optimizer update reads), the rest of the bucket is
  // all-reduced as before; both in one RCCL group.
  void set_shard(int i, int64_t start, int64_t count) {
    TORCH_CHECK(i >= 0 && i < (int)starts_.size(), "bad bucket index");
    const int64_t n = (int64_t)comm_.size() * count;
    TORCH_CHECK(count > 0 && start >= starts_[i] && start + n <= starts_[i] + counts_[i],
                "shard outside its bucket");
    shard_bucket_ = i;
    shard_start_ = start;
    shard_count_ = count;
  }
  void clear_shard() { shard_bucket_ = -1; }

  void bucket_ready(int i) {
    TORCH_CHECK(i >= 0 && i < (int)starts_.size(), "bad bucket index");
    hipStream_t cur = comm_.caller();
    HIP_OK(hipEventRecord(ready_[i], cur));
    HIP_OK(hipStreamWaitEvent(comm_.stream(), ready_[i], 0));
    if (i == shard_bucket_) {
      NCCL_OK(ncclGroupStart());
      enqueue_bucket(i);
      comm_.enqueued(ncclGroupEnd(), "grouped sharded bucket");
    } else {
      enqueue_bucket(i);
    }
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
    for (size_t i = 0; i < starts_.size(); ++i) enqueue_bucket((int)i);
    comm_.enqueued(ncclGroupEnd(), "grouped bucket all-reduce");
    for (auto& e : reduced_) HIP_OK(hipEventRecord(e, comm_.stream()));
    pending_ = true;
  }

  // in-place all-gather of `t` (rank r owns t's slice r of nranks equal slices) on the comm
  // stream, after the caller's current stream; wait_gather() joins it back
  void gather(at::Tensor t) {
    check_dev(t, comm_.device());
    const int64_t n = comm_.size();
    TORCH_CHECK(t.numel() % n == 0, "all-gather tensor must split into ", n, " equal slices");
    hipStream_t cur = comm_.caller();
    HIP_OK(hipEventRecord(gready_, cur));
    HIP_OK(hipStreamWaitEvent(comm_.stream(), gready_, 0));
    comm_.all_gather_range(t.data_ptr(), (size_t)(t.numel() / n), nccl_dtype(t), t.element_size());
    HIP_OK(hipEventRecord(gdone_, comm_.stream()));
  }
  void wait_gather() { HIP_OK(hipStreamWaitEvent(comm_.caller(), gdone_, 0)); }

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
  // the collectives of bucket i (inside the caller's group when sharded)
  void enqueue_bucket(int i) {
    float* g = grads_.data_ptr<float>();
    const int64_t s = starts_[i], e = starts_[i] + counts_[i];
    if (i != shard_bucket_) {
      comm_.all_reduce_range(g + s, (size_t)counts_[i], ncclFloat32);
      return;
    }
    const int64_t ss = shard_start_, se = shard_start_ + (int64_t)comm_.size() * shard_count_;
    if (ss > s) comm_.all_reduce_range(g + s, (size_t)(ss - s), ncclFloat32);
    comm_.reduce_scatter_range(g + ss, (size_t)shard_count_);
    if (e > se) comm_.all_reduce_range(g + se, (size_t)(e - se), ncclFloat32);
  }

  RcclComm& comm_;
  at::Tensor grads_;
  std::vector<int64_t> starts_, counts_;
  std::vector<hipEvent_t> ready_, reduced_;
  hipEvent_t done_ = nullptr, gready_ = nullptr, gdone_ = nullptr;
  bool pending_ = false;
  int shard_bucket_ = -1;
  int64_t shard_start_ = 0, shard_count_ = 0;
};

void register_comm(py::module& m) {
  m.def("rccl_unique_id", &rccl_unique_id, "ncclGetUniqueId() as 128 bytes");
  m.def("rccl_cancel_init", &rccl_cancel_init, "cancel the RCCL bring-up holding this token");
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<const std::string&, int, int, int, double, int64_t>(), py::arg("uid"),
           py::arg("rank"), py::arg("nranks"), py::arg("device"), py::arg("timeout_s") = 1800.0,
           py::arg("cancel_token") = 0, py::call_guard<py::gil_scoped_release>())
      .def("all_reduce_", &RcclComm::all_reduce_)
      .def("abort", &RcclComm::abort)
      .def("comm_count", &RcclComm::comm_count)
      .def("comm_user_rank", &RcclComm::comm_user_rank)
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("timeout_s", &RcclComm::timeout_s)
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
      .def("set_shard", &GradReducer::set_shard)
      .def("clear_shard", &GradReducer::clear_shard)
      .def("gather", &GradReducer::gather)
      .def("wait_gather", &GradReducer::wait_gather)
      .def_property_readonly("num_buckets", &GradReducer::num_buckets);
}
