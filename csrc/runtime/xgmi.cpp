// Host side of the direct xGMI gradient all-reduce (kernel + protocol: csrc/xgmi.h,
// csrc/kernels/xgmi.hip).  Replaces the RCCL data plane for the gradient buckets;
// the RCCL communicator stays for the parameter broadcast and as the fallback.
//
// XgmiReducer — one rank's end:
//   * one uncached device allocation (flags | result arena | per-bucket stage),
//     exported with hipIpcGetMemHandle; the peers' allocations are mapped with
//     hipIpcOpenMemHandle (dmabuf), so a kernel addresses every rank's buffers;
//   * one channel per gradient bucket: one-shot (whole bucket to every peer) for
//     small buckets or two ranks, two-shot (reduce-scatter + all-gather push) for
//     the 4.7 MB fc bucket at 4 and 8 ranks;
//   * the GradReducer stream protocol (bucket_ready / all_ready / wait_bucket /
//     finalize): each bucket's kernel runs on a high-priority stream behind an
//     event recorded on the caller's stream, so the whole exchange is captured in
//     the step's hipGraph and overlaps whatever the compute stream runs next.
#include <c10/hip/HIPStream.h>
#include <torch/extension.h>

#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "xgmi.h"

namespace py = pybind11;

#define XG_HIP_OK(x)                                                                      \
  do {                                                                                    \
    hipError_t _e = (x);                                                                  \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ", #x);       \
  } while (0)

namespace {

constexpr size_t kAlign = 1 << 16;
constexpr int64_t kOneShotMaxBytes = 256 << 10;   // buckets up to this size go one-shot

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Process-wide registry of exported heaps and opened peer mappings.  A heap is
// exported once and reused by later reducers of the process (re-zeroed), and a
// peer's handle is opened once: freeing an exported allocation and allocating a
// new one let hipIpcGetMemHandle fail with "invalid argument" on ROCm 7.0, and a
// re-opened handle of a recycled address could map the old pages.
struct Heap {
  void* ptr = nullptr;
  size_t bytes = 0;
  bool in_use = false;
  bool exported = false;
  hipIpcMemHandle_t handle;
};
std::mutex g_mu;
std::map<int, std::vector<Heap*>> g_heaps;          // device -> heaps (never freed)
std::map<std::string, void*> g_peer_maps;            // handle bytes -> local mapping

Heap* acquire_heap(int device, size_t bytes) {
  std::lock_guard<std::mutex> lk(g_mu);
  for (Heap* h : g_heaps[device])
    if (!h->in_use && h->bytes >= bytes) {
      h->in_use = true;
      return h;
    }
  Heap* h = new Heap();
  XG_HIP_OK(hipExtMallocWithFlags(&h->ptr, bytes, hipDeviceMallocUncached));
  h->bytes = bytes;
  h->in_use = true;
  g_heaps[device].push_back(h);
  return h;
}

void* open_peer(const std::string& key) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_peer_maps.find(key);
  if (it != g_peer_maps.end()) return it->second;
  hipIpcMemHandle_t h;
  memcpy(&h, key.data(), sizeof(h));
  void* p = nullptr;
  XG_HIP_OK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  g_peer_maps[key] = p;
  return p;
}

struct Channel {
  int64_t start, n, chunk;
  int mode, nblk;
  size_t stage_off;   // byte offset of this channel's stage area in the heap
};

}  // namespace

class XgmiReducer {
 public:
  XgmiReducer(int rank, int nranks, int device, at::Tensor grads, std::vector<int64_t> bounds,
              double timeout_s, std::string mode)
      : rank_(rank), nranks_(nranks), device_(device), grads_(grads) {
    TORCH_CHECK(nranks >= 1 && nranks <= XG_MAX_RANKS, "xgmi all-reduce supports 1..",
                XG_MAX_RANKS, " ranks, got ", nranks);
    TORCH_CHECK(rank >= 0 && rank < nranks, "bad rank");
    TORCH_CHECK(grads.is_cuda() && grads.get_device() == device, "grads must live on device ", device);
    TORCH_CHECK(grads.scalar_type() == at::kFloat && grads.is_contiguous(), "grads must be contiguous fp32");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(grads.data_ptr()) % 256 == 0, "grads must be 256-B aligned");
    TORCH_CHECK(bounds.size() % 2 == 0 && !bounds.empty() && bounds.size() / 2 <= XG_MAX_CH,
                "1..", XG_MAX_CH, " buckets as (start, end) pairs");
    TORCH_CHECK(mode == "auto" || mode == "one" || mode == "two", "mode must be auto|one|two");
    arena_ = grads.numel();
    // heap layout: flags | result arena | stage of channel 0 | stage of channel 1 | ...
    size_t off = round_up((size_t)XG_FLAG_WORDS_ALL * 4, kAlign);
    result_off_ = off;
    off += round_up((size_t)arena_ * 4, kAlign);
    for (size_t i = 0; i < bounds.size(); i += 2) {
      Channel c;
      c.start = bounds[i];
      c.n = bounds[i + 1] - bounds[i];
      TORCH_CHECK(c.start >= 0 && c.n > 0 && bounds[i + 1] <= arena_, "bucket out of range");
      TORCH_CHECK(c.start % 64 == 0 && c.n % 64 == 0, "buckets must be 64-float aligned");
      bool two = nranks > 2 && c.n * 4 > kOneShotMaxBytes;
      if (mode == "one") two = false;
      if (mode == "two") two = nranks > 1;
      c.mode = two ? XG_TWO_SHOT : XG_ONE_SHOT;
      c.chunk = two ? (int64_t)round_up((size_t)((c.n + nranks - 1) / nranks), 64) : c.n;
      const int64_t c4 = c.chunk / 4;
      // the same workgroup split serves the per-call kernel and the persistent one
      c.nblk = (int)std::min<int64_t>(XG_STREAM_WG, std::max<int64_t>(1, (c4 + XG_THREADS - 1) / XG_THREADS));
      c.stage_off = off;
      const size_t stage_floats = two ? (size_t)nranks * c.chunk : 2 * (size_t)nranks * c.n;
      TORCH_CHECK(stage_floats * 4 < (size_t)0x7fffffff, "stage area exceeds the 2 GB buffer window");
      off += round_up(stage_floats * 4, kAlign);
      ch_.push_back(c);
    }
    heap_bytes_ = off;
    timeout_ticks_ = (long long)(timeout_s * 1e8);   // s_memrealtime runs at 100 MHz
    XG_HIP_OK(hipSetDevice(device));
    heap_rec_ = acquire_heap(device, heap_bytes_);
    heap_ = heap_rec_->ptr;
    // zeroed before this rank publishes its handle, so no peer can signal into stale flags
    XG_HIP_OK(hipMemset(heap_, 0, heap_bytes_));
    XG_HIP_OK(hipMalloc(&local_, XG_LOC_WORDS * sizeof(unsigned)));
    XG_HIP_OK(hipMemset(local_, 0, XG_LOC_WORDS * sizeof(unsigned)));
    XG_HIP_OK(hipDeviceSynchronize());
    for (int r = 0; r < XG_MAX_RANKS; ++r) peers_[r] = nullptr;
    peers_[rank] = heap_;
    int lo = 0, hi = 0;
    XG_HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    XG_HIP_OK(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, hi));
    ready_.resize(ch_.size());
    reduced_.resize(ch_.size());
    for (auto& e : ready_) XG_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : reduced_) XG_HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    XG_HIP_OK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }

  ~XgmiReducer() { close(); }

  py::bytes ipc_handle() const {
    alive();
    {
      std::lock_guard<std::mutex> lk(g_mu);
      if (!heap_rec_->exported) {
        XG_HIP_OK(hipIpcGetMemHandle(&heap_rec_->handle, heap_));
        heap_rec_->exported = true;
      }
    }
    return py::bytes(reinterpret_cast<const char*>(&heap_rec_->handle), sizeof(hipIpcMemHandle_t));
  }

  // handles[r] = rank r's ipc_handle() (own entry ignored)
  void open_peers(std::vector<std::string> handles) {
    alive();
    TORCH_CHECK((int)handles.size() == nranks_, "need one handle per rank");
    XG_HIP_OK(hipSetDevice(device_));
    for (int r = 0; r < nranks_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "bad ipc handle size");
      peers_[r] = open_peer(handles[r]);
    }
    open_ = true;
  }

  at::Tensor result() const {
    alive();
    auto opts = at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, device_);
    return torch::from_blob(static_cast<char*>(heap_) + result_off_, {arena_}, [](void*) {}, opts);
  }

  void bucket_ready(int i) {
    check_bucket(i);
    hipStream_t cur = caller();
    XG_HIP_OK(hipEventRecord(ready_[i], cur));
    XG_HIP_OK(hipStreamWaitEvent(stream_, ready_[i], 0));
    launch(i);
    XG_HIP_OK(hipEventRecord(reduced_[i], stream_));
    pending_ = true;
  }

  void all_ready() {
    TORCH_CHECK(open_ || nranks_ == 1, "open_peers() first");
    hipStream_t cur = caller();
    XG_HIP_OK(hipEventRecord(ready_[0], cur));
    XG_HIP_OK(hipStreamWaitEvent(stream_, ready_[0], 0));
    for (size_t i = 0; i < ch_.size(); ++i) {
      launch((int)i);
      XG_HIP_OK(hipEventRecord(reduced_[i], stream_));
    }
    pending_ = true;
  }

  void wait_bucket(int i) {
    check_bucket(i);
    XG_HIP_OK(hipStreamWaitEvent(caller(), reduced_[i], 0));
  }

  // streamed mode: one persistent collective launch covering the next `nsteps` steps
  // (fork: ordered after the caller's stream); the step kernels hand buckets over
  // through the sync words, end() joins the caller's stream back
  // nch: how many leading buckets the persistent launch carries (-1: all); the others are
  // all-reduced in-launch by the kernels that produce them (fill_exchange)
  void begin(int nsteps, int nch = -1, bool wide = false) {
    TORCH_CHECK(open_ || nranks_ == 1, "open_peers() first");
    TORCH_CHECK(nsteps >= 1, "nsteps must be >= 1");
    TORCH_CHECK(nch == -1 || (nch >= 1 && nch <= (int)ch_.size()), "bad channel count");
    hipStream_t cur = caller();
    XG_HIP_OK(hipEventRecord(ready_[0], cur));
    XG_HIP_OK(hipStreamWaitEvent(stream_, ready_[0], 0));
    XgmiStreamArgs sa{};
    for (size_t i = 0; i < ch_.size(); ++i) fill_args((int)i, sa.ch[i]);
    sa.loc = static_cast<unsigned*>(local_);
    sa.nch = nch < 0 ? (int)ch_.size() : nch;
    sa.nsteps = nsteps;
    launch_xgmi_stream(sa, stream_, wide);
    XG_HIP_OK(hipGetLastError());
    pending_ = true;
  }

  void end() { finalize(); }

  // how many leading channels the conv backward publishes (those of the first bucket)
  void set_backward_channels(int n) {
    alive();
    TORCH_CHECK(n >= 1 && n <= (int)ch_.size(), "backward channels: 1..", ch_.size());
    npub_ = (unsigned)n;
    XG_HIP_OK(hipSetDevice(device_));
    XG_HIP_OK(hipMemcpy(static_cast<unsigned*>(local_) + XG_LOC_NPUB, &npub_, sizeof(npub_),
                        hipMemcpyHostToDevice));
  }

  // Every protocol word back to its state after construction: this rank's heap (flags,
  // stage rows, result arena) and local words (step / ready / done counters, call
  // generations, error words).  The counters of a step structure that carried other
  // channels in the persistent launch (with or without the in-launch exchange), or that
  // stopped at a device deadline, no longer match what the next structure's kernels expect.
  // Collective in effect: every rank resets between the same two control-plane agreements
  // with every device drained, so no peer kernel writes into the zeroed heap and every
  // rank's counters restart together (bench.py / parallel/startup.py candidate setup).
  void reset() {
    alive();
    XG_HIP_OK(hipSetDevice(device_));
    XG_HIP_OK(hipStreamSynchronize(stream_));
    XG_HIP_OK(hipDeviceSynchronize());
    XG_HIP_OK(hipMemset(heap_, 0, heap_bytes_));
    XG_HIP_OK(hipMemset(local_, 0, XG_LOC_WORDS * sizeof(unsigned)));
    XG_HIP_OK(hipMemcpy(static_cast<unsigned*>(local_) + XG_LOC_NPUB, &npub_, sizeof(npub_),
                        hipMemcpyHostToDevice));
    XG_HIP_OK(hipDeviceSynchronize());
    pending_ = false;
  }

  at::Tensor sync() const {
    alive();
    auto opts = at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device_);
    return torch::from_blob(local_, {XG_LOC_WORDS}, [](void*) {}, opts);
  }

  int blocks(int i) const {
    TORCH_CHECK(i >= 0 && i < (int)ch_.size(), "bad bucket index");
    return ch_[i].nblk;
  }

  void finalize() {
    if (!pending_) return;
    XG_HIP_OK(hipEventRecord(done_, stream_));
    XG_HIP_OK(hipStreamWaitEvent(caller(), done_, 0));
    pending_ = false;
  }

  // error word (XG_ERR_* in xgmi.h): every cause any wait gave up for, including
  // XG_ERR_FAILFAST for waits that only saw an earlier error
  int64_t error() { return read_err_words().first; }

  // the cause bit of the first wait that gave up at its deadline (0: none)
  int64_t first_error() { return read_err_words().second; }


  // peers whose buffers this rank has mapped through hipIpc (own rank excluded)
  int peers_mapped() const {
    int n = 0;
    for (int r = 0; r < nranks_; ++r) n += (r != rank_ && peers_[r] != nullptr);
    return n;
  }

  py::list describe() const {
    py::list out;
    for (const auto& c : ch_) {
      py::dict d;
      d["start"] = c.start;
      d["n"] = c.n;
      d["mode"] = c.mode == XG_TWO_SHOT ? "two-shot" : "one-shot";
      d["chunk"] = c.chunk;
      d["blocks"] = c.nblk;
      out.append(d);
    }
    return out;
  }

  void close() {
    if (!heap_) return;
    hipStreamSynchronize(stream_);
    // peer mappings and the exported heap stay cached for the next reducer (see Heap)
    for (auto& e : ready_) hipEventDestroy(e);
    for (auto& e : reduced_) hipEventDestroy(e);
    hipEventDestroy(done_);
    hipStreamDestroy(stream_);
    hipFree(local_);
    {
      std::lock_guard<std::mutex> lk(g_mu);
      heap_rec_->in_use = false;
    }
    heap_ = nullptr;
    open_ = false;
  }

  int num_buckets() const { return (int)ch_.size(); }

  // the in-launch exchange of bucket i (XgmiExch, xgmi.h): its one-shot stage rows on every
  // rank, the exchange flag slots and this rank's per-slot counters
  void fill_exchange(int i, XgmiExch& x) const {
    check_bucket(i);
    const Channel& c = ch_[i];
    TORCH_CHECK(c.mode == XG_ONE_SHOT, "the in-launch exchange needs a one-shot bucket");
    for (int r = 0; r < XG_MAX_RANKS; ++r) {
      char* base = static_cast<char*>(r < nranks_ ? peers_[r] : nullptr);
      x.stage[r] = base ? reinterpret_cast<float*>(base + c.stage_off) : nullptr;
      x.flags[r] = base ? reinterpret_cast<unsigned*>(base) : nullptr;
    }
    x.gen = static_cast<unsigned*>(local_) + XG_LOC_XGEN;
    x.err = err_ptr();
    x.off = c.start;
    x.n = c.n;
    x.timeout = timeout_ticks_;
    x.rank = rank_;
    x.nranks = nranks_;
  }

 private:
  void alive() const { TORCH_CHECK(heap_ != nullptr, "xgmi reducer closed"); }
  void check_bucket(int i) const {
    alive();
    TORCH_CHECK(i >= 0 && i < (int)ch_.size(), "bad bucket index");
    TORCH_CHECK(open_ || nranks_ == 1, "open_peers() first");
  }
  hipStream_t caller() const { return c10::hip::getCurrentHIPStream(device_).stream(); }
  unsigned* err_ptr() const { return static_cast<unsigned*>(local_) + XG_LOC_ERR; }

  std::pair<unsigned, unsigned> read_err_words() {
    alive();
    XG_HIP_OK(hipStreamSynchronize(stream_));
    unsigned w[XG_LOC_FIRST - XG_LOC_ERR + 1] = {};
    XG_HIP_OK(hipMemcpy(w, err_ptr(), sizeof(w), hipMemcpyDeviceToHost));
    return {w[0], w[XG_LOC_FIRST - XG_LOC_ERR]};
  }

  void launch(int i) {
    XgmiArgs a{};
    fill_args(i, a);
    launch_xgmi_allreduce(a, ch_[i].nblk, stream_);
    XG_HIP_OK(hipGetLastError());
  }

  void fill_args(int i, XgmiArgs& a) const {
    const Channel& c = ch_[i];
    for (int r = 0; r < XG_MAX_RANKS; ++r) {
      char* base = static_cast<char*>(r < nranks_ ? peers_[r] : nullptr);
      a.stage[r] = base ? reinterpret_cast<float*>(base + c.stage_off) : nullptr;
      a.result[r] = base ? reinterpret_cast<float*>(base + result_off_) : nullptr;
      a.flags[r] = base ? reinterpret_cast<unsigned*>(base) : nullptr;
    }
    a.src = grads_.data_ptr<float>() + c.start;
    a.gen = static_cast<unsigned*>(local_) + XG_LOC_GEN + i * XG_MAX_WG;
    a.err = err_ptr();
    a.off = c.start;
    a.n = c.n;
    a.chunk = c.chunk;
    a.timeout = timeout_ticks_;
    a.rank = rank_;
    a.nranks = nranks_;
    a.ch = i;
    a.mode = c.mode;
    a.nblk = c.nblk;
  }

  int rank_, nranks_, device_;
  at::Tensor grads_;
  int64_t arena_ = 0;
  size_t result_off_ = 0, heap_bytes_ = 0;
  long long timeout_ticks_ = 0;
  unsigned npub_ = 0;
  std::vector<Channel> ch_;
  Heap* heap_rec_ = nullptr;
  void* heap_ = nullptr;
  void* local_ = nullptr;
  void* peers_[XG_MAX_RANKS];
  bool open_ = false, pending_ = false;
  hipStream_t stream_ = nullptr;
  std::vector<hipEvent_t> ready_, reduced_;
  hipEvent_t done_ = nullptr;
};

// bind.cpp's optimizer entry fills the in-launch exchange from a Python-held reducer
void xgmi_fill_exchange(py::handle reducer, int bucket, XgmiExch& x) {
  reducer.cast<const XgmiReducer&>().fill_exchange(bucket, x);
}

void register_xgmi(py::module& m) {
  m.attr("XG_MAX_RANKS") = XG_MAX_RANKS;
  py::class_<XgmiReducer>(m, "XgmiReducer")
      .def(py::init<int, int, int, at::Tensor, std::vector<int64_t>, double, std::string>(),
           py::arg("rank"), py::arg("nranks"), py::arg("device"), py::arg("grads"),
           py::arg("bounds"), py::arg("timeout_s") = 60.0, py::arg("mode") = "auto")
      .def("ipc_handle", &XgmiReducer::ipc_handle)
      .def("open_peers", &XgmiReducer::open_peers)
      .def("result", &XgmiReducer::result)
      .def("bucket_ready", &XgmiReducer::bucket_ready)
      .def("all_ready", &XgmiReducer::all_ready)
      .def("wait_bucket", &XgmiReducer::wait_bucket)
      .def("finalize", &XgmiReducer::finalize)
      .def("begin", &XgmiReducer::begin, py::arg("nsteps"), py::arg("nch") = -1,
           py::arg("wide") = false)
      .def("end", &XgmiReducer::end)
      .def("sync", &XgmiReducer::sync)
      .def("set_backward_channels", &XgmiReducer::set_backward_channels)
      .def("reset", &XgmiReducer::reset)
      .def("blocks", &XgmiReducer::blocks)
      .def("error", &XgmiReducer::error)
      .def("first_error", &XgmiReducer::first_error)
      .def("describe", &XgmiReducer::describe)
      .def("peers_mapped", &XgmiReducer::peers_mapped)
      .def("close", &XgmiReducer::close)
      .def_property_readonly("num_buckets", &XgmiReducer::num_buckets);
}
