// RCCL communicator owned by the framework (not by torch.distributed).
//
// The reference moves hidden states between stages over hivemind/libp2p + protobuf (SURVEY N5,
// §5.8).  On one MI355X node every GPU pair has a direct xGMI link, so stage i -> i+1 activations
// are plain RCCL point-to-point transfers.  Owning the ncclComm_t here (instead of going through
// ProcessGroupNCCL) lets the runtime put sends and receives on its own HIP streams, ordered against
// compute with HIP events, on one 2-rank communicator per neighbouring stage pair.
//
// Communicators are created NON-BLOCKING and initialisation is polled with a deadline: a peer that
// never shows up (or fails) turns into a Python exception after `timeout_s` instead of a process
// stuck forever inside ncclCommInitRank, so the pipeline can agree on a fallback transport.
// The unique id is distributed through the torch.distributed TCP store.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <rccl/rccl.h>

#include <chrono>
#include <string>
#include <thread>

namespace {

#define RCCL_CHECK(expr)                                                              \
  do {                                                                                \
    ncclResult_t _r = (expr);                                                         \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error ", ncclGetErrorString(_r), " in ", #expr); \
  } while (0)

inline hipStream_t resolve_stream(int64_t s) {
  return s ? reinterpret_cast<hipStream_t>(s) : c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

ncclDataType_t to_nccl(const at::Tensor& t) {
  switch (t.scalar_type()) {
    case at::kFloat: return ncclFloat32;
    case at::kBFloat16: return ncclBfloat16;
    case at::kHalf: return ncclFloat16;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    default: return ncclUint8;
  }
}

class RcclComm {
 public:
  // wait=false returns with the (non-blocking) init still in flight: the caller polls ready()
  // and can give up early (another rank failed, a peer never answered) with abort().
  RcclComm(const std::string& uid, int rank, int world, int device, double timeout_s, bool wait)
      : rank_(rank), world_(world), device_(device),
        enqueue_timeout_s_(timeout_s < 60.0 ? timeout_s : 60.0) {
    TORCH_CHECK(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    memcpy(&id, uid.data(), sizeof(id));
    TORCH_CHECK(hipSetDevice(device) == hipSuccess, "hipSetDevice failed");
    ncclConfig_t config = NCCL_CONFIG_INITIALIZER;
    config.blocking = 0;
    pybind11::gil_scoped_release nogil;
    const ncclResult_t r = ncclCommInitRankConfig(&comm_, world, id, rank, &config);
    if (r != ncclSuccess && r != ncclInProgress) {
      if (comm_) ncclCommAbort(comm_);
      comm_ = nullptr;
      TORCH_CHECK(false, "RCCL error ", ncclGetErrorString(r), " in ncclCommInitRankConfig");
    }
    if (wait) wait_ready(timeout_s, "ncclCommInitRankConfig");
  }
  ~RcclComm() { destroy(); }

  // true once initialised; false while the init is in flight; raises (and aborts) on an error.
  bool ready() {
    TORCH_CHECK(comm_ != nullptr, "communicator destroyed");
    ncclResult_t st = ncclInProgress;
    const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
    if (q != ncclSuccess) st = q;
    if (st == ncclInProgress) return false;
    if (st != ncclSuccess) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      TORCH_CHECK(false, "RCCL error ", ncclGetErrorString(st), " in ncclCommInitRankConfig");
    }
    return true;
  }

  void destroy() {
    if (comm_) {
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  void send(const at::Tensor& t, int peer, int64_t stream) {
    check(t);
    enq(ncclSend(t.data_ptr(), t.nbytes(), ncclUint8, peer, comm_, resolve_stream(stream)), "ncclSend");
  }
  void recv(at::Tensor& t, int peer, int64_t stream) {
    check(t);
    enq(ncclRecv(t.data_ptr(), t.nbytes(), ncclUint8, peer, comm_, resolve_stream(stream)), "ncclRecv");
  }
  void group_start() { RCCL_CHECK(ncclGroupStart()); }
  void group_end() { enq(ncclGroupEnd(), "ncclGroupEnd"); }

  void all_reduce(at::Tensor& t, int64_t stream) {
    check(t);
    enq(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t), ncclSum, comm_,
                      resolve_stream(stream)), "ncclAllReduce");
  }
  void broadcast(at::Tensor& t, int root, int64_t stream) {
    check(t);
    enq(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.nbytes(), ncclUint8, root, comm_,
                      resolve_stream(stream)), "ncclBroadcast");
  }
  void all_gather(const at::Tensor& in, at::Tensor& out, int64_t stream) {
    check(in);
    check(out);
    TORCH_CHECK(out.nbytes() == in.nbytes() * (size_t)world_, "all_gather: out size mismatch");
    enq(ncclAllGather(in.data_ptr(), out.data_ptr(), in.nbytes(), ncclUint8, comm_,
                      resolve_stream(stream)), "ncclAllGather");
  }
  int rank() const { return rank_; }
  int world() const { return world_; }

 private:
  // Poll the (non-blocking) communicator until it leaves ncclInProgress; abort it on an error or
  // when the deadline passes.
  void wait_ready(double timeout_s, const char* what) {
    const auto deadline = std::chrono::steady_clock::now() +
                          std::chrono::microseconds((int64_t)(timeout_s * 1e6));
    ncclResult_t st = ncclInProgress;
    while (true) {
      const ncclResult_t q = ncclCommGetAsyncError(comm_, &st);
      if (q != ncclSuccess) st = q;
      if (st != ncclInProgress) break;
      if (std::chrono::steady_clock::now() > deadline) {
        ncclCommAbort(comm_);
        comm_ = nullptr;
        TORCH_CHECK(false, "RCCL ", what, " timed out after ", timeout_s, " s");
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    if (st != ncclSuccess) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
      TORCH_CHECK(false, "RCCL error ", ncclGetErrorString(st), " in ", what);
    }
  }
  // A non-blocking communicator may return ncclInProgress from an enqueue call.
  void enq(ncclResult_t r, const char* what) {
    if (r == ncclInProgress) {
      wait_ready(enqueue_timeout_s_, what);
      return;
    }
    TORCH_CHECK(r == ncclSuccess, "RCCL error ", ncclGetErrorString(r), " in ", what);
  }
  void check(const at::Tensor& t) const {
    TORCH_CHECK(comm_ != nullptr, "communicator destroyed");
    TORCH_CHECK(t.is_cuda() && t.is_contiguous(), "RCCL tensors must be contiguous GPU tensors");
    TORCH_CHECK(t.get_device() == device_, "tensor on wrong device");
  }
  ncclComm_t comm_ = nullptr;
  int rank_, world_, device_;
  double enqueue_timeout_s_;
};

pybind11::bytes get_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return pybind11::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

int rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

}  // namespace

void register_rccl(pybind11::module_& m) {
  m.def("rccl_unique_id", &get_unique_id);
  m.def("rccl_version", &rccl_version);
  pybind11::class_<RcclComm>(m, "RcclComm")
      .def(pybind11::init<const std::string&, int, int, int, double, bool>(), pybind11::arg("uid"),
           pybind11::arg("rank"), pybind11::arg("world"), pybind11::arg("device"),
           pybind11::arg("timeout_s") = 120.0, pybind11::arg("wait") = true)
      .def("ready", &RcclComm::ready, pybind11::call_guard<pybind11::gil_scoped_release>())
      .def("send", &RcclComm::send, pybind11::arg("t"), pybind11::arg("peer"),
           pybind11::arg("stream") = 0)
      .def("recv", &RcclComm::recv, pybind11::arg("t"), pybind11::arg("peer"),
           pybind11::arg("stream") = 0)
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end)
      .def("all_reduce", &RcclComm::all_reduce, pybind11::arg("t"), pybind11::arg("stream") = 0)
      .def("broadcast", &RcclComm::broadcast, pybind11::arg("t"), pybind11::arg("root"),
           pybind11::arg("stream") = 0)
      .def("all_gather", &RcclComm::all_gather, pybind11::arg("inp"), pybind11::arg("out"),
           pybind11::arg("stream") = 0)
      .def("destroy", &RcclComm::destroy)
      .def("abort", &RcclComm::abort)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("world", &RcclComm::world);
}
