// Streams with a hardware queue of their own, device-side signal / wait primitives and
// cross-process device memory (IPC) for the pipeline transports.
//
// Why this exists (round-2 verdict, "hardware-queue hazard"): a pipeline rank keeps kernels that
// WAIT on other ranks (RCCL send/recv, the rotating head's receive) on side streams next to its
// compute.  HIP multiplexes streams onto a small pool of HSA hardware queues per priority
// (GPU_MAX_HW_QUEUES, 4 by default); AQL packets of one queue run in order, so a waiting kernel or
// a cross-stream barrier packet that lands on the compute stream's queue stalls compute until the
// peer arrives.  Streams created with a CU mask are given a queue of their own (never shared); with
// the full mask they run on every CU like an ordinary stream.  ``tests/test_streams_gpu.py`` checks
// the isolation on the hardware by spinning a kernel on each stream in turn and requiring every
// other stream to make progress.
//
// The signal / wait kernels are the device half of the IPC transport (parallel/ipc_transport.py),
// used where RCCL cannot run (several ranks on one GPU) and as the spin kernel of the isolation
// test.  Every wait has a deadline: a peer that never arrives turns into a status word the host
// reads (and a Python error), never a wave that spins forever.
#include <torch/extension.h>
#include <pybind11/stl.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

namespace {

#define HIP_OK(expr)                                                                   \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    TORCH_CHECK(_e == hipSuccess, #expr, " failed: ", hipGetErrorString(_e));          \
  } while (0)

inline hipStream_t as_stream(int64_t s) {
  return s ? reinterpret_cast<hipStream_t>(s)
           : c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream();
}

// ------------------------------------------------------------------------------------ streams
// mode 0: ordinary non-blocking stream (shares the per-priority hardware-queue pool)
// mode 1: full-CU-mask stream -> a hardware queue of its own
int64_t stream_create(int device, int mode, int priority) {
  int prev = 0;
  HIP_OK(hipGetDevice(&prev));
  HIP_OK(hipSetDevice(device));
  hipStream_t s = nullptr;
  if (mode == 1) {
    hipDeviceProp_t p;
    HIP_OK(hipGetDeviceProperties(&p, device));
    const int ncu = p.multiProcessorCount;
    std::vector<uint32_t> mask((ncu + 31) / 32, 0xffffffffu);
    if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1u;
    HIP_OK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  } else {
    HIP_OK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority));
  }
  HIP_OK(hipSetDevice(prev));
  return reinterpret_cast<int64_t>(s);
}

void stream_destroy(int64_t s) {
  if (s) HIP_OK(hipStreamDestroy(reinterpret_cast<hipStream_t>(s)));
}

int64_t stream_cu_count(int64_t s) {
  std::vector<uint32_t> mask(16, 0);
  HIP_OK(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(s), (uint32_t)mask.size(), mask.data()));
  int64_t n = 0;
  for (uint32_t m : mask) n += __builtin_popcount(m);
  return n;
}

double wall_clock_hz(int device) {
  int khz = 0;
  HIP_OK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  return khz * 1e3;
}

// ---------------------------------------------------------------------------------- kernels
// One lane polls; the other lanes of the (single, 64-wide) wave only keep the launch shape legal.
// ``status`` (host-mapped) receives ``code`` if the deadline passes; the wave always exits.
// ``abort`` (host-mapped, optional): a nonzero word ends the wait at once (the job is leaving);
// ``progress`` (host-mapped, optional, 2 words): [0] receives ``target`` when the wave starts
// waiting, [1] once the wait is satisfied - the host tells which wait of a stuck pipeline its
// stream reached and never passed (or never reached) without touching the GPU.
__global__ void __launch_bounds__(64) wait_geq_kernel(const uint32_t* flag, uint32_t target,
                                                      uint64_t max_ticks, uint32_t* status,
                                                      uint32_t code, const uint32_t* abort,
                                                      uint32_t* progress) {
  if (threadIdx.x != 0) return;
  if (progress) __hip_atomic_store(progress, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < target) {
    const bool aborted =
        abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u;
    if (aborted || (uint64_t)(wall_clock64() - t0) > max_ticks) {
      if (status) __hip_atomic_store(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return;
    }
    __builtin_amdgcn_s_sleep(8);
  }
  if (progress) __hip_atomic_store(progress + 1, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Release-store ``value`` (every write queued before this kernel on its stream has completed:
// stream order + the system-scope release make the data visible before the flag); ``progress``
// (host-mapped, optional) records the value for the host.  ``status`` / ``abort`` (host-mapped,
// optional): when either is nonzero - a wait of this process expired, or the job is leaving -
// nothing is released, so a failed wait never lets garbage flow on to the peer and every
// progress word stays where the failure froze it.
__global__ void __launch_bounds__(64) signal_kernel(uint32_t* flag, uint32_t value,
                                                    uint32_t* progress, const uint32_t* status,
                                                    const uint32_t* abort) {
  if (threadIdx.x == 0) {
    if (status && __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    if (abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
    __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (progress) __hip_atomic_store(progress, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Stream-ordered device copy as a KERNEL on the caller's stream.  hipMemcpyAsync may be carried
// out on a copy queue that the process's streams share (see copy_segments below): a copy that
// must wait for a spinning credit wait on one stream would then block, in that shared in-order
// queue, the copy another stream needs to release its peer.  A copy kernel stays on its own
// stream's hardware queue.
__global__ void __launch_bounds__(256) dev_copy_kernel(uint4* __restrict__ dst,
                                                       const uint4* __restrict__ src, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// Up to kMaxSegs (offset, bytes) segments copied src_base + off -> dst_base + off in ONE launch on
// the caller's stream: the per-step host -> device metadata uploads (the source is coherent,
// device-mapped host memory, read directly by the kernel) and the device -> host token returns.
// Measured on MI355X (scripts/queue_probe.py --copies-only, profiles/streams/): a host <-> device
// hipMemcpyAsync is carried out on a copy queue shared by the process's streams - with SDMA (the
// default) by an engine queue, with HSA_ENABLE_SDMA=0 by a blit queue - so a copy that a stream
// orders behind a spinning receive (the rotating head's staging uploads) holds up every other
// stream's copies, the compute stream's step uploads included.  Kernels run on their own stream.
constexpr int kMaxSegs = 24;
struct Segs {
  long long off[kMaxSegs];
  long long n[kMaxSegs];
  int count;
};

__global__ void __launch_bounds__(256) copy_segments_kernel(char* dst, const char* src, Segs segs) {
  const int sg = blockIdx.y;
  if (sg >= segs.count) return;
  const long long off = segs.off[sg], n = segs.n[sg];
  char* d = dst + off;
  const char* s = src + off;
  const long long tid = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  const long long nth = (long long)gridDim.x * blockDim.x;
  if ((((unsigned long long)d | (unsigned long long)s) & 15ull) == 0) {
    const long long n16 = n >> 4;
    for (long long i = tid; i < n16; i += nth)
      reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
    for (long long i = (n16 << 4) + tid; i < n; i += nth) d[i] = s[i];
  } else {
    for (long long i = tid; i < n; i += nth) d[i] = s[i];
  }
}

// A trivial kernel for progress probes: out[0] += 1.
__global__ void __launch_bounds__(64) touch_kernel(uint32_t* out) {
  if (threadIdx.x == 0) out[0] += 1u;
}

void wait_geq(int64_t flag_ptr, int64_t target, double timeout_s, int64_t status_ptr, int64_t code,
              int64_t stream, int device, int64_t abort_ptr, int64_t progress_ptr) {
  TORCH_CHECK(flag_ptr != 0, "wait_geq: null flag");
  TORCH_CHECK(timeout_s > 0 && timeout_s < 3600, "wait_geq: timeout must be in (0, 3600) s");
  const uint64_t ticks = (uint64_t)(timeout_s * wall_clock_hz(device));
  hipLaunchKernelGGL(wait_geq_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                     reinterpret_cast<const uint32_t*>(flag_ptr), (uint32_t)target, ticks,
                     reinterpret_cast<uint32_t*>(status_ptr), (uint32_t)code,
                     reinterpret_cast<const uint32_t*>(abort_ptr),
                     reinterpret_cast<uint32_t*>(progress_ptr));
  HIP_OK(hipGetLastError());
}

void signal(int64_t flag_ptr, int64_t value, int64_t stream, int64_t progress_ptr,
            int64_t status_ptr, int64_t abort_ptr) {
  TORCH_CHECK(flag_ptr != 0, "signal: null flag");
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                     reinterpret_cast<uint32_t*>(flag_ptr), (uint32_t)value,
                     reinterpret_cast<uint32_t*>(progress_ptr),
                     reinterpret_cast<const uint32_t*>(status_ptr),
                     reinterpret_cast<const uint32_t*>(abort_ptr));
  HIP_OK(hipGetLastError());
}

void dev_copy(int64_t dst, int64_t src, int64_t nbytes, int64_t stream) {
  TORCH_CHECK(dst && src && nbytes >= 0, "dev_copy: bad arguments");
  TORCH_CHECK(nbytes % 16 == 0 && dst % 16 == 0 && src % 16 == 0,
              "dev_copy: 16-byte aligned pointers and sizes");
  if (nbytes == 0) return;
  const size_t n16 = (size_t)nbytes / 16;
  const size_t blocks = std::min<size_t>((n16 + 255) / 256, 2048);
  hipLaunchKernelGGL(dev_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<uint4*>(dst), reinterpret_cast<const uint4*>(src), n16);
  HIP_OK(hipGetLastError());
}

void copy_segments(int64_t dst_base, int64_t src_base, std::vector<std::pair<int64_t, int64_t>> segs,
                   int64_t stream) {
  TORCH_CHECK(dst_base && src_base, "copy_segments: null base");
  TORCH_CHECK((int)segs.size() <= kMaxSegs, "copy_segments: at most ", kMaxSegs, " segments");
  Segs a{};
  long long most = 0;
  for (const auto& sg : segs) {
    TORCH_CHECK(sg.first >= 0 && sg.second >= 0, "copy_segments: bad segment");
    if (sg.second == 0) continue;
    a.off[a.count] = sg.first;
    a.n[a.count] = sg.second;
    ++a.count;
    most = std::max(most, (long long)sg.second);
  }
  if (a.count == 0) return;
  const long long blocks = std::min<long long>((most / 16 + 255) / 256 + 1, 64);
  hipLaunchKernelGGL(copy_segments_kernel, dim3((unsigned)blocks, (unsigned)a.count), dim3(256), 0,
                     as_stream(stream), reinterpret_cast<char*>(dst_base),
                     reinterpret_cast<const char*>(src_base), a);
  HIP_OK(hipGetLastError());
}

void touch(at::Tensor out, int64_t stream) {
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kInt && out.numel() >= 1, "touch: int32 GPU tensor");
  hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, as_stream(stream),
                     reinterpret_cast<uint32_t*>(out.data_ptr()));
  HIP_OK(hipGetLastError());
}

// ----------------------------------------------------------------------- host-mapped flag words
// Coherent pinned host memory the GPU reads / writes directly: the host sets a flag the GPU
// waits on (isolation test) and reads the status words wait kernels leave on a timeout.
// Coherent, device-mapped pinned host buffer: the host fills it through a CPU tensor view, kernels
// read (or write) it through the device pointer - no copy engine in between.
class HostBuffer {
 public:
  explicit HostBuffer(int64_t nbytes) : n_(nbytes) {
    TORCH_CHECK(nbytes > 0, "HostBuffer: size");
    HIP_OK(hipHostMalloc(&h_, nbytes, hipHostMallocMapped | hipHostMallocCoherent |
                                          hipHostMallocPortable));
    std::memset(h_, 0, nbytes);
    HIP_OK(hipHostGetDevicePointer(&d_, h_, 0));
  }
  ~HostBuffer() {
    if (h_) (void)hipHostFree(h_);
  }
  at::Tensor tensor() const {   // CPU uint8 view (the buffer must outlive it)
    return torch::from_blob(h_, {n_}, at::TensorOptions().dtype(at::kByte));
  }
  int64_t dev_ptr() const { return reinterpret_cast<int64_t>(d_); }
  int64_t nbytes() const { return n_; }

 private:
  int64_t n_;
  void* h_ = nullptr;
  void* d_ = nullptr;
};

class HostWords {
 public:
  explicit HostWords(int64_t n) : n_(n) {
    TORCH_CHECK(n > 0 && n <= (1 << 20), "HostWords: bad size");
    HIP_OK(hipHostMalloc(reinterpret_cast<void**>(&h_), n * sizeof(uint32_t),
                         hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
    std::memset(h_, 0, n * sizeof(uint32_t));
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_), h_, 0));
  }
  ~HostWords() {
    if (h_) (void)hipHostFree(h_);
  }
  void set(int64_t i, int64_t v) {
    idx(i);
    __atomic_store_n(h_ + i, (uint32_t)v, __ATOMIC_SEQ_CST);
  }
  int64_t get(int64_t i) const {
    idx(i);
    return __atomic_load_n(h_ + i, __ATOMIC_SEQ_CST);
  }
  int64_t dev_ptr(int64_t i) const {
    idx(i);
    return reinterpret_cast<int64_t>(d_ + i);
  }
  int64_t size() const { return n_; }

 private:
  void idx(int64_t i) const { TORCH_CHECK(i >= 0 && i < n_, "HostWords index out of range"); }
  int64_t n_;
  uint32_t* h_ = nullptr;
  uint32_t* d_ = nullptr;
};

// ------------------------------------------------------------------------ IPC device memory
// A device allocation of our own (hipMalloc, not the torch caching allocator) so its IPC handle
// names exactly this buffer; the peer opens it and gets a pointer into the same memory.
class IpcBuffer {
 public:
  IpcBuffer(int64_t nbytes, int device) : nbytes_(nbytes), device_(device), owner_(true) {
    TORCH_CHECK(nbytes > 0, "IpcBuffer: size");
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device));
    HIP_OK(hipMalloc(&p_, nbytes));
    HIP_OK(hipMemset(p_, 0, nbytes));
  }
  IpcBuffer(const std::string& handle, int64_t nbytes, int device)
      : nbytes_(nbytes), device_(device), owner_(false) {
    TORCH_CHECK(handle.size() == sizeof(hipIpcMemHandle_t), "IpcBuffer: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle.data(), sizeof(h));
    const c10::hip::HIPGuardMasqueradingAsCUDA g(c10::Device(c10::DeviceType::CUDA, device));
    HIP_OK(hipIpcOpenMemHandle(&p_, h, hipIpcMemLazyEnablePeerAccess));
  }
  ~IpcBuffer() { close(); }
  void close() {
    if (!p_) return;
    if (owner_) (void)hipFree(p_);
    else (void)hipIpcCloseMemHandle(p_);
    p_ = nullptr;
  }
  pybind11::bytes handle() const {
    TORCH_CHECK(owner_ && p_, "IpcBuffer: only the owner exports a handle");
    hipIpcMemHandle_t h;
    HIP_OK(hipIpcGetMemHandle(&h, p_));
    return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  int64_t ptr() const { return reinterpret_cast<int64_t>(p_); }
  int64_t nbytes() const { return nbytes_; }
  // a non-owning tensor view [offset, offset + numel * itemsize) (the buffer must outlive it)
  at::Tensor view(int64_t offset, std::vector<int64_t> shape, at::ScalarType dt) const {
    TORCH_CHECK(p_, "IpcBuffer closed");
    int64_t n = 1;
    for (auto s : shape) n *= s;
    const int64_t bytes = n * (int64_t)c10::elementSize(dt);
    TORCH_CHECK(offset >= 0 && offset + bytes <= nbytes_, "IpcBuffer.view out of range");
    auto opts = at::TensorOptions().dtype(dt).device(c10::Device(c10::DeviceType::CUDA, device_));
    return torch::from_blob(static_cast<char*>(p_) + offset, shape, opts);
  }

 private:
  void* p_ = nullptr;
  int64_t nbytes_;
  int device_;
  bool owner_;
};

}  // namespace

void register_streams(pybind11::module_& m) {
  m.def("stream_create", &stream_create, pybind11::arg("device"), pybind11::arg("mode") = 1,
        pybind11::arg("priority") = 0);
  m.def("stream_destroy", &stream_destroy);
  m.def("stream_cu_count", &stream_cu_count);
  m.def("wall_clock_hz", &wall_clock_hz);
  m.def("wait_geq", &wait_geq, pybind11::arg("flag_ptr"), pybind11::arg("target"),
        pybind11::arg("timeout_s"), pybind11::arg("status_ptr"), pybind11::arg("code"),
        pybind11::arg("stream"), pybind11::arg("device"), pybind11::arg("abort_ptr") = 0,
        pybind11::arg("progress_ptr") = 0);
  m.def("signal", &signal, pybind11::arg("flag_ptr"), pybind11::arg("value"),
        pybind11::arg("stream"), pybind11::arg("progress_ptr") = 0,
        pybind11::arg("status_ptr") = 0, pybind11::arg("abort_ptr") = 0);
  m.def("touch", &touch, pybind11::arg("out"), pybind11::arg("stream") = 0);
  m.def("dev_copy", &dev_copy, pybind11::arg("dst"), pybind11::arg("src"), pybind11::arg("nbytes"),
        pybind11::arg("stream"));
  m.def("copy_segments", &copy_segments, pybind11::arg("dst_base"), pybind11::arg("src_base"),
        pybind11::arg("segments"), pybind11::arg("stream"));
  pybind11::class_<HostBuffer>(m, "HostBuffer")
      .def(pybind11::init<int64_t>())
      .def("tensor", &HostBuffer::tensor)
      .def_property_readonly("dev_ptr", &HostBuffer::dev_ptr)
      .def_property_readonly("nbytes", &HostBuffer::nbytes);
  pybind11::class_<HostWords>(m, "HostWords")
      .def(pybind11::init<int64_t>())
      .def("set", &HostWords::set)
      .def("get", &HostWords::get)
      .def("dev_ptr", &HostWords::dev_ptr)
      .def("__len__", &HostWords::size);
  pybind11::class_<IpcBuffer>(m, "IpcBuffer")
      .def(pybind11::init<int64_t, int>(), pybind11::arg("nbytes"), pybind11::arg("device"))
      .def(pybind11::init<const std::string&, int64_t, int>(), pybind11::arg("handle"),
           pybind11::arg("nbytes"), pybind11::arg("device"))
      .def("handle", &IpcBuffer::handle)
      .def("close", &IpcBuffer::close)
      .def("view", &IpcBuffer::view)
      .def_property_readonly("ptr", &IpcBuffer::ptr)
      .def_property_readonly("nbytes", &IpcBuffer::nbytes);
}
