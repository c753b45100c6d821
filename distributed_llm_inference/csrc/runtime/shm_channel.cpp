// Single-producer / multi-consumer broadcast ring in POSIX shared memory.
//
// Control plane between the per-GPU stage processes of one node.  Hidden states travel over RCCL
// (device memory, xGMI); what each stage's HOST needs to know to launch its part of a micro-batch
// (which sequences, how many new tokens each, which are finished) travels here, so no stage ever
// has to synchronise on a device->host copy of a metadata tensor.  The reference's equivalent is
// hivemind's RPC / protobuf path — microseconds here instead of network RTTs.
//
// Layout: [Header][slot 0]...[slot n-1]; slot = {uint32 len; bytes payload}.  The producer may
// only reuse a slot once every consumer has advanced past it.  Every wait is bounded by a timeout
// (-> Python TimeoutError), which the server's health checker uses to detect a dead peer.
#include <fcntl.h>
#include <pybind11/pybind11.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace dli_rt {

constexpr int kMaxReaders = 64;
constexpr uint64_t kMagic = 0x444c4953484d3031ull;  // "DLISHM01"

struct alignas(64) Header {
  uint64_t magic;
  uint32_t nslots, slot_size, nreaders, pad;
  alignas(64) std::atomic<uint64_t> write_seq;
  alignas(64) std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint64_t> read_seq[kMaxReaders];
  std::atomic<uint64_t> heartbeat_ns[kMaxReaders + 1];  // readers + writer (last)
};

static uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

class ShmChannel {
 public:
  // role: -1 = producer, >= 0 = consumer index.
  ShmChannel(const std::string& name, int role, uint32_t nslots, uint32_t slot_size,
             uint32_t nreaders, bool create, double open_timeout_s)
      : name_(name), role_(role), creator_(create) {
    if (nreaders > (uint32_t)kMaxReaders) throw std::invalid_argument("too many readers");
    const size_t total = sizeof(Header) + (size_t)nslots * (slot_size + 8);
    int fd = -1;
    if (create) {
      shm_unlink(name.c_str());
      fd = shm_open(name.c_str(), O_CREAT | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name);
      if (ftruncate(fd, (off_t)total) != 0) {
        close(fd);
        throw std::runtime_error("ftruncate failed");
      }
    } else {
      // wait for the creator without the GIL (it may be another thread of this process)
      py::gil_scoped_release nogil;
      const uint64_t deadline = now_ns() + (uint64_t)(open_timeout_s * 1e9);
      while (true) {
        fd = shm_open(name.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(Header)) break;
          close(fd);
          fd = -1;
        }
        if (now_ns() > deadline) throw std::runtime_error("timed out opening shm channel " + name);
        std::this_thread::sleep_for(std::chrono::milliseconds(2));
      }
    }
    struct stat st;
    fstat(fd, &st);
    size_ = (size_t)st.st_size;
    base_ = (uint8_t*)mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = reinterpret_cast<Header*>(base_);
    if (create) {
      hdr_->nslots = nslots;
      hdr_->slot_size = slot_size;
      hdr_->nreaders = nreaders;
      hdr_->write_seq.store(0);
      hdr_->closed.store(0);
      for (int i = 0; i < kMaxReaders; ++i) hdr_->read_seq[i].store(0);
      for (int i = 0; i <= kMaxReaders; ++i) hdr_->heartbeat_ns[i].store(now_ns());
      std::atomic_thread_fence(std::memory_order_release);
      reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->store(kMagic, std::memory_order_release);
    } else {
      py::gil_scoped_release nogil;
      const uint64_t deadline = now_ns() + (uint64_t)(open_timeout_s * 1e9);
      while (reinterpret_cast<std::atomic<uint64_t>*>(&hdr_->magic)->load(std::memory_order_acquire) != kMagic) {
        if (now_ns() > deadline) throw std::runtime_error("shm channel never initialised");
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    }
    if (role_ >= (int)hdr_->nreaders) throw std::invalid_argument("reader index out of range");
  }

  ~ShmChannel() {
    if (base_ && base_ != MAP_FAILED) munmap(base_, size_);
    unlink();
  }

  // Remove the name from /dev/shm (creator only).  Existing mappings stay valid, so calling this
  // once every peer has attached leaves nothing behind even if a process is killed later.
  void unlink() {
    if (creator_) shm_unlink(name_.c_str());
    creator_ = false;
  }

  void send(const py::bytes& msg, double timeout_s) {
    if (role_ != -1) throw std::logic_error("only the producer can send");
    std::string s = msg;
    if (s.size() > hdr_->slot_size) throw std::invalid_argument("message larger than slot");
    const uint64_t seq = hdr_->write_seq.load(std::memory_order_relaxed);
    {
      py::gil_scoped_release nogil;
      wait([&] {
        for (uint32_t r = 0; r < hdr_->nreaders; ++r)
          if (seq - hdr_->read_seq[r].load(std::memory_order_acquire) >= hdr_->nslots) return false;
        return true;
      }, timeout_s, "send");
    }
    uint8_t* slot = slot_ptr(seq);
    const uint32_t len = (uint32_t)s.size();
    std::memcpy(slot, &len, 4);
    std::memcpy(slot + 8, s.data(), s.size());
    hdr_->write_seq.store(seq + 1, std::memory_order_release);
    hdr_->heartbeat_ns[kMaxReaders].store(now_ns(), std::memory_order_relaxed);
  }

  py::bytes recv(double timeout_s) {
    if (role_ < 0) throw std::logic_error("producer cannot recv");
    const uint64_t seq = hdr_->read_seq[role_].load(std::memory_order_relaxed);
    {
      py::gil_scoped_release nogil;
      wait([&] { return hdr_->write_seq.load(std::memory_order_acquire) > seq; }, timeout_s, "recv");
    }
    const uint8_t* slot = slot_ptr(seq);
    uint32_t len;
    std::memcpy(&len, slot, 4);
    py::bytes out(reinterpret_cast<const char*>(slot + 8), len);
    hdr_->read_seq[role_].store(seq + 1, std::memory_order_release);
    hdr_->heartbeat_ns[role_].store(now_ns(), std::memory_order_relaxed);
    return out;
  }

  bool poll() const {
    if (role_ < 0) return false;
    return hdr_->write_seq.load(std::memory_order_acquire) > hdr_->read_seq[role_].load();
  }

  void close_channel() { hdr_->closed.store(1, std::memory_order_release); }
  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  void heartbeat() { hdr_->heartbeat_ns[role_ < 0 ? kMaxReaders : role_].store(now_ns()); }
  // seconds since participant `who` (-1 = producer) last made progress
  double idle_seconds(int who) const {
    const uint64_t t = hdr_->heartbeat_ns[who < 0 ? kMaxReaders : who].load();
    return (double)(now_ns() - t) * 1e-9;
  }
  uint64_t write_seq() const { return hdr_->write_seq.load(); }
  uint64_t read_seq(int r) const { return hdr_->read_seq[r].load(); }

 private:
  template <typename Pred>
  void wait(Pred ready, double timeout_s, const char* what) {
    const uint64_t deadline = timeout_s > 0 ? now_ns() + (uint64_t)(timeout_s * 1e9) : 0;
    for (uint64_t spin = 0;; ++spin) {
      if (ready()) return;
      if (hdr_->closed.load(std::memory_order_acquire)) throw ChannelClosed();
      if (spin < 2000) continue;
      if (spin < 4000) {
        sched_yield();
        continue;
      }
      if (deadline && now_ns() > deadline) throw ChannelTimeout(what);
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  uint8_t* slot_ptr(uint64_t seq) const {
    return base_ + sizeof(Header) + (size_t)(seq % hdr_->nslots) * (hdr_->slot_size + 8);
  }

 public:
  struct ChannelClosed : std::runtime_error {
    ChannelClosed() : std::runtime_error("shm channel closed") {}
  };
  struct ChannelTimeout : std::runtime_error {
    explicit ChannelTimeout(const char* w) : std::runtime_error(std::string("shm channel ") + w + " timed out") {}
  };

 private:
  std::string name_;
  int role_;
  bool creator_;
  uint8_t* base_ = nullptr;
  size_t size_ = 0;
  Header* hdr_ = nullptr;
};

void register_shm_channel(py::module_& m) {
  static py::exception<ShmChannel::ChannelClosed> closed_exc(m, "ChannelClosed", PyExc_EOFError);
  static py::exception<ShmChannel::ChannelTimeout> timeout_exc(m, "ChannelTimeout", PyExc_TimeoutError);
  py::register_exception_translator([](std::exception_ptr p) {
    try {
      if (p) std::rethrow_exception(p);
    } catch (const ShmChannel::ChannelClosed& e) {
      py::set_error(closed_exc, e.what());
    } catch (const ShmChannel::ChannelTimeout& e) {
      py::set_error(timeout_exc, e.what());
    }
  });
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, int, uint32_t, uint32_t, uint32_t, bool, double>(),
           py::arg("name"), py::arg("role"), py::arg("nslots") = 64, py::arg("slot_size") = 65536,
           py::arg("nreaders") = 1, py::arg("create") = false, py::arg("open_timeout") = 60.0)
      .def("send", &ShmChannel::send, py::arg("msg"), py::arg("timeout") = 0.0)
      .def("recv", &ShmChannel::recv, py::arg("timeout") = 0.0)
      .def("poll", &ShmChannel::poll)
      .def("close", &ShmChannel::close_channel)
      .def("unlink", &ShmChannel::unlink)
      .def_property_readonly("closed", &ShmChannel::closed)
      .def("heartbeat", &ShmChannel::heartbeat)
      .def("idle_seconds", &ShmChannel::idle_seconds)
      .def_property_readonly("write_seq", &ShmChannel::write_seq)
      .def("read_seq", &ShmChannel::read_seq);
}

void register_block_manager(py::module_& m);

}  // namespace dli_rt

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "native host runtime of distributed_llm_inference (block manager, shm channels)";
  dli_rt::register_block_manager(m);
  dli_rt::register_shm_channel(m);
}
