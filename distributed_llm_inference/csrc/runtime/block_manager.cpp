// Paged KV-cache block manager (host side, C++).
//
// The reference keeps per-session KV as Python dicts of growing tensors keyed by generation_id
// (models/llama/cache.py:14-19, 78-109) — every decode token re-allocates and copies the whole
// cache.  Here each pipeline stage owns ONE preallocated KV pool sized from HBM; this class hands
// out fixed-size blocks of it to sequences and produces, per batch, the device-side metadata the
// kernels consume (slot_mapping, positions, block_tables, seq_lens, q_start) directly into pinned
// host buffers — no Python loops on the per-step host path.
//
// Two slot policies:
//   * full cache: slot(a) = a (token a of the sequence), the cache grows one block at a time;
//   * attention-sink window (StreamingLLM, the reference's PartialLlamaSinkCache semantics):
//       sink tokens a < n_sink       -> slot a                       (never evicted)
//       rolling tokens a >= n_sink   -> slot sink_pad + (a - n_sink) % ring
//     so a sequence never holds more than sink_pad + ring slots; old rolling tokens are
//     overwritten in place (eviction costs nothing, see attention.hip for the position algebra).
//
// Allocation is deterministic (LIFO free list seeded in a fixed order), so every pipeline stage
// running the same sequence of calls produces identical block tables.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace py = pybind11;

namespace dli_rt {

struct SeqState {
  int64_t length = 0;            // tokens stored so far (absolute count)
  std::vector<int32_t> blocks;   // physical block ids, in slot order
};

class BlockManager {
 public:
  BlockManager(int64_t num_blocks, int block_size, int window_length, int num_sink_tokens,
               int max_chunk)
      : num_blocks_(num_blocks), bs_(block_size), window_(window_length), n_sink_(num_sink_tokens) {
    if (num_blocks <= 0 || block_size <= 0 || block_size % 32 != 0)
      throw std::invalid_argument("block_size must be a positive multiple of 32");
    if (window_ > 0) {
      if (n_sink_ < 0 || n_sink_ >= window_)
        throw std::invalid_argument("need 0 <= num_sink_tokens < window_length");
      sink_pad_ = ((n_sink_ + 31) / 32) * 32;
      const int need = window_ - n_sink_ + std::max(0, max_chunk - 1);
      ring_ = ((need + 31) / 32) * 32;
    }
    free_.reserve(num_blocks);
    for (int64_t b = num_blocks - 1; b >= 0; --b) free_.push_back((int32_t)b);
  }

  // ---------------------------------------------------------------- sequence lifecycle
  bool has_sequence(int64_t sid) const { return seqs_.count(sid) != 0; }

  void add_sequence(int64_t sid) {
    if (seqs_.count(sid)) throw std::invalid_argument("sequence already exists");
    seqs_.emplace(sid, SeqState());
  }

  void free_sequence(int64_t sid) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) return;
    for (auto b = it->second.blocks.rbegin(); b != it->second.blocks.rend(); ++b) free_.push_back(*b);
    seqs_.erase(it);
  }

  int64_t length(int64_t sid) const { return get(sid).length; }

  // Slots (not tokens) a sequence of `len` tokens occupies.
  int64_t slots_for(int64_t len) const {
    if (window_ <= 0) return len;
    if (len <= n_sink_) return len;
    return sink_pad_ + std::min<int64_t>(ring_, len - n_sink_);
  }
  int64_t blocks_for(int64_t len) const { return (slots_for(len) + bs_ - 1) / bs_; }

  // Extra blocks needed to grow `sid` by n tokens (sid may not exist yet -> from zero).
  int64_t blocks_needed(int64_t sid, int64_t n) const {
    auto it = seqs_.find(sid);
    const int64_t cur = it == seqs_.end() ? 0 : (int64_t)it->second.blocks.size();
    const int64_t len = it == seqs_.end() ? 0 : it->second.length;
    return std::max<int64_t>(0, blocks_for(len + n) - cur);
  }

  bool can_append(const std::vector<int64_t>& sids, const std::vector<int64_t>& ns) const {
    int64_t need = 0;
    for (size_t i = 0; i < sids.size(); ++i) need += blocks_needed(sids[i], ns[i]);
    return need <= (int64_t)free_.size();
  }

  // Reserve space for n more tokens; creates the sequence on first use.  Returns false (and
  // changes nothing) if the pool is exhausted.
  bool append(int64_t sid, int64_t n) {
    if (!seqs_.count(sid)) seqs_.emplace(sid, SeqState());
    SeqState& s = seqs_.at(sid);
    const int64_t need = blocks_for(s.length + n) - (int64_t)s.blocks.size();
    if (need > (int64_t)free_.size()) return false;
    for (int64_t i = 0; i < need; ++i) {
      s.blocks.push_back(free_.back());
      free_.pop_back();
    }
    s.length += n;
    return true;
  }

  // All-or-nothing batch reservation: grows every sids[i] by ns[i] tokens if the pool can hold
  // all of them, otherwise changes nothing and returns false (one call per step instead of B).
  bool append_batch(const std::vector<int64_t>& sids, const std::vector<int64_t>& ns) {
    if (sids.size() != ns.size()) throw std::invalid_argument("append_batch: size mismatch");
    if (!can_append(sids, ns)) return false;
    for (size_t i = 0; i < sids.size(); ++i) append(sids[i], ns[i]);
    return true;
  }

  // Undo the last reservation of n tokens: shrink the length and return the blocks the shorter
  // sequence no longer covers to the free list (in the reverse order they were taken, so the LIFO
  // allocation order -- and every stage's block tables -- stay what they were).  A sequence that
  // shrinks to zero tokens is dropped, as if it had never been appended to.  With a sink window
  // the ring slots the undone tokens wrapped onto are not restored: callers roll back before any
  // KV is written (validation failures) or accept that the overwritten window tokens are lost.
  void rollback(int64_t sid, int64_t n) {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::out_of_range("unknown sequence " + std::to_string(sid));
    SeqState& s = it->second;
    if (n < 0 || n > s.length) throw std::invalid_argument("rollback beyond the sequence start");
    s.length -= n;
    const int64_t keep = blocks_for(s.length);
    while ((int64_t)s.blocks.size() > keep) {
      free_.push_back(s.blocks.back());
      s.blocks.pop_back();
    }
    if (s.length == 0) seqs_.erase(it);
  }

  void rollback_batch(const std::vector<int64_t>& sids, const std::vector<int64_t>& ns) {
    if (sids.size() != ns.size()) throw std::invalid_argument("rollback_batch: size mismatch");
    for (size_t i = sids.size(); i-- > 0;) rollback(sids[i], ns[i]);  // reverse of append order
  }

  int64_t slot_of(int64_t sid, int64_t a) const {
    const SeqState& s = get(sid);
    return physical(s, logical_slot(a));
  }

  std::vector<int32_t> block_table(int64_t sid) const { return get(sid).blocks; }

  // ---------------------------------------------------------------- batch metadata
  // For a batch whose sequence i contributes q_lens[i] NEW tokens (already reserved with append()),
  // fill (all pointers are host buffers, e.g. pinned torch tensors):
  //   slot_mapping[T] int64, positions[T] int32, block_tables[B, bt_cols] int32 (-> 0-padded),
  //   seq_lens[B] int32, q_start[B+1] int32.
  // pos_offsets (optional, B entries) shifts the RoPE position of every token of sequence i.
  // Rows >= sids.size() up to pad_rows are filled as empty sequences (seq_len 0), so a captured
  // graph of a larger batch bucket stays valid.  Returns T.
  int64_t prepare(const std::vector<int64_t>& sids, const std::vector<int64_t>& q_lens,
                  uintptr_t slot_mapping, uintptr_t positions, uintptr_t block_tables,
                  int64_t bt_cols, uintptr_t seq_lens, uintptr_t q_start, int64_t pad_rows,
                  const std::vector<int64_t>& pos_offsets) const {
    if (sids.size() != q_lens.size()) throw std::invalid_argument("sids/q_lens length mismatch");
    auto* sm = reinterpret_cast<int64_t*>(slot_mapping);
    auto* pos = reinterpret_cast<int32_t*>(positions);
    auto* bt = reinterpret_cast<int32_t*>(block_tables);
    auto* sl = reinterpret_cast<int32_t*>(seq_lens);
    auto* qs = reinterpret_cast<int32_t*>(q_start);
    const int64_t B = (int64_t)sids.size();
    const int64_t rows = std::max<int64_t>(B, pad_rows);
    int64_t t = 0;
    for (int64_t i = 0; i < B; ++i) {
      const SeqState& s = get(sids[i]);
      const int64_t q = q_lens[i];
      if (q > s.length) throw std::invalid_argument("q_len exceeds reserved length");
      if ((int64_t)s.blocks.size() > bt_cols) throw std::invalid_argument("block table too narrow");
      if (qs) qs[i] = (int32_t)t;
      const int64_t off = pos_offsets.empty() ? 0 : pos_offsets[i];
      for (int64_t a = s.length - q; a < s.length; ++a, ++t) {
        if (sm) sm[t] = physical(s, logical_slot(a));
        if (pos) pos[t] = (int32_t)(a + off);
      }
      if (sl) sl[i] = (int32_t)s.length;
      if (bt) {
        int32_t* row = bt + i * bt_cols;
        std::memcpy(row, s.blocks.data(), s.blocks.size() * sizeof(int32_t));
        std::memset(row + s.blocks.size(), 0, (bt_cols - s.blocks.size()) * sizeof(int32_t));
      }
    }
    for (int64_t i = B; i < rows; ++i) {
      if (qs) qs[i] = (int32_t)t;
      if (sl) sl[i] = 0;
      if (bt) std::memset(bt + i * bt_cols, 0, bt_cols * sizeof(int32_t));
    }
    if (qs) qs[rows] = (int32_t)t;
    return t;
  }

  // ---------------------------------------------------------------- properties
  int64_t num_free_blocks() const { return (int64_t)free_.size(); }
  int64_t num_blocks() const { return num_blocks_; }
  int block_size() const { return bs_; }
  int window_length() const { return window_; }
  int num_sink_tokens() const { return n_sink_; }
  int sink_pad() const { return sink_pad_; }
  int ring() const { return ring_; }
  int64_t max_blocks_per_seq(int64_t max_len) const { return blocks_for(max_len); }
  std::vector<int64_t> sequences() const {
    std::vector<int64_t> out;
    for (auto& kv : seqs_) out.push_back(kv.first);
    std::sort(out.begin(), out.end());
    return out;
  }

 private:
  const SeqState& get(int64_t sid) const {
    auto it = seqs_.find(sid);
    if (it == seqs_.end()) throw std::out_of_range("unknown sequence " + std::to_string(sid));
    return it->second;
  }
  int64_t logical_slot(int64_t a) const {
    if (window_ <= 0 || a < n_sink_) return a;
    return sink_pad_ + (a - n_sink_) % ring_;
  }
  int64_t physical(const SeqState& s, int64_t slot) const {
    const int64_t bi = slot / bs_;
    if (bi >= (int64_t)s.blocks.size()) throw std::out_of_range("slot beyond reserved blocks");
    return (int64_t)s.blocks[bi] * bs_ + slot % bs_;
  }

  int64_t num_blocks_;
  int bs_, window_, n_sink_;
  int sink_pad_ = 0, ring_ = 0;
  std::vector<int32_t> free_;
  std::unordered_map<int64_t, SeqState> seqs_;
};

void register_block_manager(py::module_& m) {
  py::class_<BlockManager>(m, "BlockManager")
      .def(py::init<int64_t, int, int, int, int>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("window_length") = 0, py::arg("num_sink_tokens") = 0,
           py::arg("max_chunk") = 512)
      .def("has_sequence", &BlockManager::has_sequence)
      .def("add_sequence", &BlockManager::add_sequence)
      .def("free_sequence", &BlockManager::free_sequence)
      .def("length", &BlockManager::length)
      .def("slots_for", &BlockManager::slots_for)
      .def("blocks_for", &BlockManager::blocks_for)
      .def("blocks_needed", &BlockManager::blocks_needed)
      .def("can_append", &BlockManager::can_append)
      .def("append", &BlockManager::append)
      .def("append_batch", &BlockManager::append_batch)
      .def("rollback", &BlockManager::rollback)
      .def("rollback_batch", &BlockManager::rollback_batch)
      .def("slot_of", &BlockManager::slot_of)
      .def("block_table", &BlockManager::block_table)
      .def("prepare", &BlockManager::prepare, py::arg("sids"), py::arg("q_lens"),
           py::arg("slot_mapping"), py::arg("positions"), py::arg("block_tables"),
           py::arg("bt_cols"), py::arg("seq_lens"), py::arg("q_start"), py::arg("pad_rows") = 0,
           py::arg("pos_offsets") = std::vector<int64_t>())
      .def_property_readonly("num_free_blocks", &BlockManager::num_free_blocks)
      .def_property_readonly("num_blocks", &BlockManager::num_blocks)
      .def_property_readonly("block_size", &BlockManager::block_size)
      .def_property_readonly("window_length", &BlockManager::window_length)
      .def_property_readonly("num_sink_tokens", &BlockManager::num_sink_tokens)
      .def_property_readonly("sink_pad", &BlockManager::sink_pad)
      .def_property_readonly("ring", &BlockManager::ring)
      .def("max_blocks_per_seq", &BlockManager::max_blocks_per_seq)
      .def("sequences", &BlockManager::sequences);
}

}  // namespace dli_rt
