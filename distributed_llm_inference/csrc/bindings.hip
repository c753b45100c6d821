// Torch bindings for the CDNA4 kernels and the RCCL point-to-point communicator.
//
// Every entry point validates device / dtype / contiguity / shapes on the host before launching:
// a mis-shaped operand must raise a Python error, never become an out-of-bounds GPU access.
// Kernels run on the caller's current HIP stream (so they are hipGraph-capturable).
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <cstdlib>

#include "kernels/kernels.h"

using at::Tensor;
using c10::optional;

namespace {

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")
#define CHECK_BF16(t) TORCH_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bfloat16")
#define CHECK_I32(t) TORCH_CHECK((t).scalar_type() == at::kInt, #t " must be int32")
#define CHECK_I64(t) TORCH_CHECK((t).scalar_type() == at::kLong, #t " must be int64")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_IN(t) \
  CHECK_DEV(t);     \
  CHECK_CONTIG(t)

inline dli::bf16* bp(const Tensor& t) { return reinterpret_cast<dli::bf16*>(t.data_ptr()); }
inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }
inline void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, ": unsupported shape/configuration (rc=", rc, ")");
}

// ------------------------------------------------------------------------------ normalisation
void rms_norm(Tensor out, Tensor x, optional<Tensor> residual, Tensor w, double eps,
              optional<Tensor> residual_out) {
  CHECK_IN(out); CHECK_IN(x); CHECK_IN(w);
  CHECK_BF16(out); CHECK_BF16(x); CHECK_BF16(w);
  const int64_t hidden = x.size(-1);
  const int64_t rows = x.numel() / hidden;
  TORCH_CHECK(w.numel() == hidden && out.numel() == x.numel(), "rms_norm: shape mismatch");
  const dli::bf16* r = nullptr;
  dli::bf16* ro = nullptr;
  if (residual.has_value()) {
    CHECK_IN(*residual); CHECK_BF16(*residual);
    TORCH_CHECK(residual->numel() == x.numel(), "rms_norm: residual shape mismatch");
    r = bp(*residual);
    ro = bp(*residual);
    if (residual_out.has_value()) {
      CHECK_IN(*residual_out); CHECK_BF16(*residual_out);
      TORCH_CHECK(residual_out->numel() == x.numel(), "rms_norm: residual_out shape mismatch");
      ro = bp(*residual_out);
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_rms_norm(bp(out), bp(x), r, ro, bp(w), (float)eps, (int)rows, (int)hidden,
                                cur_stream()), "rms_norm");
}

void splitk_reduce(Tensor out, Tensor parts) {
  CHECK_IN(out); CHECK_IN(parts); CHECK_BF16(out); CHECK_F32(parts);
  TORCH_CHECK(parts.dim() == 3 && out.numel() == parts.size(1) * parts.size(2),
              "splitk_reduce: parts [S, M, N] and out [M, N]");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(parts.device());
  check_rc(dli::launch_splitk_reduce(bp(out), parts.data_ptr<float>(), (int)parts.size(0),
                                     (size_t)out.numel(), cur_stream()), "splitk_reduce");
}

// RMSNorm whose input is the un-reduced fp32 split-K output of gemm_tile(defer_reduce=True):
// parts [splits, rows, hidden]; the sum (rounded to bf16) replaces x.
void rms_norm_splitk(Tensor out, Tensor parts, optional<Tensor> residual, Tensor w, double eps,
                     optional<Tensor> residual_out) {
  CHECK_IN(out); CHECK_IN(parts); CHECK_IN(w);
  CHECK_BF16(out); CHECK_BF16(w);
  // fp32 partials, or bf16 ones (8-bit weight modes: gemm_tile epilogue 4)
  const bool parts_bf16 = parts.scalar_type() == at::kBFloat16;
  TORCH_CHECK(parts_bf16 || parts.scalar_type() == at::kFloat, "rms_norm_splitk: fp32 or bf16 parts");
  TORCH_CHECK(parts.dim() == 3, "rms_norm_splitk: parts must be [splits, rows, hidden]");
  const int64_t splits = parts.size(0), rows = parts.size(1), hidden = parts.size(2);
  TORCH_CHECK(splits >= 1 && w.numel() == hidden && out.numel() == rows * hidden,
              "rms_norm_splitk: shape mismatch");
  const dli::bf16* r = nullptr;
  dli::bf16* ro = nullptr;
  if (residual.has_value()) {
    CHECK_IN(*residual); CHECK_BF16(*residual);
    TORCH_CHECK(residual->numel() == rows * hidden, "rms_norm_splitk: residual shape mismatch");
    r = bp(*residual);
    ro = bp(*residual);
    if (residual_out.has_value()) {
      CHECK_IN(*residual_out); CHECK_BF16(*residual_out);
      TORCH_CHECK(residual_out->numel() == rows * hidden, "rms_norm_splitk: residual_out shape");
      ro = bp(*residual_out);
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(parts.device());
  check_rc(dli::launch_rms_norm(bp(out), nullptr, r, ro, bp(w), (float)eps, (int)rows,
                                (int)hidden, cur_stream(), parts.data_ptr(), (int)splits,
                                parts_bf16),
           "rms_norm_splitk");
}

void layer_norm(Tensor out, Tensor x, optional<Tensor> residual, Tensor w, Tensor b, double eps,
                optional<Tensor> residual_out) {
  CHECK_IN(out); CHECK_IN(x); CHECK_IN(w); CHECK_IN(b);
  CHECK_BF16(out); CHECK_BF16(x); CHECK_BF16(w); CHECK_BF16(b);
  const int64_t hidden = x.size(-1);
  const int64_t rows = x.numel() / hidden;
  TORCH_CHECK(w.numel() == hidden && b.numel() == hidden && out.numel() == x.numel(),
              "layer_norm: shape mismatch");
  const dli::bf16* r = nullptr;
  dli::bf16* ro = nullptr;
  if (residual.has_value()) {
    CHECK_IN(*residual); CHECK_BF16(*residual);
    TORCH_CHECK(residual->numel() == x.numel(), "layer_norm: residual shape mismatch");
    r = bp(*residual);
    ro = bp(*residual);
    if (residual_out.has_value()) {
      CHECK_IN(*residual_out); CHECK_BF16(*residual_out);
      TORCH_CHECK(residual_out->numel() == x.numel(), "layer_norm: residual_out shape mismatch");
      ro = bp(*residual_out);
    }
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_layer_norm(bp(out), bp(x), r, ro, bp(w), bp(b), (float)eps, (int)rows,
                                  (int)hidden, cur_stream()), "layer_norm");
}

// ------------------------------------------------------------------------------ activations
void silu_mul(Tensor out, Tensor x, bool interleaved) {
  CHECK_IN(out); CHECK_IN(x); CHECK_BF16(out); CHECK_BF16(x);
  const int64_t two_i = x.size(-1);
  TORCH_CHECK(two_i % 2 == 0, "silu_mul: last dim must be even");
  const int64_t rows = x.numel() / two_i;
  TORCH_CHECK(out.numel() == rows * (two_i / 2), "silu_mul: out shape mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_silu_mul(bp(out), bp(x), (int)rows, (int)(two_i / 2), interleaved,
                                cur_stream()),
           "silu_mul");
}

void gelu_bias(Tensor out, Tensor x, optional<Tensor> bias) {
  CHECK_IN(out); CHECK_IN(x); CHECK_BF16(out); CHECK_BF16(x);
  const int64_t cols = x.size(-1);
  const int64_t rows = x.numel() / cols;
  TORCH_CHECK(out.numel() == x.numel(), "gelu: out shape mismatch");
  dli::bf16* bb = nullptr;
  if (bias.has_value()) {
    CHECK_IN(*bias); CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == cols, "gelu: bias shape mismatch");
    bb = bp(*bias);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_gelu_bias(bp(out), bp(x), bb, (int)rows, (int)cols, cur_stream()), "gelu");
}

void add(Tensor out, Tensor a, Tensor b) {
  CHECK_IN(out); CHECK_IN(a); CHECK_IN(b);
  CHECK_BF16(out); CHECK_BF16(a); CHECK_BF16(b);
  TORCH_CHECK(a.numel() == b.numel() && out.numel() == a.numel(), "add: shape mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  check_rc(dli::launch_add(bp(out), bp(a), bp(b), (size_t)a.numel(), cur_stream()), "add");
}

// ------------------------------------------------------------------------------ rope + cache
// Returns true for an fp8 (e4m3fn) cache, false for bf16.
bool check_cache(const Tensor& k_cache, const Tensor& v_cache, int64_t nkv, int64_t D) {
  CHECK_IN(k_cache); CHECK_IN(v_cache);
  const bool fp8 = k_cache.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(fp8 || k_cache.scalar_type() == at::kBFloat16, "KV cache must be bf16 or fp8 e4m3fn");
  TORCH_CHECK(v_cache.scalar_type() == k_cache.scalar_type(), "k/v caches must share a dtype");
  TORCH_CHECK(k_cache.dim() == 4 && v_cache.dim() == 5, "k_cache must be 4-D, v_cache 5-D");
  // k: [blocks, nkv, bs, D]; v: [blocks, nkv, bs/8, D, 8]
  TORCH_CHECK(k_cache.size(1) == nkv && k_cache.size(3) == D, "k_cache must be [blocks, nkv, bs, D]");
  TORCH_CHECK(v_cache.size(0) == k_cache.size(0) && v_cache.size(1) == nkv &&
                  v_cache.size(2) * 8 == k_cache.size(2) && v_cache.size(3) == D &&
                  v_cache.size(4) == 8,
              "v_cache must be [blocks, nkv, bs/8, D, 8]");
  return fp8;
}

void rope_cache(Tensor qkv, optional<Tensor> positions, optional<Tensor> slot_mapping,
                optional<Tensor> cos_sin, Tensor q_out, optional<Tensor> q_sink_out,
                int64_t window, Tensor k_cache, Tensor v_cache, int64_t nh, int64_t nkv,
                double k_scale, double v_scale) {
  CHECK_DEV(qkv);
  // qkv: the bf16 GEMM output [T, *], or its un-reduced split-K partials [S, T, N] (fp32, or
  // bf16 from the fp8 path's gemm_tile epilogue 4)
  const bool parts_bf16 = qkv.scalar_type() == at::kBFloat16 && qkv.dim() == 3;
  const bool parts = qkv.scalar_type() == at::kFloat || parts_bf16;
  if (parts) {
    TORCH_CHECK(qkv.dim() == 3 && qkv.is_contiguous(), "qkv partials must be contiguous [S, T, N]");
  } else {
    CHECK_BF16(qkv);
    TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv must be [T, *] with unit inner stride");
  }
  const int64_t T = parts ? qkv.size(1) : qkv.size(0);
  CHECK_IN(q_out); CHECK_BF16(q_out);
  TORCH_CHECK(q_out.dim() == 3 && q_out.size(0) == T && q_out.size(1) == nh, "q_out must be [T, nh, D]");
  const int64_t D = q_out.size(2);
  TORCH_CHECK(qkv.size(qkv.dim() - 1) >= (nh + 2 * nkv) * D, "qkv too narrow for nh/nkv/D");
  const bool fp8 = check_cache(k_cache, v_cache, nkv, D);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "KV scales must be positive");
  dli::RopeCacheParams p{};
  p.kv_fp8 = fp8 ? 1 : 0;
  p.k_inv_scale = (float)(1.0 / k_scale);
  p.v_inv_scale = (float)(1.0 / v_scale);
  if (parts) {
    p.qkv = nullptr;
    p.qkv_parts = qkv.data_ptr();
    p.parts_bf16 = parts_bf16 ? 1 : 0;
    p.splits = (int)qkv.size(0);
    p.qkv_stride = qkv.size(2);
    p.split_stride = (long)(T * qkv.size(2));
  } else {
    p.qkv = bp(qkv);
    p.qkv_stride = qkv.stride(0);
  }
  if (positions.has_value()) {
    CHECK_IN(*positions); CHECK_I32(*positions);
    TORCH_CHECK(positions->numel() == T, "positions must have T entries");
    p.positions = positions->data_ptr<int>();
  }
  if (slot_mapping.has_value()) {
    CHECK_IN(*slot_mapping); CHECK_I64(*slot_mapping);
    TORCH_CHECK(slot_mapping->numel() == T, "slot_mapping must have T entries");
    p.slot_mapping = reinterpret_cast<const long*>(slot_mapping->data_ptr<int64_t>());
  }
  if (cos_sin.has_value()) {
    CHECK_IN(*cos_sin); CHECK_F32(*cos_sin);
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == D, "cos_sin must be [max_pos, D]");
    TORCH_CHECK(positions.has_value(), "rope needs positions");
    p.cos_sin = cos_sin->data_ptr<float>();
    p.max_pos = (int)cos_sin->size(0);
  }
  p.q_out = bp(q_out);
  if (q_sink_out.has_value()) {
    CHECK_IN(*q_sink_out); CHECK_BF16(*q_sink_out);
    TORCH_CHECK(q_sink_out->sizes() == q_out.sizes(), "q_sink_out shape mismatch");
    TORCH_CHECK(window > 0, "q_sink_out requires window > 0");
    p.q_sink_out = bp(*q_sink_out);
  }
  p.window = (int)window;
  p.k_cache = k_cache.data_ptr();
  p.v_cache = v_cache.data_ptr();
  p.nh = (int)nh;
  p.nkv = (int)nkv;
  p.D = (int)D;
  p.bs = (int)k_cache.size(2);
  const c10::hip::HIPGuardMasqueradingAsCUDA g(qkv.device());
  check_rc(dli::launch_rope_cache(p, (int)T, cur_stream()), "rope_cache");
}

// ------------------------------------------------------------------------------ attention
dli::AttnParams attn_common(Tensor& out, Tensor& q, optional<Tensor>& q_sink, Tensor& k_cache,
                            Tensor& v_cache, Tensor& block_tables, Tensor& seq_lens, double scale,
                            int64_t n_sink, int64_t sink_pad, int64_t ring, int64_t window,
                            double k_scale, double v_scale, int64_t& D,
                            bool allow_empty_out = false) {
  CHECK_IN(out); CHECK_IN(q); CHECK_BF16(out); CHECK_BF16(q);
  TORCH_CHECK(q.dim() == 3, "q must be [T, nh, D]");
  // empty `out`: only for an MX-output decode, whose kernel never touches the bf16 output
  TORCH_CHECK(out.sizes() == q.sizes() || (allow_empty_out && out.numel() == 0),
              "out must match q");
  const int64_t nh = q.size(1);
  D = q.size(2);
  const int64_t nkv = k_cache.size(1);
  TORCH_CHECK(nkv > 0 && nh % nkv == 0, "nh must be a multiple of nkv");
  const bool fp8 = check_cache(k_cache, v_cache, nkv, D);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "KV scales must be positive");
  CHECK_IN(block_tables); CHECK_I32(block_tables); CHECK_IN(seq_lens); CHECK_I32(seq_lens);
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) == seq_lens.size(0),
              "block_tables must be [B, max_blocks]");
  dli::AttnParams p{};
  p.q = bp(q);
  if (ring > 0) {
    TORCH_CHECK(q_sink.has_value() || n_sink == 0, "window mode with sinks needs q_sink");
    TORCH_CHECK(window > n_sink && sink_pad >= n_sink && sink_pad % 32 == 0 && ring % 32 == 0,
                "invalid window configuration");
  }
  if (q_sink.has_value()) {
    CHECK_IN(*q_sink); CHECK_BF16(*q_sink);
    TORCH_CHECK(q_sink->sizes() == q.sizes(), "q_sink must match q");
    p.q_sink = bp(*q_sink);
  }
  p.k_cache = k_cache.data_ptr();
  p.v_cache = v_cache.data_ptr();
  p.kv_fp8 = fp8 ? 1 : 0;
  p.k_scale = (float)k_scale;
  p.v_scale = (float)v_scale;
  p.out = out.numel() ? bp(out) : nullptr;
  p.block_tables = block_tables.data_ptr<int>();
  p.bt_stride = (int)block_tables.size(1);
  p.seq_lens = seq_lens.data_ptr<int>();
  p.scale_log2 = (float)(scale * 1.4426950408889634);
  p.nh = (int)nh;
  p.nkv = (int)nkv;
  p.bs = (int)k_cache.size(2);
  p.n_sink = (int)n_sink;
  p.sink_pad = (int)sink_pad;
  p.ring = (int)ring;
  p.window = (int)window;
  p.num_splits = 1;
  TORCH_CHECK(p.bs % 32 == 0, "cache block size must be a multiple of 32");
  return p;
}

void attn_decode(Tensor out, Tensor q, optional<Tensor> q_sink, Tensor k_cache, Tensor v_cache,
                 Tensor block_tables, Tensor seq_lens, double scale, int64_t n_sink,
                 int64_t sink_pad, int64_t ring, int64_t window, int64_t num_splits,
                 optional<Tensor> part_o, optional<Tensor> part_ml, double k_scale,
                 double v_scale, optional<Tensor> out_q, optional<Tensor> out_mx) {
  int64_t D = 0;
  auto p = attn_common(out, q, q_sink, k_cache, v_cache, block_tables, seq_lens, scale, n_sink,
                       sink_pad, ring, window, k_scale, v_scale, D, out_q.has_value());
  const int64_t B = q.size(0);
  TORCH_CHECK(seq_lens.numel() == B, "decode: one token per sequence (seq_lens must have T entries)");
  TORCH_CHECK(num_splits >= 1, "num_splits >= 1");
  p.num_splits = (int)num_splits;
  TORCH_CHECK(out_q.has_value() == out_mx.has_value(), "attn_decode: out_q and out_mx go together");
  if (out_q.has_value()) {   // MX fp8 output for the fp8 O projection
    CHECK_IN(*out_q); CHECK_IN(*out_mx);
    TORCH_CHECK(D == 128 && num_splits == 1, "attn_decode: MX output needs head_dim 128, one split");
    TORCH_CHECK(out_q->element_size() == 1 && out_q->numel() == B * p.nh * D,
                "attn_decode: out_q = fp8 [T, nh * D]");
    TORCH_CHECK(out_mx->element_size() == 1 && out_mx->numel() == p.nh * ((B + 63) / 64) * 64,
                "attn_decode: out_mx = e8m0 [nh][ceil(T / 64) * 64]");
    p.out_q = static_cast<uint8_t*>(out_q->data_ptr());
    p.out_mx = static_cast<uint8_t*>(out_mx->data_ptr());
  }
  if (num_splits > 1) {
    TORCH_CHECK(part_o.has_value() && part_ml.has_value(), "split-K needs workspaces");
    CHECK_IN(*part_o); CHECK_IN(*part_ml); CHECK_F32(*part_o); CHECK_F32(*part_ml);
    TORCH_CHECK(part_o->numel() >= num_splits * B * p.nh * D, "part_o workspace too small");
    TORCH_CHECK(part_ml->numel() >= num_splits * B * p.nh * 2, "part_ml workspace too small");
    p.part_o = part_o->data_ptr<float>();
    p.part_ml = part_ml->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  check_rc(dli::launch_attn_decode(p, (int)B, (int)D, cur_stream()), "attn_decode");
}

void attn_prefill(Tensor out, Tensor q, optional<Tensor> q_sink, Tensor k_cache, Tensor v_cache,
                  Tensor block_tables, Tensor seq_lens, Tensor q_start, int64_t max_q,
                  double scale, int64_t n_sink, int64_t sink_pad, int64_t ring, int64_t window,
                  double k_scale, double v_scale, optional<Tensor> tile_map, int64_t qb,
                  optional<Tensor> mask, bool m32) {
  int64_t D = 0;
  auto p = attn_common(out, q, q_sink, k_cache, v_cache, block_tables, seq_lens, scale, n_sink,
                       sink_pad, ring, window, k_scale, v_scale, D);
  CHECK_IN(q_start); CHECK_I32(q_start);
  const int64_t B = seq_lens.numel();
  TORCH_CHECK(q_start.numel() == B + 1, "q_start must have B+1 entries");
  p.q_start = q_start.data_ptr<int>();
  if (tile_map.has_value()) {
    CHECK_IN(*tile_map); CHECK_I32(*tile_map);
    TORCH_CHECK(tile_map->dim() == 2 && tile_map->size(1) == 2, "tile_map must be [n_tiles, 2]");
    p.tile_map = tile_map->data_ptr<int>();
    p.n_tiles = (int)tile_map->size(0);
  }
  TORCH_CHECK(qb == 1 || qb == 2, "attn_prefill: qb (query blocks per wave) must be 1 or 2");
  p.prefill_qb = (int)qb;
  p.prefill_m32 = m32 ? 1 : 0;
  if (mask.has_value()) {   // reference 4-D additive mask [B, 1 | nh, Tm, Km], fp32
    CHECK_IN(*mask); CHECK_F32(*mask);
    TORCH_CHECK(mask->dim() == 4 && mask->size(0) == B &&
                    (mask->size(1) == 1 || mask->size(1) == q.size(1)),
                "attn_prefill: mask must be [B, 1 | nh, T, keys]");
    TORCH_CHECK(ring == 0 && !tile_map.has_value(),
                "attn_prefill: a custom mask needs a full cache and the dense grid");
    p.mask = mask->data_ptr<float>();
    p.mask_heads = (int)mask->size(1);
    p.mask_q = (int)mask->size(2);
    p.mask_k = (int)mask->size(3);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(q.device());
  check_rc(dli::launch_attn_prefill(p, (int)B, (int)max_q, (int)D, cur_stream()), "attn_prefill");
}

// ------------------------------------------------------------------------------ sampling
void sample(Tensor out_tokens, optional<Tensor> out_logprobs, Tensor logits,
            optional<Tensor> temperature, optional<Tensor> top_k, optional<Tensor> top_p,
            optional<Tensor> seeds, optional<Tensor> step, optional<Tensor> ctr) {
  CHECK_DEV(logits);
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits must be [B, V] row-major");
  TORCH_CHECK(logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat,
              "logits must be bf16 or f32");
  const int64_t B = logits.size(0);
  CHECK_IN(out_tokens); CHECK_I32(out_tokens);
  TORCH_CHECK(out_tokens.numel() == B, "out_tokens must have B entries");
  dli::SampleParams p{};
  p.logits = logits.data_ptr();
  p.logits_is_f32 = logits.scalar_type() == at::kFloat;
  p.row_stride = logits.stride(0);
  p.V = (int)logits.size(1);
  auto opt_f = [&](optional<Tensor>& t, const char* n) -> const float* {
    if (!t.has_value()) return nullptr;
    CHECK_IN(*t); CHECK_F32(*t);
    TORCH_CHECK(t->numel() == B, n, " must have B entries");
    return t->data_ptr<float>();
  };
  p.temperature = opt_f(temperature, "temperature");
  p.top_p = opt_f(top_p, "top_p");
  if (top_k.has_value()) {
    CHECK_IN(*top_k); CHECK_I32(*top_k);
    TORCH_CHECK(top_k->numel() == B, "top_k must have B entries");
    p.top_k = top_k->data_ptr<int>();
  }
  if (seeds.has_value()) {
    CHECK_IN(*seeds); CHECK_I64(*seeds);
    TORCH_CHECK(seeds->numel() == B, "seeds must have B entries");
    p.seeds = reinterpret_cast<const unsigned long long*>(seeds->data_ptr<int64_t>());
  }
  if (step.has_value()) {
    CHECK_IN(*step); CHECK_I64(*step);
    p.step = reinterpret_cast<const long*>(step->data_ptr<int64_t>());
  }
  if (ctr.has_value()) {
    CHECK_IN(*ctr); CHECK_I64(*ctr);
    TORCH_CHECK(ctr->numel() == B, "ctr must have B entries");
    p.ctr = reinterpret_cast<const long*>(ctr->data_ptr<int64_t>());
  }
  p.out_tokens = out_tokens.data_ptr<int>();
  if (out_logprobs.has_value()) {
    CHECK_IN(*out_logprobs); CHECK_F32(*out_logprobs);
    TORCH_CHECK(out_logprobs->numel() == B, "out_logprobs must have B entries");
    p.out_logprobs = out_logprobs->data_ptr<float>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(logits.device());
  check_rc(dli::launch_sample(p, (int)B, cur_stream()), "sample");
}

// ------------------------------------------------------------------------------ fp8 quant
void quant_rowwise(Tensor q_out, Tensor scale, Tensor x, optional<Tensor> residual,
                   optional<Tensor> norm_w, double eps, optional<Tensor> residual_out) {
  CHECK_IN(q_out); CHECK_IN(scale); CHECK_IN(x); CHECK_F32(scale);
  // x: bf16 [rows, K], or split-K partials [S, rows, K] summed on load (fp32, or bf16 from the
  // fp8 path's gemm_tile epilogue 4)
  const bool parts_bf16 = x.scalar_type() == at::kBFloat16 && x.dim() == 3;
  const bool parts = x.scalar_type() == at::kFloat || parts_bf16;
  if (parts) {
    TORCH_CHECK(x.dim() == 3, "quant: partials must be [S, rows, K]");
  } else {
    CHECK_BF16(x);
  }
  TORCH_CHECK(q_out.element_size() == 1, "q_out must be an 8-bit tensor");
  const int64_t K = x.size(-1);
  const int64_t n = parts ? x.numel() / x.size(0) : x.numel();
  const int64_t rows = n / K;
  TORCH_CHECK(q_out.numel() == n && scale.numel() == rows, "quant: shape mismatch");
  const dli::bf16* ri = nullptr;
  dli::bf16* ro = nullptr;
  if (residual.has_value()) {
    CHECK_IN(*residual); CHECK_BF16(*residual);
    TORCH_CHECK(residual->numel() == n, "quant: residual shape mismatch");
    ri = bp(*residual);
    ro = bp(*residual);
    if (residual_out.has_value()) {
      CHECK_IN(*residual_out); CHECK_BF16(*residual_out);
      TORCH_CHECK(residual_out->numel() == n, "quant: residual_out shape mismatch");
      ro = bp(*residual_out);
    }
  }
  const dli::bf16* w = nullptr;
  if (norm_w.has_value()) {
    CHECK_IN(*norm_w); CHECK_BF16(*norm_w);
    TORCH_CHECK(norm_w->numel() == K, "quant: norm weight shape mismatch");
    w = bp(*norm_w);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_quant_rowwise(reinterpret_cast<uint8_t*>(q_out.data_ptr()),
                                     scale.data_ptr<float>(), parts ? nullptr : bp(x), ri, ro, w,
                                     (float)eps, (int)rows, (int)K, cur_stream(),
                                     parts ? x.data_ptr() : nullptr,
                                     parts ? (int)x.size(0) : 0, parts_bf16),
           "quant_rowwise");
}

// Payload digest partials of the hop-integrity check (parallel/integrity.py): part [nblocks, 2]
// int64 receives per-workgroup sums over t's 32-bit words; the host folds them (mod 2^64).
void digest(Tensor part, Tensor t) {
  CHECK_DEV(t); CHECK_CONTIG(t); CHECK_IN(part); CHECK_I64(part);
  const int64_t nbytes = t.numel() * t.element_size();
  TORCH_CHECK(nbytes % 4 == 0, "digest: payload must be a whole number of 32-bit words");
  TORCH_CHECK(part.dim() == 2 && part.size(1) == 2 && part.size(0) >= 1, "digest: part must be [nblocks, 2]");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(t.device());
  check_rc(dli::launch_digest(t.data_ptr(), (long)(nbytes / 4), part.data_ptr<int64_t>(),
                              (int)part.size(0), cur_stream()), "digest");
}

void quant_rowwise_int8(Tensor q_out, Tensor scale, Tensor x, optional<Tensor> outlier) {
  CHECK_IN(q_out); CHECK_IN(scale); CHECK_IN(x); CHECK_BF16(x); CHECK_F32(scale);
  TORCH_CHECK(q_out.scalar_type() == at::kChar, "q_out must be int8");
  TORCH_CHECK(x.dim() == 2, "quant_rowwise_int8: x must be [rows, K]");
  const int64_t rows = x.size(0), K = x.size(1);
  TORCH_CHECK(q_out.numel() == x.numel() && scale.numel() == rows, "quant_rowwise_int8: shape mismatch");
  const uint8_t* f = nullptr;
  if (outlier.has_value()) {
    CHECK_IN(*outlier);
    TORCH_CHECK(outlier->element_size() == 1 && outlier->numel() == K,
                "quant_rowwise_int8: outlier must be K bytes");
    f = reinterpret_cast<const uint8_t*>(outlier->data_ptr());
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_quant_rowwise_int8(reinterpret_cast<int8_t*>(q_out.data_ptr()),
                                          scale.data_ptr<float>(), bp(x), f, (int)rows, (int)K,
                                          cur_stream()),
           "quant_rowwise_int8");
}

// LLM.int8 outlier columns of x [M, K] against int8 weights wq [N, K] (scale ws [N]): returns
// (flags uint8 [K], x_out bf16 [M, max_out], w_out bf16 [N, max_out]) with x_out . w_out^T the
// bf16 outlier product (padding columns are zero).  Four kernels, static shapes, no host sync.
// Returns (flags [K] u8, x_out [M, max_out], w_out [N, max_out], cnt [1] i32 = columns kept).
// dynamic: the gathers write only the first ceil(cnt / 32) 32-column chunks of x_out / w_out (the
// rest is left unwritten) -- for the int8 tile GEMM, which given `cnt` reads no further.
std::vector<Tensor> llm_int8_outliers(Tensor x, Tensor wq, Tensor ws, double threshold,
                                      int64_t max_out, optional<Tensor> wq_t, bool dynamic) {
  CHECK_IN(x); CHECK_BF16(x); CHECK_IN(wq); CHECK_IN(ws); CHECK_F32(ws);
  TORCH_CHECK(wq.scalar_type() == at::kChar, "llm_int8_outliers: wq must be int8");
  TORCH_CHECK(x.dim() == 2 && wq.dim() == 2 && wq.size(1) == x.size(1) && ws.numel() == wq.size(0),
              "llm_int8_outliers: shape mismatch");
  const int64_t M = x.size(0), K = x.size(1), N = wq.size(0);
  TORCH_CHECK(K % 8 == 0 && max_out > 0 && max_out <= K, "llm_int8_outliers: K % 8 and 0 < max_out <= K");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  auto o = x.options();
  Tensor colmax = at::empty({K}, o.dtype(at::kFloat));
  Tensor idx = at::empty({max_out}, o.dtype(at::kLong));
  Tensor sel = at::empty({max_out}, o.dtype(at::kFloat));
  Tensor flags = at::empty({K}, o.dtype(at::kByte));
  Tensor xo = at::empty({M, max_out}, o);
  Tensor wo = at::empty({N, max_out}, o);
  Tensor cnt = at::empty({1}, o.dtype(at::kInt));
  const int* dyn = dynamic ? cnt.data_ptr<int>() : nullptr;
  hipStream_t st = cur_stream();
  check_rc(dli::launch_llm_int8_colmax(colmax.data_ptr<float>(), bp(x), (int)M, (int)K, st),
           "llm_int8_colmax");
  check_rc(dli::launch_llm_int8_select(colmax.data_ptr<float>(), (int)K, (float)threshold,
                                       (int)max_out, idx.data_ptr<int64_t>(), sel.data_ptr<float>(),
                                       flags.data_ptr<uint8_t>(), st, cnt.data_ptr<int>()),
           "llm_int8_select");
  check_rc(dli::launch_llm_int8_gather_x(bp(xo), bp(x), idx.data_ptr<int64_t>(),
                                         sel.data_ptr<float>(), (int)M, (int)K, (int)max_out, st,
                                         dyn),
           "llm_int8_gather_x");
  if (wq_t.has_value()) {   // transposed copy [K, N]: coalesced column gather
    CHECK_IN((*wq_t));
    TORCH_CHECK(wq_t->scalar_type() == at::kChar && wq_t->dim() == 2 && wq_t->size(0) == K &&
                    wq_t->size(1) == N, "llm_int8_outliers: wq_t must be int8 [K, N]");
    check_rc(dli::launch_llm_int8_gather_wt(bp(wo), reinterpret_cast<const int8_t*>(wq_t->data_ptr()),
                                            ws.data_ptr<float>(), idx.data_ptr<int64_t>(),
                                            sel.data_ptr<float>(), (int)N, (int)max_out, st, dyn),
             "llm_int8_gather_wt");
  } else {
    check_rc(dli::launch_llm_int8_gather_w(bp(wo), reinterpret_cast<const int8_t*>(wq.data_ptr()),
                                           ws.data_ptr<float>(), idx.data_ptr<int64_t>(),
                                           sel.data_ptr<float>(), (int)N, (int)K, (int)max_out, st,
                                           dyn),
             "llm_int8_gather_w");
  }
  return {flags, xo, wo, cnt};
}

void silu_mul_quant(Tensor q_out, Tensor scale, Tensor x) {
  CHECK_IN(q_out); CHECK_IN(scale); CHECK_IN(x); CHECK_BF16(x); CHECK_F32(scale);
  TORCH_CHECK(q_out.element_size() == 1, "q_out must be an 8-bit tensor");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 2 == 0, "silu_mul_quant: x must be [rows, 2I]");
  const int64_t rows = x.size(0), I = x.size(1) / 2;
  TORCH_CHECK(q_out.numel() == rows * I && scale.numel() == rows, "silu_mul_quant: shape mismatch");
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_silu_mul_quant(reinterpret_cast<uint8_t*>(q_out.data_ptr()),
                                      scale.data_ptr<float>(), bp(x), (int)rows, (int)I,
                                      cur_stream()),
           "silu_mul_quant");
}

// ------------------------------------------------------------------------------ tile GEMM
// epilogue 0: out = A . B^T (bf16); 2: out[:, n] = silu(g) * u with B rows interleaved by
// ops.swiglu_interleave (out has N / 2 columns).  splits > 1 (epilogue 0 only) needs an fp32
// workspace of splits * M * N.  fp8: A, B are e4m3 bytes with a_scale [M] and b_scale [N] (fp32,
// both required); out = (A . B^T) * a_scale[:, None] * b_scale[None, :].
void gemm_tile(Tensor out, Tensor a, Tensor b, int64_t splits, int64_t epilogue,
               optional<Tensor> workspace, optional<Tensor> a_scale, optional<Tensor> b_scale,
               optional<Tensor> x_out, optional<Tensor> w_out, optional<Tensor> a_mx,
               optional<Tensor> out_mx, optional<Tensor> ol_cnt) {
  CHECK_IN(out); CHECK_IN(a); CHECK_IN(b);
  TORCH_CHECK(epilogue == 3 ? out.element_size() == 1 : out.scalar_type() == at::kBFloat16,
              "gemm_tile: bf16 output (fp8 bytes for epilogue 3)");
  const bool bf16_parts = epilogue == 4;   // bf16 split-K partials into out [S, M, N]
  const bool fp8 = a.element_size() == 1;   // 1-byte operands: fp8 e4m3 or int8
  TORCH_CHECK(a.scalar_type() == b.scalar_type(), "gemm_tile: a and b must share a dtype");
  TORCH_CHECK(fp8 || a.scalar_type() == at::kBFloat16, "gemm_tile: bf16, fp8 (e4m3) or int8 operands");
  int precision = !fp8 ? 0 : (a.scalar_type() == at::kChar ? 2 : 1);
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2 && (out.dim() == 2 || bf16_parts), "gemm_tile: 2-D tensors");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K && (bf16_parts || out.size(0) == M), "gemm_tile: shape mismatch");
  TORCH_CHECK(epilogue >= 0 && epilogue <= 4,
              "gemm_tile: epilogue must be 0 (store), 1 (split-K partials only), 2 (swiglu), 3 "
              "(swiglu -> fp8 with MX scales) or 4 (bf16 split-K partials)");
  TORCH_CHECK(epilogue == 1 || bf16_parts || out.size(1) == (epilogue >= 2 ? N / 2 : N),
              "gemm_tile: output columns");
  TORCH_CHECK(!bf16_parts || (splits > 1 && out.is_contiguous() && out.numel() == splits * M * N),
              "gemm_tile: epilogue 4 = splits > 1, out [splits, M, N] bf16");
  // fp8 MX activations: e8m0 scale per (row, 128-column block), layout of gemm_tile.hip mx_off
  const int64_t nb = (M + 63) / 64;
  const uint8_t* amx = nullptr;
  uint8_t* omx = nullptr;
  if (a_mx.has_value()) {
    CHECK_IN(*a_mx);
    TORCH_CHECK(precision == 1 && a_mx->element_size() == 1 && a_mx->numel() == (K / 128) * nb * 64,
                "gemm_tile: a_mx = fp8 A's e8m0 scales [K / 128][ceil(M / 64) * 64]");
    amx = static_cast<const uint8_t*>(a_mx->data_ptr());
    precision = 3;
  }
  if (epilogue == 3) {
    TORCH_CHECK(precision == 1 && splits == 1 && out_mx.has_value(),
                "gemm_tile: epilogue 3 needs fp8 operands with per-row scales, splits 1, out_mx");
    CHECK_IN(*out_mx);
    TORCH_CHECK(out_mx->element_size() == 1 && out_mx->numel() == (N / 2 / 128) * nb * 64,
                "gemm_tile: out_mx = [N / 256][ceil(M / 64) * 64] bytes");
    omx = static_cast<uint8_t*>(out_mx->data_ptr());
  }
  TORCH_CHECK(epilogue != 1 || splits > 1, "gemm_tile: epilogue 1 (partials only) needs splits > 1");
  const int64_t kt = K * a.element_size() / 128;
  TORCH_CHECK(M >= 1 && M <= (1 << 20) && N % 256 == 0 && (K * a.element_size()) % 128 == 0 && K > 0,
              "gemm_tile: needs N % 256 == 0 and 128-byte multiples of K");
  TORCH_CHECK(splits >= 0 && splits <= kt, "gemm_tile: 0 (stream-K tail) <= splits <= k-tiles");
  const float* sa = nullptr;
  const float* sb = nullptr;
  if (fp8) {
    TORCH_CHECK((a_scale.has_value() || precision == 3) && b_scale.has_value(),
                "gemm_tile: 8-bit needs a_scale (or a_mx) and b_scale");
    CHECK_IN(*b_scale); CHECK_F32(*b_scale);
    TORCH_CHECK(b_scale->numel() == N, "gemm_tile: scale sizes");
    sb = b_scale->data_ptr<float>();
    if (precision != 3) {
      CHECK_IN(*a_scale); CHECK_F32(*a_scale);
      TORCH_CHECK(a_scale->numel() == M, "gemm_tile: scale sizes");
      sa = a_scale->data_ptr<float>();
    }
  }
  float* ws = nullptr;
  if (splits == 0) {
    TORCH_CHECK(workspace.has_value(), "gemm_tile: the stream-K tail needs a workspace");
    CHECK_IN(*workspace); CHECK_F32(*workspace);
    const c10::hip::HIPGuardMasqueradingAsCUDA g0(a.device());
    TORCH_CHECK(workspace->numel() >= dli::gemm_tile_sk_workspace_floats(),
                "gemm_tile: stream-K workspace too small");
    ws = workspace->data_ptr<float>();
  } else if (splits > 1 && !bf16_parts) {
    TORCH_CHECK(epilogue != 2, "gemm_tile: split-K only with the store / partials epilogues");
    TORCH_CHECK(workspace.has_value(), "gemm_tile: split-K needs a workspace");
    CHECK_IN(*workspace); CHECK_F32(*workspace);
    TORCH_CHECK(workspace->numel() >= splits * M * N, "gemm_tile: workspace too small");
    ws = workspace->data_ptr<float>();
  }
  // LLM.int8 outlier columns (int8 only): out += x_out [M, J] . w_out [N, J]^T in the epilogue
  const dli::bf16* xo = nullptr;
  const dli::bf16* wo = nullptr;
  int J = 0;
  TORCH_CHECK(x_out.has_value() == w_out.has_value(), "gemm_tile: x_out and w_out go together");
  if (x_out.has_value()) {
    TORCH_CHECK(precision == 2, "gemm_tile: outlier columns are an int8 (LLM.int8) feature");
    CHECK_IN(*x_out); CHECK_IN(*w_out); CHECK_BF16(*x_out); CHECK_BF16(*w_out);
    TORCH_CHECK(x_out->dim() == 2 && w_out->dim() == 2 && x_out->size(0) == M &&
                w_out->size(0) == N && x_out->size(1) == w_out->size(1),
                "gemm_tile: x_out [M, J], w_out [N, J]");
    J = (int)x_out->size(1);
    TORCH_CHECK(J % 32 == 0, "gemm_tile: J (outlier columns) must be a multiple of 32");
    xo = bp(*x_out);
    wo = bp(*w_out);
  }
  const int* olc = nullptr;   // live outlier columns (llm_int8_outliers(..., dynamic=True))
  if (ol_cnt.has_value()) {
    CHECK_IN(*ol_cnt);
    TORCH_CHECK(x_out.has_value() && ol_cnt->scalar_type() == at::kInt && ol_cnt->numel() == 1,
                "gemm_tile: ol_cnt = int32 [1] count of the live outlier columns (with x_out)");
    olc = ol_cnt->data_ptr<int>();
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  check_rc(dli::launch_gemm_tile(out.data_ptr(), a.data_ptr(), b.data_ptr(), sa, sb, ws, (int)M,
                                 (int)N, (int)K, (int)splits, (int)epilogue, precision, cur_stream(),
                                 xo, wo, J, amx, omx, olc),
           "gemm_tile");
}

// one-wave-per-SIMD tile GEMM (gemm4.hip), bf16: epilogue 0 = bf16 [M, N], 2 = SwiGLU [M, N/2]
// (splits 1); 1 = fp32 partials, 4 = bf16 partials [splits, M, N] (splits > 1)
// fp8 e4m3 operands (1-byte a / b) take per-row a_scale [M] and per-channel b_scale [N] (fp32)
void gemm4(Tensor out, Tensor a, Tensor b, int64_t splits, int64_t epilogue, int64_t grid,
           optional<Tensor> a_scale, optional<Tensor> b_scale, int64_t variant,
           optional<Tensor> a_mx, optional<Tensor> out_mx) {
  CHECK_IN(out); CHECK_IN(a); CHECK_IN(b);
  const bool fp8 = a.element_size() == 1;
  TORCH_CHECK(a.scalar_type() == b.scalar_type() && a.scalar_type() != at::kChar,
              "gemm4: bf16 or fp8 e4m3 operands of one dtype");
  if (!fp8) { CHECK_BF16(a); }
  TORCH_CHECK(a.dim() == 2 && b.dim() == 2, "gemm4: 2-D operands");
  const int64_t M = a.size(0), K = a.size(1), N = b.size(0);
  TORCH_CHECK(b.size(1) == K, "gemm4: shape mismatch");
  const int64_t nb = (M + 63) / 64;
  const float* sa = nullptr;
  const float* sb = nullptr;
  const uint8_t* amx = nullptr;
  uint8_t* omx = nullptr;
  int precision = 0;
  if (fp8) {
    TORCH_CHECK(b_scale.has_value(), "gemm4: fp8 needs b_scale");
    CHECK_IN(*b_scale); CHECK_F32(*b_scale);
    TORCH_CHECK(b_scale->numel() == N, "gemm4: b_scale [N]");
    sb = b_scale->data_ptr<float>();
    if (a_mx.has_value()) {   // MX activations: e8m0 per (row, 128-column block)
      CHECK_IN(*a_mx);
      TORCH_CHECK(a_mx->element_size() == 1 && a_mx->numel() == (K / 128) * nb * 64,
                  "gemm4: a_mx = e8m0 [K / 128][ceil(M / 64) * 64] (mx_off layout)");
      amx = static_cast<const uint8_t*>(a_mx->data_ptr());
      precision = 2;
    } else {
      TORCH_CHECK(a_scale.has_value(), "gemm4: fp8 needs a_scale (or a_mx)");
      CHECK_IN(*a_scale); CHECK_F32(*a_scale);
      TORCH_CHECK(a_scale->numel() == M, "gemm4: a_scale [M]");
      sa = a_scale->data_ptr<float>();
      precision = 1;
    }
  }
  int64_t want = 0;
  if (epilogue == 0) want = M * N;
  else if (epilogue == 2 || epilogue == 3) want = M * (N / 2);
  else if (epilogue == 1 || epilogue == 4) want = splits * M * N;
  else TORCH_CHECK(false, "gemm4: epilogue 0, 1, 2, 3 or 4");
  const auto odt = out.scalar_type();
  TORCH_CHECK(out.is_contiguous() && out.numel() == want &&
              (epilogue == 3 ? out.element_size() == 1
                             : odt == (epilogue == 1 ? at::kFloat : at::kBFloat16)),
              "gemm4: output size / dtype");
  if (epilogue == 3) {
    TORCH_CHECK(precision == 1 && splits == 1, "gemm4: the MX SwiGLU epilogue takes per-row fp8, one split");
    TORCH_CHECK(out_mx.has_value(), "gemm4: epilogue 3 needs out_mx");
    CHECK_IN(*out_mx);
    TORCH_CHECK(out_mx->element_size() == 1 && out_mx->numel() == (N / 2 / 128) * nb * 64,
                "gemm4: out_mx = e8m0 [N / 256][ceil(M / 64) * 64]");
    omx = static_cast<uint8_t*>(out_mx->data_ptr());
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(a.device());
  check_rc(dli::launch_gemm4(out.data_ptr(), a.data_ptr(), b.data_ptr(), (int)M, (int)N, (int)K,
                             (int)splits, (int)epilogue, (int)grid, cur_stream(), (int)variant,
                             precision, sa, sb, amx, omx),
           "gemm4");
}

// ------------------------------------------------------------------------------ skinny GEMM
// fused input RMSNorm of a skinny GEMM's rows: norm_w given -> x' = rmsnorm(x + res_in) * norm_w
struct GemvNormArgs {
  dli::GemvNorm nm{};
  bool on = false;
};
static GemvNormArgs gemv_norm_args(const Tensor& x, const optional<Tensor>& norm_w,
                                   const optional<Tensor>& res_in, const optional<Tensor>& res_out,
                                   double eps, const char* what) {
  GemvNormArgs a;
  if (!norm_w.has_value()) {
    TORCH_CHECK(!res_in.has_value() && !res_out.has_value(), what, ": residuals need norm_w");
    return a;
  }
  CHECK_IN(*norm_w); CHECK_BF16(*norm_w); CHECK_BF16(x);
  TORCH_CHECK(norm_w->numel() == x.size(1) && x.size(0) <= 2, what, ": norm_w [K], M <= 2");
  a.on = true;
  a.nm.w = bp(*norm_w);
  a.nm.eps = (float)eps;
  if (res_in.has_value()) {
    CHECK_IN(*res_in); CHECK_BF16(*res_in);
    TORCH_CHECK(res_in->sizes() == x.sizes(), what, ": res_in shape");
    a.nm.res_in = bp(*res_in);
  }
  if (res_out.has_value()) {
    CHECK_IN(*res_out); CHECK_BF16(*res_out);
    TORCH_CHECK(res_out->sizes() == x.sizes() && res_in.has_value(), what, ": res_out needs res_in");
    TORCH_CHECK(res_out->data_ptr() != res_in->data_ptr(), what, ": res_out must not alias res_in");
    a.nm.res_out = bp(*res_out);
  }
  return a;
}

// swiglu: w is a swiglu_interleave'd gate|up weight [2I, K]; out = silu(gate) * up [M, I]
static int64_t gemv_out_cols(int64_t N, bool swiglu, const char* what) {
  TORCH_CHECK(!swiglu || N % 32 == 0, what, ": swiglu needs 32 | N");
  return swiglu ? N / 2 : N;
}

void skinny_gemm(Tensor out, Tensor x, Tensor w, optional<Tensor> bias, bool swiglu,
                 optional<Tensor> norm_w, optional<Tensor> res_in, optional<Tensor> res_out,
                 double eps) {
  const GemvNormArgs na = gemv_norm_args(x, norm_w, res_in, res_out, eps, "skinny_gemm");
  CHECK_IN(out); CHECK_IN(x); CHECK_IN(w);
  CHECK_BF16(out); CHECK_BF16(x); CHECK_BF16(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_gemm: 2-D tensors");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M && out.size(1) == gemv_out_cols(N, swiglu, "skinny_gemm"),
              "skinny_gemm: shape mismatch");
  TORCH_CHECK(!swiglu || M <= 2, "skinny_gemm: swiglu for M <= 2");
  TORCH_CHECK(M >= 1 && M <= 4 && K % 8 == 0, "skinny_gemm: M in [1, 4], K % 8 == 0");
  const dli::bf16* b = nullptr;
  if (bias.has_value()) {
    CHECK_IN(*bias); CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N, "skinny_gemm: bias must have N entries");
    b = bp(*bias);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_skinny_gemm(bp(out), bp(x), bp(w), b, (int)M, (int)N, (int)K,
                                   cur_stream(), swiglu, na.on ? &na.nm : nullptr), "skinny_gemm");
}

// int8 weights [N, K] with fp32 per-row scales [N], bf16 activations (weight-only dequantisation)
void skinny_gemm_int8(Tensor out, Tensor x, Tensor w, Tensor wscale, optional<Tensor> bias,
                      bool swiglu, optional<Tensor> norm_w, optional<Tensor> res_in,
                      optional<Tensor> res_out, double eps) {
  const GemvNormArgs na = gemv_norm_args(x, norm_w, res_in, res_out, eps, "skinny_gemm_int8");
  CHECK_IN(out); CHECK_IN(x); CHECK_IN(w); CHECK_IN(wscale);
  CHECK_BF16(out); CHECK_BF16(x); CHECK_F32(wscale);
  TORCH_CHECK(w.scalar_type() == at::kChar, "skinny_gemm_int8: int8 weights");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_gemm_int8: 2-D tensors");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M &&
              out.size(1) == gemv_out_cols(N, swiglu, "skinny_gemm_int8") && wscale.numel() == N,
              "skinny_gemm_int8: shape mismatch");
  TORCH_CHECK(M >= 1 && M <= 2 && K % 16 == 0, "skinny_gemm_int8: M in [1, 2], K % 16 == 0");
  const dli::bf16* b = nullptr;
  if (bias.has_value()) {
    CHECK_IN(*bias); CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N, "skinny_gemm_int8: bias must have N entries");
    b = bp(*bias);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_skinny_gemm_int8(bp(out), bp(x), w.data_ptr<int8_t>(),
                                        wscale.data_ptr<float>(), b, (int)M, (int)N, (int)K,
                                        cur_stream(), swiglu, na.on ? &na.nm : nullptr),
           "skinny_gemm_int8");
}

// fp8 e4m3 weights [N, K] (1-byte storage), fp32 per-row scales [N]; activations bf16, or fp8
// [M, K] with fp32 per-row scales xscale [M] (the fused RMSNorm quantiser's output)
void skinny_gemm_fp8(Tensor out, Tensor x, optional<Tensor> xscale, Tensor w, Tensor wscale,
                     optional<Tensor> bias, bool swiglu, optional<Tensor> norm_w,
                     optional<Tensor> res_in, optional<Tensor> res_out, double eps) {
  const GemvNormArgs na = gemv_norm_args(x, norm_w, res_in, res_out, eps, "skinny_gemm_fp8");
  TORCH_CHECK(!na.on || !xscale.has_value(), "skinny_gemm_fp8: the fused norm takes bf16 rows");
  CHECK_IN(out); CHECK_IN(x); CHECK_IN(w); CHECK_IN(wscale);
  CHECK_BF16(out); CHECK_F32(wscale);
  TORCH_CHECK(w.element_size() == 1, "skinny_gemm_fp8: 1-byte (fp8 e4m3) weights");
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && out.dim() == 2, "skinny_gemm_fp8: 2-D tensors");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == K && out.size(0) == M &&
              out.size(1) == gemv_out_cols(N, swiglu, "skinny_gemm_fp8") && wscale.numel() == N,
              "skinny_gemm_fp8: shape mismatch");
  TORCH_CHECK(M >= 1 && M <= 2 && K % 16 == 0, "skinny_gemm_fp8: M in [1, 2], K % 16 == 0");
  const float* xs = nullptr;
  if (xscale.has_value()) {
    CHECK_IN(*xscale); CHECK_F32(*xscale);
    TORCH_CHECK(x.element_size() == 1 && xscale->numel() == M,
                "skinny_gemm_fp8: fp8 activations need one scale per row");
    xs = xscale->data_ptr<float>();
  } else {
    CHECK_BF16(x);
  }
  const dli::bf16* b = nullptr;
  if (bias.has_value()) {
    CHECK_IN(*bias); CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N, "skinny_gemm_fp8: bias must have N entries");
    b = bp(*bias);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  check_rc(dli::launch_skinny_gemm_fp8(bp(out), x.data_ptr(), xs,
                                       static_cast<const uint8_t*>(w.data_ptr()),
                                       wscale.data_ptr<float>(), b, (int)M, (int)N, (int)K,
                                       cur_stream(), swiglu, na.on ? &na.nm : nullptr),
           "skinny_gemm_fp8");
}

// 1-2 decode rows: the fused QKV GEMV whose epilogue does rope_cache's work (q rotated into q_out,
// k rotated and v written into the paged caches), optionally with the fused input RMSNorm.
// w: bf16 [N, K], fp8 e4m3 / int8 [N, K] with fp32 per-row wscale; N = (nh + 2 nkv) D.
void skinny_gemm_qkv_rope(Tensor q_out, Tensor x, Tensor w, optional<Tensor> wscale,
                          optional<Tensor> bias, optional<Tensor> positions,
                          optional<Tensor> slot_mapping, optional<Tensor> cos_sin, Tensor k_cache,
                          Tensor v_cache, int64_t nh, int64_t nkv, double k_scale, double v_scale,
                          optional<Tensor> norm_w, optional<Tensor> res_in,
                          optional<Tensor> res_out, double eps) {
  CHECK_IN(q_out); CHECK_IN(x); CHECK_IN(w);
  CHECK_BF16(q_out); CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && q_out.dim() == 3, "skinny_gemm_qkv_rope: shapes");
  const int64_t M = x.size(0), K = x.size(1), N = w.size(0), D = q_out.size(2);
  TORCH_CHECK(M >= 1 && M <= 2 && w.size(1) == K && q_out.size(0) == M && q_out.size(1) == nh &&
                  N == (nh + 2 * nkv) * D,
              "skinny_gemm_qkv_rope: x [M <= 2, K], w [(nh + 2 nkv) D, K], q_out [M, nh, D]");
  const bool fp8 = check_cache(k_cache, v_cache, nkv, D);
  TORCH_CHECK(k_scale > 0 && v_scale > 0, "KV scales must be positive");
  dli::GemvRope rp{};
  rp.kv_fp8 = fp8 ? 1 : 0;
  rp.k_inv_scale = (float)(1.0 / k_scale);
  rp.v_inv_scale = (float)(1.0 / v_scale);
  if (positions.has_value()) {
    CHECK_IN(*positions); CHECK_I32(*positions);
    TORCH_CHECK(positions->numel() == M, "positions must have M entries");
    rp.positions = positions->data_ptr<int>();
  }
  if (slot_mapping.has_value()) {
    CHECK_IN(*slot_mapping); CHECK_I64(*slot_mapping);
    TORCH_CHECK(slot_mapping->numel() == M, "slot_mapping must have M entries");
    rp.slot_mapping = reinterpret_cast<const long*>(slot_mapping->data_ptr<int64_t>());
  }
  if (cos_sin.has_value()) {
    CHECK_IN(*cos_sin); CHECK_F32(*cos_sin);
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == D && positions.has_value(),
                "cos_sin must be [max_pos, D] (with positions)");
    rp.cos_sin = cos_sin->data_ptr<float>();
    rp.max_pos = (int)cos_sin->size(0);
  }
  rp.q_out = bp(q_out);
  rp.k_cache = k_cache.data_ptr();
  rp.v_cache = v_cache.data_ptr();
  rp.nh = (int)nh;
  rp.nkv = (int)nkv;
  rp.D = (int)D;
  rp.bs = (int)k_cache.size(2);
  const GemvNormArgs na = gemv_norm_args(x, norm_w, res_in, res_out, eps, "skinny_gemm_qkv_rope");
  const dli::GemvNorm* nm = na.on ? &na.nm : nullptr;
  const dli::bf16* b = nullptr;
  if (bias.has_value()) {
    CHECK_IN(*bias); CHECK_BF16(*bias);
    TORCH_CHECK(bias->numel() == N, "skinny_gemm_qkv_rope: bias must have N entries");
    b = bp(*bias);
  }
  const c10::hip::HIPGuardMasqueradingAsCUDA g(x.device());
  int rc;
  if (w.scalar_type() == at::kBFloat16) {
    rc = dli::launch_skinny_gemm(nullptr, bp(x), bp(w), b, (int)M, (int)N, (int)K, cur_stream(),
                                 false, nm, &rp);
  } else {
    TORCH_CHECK(wscale.has_value() && w.element_size() == 1, "8-bit weights need wscale");
    CHECK_IN(*wscale); CHECK_F32(*wscale);
    TORCH_CHECK(wscale->numel() == N, "wscale must have N entries");
    if (w.scalar_type() == at::kChar)
      rc = dli::launch_skinny_gemm_int8(nullptr, bp(x), w.data_ptr<int8_t>(),
                                        wscale->data_ptr<float>(), b, (int)M, (int)N, (int)K,
                                        cur_stream(), false, nm, &rp);
    else
      rc = dli::launch_skinny_gemm_fp8(nullptr, x.data_ptr(), nullptr,
                                       static_cast<const uint8_t*>(w.data_ptr()),
                                       wscale->data_ptr<float>(), b, (int)M, (int)N, (int)K,
                                       cur_stream(), false, nm, &rp);
  }
  check_rc(rc, "skinny_gemm_qkv_rope");
}


}  // namespace

void register_rccl(pybind11::module_& m);  // comm/rccl_p2p.hip
void register_streams(pybind11::module_& m);  // comm/streams.hip

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "CDNA4 (gfx950) kernels of distributed_llm_inference";
  m.def("rms_norm", &rms_norm, "RMSNorm (+fused residual add)", py::arg("out"), py::arg("x"),
        py::arg("residual"), py::arg("w"), py::arg("eps"), py::arg("residual_out") = py::none());
  m.def("layer_norm", &layer_norm, "LayerNorm (+fused residual add)", py::arg("out"),
        py::arg("x"), py::arg("residual"), py::arg("w"), py::arg("b"), py::arg("eps"),
        py::arg("residual_out") = py::none());
  m.def("silu_mul", &silu_mul, "SwiGLU: out = silu(x[:, :I]) * x[:, I:] (or tile-interleaved)",
        py::arg("out"), py::arg("x"), py::arg("interleaved") = false);
  m.def("gelu_bias", &gelu_bias, "gelu_tanh(x + bias)");
  m.def("add", &add, "out = a + b");
  m.def("rope_cache", &rope_cache, "fused RoPE + paged KV cache write");
  m.def("attn_decode", &attn_decode, "paged GQA decode attention (split-K)", py::arg("out"),
        py::arg("q"), py::arg("q_sink"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("block_tables"), py::arg("seq_lens"), py::arg("scale"), py::arg("n_sink"),
        py::arg("sink_pad"), py::arg("ring"), py::arg("window"), py::arg("num_splits"),
        py::arg("part_o"), py::arg("part_ml"), py::arg("k_scale"), py::arg("v_scale"),
        py::arg("out_q") = py::none(), py::arg("out_mx") = py::none());
  m.def("attn_prefill", &attn_prefill, "paged causal prefill attention (varlen)", py::arg("out"),
        py::arg("q"), py::arg("q_sink"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("block_tables"), py::arg("seq_lens"), py::arg("q_start"), py::arg("max_q"),
        py::arg("scale"), py::arg("n_sink"), py::arg("sink_pad"), py::arg("ring"),
        py::arg("window"), py::arg("k_scale"), py::arg("v_scale"), py::arg("tile_map"),
        py::arg("qb"), py::arg("mask") = py::none(), py::arg("m32") = true);
  m.def("sample", &sample, "greedy / temperature / top-k / top-p sampling", py::arg("out_tokens"),
        py::arg("out_logprobs"), py::arg("logits"), py::arg("temperature"), py::arg("top_k"),
        py::arg("top_p"), py::arg("seeds"), py::arg("step"), py::arg("ctr") = py::none());
  m.def("digest", &digest, "hop-integrity payload digest partials", py::arg("part"), py::arg("t"));
  m.def("quant_rowwise", &quant_rowwise, "row-wise fp8 e4m3 quantisation (+fused RMSNorm)",
        py::arg("q_out"), py::arg("scale"), py::arg("x"), py::arg("residual"), py::arg("norm_w"),
        py::arg("eps"), py::arg("residual_out") = py::none());
  m.def("quant_rowwise_int8", &quant_rowwise_int8, "LLM.int8 row-wise int8 quantisation (outlier columns zeroed)",
        py::arg("q_out"), py::arg("scale"), py::arg("x"), py::arg("outlier") = py::none());
  m.def("llm_int8_outliers", &llm_int8_outliers,
        "LLM.int8 outlier columns: (flags, x_out, w_out, cnt) for the bf16 outlier product",
        py::arg("x"), py::arg("wq"), py::arg("ws"), py::arg("threshold"), py::arg("max_out"),
        py::arg("wq_t") = py::none(), py::arg("dynamic") = false);
  m.def("silu_mul_quant", &silu_mul_quant, "SwiGLU fused with row-wise fp8 quantisation");
  m.def("gemm_tile", &gemm_tile, "C = A . B^T, 256x256 LDS-DMA 8-phase MFMA tile GEMM",
        py::arg("out"), py::arg("a"), py::arg("b"), py::arg("splits") = 1,
        py::arg("epilogue") = 0, py::arg("workspace") = py::none(),
        py::arg("a_scale") = py::none(), py::arg("b_scale") = py::none(),
        py::arg("x_out") = py::none(), py::arg("w_out") = py::none(),
        py::arg("a_mx") = py::none(), py::arg("out_mx") = py::none(),
        py::arg("ol_cnt") = py::none());
  m.def("rms_norm_splitk", &rms_norm_splitk, "residual add + RMSNorm over un-reduced split-K partials",
        py::arg("out"), py::arg("parts"), py::arg("residual"), py::arg("w"), py::arg("eps"),
        py::arg("residual_out") = py::none());
  m.def("splitk_reduce", &splitk_reduce, "bf16 out = sum of fp32 split-K partials [S, M, N]");
  m.def("gemm_tile_sk_workspace_floats", []() { return dli::gemm_tile_sk_workspace_floats(); },
        "fp32 workspace elements gemm_tile(splits=0) needs on the current device");
  m.def("skinny_gemm_qkv_rope", &skinny_gemm_qkv_rope,
        "1-2 row fused QKV GEMV with RoPE + paged KV write in its epilogue (+ fused input RMSNorm)",
        py::arg("q_out"), py::arg("x"), py::arg("w"), py::arg("wscale"), py::arg("bias"),
        py::arg("positions"), py::arg("slot_mapping"), py::arg("cos_sin"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("nh"), py::arg("nkv"), py::arg("k_scale") = 1.0,
        py::arg("v_scale") = 1.0, py::arg("norm_w") = py::none(), py::arg("res_in") = py::none(),
        py::arg("res_out") = py::none(), py::arg("eps") = 1e-5);
  m.def("gemm4", &gemm4, "C = A . B^T, one-wave-per-SIMD 256x256 MFMA tile GEMM (gemm4.hip)",
        py::arg("out"), py::arg("a"), py::arg("b"), py::arg("splits") = 1,
        py::arg("epilogue") = 0, py::arg("grid") = 0, py::arg("a_scale") = py::none(),
        py::arg("b_scale") = py::none(), py::arg("variant") = -1, py::arg("a_mx") = py::none(),
        py::arg("out_mx") = py::none());
  m.def("skinny_gemm_int8", &skinny_gemm_int8,
        "y = (x . W8^T) * scale (+ bias), int8 weights, bf16 rows, M <= 2 (weight-streaming GEMV)",
        py::arg("out"), py::arg("x"), py::arg("w"), py::arg("wscale"), py::arg("bias") = py::none(),
        py::arg("swiglu") = false, py::arg("norm_w") = py::none(), py::arg("res_in") = py::none(),
        py::arg("res_out") = py::none(), py::arg("eps") = 1e-5);
  m.def("skinny_gemm_fp8", &skinny_gemm_fp8,
        "y = (x . W8^T) * scale (+ bias), fp8 e4m3 weights, M <= 2 (weight-streaming GEMV)",
        py::arg("out"), py::arg("x"), py::arg("xscale"), py::arg("w"), py::arg("wscale"),
        py::arg("bias") = py::none(), py::arg("swiglu") = false, py::arg("norm_w") = py::none(),
        py::arg("res_in") = py::none(), py::arg("res_out") = py::none(), py::arg("eps") = 1e-5);
  m.def("skinny_gemm", &skinny_gemm, "y = x . W^T (+ bias) for M <= 4 (weight-streaming GEMV)",
        py::arg("out"), py::arg("x"), py::arg("w"), py::arg("bias") = py::none(),
        py::arg("swiglu") = false, py::arg("norm_w") = py::none(), py::arg("res_in") = py::none(),
        py::arg("res_out") = py::none(), py::arg("eps") = 1e-5);
  register_rccl(m);
  register_streams(m);
}
