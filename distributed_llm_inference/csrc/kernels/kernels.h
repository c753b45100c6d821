// Launch interface of the CDNA4 kernels (shared by the .hip kernel TUs and the torch bindings).
#pragma once
#include "common.h"

namespace dli {

struct AttnParams {
  const bf16* q;        // [T, nh, D]
  const bf16* q_sink;   // [T, nh, D] or nullptr (window mode only)
  const void* k_cache;  // [blocks, nkv, bs, D]           bf16, or fp8 e4m3 if kv_fp8
  const void* v_cache;  // [blocks, nkv, bs/8, D, 8]      (V^T in 8-key groups), same dtype
  int kv_fp8;           // caches hold fp8 e4m3: stored = x / scale
  float k_scale, v_scale;
  bf16* out;            // [T, nh, D]
  const int* block_tables;  // [B, bt_stride]
  int bt_stride;
  const int* seq_lens;  // [B] absolute length incl. this step's tokens
  const int* q_start;   // [B+1] prefill token offsets; nullptr for decode (token b == seq b)
  const int* tile_map;  // prefill: [n_tiles, 2] (sequence, token tile) work list, or nullptr
  int n_tiles;          //   (nullptr: dense grid over max_q x B)
  int prefill_qb = 1;   // prefill: 16-token query blocks per wave (1 or 2); a tile = 16 TPW QB tokens
  int prefill_m32 = 1;  // prefill: the 32x32x16-MFMA kernel (attn_prefill32.hip) where eligible
  float scale_log2;     // softmax scale * log2(e)
  int nh, nkv, bs;
  int n_sink, sink_pad, ring, window;  // window mode iff ring > 0
  float* part_o;        // [splits, T, nh, D]     (decode, num_splits > 1)
  float* part_ml;       // [splits, T, nh, 2]
  int num_splits;
  // decode, one split, D = 128: write the output as MX fp8 for the fp8 O projection instead of
  // bf16 -- e4m3 bytes [T, nh * D] and one e8m0 scale per (token, head) in mx_off layout
  uint8_t* out_q = nullptr;
  uint8_t* out_mx = nullptr;
  // prefill with the reference API's pre-inverted 4-D additive mask (full cache only):
  // fp32 [B, mask_heads (1 | nh), mask_q, mask_k]; query token t of sequence b uses row
  // mask_q - qlen_b + t (the last qlen_b rows), key k column k.  No causal mask is added.
  const float* mask = nullptr;
  int mask_heads = 0, mask_q = 0, mask_k = 0;
};

struct RopeCacheParams {
  const bf16* qkv;        // [T, qkv_stride]
  long qkv_stride;        // elements
  const int* positions;   // [T] rope positions
  const long* slot_mapping;  // [T]
  const float* cos_sin;   // [max_pos, D] (cos | sin) or nullptr (no rope, e.g. GPT-2)
  int max_pos;
  bf16* q_out;            // [T, nh, D]
  bf16* q_sink_out;       // [T, nh, D] or nullptr
  int window;             // > 0: q_sink rotated at min(pos, window-1)
  void* k_cache;          // [blocks, nkv, bs, D]        bf16, or fp8 e4m3 if kv_fp8
  void* v_cache;          // [blocks, nkv, bs/8, D, 8]
  int kv_fp8;
  float k_inv_scale, v_inv_scale;  // fp8: stored = x * inv_scale
  int nh, nkv, D, bs;
  // optional: qkv given as un-reduced fp32 split-K partials [splits, T, qkv_stride] of the QKV
  // tile GEMM (summed and rounded to bf16 on load, as the reduce pass would); qkv is unused then
  const void* qkv_parts;  // fp32, or bf16 with parts_bf16 (the fp8 path's gemm_tile epilogue 4)
  int parts_bf16;
  int splits;
  long split_stride;      // elements between consecutive partials (T * qkv_stride)
};

struct SampleParams {
  const void* logits;       // [B, row_stride] bf16 or f32
  int logits_is_f32;
  long row_stride;
  int V;
  const float* temperature; // [B]
  const int* top_k;         // [B] (<=0 or >=V: disabled)
  const float* top_p;       // [B] (>=1: disabled)
  const unsigned long long* seeds;  // [B]
  const long* step;         // [1] device counter (read only) or nullptr
  const long* ctr;          // [B] per-row counters (the sampled token's position in its
                            // sequence) or nullptr: then (step, row) key the randomness
  int* out_tokens;          // [B]
  float* out_logprobs;      // [B] or nullptr
};

int launch_rms_norm(bf16* out, const bf16* x, const bf16* residual_in, bf16* residual_out,
                    const bf16* w, float eps, int rows, int hidden, hipStream_t stream,
                    const void* x_parts = nullptr, int splits = 0, bool parts_bf16 = false);
int launch_layer_norm(bf16* out, const bf16* x, const bf16* residual_in, bf16* residual_out,
                      const bf16* w, const bf16* b, float eps, int rows, int hidden,
                      hipStream_t stream);
int launch_silu_mul(bf16* out, const bf16* x, int rows, int inter, bool interleaved,
                    hipStream_t stream);
int launch_gelu_bias(bf16* out, const bf16* x, const bf16* bias, int rows, int cols,
                     hipStream_t stream);
int launch_add(bf16* out, const bf16* a, const bf16* b, size_t n, hipStream_t stream);
// hop-integrity payload digest (digest.hip): [nblocks][2] int64 partial sums
int launch_digest(const void* data, long nwords, int64_t* part, int nblocks, hipStream_t stream);
int launch_rope_cache(const RopeCacheParams& p, int num_tokens, hipStream_t stream);
int launch_attn_decode(const AttnParams& p, int B, int D, hipStream_t stream);
int launch_attn_prefill(const AttnParams& p, int B, int max_q, int D, hipStream_t stream);
bool attn_prefill32_eligible(const AttnParams& p, int D);
int launch_attn_prefill32(const AttnParams& p, int B, int max_q, hipStream_t stream);
int launch_sample(const SampleParams& p, int B, hipStream_t stream);
int launch_gemm_tile(void* C, const void* A, const void* B, const float* a_scale,
                     const float* b_scale, float* workspace, int M, int N, int K, int splits,
                     int epilogue, int precision, hipStream_t stream,
                     const bf16* x_out = nullptr, const bf16* w_out = nullptr, int J = 0,
                     const uint8_t* a_mx = nullptr, uint8_t* out_mx = nullptr,
                     const int* ol_cnt = nullptr);
// C[MN] (bf16) = sum over `splits` fp32 partial products parts[splits][MN]
int launch_splitk_reduce(bf16* C, const float* parts, int splits, size_t MN, hipStream_t stream);
// fp32 elements of the workspace gemm_tile needs for splits == 0 (stream-K tail) on this device
long long gemm_tile_sk_workspace_floats();
// skinny GEMMs (gemv.hip); swiglu: W is a swiglu_interleave'd gate|up weight [2I, K] and y is
// silu(gate) * up [M, I].  nm: fused input RMSNorm of x (M <= 2, bf16 rows): x' = rmsnorm(x +
// res_in) * w, res_out = x + res_in (written once; must not alias res_in)
struct GemvNorm {
  const bf16* res_in;   // nullptr: no residual add
  bf16* res_out;        // nullptr: not written
  const bf16* w;        // [K]
  float eps;
};
// rp: W is the fused QKV weight [(nh + 2 nkv) D, K] and the GEMV's epilogue does rope_cache's
// work (q rotated into q_out [M, nh, D], k rotated and v into the paged caches); y is unused
struct GemvRope {
  const int* positions;       // [M]
  const long* slot_mapping;   // [M] (-1: no cache write)
  const float* cos_sin;       // [max_pos, D] (cos | sin), nullptr: no rotation
  int max_pos;
  bf16* q_out;                // [M, nh, D]
  void* k_cache;              // [blocks, nkv, bs, D]
  void* v_cache;              // [blocks, nkv, bs/8, D, 8]
  int kv_fp8;
  float k_inv_scale, v_inv_scale;
  int nh, nkv, D, bs;
};
int launch_skinny_gemm_fp8(bf16* y, const void* x, const float* xscale, const uint8_t* W,
                           const float* wscale, const bf16* bias, int M, int N, int K,
                           hipStream_t stream, bool swiglu = false, const GemvNorm* nm = nullptr,
                           const GemvRope* rp = nullptr);
int launch_skinny_gemm_int8(bf16* y, const bf16* x, const int8_t* W, const float* wscale,
                            const bf16* bias, int M, int N, int K, hipStream_t stream,
                            bool swiglu = false, const GemvNorm* nm = nullptr,
                            const GemvRope* rp = nullptr);
int launch_skinny_gemm(bf16* y, const bf16* x, const bf16* W, const bf16* bias, int M, int N,
                       int K, hipStream_t stream, bool swiglu = false,
                       const GemvNorm* nm = nullptr, const GemvRope* rp = nullptr);
// one-wave-per-SIMD 256x256 GEMM (gemm4.hip); epilogue 0 bf16, 1 fp32 partials, 2 SwiGLU,
// 3 SwiGLU quantised to MX fp8 (precision 1; scales into out_mx), 4 bf16 partials; grid <= 0:
// automatic persistent grid; variant < 0: default k-loop schedule.  precision 1: fp8 e4m3
// operands with per-row a_scale [M] and per-channel b_scale [N]; 2: fp8 with MX activation
// scales a_mx (mx_off layout) and per-channel b_scale
int launch_gemm4(void* C, const void* A, const void* B, int M, int N, int K, int splits,
                 int epilogue, int grid, hipStream_t stream, int variant = -1, int precision = 0,
                 const float* a_scale = nullptr, const float* b_scale = nullptr,
                 const uint8_t* a_mx = nullptr, uint8_t* out_mx = nullptr);
int gemm4_grid(int items, int cus);
int launch_quant_rowwise(uint8_t* q, float* scale, const bf16* x, const bf16* residual_in,
                         bf16* residual_out, const bf16* norm_w, float eps, int rows, int K,
                         hipStream_t stream, const void* x_parts = nullptr, int splits = 0,
                         bool parts_bf16 = false);
int launch_quant_rowwise_int8(int8_t* q, float* scale, const bf16* x, const uint8_t* outlier,
                              int rows, int K, hipStream_t stream);
// LLM.int8 outlier bookkeeping (int8_outlier.hip)
int launch_llm_int8_colmax(float* colmax, const bf16* x, int rows, int K, hipStream_t stream);
int launch_llm_int8_select(const float* colmax, int K, float threshold, int max_out, long* idx,
                           float* sel, uint8_t* flags, hipStream_t stream, int* cnt = nullptr);
// gathers: `cnt` (optional, written by the select kernel) = only the first ceil(cnt / 32) * 32
// columns are written (the rest keep stale data: for consumers that read no further)
int launch_llm_int8_gather_w(bf16* w_out, const int8_t* wq, const float* ws, const long* idx,
                             const float* sel, int N, int K, int max_out, hipStream_t stream,
                             const int* cnt = nullptr);
int launch_llm_int8_gather_wt(bf16* w_out, const int8_t* wqT, const float* ws, const long* idx,
                              const float* sel, int N, int max_out, hipStream_t stream,
                              const int* cnt = nullptr);
int launch_llm_int8_gather_x(bf16* x_out, const bf16* x, const long* idx, const float* sel, int M,
                             int K, int max_out, hipStream_t stream, const int* cnt = nullptr);
int launch_silu_mul_quant(uint8_t* q, float* scale, const bf16* x, int rows, int inter,
                          hipStream_t stream);

}  // namespace dli
