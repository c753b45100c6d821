// Retired round 5: csrc/kernels/kernels.h declarations of the decode-layer kernel.
// One Llama decoder layer for a single decode row in one persistent launch (decode_layer.hip).
struct DecodeProj {
  const void* w;       // [N, K]: bf16, fp8 e4m3 or int8
  const float* ws;     // [N] per-row scale (8-bit weights) or nullptr
  const bf16* bias;    // [N] or nullptr
  int N, K;
};
struct DecodeLayerParams {
  const bf16* h;        // [K] layer input (previous down output, or the embedding)
  const bf16* r;        // [K] residual stream, or nullptr (first layer: h is the residual)
  bf16* res1;           // [K] h + r (== h when r is nullptr: not written then)
  bf16* res2;           // [K] o_out + res1 (the layer's residual output)
  bf16* out;            // [K] down output (the layer's hidden output)
  const bf16* ln1;
  const bf16* ln2;
  float eps1, eps2;
  DecodeProj qkv, o, gu, down;   // gu: swiglu_interleave'd gate|up
  GemvRope rp;          // QKV epilogue: q -> rp.q_out, k / v -> the paged caches
  AttnParams ap;        // decode attention over rp.q_out (B = 1), split partials
  int gs;               // splits merged per 4-wave group
  bf16* attn;           // [nh * D] scratch
  bf16* o_out;          // [K] scratch
  bf16* act;            // [I] scratch
  unsigned long long* bar;   // grid-barrier arrival counters [8][16] (zero once, never reset)
  unsigned* err;        // barrier spin-timeout count (0 = every barrier completed)
  unsigned long long* stamps = nullptr;   // diagnostics: [grid][24] 100 MHz wall ticks per phase
  int flags = 0;        // bit 0: issue the O weights' first chunk at the attention barrier
  unsigned* merge_cnt = nullptr;   // [64] attention-merge arrival counters (zeroed in-kernel)
};
int launch_decode_layer(const DecodeLayerParams& p, int wq, hipStream_t stream);
int decode_layer_grid();
