// Retired round 5: the torch binding of the persistent single-row
// decode-layer kernel (decode_layer.hip), as it was in csrc/bindings.hip.

// one Llama decoder layer for a single decode row, one persistent launch (decode_layer.hip)
dli::DecodeProj decode_proj(const Tensor& w, const optional<Tensor>& ws, const optional<Tensor>& b,
                            int& wq, const char* what) {
  CHECK_IN(w);
  TORCH_CHECK(w.dim() == 2, what, ": weight must be [N, K]");
  const int q = w.scalar_type() == at::kBFloat16 ? 0 : w.scalar_type() == at::kChar ? 2
                : w.element_size() == 1 ? 1 : -1;
  TORCH_CHECK(q >= 0 && (wq < 0 || wq == q), what, ": bf16 / fp8 / int8 weights, one format per layer");
  wq = q;
  dli::DecodeProj d{};
  d.w = w.data_ptr();
  d.N = (int)w.size(0);
  d.K = (int)w.size(1);
  if (q != 0) {
    TORCH_CHECK(ws.has_value(), what, ": 8-bit weights need their per-row scales");
    CHECK_IN(*ws); CHECK_F32(*ws);
    TORCH_CHECK(ws->numel() == d.N, what, ": scale must have N entries");
    d.ws = ws->data_ptr<float>();
  }
  if (b.has_value()) {
    CHECK_IN(*b); CHECK_BF16(*b);
    TORCH_CHECK(b->numel() == d.N, what, ": bias must have N entries");
    d.bias = bp(*b);
  }
  return d;
}

void decode_layer(Tensor h, optional<Tensor> r, Tensor res1, Tensor res2, Tensor out, Tensor ln1,
                  Tensor ln2, double eps1, double eps2, Tensor w_qkv, optional<Tensor> s_qkv,
                  optional<Tensor> b_qkv, Tensor w_o, optional<Tensor> s_o, optional<Tensor> b_o,
                  Tensor w_gu, optional<Tensor> s_gu, optional<Tensor> b_gu, Tensor w_down,
                  optional<Tensor> s_down, optional<Tensor> b_down, Tensor positions,
                  Tensor slot_mapping, optional<Tensor> cos_sin, Tensor q_out, Tensor k_cache,
                  Tensor v_cache, double k_scale, double v_scale, Tensor block_tables,
                  Tensor seq_lens, double scale, int64_t num_splits, optional<Tensor> part_o,
                  optional<Tensor> part_ml, Tensor attn, Tensor o_out, Tensor act, Tensor bar,
                  optional<Tensor> stamps, int64_t flags) {
  for (const Tensor* t : {&h, &res1, &res2, &out, &ln1, &ln2, &attn, &o_out, &act, &q_out}) {
    CHECK_IN(*t); CHECK_BF16(*t);
  }
  const int64_t K = h.numel();
  TORCH_CHECK(res1.numel() == K && res2.numel() == K && out.numel() == K && ln1.numel() == K &&
                  ln2.numel() == K && o_out.numel() == K,
              "decode_layer: hidden-size vectors");
  if (r.has_value()) {
    CHECK_IN(*r); CHECK_BF16(*r);
    TORCH_CHECK(r->numel() == K, "decode_layer: residual size");
    TORCH_CHECK(res1.data_ptr() != r->data_ptr() && res1.data_ptr() != h.data_ptr(),
                "decode_layer: res1 must not alias the inputs");
  } else {
    TORCH_CHECK(res1.data_ptr() == h.data_ptr(), "decode_layer: first layer passes res1 = h");
  }
  TORCH_CHECK(res2.data_ptr() != res1.data_ptr(), "decode_layer: res2 must not alias res1");
  CHECK_IN(bar);
  TORCH_CHECK(bar.scalar_type() == at::kLong && bar.numel() >= 168,
              "decode_layer: bar = int64 [168] (8 counters x 16, error word at 128, merge "
              "counters from 136)");
  int wq = -1;
  dli::DecodeLayerParams p{};
  p.qkv = decode_proj(w_qkv, s_qkv, b_qkv, wq, "decode_layer qkv");
  p.o = decode_proj(w_o, s_o, b_o, wq, "decode_layer o");
  p.gu = decode_proj(w_gu, s_gu, b_gu, wq, "decode_layer gate_up");
  p.down = decode_proj(w_down, s_down, b_down, wq, "decode_layer down");
  TORCH_CHECK(p.qkv.K == K && act.numel() == p.down.K, "decode_layer: projection shapes");
  TORCH_CHECK(q_out.dim() == 3 && q_out.size(0) == 1, "decode_layer: q_out [1, nh, D]");
  const int64_t nh = q_out.size(1), D = q_out.size(2);
  TORCH_CHECK(attn.numel() == nh * D, "decode_layer: attn [nh * D]");
  const int64_t nkv = (p.qkv.N / D - nh) / 2;
  TORCH_CHECK(p.qkv.N == (nh + 2 * nkv) * D && nkv >= 1, "decode_layer: qkv rows");
  // attention (B = 1) over q_out
  Tensor qv = q_out.view({1, nh, D});
  Tensor qo = qv;
  optional<Tensor> no_sink = c10::nullopt;
  int64_t Dq = 0;
  dli::AttnParams ap = attn_common(qo, qv, no_sink, k_cache, v_cache, block_tables, seq_lens,
                                   scale, 0, 0, 0, 0, k_scale, v_scale, Dq, false);
  ap.out = nullptr;
  TORCH_CHECK(seq_lens.numel() == 1 && num_splits >= 1, "decode_layer: one sequence");
  ap.num_splits = (int)num_splits;
  const int gs = num_splits % 4 == 0 ? 4 : num_splits % 2 == 0 ? 2 : 1;
  if (num_splits / gs > 1) {
    TORCH_CHECK(part_o.has_value() && part_ml.has_value(), "decode_layer: split workspaces");
    CHECK_IN(*part_o); CHECK_IN(*part_ml); CHECK_F32(*part_o); CHECK_F32(*part_ml);
    TORCH_CHECK(part_o->numel() >= num_splits / gs * nh * D && part_ml->numel() >= num_splits / gs * nh * 2,
                "decode_layer: split workspaces too small");
    ap.part_o = part_o->data_ptr<float>();
    ap.part_ml = part_ml->data_ptr<float>();
  }
  // QKV epilogue
  dli::GemvRope rp{};
  rp.kv_fp8 = ap.kv_fp8;
  rp.k_inv_scale = (float)(1.0 / k_scale);
  rp.v_inv_scale = (float)(1.0 / v_scale);
  CHECK_IN(positions); CHECK_I32(positions); CHECK_IN(slot_mapping); CHECK_I64(slot_mapping);
  TORCH_CHECK(positions.numel() == 1 && slot_mapping.numel() == 1, "decode_layer: one row");
  rp.positions = positions.data_ptr<int>();
  rp.slot_mapping = reinterpret_cast<const long*>(slot_mapping.data_ptr<int64_t>());
  if (cos_sin.has_value()) {
    CHECK_IN(*cos_sin); CHECK_F32(*cos_sin);
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == D, "cos_sin must be [max_pos, D]");
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
  p.h = bp(h);
  p.r = r.has_value() ? bp(*r) : nullptr;
  p.res1 = bp(res1);
  p.res2 = bp(res2);
  p.out = bp(out);
  p.ln1 = bp(ln1);
  p.ln2 = bp(ln2);
  p.eps1 = (float)eps1;
  p.eps2 = (float)eps2;
  p.rp = rp;
  p.ap = ap;
  p.gs = gs;
  p.attn = bp(attn);
  p.o_out = bp(o_out);
  p.act = bp(act);
  p.bar = reinterpret_cast<unsigned long long*>(bar.data_ptr<int64_t>());
  p.err = reinterpret_cast<unsigned*>(bar.data_ptr<int64_t>() + 128);
  p.merge_cnt = (flags & 2) ? nullptr : reinterpret_cast<unsigned*>(bar.data_ptr<int64_t>() + 136);
  if (stamps.has_value()) {
    CHECK_IN(*stamps);
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->numel() >= 24 * dli::decode_layer_grid(),
                "decode_layer: stamps = int64 [grid * 24]");
    p.stamps = reinterpret_cast<unsigned long long*>(stamps->data_ptr<int64_t>());
  }
  p.flags = (int)flags;
  const c10::hip::HIPGuardMasqueradingAsCUDA g(h.device());
  check_rc(dli::launch_decode_layer(p, wq, cur_stream()), "decode_layer");
}
