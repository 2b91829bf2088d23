// libmtts engine: weights, KV cache, workspaces, prefill, hipGraph-captured decode steps,
// and the C ABI declared in include/mtts.h.
//
// Reference behaviour restated here (everything device-side lives in the .hip files):
//   MossTTSDelayModel.forward   moss_tts_delay/modeling_moss_tts.py:225-300
//   MossTTSDelayModel.generate  moss_tts_delay/modeling_moss_tts.py:392-525
//   Qwen3Model.forward          transformers/models/qwen3/modeling_qwen3.py:367-427
#include "engine_internal.h"

static int trace_rows(const mtts_config& c) { return std::max(c.layers, c.model_kind == MTTS_MODEL_LOCAL ? c.local_layers : 0); }

static thread_local std::string g_err;
int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// ---------------------------------------------------------------------------
// RoPE table (TF/.../modeling_qwen3.py:106-137): inv_freq = 1/theta^(2i/D) with the power
// correctly rounded to fp32 and an fp32 division; freqs = fp32(inv_freq * pos); cos/sin
// evaluated in double, rounded to fp32, then to bf16 (RNE).
static uint16_t host_f2bf(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
extern "C" int mtts_rope_table(float theta, int D, int n_pos, uint16_t* cos_h, uint16_t* sin_h) {
  if (D <= 0 || D % 2 || n_pos <= 0 || !cos_h || !sin_h) return fail(MTTS_E_INVALID, "bad rope table args");
  std::vector<float> inv(D / 2);
  for (int i = 0; i < D / 2; ++i) {
    const float e = (float)(2 * i) / (float)D;
    const float p = (float)std::pow((double)theta, (double)e);
    inv[i] = 1.0f / p;
  }
  for (int pos = 0; pos < n_pos; ++pos)
    for (int d = 0; d < D; ++d) {
      const float f = inv[d % (D / 2)] * (float)pos;
      cos_h[(size_t)pos * D + d] = host_f2bf((float)std::cos((double)f));
      sin_h[(size_t)pos * D + d] = host_f2bf((float)std::sin((double)f));
    }
  return 0;
}

extern "C" const char* mtts_last_error(void) { return g_err.c_str(); }
extern "C" int mtts_version(void) { return 1; }

extern "C" int mtts_engine_destroy(mtts_engine* e) {
  if (!e) return 0;
  hipSetDevice(e->device);
  for (auto& kv : e->graphs) hipGraphExecDestroy(kv.second.exec);
  local_destroy(e);
  for (void* p : e->allocs) hipFree(p);
  for (void* p : e->cap_allocs) hipFree(p);
  if (e->staging) hipFree(e->staging);
  if (e->ev_in) hipEventDestroy(e->ev_in);
  if (e->ev_pse) hipEventDestroy(e->ev_pse);
  if (e->pse_err_host) hipHostFree(e->pse_err_host);
  if (e->ev_out) hipEventDestroy(e->ev_out);
  if (e->stream) hipStreamDestroy(e->stream);
  delete e;
  return 0;
}

// capacity-dependent buffers (KV cache, RoPE table, mask, workspaces, generate state);
// weights are untouched, so mtts_engine_reserve can grow these without a reload
static int alloc_capacity(mtts_engine* e) {
  const mtts_config& c = e->c;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv, I = c.inter;
  int rc = 0;
  e->cap_mode = true;
  // KV cache [layer][Bmax][Hkv][Cmax][D]
  e->layer_kv = (size_t)c.max_batch * Hkv * c.max_ctx * D;
  if ((rc = e->alloc(&e->kc, e->layer_kv * c.layers)) || (rc = e->alloc(&e->vc, e->layer_kv * c.layers))) return rc;
  if ((rc = e->alloc(&e->cos_t, (size_t)c.max_ctx * D)) || (rc = e->alloc(&e->sin_t, (size_t)c.max_ctx * D))) return rc;
  {
    std::vector<uint16_t> cs((size_t)c.max_ctx * D), sn((size_t)c.max_ctx * D);
    mtts_rope_table(c.rope_theta, D, c.max_ctx, cs.data(), sn.data());
    hipMemcpy(e->cos_t, cs.data(), cs.size() * 2, hipMemcpyHostToDevice);
    hipMemcpy(e->sin_t, sn.data(), sn.size() * 2, hipMemcpyHostToDevice);
  }
  if ((rc = e->alloc(&e->mask, (size_t)c.max_batch * c.max_ctx))) return rc;
  // workspaces
  e->Mmax = std::max(c.max_batch, c.max_prefill_tokens);
  const size_t M = e->Mmax;
  if ((rc = e->alloc(&e->ss, M * (H / 16))) || (rc = e->alloc(&e->h, M * H)) || (rc = e->alloc(&e->xn, M * H)) || (rc = e->alloc(&e->qkvb, M * e->qkv_rows)) ||
      (rc = e->alloc(&e->qb, M * Hq * D)) || (rc = e->alloc(&e->attnb, M * Hq * D)) || (rc = e->alloc(&e->act, M * I)))
    return rc;
  const size_t ns_dec = (c.max_ctx + CH_DECODE - 1) / CH_DECODE;
  const size_t ns_pf = (c.max_ctx + CH_PREFILL - 1) / CH_PREFILL;
  // decode-attention split partials; the per-token split-K prefill attention (MTTS_OLD_PREFILL_ATTN,
  // A/B only) also keeps M x ns_pf of them -- 17 GB at an 8,192-token chunk and 32 K context,
  // which the flash prefill attention does not need
  e->part_floats = std::max((size_t)c.max_batch * ns_dec, e->old_prefill_attn ? M * ns_pf : 0) * Hq * (D + 2);
  if ((rc = e->alloc(&e->part, e->part_floats))) return rc;
  if ((rc = e->alloc(&e->logits, (size_t)c.max_batch * e->heads_ld))) return rc;
  if ((rc = e->alloc(&e->d_pos, 4))) return rc;
  if ((rc = e->alloc(&e->rope_off, (size_t)c.max_batch))) return rc;
  if (hipMemset(e->rope_off, 0, (size_t)c.max_batch * sizeof(int)) != hipSuccess) return fail(MTTS_E_HIP, "memset");
  if ((rc = e->alloc(&e->att_cnt, (size_t)c.max_batch * Hkv))) return rc;
  if (hipMemset(e->att_cnt, 0, (size_t)c.max_batch * Hkv * sizeof(int)) != hipSuccess) return fail(MTTS_E_HIP, "memset");
  if ((rc = e->alloc(&e->sk_part, SK_PART_FLOATS)) || (rc = e->alloc(&e->sk_cnt, (size_t)SK_TILES))) return rc;
  if ((rc = e->alloc(&e->gk_ws, GK_WS_FLOATS))) return rc;
  if (hipMemset(e->sk_cnt, 0, SK_TILES * sizeof(int)) != hipSuccess) return fail(MTTS_E_HIP, "memset");
  // persistent decode launch: per-layer pointers (the caches move with the capacity) + counters
  {
    std::vector<PseLayer> pl(c.layers);
    for (int l = 0; l < c.layers; ++l) {
      const LayerW& w = e->L[l];
      pl[l] = PseLayer{w.qkv, w.o, w.gu, w.down, w.in_norm, w.post_norm, w.q_norm, w.k_norm,
                       e->kc + l * e->layer_kv, e->vc + l * e->layer_kv};
    }
    if ((rc = e->alloc(&e->pse_L, (size_t)c.layers)) || (rc = e->alloc(&e->pse_ws, pse_ws_bytes()))) return rc;
    if (hipMemcpy(e->pse_L, pl.data(), pl.size() * sizeof(PseLayer), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(e->pse_ws, 0, pse_ws_bytes()) != hipSuccess)
      return fail(MTTS_E_HIP, "pse state");
    e->pse_ok = pse_supported(e->device, 1, c.layers, H, Hq, Hkv, D, I, e->qkv_rows, c.max_ctx);
    e->pse4_ok = c.max_batch >= 4 && pse4_supported(e->device, c.layers, H, Hq, Hkv, D, I, e->qkv_rows, c.max_ctx);
    if (e->pse4_ok) {
      if ((rc = e->alloc(&e->pse4_ws, pse4_ws_bytes()))) return rc;
      if (hipMemset(e->pse4_ws, 0, pse4_ws_bytes()) != hipSuccess) return fail(MTTS_E_HIP, "pse4 state");
    } else {
      e->pse4_ws = nullptr;
    }
    // (rows: the backbone's layers, or MossTTSLocal's depth layers if more -- lpse.hip stamps those)
  if (getenv("MTTS_PSE_TRACE") && (rc = e->alloc(&e->pse_trace, (size_t)trace_rows(c) * PSE_TRACE_EV * 256))) return rc;
  }
  // generate state
  const int B = c.max_batch;
  if ((rc = e->alloc(&e->st, 1)) || (rc = e->alloc(&e->is_stopping, B)) || (rc = e->alloc(&e->is_audio, B)) ||
      (rc = e->alloc(&e->text_cand, B)) || (rc = e->alloc(&e->audio_cand, (size_t)B * c.n_vq)) ||
      (rc = e->alloc(&e->part_idx, (size_t)B * TEXT_PARTS)) || (rc = e->alloc(&e->part_val, (size_t)B * TEXT_PARTS)) ||
      (rc = e->alloc(&e->audio_len, B)) || (rc = e->alloc(&e->delayed, B)) || (rc = e->alloc(&e->cur_ids, (size_t)B * (c.n_vq + 1))) ||
      (rc = e->alloc(&e->gen_ids, (size_t)B * c.max_ctx * (c.n_vq + 1))) || (rc = e->alloc(&e->seen, 2 * e->audio_rows)) ||
      (rc = e->alloc(&e->wide_hist, (size_t)B * 65536)))
    return rc;
  e->cap_mode = false;
  return 0;
}

extern "C" int mtts_engine_create(const mtts_config* cfg, int device, mtts_engine** out) {
  if (!cfg || !out) return fail(MTTS_E_INVALID, "null argument");
  const mtts_config& c = *cfg;
  if (c.hidden % 32 || c.inter % 32 || c.head_dim % 8 || c.head_dim > 128 || c.n_heads % c.n_kv ||
      (c.n_heads * c.head_dim) % 32 || c.max_batch <= 0 || c.max_batch > 256 || c.max_ctx <= 0 || c.max_ctx > MTTS_MAX_CTX || c.n_vq < 1)
    return fail(MTTS_E_UNSUPPORTED, "unsupported model shape");
  const int G = c.n_heads / c.n_kv;
  if (G != 1 && G != 2 && G != 4 && G != 8) return fail(MTTS_E_UNSUPPORTED, "GQA group must be 1/2/4/8");
  if ((c.vocab + TEXT_PARTS - 1) / TEXT_PARTS > 4096) return fail(MTTS_E_UNSUPPORTED, "text vocab too large");
  if (c.audio_vocab + 1 > 1040) return fail(MTTS_E_UNSUPPORTED, "audio vocab too large");
  if (c.model_kind != MTTS_MODEL_DELAY && c.model_kind != MTTS_MODEL_LOCAL) return fail(MTTS_E_UNSUPPORTED, "model_kind");
  if (c.model_kind == MTTS_MODEL_LOCAL &&
      (c.local_hidden <= 0 || c.local_hidden % 64 || c.local_hidden > 4096 || c.local_inter <= 0 || c.local_inter % 32 ||
       c.local_mlp_ffn <= 0 || c.local_mlp_ffn % 32 || c.local_layers <= 0 || c.n_vq + 1 > 64 || c.hidden % 64))
    return fail(MTTS_E_UNSUPPORTED, "unsupported MossTTSLocal shape");
  if (hipSetDevice(device) != hipSuccess) return fail(MTTS_E_HIP, "hipSetDevice failed");
  mtts_engine* e = new mtts_engine();
  e->c = c;
  e->c.max_ctx = (c.max_ctx + 63) / 64 * 64;  // 16-byte V^T fragments, whole 64-key chunks
  if (e->c.max_prefill_tokens <= 0) e->c.max_prefill_tokens = 8192;
  e->device = device;
  if (const char* v = getenv("MTTS_UNFUSED_NORM")) e->unfused_norm = v[0] == '1';
  if (const char* v = getenv("MTTS_FULL_TEXT_HEAD")) e->full_text_head = v[0] == '1';
  if (const char* v = getenv("MTTS_GEMV_PREFILL")) e->gemv_prefill = v[0] == '1';
  if (const char* v = getenv("MTTS_UNFUSED_ATTN")) e->unfused_attn = v[0] == '1';
  if (const char* v = getenv("MTTS_OLD_PREFILL_ATTN")) e->old_prefill_attn = v[0] == '1';
  if (const char* v = getenv("MTTS_PSE")) e->pse = v[0] == '1';
  if (const char* v = getenv("MTTS_PSE_CTX")) e->pse_ctx_max = atoi(v);
  if (const char* v = getenv("MTTS_PSE_COOP")) e->pse_coop = v[0] == '1';
  if (const char* v = getenv("MTTS_PSE4")) e->pse4 = v[0] == '1';
  if (const char* v = getenv("MTTS_PSE_LONG")) e->pse_long = v[0] == '1';
  if (const char* v = getenv("MTTS_ATTN_LONG")) e->attn_long_ctx = atoi(v);
  if (const char* v = getenv("MTTS_XPACK")) e->xpack = v[0] == '1';
  if (const char* v = getenv("MTTS_SPLITK")) e->splitk = v[0] == '1';
  if (const char* v = getenv("MTTS_NW")) sscanf(v, "%d,%d,%d,%d,%d", &e->nw[0], &e->nw[1], &e->nw[2], &e->nw[3], &e->nw[4]);
  if (const char* v = getenv("MTTS_U")) sscanf(v, "%d,%d,%d,%d,%d", &e->nu[0], &e->nu[1], &e->nu[2], &e->nu[3], &e->nu[4]);
  auto bail = [&](int rc) {
    mtts_engine_destroy(e);
    return rc;
  };
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) return bail(fail(MTTS_E_HIP, "stream"));
  hipEventCreateWithFlags(&e->ev_in, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_out, hipEventDisableTiming);
  hipEventCreateWithFlags(&e->ev_pse, hipEventDisableTiming);
  if (hipHostMalloc((void**)&e->pse_err_host, 4, hipHostMallocDefault) != hipSuccess) return bail(fail(MTTS_E_OOM, "pinned word"));
  *e->pse_err_host = 0;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv, I = c.inter;
  e->qkv_rows = (Hq + 2 * Hkv) * D;
  e->audio_rows = c.audio_vocab + 1;
  e->heads_rows = c.vocab + c.n_vq * e->audio_rows;
  e->heads_ld = e->heads_rows;
  e->text_tile_lo = std::min({c.im_end_token_id, c.audio_assistant_gen_slot_token_id,
                              c.audio_assistant_delay_slot_token_id, c.vocab}) / 16;
  int rc = 0;
  e->L.resize(c.layers);
  uint64_t wb = 0;
  for (int l = 0; l < c.layers; ++l) {
    LayerW& w = e->L[l];
    if ((rc = e->alloc(&w.qkv, packed_bytes(e->qkv_rows, H) / 2))) return bail(rc);
    if ((rc = e->alloc(&w.o, packed_bytes(H, Hq * D) / 2))) return bail(rc);
    if ((rc = e->alloc(&w.gu, packed_bytes(2 * I, H) / 2))) return bail(rc);
    if ((rc = e->alloc(&w.down, packed_bytes(H, I) / 2))) return bail(rc);
    if ((rc = e->alloc(&w.in_norm, H)) || (rc = e->alloc(&w.post_norm, H)) || (rc = e->alloc(&w.q_norm, D)) ||
        (rc = e->alloc(&w.k_norm, D)))
      return bail(rc);
    hipMemset(w.qkv, 0, packed_bytes(e->qkv_rows, H));
    hipMemset(w.o, 0, packed_bytes(H, Hq * D));
    wb += 2ull * ((uint64_t)e->qkv_rows * H + (uint64_t)H * Hq * D + 2ull * I * H + (uint64_t)H * I) + 2ull * 2 * H + 2ull * 2 * D;
  }
  if ((rc = e->alloc(&e->emb_text, (size_t)c.vocab * H)) || (rc = e->alloc(&e->emb_audio, (size_t)c.n_vq * e->audio_rows * H)) ||
      (rc = e->alloc(&e->final_norm, H)))
    return bail(rc);
  wb += 2ull * H;
  if (c.model_kind == MTTS_MODEL_DELAY) {  // MossTTSLocal keeps one packed head per channel (local.cpp)
    if ((rc = e->alloc(&e->heads, packed_bytes(e->heads_rows, H) / 2))) return bail(rc);
    hipMemset(e->heads, 0, packed_bytes(e->heads_rows, H));
    wb += 2ull * (uint64_t)e->heads_rows * H;
  }
  e->step_weight_bytes = wb;
  if ((rc = alloc_capacity(e))) return bail(rc);
  if (c.model_kind == MTTS_MODEL_LOCAL && ((rc = local_create(e)) || (rc = local_alloc_capacity(e)))) return bail(rc);
  if (hipDeviceSynchronize() != hipSuccess) return bail(fail(MTTS_E_HIP, "init sync failed"));
  *out = e;
  return 0;
}

extern "C" int mtts_engine_reserve(mtts_engine* e, int max_batch, int max_ctx, int max_prefill_tokens) {
  if (!e || max_batch <= 0 || max_batch > 256 || max_ctx <= 0 || max_ctx > MTTS_MAX_CTX) return fail(MTTS_E_INVALID, "bad capacity");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  for (auto& kv : e->graphs) hipGraphExecDestroy(kv.second.exec);
  e->graphs.clear();
  local_clear_graphs(e);
  for (void* p : e->cap_allocs) hipFree(p);
  e->cap_allocs.clear();
  e->c.max_batch = max_batch;
  e->c.max_ctx = (max_ctx + 63) / 64 * 64;
  e->c.max_prefill_tokens = max_prefill_tokens > 0 ? max_prefill_tokens : 8192;
  e->gen_B = 0;
  int rc = alloc_capacity(e);
  if (!rc && e->lp) rc = local_alloc_capacity(e);
  if (rc) return rc;
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

extern "C" int mtts_engine_weight_bytes(const mtts_engine* e, uint64_t* bytes) {
  if (!e || !bytes) return fail(MTTS_E_INVALID, "null argument");
  *bytes = e->step_weight_bytes;
  return 0;
}
extern "C" int mtts_heads_ld(const mtts_engine* e) { return e ? e->heads_ld : 0; }
uint32_t* mtts_engine::pse_err(int B) const {
  return B == 4 ? (pse4_ws ? pse4_err_word(pse4_ws) : nullptr) : (pse_ws ? pse_err_word(pse_ws) : nullptr);
}
extern "C" int mtts_pse_active(const mtts_engine* e) { return e && e->pse && e->pse_ok ? 1 : 0; }
extern "C" int mtts_pse4_active(const mtts_engine* e) { return e && e->pse_takes(4) ? 1 : 0; }
extern "C" int mtts_pse_long_active(const mtts_engine* e) { return e && e->pse_takes(1) && e->pse_long ? 1 : 0; }
extern "C" int mtts_pse_inject_timeout(mtts_engine* e) {
  if (e && e->lp) {
    hipSetDevice(e->device);
    return local_lpse_inject(e);
  }
  if (!e || !e->pse_ws) return fail(MTTS_E_INVALID, "no persistent launch state");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint32_t code = 0x7e57u;
  HIPCHK(hipMemcpy(pse_err_word(e->pse_ws), &code, 4, hipMemcpyHostToDevice));
  if (e->pse4_ws) HIPCHK(hipMemcpy(pse4_err_word(e->pse4_ws), &code, 4, hipMemcpyHostToDevice));
  return 0;
}
extern "C" int mtts_pse_ctx_max(const mtts_engine* e) {
  return e && e->pse && (e->pse_ok || (e->pse4 && e->pse4_ok)) ? e->pse_ctx_max : 0;
}
extern "C" int mtts_pse_trace(mtts_engine* e, uint64_t* host, size_t n) {
  if (!e || !host) return fail(MTTS_E_INVALID, "null argument");
  if (!e->pse_trace) return fail(MTTS_E_UNSUPPORTED, "engine created without MTTS_PSE_TRACE=1");
  const size_t have = (size_t)trace_rows(e->c) * PSE_TRACE_EV * 256;
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemcpy(host, e->pse_trace, std::min(n, have) * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return 0;
}

// ---------------------------------------------------------------------------
// weight loading by reference state_dict name
int ensure_staging(mtts_engine* e, size_t bytes) {
  if (e->staging_bytes >= bytes) return 0;
  if (e->staging) hipFree(e->staging);
  e->staging = nullptr;
  e->staging_bytes = 0;
  if (hipMalloc(&e->staging, bytes) != hipSuccess) return fail(MTTS_E_OOM, "staging alloc");
  e->staging_bytes = bytes;
  return 0;
}

bool parse_layer(const char* name, int* layer, std::string* rest) {
  const char* p = "language_model.layers.";
  if (std::strncmp(name, p, std::strlen(p)) != 0) return false;
  const char* q = name + std::strlen(p);
  char* end = nullptr;
  long l = std::strtol(q, &end, 10);
  if (end == q || *end != '.') return false;
  *layer = (int)l;
  *rest = std::string(end + 1);
  return true;
}

bool layer_target(const LayerW& w, const std::string& rest, int H, int I, int Hq, int Hkv, int D, WTarget* t) {
  WTarget r;
  r.pack = true;
  if (rest == "self_attn.q_proj.weight") { r.dst = w.qkv; r.rows = Hq * D; r.K = H; r.row_off = 0; }
  else if (rest == "self_attn.k_proj.weight") { r.dst = w.qkv; r.rows = Hkv * D; r.K = H; r.row_off = Hq * D; }
  else if (rest == "self_attn.v_proj.weight") { r.dst = w.qkv; r.rows = Hkv * D; r.K = H; r.row_off = (Hq + Hkv) * D; }
  else if (rest == "self_attn.o_proj.weight") { r.dst = w.o; r.rows = H; r.K = Hq * D; }
  else if (rest == "mlp.gate_proj.weight") { r.dst = w.gu; r.rows = I; r.K = H; r.inter = 1; r.which = 0; }
  else if (rest == "mlp.up_proj.weight") { r.dst = w.gu; r.rows = I; r.K = H; r.inter = 1; r.which = 1; }
  else if (rest == "mlp.down_proj.weight") { r.dst = w.down; r.rows = H; r.K = I; }
  else {
    r.pack = false;
    if (rest == "self_attn.q_norm.weight") { r.dst = w.q_norm; r.expect = D; }
    else if (rest == "self_attn.k_norm.weight") { r.dst = w.k_norm; r.expect = D; }
    else if (rest == "input_layernorm.weight") { r.dst = w.in_norm; r.expect = H; }
    else if (rest == "post_attention_layernorm.weight") { r.dst = w.post_norm; r.expect = H; }
    else return false;
  }
  if (r.pack) r.expect = (size_t)r.rows * r.K;
  *t = r;
  return true;
}

int store_weight(mtts_engine* e, const WTarget& t, const char* name, const void* src, size_t bytes, int on_dev) {
  if (bytes != t.expect * 2) return fail(MTTS_E_INVALID, std::string("size mismatch for ") + name);
  // a device source may still be in flight on the caller's stream (e.g. a torch tensor just
  // produced there): the engine stream orders after that stream by an event (enter), and the
  // caller's later work -- e.g. freeing the source -- after the repack (leave).  No device-wide
  // sync per tensor (a state_dict is ~400 of them; a device sync also stalls other streams).
  hipStream_t s = enter(e, e->load_stream);
  if (!t.pack) {
    HIPCHK(hipMemcpyAsync(t.dst, src, bytes, on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  } else {
    const bf16_t* from = reinterpret_cast<const bf16_t*>(src);
    if (!on_dev) {
      int rc = ensure_staging(e, bytes);
      if (rc) return rc;
      HIPCHK(hipMemcpyAsync(e->staging, src, bytes, hipMemcpyHostToDevice, s));
      from = e->staging;
    }
    HIPCHK(pack_weight(from, t.dst, t.rows, t.K, t.row_off, t.inter, t.which, s));
  }
  // a host source must stay untouched until its copy has landed: wait for those only
  if (!on_dev) HIPCHK(hipStreamSynchronize(s));
  leave(e, e->load_stream);
  return 0;
}

extern "C" int mtts_engine_load_weight_stream(mtts_engine* e, const char* name, const void* src, size_t bytes,
                                              int on_dev, void* stream) {
  if (!e || !name || !src) return fail(MTTS_E_INVALID, "null argument");
  e->load_stream = stream;
  const int rc = load_weight_impl(e, name, src, bytes, on_dev);
  e->load_stream = nullptr;
  return rc;
}
// the legacy default stream orders the source (what torch's default stream is)
extern "C" int mtts_engine_load_weight(mtts_engine* e, const char* name, const void* src, size_t bytes, int on_dev) {
  return mtts_engine_load_weight_stream(e, name, src, bytes, on_dev, nullptr);
}
int load_weight_impl(mtts_engine* e, const char* name, const void* src, size_t bytes, int on_dev) {
  hipSetDevice(e->device);
  if (e->lp) {  // MossTTSLocal names (model.embedding_list.*, local_transformer.*, ...)
    int rc = 0;
    if (local_load_weight(e, name, src, bytes, on_dev, &rc)) return rc;
  }
  const mtts_config& c = e->c;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv, I = c.inter;
  WTarget t;
  int layer = -1;
  std::string rest;
  if (!std::strcmp(name, "language_model.embed_tokens.weight")) {
    t.dst = e->emb_text; t.expect = (size_t)c.vocab * H;
  } else if (!std::strcmp(name, "language_model.norm.weight")) {
    t.dst = e->final_norm; t.expect = H;
  } else if (!std::strncmp(name, "emb_ext.", 8)) {
    const int j = std::atoi(name + 8);
    if (j < 0 || j >= c.n_vq) return fail(MTTS_E_INVALID, std::string("bad name ") + name);
    t.dst = e->emb_audio + (size_t)j * e->audio_rows * H; t.expect = (size_t)e->audio_rows * H;
  } else if (!std::strncmp(name, "lm_heads.", 9) && !e->lp) {
    const int j = std::atoi(name + 9);
    if (j < 0 || j > c.n_vq) return fail(MTTS_E_INVALID, std::string("bad name ") + name);
    t.pack = true; t.dst = e->heads; t.K = H;
    t.rows = j == 0 ? c.vocab : e->audio_rows;
    t.row_off = j == 0 ? 0 : c.vocab + (j - 1) * e->audio_rows;
    t.expect = (size_t)t.rows * H;
  } else if (parse_layer(name, &layer, &rest)) {
    if (layer < 0 || layer >= c.layers) return fail(MTTS_E_INVALID, std::string("bad layer in ") + name);
    if (!layer_target(e->L[layer], rest, H, I, Hq, Hkv, D, &t))
      return fail(MTTS_E_INVALID, std::string("unknown weight ") + name);
  } else {
    return fail(MTTS_E_INVALID, std::string("unknown weight ") + name);
  }
  return store_weight(e, t, name, src, bytes, on_dev);
}

// same tensor order / init as oracle.moss_delay.weight_specs + scale_for (no text boost)
extern "C" int mtts_engine_init_random(mtts_engine* e, uint64_t seed) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  hipSetDevice(e->device);
  if (e->lp) return local_init_random(e, seed);
  const mtts_config& c = e->c;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv, I = c.inter;
  struct Spec { std::string name; size_t rows, cols; int kind; };  // 0 lin 1 norm 2 emb 3 head
  std::vector<Spec> sp;
  sp.push_back({"language_model.embed_tokens.weight", (size_t)c.vocab, (size_t)H, 2});
  for (int l = 0; l < c.layers; ++l) {
    const std::string p = "language_model.layers." + std::to_string(l) + ".";
    sp.push_back({p + "self_attn.q_proj.weight", (size_t)Hq * D, (size_t)H, 0});
    sp.push_back({p + "self_attn.k_proj.weight", (size_t)Hkv * D, (size_t)H, 0});
    sp.push_back({p + "self_attn.v_proj.weight", (size_t)Hkv * D, (size_t)H, 0});
    sp.push_back({p + "self_attn.o_proj.weight", (size_t)H, (size_t)Hq * D, 0});
    sp.push_back({p + "self_attn.q_norm.weight", 1, (size_t)D, 1});
    sp.push_back({p + "self_attn.k_norm.weight", 1, (size_t)D, 1});
    sp.push_back({p + "mlp.gate_proj.weight", (size_t)I, (size_t)H, 0});
    sp.push_back({p + "mlp.up_proj.weight", (size_t)I, (size_t)H, 0});
    sp.push_back({p + "mlp.down_proj.weight", (size_t)H, (size_t)I, 0});
    sp.push_back({p + "input_layernorm.weight", 1, (size_t)H, 1});
    sp.push_back({p + "post_attention_layernorm.weight", 1, (size_t)H, 1});
  }
  sp.push_back({"language_model.norm.weight", 1, (size_t)H, 1});
  for (int j = 0; j < c.n_vq; ++j) sp.push_back({"emb_ext." + std::to_string(j) + ".weight", (size_t)e->audio_rows, (size_t)H, 2});
  sp.push_back({"lm_heads.0.weight", (size_t)c.vocab, (size_t)H, 3});
  for (int j = 0; j < c.n_vq; ++j) sp.push_back({"lm_heads." + std::to_string(j + 1) + ".weight", (size_t)e->audio_rows, (size_t)H, 3});
  size_t mx = 0;
  for (auto& s : sp) mx = std::max(mx, s.rows * s.cols);
  int rc = ensure_staging(e, mx * 2);
  if (rc) return rc;
  for (size_t tid = 0; tid < sp.size(); ++tid) {
    const Spec& s = sp[tid];
    float scale = 1.f, offset = 0.f;
    if (s.kind == 0 || s.kind == 3) scale = (float)std::sqrt(3.0 / (double)s.cols);
    else if (s.kind == 1) { scale = 0.25f; offset = 1.0f; }
    HIPCHK(fill_uniform_bf16(e->staging, s.rows * s.cols, seed, tid, scale, offset, e->stream));
    rc = mtts_engine_load_weight(e, s.name.c_str(), e->staging, s.rows * s.cols * 2, 1);
    if (rc) return rc;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// The GEMV `g` reads Qwen3RMSNorm(h) with weight `nw`.  Small decode batches fold the norm
// into the GEMV prologue (normalised rows staged in LDS per block, no extra launch); larger
// ones run the single-pass rmsnorm_ss kernel into e->xn first.  Both read the residual
// stream's per-16-column sums of squares e->ss.
int normed_input(mtts_engine* e, const Stack& st, GemvArgs& g, const bf16_t* nw, int M, hipStream_t s, int tiles) {
  const int H = st.H, NT = H / 16;
  // (packed prefills, tiles > 2, run the GEMM, which has no norm prologue)
  if (tiles <= 2 && norm_lds_bytes(M, H) <= NORM_LDS_MAX && !e->unfused_norm) {
    g.x = st.h; g.ldx = H;
    g.ss_in = st.ss; g.ld_ss = NT; g.n_ss = NT; g.nw = nw; g.eps = e->c.rms_eps;
    return 0;
  }
  HIPCHK(rmsnorm_ss(st.h, 0, H, st.ss, 0, NT, nw, st.xn, M, H, e->c.rms_eps, s, tiles));
  g.x = st.xn; g.ldx = H; g.x_packed = tiles ? 1 : 0;
  g.pk_tiles = tiles > 2 ? tiles : 0;  // > 2: the prefill GEMM's form
  return 0;
}

Stack backbone_stack(mtts_engine* e) {
  const mtts_config& c = e->c;
  Stack st;
  st.L = e->L.data(); st.layers = c.layers; st.H = c.hidden; st.Hq = c.n_heads; st.Hkv = c.n_kv; st.D = c.head_dim;
  st.I = c.inter; st.qkv_rows = e->qkv_rows;
  st.kc = e->kc; st.vc = e->vc; st.layer_kv = e->layer_kv; st.Cmax = c.max_ctx;
  st.cos_t = e->cos_t; st.sin_t = e->sin_t; st.mask = e->mask;
  st.h = e->h; st.xn = e->xn; st.qkvb = e->qkvb; st.qb = e->qb; st.attnb = e->attnb; st.act = e->act;
  st.rows = e->Mmax;
  st.ss = e->ss; st.part = e->part; st.att_cnt = e->att_cnt;
  // MossTTSLocal: its `generate` is GenerationMixin's, whose position ids exclude a row's left pads
  // (cumsum(mask) - 1, transformers/generation/utils.py:751-773); MossTTSDelay's own loop
  // includes them (positions = cache slots, TF/.../modeling_qwen3.py:386-389)
  st.rope_off = e->lp ? e->rope_off : nullptr;
  return st;
}

// ---------------------------------------------------------------------------
// forward over rows [b0, b0+B) with S tokens each; pos_base device pointer.
// Per layer: input RMSNorm (from the residual epilogue's sums of squares; fused into the
// GEMV prologue for small batches) -> q|k|v GEMV -> attention (decode: one fused kernel incl. q/k norm, RoPE, KV append;
// prefill: norm/rope/append + split-K attention + combine) -> o_proj GEMV (+residual,
// +sums of squares) -> post-attention RMSNorm (fused as above) -> gate|up GEMV (SwiGLU epilogue) -> down
// GEMV (+residual, +sums of squares).
// token-parallel projections: the decode GEMV for a handful of rows, the prefill GEMM
// (weights read once per 256 tokens instead of once per 32) beyond that
static int gemm_min_rows() {  // MTTS_GEMM_MIN_ROWS (A/B): token rows from which projections use the GEMM
  static const int v = getenv("MTTS_GEMM_MIN_ROWS") ? atoi(getenv("MTTS_GEMM_MIN_ROWS")) : 33;
  return v;
}
hipError_t proj(mtts_engine* e, const GemvArgs& g, int epi, hipStream_t s) {
  if (g.B >= gemm_min_rows() && !g.ss_in && !e->gemv_prefill && (!(g.x_packed || g.y_packed) || g.pk_tiles > 0)) {
    GemvArgs gg = g;  // short prompts split K over workgroups (gemm.hip)
    gg.ws = e->gk_ws;
    gg.ws_floats = e->gk_ws ? GK_WS_FLOATS : 0;
    return gemm_ex(gg, epi, s);
  }
  // residual projections with too few output tiles to fill the chip (MossTTSLocal's depth
  // down_proj: 96 tiles): split K over workgroups (splitk.hip)
  if (epi == EPI_RESADD && e->splitk && e->sk_part && g.res && !g.ss_in && !g.attn.part && !g.gate && !g.tile0 &&
      !g.x_packed) {
    const int tiles = (g.N + 15) / 16, S = gemv_splitk_splits(tiles, g.K / 32, g.B);
    if (S > 1 && tiles <= SK_TILES && gemv_splitk_ws_floats(tiles, S) <= SK_PART_FLOATS)
      return gemv_splitk(g, S, e->sk_part, e->sk_cnt, s);
  }
  // 17-32 packed rows (B = 32 decode o_proj / down_proj): row tiles share the x fragments,
  // K split to keep the grid full (splitk.hip)
  if (epi == EPI_RESADD && e->splitk && e->sk_part && g.res && !g.ss_in && !g.attn.part && !g.gate && !g.tile0 &&
      g.x_packed) {
    const int tiles = (g.N + 15) / 16;
    int RT = 0, S = 0;
    if (gemv_splitk2_pick(tiles, g.K / 32, g.B, &RT, &S) && tiles / RT <= SK_TILES &&
        gemv_splitk2_ws_floats(tiles, S) <= SK_PART_FLOATS)
      return gemv_splitk2(g, RT, S, e->sk_part, e->sk_cnt, s);
  }
  return gemv_ex(g, epi, s);
}

// the decoder layers of a stack over rows [b0, b0+B), S tokens each, token s of a row at
// position *pos_base + s
int run_layers(mtts_engine* e, const Stack& st, int b0, int B, int S, const int* pos_base, int CH, int n_split,
               hipStream_t s) {
  const int H = st.H, D = st.D, Hq = st.Hq, Hkv = st.Hkv, I = st.I;
  const int M = B * S;
  const int NT = H / 16;  // per-row sum-of-squares partials (one per 16-column tile)
  const float eps = e->c.rms_eps;
  if (S == 1 && B == 1 && b0 == 0 && e->pse && e->pse_ok && (e->pse_now || e->pse_long_now) && st.cos_t &&
      st.L == e->L.data()) {
    // the whole stack as one persistent launch with run-ahead weight streaming (pse.hip)
    PseArgs pa{};
    pa.L = e->pse_L; pa.layers = st.layers; pa.h = st.h; pa.ss = st.ss; pa.cos_t = st.cos_t; pa.sin_t = st.sin_t;
    pa.mask = st.mask; pa.pos = pos_base; pa.Cmax = st.Cmax; pa.eps = e->c.rms_eps;
    pa.scale = 1.0f / std::sqrt((float)D);
    pa.trace = e->pse_trace;
    static const int pse_probe = getenv("MTTS_PSE_PROBE") ? atoi(getenv("MTTS_PSE_PROBE")) : 0;
    pa.probe = pse_probe;
    HIPCHK(pse_decode(pa, e->pse_ws, s, e->pse_coop, !e->pse_now));
    return 0;
  }
  if (S == 1 && B == 4 && b0 == 0 && e->pse_takes(4) && e->pse_now && st.cos_t && st.L == e->L.data()) {
    // the batch-4 form (pse4.hip): rows 0-3 of the residual stream, masks and caches
    PseArgs pa{};
    pa.L = e->pse_L; pa.layers = st.layers; pa.h = st.h; pa.ss = st.ss; pa.cos_t = st.cos_t; pa.sin_t = st.sin_t;
    pa.mask = st.mask; pa.pos = pos_base; pa.Cmax = st.Cmax; pa.eps = e->c.rms_eps;
    pa.scale = 1.0f / std::sqrt((float)D);
    pa.trace = e->pse_trace;
    HIPCHK(pse4_decode(pa, e->pse4_ws, s, e->pse_coop));
    return 0;
  }
  // decode: o_proj merges the attention's split partials in its prologue when it preloads one
  // merged element per thread (gemv_attn_preload: batch 1-2 at K 4096) and the context is short
  // (the long-context graphs' attention merges its many splits itself); otherwise the attention
  // writes its rows and o_proj is a plain GEMV
  const bool fuse_attn = S == 1 && M <= 16 && (size_t)M * Hq * D * 2 <= NORM_LDS_MAX && !e->unfused_attn &&
                         !st.attn_direct && !e->long_now && gemv_attn_preload(M, Hq * D, H, e->nw[1]);
  // batch-1 decode at long contexts (e->long_now): 16-wave (512-key) attention blocks
  const int dec_nwv = st.attn_nwv ? st.attn_nwv : ((S == 1 && B == 1 && e->long_now && st.cos_t) ? 16 : 0);
  // 17-32 row decode: the GEMV inputs (xn, the attention output, the SwiGLU output) travel in
  // the fragment-packed layout, so each x fragment is one 1 KiB load (B=32 per layer: x loads
  // cost ~22 of 129 us row-major)
  const bool xpk = S == 1 && M > 16 && M <= 32 && st.rows >= 32 && e->xpack;
  // long prefills (the 32-utterance batch): the same for the 128 x 128 GEMM, T = M / 16 token
  // tiles (its x loads were 81 of 191 ms row-major)
  // prefills of >= 128 token rows (the 128 x 128 GEMM's range): packed GEMM inputs.  B=1 clone
  // prompt (181 rows) 12.6 -> 9.5 ms with the split-K partial launches reading them packed
  // (MTTS_PK_MIN / MTTS_PK_SPLIT=0 for A/B)
  // (from 33 rows since round 5: the <= 192-row GEMM form takes 3-12 token tiles)
  static const int pk_min = getenv("MTTS_PK_MIN") ? atoi(getenv("MTTS_PK_MIN")) : 33;
  const int pkT = (S > 1 && M >= pk_min && e->xpack && !e->gemv_prefill && !e->old_prefill_attn &&
                   M >= gemm_min_rows() && (M + 15) / 16 * 16 <= st.rows) ? (M + 15) / 16 : 0;
  const int ntiles = xpk ? 2 : pkT;  // packed activations of this call (0: row-major)
  // packed split prefills: the residual GEMMs' split-K reduce also writes the next op's normed,
  // packed input (GemvArgs::pn_w; MTTS_FUSE_PN=0 for A/B), and that op skips its rmsnorm_ss
  static const bool fuse_pn = !getenv("MTTS_FUSE_PN") || getenv("MTTS_FUSE_PN")[0] != '0';
  int xn_ready = 0;  // st.xn holds the next op's normed packed input
  auto input = [&](GemvArgs& g, const bf16_t* nw) -> int {
    if (xn_ready) {
      g.x = st.xn; g.ldx = H; g.x_packed = 1; g.pk_tiles = pkT;
      xn_ready = 0;
      return 0;
    }
    return normed_input(e, st, g, nw, M, s, ntiles);
  };
  auto fuse_next = [&](GemvArgs& g, const bf16_t* nw) {
    if (!fuse_pn || pkT <= 2 || !nw) return;
    g.pn_w = nw; g.pn_y = st.xn; g.pn_tiles = pkT; g.pn_eps = eps; g.pn_done = &xn_ready;
  };
  for (int l = 0; l < st.layers; ++l) {
    const LayerW& w = st.L[l];
    bf16_t* kc = st.kc + l * st.layer_kv + (size_t)b0 * Hkv * st.Cmax * D;
    bf16_t* vc = st.vc + l * st.layer_kv + (size_t)b0 * Hkv * st.Cmax * D;
    GemvArgs g = gemv_args(w.qkv, st.xn, H, st.qkvb, st.qkv_rows, M, st.qkv_rows, H);
    if (int rc = input(g, w.in_norm)) return rc;
    g.force_nw = e->nw[0]; g.force_u = e->nu[0];
    DecAttnArgs da{};
    da.qkv = st.qkvb; da.qn_w = w.q_norm; da.kn_w = w.k_norm; da.cos_t = st.cos_t; da.sin_t = st.sin_t;
    da.kc = kc; da.vc = vc; da.mask = st.mask + (size_t)b0 * st.Cmax; da.pos = pos_base; da.out = st.attnb;
    da.rope_off = st.rope_off ? st.rope_off + b0 : nullptr;
    da.part = st.part; da.cnt = st.att_cnt;
    // small batches: blocks only publish partials; the o_proj GEMV merges them in its prologue
    da.publish_only = fuse_attn ? 1 : 0;
    da.po_max = attn_publish_max_splits();
    da.out_packed = xpk ? 1 : 0;
    da.nwv_force = dec_nwv;
    da.Hq = Hq; da.Hkv = Hkv; da.D = D; da.Cmax = st.Cmax; da.eps = eps; da.scale = 1.0f / std::sqrt((float)D);
    QKRopeArgs qa{};
    qa.qkv = st.qkvb; qa.q_out = st.qb; qa.kc = kc; qa.vc = vc;
    qa.qn_w = w.q_norm; qa.kn_w = w.k_norm; qa.cos_t = st.cos_t; qa.sin_t = st.sin_t;
    qa.pos_base = pos_base; qa.S = S; qa.Hq = Hq; qa.Hkv = Hkv; qa.D = D; qa.Cmax = st.Cmax; qa.eps = eps; qa.M = M;
    qa.rope_off = st.rope_off ? st.rope_off + b0 : nullptr;
    // packed split prefills: the q|k|v reduce runs the q/k norm + RoPE + KV append itself
    // (MTTS_FUSE_QKR=0 for A/B)
    static const bool fuse_qkr = !getenv("MTTS_FUSE_QKR") || getenv("MTTS_FUSE_QKR")[0] != '0';
    int qk_done = 0;
    if (fuse_qkr && S > 1 && pkT > 2 && D == 128 && st.cos_t) {
      g.qkr = &qa;
      g.qkr_done = &qk_done;
    }
    HIPCHK(proj(e, g, EPI_STORE, s));
    if (S == 1) {
      HIPCHK(attn_decode(da, B, s));
    } else {
      if (!st.cos_t) return fail(MTTS_E_UNSUPPORTED, "multi-token forward of a stack without positions");
      if (!qk_done) HIPCHK(qk_norm_rope(qa, s));
      AttnArgs aa;
      aa.q = st.qb; aa.kc = kc; aa.vc = vc; aa.mask = st.mask + (size_t)b0 * st.Cmax; aa.pos_base = pos_base;
      aa.part_o = st.part; aa.part_ml = st.part + (size_t)M * n_split * Hq * D; aa.out = st.attnb;
      aa.S = S; aa.Hq = Hq; aa.Hkv = Hkv; aa.D = D; aa.Cmax = st.Cmax; aa.CH = CH; aa.n_split = n_split; aa.M = M;
      aa.out_tiles = pkT;
      aa.scale = 1.0f / std::sqrt((float)D);
      if (e->old_prefill_attn) HIPCHK(attention(aa, s));
      else HIPCHK(attention_prefill(aa, s));
    }
    g = gemv_args(w.o, st.attnb, Hq * D, st.h, H, M, H, Hq * D);
    g.res = st.h; g.ldres = H; g.ss_out = st.ss; g.ld_ss_out = NT; g.force_nw = e->nw[1]; g.force_u = e->nu[1];
    g.x_packed = ntiles ? 1 : 0; g.pk_tiles = pkT;
    if (fuse_attn) {
      g.attn.part = st.part; g.attn.pos = pos_base; g.attn.Hkv = Hkv; g.attn.G = Hq / Hkv; g.attn.D = D;
      g.attn.kb = attn_decode_keys_per_block_nwv(dec_nwv);
      g.attn.ns = (st.Cmax + g.attn.kb - 1) / g.attn.kb;
      g.attn.po_max = attn_publish_max_splits();
    }
    fuse_next(g, w.post_norm);
    HIPCHK(proj(e, g, EPI_RESADD, s));
    g = gemv_args(w.gu, st.xn, H, st.act, I, M, I, H);
    if (int rc = input(g, w.post_norm)) return rc;
    g.force_nw = e->nw[2]; g.force_u = e->nu[2];
    g.y_packed = ntiles ? 1 : 0;
    HIPCHK(proj(e, g, EPI_SWIGLU, s));
    g = gemv_args(w.down, st.act, I, st.h, H, M, H, I);
    g.res = st.h; g.ldres = H; g.ss_out = st.ss; g.ld_ss_out = NT; g.force_nw = e->nw[3]; g.force_u = e->nu[3];
    g.x_packed = ntiles ? 1 : 0; g.pk_tiles = pkT;
    if (l + 1 < st.layers) fuse_next(g, st.L[l + 1].in_norm);
    HIPCHK(proj(e, g, EPI_RESADD, s));
  }
  return 0;
}

int forward_rows(mtts_engine* e, const int64_t* ids, int b0, int B, int S, const int* pos_base, int CH,
                 int n_split, bf16_t* logits_out, hipStream_t s, const int* text_gate, bool heads, bf16_t* hidden,
                 int n_embed) {
  const mtts_config& c = e->c;
  const int H = c.hidden, C = c.n_vq + 1;
  const int M = B * S;
  const int NT = H / 16;
  const float eps = c.rms_eps;
  const Stack st = backbone_stack(e);
  HIPCHK(embed(ids, n_embed > 0 ? n_embed : C, e->emb_text, e->emb_audio, e->audio_rows, H, e->h, M, s, e->ss, NT, C));
  if (int rc = run_layers(e, st, b0, B, S, pos_base, CH, n_split, s)) return rc;
  if (!heads && hidden) {  // final-normed hidden state of each row's last token (MossTTSLocal)
    HIPCHK(rmsnorm_ss(e->h, (size_t)(S - 1) * H, (size_t)S * H, e->ss, (size_t)(S - 1) * NT, (size_t)S * NT,
                      e->final_norm, hidden, B, H, eps, s));
    return 0;
  }
  if (!heads) return 0;  // a leading chunk of a position-chunked prefill: KV cache only
  // final norm on the last token of each row, then the 1+n_vq heads (audio pad column -inf)
  GemvArgs g = gemv_args(e->heads, e->xn, H, logits_out, e->heads_ld, B, e->heads_rows, H);
  if (S == 1) {
    // 17-32 rows: the heads' input packed too (one 1 KiB load per x fragment)
    const bool hpk = B > 16 && B <= 32 && st.rows >= 32 && e->xpack;
    if (int rc = normed_input(e, st, g, e->final_norm, B, s, hpk ? 2 : 0)) return rc;
  } else {
    HIPCHK(rmsnorm_ss(e->h, (size_t)(S - 1) * H, (size_t)S * H, e->ss, (size_t)(S - 1) * NT, (size_t)S * NT,
                      e->final_norm, e->xn, B, H, eps, s));
  }
  g.pad_start = c.vocab; g.pad_period = e->audio_rows; g.pad_off = e->audio_rows - 1;
  // decode at <= 16 rows: 4-wave blocks for the heads (B=4 3.052 -> 3.034 ms/step, B=1 even;
  // profiles/r05_v_ab_heads_nw.txt); MTTS_NW's fifth entry overrides
  g.force_nw = e->nw[4] ? e->nw[4] : (S == 1 && B <= 16 ? 4 : 0);
  g.force_u = e->nu[4];
  if (text_gate && e->text_tile_lo > 0) {
    // decode: text rows below the special ids only when some row samples text freely.
    // Audio-mode rows see every text logit except gen_slot / delay_slot masked to -inf
    // (modeling_moss_tts.py:459-460), so those are the only text logits they need.
    GemvArgs gt = g;
    gt.N = e->text_tile_lo * 16;
    gt.gate = text_gate;
    HIPCHK(gemv_ex(gt, EPI_LOGITS, s));
    g.tile0 = e->text_tile_lo;
  }
  HIPCHK(gemv_ex(g, EPI_LOGITS, s));
  return 0;
}

// prefill / teacher-forced forward of S tokens at position `past` (host int).  Rows are
// chunked so that rows x S <= max_prefill_tokens; a prompt longer than that is prefilled one
// row at a time in position chunks of max_prefill_tokens (each chunk attends to the cache the
// previous ones wrote; only the last chunk evaluates the heads) -- the long-form (TTSD) path.
int forward_chunked(mtts_engine* e, const int64_t* ids, int B, int S, int past, bf16_t* logits_out, hipStream_t s,
                    bf16_t* hidden, int n_embed, const int* text_gate) {
  const mtts_config& c = e->c;
  const int C = c.n_vq + 1;
  const int CH = S == 1 ? CH_DECODE : CH_PREFILL;
  if (S > e->Mmax) {
    const int P = e->Mmax;
    for (int b = 0; b < B; ++b) {
      for (int s0 = 0; s0 < S; s0 += P) {
        const int len = std::min(P, S - s0);
        HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(e->d_pos), past + s0, 1, s));
        const int n_split = (past + s0 + len + CH - 1) / CH;
        const bool last = s0 + len == S;
        int rc = forward_rows(e, ids + ((size_t)b * S + s0) * C, b, 1, len, e->d_pos, CH, n_split,
                              logits_out ? logits_out + (size_t)b * e->heads_ld : nullptr, s, text_gate,
                              last && !hidden, last && hidden ? hidden + (size_t)b * c.hidden : nullptr, n_embed);
        if (rc) return rc;
      }
    }
    return 0;
  }
  HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(e->d_pos), past, 1, s));
  const int rows_per = std::max(1, e->Mmax / S);
  const int n_split = (past + S + CH - 1) / CH;
  for (int b0 = 0; b0 < B; b0 += rows_per) {
    const int nb = std::min(rows_per, B - b0);
    int rc = forward_rows(e, ids + (size_t)b0 * S * C, b0, nb, S, e->d_pos, CH, n_split,
                          logits_out ? logits_out + (size_t)b0 * e->heads_ld : nullptr, s, text_gate, !hidden,
                          hidden ? hidden + (size_t)b0 * c.hidden : nullptr, n_embed);
    if (rc) return rc;
  }
  return 0;
}

// The engine works on its own non-blocking stream, ordered after / before the caller's
// stream by events.  A NULL caller stream is the legacy default stream (what torch's
// default `cuda_stream` handle is), which a non-blocking stream does NOT synchronise with
// implicitly, so it gets the same event fences.
hipStream_t enter(mtts_engine* e, void* user) {
  hipSetDevice(e->device);
  hipEventRecord(e->ev_in, (hipStream_t)user);
  hipStreamWaitEvent(e->stream, e->ev_in, 0);
  return e->stream;
}
void leave(mtts_engine* e, void* user) {
  hipEventRecord(e->ev_out, e->stream);
  hipStreamWaitEvent((hipStream_t)user, e->ev_out, 0);
}

// The persistent streaming launch's error word (pse.hip: a bounded wait timed out).  When set:
// clear it, turn the launch off for this engine (every later step takes the per-op launches)
// and report true; synchronises the engine stream.
bool pse_tripped(mtts_engine* e, hipStream_t s) {
  if (e->lp) return local_lpse_tripped(e, s);
  if (!e->pse_ws) return false;
  uint32_t err = 0, err4 = 0;
  if (hipStreamSynchronize(s) != hipSuccess || hipMemcpy(&err, pse_err_word(e->pse_ws), 4, hipMemcpyDeviceToHost) != hipSuccess)
    return false;
  if (e->pse4_ws && hipMemcpy(&err4, pse4_err_word(e->pse4_ws), 4, hipMemcpyDeviceToHost) != hipSuccess) return false;
  if (!err && !err4) return false;
  err |= err4;
  hipMemset(e->pse_ws, 0, pse_ws_bytes());
  if (e->pse4_ws) hipMemset(e->pse4_ws, 0, pse4_ws_bytes());
  e->pse = false;
  e->pse_timeouts += 1;
  fprintf(stderr, "libmtts: persistent streaming decode timed out (code %u; device shared with other work?); "
                  "this engine continues on the per-op launches\n", err);
  return true;
}

// A teacher-forced forward through the persistent launch leaves its error word on the way to
// pinned host memory (an async copy + event): no host sync per step, legal under a caller's
// stream capture.  The word is checked lazily: without blocking at the start of the next forward
// / generation (pse_lazy_check(e, false)), blocking in mtts_pse_check.  A tripped launch (a wait
// timed out: its workgroups were not all resident, other work on the device) turns the launch
// off for this engine and is reported ONCE as MTTS_E_PSE_TIMEOUT: the logits of the forwards
// since the last clean check are invalid and must be recomputed (the forward is idempotent: it
// rewrites the KV rows at past..), which the per-op launches then do.
static void pse_trip(mtts_engine* e, uint32_t err) {
  hipMemsetAsync(pse_err_word(e->pse_ws), 0, 4, e->stream);
  if (e->pse4_ws) hipMemsetAsync(pse4_err_word(e->pse4_ws), 0, 4, e->stream);
  e->pse = false;
  e->pse_timeouts += 1;
  fprintf(stderr, "libmtts: persistent streaming decode timed out (code %u; device shared with other work?); "
                  "this engine continues on the per-op launches\n", err);
}
static int pse_lazy_check(mtts_engine* e, bool block) {
  if (!e->pse_pending) return 0;
  if (block) {
    HIPCHK(hipEventSynchronize(e->ev_pse));
  } else if (hipEventQuery(e->ev_pse) != hipSuccess) {
    return 0;  // not landed yet: a later call reports it
  }
  e->pse_pending = false;
  const uint32_t err = *(volatile uint32_t*)e->pse_err_host;
  if (!err) return 0;
  pse_trip(e, err);
  return fail(MTTS_E_PSE_TIMEOUT, "persistent streaming decode: a wait timed out; the logits of the forwards since "
                                  "the last check are invalid (recompute them: the engine now runs the per-op launches)");
}

static int pse_report_owed(mtts_engine* e) {
  if (!e->pse_unreported) return 0;
  e->pse_unreported = false;
  return fail(MTTS_E_PSE_TIMEOUT, "persistent streaming decode: a wait timed out in a teacher-forced forward before "
                                  "the last generation; those forwards' logits are invalid (the engine now runs the "
                                  "per-op launches)");
}

extern "C" int mtts_engine_set_pse_lazy(mtts_engine* e, int lazy) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  e->pse_lazy = lazy != 0;
  return 0;
}

extern "C" int mtts_pse_check(mtts_engine* e) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  hipSetDevice(e->device);
  if (int rc = pse_lazy_check(e, true)) return rc;
  if (int rc = pse_report_owed(e)) return rc;
  // forwards the caller captured into its own graph: read the word itself
  if (e->pse_ws && pse_tripped(e, e->stream))
    return fail(MTTS_E_PSE_TIMEOUT, "persistent streaming decode: a wait timed out (results since the last check "
                                    "are invalid; the engine now runs the per-op launches)");
  return 0;
}

extern "C" int mtts_forward(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int S, int past,
                            uint16_t* logits, void* stream) {
  if (!e || !ids || !mask || !logits) return fail(MTTS_E_INVALID, "null argument");
  if (e->lp) return fail(MTTS_E_UNSUPPORTED, "MossTTSLocal engine: use mtts_local_forward");
  const mtts_config& c = e->c;
  if (B <= 0 || B > c.max_batch || S <= 0 || past < 0 || past + S > c.max_ctx) return fail(MTTS_E_INVALID, "bad B/S/past");
  hipSetDevice(e->device);
  if (int rc = pse_lazy_check(e, false)) return rc;
  if (int rc = pse_report_owed(e)) return rc;
  hipStream_t s = enter(e, stream);
  HIPCHK(hipMemcpy2DAsync(e->mask, c.max_ctx, mask, past + S, past + S, B, hipMemcpyDeviceToDevice, s));
  e->pse_choose(past + S);
  e->long_now = e->attn_long_ctx > 0 && past + S > e->attn_long_ctx;
  int rc = forward_chunked(e, ids, B, S, past, reinterpret_cast<bf16_t*>(logits), s);
  if (!rc && S == 1 && e->pse_takes(B) && (e->pse_now || (B == 1 && e->pse_long_now)) && e->pse_err(B)) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(s, &cs));
    if (cs != hipStreamCaptureStatusNone) {
      // inside a caller's capture: mtts_pse_check reads the word
    } else if (!e->pse_lazy) {
      // default: check now; a timed-out launch wrote only its own granules, the residual and this
      // step's KV rows, so the step is recomputed on the per-op launches (which rewrite those rows)
      // and the caller gets valid logits from this very call
      if (pse_tripped(e, s)) {
        e->pse_choose(past + S);
        rc = forward_chunked(e, ids, B, S, past, reinterpret_cast<bf16_t*>(logits), s);
      }
    } else {
      HIPCHK(hipMemcpyAsync(e->pse_err_host, e->pse_err(B), 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipEventRecord(e->ev_pse, s));
      e->pse_pending = true;
    }
  }
  leave(e, stream);
  return rc;
}

// ---------------------------------------------------------------------------
// test hooks: write K / V rows of the cache directly (host bf16 k, v [Hkv][n][D] at positions
// pos0 .. pos0 + n - 1 of row b, layer l; V is stored transposed), or fill the whole cache with
// one bf16 pattern (e.g. NaN: rows never written must never reach a result)
extern "C" int mtts_engine_kv_write(mtts_engine* e, int layer, int b, int pos0, int n, const uint16_t* k,
                                    const uint16_t* v) {
  if (!e || !k || !v) return fail(MTTS_E_INVALID, "null argument");
  const mtts_config& c = e->c;
  if (e->lp || layer < 0 || layer >= c.layers || b < 0 || b >= c.max_batch || pos0 < 0 || n <= 0 || pos0 + n > c.max_ctx)
    return fail(MTTS_E_INVALID, "bad kv_write args");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  const int D = c.head_dim, Hkv = c.n_kv, Cm = c.max_ctx;
  bf16_t* kc = e->kc + layer * e->layer_kv + (size_t)b * Hkv * Cm * D;
  bf16_t* vc = e->vc + layer * e->layer_kv + (size_t)b * Hkv * Cm * D;
  std::vector<uint16_t> vt((size_t)D * n);
  for (int g = 0; g < Hkv; ++g) {
    HIPCHK(hipMemcpy(kc + ((size_t)g * Cm + pos0) * D, k + (size_t)g * n * D, (size_t)n * D * 2, hipMemcpyHostToDevice));
    for (int i = 0; i < n; ++i)
      for (int d = 0; d < D; ++d) vt[(size_t)d * n + i] = v[((size_t)g * n + i) * D + d];
    HIPCHK(hipMemcpy2D(vc + (size_t)g * D * Cm + pos0, (size_t)Cm * 2, vt.data(), (size_t)n * 2, (size_t)n * 2, D,
                       hipMemcpyHostToDevice));
  }
  return 0;
}
extern "C" int mtts_engine_kv_fill(mtts_engine* e, uint16_t bits) {
  if (!e || e->lp) return fail(MTTS_E_INVALID, "bad engine");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  HIPCHK(hipMemsetD16(reinterpret_cast<hipDeviceptr_t>(e->kc), bits, e->layer_kv * e->c.layers));
  HIPCHK(hipMemsetD16(reinterpret_cast<hipDeviceptr_t>(e->vc), bits, e->layer_kv * e->c.layers));
  HIPCHK(hipDeviceSynchronize());
  return 0;
}

// ---------------------------------------------------------------------------
static int decode_step_launch(mtts_engine* e, hipStream_t s) {
  const int B = e->gen_B;
  const int n_split = (e->c.max_ctx + CH_DECODE - 1) / CH_DECODE;
  int rc = forward_rows(e, e->cur_ids, 0, B, 1, &e->st->fwd_pos, CH_DECODE, n_split, e->logits, s,
                        e->full_text_head ? nullptr : &e->st->need_text);
  if (rc) return rc;
  HIPCHK(sample_step(e->bufs(), B, e->c.n_vq, TEXT_PARTS, s));
  return 0;
}

extern "C" int mtts_generate_begin(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int T, int max_new,
                                   const mtts_sampling* sp, const int32_t* forced, void* stream) {
  if (!e || !ids || !sp) return fail(MTTS_E_INVALID, "null argument");
  if (e->lp) return fail(MTTS_E_UNSUPPORTED, "MossTTSLocal engine: use mtts_local_generate_begin");
  const mtts_config& c = e->c;
  if (B <= 0 || B > c.max_batch || T <= 0 || max_new <= 0 || T + max_new > c.max_ctx)
    return fail(MTTS_E_INVALID, "B/T/max_new_tokens exceed the engine capacity");
  hipSetDevice(e->device);
  // a tripped teacher-forced launch of earlier (lazily checked) forwards: switch before this
  // generation, which is valid; the timeout stays owed to the caller (pse_report_owed)
  if (pse_lazy_check(e, true)) {
    g_err.clear();
    e->pse_unreported = true;
  }
  hipStream_t s = enter(e, stream);
  GenDev& g = e->hst;
  std::memset(&g, 0, sizeof(g));
  g.T0 = T; g.step = 0; g.fwd_pos = 0; g.done_step = -1;
  g.B = B; g.n_vq = c.n_vq; g.C = c.n_vq + 1; g.Ltot = c.max_ctx; g.Cmax = c.max_ctx;
  g.vocab = c.vocab; g.audio_rows = e->audio_rows; g.heads_ld = e->heads_ld;
  g.P = TEXT_PARTS; g.part_len = (c.vocab + TEXT_PARTS - 1) / TEXT_PARTS;
  g.text_sample = sp->text_temperature > 0.f;
  g.audio_sample = sp->audio_temperature > 0.f;
  g.text_temp = g.text_sample ? sp->text_temperature : 1.f;
  g.audio_temp = g.audio_sample ? sp->audio_temperature : 1.f;
  g.text_top_p = sp->text_top_p; g.audio_top_p = sp->audio_top_p;
  g.text_top_k = sp->text_top_k; g.audio_top_k = sp->audio_top_k;
  g.rep_penalty = sp->audio_repetition_penalty;
  g.seed = sp->seed;
  g.ids.pad = c.pad_token_id; g.ids.im_start = c.im_start_token_id; g.ids.im_end = c.im_end_token_id;
  g.ids.audio_start = c.audio_start_token_id; g.ids.audio_end = c.audio_end_token_id;
  g.ids.user_slot = c.audio_user_slot_token_id; g.ids.gen_slot = c.audio_assistant_gen_slot_token_id;
  g.ids.delay_slot = c.audio_assistant_delay_slot_token_id; g.ids.audio_pad = c.audio_pad_code;
  // sampled text: top_k 1..TOPK_CAP sorts its candidates; <= 0 (no filter, inference_utils.py:136)
  // or larger runs the key-bin sampler over the whole row (topk.h block_wide_draw); audio rows
  // have 1,025 codes, so any audio top_k (<= 0: no filter) fits the sorted form
  if (e->audio_rows > TOPK_CAP) return fail(MTTS_E_UNSUPPORTED, "audio vocab above 2048");
  e->gen_B = B; e->gen_T = T; e->gen_max_new = max_new; e->forced = forced;
  HIPCHK(hipMemcpyAsync(e->st, &g, sizeof(g), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(e->seen, 0, 2 * e->audio_rows, s));
  HIPCHK(gen_init(e->bufs(), ids, mask, B, T, c.n_vq + 1, s));
  e->pse_choose(T);  // (a prefill takes the launch only as a one-token prompt)
  e->long_now = e->attn_long_ctx > 0 && T > e->attn_long_ctx;
  // the step-0 text rows only when some row continues in text mode (gen_init sets need_text)
  int rc = forward_chunked(e, ids, B, T, 0, e->logits, s, nullptr, 0, e->full_text_head ? nullptr : &e->st->need_text);
  if (rc) return rc;
  HIPCHK(sample_step(e->bufs(), B, c.n_vq, TEXT_PARTS, s));
  e->steps_issued = 1;
  leave(e, stream);
  return 0;
}

extern "C" int mtts_generate_decode(mtts_engine* e, int n_steps, void* stream) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  if (e->lp) return fail(MTTS_E_UNSUPPORTED, "MossTTSLocal engine: use mtts_local_generate_decode");
  if (e->gen_B <= 0) return fail(MTTS_E_INVALID, "generate_begin not called");
  hipStream_t s = enter(e, stream);
  // the graph bakes the kernel arguments (buffers, B, the forced-schedule pointer);
  // every step-dependent value is read from device state, so one graph serves all steps --
  // one per path: the persistent streaming launch (pse.hip) while the context stays in its
  // range, the per-op launches beyond (the choice is per step, from the host's step count)
  auto graph_for = [&](bool pse, bool lng, bool plong, hipGraphExec_t* exec) -> int {
    const int key = e->gen_B * 8 + (plong ? 4 : 0) + (lng ? 2 : 0) + (pse ? 1 : 0);
    auto it = e->graphs.find(key);
    if (it != e->graphs.end() && it->second.forced == e->forced) {
      *exec = it->second.exec;
      return 0;
    }
    if (it != e->graphs.end()) {
      hipGraphExecDestroy(it->second.exec);
      e->graphs.erase(it);
    }
    e->pse_now = pse;
    e->pse_long_now = plong;
    e->long_now = lng;
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = decode_step_launch(e, s);
    hipError_t ce = hipStreamEndCapture(s, &graph);
    if (rc) return rc;
    if (ce != hipSuccess) return fail(MTTS_E_HIP, std::string("capture: ") + hipGetErrorString(ce));
    HIPCHK(hipGraphInstantiate(exec, graph, nullptr, nullptr, 0));
    hipGraphDestroy(graph);
    e->graphs[key] = mtts_engine::Graph{*exec, e->forced, pse || plong};
    return 0;
  };
  for (int i = 0; i < n_steps && e->steps_issued < e->gen_max_new; ++i) {
    // context of this step <= prompt + steps so far + 1
    const int ctx = e->gen_T + e->steps_issued + 1;
    const bool pse = e->pse_takes(e->gen_B) && ctx <= e->pse_ctx_max;
    // batch 1 past the short form's range: the launch's all-CU attention form
    const bool plong = !pse && e->gen_B == 1 && e->pse_takes(1) && e->pse_long;
    const bool lng = !pse && !plong && e->gen_B == 1 && e->attn_long_ctx > 0 && ctx > e->attn_long_ctx;
    hipGraphExec_t exec = nullptr;
    if (int rc = graph_for(pse, lng, plong, &exec)) return rc;
    HIPCHK(hipGraphLaunch(exec, s));
    ++e->steps_issued;
  }
  leave(e, stream);
  return 0;
}

extern "C" int mtts_generate_poll(mtts_engine* e, int* steps, int* done_step, void* stream) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  GenDev g;
  HIPCHK(hipMemcpy(&g, e->st, sizeof(g), hipMemcpyDeviceToHost));
  if (pse_tripped(e, e->stream))  // the persistent streaming launch gave up waiting: the run is invalid
    return fail(MTTS_E_PSE_TIMEOUT, "persistent streaming decode: a wait timed out (results invalid; the engine "
                                    "now runs the per-op launches: restart the generation)");
  if (g.topk_overflow)
    return fail(MTTS_E_UNSUPPORTED, "top-k: ties at the k-th score exceed 2048 candidates (lower top_k)");
  if (steps) *steps = g.step;
  if (done_step) *done_step = g.done_step;
  (void)stream;
  return 0;
}

extern "C" int mtts_generate_stats(mtts_engine* e, int* text_head_steps) {
  if (!e || !text_head_steps) return fail(MTTS_E_INVALID, "null argument");
  hipSetDevice(e->device);
  HIPCHK(hipStreamSynchronize(e->stream));
  GenDev g;
  HIPCHK(hipMemcpy(&g, e->st, sizeof(g), hipMemcpyDeviceToHost));
  *text_head_steps = g.text_head_steps;
  return 0;
}

extern "C" int mtts_generate(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int T, int max_new,
                             const mtts_sampling* sp, const int32_t* forced, int chunk, int* n_rows, void* stream) {
  if (chunk <= 0) chunk = 16;
  // a persistent-launch timeout (MTTS_E_PSE_TIMEOUT) turned that launch off: the generation
  // restarts once from the prompt on the per-op launches (the inputs are the caller's)
  for (int attempt = 0;; ++attempt) {
    int rc = mtts_generate_begin(e, ids, mask, B, T, max_new, sp, forced, stream);
    if (rc) return rc;
    int steps = 1, done = -1;
    while (true) {
      rc = mtts_generate_poll(e, &steps, &done, stream);
      if (rc) break;
      if (done >= 0 || steps >= max_new) break;
      // every issued step advances the device's step counter (finalize), so a counter behind the
      // issued steps with nothing left to issue is a broken state, not a wait: fail, never spin
      if (e->steps_issued >= e->gen_max_new)
        return fail(MTTS_E_HIP, "generation stalled: the device step counter is at " + std::to_string(steps) + " of " +
                                    std::to_string(e->steps_issued) + " issued steps");
      rc = mtts_generate_decode(e, std::min(chunk, max_new - steps), stream);
      if (rc) break;
    }
    if (rc == MTTS_E_PSE_TIMEOUT && attempt == 0) continue;
    if (rc) return rc;
    if (n_rows) *n_rows = done >= 0 ? done + 1 : steps;
    return 0;
  }
}

extern "C" int mtts_generate_fetch(mtts_engine* e, int64_t* out, int n_rows, void* stream) {
  if (!e || !out) return fail(MTTS_E_INVALID, "null argument");
  const int C = e->c.n_vq + 1;
  if (n_rows < 0 || e->gen_T + n_rows > e->c.max_ctx) return fail(MTTS_E_INVALID, "bad n_rows");
  hipStream_t s = enter(e, stream);
  const size_t w = (size_t)(e->gen_T + n_rows) * C * sizeof(int64_t);
  HIPCHK(hipMemcpy2DAsync(out, w, e->gen_ids, (size_t)e->c.max_ctx * C * sizeof(int64_t), w, e->gen_B,
                          hipMemcpyDeviceToDevice, s));
  leave(e, stream);
  return 0;
}

extern "C" int mtts_generate_logits(mtts_engine* e, uint16_t* out, void* stream) {
  if (!e || !out) return fail(MTTS_E_INVALID, "null argument");
  if (e->lp) return fail(MTTS_E_UNSUPPORTED, "MossTTSLocal engine: logits are per channel");
  if (e->gen_B <= 0) return fail(MTTS_E_INVALID, "generate_begin not called");
  hipStream_t s = enter(e, stream);
  HIPCHK(hipMemcpyAsync(out, e->logits, (size_t)e->gen_B * e->heads_ld * sizeof(bf16_t), hipMemcpyDeviceToDevice, s));
  leave(e, stream);
  return 0;
}

// ---------------------------------------------------------------------------
// kernel-level entry points
extern "C" size_t mtts_k_packed_bytes(int rows, int K) { return packed_bytes(rows, K); }
extern "C" int mtts_k_pack(const uint16_t* src, uint16_t* dst, int rows, int K, int row_offset, int interleave, int which,
                           void* stream) {
  HIPCHK(pack_weight(src, dst, rows, K, row_offset, interleave, which, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_gemv(const uint16_t* w, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                           int ldres, int B, int N, int K, int epi, int ps, int pp, int po, void* stream) {
  if (K % 32) return fail(MTTS_E_INVALID, "K must be a multiple of 32");
  HIPCHK(gemv(w, x, ldx, y, ldy, res, ldres, B, N, K, epi, ps, pp, po, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_rmsnorm(const uint16_t* x, size_t xo, size_t xs, const uint16_t* w, uint16_t* y, int M, int H,
                              float eps, void* stream) {
  HIPCHK(rmsnorm(x, xo, xs, w, y, M, H, eps, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_embed(const int64_t* ids, int C, const uint16_t* et, const uint16_t* ea, int ar, int H, uint16_t* h,
                            int M, void* stream) {
  HIPCHK(embed(ids, C, et, ea, ar, H, h, M, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_qk_norm_rope(const uint16_t* qkv, uint16_t* q_out, uint16_t* kc, uint16_t* vc, const uint16_t* qn,
                                   const uint16_t* kn, const uint16_t* cs, const uint16_t* sn, const int32_t* pos, int M,
                                   int S, int Hq, int Hkv, int D, int Cmax, float eps, void* stream) {
  QKRopeArgs a;
  a.qkv = qkv; a.q_out = q_out; a.kc = kc; a.vc = vc; a.qn_w = qn; a.kn_w = kn; a.cos_t = cs; a.sin_t = sn;
  a.pos_base = pos; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.D = D; a.Cmax = Cmax; a.eps = eps; a.M = M;
  a.rope_off = nullptr;
  HIPCHK(qk_norm_rope(a, (hipStream_t)stream));
  return 0;
}
extern "C" size_t mtts_k_attention_ws_bytes(int M, int Hq, int D, int n_split) {
  return (size_t)M * n_split * Hq * (D + 2) * sizeof(float);
}
extern "C" int mtts_k_attention(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const uint8_t* mask,
                                const int32_t* pos, uint16_t* out, void* ws, int M, int S, int Hq, int Hkv, int D,
                                int Cmax, int CH, int n_split, void* stream) {
  AttnArgs a{};
  a.q = q; a.kc = kc; a.vc = vc; a.mask = mask; a.pos_base = pos;
  a.part_o = reinterpret_cast<float*>(ws);
  a.part_ml = a.part_o + (size_t)M * n_split * Hq * D;
  a.out = out; a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.D = D; a.Cmax = Cmax; a.CH = CH; a.n_split = n_split; a.M = M;
  a.scale = 1.0f / std::sqrt((float)D);
  HIPCHK(attention(a, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_attention_prefill(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const uint8_t* mask,
                                        const int32_t* pos, uint16_t* out, int M, int S, int Hq, int Hkv, int D, int Cmax,
                                        void* stream) {
  AttnArgs a{};
  a.q = q; a.kc = kc; a.vc = vc; a.mask = mask; a.pos_base = pos; a.out = out;
  a.S = S; a.Hq = Hq; a.Hkv = Hkv; a.D = D; a.Cmax = Cmax; a.M = M;
  a.scale = 1.0f / std::sqrt((float)D);
  HIPCHK(attention_prefill(a, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_fill_uniform(uint16_t* dst, size_t n, uint64_t seed, uint64_t tid, float scale, float offset,
                                   void* stream) {
  HIPCHK(fill_uniform_bf16(dst, n, seed, tid, scale, offset, (hipStream_t)stream));
  return 0;
}

// ---------------------------------------------------------------------------
// roofline probe: time one weight-streaming GEMV of the loaded model on the engine
// stream with HIP events (which: 0 q|k|v, 1 o_proj, 2 gate|up (SwiGLU), 3 down, 4 heads,
// 5 the persistent streaming decode stack of every layer, batch 1)
extern "C" int mtts_engine_time_gemv(mtts_engine* e, int which, int layer, int B, int iters, float* avg_ms,
                                     uint64_t* alg_bytes) {
  if (!e || !avg_ms || !alg_bytes || iters <= 0) return fail(MTTS_E_INVALID, "null argument");
  const mtts_config& c = e->c;
  if (which == 6 || which == 7) {
    // MossTTSLocal: the depth stack's gate|up (6) / down (7), the Local frame's dominant launches
    if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "no depth stack in a MossTTSDelay engine");
    hipSetDevice(e->device);
    return local_time_proj(e, which - 4, layer, B, iters, avg_ms, alg_bytes);
  }
  if (layer < 0 || layer >= c.layers || B <= 0 || B > c.max_batch) return fail(MTTS_E_INVALID, "bad layer/B");
  hipSetDevice(e->device);
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, I = c.inter;
  if (which == 5) {
    // the persistent streaming decode stack (pse.hip): ONE launch streams every layer, at the
    // engine's current decode position `layer` ignored; the cached keys up to pos are read
    if (e->lp || (B != 1 && B != 4) || !e->pse_takes(B)) return fail(MTTS_E_UNSUPPORTED, "persistent streaming decode inactive");
    hipStream_t s = e->stream;
    const Stack st = backbone_stack(e);
    int pos = 0;
    HIPCHK(hipMemcpy(&pos, &e->st->fwd_pos, sizeof(int), hipMemcpyDeviceToHost));
    pos = std::min(std::max(pos, 0), c.max_ctx - 1);
    HIPCHK(hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(e->d_pos), pos, 1, s));
    const int n_split = (c.max_ctx + CH_DECODE - 1) / CH_DECODE;
    hipEvent_t a, b;
    HIPCHK(hipEventCreate(&a));
    HIPCHK(hipEventCreate(&b));
    e->pse_choose(pos + 1);  // the form a decode step at this context takes (batch 1: short or long)
    if (B == 4) e->pse_now = true;
    if (B == 1 && !e->pse_now && !e->pse_long_now) return fail(MTTS_E_UNSUPPORTED, "no persistent form at this context");
    if (int rc = run_layers(e, st, 0, B, 1, e->d_pos, CH_DECODE, n_split, s)) return rc;
    HIPCHK(hipEventRecord(a, s));
    for (int i = 0; i < iters; ++i)
      if (int rc = run_layers(e, st, 0, B, 1, e->d_pos, CH_DECODE, n_split, s)) return rc;
    HIPCHK(hipEventRecord(b, s));
    HIPCHK(hipEventSynchronize(b));
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    hipEventDestroy(a);
    hipEventDestroy(b);
    uint32_t err = 0;
    HIPCHK(hipMemcpy(&err, e->pse_err(B), 4, hipMemcpyDeviceToHost));
    if (err) {
      hipMemset(e->pse_err(B), 0, 4);
      return fail(MTTS_E_HIP, "persistent streaming decode: a wait timed out (timing invalid)");
    }
    *avg_ms = ms / iters;
    // every layer's weights once + its K / V rows 0..pos read and row pos written
    const uint64_t wl = 2ull * ((uint64_t)e->qkv_rows * H + (uint64_t)H * Hq * D + 3ull * I * H);
    const uint64_t kv = 2ull * 2 * c.n_kv * D * (uint64_t)(pos + 1) * B;
    *alg_bytes = (uint64_t)st.layers * (wl + kv);
    return 0;
  }
  const LayerW& w = e->L[layer];
  hipStream_t s = e->stream;
  const bf16_t* W = nullptr;
  const bf16_t* x = e->xn;
  bf16_t* y = e->qkvb;
  const bf16_t* res = nullptr;
  int N = 0, K = H, epi = EPI_STORE, ps = 0, pp = 1, po = 0, ldx = H, ldy = 0, ldres = 0;
  uint64_t wrows = 0;
  switch (which) {
    case 0: W = w.qkv; N = e->qkv_rows; ldy = N; wrows = N; break;
    case 1: W = w.o; N = H; K = Hq * D; x = e->attnb; ldx = K; y = e->h; res = e->h; ldy = H; ldres = H; epi = EPI_RESADD; wrows = H; break;
    case 2: W = w.gu; N = I; y = e->act; ldy = I; epi = EPI_SWIGLU; wrows = 2ull * I; break;
    case 3: W = w.down; N = H; K = I; x = e->act; ldx = I; y = e->h; res = e->h; ldy = H; ldres = H; epi = EPI_RESADD; wrows = H; break;
    case 4: if (!e->heads) return fail(MTTS_E_UNSUPPORTED, "no joint heads in a MossTTSLocal engine");
      W = e->heads; N = e->heads_rows; y = e->logits; ldy = e->heads_ld; epi = EPI_LOGITS; ps = c.vocab;
      pp = e->audio_rows; po = e->audio_rows - 1; wrows = N; break;
    default: return fail(MTTS_E_INVALID, "bad which");
  }
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  // consecutive launches walk the layers (same shape, different weights), so the matrix is
  // not resident in the 256 MB MALL from the previous launch: HBM-honest timing
  auto wl = [&](int i) -> const bf16_t* {
    const LayerW& q = e->L[(layer + i) % c.layers];
    switch (which) {
      case 0: return q.qkv;
      case 1: return q.o;
      case 2: return q.gu;
      case 3: return q.down;
      default: return W;
    }
  };
  // the kernel instance the decode step launches: q|k|v and gate|up read RMSNorm(h) through
  // the same normed_input choice (fused prologue for small batches), the rest plain
  const Stack st = backbone_stack(e);
  // 17-32 rows: the decode step's packed-activation instances (xpk_index inputs / SwiGLU output);
  // the standalone RMSNorm runs once before the timed launches
  const bool pk = B > 16 && B <= 32 && e->xpack && which != 4;
  if (pk && (which == 0 || which == 2)) {
    GemvArgs g0 = gemv_args(W, e->xn, H, y, ldy, B, N, H);
    if (int rc = normed_input(e, st, g0, which == 0 ? w.in_norm : w.post_norm, B, s, 2)) return rc;
  }
  auto launch = [&](const bf16_t* Wi) -> int {
    if (pk) {
      GemvArgs g = gemv_args(Wi, x, ldx, y, ldy, B, N, K);
      g.res = res; g.ldres = ldres; g.x_packed = 1; g.y_packed = which == 2 ? 1 : 0;
      g.force_nw = e->nw[which]; g.force_u = e->nu[which];
      HIPCHK(gemv_ex(g, epi, s));
      return 0;
    }
    if (which == 0 || which == 2) {
      GemvArgs g = gemv_args(Wi, e->xn, H, y, ldy, B, N, H);
      if (int rc = normed_input(e, st, g, which == 0 ? w.in_norm : w.post_norm, B, s)) return rc;
      g.force_nw = e->nw[which]; g.force_u = e->nu[which];
      HIPCHK(gemv_ex(g, epi, s));
      return 0;
    }
    HIPCHK(gemv(Wi, x, ldx, y, ldy, res, ldres, B, N, K, epi, ps, pp, po, s));
    return 0;
  };
  HIPCHK(hipMemsetAsync(e->ss, 0, (size_t)B * (H / 16) * sizeof(float), s));
  if (int rc = launch(W)) return rc;
  HIPCHK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i)
    if (int rc = launch(wl(i + 1))) return rc;
  HIPCHK(hipEventRecord(b, s));
  HIPCHK(hipEventSynchronize(b));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  hipEventDestroy(a);
  hipEventDestroy(b);
  *avg_ms = ms / iters;
  // algorithmic bytes: weights once + activations in + outputs (+ residual read)
  *alg_bytes = 2ull * wrows * K + 2ull * B * K + 2ull * B * N * (res ? 2 : 1);
  return 0;
}

extern "C" size_t mtts_k_attn_decode_ws_bytes(int B, int Hq, int Hkv, int D, int Cmax) {
  return attn_decode_ws_bytes(B, Hq, Hkv, D, Cmax);
}
extern "C" int mtts_k_attn_decode(const uint16_t* qkv, const uint16_t* qn_w, const uint16_t* kn_w, const uint16_t* cos_t,
                                  const uint16_t* sin_t, uint16_t* kc, uint16_t* vc, const uint8_t* mask,
                                  const int32_t* pos, uint16_t* out, void* ws, int B, int Hq, int Hkv, int D, int Cmax,
                                  float eps, void* stream) {
  if (!ws) return fail(MTTS_E_INVALID, "workspace required");
  DecAttnArgs a{};
  a.qkv = qkv; a.qn_w = qn_w; a.kn_w = kn_w; a.cos_t = cos_t; a.sin_t = sin_t; a.kc = kc; a.vc = vc; a.mask = mask;
  a.pos = pos; a.out = out; a.Hq = Hq; a.Hkv = Hkv; a.D = D; a.Cmax = Cmax; a.eps = eps;
  a.cnt = reinterpret_cast<int*>(ws);
  a.part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + ((size_t)B * Hkv * sizeof(int) + 255) / 256 * 256);
  a.scale = 1.0f / std::sqrt((float)D);
  HIPCHK(attn_decode(a, B, (hipStream_t)stream));
  return 0;
}

extern "C" size_t mtts_k_gemv_splitk_ws_bytes(int N, int splits) {
  const int tiles = (N + 15) / 16;
  return ((size_t)tiles * sizeof(int) + 255) / 256 * 256 + gemv_splitk_ws_floats(tiles, splits) * sizeof(float);
}
extern "C" int mtts_k_gemv_splitk(const uint16_t* w, const uint16_t* x, int ldx, uint16_t* y, int ldy,
                                  const uint16_t* res, int ldres, int B, int N, int K, int splits, float* ss_out,
                                  int ld_ss_out, void* ws, void* stream) {
  if (!ws || !res || K % 32 || B <= 0 || B > 16 || splits < 2) return fail(MTTS_E_INVALID, "bad split-K GEMV args");
  GemvArgs a = gemv_args(w, x, ldx, y, ldy, B, N, K);
  a.res = res; a.ldres = ldres; a.ss_out = ss_out; a.ld_ss_out = ld_ss_out;
  const int tiles = (N + 15) / 16;
  int* cnt = reinterpret_cast<int*>(ws);
  float* part = reinterpret_cast<float*>(reinterpret_cast<char*>(ws) + ((size_t)tiles * sizeof(int) + 255) / 256 * 256);
  HIPCHK(gemv_splitk(a, splits, part, cnt, (hipStream_t)stream));
  return 0;
}
extern "C" int mtts_k_gemv_splitk_splits(int N, int K, int B) { return gemv_splitk_splits((N + 15) / 16, K / 32, B); }

extern "C" int mtts_k_gemm(const uint16_t* w, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                           int ldres, int M, int N, int K, int epi, float* ss_out, int ld_ss_out, void* stream) {
  if (K % 32) return fail(MTTS_E_INVALID, "K must be a multiple of 32");
  if (epi != EPI_STORE && epi != EPI_RESADD && epi != EPI_SWIGLU) return fail(MTTS_E_INVALID, "epi 0/1/2 only");
  GemvArgs a = gemv_args(w, x, ldx, y, ldy, M, N, K);
  a.res = res; a.ldres = ldres; a.ss_out = ss_out; a.ld_ss_out = ld_ss_out;
  HIPCHK(gemm_ex(a, epi, (hipStream_t)stream));
  return 0;
}

extern "C" int mtts_k_gemm_packed(const uint16_t* w, const uint16_t* x, uint16_t* y, int ldy, int y_packed,
                                  const uint16_t* res, int ldres, int M, int N, int K, int epi, float* ss_out,
                                  int ld_ss_out, float* ws, size_t ws_floats, void* stream) {
  if (K % 64 || M < 33) return fail(MTTS_E_INVALID, "packed prefill GEMM: K % 64 == 0 and M >= 33");
  if (epi != EPI_STORE && epi != EPI_RESADD && epi != EPI_SWIGLU) return fail(MTTS_E_INVALID, "epi 0/1/2 only");
  if (y_packed && epi != EPI_SWIGLU) return fail(MTTS_E_INVALID, "packed outputs: epi 2 only");
  GemvArgs a = gemv_args(w, x, K, y, ldy, M, N, K);
  a.res = res; a.ldres = ldres; a.ss_out = ss_out; a.ld_ss_out = ld_ss_out;
  a.x_packed = 1; a.y_packed = y_packed ? 1 : 0; a.pk_tiles = (M + 15) / 16;
  a.ws = ws; a.ws_floats = ws ? ws_floats : 0;
  HIPCHK(gemm_ex(a, epi, (hipStream_t)stream));
  return 0;
}

// full-control GEMV (fused norm prologue, sum-of-squares epilogue, waves-per-block override)
extern "C" int mtts_k_gemv_ex(const uint16_t* w, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                              int ldres, int B, int N, int K, int epi, const float* ss_in, int ld_ss, int n_ss,
                              const uint16_t* norm_w, float eps, float* ss_out, int ld_ss_out, int force_nw,
                              void* stream) {
  GemvArgs a = gemv_args(w, x, ldx, y, ldy, B, N, K);
  a.res = res; a.ldres = ldres;
  a.ss_in = ss_in; a.ld_ss = ld_ss; a.n_ss = n_ss; a.nw = norm_w; a.eps = eps;
  a.ss_out = ss_out; a.ld_ss_out = ld_ss_out; a.force_nw = force_nw;
  if (epi == EPI_LOGITS) return fail(MTTS_E_INVALID, "use mtts_k_gemv for logits");
  HIPCHK(gemv_ex(a, epi, (hipStream_t)stream));
  return 0;
}
