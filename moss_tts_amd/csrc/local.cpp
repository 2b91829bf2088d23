// MossTTSLocal on the engine: the Qwen3 backbone of engine.cpp plus the per-frame depth stage
// of `CustomMixin._sample` (moss_tts_local/modeling_moss_tts.py:377-456):
//
//   g   = final-normed backbone state of the last position                     (:384-390)
//   x_0 = speech_embedding_to_local_mlp(g)                                      (:395)
//   for channel i < n_ch = min(1+n_vq, 1+n_vq_for_inference):
//     local transformer over x_0..x_i (4 Qwen3 layers, no RoPE, causal)        (:397-401)
//     logits_i = lm_heads[i](MossTTSRMSNorm_i(local_to_speech_embedding_mlps[i](h_i)))  (:402-410)
//     pad column -inf for i >= 1; token = argmax                               (:411-419)
//     x_{i+1} = speech_embedding_to_local_mlp(embedding_list[i](token))        (:421-423)
//   finished rows emit eos / pad; append; stop on eos in channel 0             (:425-446)
//
// The reference re-runs the local transformer over the whole prefix per channel; attention
// is causal and position-free, so the depth stack keeps a KV cache over channel positions
// instead (same function, one new position per channel).  Everything here is launched on
// the engine stream; one decode frame is captured as a hipGraph per (batch, n_ch).
#include "engine_internal.h"

constexpr int LOCAL_CMAX = 64;  // channel positions of the depth stack's KV cache (1 + n_vq <= 64)

struct LocalParts {
  int LH = 0, LL = 0, LI = 0, F = 0, C = 0, qkv_rows = 0;
  std::vector<LayerW> L;
  bf16_t* norm = nullptr;                       // local_transformer.norm
  bf16_t *mi_gu = nullptr, *mi_down = nullptr;  // speech_embedding_to_local_mlp (gate|up interleaved), down
  std::vector<bf16_t*> mo_gu, mo_down;          // local_to_speech_embedding_mlps[i]
  std::vector<bf16_t*> ln, head;                // layer_norm_before_lm_heads[i], lm_heads[i] (packed)
  uint64_t backbone_bytes = 0, channel_bytes = 0, text_head_bytes = 0, audio_head_bytes = 0;
  // capacity
  bf16_t *kc = nullptr, *vc = nullptr;
  size_t layer_kv = 0;
  uint8_t* mask = nullptr;
  int* lpos = nullptr;  // [LOCAL_CMAX]: position i of channel i
  bf16_t *h = nullptr, *xn = nullptr, *qkvb = nullptr, *attnb = nullptr, *act = nullptr;
  float* ss = nullptr;
  float* part = nullptr;
  int* att_cnt = nullptr;
  bf16_t *hid = nullptr, *eb = nullptr, *actF = nullptr, *zero = nullptr, *z = nullptr, *zn = nullptr, *logits = nullptr;
  int ld_logits = 0;
  int64_t* next = nullptr;  // [Bmax][C] tokens of the frame being built (the next forward's input)
  int* finished = nullptr;  // [Bmax]
  uint8_t* seen = nullptr;  // [Bmax][C][audio_rows] channel histories (repetition penalty)
  int n_ch = 0;
  std::vector<ChSampling> ch_table;  // mtts_local_set_sampling: per-channel processors (empty: from mtts_sampling)
  bool no_graph = false;
  std::unordered_map<long long, hipGraphExec_t> graphs;
  // one channel's depth stage as one persistent launch (lpse.hip); MTTS_LPSE=1 turns it on.  Off by
  // default: 9.98 ms per frame against 8.40 for the per-op launches (profiles/r04_b_*)
  bool lpse = false, lpse_ok = false;
  void* lpse_ws = nullptr;  // lpse_ws_bytes(), zero-filled
  int lpse_timeouts = 0;
  int* mask_bad = nullptr;  // row_pad_count's flag: some row of the mask is not left-padded
};

static Stack local_stack(mtts_engine* e) {
  const LocalParts& p = *e->lp;
  const mtts_config& c = e->c;
  Stack st;
  st.L = p.L.data(); st.layers = p.LL; st.H = p.LH; st.Hq = c.n_heads; st.Hkv = c.n_kv; st.D = c.head_dim;
  st.I = p.LI; st.qkv_rows = p.qkv_rows;
  st.kc = p.kc; st.vc = p.vc; st.layer_kv = p.layer_kv; st.Cmax = LOCAL_CMAX;
  st.cos_t = nullptr; st.sin_t = nullptr;  // MossTTSLocalTransformer: no positional embedding
  st.mask = p.mask;
  st.h = p.h; st.xn = p.xn; st.qkvb = p.qkvb; st.qb = nullptr; st.attnb = p.attnb; st.act = p.act;
  st.ss = p.ss; st.part = p.part; st.att_cnt = p.att_cnt;
  // <= 33 channel positions: one attention block per head, so it writes its rows itself and
  // the depth o_proj reads them as a plain GEMV (no partial merge in its prologue)
  static const bool no_direct = getenv("MTTS_LOCAL_ATTN_MERGE") && getenv("MTTS_LOCAL_ATTN_MERGE")[0] == '1';
  st.attn_direct = !no_direct && LOCAL_CMAX <= attn_decode_keys_per_block();
  // the direct form's block: 4 waves (128 keys) hold the <= 33 positions, a 4-wave merge instead
  // of 8 (frame 8.57 -> 8.53 ms in two same-box pairs; MTTS_LOCAL_ATTN_NWV=8 for A/B)
  static const int nwv = getenv("MTTS_LOCAL_ATTN_NWV") ? atoi(getenv("MTTS_LOCAL_ATTN_NWV")) : 4;
  if (st.attn_direct && (nwv == 4 || nwv == 8) && LOCAL_CMAX <= 32 * nwv) st.attn_nwv = nwv;
  return st;
}

int local_create(mtts_engine* e) {
  const mtts_config& c = e->c;
  e->lp = new LocalParts();
  LocalParts& p = *e->lp;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv;
  p.LH = c.local_hidden; p.LL = c.local_layers; p.LI = c.local_inter; p.F = c.local_mlp_ffn; p.C = c.n_vq + 1;
  p.qkv_rows = (Hq + 2 * Hkv) * D;
  if (const char* v = getenv("MTTS_LOCAL_NO_GRAPH")) p.no_graph = v[0] == '1';
  if (const char* v = getenv("MTTS_LPSE")) p.lpse = v[0] == '1';
  const int LH = p.LH, LI = p.LI, F = p.F, C = p.C;
  int rc = 0;
  p.L.resize(p.LL);
  uint64_t lb = 0;
  for (int l = 0; l < p.LL; ++l) {
    LayerW& w = p.L[l];
    if ((rc = e->alloc(&w.qkv, packed_bytes(p.qkv_rows, LH) / 2)) || (rc = e->alloc(&w.o, packed_bytes(LH, Hq * D) / 2)) ||
        (rc = e->alloc(&w.gu, packed_bytes(2 * LI, LH) / 2)) || (rc = e->alloc(&w.down, packed_bytes(LH, LI) / 2)) ||
        (rc = e->alloc(&w.in_norm, LH)) || (rc = e->alloc(&w.post_norm, LH)) || (rc = e->alloc(&w.q_norm, D)) ||
        (rc = e->alloc(&w.k_norm, D)))
      return rc;
    hipMemset(w.qkv, 0, packed_bytes(p.qkv_rows, LH));
    hipMemset(w.o, 0, packed_bytes(LH, Hq * D));
    lb += 2ull * ((uint64_t)p.qkv_rows * LH + (uint64_t)LH * Hq * D + 2ull * LI * LH + (uint64_t)LH * LI) + 4ull * LH + 4ull * D;
  }
  if ((rc = e->alloc(&p.norm, LH)) || (rc = e->alloc(&p.mi_gu, packed_bytes(2 * F, H) / 2)) ||
      (rc = e->alloc(&p.mi_down, packed_bytes(LH, F) / 2)))
    return rc;
  p.mo_gu.assign(C, nullptr); p.mo_down.assign(C, nullptr); p.ln.assign(C, nullptr); p.head.assign(C, nullptr);
  for (int i = 0; i < C; ++i) {
    const int V = i == 0 ? c.vocab : e->audio_rows;
    if ((rc = e->alloc(&p.mo_gu[i], packed_bytes(2 * F, LH) / 2)) || (rc = e->alloc(&p.mo_down[i], packed_bytes(H, F) / 2)) ||
        (rc = e->alloc(&p.ln[i], H)) || (rc = e->alloc(&p.head[i], packed_bytes(V, H) / 2)))
      return rc;
    hipMemset(p.head[i], 0, packed_bytes(V, H));  // pad rows of the last tile
    hipMemset(p.mo_down[i], 0, packed_bytes(H, F));
  }
  hipMemset(p.mi_down, 0, packed_bytes(LH, F));
  if ((rc = e->alloc(&p.mask_bad, 1))) return rc;
  // weight bytes one frame streams: backbone once, then per channel the depth stack, its norm,
  // both adapters, the channel norm and the channel head
  p.lpse_ok = lpse_supported(e->device, 1, p.LL, LH, Hq, Hkv, D, LI, F, H, LOCAL_CMAX) &&
              p.qkv_rows == (Hq + 2 * Hkv) * D && C <= LPSE_MAX_CHANNELS;
  if (p.lpse_ok) {
    if ((rc = e->alloc(reinterpret_cast<unsigned char**>(&p.lpse_ws), lpse_ws_bytes()))) return rc;
    HIPCHK(hipMemset(p.lpse_ws, 0, lpse_ws_bytes()));
  }
  p.backbone_bytes = e->step_weight_bytes;
  p.channel_bytes = lb + 2ull * LH + 2ull * (2ull * F * H + (uint64_t)LH * F) + 2ull * (2ull * F * LH + (uint64_t)H * F) + 2ull * H;
  p.text_head_bytes = 2ull * c.vocab * H;
  p.audio_head_bytes = 2ull * e->audio_rows * H;
  e->step_weight_bytes = p.backbone_bytes + C * p.channel_bytes + p.text_head_bytes + (C - 1) * p.audio_head_bytes;
  return 0;
}

int local_alloc_capacity(mtts_engine* e) {
  const mtts_config& c = e->c;
  LocalParts& p = *e->lp;
  const int B = c.max_batch, H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv;
  const int LH = p.LH, F = p.F, C = p.C;
  int rc = 0;
  e->cap_mode = true;
  p.layer_kv = (size_t)B * Hkv * LOCAL_CMAX * D;
  const size_t ns = attn_decode_splits(LOCAL_CMAX);
  p.ld_logits = (c.vocab + 7) / 8 * 8;
  if ((rc = e->alloc(&p.kc, p.layer_kv * p.LL)) || (rc = e->alloc(&p.vc, p.layer_kv * p.LL)) ||
      (rc = e->alloc(&p.mask, (size_t)B * LOCAL_CMAX)) || (rc = e->alloc(&p.lpos, LOCAL_CMAX)) ||
      (rc = e->alloc(&p.h, (size_t)B * LH)) || (rc = e->alloc(&p.xn, (size_t)B * LH)) ||
      (rc = e->alloc(&p.qkvb, (size_t)B * p.qkv_rows)) || (rc = e->alloc(&p.attnb, (size_t)B * Hq * D)) ||
      (rc = e->alloc(&p.act, (size_t)B * p.LI)) || (rc = e->alloc(&p.ss, (size_t)B * (LH / 16))) ||
      (rc = e->alloc(&p.part, (size_t)B * ns * Hq * (D + 2))) || (rc = e->alloc(&p.att_cnt, (size_t)B * Hkv)) ||
      (rc = e->alloc(&p.hid, (size_t)B * H)) || (rc = e->alloc(&p.eb, (size_t)B * H)) ||
      (rc = e->alloc(&p.actF, (size_t)B * F)) || (rc = e->alloc(&p.zero, (size_t)B * LH)) ||
      (rc = e->alloc(&p.z, (size_t)B * H)) || (rc = e->alloc(&p.zn, (size_t)B * H)) ||
      (rc = e->alloc(&p.logits, (size_t)B * p.ld_logits)) || (rc = e->alloc(&p.next, (size_t)B * C)) ||
      (rc = e->alloc(&p.finished, B)) || (rc = e->alloc(&p.seen, (size_t)B * C * e->audio_rows)))
    return rc;
  e->cap_mode = false;
  std::vector<int> pos(LOCAL_CMAX);
  for (int i = 0; i < LOCAL_CMAX; ++i) pos[i] = i;
  HIPCHK(hipMemcpy(p.lpos, pos.data(), LOCAL_CMAX * sizeof(int), hipMemcpyHostToDevice));
  HIPCHK(hipMemset(p.mask, 1, (size_t)B * LOCAL_CMAX));  // the depth stack attends to every channel so far
  HIPCHK(hipMemset(p.att_cnt, 0, (size_t)B * Hkv * sizeof(int)));
  HIPCHK(hipMemset(p.zero, 0, (size_t)B * LH * 2));
  HIPCHK(hipMemset(p.next, 0, (size_t)B * C * 8));
  HIPCHK(hipMemset(p.seen, 0, (size_t)B * C * e->audio_rows));
  return 0;
}

// The persistent channel launch's error word (lpse.hip: a bounded wait timed out).  When set:
// clear it, turn the launch off for this engine (the captured frames are re-captured on the
// per-op launches) and report true; synchronises the stream.
bool local_lpse_tripped(mtts_engine* e, hipStream_t s) {
  LocalParts* p = e->lp;
  if (!p || !p->lpse_ws) return false;
  uint32_t err = 0;
  if (hipStreamSynchronize(s) != hipSuccess ||
      hipMemcpy(&err, lpse_err_word(p->lpse_ws), 4, hipMemcpyDeviceToHost) != hipSuccess || !err)
    return false;
  hipMemset(p->lpse_ws, 0, lpse_ws_bytes());
  p->lpse = false;
  p->lpse_timeouts += 1;
  local_clear_graphs(e);
  fprintf(stderr, "libmtts: persistent channel launch timed out (code %u; device shared with other work?); "
                  "this engine continues on the per-op launches\n", err);
  return true;
}

int local_lpse_inject(mtts_engine* e) {
  LocalParts* p = e->lp;
  if (!p || !p->lpse_ws) return fail(MTTS_E_INVALID, "no persistent channel launch state");
  HIPCHK(hipStreamSynchronize(e->stream));
  const uint32_t code = 0x7e57u;
  HIPCHK(hipMemcpy(lpse_err_word(p->lpse_ws), &code, 4, hipMemcpyHostToDevice));
  return 0;
}

void local_clear_graphs(mtts_engine* e) {
  if (!e->lp) return;
  for (auto& kv : e->lp->graphs) hipGraphExecDestroy(kv.second);
  e->lp->graphs.clear();
}

void local_destroy(mtts_engine* e) {
  if (!e->lp) return;
  local_clear_graphs(e);
  delete e->lp;
  e->lp = nullptr;
}

// ---------------------------------------------------------------------------
// weights by the reference's state_dict names (moss_tts_local/modeling_moss_tts.py:495-512,
// :560-600): backbone names get the engine's own, the depth stage lands here
static bool channel_index(const char* name, const char* prefix, int C, int* i, std::string* rest) {
  const size_t n = std::strlen(prefix);
  if (std::strncmp(name, prefix, n) != 0) return false;
  char* end = nullptr;
  const long v = std::strtol(name + n, &end, 10);
  if (end == name + n || *end != '.' || v < 0 || v >= C) return false;
  *i = (int)v;
  *rest = std::string(end + 1);
  return true;
}

int local_load_weight(mtts_engine* e, const char* name, const void* src, size_t bytes, int on_dev, int* rc) {
  const mtts_config& c = e->c;
  LocalParts& p = *e->lp;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv;
  const int LH = p.LH, F = p.F, C = p.C;
  int i = -1;
  std::string rest;
  WTarget t;
  auto bad = [&](const char* why) {
    *rc = fail(MTTS_E_INVALID, std::string(why) + ": " + name);
    return 1;
  };
  // backbone: renamed onto the engine's names
  if (channel_index(name, "model.embedding_list.", C, &i, &rest)) {
    if (rest != "weight") return bad("unknown weight");
    const std::string to = i == 0 ? std::string("language_model.embed_tokens.weight") : "emb_ext." + std::to_string(i - 1) + ".weight";
    *rc = load_weight_impl(e, to.c_str(), src, bytes, on_dev);
    return 1;
  }
  if (!std::strcmp(name, "model.language_model.embed_tokens.weight")) {  // unused: inputs_embeds path (:515-530)
    *rc = 0;
    return 1;
  }
  if (!std::strncmp(name, "model.language_model.", 21)) {
    *rc = load_weight_impl(e, name + 6, src, bytes, on_dev);
    return 1;
  }
  // depth stage
  if (!std::strncmp(name, "local_transformer.layers.", 25)) {
    if (!channel_index(name, "local_transformer.layers.", p.LL, &i, &rest)) return bad("bad layer");
    if (!layer_target(p.L[i], rest, LH, p.LI, Hq, Hkv, D, &t)) return bad("unknown weight");
  } else if (!std::strcmp(name, "local_transformer.norm.weight")) {
    t.dst = p.norm; t.expect = LH;
  } else if (!std::strncmp(name, "speech_embedding_to_local_mlp.", 30)) {
    rest = name + 30;
    t.pack = true;
    if (rest == "gate_proj.weight") { t.dst = p.mi_gu; t.rows = F; t.K = H; t.inter = 1; t.which = 0; }
    else if (rest == "up_proj.weight") { t.dst = p.mi_gu; t.rows = F; t.K = H; t.inter = 1; t.which = 1; }
    else if (rest == "down_proj.weight") { t.dst = p.mi_down; t.rows = LH; t.K = F; }
    else return bad("unknown weight");
    t.expect = (size_t)t.rows * t.K;
  } else if (channel_index(name, "local_to_speech_embedding_mlps.", C, &i, &rest)) {
    t.pack = true;
    if (rest == "gate_proj.weight") { t.dst = p.mo_gu[i]; t.rows = F; t.K = LH; t.inter = 1; t.which = 0; }
    else if (rest == "up_proj.weight") { t.dst = p.mo_gu[i]; t.rows = F; t.K = LH; t.inter = 1; t.which = 1; }
    else if (rest == "down_proj.weight") { t.dst = p.mo_down[i]; t.rows = H; t.K = F; }
    else return bad("unknown weight");
    t.expect = (size_t)t.rows * t.K;
  } else if (channel_index(name, "layer_norm_before_lm_heads.", C, &i, &rest)) {
    if (rest != "weight") return bad("unknown weight");
    t.dst = p.ln[i]; t.expect = H;
  } else if (channel_index(name, "lm_heads.", C, &i, &rest)) {
    if (rest != "weight") return bad("unknown weight");
    t.pack = true; t.dst = p.head[i]; t.rows = i == 0 ? c.vocab : e->audio_rows; t.K = H;
    t.expect = (size_t)t.rows * H;
  } else {
    return 0;
  }
  *rc = store_weight(e, t, name, src, bytes, on_dev);
  return 1;
}

// same tensor order / init as oracle.moss_local.weight_specs + _scale
int local_init_random(mtts_engine* e, uint64_t seed) {
  const mtts_config& c = e->c;
  const LocalParts& p = *e->lp;
  const int H = c.hidden, D = c.head_dim, Hq = c.n_heads, Hkv = c.n_kv, C = p.C, LH = p.LH, F = p.F;
  struct Spec { std::string name; size_t rows, cols; int kind; };  // 0 lin/head 1 norm 2 emb
  std::vector<Spec> sp;
  sp.push_back({"model.embedding_list.0.weight", (size_t)c.vocab, (size_t)H, 2});
  for (int i = 1; i < C; ++i) sp.push_back({"model.embedding_list." + std::to_string(i) + ".weight", (size_t)e->audio_rows, (size_t)H, 2});
  auto layer = [&](const std::string& pf, int Hs, int I) {
    sp.push_back({pf + "self_attn.q_proj.weight", (size_t)Hq * D, (size_t)Hs, 0});
    sp.push_back({pf + "self_attn.k_proj.weight", (size_t)Hkv * D, (size_t)Hs, 0});
    sp.push_back({pf + "self_attn.v_proj.weight", (size_t)Hkv * D, (size_t)Hs, 0});
    sp.push_back({pf + "self_attn.o_proj.weight", (size_t)Hs, (size_t)Hq * D, 0});
    sp.push_back({pf + "self_attn.q_norm.weight", 1, (size_t)D, 1});
    sp.push_back({pf + "self_attn.k_norm.weight", 1, (size_t)D, 1});
    sp.push_back({pf + "mlp.gate_proj.weight", (size_t)I, (size_t)Hs, 0});
    sp.push_back({pf + "mlp.up_proj.weight", (size_t)I, (size_t)Hs, 0});
    sp.push_back({pf + "mlp.down_proj.weight", (size_t)Hs, (size_t)I, 0});
    sp.push_back({pf + "input_layernorm.weight", 1, (size_t)Hs, 1});
    sp.push_back({pf + "post_attention_layernorm.weight", 1, (size_t)Hs, 1});
  };
  for (int l = 0; l < c.layers; ++l) layer("model.language_model.layers." + std::to_string(l) + ".", H, c.inter);
  sp.push_back({"model.language_model.norm.weight", 1, (size_t)H, 1});
  for (int l = 0; l < p.LL; ++l) layer("local_transformer.layers." + std::to_string(l) + ".", LH, p.LI);
  sp.push_back({"local_transformer.norm.weight", 1, (size_t)LH, 1});
  sp.push_back({"speech_embedding_to_local_mlp.gate_proj.weight", (size_t)F, (size_t)H, 0});
  sp.push_back({"speech_embedding_to_local_mlp.up_proj.weight", (size_t)F, (size_t)H, 0});
  sp.push_back({"speech_embedding_to_local_mlp.down_proj.weight", (size_t)LH, (size_t)F, 0});
  for (int i = 0; i < C; ++i) {
    const std::string pf = "local_to_speech_embedding_mlps." + std::to_string(i) + ".";
    sp.push_back({pf + "gate_proj.weight", (size_t)F, (size_t)LH, 0});
    sp.push_back({pf + "up_proj.weight", (size_t)F, (size_t)LH, 0});
    sp.push_back({pf + "down_proj.weight", (size_t)H, (size_t)F, 0});
  }
  for (int i = 0; i < C; ++i) sp.push_back({"layer_norm_before_lm_heads." + std::to_string(i) + ".weight", 1, (size_t)H, 1});
  sp.push_back({"lm_heads.0.weight", (size_t)c.vocab, (size_t)H, 0});
  for (int i = 1; i < C; ++i) sp.push_back({"lm_heads." + std::to_string(i) + ".weight", (size_t)e->audio_rows, (size_t)H, 0});
  size_t mx = 0;
  for (auto& s : sp) mx = std::max(mx, s.rows * s.cols);
  int rc = ensure_staging(e, mx * 2);
  if (rc) return rc;
  for (size_t tid = 0; tid < sp.size(); ++tid) {
    const Spec& s = sp[tid];
    float scale = 1.f, offset = 0.f;
    if (s.kind == 0) scale = (float)std::sqrt(3.0 / (double)s.cols);
    else if (s.kind == 1) { scale = 0.25f; offset = 1.0f; }
    HIPCHK(fill_uniform_bf16(e->staging, s.rows * s.cols, seed, tid, scale, offset, e->stream));
    rc = load_weight_impl(e, s.name.c_str(), e->staging, s.rows * s.cols * 2, 1);
    if (rc) return rc;
  }
  return 0;
}

// One depth-stack projection at the decode shape, launched as run_layers launches it (gate|up:
// Qwen3RMSNorm prologue + SwiGLU epilogue; down: residual add + sum-of-squares epilogue, split-K
// where proj() picks it).  Consecutive launches walk the depth layers the way the channel loop
// does, so the weights come from wherever the frame finds them (the 4 depth layers stay in the
// MALL across a frame's 33 channels); the algorithmic bytes count them once per launch.
int local_time_proj(mtts_engine* e, int proj_kind, int layer, int B, int iters, float* avg_ms, uint64_t* alg_bytes) {
  const LocalParts& p = *e->lp;
  if (proj_kind != 2 && proj_kind != 3) return fail(MTTS_E_INVALID, "depth projection: 2 (gate|up) or 3 (down)");
  if (layer < 0 || layer >= p.LL || B <= 0 || B > e->c.max_batch || iters <= 0) return fail(MTTS_E_INVALID, "bad layer/B");
  const Stack st = local_stack(e);
  const int H = st.H, I = st.I, NT = H / 16;
  hipStream_t s = e->stream;
  HIPCHK(hipMemsetAsync(st.ss, 0, (size_t)B * NT * sizeof(float), s));
  auto launch = [&](int l) -> int {
    const LayerW& w = st.L[l % p.LL];
    if (proj_kind == 2) {
      GemvArgs g = gemv_args(w.gu, st.xn, H, st.act, I, B, I, H);
      if (int rc = normed_input(e, st, g, w.post_norm, B, s, 0)) return rc;
      g.force_nw = e->nw[2]; g.force_u = e->nu[2];
      HIPCHK(proj(e, g, EPI_SWIGLU, s));
    } else {
      GemvArgs g = gemv_args(w.down, st.act, I, st.h, H, B, H, I);
      g.res = st.h; g.ldres = H; g.ss_out = st.ss; g.ld_ss_out = NT; g.force_nw = e->nw[3]; g.force_u = e->nu[3];
      HIPCHK(proj(e, g, EPI_RESADD, s));
    }
    return 0;
  };
  if (int rc = launch(layer)) return rc;
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  HIPCHK(hipEventRecord(a, s));
  for (int i = 0; i < iters; ++i)
    if (int rc = launch(layer + 1 + i)) return rc;
  HIPCHK(hipEventRecord(b, s));
  HIPCHK(hipEventSynchronize(b));
  float ms = 0.f;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  hipEventDestroy(a);
  hipEventDestroy(b);
  *avg_ms = ms / iters;
  const uint64_t rows = proj_kind == 2 ? 2ull * I : (uint64_t)H, K = proj_kind == 2 ? H : I,
                 N = proj_kind == 2 ? I : H;
  *alg_bytes = 2ull * rows * K + 2ull * B * K + 2ull * B * N * (proj_kind == 3 ? 2 : 1);
  return 0;
}

// ---------------------------------------------------------------------------
// speech_embedding_to_local_mlp(x) -> the depth stack's residual stream (+ its per-16-column
// sums of squares for the first layer's input norm); x [B, H], or with tok != nullptr the
// embedding rows x + tok[b * ld_tok] * H gathered by the gate|up GEMV itself
static int mlp_in(mtts_engine* e, const Stack& st, const bf16_t* x, int B, hipStream_t s,
                  const int64_t* tok = nullptr, int ld_tok = 0) {
  LocalParts& p = *e->lp;
  const int H = e->c.hidden, LH = p.LH, F = p.F;
  GemvArgs g = gemv_args(p.mi_gu, x, H, p.actF, F, B, F, H);
  g.xtok = tok; g.ld_xtok = ld_tok;
  HIPCHK(gemv_ex(g, EPI_SWIGLU, s));
  g = gemv_args(p.mi_down, p.actF, F, st.h, LH, B, LH, F);
  g.res = p.zero; g.ldres = LH; g.ss_out = st.ss; g.ld_ss_out = LH / 16;  // bf16(0 + y) == y
  HIPCHK(gemv_ex(g, EPI_RESADD, s));
  return 0;
}

// MTTS_LOCAL_SEP_EMBED=1: the channel embedding as its own launch (the A/B side of the gather)
static bool local_sep_embed() {
  static const bool v = getenv("MTTS_LOCAL_SEP_EMBED") && getenv("MTTS_LOCAL_SEP_EMBED")[0] == '1';
  return v;
}

// The depth loop of one frame from the backbone state p.hid [B, H].  Greedy tokens go to
// p.next[b][i]; forced != nullptr feeds forced[b * ld_forced + i] to channel i+1 instead
// (teacher forcing); dump != nullptr receives channel i's logits at dump + i*B*ld_dump.
bool local_lpse_takes(const mtts_engine* e, int B) {
  const LocalParts* p = e->lp;
  return p && p->lpse && p->lpse_ok && B >= 1 && B <= LPSE_MAXB;
}

// channel i's depth stage (adapter in, the depth layers, local_transformer.norm, adapter out -> p.z)
// as one persistent launch; its input rows: the backbone state (i == 0) or the embedding rows of
// channel i - 1's tokens tok[b * ld_tok]
static int lpse_launch(mtts_engine* e, int B, int i, const int64_t* tok, int ld_tok, hipStream_t s) {
  LocalParts& p = *e->lp;
  const mtts_config& c = e->c;
  LpseArgs a{};
  for (int l = 0; l < p.LL; ++l) {
    const LayerW& w = p.L[l];
    a.L[l] = LpseLayer{w.qkv, w.o, w.gu, w.down, w.in_norm, w.post_norm, w.q_norm, w.k_norm};
  }
  a.layers = p.LL;
  if (i == 0) {
    a.in = p.hid;
  } else {
    a.in = i - 1 == 0 ? e->emb_text : e->emb_audio + (size_t)(i - 2) * e->audio_rows * c.hidden;
    a.tok = tok;
    a.ld_tok = ld_tok;
  }
  a.mi_gu = p.mi_gu; a.mi_down = p.mi_down; a.norm = p.norm; a.mo_gu = p.mo_gu[i]; a.mo_down = p.mo_down[i];
  a.h = p.h; a.qkvb = p.qkvb; a.attnb = p.attnb; a.act = p.act; a.actF = p.actF; a.z = p.z; a.ss = p.ss;
  a.kc = p.kc; a.vc = p.vc; a.layer_kv = p.layer_kv;
  a.B = B; a.pos = i; a.eps = c.rms_eps; a.scale = 1.0f / std::sqrt((float)c.head_dim);
  a.trace = e->pse_trace;  // (MTTS_PSE_TRACE=1: the stamps of the last channel launch)
  HIPCHK(lpse_channel(a, p.lpse_ws, s));
  return 0;
}

static int local_depth(mtts_engine* e, int B, int n_ch, const int64_t* forced, int ld_forced, bf16_t* dump, int ld_dump,
                       hipStream_t s) {
  LocalParts& p = *e->lp;
  const mtts_config& c = e->c;
  const int H = c.hidden, LH = p.LH, F = p.F, C = p.C;
  const Stack st = local_stack(e);
  const bool lp = local_lpse_takes(e, B);
  if (!lp)
    if (int rc = mlp_in(e, st, p.hid, B, s)) return rc;
  for (int i = 0; i < n_ch; ++i) {
    if (lp) {
      const int64_t* tok = i == 0 ? nullptr : (forced ? forced + (i - 1) : p.next + (i - 1));
      if (int rc = lpse_launch(e, B, i, tok, forced ? ld_forced : C, s)) return rc;
    } else {
      if (int rc = run_layers(e, st, 0, B, 1, p.lpos + i, CH_DECODE, 1, s)) return rc;
      GemvArgs g = gemv_args(p.mo_gu[i], st.xn, LH, p.actF, F, B, F, LH);
      if (int rc = normed_input(e, st, g, p.norm, B, s)) return rc;  // local_transformer.norm (Qwen3RMSNorm)
      HIPCHK(gemv_ex(g, EPI_SWIGLU, s));
      g = gemv_args(p.mo_down[i], p.actF, F, p.z, H, B, H, F);
      HIPCHK(gemv_ex(g, EPI_STORE, s));
    }
    HIPCHK(moss_rmsnorm(p.z, p.ln[i], p.zn, B, H, c.rms_eps, s));
    const int V = i == 0 ? c.vocab : e->audio_rows;
    bf16_t* lg = dump ? dump + (size_t)i * B * ld_dump : p.logits;
    const int ldl = dump ? ld_dump : p.ld_logits;
    GemvArgs g = gemv_args(p.head[i], p.zn, H, lg, ldl, B, V, H);
    if (i == 0) { g.pad_start = V; }
    else { g.pad_start = 0; g.pad_period = e->audio_rows; g.pad_off = c.audio_pad_code; }
    HIPCHK(gemv_ex(g, EPI_LOGITS, s));
    if (dump) HIPCHK(argmax_rows(lg, ldl, V, p.next + i, C, B, s));  // teacher forcing: no generate state
    else HIPCHK(local_pick(e->st, lg, ldl, V, i, p.seen, p.next, C, B, e->wide_hist, s));
    if (i + 1 < n_ch && !lp) {
      const int64_t* tok = forced ? forced + i : p.next + i;
      const bf16_t* table = i == 0 ? e->emb_text : e->emb_audio + (size_t)(i - 1) * e->audio_rows * H;
      const int ld_tok = forced ? ld_forced : C;
      if (B <= 16 && !local_sep_embed()) {  // the adapter's gate|up gathers the rows itself
        if (int rc = mlp_in(e, st, table, B, s, tok, ld_tok)) return rc;
      } else {
        HIPCHK(embed(tok, 1, table, nullptr, e->audio_rows, H, p.eb, B, s, nullptr, 0, ld_tok));
        if (int rc = mlp_in(e, st, p.eb, B, s)) return rc;
      }
    }
  }
  return 0;
}

static int local_frame_end(mtts_engine* e, hipStream_t s) {
  LocalParts& p = *e->lp;
  HIPCHK(local_finalize(e->st, p.next, p.finished, e->gen_ids, e->mask, p.seen, e->gen_B, p.C, p.n_ch,
                        e->c.eos_token_id, e->c.audio_pad_code, s));
  return 0;
}

static int local_step_launch(mtts_engine* e, hipStream_t s) {
  LocalParts& p = *e->lp;
  const int B = e->gen_B;
  const int n_split = (e->c.max_ctx + CH_DECODE - 1) / CH_DECODE;
  int rc = forward_rows(e, p.next, 0, B, 1, &e->st->fwd_pos, CH_DECODE, n_split, nullptr, s, nullptr, false, p.hid,
                        p.n_ch);
  if (!rc) rc = local_depth(e, B, p.n_ch, nullptr, 0, nullptr, 0, s);
  if (!rc) rc = local_frame_end(e, s);
  return rc;
}

static int n_channels(const mtts_engine* e, int n_vq_inf) {
  const int C = e->c.n_vq + 1;
  return n_vq_inf < 0 ? C : std::min(C, 1 + n_vq_inf);
}

// The backbone rows' RoPE offsets from e->mask's first n columns (the rows' left pads).
// GenerationMixin's positions are cumsum(mask) - 1 (transformers/generation/utils.py:751-773),
// which is slot - pads only for a left-padded row, so any other mask is refused (one host sync,
// outside stream capture) rather than decoded with shifted positions.
static int left_pad_offsets(mtts_engine* e, int n, int B, hipStream_t s) {
  LocalParts& p = *e->lp;
  HIPCHK(hipMemsetAsync(p.mask_bad, 0, sizeof(int), s));
  HIPCHK(row_pad_count(e->mask, e->c.max_ctx, n, B, e->rope_off, p.mask_bad, s));
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIPCHK(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) return 0;
  int bad = 0;
  HIPCHK(hipMemcpyAsync(&bad, p.mask_bad, sizeof(int), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (bad) return fail(MTTS_E_INVALID, "attention_mask must be left-padded (MossTTSLocal positions are cumsum(mask) - 1)");
  return 0;
}

// ---------------------------------------------------------------------------
// C ABI (include/mtts.h)
extern "C" int mtts_local_generate_begin(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int T,
                                         int max_new, int n_vq_for_inference, const mtts_sampling* sp, void* stream) {
  if (!e || !ids) return fail(MTTS_E_INVALID, "null argument");
  if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "not a MossTTSLocal engine");
  const mtts_config& c = e->c;
  if (B <= 0 || B > c.max_batch || T <= 0 || max_new <= 0 || T + max_new > c.max_ctx)
    return fail(MTTS_E_INVALID, "B/T/max_new_tokens exceed the engine capacity");
  LocalParts& p = *e->lp;
  // per-channel processors (:356-368): the table set by mtts_local_set_sampling, else channel 0
  // from the text_* fields and every codebook channel from the audio_* fields
  ChSampling chs[LOCAL_MAXC];
  for (int c = 0; c < p.C; ++c) {
    ChSampling& q = chs[c];
    if (c < (int)p.ch_table.size()) {
      q = p.ch_table[c];
    } else if (!sp) {
      q = ChSampling{0, 1.f, 1.f, 1.f, 0};
    } else if (c == 0) {
      q = ChSampling{sp->text_temperature > 0.f, sp->text_temperature > 0.f ? sp->text_temperature : 1.f,
                     sp->text_top_p, 1.f, sp->text_top_k};
    } else {
      q = ChSampling{sp->audio_temperature > 0.f, sp->audio_temperature > 0.f ? sp->audio_temperature : 1.f,
                     sp->audio_top_p, sp->audio_repetition_penalty, sp->audio_top_k};
    }
    if (c == 0) q.pen = 1.f;  // the reference attaches no repetition penalty to the text channel
    // any top_k (<= 0: no TopKLogitsWarper, :365-370): candidate sets past the sorted list take
    // the key-bin walk (local_pick_kernel)
    if (q.sample && !(q.temp > 0.f)) return fail(MTTS_E_INVALID, "sampled channel needs a positive temperature");
  }
  hipStream_t s = enter(e, stream);
  GenDev& g = e->hst;
  std::memset(&g, 0, sizeof(g));
  g.T0 = T; g.step = 0; g.fwd_pos = 0; g.done_step = -1;
  g.B = B; g.n_vq = c.n_vq; g.C = p.C; g.Ltot = c.max_ctx; g.Cmax = c.max_ctx;
  g.vocab = c.vocab; g.audio_rows = e->audio_rows;
  // generation_config.layers (:356-368): channel 0 <- text_*, channels >= 1 <- audio_*;
  // do_samples[i] = temperature > 0; repetition penalty on audio channels only (i != 0)
  for (int c = 0; c < p.C; ++c) g.lch[c] = chs[c];
  if (sp) g.seed = sp->seed;
  e->gen_B = B; e->gen_T = T; e->gen_max_new = max_new; e->forced = nullptr;
  p.n_ch = n_channels(e, n_vq_for_inference);
  HIPCHK(hipMemcpyAsync(e->st, &g, sizeof(g), hipMemcpyHostToDevice, s));
  HIPCHK(local_init(ids, mask, B, T, p.C, e->gen_ids, c.max_ctx, e->mask, c.max_ctx, p.finished, p.seen, e->audio_rows, s));
  int rc = left_pad_offsets(e, T, B, s);
  if (!rc) rc = forward_chunked(e, ids, B, T, 0, nullptr, s, p.hid, p.n_ch);
  if (!rc) rc = local_depth(e, B, p.n_ch, nullptr, 0, nullptr, 0, s);
  if (!rc) rc = local_frame_end(e, s);
  if (rc) return rc;
  e->steps_issued = 1;
  leave(e, stream);
  return 0;
}

extern "C" int mtts_local_set_sampling(mtts_engine* e, const mtts_channel_sampling* ch, int n) {
  if (!e || n < 0 || (n > 0 && !ch)) return fail(MTTS_E_INVALID, "null argument");
  if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "not a MossTTSLocal engine");
  if (n > e->lp->C) return fail(MTTS_E_INVALID, "more channel settings than channels");
  e->lp->ch_table.clear();
  for (int i = 0; i < n; ++i)
    e->lp->ch_table.push_back(ChSampling{ch[i].do_sample != 0, ch[i].temperature, ch[i].top_p,
                                         ch[i].repetition_penalty, ch[i].top_k});
  return 0;
}

extern "C" int mtts_local_generate_decode(mtts_engine* e, int n_steps, void* stream) {
  if (!e) return fail(MTTS_E_INVALID, "null engine");
  if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "not a MossTTSLocal engine");
  if (e->gen_B <= 0) return fail(MTTS_E_INVALID, "generate_begin not called");
  LocalParts& p = *e->lp;
  hipStream_t s = enter(e, stream);
  if (p.no_graph) {  // MTTS_LOCAL_NO_GRAPH=1: direct launches (A/B)
    for (int i = 0; i < n_steps && e->steps_issued < e->gen_max_new; ++i) {
      if (int rc = local_step_launch(e, s)) return rc;
      ++e->steps_issued;
    }
    leave(e, stream);
    return 0;
  }
  const long long key = (long long)e->gen_B * 256 + p.n_ch;
  auto it = p.graphs.find(key);
  hipGraphExec_t exec = nullptr;
  if (it != p.graphs.end()) {
    exec = it->second;
  } else {
    hipGraph_t graph;
    HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    int rc = local_step_launch(e, s);
    hipError_t ce = hipStreamEndCapture(s, &graph);
    if (rc) return rc;
    if (ce != hipSuccess) return fail(MTTS_E_HIP, std::string("capture: ") + hipGetErrorString(ce));
    HIPCHK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    hipGraphDestroy(graph);
    p.graphs[key] = exec;
  }
  for (int i = 0; i < n_steps && e->steps_issued < e->gen_max_new; ++i) {
    HIPCHK(hipGraphLaunch(exec, s));
    ++e->steps_issued;
  }
  leave(e, stream);
  return 0;
}

extern "C" int mtts_local_generate(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int T, int max_new,
                                   int n_vq_for_inference, const mtts_sampling* sp, int chunk, int* n_rows, void* stream) {
  if (chunk <= 0) chunk = 16;
  // a persistent-launch timeout (MTTS_E_PSE_TIMEOUT) turned that launch off: the generation
  // restarts once from the prompt on the per-op launches
  for (int attempt = 0;; ++attempt) {
    int rc = mtts_local_generate_begin(e, ids, mask, B, T, max_new, n_vq_for_inference, sp, stream);
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
      rc = mtts_local_generate_decode(e, std::min(chunk, max_new - steps), stream);
      if (rc) break;
    }
    if (rc == MTTS_E_PSE_TIMEOUT && attempt == 0) continue;
    if (rc) return rc;
    if (n_rows) *n_rows = done >= 0 ? done + 1 : steps;
    return 0;
  }
}

extern "C" int mtts_local_forward(mtts_engine* e, const int64_t* ids, const uint8_t* mask, int B, int S, int past,
                                  int n_vq_for_inference, const int64_t* forced, uint16_t* logits, int ld_logits,
                                  void* stream) {
  if (!e || !ids || !mask || !logits) return fail(MTTS_E_INVALID, "null argument");
  if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "not a MossTTSLocal engine");
  const mtts_config& c = e->c;
  if (B <= 0 || B > c.max_batch || S <= 0 || past < 0 || past + S > c.max_ctx) return fail(MTTS_E_INVALID, "bad B/S/past");
  if (ld_logits < c.vocab) return fail(MTTS_E_INVALID, "ld_logits < vocab");
  LocalParts& p = *e->lp;
  const int n_ch = n_channels(e, n_vq_for_inference);
  hipStream_t s = enter(e, stream);
  HIPCHK(hipMemcpy2DAsync(e->mask, c.max_ctx, mask, past + S, past + S, B, hipMemcpyDeviceToDevice, s));
  int rc = left_pad_offsets(e, past + S, B, s);
  if (!rc) rc = forward_chunked(e, ids, B, S, past, nullptr, s, p.hid, n_ch);
  if (!rc) rc = local_depth(e, B, n_ch, forced, p.C, reinterpret_cast<bf16_t*>(logits), ld_logits, s);
  if (!rc && local_lpse_takes(e, B)) {
    // (a teacher-forced frame is the parity entry: checked here, and on a timed-out launch the
    // frame is recomputed on the per-op launches -- it rewrites the same cache rows)
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIPCHK(hipStreamIsCapturing(s, &cs));
    if (cs == hipStreamCaptureStatusNone && local_lpse_tripped(e, s)) {
      rc = forward_chunked(e, ids, B, S, past, nullptr, s, p.hid, n_ch);
      if (!rc) rc = local_depth(e, B, n_ch, forced, p.C, reinterpret_cast<bf16_t*>(logits), ld_logits, s);
    }
  }
  leave(e, stream);
  return rc;
}

extern "C" int mtts_local_lpse_active(const mtts_engine* e) { return e && local_lpse_takes(e, 1) ? 1 : 0; }

extern "C" int mtts_local_frame_bytes(const mtts_engine* e, int n_vq_for_inference, uint64_t* bytes) {
  if (!e || !bytes) return fail(MTTS_E_INVALID, "null argument");
  if (!e->lp) return fail(MTTS_E_UNSUPPORTED, "not a MossTTSLocal engine");
  const LocalParts& p = *e->lp;
  const int n_ch = n_channels(e, n_vq_for_inference);
  *bytes = p.backbone_bytes + n_ch * p.channel_bytes + p.text_head_bytes + (uint64_t)(n_ch - 1) * p.audio_head_bytes;
  return 0;
}

extern "C" int mtts_k_moss_rmsnorm(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int H, float eps, void* stream) {
  HIPCHK(moss_rmsnorm(x, w, y, M, H, eps, (hipStream_t)stream));
  return 0;
}

// kernel-level channel pick (parity tests): B rows of logits [B, ld]; row b's channel history
// in seen [B][C][audio_rows] (channel ch); the draw of row b uses Philox(seed; step, b, ch)
extern "C" int mtts_k_local_pick(const uint16_t* logits, int ld, int V, int ch, const uint8_t* seen, int64_t* out, int C,
                                 int B, int audio_rows, float temperature, int top_k, float top_p, float penalty,
                                 uint64_t seed, int step, void* stream) {
  // (the per-channel table GenDev::lch holds LOCAL_MAXC channels)
  if (!logits || !out || B <= 0 || V <= 0 || C <= 0 || C > LOCAL_MAXC || ch < 0 || ch >= C || (ch > 0 && V > audio_rows))
    return fail(MTTS_E_INVALID, "bad local_pick args");
  hipStream_t s = (hipStream_t)stream;
  GenDev g;
  std::memset(&g, 0, sizeof(g));
  g.step = step; g.audio_rows = audio_rows; g.seed = seed;
  g.lch[ch] = ChSampling{temperature > 0.f, temperature > 0.f ? temperature : 1.f, top_p, penalty, top_k};
  GenDev* d = nullptr;
  HIPCHK(hipMallocAsync((void**)&d, sizeof(GenDev), s));
  HIPCHK(hipMemcpyAsync(d, &g, sizeof(g), hipMemcpyHostToDevice, s));
  int* hist = nullptr;  // key-bin scratch of the wide candidate sets
  HIPCHK(hipMallocAsync((void**)&hist, (size_t)B * 65536 * sizeof(int), s));
  hipError_t err = local_pick(d, reinterpret_cast<const bf16_t*>(logits), ld, V, ch, seen, out, C, B, hist, s);
  HIPCHK(hipFreeAsync(hist, s));
  HIPCHK(hipFreeAsync(d, s));
  HIPCHK(err);
  HIPCHK(hipStreamSynchronize(s));
  return 0;
}
