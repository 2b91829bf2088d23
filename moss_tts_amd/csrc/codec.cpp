// Codec decoder (include/mtts_codec.h): residual-vector dequantisation, stages of causal
// Transformer blocks with linear upsampling between them, waveform patches out.
//
// Every stage is a Stack of Qwen3 decoder layers run by the backbone's own run_layers
// (prefill GEMM + flash prefill attention for chunks of tokens, the decode GEMV / fused
// decode attention for one-token chunks), with its own KV cache so that decoding is
// incremental: a chunk of F frames at frame offset f0 is F * R_s tokens at positions
// f0 * R_s .. of stage s (R_s = product of the upsampling factors before s).
//
// Per chunk:  rvq_dequant -> for each stage: run_layers -> stage RMSNorm (rmsnorm_ss) ->
//             upsample projection (GEMM; [M, r*D'] row-major IS [M*r, D']) + sumsq16
//             | last stage: patch_out (fp32 samples)
#include "engine_internal.h"
#include "../../include/mtts_codec.h"

namespace mtts {
hipError_t rvq_dequant(const int64_t* codes, int ld_codes, size_t ld_b, int F, int n_q, const bf16_t* tables, int cb,
                       int D, bf16_t* x, float* ss, int M, hipStream_t s);
hipError_t sumsq16(const bf16_t* x, int H, int M, float* ss, hipStream_t s);
hipError_t patch_out(const bf16_t* x, int M, int K, const bf16_t* wt, int patch, float* wav, int S, size_t ld_wav,
                     size_t off0, hipStream_t s);
hipError_t fill_int(int* p, int v, hipStream_t s);
}  // namespace mtts

namespace {

struct CodecStage {
  mtts_codec_stage c{};
  int R = 1;         // tokens per frame
  int Cmax = 0;      // KV capacity in tokens
  int Mmax = 0;      // token rows per chunk (all streams)
  std::vector<LayerW> L;
  bf16_t* norm = nullptr;
  bf16_t* up = nullptr;  // packed [upsample * next hidden, hidden]
  int* d_pos = nullptr;
  mtts_engine E;     // run_layers context: eps, flags, stream (owns no memory)
  Stack st;
};

}  // namespace

struct mtts_codec {
  mtts_codec_config c{};
  int device = 0;
  mtts_engine W;  // stream, events, weight staging
  std::vector<CodecStage> S;
  bf16_t* tables = nullptr;  // [n_q][codebook_size][hidden_0]
  bf16_t* outw = nullptr;    // [hidden_last][patch] (transposed for patch_out)
  int spf = 0;
  int pos = 0;  // frames decoded since reset
  uint64_t weight_bytes = 0;
  std::vector<void*> mem;

  template <class T>
  int alloc(T** p, size_t n) {
    void* q = nullptr;
    if (hipMalloc(&q, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess)
      return fail(MTTS_E_OOM, "codec hipMalloc failed (" + std::to_string(n * sizeof(T)) + " B)");
    mem.push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
};

extern "C" int mtts_codec_destroy(mtts_codec* k) {
  if (!k) return 0;
  hipSetDevice(k->device);
  if (k->W.stream) hipStreamSynchronize(k->W.stream);
  for (void* p : k->mem) hipFree(p);
  if (k->W.staging) hipFree(k->W.staging);
  if (k->W.ev_in) hipEventDestroy(k->W.ev_in);
  if (k->W.ev_out) hipEventDestroy(k->W.ev_out);
  if (k->W.stream) hipStreamDestroy(k->W.stream);
  delete k;
  return 0;
}

extern "C" int mtts_codec_create(const mtts_codec_config* cfg, int device, mtts_codec** out) {
  if (!cfg || !out) return fail(MTTS_E_INVALID, "null argument");
  const mtts_codec_config& c = *cfg;
  if (c.n_q <= 0 || c.codebook_size <= 0 || c.n_stages <= 0 || c.n_stages > MTTS_CODEC_MAX_STAGES || c.patch <= 0 ||
      c.max_batch <= 0 || c.max_frames <= 0 || c.max_chunk_frames <= 0)
    return fail(MTTS_E_INVALID, "bad codec config");
  for (int s = 0; s < c.n_stages; ++s) {
    const mtts_codec_stage& g = c.stages[s];
    if (g.hidden % 32 || g.inter % 32 || g.layers <= 0 || g.n_heads % g.n_kv || g.upsample < 1 ||
        (g.head_dim != 32 && g.head_dim != 64 && g.head_dim != 128) || (s == c.n_stages - 1 && g.upsample != 1))
      return fail(MTTS_E_UNSUPPORTED, "codec stage shape not covered by the kernels");
  }
  if (c.stages[0].hidden / 8 > 256 || (size_t)8 * c.stages[c.n_stages - 1].hidden * 4 > 64 * 1024)
    return fail(MTTS_E_UNSUPPORTED, "codec dims not covered by the dequant / patch kernels");
  if (hipSetDevice(device) != hipSuccess) return fail(MTTS_E_HIP, "hipSetDevice");
  mtts_codec* k = new mtts_codec();
  k->c = c;
  k->device = device;
  auto bail = [&](int rc) {
    mtts_codec_destroy(k);
    return rc;
  };
  k->W.device = device;
  if (hipStreamCreateWithFlags(&k->W.stream, hipStreamNonBlocking) != hipSuccess) return bail(fail(MTTS_E_HIP, "stream"));
  hipEventCreateWithFlags(&k->W.ev_in, hipEventDisableTiming);
  hipEventCreateWithFlags(&k->W.ev_out, hipEventDisableTiming);
  int rc = 0;
  const int B = c.max_batch;
  k->S.resize(c.n_stages);
  int R = 1;
  uint64_t wb = 0;
  for (int s = 0; s < c.n_stages; ++s) {
    CodecStage& st = k->S[s];
    st.c = c.stages[s];
    const int H = st.c.hidden, D = st.c.head_dim, Hq = st.c.n_heads, Hkv = st.c.n_kv, I = st.c.inter;
    const int qkv_rows = (Hq + 2 * Hkv) * D;
    st.R = R;
    st.Cmax = ((c.max_frames * R + 63) / 64) * 64;
    st.Mmax = B * c.max_chunk_frames * R;
    st.L.resize(st.c.layers);
    for (auto& w : st.L) {
      if ((rc = k->alloc(&w.qkv, packed_bytes(qkv_rows, H) / 2)) || (rc = k->alloc(&w.o, packed_bytes(H, Hq * D) / 2)) ||
          (rc = k->alloc(&w.gu, packed_bytes(2 * I, H) / 2)) || (rc = k->alloc(&w.down, packed_bytes(H, I) / 2)) ||
          (rc = k->alloc(&w.in_norm, H)) || (rc = k->alloc(&w.post_norm, H)) || (rc = k->alloc(&w.q_norm, D)) ||
          (rc = k->alloc(&w.k_norm, D)))
        return bail(rc);
      wb += 2ull * ((uint64_t)qkv_rows * H + (uint64_t)H * Hq * D + 2ull * I * H + (uint64_t)H * I);
    }
    if ((rc = k->alloc(&st.norm, H))) return bail(rc);
    if (s + 1 < c.n_stages) {
      const int rows = st.c.upsample * c.stages[s + 1].hidden;
      if ((rc = k->alloc(&st.up, packed_bytes(rows, H) / 2))) return bail(rc);
      wb += 2ull * rows * H;
    }
    // the stage's Stack: caches, RoPE tables, mask (every key valid), workspaces
    Stack& t = st.st;
    t.L = st.L.data(); t.layers = st.c.layers; t.H = H; t.Hq = Hq; t.Hkv = Hkv; t.D = D; t.I = I; t.qkv_rows = qkv_rows;
    t.layer_kv = (size_t)B * Hkv * st.Cmax * D;
    t.Cmax = st.Cmax;
    bf16_t *cs = nullptr, *sn = nullptr;
    const size_t M = std::max(st.Mmax, B);
    const size_t ns_dec = (st.Cmax + CH_DECODE - 1) / CH_DECODE;
    if ((rc = k->alloc(&t.kc, t.layer_kv * st.c.layers)) || (rc = k->alloc(&t.vc, t.layer_kv * st.c.layers)) ||
        (rc = k->alloc(&cs, (size_t)st.Cmax * D)) || (rc = k->alloc(&sn, (size_t)st.Cmax * D)) ||
        (rc = k->alloc(&t.mask, (size_t)B * st.Cmax)) || (rc = k->alloc(&t.h, M * H)) || (rc = k->alloc(&t.xn, M * H)) ||
        (rc = k->alloc(&t.ss, M * (H / 16))) || (rc = k->alloc(&t.qkvb, M * qkv_rows)) ||
        (rc = k->alloc(&t.qb, M * Hq * D)) || (rc = k->alloc(&t.attnb, M * Hq * D)) || (rc = k->alloc(&t.act, M * I)) ||
        (rc = k->alloc(&t.part, (size_t)B * ns_dec * Hq * (D + 2))) || (rc = k->alloc(&t.att_cnt, (size_t)B * Hkv)) ||
        (rc = k->alloc(&st.d_pos, 1)))
      return bail(rc);
    {
      std::vector<uint16_t> ch((size_t)st.Cmax * D), sh((size_t)st.Cmax * D);
      mtts_rope_table(c.rope_theta, D, st.Cmax, ch.data(), sh.data());
      if (hipMemcpy(cs, ch.data(), ch.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemcpy(sn, sh.data(), sh.size() * 2, hipMemcpyHostToDevice) != hipSuccess ||
          hipMemset(t.mask, 1, (size_t)B * st.Cmax) != hipSuccess ||
          hipMemset(t.att_cnt, 0, (size_t)B * Hkv * sizeof(int)) != hipSuccess)
        return bail(fail(MTTS_E_HIP, "codec init"));
    }
    t.cos_t = cs; t.sin_t = sn;
    st.E.c.rms_eps = c.rms_eps;
    st.E.device = device;
    st.E.stream = k->W.stream;
    R *= st.c.upsample;
  }
  const int D0 = c.stages[0].hidden, DL = c.stages[c.n_stages - 1].hidden;
  if ((rc = k->alloc(&k->tables, (size_t)c.n_q * c.codebook_size * D0)) || (rc = k->alloc(&k->outw, (size_t)DL * c.patch)))
    return bail(rc);
  wb += 2ull * DL * c.patch;
  k->weight_bytes = wb;
  k->spf = R * c.patch;
  if (hipDeviceSynchronize() != hipSuccess) return bail(fail(MTTS_E_HIP, "codec init sync"));
  *out = k;
  return 0;
}

extern "C" int mtts_codec_samples_per_frame(const mtts_codec* k) { return k ? k->spf : 0; }
extern "C" int mtts_codec_position(const mtts_codec* k) { return k ? k->pos : 0; }
extern "C" int mtts_codec_reset(mtts_codec* k) {
  if (!k) return fail(MTTS_E_INVALID, "null codec");
  k->pos = 0;
  return 0;
}
extern "C" int mtts_codec_weight_bytes(const mtts_codec* k, uint64_t* bytes) {
  if (!k || !bytes) return fail(MTTS_E_INVALID, "null argument");
  *bytes = k->weight_bytes;
  return 0;
}

namespace {

__global__ void transpose_bf16_kernel(const bf16_t* src, bf16_t* dst, int rows, int cols) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)rows * cols) return;
  const size_t r = i / cols, cc = i % cols;
  dst[cc * rows + r] = src[i];
}

}  // namespace

extern "C" int mtts_codec_load_weight(mtts_codec* k, const char* name, const void* src, size_t bytes, int on_dev) {
  if (!k || !name || !src) return fail(MTTS_E_INVALID, "null argument");
  hipSetDevice(k->device);
  const mtts_codec_config& c = k->c;
  const std::string n(name);
  WTarget t;
  auto num = [](const std::string& s, size_t at, size_t* end) -> int {
    size_t e = at;
    while (e < s.size() && isdigit((unsigned char)s[e])) ++e;
    *end = e;
    return e > at ? std::atoi(s.c_str() + at) : -1;
  };
  const std::string pq = "quantizer.codebooks.", ps = "decoder.stages.";
  if (n.rfind(pq, 0) == 0) {
    size_t e;
    const int q = num(n, pq.size(), &e);
    if (q < 0 || q >= c.n_q || n.substr(e) != ".weight") return fail(MTTS_E_INVALID, "bad name " + n);
    t.dst = k->tables + (size_t)q * c.codebook_size * c.stages[0].hidden;
    t.expect = (size_t)c.codebook_size * c.stages[0].hidden;
  } else if (n == "decoder.out_proj.weight") {
    const int DL = c.stages[c.n_stages - 1].hidden;
    if (bytes != (size_t)c.patch * DL * 2) return fail(MTTS_E_INVALID, "size mismatch for " + n);
    const bf16_t* from = reinterpret_cast<const bf16_t*>(src);
    // the source may be in flight on the caller's (legacy default) stream: event-ordered, as store_weight
    hipStream_t ws = enter(&k->W, nullptr);
    if (!on_dev) {
      if (int rc = ensure_staging(&k->W, bytes)) return rc;
      HIPCHK(hipMemcpyAsync(k->W.staging, src, bytes, hipMemcpyHostToDevice, ws));
      from = k->W.staging;
    }
    const size_t tot = (size_t)c.patch * DL;
    hipLaunchKernelGGL(transpose_bf16_kernel, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, ws, from,
                       k->outw, c.patch, DL);
    HIPCHK(hipGetLastError());
    if (!on_dev) HIPCHK(hipStreamSynchronize(ws));
    leave(&k->W, nullptr);
    return 0;
  } else if (n.rfind(ps, 0) == 0) {
    size_t e;
    const int s = num(n, ps.size(), &e);
    if (s < 0 || s >= c.n_stages) return fail(MTTS_E_INVALID, "bad stage in " + n);
    CodecStage& st = k->S[s];
    const std::string rest = n.substr(e);
    const int H = st.c.hidden;
    if (rest == ".norm.weight") {
      t.dst = st.norm; t.expect = H;
    } else if (rest == ".upsample.weight" && st.up) {
      t.pack = true; t.dst = st.up; t.rows = st.c.upsample * c.stages[s + 1].hidden; t.K = H;
      t.expect = (size_t)t.rows * H;
    } else if (rest.rfind(".layers.", 0) == 0) {
      size_t e2;
      const int l = num(rest, 8, &e2);
      if (l < 0 || l >= st.c.layers || e2 >= rest.size() || rest[e2] != '.') return fail(MTTS_E_INVALID, "bad layer in " + n);
      if (!layer_target(st.L[l], rest.substr(e2 + 1), H, st.c.inter, st.c.n_heads, st.c.n_kv, st.c.head_dim, &t))
        return fail(MTTS_E_INVALID, "unknown weight " + n);
    } else {
      return fail(MTTS_E_INVALID, "unknown weight " + n);
    }
  } else {
    return fail(MTTS_E_INVALID, "unknown weight " + n);
  }
  return store_weight(&k->W, t, name, src, bytes, on_dev);
}

// Qwen3-block init like mtts_engine_init_random (uniform +-sqrt(3/K) matrices, norms 1 +- 0.25);
// codebooks +-sqrt(3/n_q) so that the dequantised sum has unit scale
extern "C" int mtts_codec_init_random(mtts_codec* k, uint64_t seed) {
  if (!k) return fail(MTTS_E_INVALID, "null codec");
  hipSetDevice(k->device);
  const mtts_codec_config& c = k->c;
  struct Spec { std::string name; size_t rows, cols; int kind; };
  std::vector<Spec> sp;
  for (int q = 0; q < c.n_q; ++q)
    sp.push_back({"quantizer.codebooks." + std::to_string(q) + ".weight", (size_t)c.codebook_size,
                  (size_t)c.stages[0].hidden, 2});
  for (int s = 0; s < c.n_stages; ++s) {
    const mtts_codec_stage& g = c.stages[s];
    const size_t H = g.hidden, D = g.head_dim, Hq = g.n_heads, Hkv = g.n_kv, I = g.inter;
    for (int l = 0; l < g.layers; ++l) {
      const std::string p = "decoder.stages." + std::to_string(s) + ".layers." + std::to_string(l) + ".";
      sp.push_back({p + "self_attn.q_proj.weight", Hq * D, H, 0});
      sp.push_back({p + "self_attn.k_proj.weight", Hkv * D, H, 0});
      sp.push_back({p + "self_attn.v_proj.weight", Hkv * D, H, 0});
      sp.push_back({p + "self_attn.o_proj.weight", H, Hq * D, 0});
      sp.push_back({p + "self_attn.q_norm.weight", 1, D, 1});
      sp.push_back({p + "self_attn.k_norm.weight", 1, D, 1});
      sp.push_back({p + "mlp.gate_proj.weight", I, H, 0});
      sp.push_back({p + "mlp.up_proj.weight", I, H, 0});
      sp.push_back({p + "mlp.down_proj.weight", H, I, 0});
      sp.push_back({p + "input_layernorm.weight", 1, H, 1});
      sp.push_back({p + "post_attention_layernorm.weight", 1, H, 1});
    }
    sp.push_back({"decoder.stages." + std::to_string(s) + ".norm.weight", 1, H, 1});
    if (s + 1 < c.n_stages)
      sp.push_back({"decoder.stages." + std::to_string(s) + ".upsample.weight",
                    (size_t)g.upsample * c.stages[s + 1].hidden, H, 0});
  }
  sp.push_back({"decoder.out_proj.weight", (size_t)c.patch, (size_t)c.stages[c.n_stages - 1].hidden, 0});
  size_t mx = 0;
  for (auto& s : sp) mx = std::max(mx, s.rows * s.cols);
  bf16_t* buf = nullptr;
  if (hipMalloc(&buf, mx * 2) != hipSuccess) return fail(MTTS_E_OOM, "codec init buffer");
  int rc = 0;
  for (size_t tid = 0; tid < sp.size() && !rc; ++tid) {
    const Spec& s = sp[tid];
    float scale = 1.f, offset = 0.f;
    if (s.kind == 0) scale = (float)std::sqrt(3.0 / (double)s.cols);
    else if (s.kind == 1) { scale = 0.25f; offset = 1.0f; }
    else scale = (float)std::sqrt(3.0 / (double)c.n_q);
    if (fill_uniform_bf16(buf, s.rows * s.cols, seed, tid, scale, offset, k->W.stream) != hipSuccess) {
      rc = fail(MTTS_E_HIP, "fill");
      break;
    }
    rc = mtts_codec_load_weight(k, s.name.c_str(), buf, s.rows * s.cols * 2, 1);
  }
  hipStreamSynchronize(k->W.stream);
  hipFree(buf);
  return rc;
}

// one chunk of F frames of B streams at frame offset f0
// f0: the chunk's first frame in the stream (positions); wav_off: its first sample in wav rows
static int codec_chunk(mtts_codec* k, const int64_t* codes, size_t ld_b, int B, int F, int ld_codes, int nq, float* wav,
                       size_t ld_wav, int f0, size_t wav_off, hipStream_t s) {
  const mtts_codec_config& c = k->c;
  const int D0 = c.stages[0].hidden;
  HIPCHK(rvq_dequant(codes, ld_codes, ld_b, F, nq, k->tables, c.codebook_size, D0, k->S[0].st.h, k->S[0].st.ss, B * F,
                     s));
  for (int i = 0; i < c.n_stages; ++i) {
    CodecStage& st = k->S[i];
    const int Sn = F * st.R, M = B * Sn, H = st.c.hidden;
    HIPCHK(fill_int(st.d_pos, f0 * st.R, s));
    st.E.stream = s;
    if (int rc = run_layers(&st.E, st.st, 0, B, Sn, st.d_pos, CH_PREFILL, 1, s)) return rc;
    HIPCHK(rmsnorm_ss(st.st.h, 0, H, st.st.ss, 0, H / 16, st.norm, st.st.xn, M, H, c.rms_eps, s));
    if (i + 1 < c.n_stages) {
      CodecStage& nx = k->S[i + 1];
      const int N = st.c.upsample * nx.c.hidden;
      GemvArgs g = gemv_args(st.up, st.st.xn, H, nx.st.h, N, M, N, H);
      HIPCHK(proj(&st.E, g, EPI_STORE, s));
      HIPCHK(sumsq16(nx.st.h, nx.c.hidden, M * st.c.upsample, nx.st.ss, s));
    } else {
      HIPCHK(patch_out(st.st.xn, M, H, k->outw, c.patch, wav, Sn, ld_wav, wav_off, s));
    }
  }
  return 0;
}

extern "C" int mtts_codec_decode(mtts_codec* k, const int64_t* codes, int B, int T, int ld_codes, int nq, float* wav,
                                 size_t ld_wav, void* stream) {
  if (!k || !codes || !wav) return fail(MTTS_E_INVALID, "null argument");
  const mtts_codec_config& c = k->c;
  if (B <= 0 || B > c.max_batch || T < 0 || nq <= 0 || nq > c.n_q || ld_codes < nq)
    return fail(MTTS_E_INVALID, "codec decode: bad B / T / n_q");
  if (k->pos + T > c.max_frames) return fail(MTTS_E_INVALID, "codec decode: stream longer than max_frames (reset first)");
  if (ld_wav < (size_t)T * k->spf) return fail(MTTS_E_INVALID, "codec decode: wav row too short");
  hipStream_t s = enter(&k->W, stream);
  for (int f = 0; f < T; f += c.max_chunk_frames) {
    const int F = std::min(c.max_chunk_frames, T - f);
    if (int rc = codec_chunk(k, codes + (size_t)f * ld_codes, (size_t)T * ld_codes, B, F, ld_codes, nq, wav, ld_wav,
                             k->pos, (size_t)f * k->spf, s)) {
      leave(&k->W, stream);
      return rc;
    }
    k->pos += F;
  }
  leave(&k->W, stream);
  return 0;
}
