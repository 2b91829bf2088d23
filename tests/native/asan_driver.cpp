// AddressSanitizer run of the C-ABI host code (SURVEY.md §5 "ASan for the C-ABI host code").
//
// libmtts's host side (csrc/engine.cpp, local.cpp, codec.cpp: weight repacking by name,
// capacity buffers, graph capture, the generate state machine's host part, the codec's
// chunking) is compiled with -Xarch_host -fsanitize=address into this executable (no Python,
// so the ASan runtime is linked in rather than preloaded); the device code is built as usual.
// The driver walks every C entry point on tiny shapes -- engine create / load / reserve /
// forward / generate (greedy, sampled, wide text top_k, forced schedule) / fetch / logits /
// poll / stats, the MossTTSLocal engine (per-channel sampling, teacher-forced frames), the
// codec (whole and chunked decode), the kernel-level entry points -- plus their error paths
// (null arguments, bad names and sizes, exceeded capacity), and checks every status code.
// Any heap overflow / use-after-free / leak in the host code aborts with an ASan report.
//
//   make -C tests/native && tests/native/asan_driver     (GPU box)
#include <hip/hip_runtime.h>

#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mtts.h"
#include "../../include/mtts_codec.h"

static int g_fail = 0;
#define EXPECT(cond, what)                                                                      \
  do {                                                                                          \
    if (!(cond)) {                                                                              \
      fprintf(stderr, "FAIL %s:%d %s (last error: %s)\n", __FILE__, __LINE__, what, mtts_last_error()); \
      ++g_fail;                                                                                 \
    }                                                                                           \
  } while (0)
#define OK(x) EXPECT((x) == 0, #x)

// Progress log + watchdog (round 5).  One run of this driver inside the GPU
// suite once went silent for 180 s and was killed with its output captured, so nothing said where
// it was.  Every phase now writes a line (flushed) to $MTTS_ASAN_LOG (else stderr) before it
// starts, and a watchdog thread ends the process with exit code 3, naming the phase, when one
// phase runs longer than $MTTS_ASAN_PHASE_TIMEOUT seconds (default 90).  The last line before
// `return` says "exit": a stall after it is the LeakSanitizer leak check or the runtime's teardown
// (the watchdog is suspended with every other thread during the leak check; the test's own
// subprocess timeout covers that window).
static FILE* g_log = nullptr;
static std::atomic<int> g_phase_id{0};
static std::atomic<long long> g_phase_t0{0};
static const char* volatile g_phase = "start";
static long long now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static long long g_start_ms = now_ms();
static void phase(const char* name) {
  g_phase = name;
  g_phase_t0.store(now_ms());
  g_phase_id.fetch_add(1);
  fprintf(g_log, "[%8.3f s] %s\n", (now_ms() - g_start_ms) / 1000.0, name);
  fflush(g_log);
}
static void watchdog(int limit_s) {
  for (;;) {
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    const long long age = now_ms() - g_phase_t0.load();
    if (age > (long long)limit_s * 1000) {
      fprintf(g_log, "[%8.3f s] STALL: phase '%s' has run %.1f s (limit %d s)\n", (now_ms() - g_start_ms) / 1000.0,
              (const char*)g_phase, age / 1000.0, limit_s);
      fflush(g_log);
      fprintf(stderr, "asan driver: STALL in phase '%s' after %.1f s\n", (const char*)g_phase, age / 1000.0);
      fflush(stderr);
      _exit(3);
    }
  }
}

template <class T>
static T* dev(size_t n) {
  void* p = nullptr;
  if (hipMalloc(&p, n * sizeof(T) + 16) != hipSuccess) {
    fprintf(stderr, "hipMalloc failed\n");
    exit(2);
  }
  hipMemset(p, 0, n * sizeof(T) + 16);
  return reinterpret_cast<T*>(p);
}

static mtts_config tiny(int n_vq, int kind) {
  mtts_config c{};
  c.hidden = 64; c.layers = 2; c.n_heads = 4; c.n_kv = 2; c.head_dim = 16; c.inter = 128; c.vocab = 151936;
  c.n_vq = n_vq; c.audio_vocab = 1024; c.rope_theta = 10000.f; c.rms_eps = 1e-6f;
  c.pad_token_id = 151643; c.im_start_token_id = 151644; c.im_end_token_id = 151645;
  c.audio_start_token_id = 151652; c.audio_end_token_id = 151653; c.audio_user_slot_token_id = 151654;
  c.audio_assistant_gen_slot_token_id = 151656; c.audio_assistant_delay_slot_token_id = 151662;
  c.audio_pad_code = 1024; c.max_batch = 3; c.max_ctx = 128; c.max_prefill_tokens = 64;
  c.model_kind = kind; c.eos_token_id = 151653;
  if (kind == MTTS_MODEL_LOCAL) {
    c.local_hidden = 64; c.local_layers = 2; c.local_inter = 128; c.local_mlp_ffn = 96;
  }
  return c;
}

// prompt rows: random text ids, an audio block of user-slot rows with codes, ending in audio_start
static std::vector<int64_t> prompt(int B, int T, int C, unsigned seed) {
  std::vector<int64_t> ids((size_t)B * T * C, 1024);
  srand(seed);
  for (int b = 0; b < B; ++b)
    for (int t = 0; t < T; ++t) {
      int64_t* r = &ids[((size_t)b * T + t) * C];
      r[0] = 200 + rand() % 20000;
      if (t >= 3 && t < 8) {
        r[0] = 151654;
        for (int c = 1; c < C; ++c) r[c] = rand() % 1024;
      }
      if (t == T - 1) r[0] = 151652;
    }
  return ids;
}

static void delay_engine() {
  const int n_vq = 4, C = n_vq + 1, B = 3, T = 20, max_new = 24;
  mtts_config c = tiny(n_vq, MTTS_MODEL_DELAY);
  mtts_engine* e = nullptr;
  phase("delay: create + init_random");
  OK(mtts_engine_create(&c, 0, &e));
  if (!e) return;
  OK(mtts_engine_init_random(e, 7));
  uint64_t wb = 0;
  OK(mtts_engine_weight_bytes(e, &wb));
  EXPECT(wb > 0, "weight bytes");
  // weight loading by name: host and device sources, bad names and sizes
  phase("delay: load_weight by name");
  const int H = c.hidden;
  std::vector<uint16_t> host((size_t)c.vocab * H, 0x3f80);
  OK(mtts_engine_load_weight(e, "language_model.norm.weight", host.data(), H * 2, 0));
  OK(mtts_engine_load_weight(e, "language_model.layers.1.mlp.down_proj.weight", host.data(), (size_t)H * c.inter * 2, 0));
  uint16_t* dsrc = dev<uint16_t>((size_t)c.n_heads * c.head_dim * H);
  OK(mtts_engine_load_weight(e, "language_model.layers.0.self_attn.q_proj.weight", dsrc, (size_t)c.n_heads * c.head_dim * H * 2, 1));
  EXPECT(mtts_engine_load_weight(e, "language_model.layers.9.mlp.up_proj.weight", host.data(), (size_t)H * c.inter * 2, 0) ==
             MTTS_E_INVALID, "bad layer index");
  EXPECT(mtts_engine_load_weight(e, "no.such.weight", host.data(), 2, 0) == MTTS_E_INVALID, "unknown name");
  EXPECT(mtts_engine_load_weight(e, "lm_heads.1.weight", host.data(), 2, 0) == MTTS_E_INVALID, "size mismatch");
  EXPECT(mtts_engine_load_weight(e, "emb_ext.99.weight", host.data(), 2, 0) == MTTS_E_INVALID, "bad channel");
  EXPECT(mtts_engine_load_weight(nullptr, "x", host.data(), 2, 0) == MTTS_E_INVALID, "null engine");
  OK(mtts_engine_init_random(e, 7));
  // forward: prefill + 3 decode steps, ragged mask
  phase("delay: teacher-forced forward (prefill + 3 steps)");
  std::vector<int64_t> ids = prompt(B, T + 3, C, 1);
  int64_t* d_ids = dev<int64_t>(ids.size());
  hipMemcpy(d_ids, ids.data(), ids.size() * 8, hipMemcpyHostToDevice);
  std::vector<uint8_t> mask((size_t)B * (T + 3), 1);
  for (int t = 0; t < 5; ++t) mask[(size_t)2 * (T + 3) + t] = 0;
  const int ld = mtts_heads_ld(e);
  EXPECT(ld == c.vocab + n_vq * 1025, "heads_ld");
  uint16_t* d_logits = dev<uint16_t>((size_t)B * ld);
  // forward reads mask [B, past + S]: pack per call
  for (int s = 0; s <= 3; ++s) {
    const int past = s == 0 ? 0 : T + s - 1, S = s == 0 ? T : 1;
    std::vector<int64_t> x((size_t)B * S * C);
    std::vector<uint8_t> m((size_t)B * (past + S));
    for (int b = 0; b < B; ++b) {
      memcpy(&x[(size_t)b * S * C], &ids[((size_t)b * (T + 3) + past) * C], (size_t)S * C * 8);
      memcpy(&m[(size_t)b * (past + S)], &mask[(size_t)b * (T + 3)], past + S);
    }
    int64_t* dx = dev<int64_t>(x.size());
    uint8_t* dm = dev<uint8_t>(m.size());
    hipMemcpy(dx, x.data(), x.size() * 8, hipMemcpyHostToDevice);
    hipMemcpy(dm, m.data(), m.size(), hipMemcpyHostToDevice);
    OK(mtts_forward(e, dx, dm, B, S, past, d_logits, nullptr));
    hipFree(dx);
    hipFree(dm);
  }
  EXPECT(mtts_forward(e, d_ids, nullptr, B, 1, 0, d_logits, nullptr) == MTTS_E_INVALID, "null mask");
  EXPECT(mtts_forward(e, d_ids, mask.data(), B, 1, c.max_ctx, d_logits, nullptr) == MTTS_E_INVALID, "past beyond capacity");
  // generate: greedy, sampled (default kwargs), wide text top_k, forced schedule
  std::vector<int64_t> gp = prompt(B, T, C, 2);
  int64_t* d_gp = dev<int64_t>(gp.size());
  hipMemcpy(d_gp, gp.data(), gp.size() * 8, hipMemcpyHostToDevice);
  uint8_t* d_gm = dev<uint8_t>((size_t)B * T);
  hipMemset(d_gm, 1, (size_t)B * T);
  int32_t* d_forced = dev<int32_t>(max_new);
  std::vector<int32_t> forced(max_new, 151656);
  hipMemcpy(d_forced, forced.data(), max_new * 4, hipMemcpyHostToDevice);
  mtts_sampling greedy{0.f, 1.f, 50, 0.f, 1.f, 25, 1.f, 1};
  mtts_sampling sampled{1.5f, 1.f, 50, 1.7f, 0.8f, 25, 1.1f, 2};
  mtts_sampling wide{1.0f, 0.9f, 0, 1.2f, 0.95f, 0, 1.0f, 3};
  int64_t* d_out = dev<int64_t>((size_t)B * (T + max_new) * C);
  const char* gen_names[3][2] = {{"delay: generate greedy", "delay: generate greedy, forced"},
                                 {"delay: generate sampled", "delay: generate sampled, forced"},
                                 {"delay: generate wide text top_k", "delay: generate wide text top_k, forced"}};
  int gi = 0;
  for (const mtts_sampling* sp : {&greedy, &sampled, &wide}) {
    int fi = 0;
    for (const int32_t* f : {(const int32_t*)nullptr, (const int32_t*)d_forced}) {
      phase(gen_names[gi][fi++]);
      int n = 0;
      OK(mtts_generate(e, d_gp, d_gm, B, T, max_new, sp, f, 8, &n, nullptr));
      EXPECT(n >= 1 && n <= max_new, "generated rows");
      OK(mtts_generate_fetch(e, d_out, n, nullptr));
      OK(mtts_generate_logits(e, d_logits, nullptr));
      int hs = -1;
      OK(mtts_generate_stats(e, &hs));
      // (0 is valid: a prompt continuing in audio mode gates the text head from step 0 on)
      EXPECT(hs >= 0 && hs <= max_new, "text head steps");
    }
    ++gi;
  }
  // stepwise API
  phase("delay: stepwise begin / poll / decode");
  OK(mtts_generate_begin(e, d_gp, d_gm, B, T, max_new, &sampled, nullptr, nullptr));
  int steps = 0, done = -2;
  OK(mtts_generate_poll(e, &steps, &done, nullptr));
  OK(mtts_generate_decode(e, 5, nullptr));
  OK(mtts_generate_poll(e, &steps, &done, nullptr));
  EXPECT(steps >= 1, "steps");
  EXPECT(mtts_generate(e, d_gp, d_gm, B, T, c.max_ctx, &greedy, nullptr, 8, &steps, nullptr) == MTTS_E_INVALID,
         "max_new beyond capacity");
  EXPECT(mtts_generate_fetch(e, d_out, -1, nullptr) == MTTS_E_INVALID, "bad n_rows");
  // capacity regrow keeps the weights; generate again at the larger size
  phase("delay: reserve + generate at the larger capacity");
  OK(mtts_engine_reserve(e, 4, 256, 128));
  {
    int n = 0;
    OK(mtts_generate(e, d_gp, d_gm, B, T, 40, &greedy, nullptr, 16, &n, nullptr));
  }
  EXPECT(mtts_engine_reserve(e, 0, 256, 0) == MTTS_E_INVALID, "bad reserve");
  // roofline probe
  phase("delay: time_gemv probes");
  float ms = 0.f;
  uint64_t nb = 0;
  for (int which = 0; which < 5; ++which) OK(mtts_engine_time_gemv(e, which, 0, 2, 3, &ms, &nb));
  EXPECT(mtts_engine_time_gemv(e, 9, 0, 1, 1, &ms, &nb) == MTTS_E_INVALID, "bad which");
  EXPECT(mtts_engine_time_gemv(e, 6, 0, 1, 1, &ms, &nb) == MTTS_E_UNSUPPORTED, "depth stack on a Delay engine");
  EXPECT(mtts_local_forward(e, d_ids, mask.data(), 1, 1, 0, -1, nullptr, d_logits, ld, nullptr) == MTTS_E_UNSUPPORTED,
         "local entry point on a MossTTSDelay engine");
  phase("delay: destroy");
  OK(mtts_engine_destroy(e));
  for (void* p : {(void*)dsrc, (void*)d_ids, (void*)d_logits, (void*)d_gp, (void*)d_gm, (void*)d_forced, (void*)d_out})
    hipFree(p);
}

static void local_engine() {
  const int n_vq = 4, C = n_vq + 1, B = 2, T = 12;
  mtts_config c = tiny(n_vq, MTTS_MODEL_LOCAL);
  mtts_engine* e = nullptr;
  phase("local: create + init_random");
  OK(mtts_engine_create(&c, 0, &e));
  if (!e) return;
  OK(mtts_engine_init_random(e, 5));
  std::vector<int64_t> ids = prompt(B, T + 1, C, 3);
  int64_t* d_ids = dev<int64_t>(ids.size());
  hipMemcpy(d_ids, ids.data(), ids.size() * 8, hipMemcpyHostToDevice);
  uint8_t* d_m = dev<uint8_t>((size_t)B * (T + 1));
  hipMemset(d_m, 1, (size_t)B * (T + 1));
  const int ld = (c.vocab + 7) / 8 * 8;
  uint16_t* d_lg = dev<uint16_t>((size_t)C * B * ld);
  int64_t* d_forced = dev<int64_t>((size_t)B * C);
  phase("local: teacher-forced frames");
  OK(mtts_local_forward(e, d_ids, d_m, B, T, 0, -1, d_forced, d_lg, ld, nullptr));
  OK(mtts_local_forward(e, d_ids, d_m, B, T, 0, 2, d_forced, d_lg, ld, nullptr));
  EXPECT(mtts_local_forward(e, d_ids, d_m, B, T, 0, -1, d_forced, d_lg, 8, nullptr) == MTTS_E_INVALID, "small ld");
  mtts_sampling sp{1.5f, 1.f, 50, 1.0f, 0.95f, 50, 1.1f, 4};
  int64_t* d_out = dev<int64_t>((size_t)B * (T + 16) * C);
  int n = 0;
  phase("local: generate greedy / sampled");
  OK(mtts_local_generate(e, d_ids, nullptr, B, T, 8, -1, nullptr, 4, &n, nullptr));
  OK(mtts_local_generate(e, d_ids, nullptr, B, T, 8, 2, &sp, 4, &n, nullptr));
  OK(mtts_generate_fetch(e, d_out, n, nullptr));
  phase("local: per-channel sampling tables");
  std::vector<mtts_channel_sampling> ch(C);
  for (int i = 0; i < C; ++i) ch[i] = mtts_channel_sampling{i % 2, 1.0f + 0.5f * i, i == 0 ? 20 : 0, 0.9f, 1.2f};
  OK(mtts_local_set_sampling(e, ch.data(), C));
  OK(mtts_local_generate(e, d_ids, nullptr, B, T, 8, -1, &sp, 4, &n, nullptr));
  ch[0] = mtts_channel_sampling{1, 1.0f, 0, 1.0f, 1.0f};  // sampled text without top_k: the key-bin walk
  OK(mtts_local_set_sampling(e, ch.data(), C));
  OK(mtts_local_generate(e, d_ids, nullptr, B, T, 8, -1, &sp, 4, &n, nullptr));
  OK(mtts_local_set_sampling(e, nullptr, 0));
  EXPECT(mtts_local_set_sampling(e, ch.data(), C + 1) == MTTS_E_INVALID, "too many channels");
  phase("local: frame bytes + time_gemv probes + destroy");
  uint64_t fb = 0;
  OK(mtts_local_frame_bytes(e, -1, &fb));
  float ms = 0.f;
  uint64_t nb = 0;
  OK(mtts_engine_time_gemv(e, 6, 1, B, 5, &ms, &nb));
  OK(mtts_engine_time_gemv(e, 7, 0, B, 5, &ms, &nb));
  EXPECT(mtts_engine_time_gemv(e, 6, c.local_layers, B, 1, &ms, &nb) == MTTS_E_INVALID, "bad depth layer");
  OK(mtts_engine_destroy(e));
  for (void* p : {(void*)d_ids, (void*)d_m, (void*)d_lg, (void*)d_forced, (void*)d_out}) hipFree(p);
}

static void codec() {
  mtts_codec_config k{};
  k.n_q = 4; k.codebook_size = 1024; k.n_stages = 2;
  k.stages[0] = mtts_codec_stage{128, 2, 2, 1, 64, 256, 2};
  k.stages[1] = mtts_codec_stage{64, 1, 2, 2, 32, 128, 1};
  k.patch = 24; k.rope_theta = 10000.f; k.rms_eps = 1e-6f; k.max_batch = 2; k.max_frames = 64; k.max_chunk_frames = 6;
  mtts_codec* d = nullptr;
  phase("codec: create / decode / chunked decode / load_weight / destroy");
  OK(mtts_codec_create(&k, 0, &d));
  if (!d) return;
  OK(mtts_codec_init_random(d, 3));
  const int spf = mtts_codec_samples_per_frame(d);
  EXPECT(spf == 48, "samples per frame");
  const int B = 2, T = 13;
  std::vector<int64_t> codes((size_t)B * T * 4);
  for (size_t i = 0; i < codes.size(); ++i) codes[i] = (int64_t)(i * 37 % 1024);
  int64_t* dc = dev<int64_t>(codes.size());
  hipMemcpy(dc, codes.data(), codes.size() * 8, hipMemcpyHostToDevice);
  float* wav = dev<float>((size_t)B * T * spf);
  OK(mtts_codec_decode(d, dc, B, T, 4, 4, wav, (size_t)T * spf, nullptr));
  OK(mtts_codec_reset(d));
  OK(mtts_codec_decode(d, dc, B, 5, 4, 2, wav, (size_t)T * spf, nullptr));
  EXPECT(mtts_codec_position(d) == 5, "position");
  std::vector<uint16_t> w((size_t)24 * 64, 0x3c00);
  OK(mtts_codec_load_weight(d, "decoder.out_proj.weight", w.data(), w.size() * 2, 0));
  EXPECT(mtts_codec_load_weight(d, "decoder.stages.7.norm.weight", w.data(), 128, 0) == MTTS_E_INVALID, "bad stage");
  EXPECT(mtts_codec_decode(d, dc, 3, T, 4, 4, wav, (size_t)T * spf, nullptr) != 0, "batch beyond capacity");
  uint64_t wb = 0;
  OK(mtts_codec_weight_bytes(d, &wb));
  OK(mtts_codec_destroy(d));
  hipFree(dc);
  hipFree(wav);
}

static void kernels() {
  // kernel-level entry points on caller-owned buffers
  phase("kernel-level entry points");
  const int B = 2, N = 48, K = 64;
  const size_t pb = mtts_k_packed_bytes(N, K);
  uint16_t* w = dev<uint16_t>((size_t)N * K);
  uint16_t* wp = dev<uint16_t>(pb / 2);
  uint16_t* x = dev<uint16_t>((size_t)B * K);
  uint16_t* y = dev<uint16_t>((size_t)B * N);
  OK(mtts_k_pack(w, wp, N, K, 0, 0, 0, nullptr));
  OK(mtts_k_gemv(wp, x, K, y, N, nullptr, 0, B, N, K, 0, 0, 1, 0, nullptr));
  EXPECT(mtts_k_gemv(wp, x, K, y, N, nullptr, 0, B, N, 33, 0, 0, 1, 0, nullptr) == MTTS_E_INVALID, "K % 32");
  OK(mtts_k_gemm(wp, x, K, y, N, nullptr, 0, B, N, K, 0, nullptr, 0, nullptr));
  OK(mtts_k_rmsnorm(x, 0, K, x, y, B, K, 1e-6f, nullptr));
  std::vector<uint16_t> cs(16 * 8), sn(16 * 8);
  OK(mtts_rope_table(10000.f, 16, 8, cs.data(), sn.data()));
  EXPECT(mtts_rope_table(10000.f, 15, 8, cs.data(), sn.data()) == MTTS_E_INVALID, "odd D");
  OK(mtts_k_fill_uniform(w, (size_t)N * K, 1, 2, 0.5f, 0.f, nullptr));
  hipDeviceSynchronize();
  for (void* p : {(void*)w, (void*)wp, (void*)x, (void*)y}) hipFree(p);
}

int main(int argc, char** argv) {
  // --build-id: the source hash compiled into this driver (moss_tts_amd/_buildid.py --scope asan),
  // checked against the tree before any GPU test runs (tests/conftest.py); touches no GPU
  if (argc > 1 && strcmp(argv[1], "--build-id") == 0) {
    printf("%s\n", mtts_build_id());
    return 0;
  }
  const char* lp = getenv("MTTS_ASAN_LOG");
  g_log = lp && *lp ? fopen(lp, "a") : nullptr;
  if (!g_log) g_log = stderr;
  const char* lim = getenv("MTTS_ASAN_PHASE_TIMEOUT");
  std::thread(watchdog, lim && atoi(lim) > 0 ? atoi(lim) : 90).detach();
  phase("HIP init");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    fprintf(stderr, "no GPU\n");
    return 2;
  }
  EXPECT(mtts_version() >= 1, "version");
  mtts_engine* e = nullptr;
  mtts_config bad = tiny(4, MTTS_MODEL_DELAY);
  bad.hidden = 63;
  EXPECT(mtts_engine_create(&bad, 0, &e) == MTTS_E_UNSUPPORTED && !e, "bad shape refused");
  EXPECT(mtts_engine_create(nullptr, 0, &e) == MTTS_E_INVALID, "null config");
  delay_engine();
  local_engine();
  codec();
  kernels();
  phase("final device synchronize");
  hipDeviceSynchronize();
  phase("exit (LeakSanitizer leak check, runtime teardown)");
  printf("asan driver: %s (%d failed checks)\n", g_fail ? "FAILED" : "ok", g_fail);
  return g_fail ? 1 : 0;
}
