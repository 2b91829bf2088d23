// Engine internals shared by engine.cpp (MossTTSDelay) and local.cpp (MossTTSLocal).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mtts.h"
#include "kernels.h"

using namespace mtts;

int fail(int code, const std::string& msg);
#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(MTTS_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

constexpr int CH_DECODE = 64;
constexpr int CH_PREFILL = 256;
constexpr int TEXT_PARTS = 64;

struct LayerW {
  bf16_t *qkv, *o, *gu, *down, *in_norm, *post_norm, *q_norm, *k_norm;
};

// A stack of Qwen3 decoder layers with its KV cache and activation buffers: the backbone,
// or MossTTSLocal's depth transformer (no positional embedding: cos_t == nullptr).
struct Stack {
  const LayerW* L = nullptr;
  int layers = 0, H = 0, Hq = 0, Hkv = 0, D = 0, I = 0, qkv_rows = 0;
  bf16_t *kc = nullptr, *vc = nullptr;
  size_t layer_kv = 0;
  int Cmax = 0;
  const bf16_t *cos_t = nullptr, *sin_t = nullptr;
  uint8_t* mask = nullptr;  // [Bmax][Cmax]
  bf16_t *h = nullptr, *xn = nullptr, *qkvb = nullptr, *qb = nullptr, *attnb = nullptr, *act = nullptr;
  float* ss = nullptr;      // per-16-column sums of squares of h
  float* part = nullptr;
  int* att_cnt = nullptr;
  int rows = 0;             // row capacity of xn / attnb / act (>= 32: 17-32 row decode may use the packed layout)
  bool attn_direct = false; // the context never spans two attention blocks: the attention writes its
                            // rows directly and o_proj is a plain GEMV (no split partials to merge)
  int attn_nwv = 0;         // decode attention waves per block for this stack (0: the engine default)
  const int* rope_off = nullptr;  // [rows] RoPE position offsets (MossTTSLocal backbone; null: positions = slots)
};

constexpr int SK_TILES = 256;                   // split-K GEMV: most output tiles, and
constexpr size_t SK_PART_FLOATS = 4096 * 256;   // its partial workspace (tiles x splits x 256; x 2 rows halves)
constexpr size_t GK_WS_FLOATS = 8u << 20;       // prefill GEMM split-K partials (32 MB)

inline size_t packed_bytes(int rows, int K) { return (size_t)((rows + 15) / 16) * 16 * K * sizeof(bf16_t); }

struct LocalParts;  // MossTTSLocal depth stage (local.cpp)

struct mtts_engine {
  mtts_config c{};
  LocalParts* lp = nullptr;
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  int qkv_rows = 0, audio_rows = 0, heads_rows = 0, heads_ld = 0;
  std::vector<LayerW> L;
  bf16_t *emb_text = nullptr, *emb_audio = nullptr, *final_norm = nullptr, *heads = nullptr;
  bf16_t *kc = nullptr, *vc = nullptr;
  size_t layer_kv = 0;  // elements per layer in kc / vc
  bf16_t *cos_t = nullptr, *sin_t = nullptr;
  uint8_t* mask = nullptr;
  // workspace
  int Mmax = 0;
  float* ss = nullptr;  // [Mmax, H/16] per-tile sums of squares of the residual stream
  bf16_t *h = nullptr, *xn = nullptr, *qkvb = nullptr, *qb = nullptr, *attnb = nullptr, *act = nullptr;
  float* part = nullptr;
  size_t part_floats = 0;
  bf16_t* logits = nullptr;
  int* d_pos = nullptr;     // pos_base for teacher-forced forwards / prefill
  int* rope_off = nullptr;  // [max_batch]: MossTTSLocal backbone rows' left-pad counts (Stack::rope_off)
  int* att_cnt = nullptr;  // decode-attention arrival tickets [Bmax][Hkv] (zero between launches)
  int text_tile_lo = 0;    // first 16-row text-head tile holding a special id the sampler reads
  bool full_text_head = false;    // MTTS_FULL_TEXT_HEAD=1: evaluate the whole text head every step (A/B)
  bool gemv_prefill = false;      // MTTS_GEMV_PREFILL=1: prefill through the decode GEMV (A/B)
  bool unfused_attn = false;      // MTTS_UNFUSED_ATTN=1: decode attention combines in its own kernel (A/B)
  bool old_prefill_attn = false;  // MTTS_OLD_PREFILL_ATTN=1: per-token split-K prefill attention (A/B)
  // split-K residual GEMV for few-tile projections (splitk.hip); MTTS_SPLITK=0 turns it off (A/B)
  bool splitk = true;
  float* gk_ws = nullptr;    // prefill GEMM split-K partials (GK_WS_FLOATS; gemm.hip)
  float* sk_part = nullptr;  // SK_PART_FLOATS
  int* sk_cnt = nullptr;     // SK_TILES tickets, zero between launches
  // 17-32 row decode: xn / attnb / act in the fragment-packed layout (xpk_index; MTTS_XPACK=0: row-major)
  bool xpack = true;
  // persistent streaming engine (pse.hip) for the batch-1 decode stack: MTTS_PSE=1 (A/B)
  bool pse = true;               // MTTS_PSE=0: per-op launches for batch-1 decode too
  int pse_ctx_max = 768;         // PSE only while the context stays within this (MTTS_PSE_CTX):
                                 // its attention (2 CUs per KV head, every key each) loses to
                                 // the per-op split-K attention beyond ~850 cached keys
                                 // (scripts/pse_ctx_sweep.py, round 3: 0.97 at 700, 1.02 at 900)
  bool pse_now = false;          // this forward / captured decode step may take the PSE path
  // batch-1 per-op decode past this context (TTSD long form): 16-wave decode attention blocks of
  // 512 keys, half the splits to merge (MTTS_ATTN_LONG; 0: off).  TTSD shape, same box: 8 K keys
  // 3.74 -> 3.59 ms/step, but 2 K keys 3.33 -> 3.49 (too few blocks), hence the switch
  int attn_long_ctx = 4096;
  bool long_now = false;         // this forward / captured decode step takes the long form
  // batch-1 contexts past pse_ctx_max: the launch's all-CU attention form (pse.hip, round 4;
  // MTTS_PSE_LONG=0: the per-op launches there, as before)
  bool pse_long = true;
  bool pse_long_now = false;
  void pse_choose(int ctx) {
    pse_now = ctx <= pse_ctx_max;
    pse_long_now = !pse_now && pse_long;
  }
  bool pse_ok = false;           // the shape and the device support it
  // batch-4 form (pse4.hip, configs[2]'s per-GPU share): MTTS_PSE4=0 turns it off (A/B)
  bool pse4 = true;
  bool pse4_ok = false;
  unsigned char* pse4_ws = nullptr;  // pse4_ws_bytes(), zero-filled
  // the persistent launch a decode of B rows takes (when its context is in range)
  bool pse_takes(int B) const { return pse && ((B == 1 && pse_ok) || (B == 4 && pse4 && pse4_ok)); }
  uint32_t* pse_err(int B) const;
  int pse_timeouts = 0;          // launches that gave up waiting (each turns `pse` off)
  PseLayer* pse_L = nullptr;     // device [layers]
  unsigned char* pse_ws = nullptr;  // pse_ws_bytes(), zero-filled
  // teacher-forced forwards through the launch: its error word is copied asynchronously into
  // pinned host memory (no host sync per step) and checked lazily (pse_lazy_check)
  uint32_t* pse_err_host = nullptr;
  hipEvent_t ev_pse = nullptr;
  bool pse_pending = false;
  // teacher-forced forwards through a launch: by default checked synchronously (a timed-out launch
  // is recomputed on the per-op launches inside the same call); mtts_engine_set_pse_lazy(e, 1)
  // opts into the async check above (no host sync per forward; errors surface on a later call)
  bool pse_lazy = false;
  // a lazily detected timeout that a generation start swallowed (that generation is valid) is
  // still owed to the caller: the next mtts_pse_check / mtts_forward reports it once
  bool pse_unreported = false;
  bool pse_coop = false;            // MTTS_PSE_COOP=1: cooperative launch (hipLaunchCooperativeKernel)
  uint64_t* pse_trace = nullptr;    // MTTS_PSE_TRACE=1: per-layer event stamps of the last launch
  // generate state
  GenDev* st = nullptr;
  GenDev hst{};
  int *is_stopping = nullptr, *is_audio = nullptr, *text_cand = nullptr, *audio_cand = nullptr, *part_idx = nullptr;
  int64_t *audio_len = nullptr, *delayed = nullptr, *cur_ids = nullptr, *gen_ids = nullptr;
  uint8_t* seen = nullptr;
  int* wide_hist = nullptr;  // [max_batch][65536] (sampled text without a top-k cap)
  float* part_val = nullptr;
  const int* forced = nullptr;
  int gen_B = 0, gen_T = 0, gen_max_new = 0, steps_issued = 0;
  struct Graph { hipGraphExec_t exec; const int* forced; bool pse; };  // key: 8 B + 4 pse-long + 2 long + pse
  std::unordered_map<int, Graph> graphs;  // decode-step graph per batch size
  std::vector<void*> allocs;      // weights
  std::vector<void*> cap_allocs;  // capacity buffers (see alloc_capacity)
  bool cap_mode = false;
  bool unfused_norm = false;  // MTTS_UNFUSED_NORM=1: always run the separate RMSNorm kernel (A/B timing)
  int nw[5] = {0, 0, 0, 0, 0};  // waves-per-block overrides (MTTS_NW="qkv,o,gu,down,heads"; 0 = auto)
  int nu[5] = {0, 0, 0, 0, 0};  // load-batch depth overrides (MTTS_U="qkv,o,gu,down,heads"; 0 = auto, 4 / 8)
  bf16_t* staging = nullptr;
  void* load_stream = nullptr;  // the caller's stream of the weight load in progress (NULL: legacy default)
  size_t staging_bytes = 0;
  uint64_t step_weight_bytes = 0;

  template <class T>
  int alloc(T** p, size_t n) {
    void* q = nullptr;
    if (n == 0) n = 1;
    if (hipMalloc(&q, n * sizeof(T)) != hipSuccess) return fail(MTTS_E_OOM, "hipMalloc failed (" + std::to_string(n * sizeof(T)) + " B)");
    (cap_mode ? cap_allocs : allocs).push_back(q);
    *p = reinterpret_cast<T*>(q);
    return 0;
  }
  GenBufs bufs() const {
    GenBufs g;
    g.st = st; g.logits = logits; g.is_stopping = is_stopping; g.is_audio = is_audio;
    g.audio_len = audio_len; g.delayed = delayed; g.cur_ids = cur_ids; g.gen_ids = gen_ids; g.mask = mask;
    g.seen = seen; g.part_val = part_val; g.part_idx = part_idx; g.text_cand = text_cand; g.audio_cand = audio_cand;
    g.forced = forced;
    g.wide_hist = wide_hist;
    return g;
  }
};

// where a reference tensor lands: a raw copy (norms, embeddings) or an MFMA-tile repack
struct WTarget {
  bf16_t* dst = nullptr;
  bool pack = false;
  int rows = 0, K = 0, row_off = 0, inter = 0, which = 0;
  size_t expect = 0;  // elements
};

// ---- shared engine internals (engine.cpp) ----
bool layer_target(const LayerW& w, const std::string& rest, int H, int I, int Hq, int Hkv, int D, WTarget* t);
int store_weight(mtts_engine* e, const WTarget& t, const char* name, const void* src, size_t bytes, int on_dev);
// mtts_engine_load_weight without the public entry's stream bookkeeping (orders after e->load_stream)
int load_weight_impl(mtts_engine* e, const char* name, const void* src, size_t bytes, int on_dev);
int ensure_staging(mtts_engine* e, size_t bytes);
bool parse_layer(const char* name, int* layer, std::string* rest);
int normed_input(mtts_engine* e, const Stack& st, GemvArgs& g, const bf16_t* nw, int M, hipStream_t s,
                 int tiles = 0);
Stack backbone_stack(mtts_engine* e);
hipError_t proj(mtts_engine* e, const GemvArgs& g, int epi, hipStream_t s);
int run_layers(mtts_engine* e, const Stack& st, int b0, int B, int S, const int* pos_base, int CH, int n_split,
               hipStream_t s);
// backbone forward; heads == false: KV cache only, or (hidden != nullptr) the final-normed
// hidden state of each row's last token into hidden [B, H]; n_embed: channels summed (0 = all)
int forward_rows(mtts_engine* e, const int64_t* ids, int b0, int B, int S, const int* pos_base, int CH, int n_split,
                 bf16_t* logits_out, hipStream_t s, const int* text_gate = nullptr, bool heads = true,
                 bf16_t* hidden = nullptr, int n_embed = 0);
// text_gate: device flag gating the heads' text rows below the special ids (generate_begin's
// prefill: GenDev::need_text); nullptr: every head row
int forward_chunked(mtts_engine* e, const int64_t* ids, int B, int S, int past, bf16_t* logits_out, hipStream_t s,
                    bf16_t* hidden = nullptr, int n_embed = 0, const int* text_gate = nullptr);
hipStream_t enter(mtts_engine* e, void* user);
bool pse_tripped(mtts_engine* e, hipStream_t s);
void leave(mtts_engine* e, void* user);
// local.cpp (MossTTSLocal)
int local_create(mtts_engine* e);
int local_alloc_capacity(mtts_engine* e);
void local_destroy(mtts_engine* e);
void local_clear_graphs(mtts_engine* e);
int local_init_random(mtts_engine* e, uint64_t seed);
// 1: the name belongs to the local stage and was loaded (or failed: *rc set); 0: not a local name
int local_load_weight(mtts_engine* e, const char* name, const void* src, size_t bytes, int on_dev, int* rc);
// mtts_engine_time_gemv's depth-stack cases: proj 2 = gate|up, 3 = down of depth layer `layer`
int local_time_proj(mtts_engine* e, int proj_kind, int layer, int B, int iters, float* avg_ms, uint64_t* alg_bytes);
// the persistent channel launch (lpse.hip): taken for B rows; its error word (clears it, turns the
// launch off and drops the captured frames when set); the fault-injection hook
bool local_lpse_takes(const mtts_engine* e, int B);
bool local_lpse_tripped(mtts_engine* e, hipStream_t s);
int local_lpse_inject(mtts_engine* e);
