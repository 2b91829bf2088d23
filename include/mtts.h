/* mtts.h -- C ABI of libmtts.so, the MI355X (gfx950) MossTTSDelay decode engine.
 *
 * Drop-in boundary.  The Python package `moss_tts_amd` binds these
 * entry points with ctypes; any other host (cgo, JNI, N-API) can bind them the same
 * way.  No torch types cross this boundary: plain pointers, sizes
 * and a hipStream_t (passed as void*; NULL = the legacy default stream).  Engine calls
 * run on the engine's own stream, fenced by events after the caller's stream and before
 * its later work, so results are ordered like any other work on the caller's stream.
 * All `*_dev` pointers are device memory owned by the caller; the engine owns weights,
 * KV cache and workspaces.
 *
 * Errors: every function returns 0 on success or a negative MTTS_E_* code;
 * mtts_last_error() returns a thread-local message.  Threading: one engine = one
 * device = one stream at a time (not re-entrant per engine); engines on different
 * devices may run concurrently (one process per GPU for data parallelism).
 */
#ifndef MTTS_H
#define MTTS_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTTS_OK 0
#define MTTS_E_INVALID -1     /* bad shape / argument (reference raises ValueError) */
#define MTTS_E_OOM -2
#define MTTS_E_HIP -3         /* HIP runtime error */
#define MTTS_E_UNSUPPORTED -4 /* config the kernels do not cover */
#define MTTS_E_PSE_TIMEOUT -5 /* the batch-1 persistent decode launch timed out (device shared): results of
                                 the current generation are invalid; the engine has switched to the per-op
                                 launches, so restarting the generation succeeds (mtts_generate does) */

typedef struct mtts_engine mtts_engine;

/* longest context (prompt + max_new_tokens) an engine reserves: 2.9 hours of 12.5 Hz frames, past
 * the 60-minute single session of the TTSD model card (docs/moss_ttsd_model_card.md:21) */
#define MTTS_MAX_CTX 131072

/* Model + capacity configuration.  Model fields restate MossTTSDelayConfig
 * (moss_tts_delay/configuration_moss_tts.py:62-103) and the nested Qwen3Config. */
typedef struct mtts_config {
  int hidden, layers, n_heads, n_kv, head_dim, inter, vocab;
  int n_vq, audio_vocab; /* audio heads/embeddings have audio_vocab + 1 rows */
  float rope_theta, rms_eps;
  int pad_token_id, im_start_token_id, im_end_token_id, audio_start_token_id, audio_end_token_id;
  int audio_user_slot_token_id, audio_assistant_gen_slot_token_id, audio_assistant_delay_slot_token_id;
  int audio_pad_code;
  /* capacity */
  int max_batch;          /* rows per generate() call */
  int max_ctx;            /* prompt + max_new_tokens */
  int max_prefill_tokens; /* rows x prompt tokens processed per prefill chunk */
  /* model family: MTTS_MODEL_DELAY (MossTTSDelay) or MTTS_MODEL_LOCAL (MossTTSLocal:
   * backbone + depth transformer, moss_tts_local/configuration_moss_tts.py:60-110) */
  int model_kind;
  int local_hidden, local_layers, local_inter; /* depth transformer (local_*_size) */
  int local_mlp_ffn;                           /* additional_mlp_ffn_hidden_size of the adapters */
  int eos_token_id;                            /* generation_config.eos_token_id (Local stop id) */
} mtts_config;

#define MTTS_MODEL_DELAY 0
#define MTTS_MODEL_LOCAL 1

/* generate() keyword arguments (modeling_moss_tts.py:393-405); temperature <= 0 = greedy */
typedef struct mtts_sampling {
  float text_temperature, text_top_p;
  int text_top_k;
  float audio_temperature, audio_top_p;
  int audio_top_k;
  float audio_repetition_penalty;
  uint64_t seed; /* Philox key for the multinomial draws */
} mtts_sampling;

const char* mtts_last_error(void);
int mtts_version(void);
/* sha256 (hex) of the sources this library was built from (moss_tts_amd/_buildid.py): ties a
 * prebuilt binary to its tree; the Python binding refuses a mismatch. */
const char* mtts_build_id(void);

/* ---- engine lifecycle --------------------------------------------------- */
/* replaces AutoModel.from_pretrained(...).to(device) (clis/moss_tts_app.py:95-107) */
int mtts_engine_create(const mtts_config* cfg, int device, mtts_engine** out);
int mtts_engine_destroy(mtts_engine* eng);
/* Re-size the capacity buffers (KV cache, workspaces, generate state); weights are kept. */
int mtts_engine_reserve(mtts_engine* eng, int max_batch, int max_ctx, int max_prefill_tokens);
/* Load one tensor by its reference state_dict name (modeling_moss_tts.py:170-191,
 * e.g. "language_model.layers.3.mlp.gate_proj.weight"); src is bf16 row-major in the
 * reference shape, on the host (src_on_device = 0) or the device (1).  The engine
 * repacks matrices into its MFMA-tile layout. */
int mtts_engine_load_weight(mtts_engine* eng, const char* name, const void* src, size_t bytes, int src_on_device);
/* The same, ordered after `stream` (a device source may still be being written there): the
 * repack runs on the engine stream behind an event of `stream`, and `stream`'s later work waits
 * for it -- no device-wide sync.  mtts_engine_load_weight = this with the legacy default stream. */
int mtts_engine_load_weight_stream(mtts_engine* eng, const char* name, const void* src, size_t bytes,
                                   int src_on_device, void* stream);
/* Fill every weight with the portable splitmix64 init of oracle/prng.py (benchmarks). */
int mtts_engine_init_random(mtts_engine* eng, uint64_t seed);
/* Total bytes of weights streamed per decode step (for roofline accounting). */
int mtts_engine_weight_bytes(const mtts_engine* eng, uint64_t* bytes);
/* Roofline probe: average duration (HIP events, engine stream) of one GEMV of the loaded
 * model -- which: 0 q|k|v, 1 o_proj, 2 gate|up+SwiGLU, 3 down, 4 heads -- and its
 * algorithmic bytes per launch (weights once + activations + outputs); which 5: the
 * persistent streaming decode stack (every layer in one launch, B = 1 or 4, at the engine's
 * current decode position; bytes = all layer weights + the K/V rows read); which 6 / 7
 * (MossTTSLocal): the depth stack's gate|up+SwiGLU / down of depth layer `layer`, launched as
 * the channel loop launches them, walking the depth layers. */
int mtts_engine_time_gemv(mtts_engine* eng, int which, int layer, int B, int iters, float* avg_ms,
                          uint64_t* alg_bytes);

/* ---- forward (teacher-forced; MossTTSDelayModel.forward, modeling_moss_tts.py:225-300) ----
 * Appends S tokens per row at positions past..past+S-1 (left pads included, like
 * TF/.../modeling_qwen3.py:386-389).  ids_dev int64 [B,S,1+n_vq]; mask_dev uint8
 * [B, past+S] (1 = attend); logits_dev bf16 [B, heads_ld] receives the last position's
 * logits of all 1+n_vq heads concatenated (text | audio_0 | ...), audio pad column = -inf. */
int mtts_forward(mtts_engine* eng, const int64_t* ids_dev, const uint8_t* mask_dev, int B, int S, int past,
                 uint16_t* logits_dev, void* stream);
int mtts_heads_ld(const mtts_engine* eng);
/* 1 when batch-1 decode steps run the decoder stack as one persistent launch with run-ahead
 * weight streaming (default; MTTS_PSE=0 at creation turns it off; MossTTSDelay-8B shape,
 * 256 CUs), else 0.  It is taken by the decode steps of a generation (and teacher-forced
 * forwards) whose context stays within mtts_pse_ctx_max (MTTS_PSE_CTX); later steps of the
 * same generation take the per-op launches. */
int mtts_pse_active(const mtts_engine* eng);
/* the same for batch-4 decode steps (configs[2]'s per-GPU share: pse4.hip; MTTS_PSE4=0 turns it off) */
int mtts_pse4_active(const mtts_engine* eng);
/* 1 when batch-1 steps past mtts_pse_ctx_max take the launch's long-context form (every CU scores a
 * slice of each KV head's cached keys, merge units combine them; MTTS_PSE_LONG=0: per-op launches) */
int mtts_pse_long_active(const mtts_engine* eng);
int mtts_pse_ctx_max(const mtts_engine* eng);
/* MossTTSLocal engines: 1 when each channel of a frame's depth stage (adapter in, the depth layers,
 * local_transformer.norm, adapter out) runs as one persistent launch (lpse.hip; the 1.7B depth
 * shape, <= 8 rows, 256 CUs; opt-in: MTTS_LPSE=1 at creation), else 0.  A timed-out launch
 * is handled like the Delay launch's: mtts_generate_poll reports MTTS_E_PSE_TIMEOUT and the engine
 * continues on the per-op launches (mtts_local_generate restarts once); mtts_local_forward checks
 * its own launches and recomputes the frame. */
int mtts_local_lpse_active(const mtts_engine* eng);
/* Fault injection (tests): mark the persistent launch's error word as if a wait had timed out.
 * The next check (a teacher-forced batch-1 forward, or mtts_generate_poll) takes the fallback:
 * the launch is turned off for this engine and the work re-runs on the per-op launches.
 * (MossTTSLocal engines: the persistent channel launch's word.) */
int mtts_pse_inject_timeout(mtts_engine* eng);
/* A one-token mtts_forward through a persistent launch checks the launch's error word before it
 * returns (default): a timed-out launch is recomputed on the per-op launches inside the same call,
 * so the logits it returns are valid (the engine then stays on the per-op launches).
 * mtts_engine_set_pse_lazy(eng, 1) opts into the non-synchronising form: the word is copied
 * asynchronously and checked lazily -- without blocking at the next mtts_forward, blocking here
 * and at mtts_generate_begin.  MTTS_E_PSE_TIMEOUT (reported once, by this call or the next
 * mtts_forward, also when a generation start found it first): a launch timed out, the logits of
 * the lazy forwards since the last clean check are invalid, and the engine now runs the per-op
 * launches (recompute those forwards).  Also reads the word of forwards the caller captured into
 * its own graph.  0: every forward so far is valid. */
int mtts_engine_set_pse_lazy(mtts_engine* eng, int lazy);
int mtts_pse_check(mtts_engine* eng);
/* per-layer event stamps (s_memrealtime, 100 MHz) of the last persistent streaming launch:
 * [layers][20][256 workgroups] (engine created with MTTS_PSE_TRACE=1; see pse.hip) */
int mtts_pse_trace(mtts_engine* eng, uint64_t* host, size_t n);

/* test hooks: write bf16 K / V rows [n_kv][n][head_dim] (host) at positions pos0.. of batch row
 * b, layer `layer` (the cache of a long context without prefilling it); fill the whole KV cache
 * with one bf16 bit pattern (e.g. NaN: rows never written must never reach a result) */
int mtts_engine_kv_write(mtts_engine* eng, int layer, int b, int pos0, int n, const uint16_t* k_host,
                         const uint16_t* v_host);
int mtts_engine_kv_fill(mtts_engine* eng, uint16_t bits);

/* ---- generate (MossTTSDelayModel.generate, modeling_moss_tts.py:392-525) ----
 * begin: state init + prefill + the step-0 sampling.  decode: n more steps (hipGraph).
 * forced_text_dev (int32 [max_new_tokens], -1 = free) optionally overrides the text token
 * of rows that sample the text channel (benchmark schedule); pass NULL normally. */
int mtts_generate_begin(mtts_engine* eng, const int64_t* ids_dev, const uint8_t* mask_dev, int B, int T,
                        int max_new_tokens, const mtts_sampling* sp, const int32_t* forced_text_dev, void* stream);
int mtts_generate_decode(mtts_engine* eng, int n_steps, void* stream);
/* synchronises the stream; *steps = sampled steps so far, *done_step = step at which
 * every row had emitted im_end (-1 if none) */
int mtts_generate_poll(mtts_engine* eng, int* steps, int* done_step, void* stream);
/* accounting: decode steps (step 0 included) whose logits needed the full text head, i.e.
 * some row sampled the text channel outside audio mode.  Other steps evaluate only the
 * 16-row text tiles holding the special ids plus the audio heads. */
int mtts_generate_stats(mtts_engine* eng, int* text_head_steps);
/* whole loop: begin + decode in chunks until every row stopped or max_new_tokens;
 * *n_rows = generated rows per sequence (reference generation_ids width - T) */
int mtts_generate(mtts_engine* eng, const int64_t* ids_dev, const uint8_t* mask_dev, int B, int T,
                  int max_new_tokens, const mtts_sampling* sp, const int32_t* forced_text_dev, int chunk,
                  int* n_rows, void* stream);
/* copy generation_ids [B, T + n_rows, 1+n_vq] (prompt included) to out_dev */
int mtts_generate_fetch(mtts_engine* eng, int64_t* out_dev, int n_rows, void* stream);
/* parity hook: copy the logits the last sampled step drew from (bf16 [B, heads_ld], the
 * layout of mtts_forward; when no row sampled text outside audio mode, only the text tiles
 * holding the special ids are current) to out_dev */
int mtts_generate_logits(mtts_engine* eng, uint16_t* out_dev, void* stream);

/* ---- MossTTSLocal (model_kind == MTTS_MODEL_LOCAL) -------------------------------------
 * Weights load by the reference names of moss_tts_local/modeling_moss_tts.py
 * (model.embedding_list.{i}, model.language_model.*, local_transformer.*,
 * speech_embedding_to_local_mlp.*, local_to_speech_embedding_mlps.{i}.*,
 * layer_norm_before_lm_heads.{i}, lm_heads.{i}).  Poll and fetch are mtts_generate_poll /
 * mtts_generate_fetch.  n_vq_for_inference < 0: all channels.
 * Replaces CustomMixin._sample (moss_tts_local/modeling_moss_tts.py:315-477): greedy channels
 * (temperature <= 0) or the HF processor chain with any top_k (<= 0: none), top_p, penalty. */
int mtts_local_generate_begin(mtts_engine* eng, const int64_t* input_ids_dev, const uint8_t* attention_mask_dev, int B,
                              int T, int max_new_tokens, int n_vq_for_inference, const mtts_sampling* sampling,
                              void* stream);
int mtts_local_generate_decode(mtts_engine* eng, int n_steps, void* stream);
/* Per-channel processors of generation_config.do_samples / .layers (:356-368) for the next
 * mtts_local_generate_begin / mtts_local_generate calls: channel i < n takes ch[i] (temperature,
 * top_k <= 0 = none, top_p 1 = none, repetition_penalty, ignored on channel 0); the sampling
 * struct then only supplies the seed.  n = 0 reverts to its text_* / audio_* split. */
typedef struct mtts_channel_sampling {
  int do_sample;
  float temperature;
  int top_k;
  float top_p;
  float repetition_penalty;
} mtts_channel_sampling;
int mtts_local_set_sampling(mtts_engine* eng, const mtts_channel_sampling* ch, int n);
int mtts_local_generate(mtts_engine* eng, const int64_t* input_ids_dev, const uint8_t* attention_mask_dev, int B, int T,
                        int max_new_tokens, int n_vq_for_inference, const mtts_sampling* sampling, int chunk_steps,
                        int* n_rows, void* stream);
/* Teacher-forced frame: backbone over S tokens at `past` (mask [B, past+S]), then the depth
 * loop feeding forced_dev[b, i] ([B, 1+n_vq] int64) to channel i+1.  logits_dev receives
 * channel i's logits at + i*B*ld (bf16 [n_ch][B][ld], ld >= vocab; audio pad column -inf). */
int mtts_local_forward(mtts_engine* eng, const int64_t* ids_dev, const uint8_t* mask_dev, int B, int S, int past,
                       int n_vq_for_inference, const int64_t* forced_dev, uint16_t* logits_dev, int ld, void* stream);
/* weight bytes one frame streams (backbone + n_ch x depth stage + heads) */
int mtts_local_frame_bytes(const mtts_engine* eng, int n_vq_for_inference, uint64_t* bytes);
/* MossTTSLocal channel pick on B rows of bf16 logits [B, ld] (V columns) for channel ch:
 * temperature <= 0: argmax; else HF RepetitionPenalty (ch >= 1, over seen [B][C][audio_rows])
 * -> Temperature -> TopK -> TopP -> multinomial (Philox(seed; step, row, ch)).  out[b*C + ch].
 * Restates the realprocessor chain of moss_tts_local/modeling_moss_tts.py:356-419. */
int mtts_k_local_pick(const uint16_t* logits, int ld, int V, int ch, const uint8_t* seen_dev, int64_t* out_dev, int C,
                      int B, int audio_rows, float temperature, int top_k, float top_p, float penalty, uint64_t seed,
                      int step, void* stream);
/* bf16 MossTTSRMSNorm (no fp32 upcast, modeling_moss_tts.py:34-44), x/y [M, H] */
int mtts_k_moss_rmsnorm(const uint16_t* x, const uint16_t* w, uint16_t* y, int M, int H, float eps, void* stream);

/* ---- kernel-level entry points (unit parity; device pointers, explicit shapes) ---- */
/* pack W [rows,K] bf16 into MFMA tiles; interleave=1 places gate/up tile pairs */
int mtts_k_pack(const uint16_t* src, uint16_t* dst, int rows, int K, int row_offset, int interleave, int which,
                void* stream);
size_t mtts_k_packed_bytes(int rows, int K);
/* y[B,N] = epi(x[B,K] . W^T); epi 0 store, 1 residual add (res), 2 swiglu (N = I), 3 logits */
int mtts_k_gemv(const uint16_t* wpacked, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                int ldres, int B, int N, int K, int epi, int pad_start, int pad_period, int pad_off, void* stream);
/* as mtts_k_gemv plus the fused RMSNorm prologue (ss_in: per-16-column sums of squares of x,
 * norm_w: RMSNorm weight; NULL = off; needs (min(B,32)+1)*K*2 <= 48 KiB, the normalised rows
 * are staged in LDS), the residual epilogue's sums of squares (ss_out) and a waves-per-block
 * override (0 = automatic, 4/8/16) */
int mtts_k_gemv_ex(const uint16_t* wpacked, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                   int ldres, int B, int N, int K, int epi, const float* ss_in, int ld_ss, int n_ss,
                   const uint16_t* norm_w, float eps, float* ss_out, int ld_ss_out, int force_nw, void* stream);
/* split-K form of the residual GEMV (epi 1) for projections with few 16-row output tiles:
 * y[B,N] = res + bf16(x . W^T), ss_out per-16-column sums of squares (NULL: skip); B <= 16,
 * splits >= 2 (mtts_k_gemv_splitk_splits gives the engine's choice, 1 = not worth splitting);
 * ws_dev: mtts_k_gemv_splitk_ws_bytes bytes, zero-filled before the first call (kept zero). */
size_t mtts_k_gemv_splitk_ws_bytes(int N, int splits);
int mtts_k_gemv_splitk_splits(int N, int K, int B);
int mtts_k_gemv_splitk(const uint16_t* wpacked, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                       int ldres, int B, int N, int K, int splits, float* ss_out, int ld_ss_out, void* ws_dev,
                       void* stream);
/* prefill form: y[M,N] = epi(x[M,K] . W^T) for any token count M (epi 0 store, 1 residual
 * add + per-16-column sums of squares into ss_out when non-NULL, 2 swiglu) */
int mtts_k_gemm(const uint16_t* wpacked, const uint16_t* x, int ldx, uint16_t* y, int ldy, const uint16_t* res,
                int ldres, int M, int N, int K, int epi, float* ss_out, int ld_ss_out, void* stream);
/* the prefill projections' packed-activation form (the engine's >= 33-row prompts; M >= 33): x_packed holds
 * ceil(M / 16) token tiles in the fragment order xpkT_index (kernels.h: u16 index
 * ((((k / 32) T + m / 16) 64 + m % 16 + 16 ((k % 32) / 8)) 8 + k % 8), T = ceil(M / 16)); y row-major
 * (epi 0 / 1) or, y_packed = 1 (epi 2 only, the down projection's input), packed the same way over
 * N columns.  ws_dev / ws_floats: fp32 split-K partials (0: no split). */
int mtts_k_gemm_packed(const uint16_t* wpacked, const uint16_t* x_packed, uint16_t* y, int ldy, int y_packed,
                       const uint16_t* res, int ldres, int M, int N, int K, int epi, float* ss_out, int ld_ss_out,
                       float* ws_dev, size_t ws_floats, void* stream);
int mtts_k_rmsnorm(const uint16_t* x, size_t x_off, size_t x_stride, const uint16_t* w, uint16_t* y, int M, int H,
                   float eps, void* stream);
int mtts_k_embed(const int64_t* ids, int C, const uint16_t* emb_text, const uint16_t* emb_audio, int audio_rows,
                 int H, uint16_t* h, int M, void* stream);
/* q/k RMSNorm + RoPE (cos/sin bf16 [max_pos, D]) + cache append; pos_base_dev int32 */
int mtts_k_qk_norm_rope(const uint16_t* qkv, uint16_t* q_out, uint16_t* kc, uint16_t* vc, const uint16_t* qn_w,
                        const uint16_t* kn_w, const uint16_t* cos_t, const uint16_t* sin_t, const int32_t* pos_base_dev,
                        int M, int S, int Hq, int Hkv, int D, int Cmax, float eps, void* stream);
/* attention over the cache; q [M, Hq*D]; workspace_dev >= mtts_k_attention_ws_bytes */
size_t mtts_k_attention_ws_bytes(int M, int Hq, int D, int n_split);
int mtts_k_attention(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const uint8_t* mask,
                     const int32_t* pos_base_dev, uint16_t* out, void* workspace_dev, int M, int S, int Hq, int Hkv,
                     int D, int Cmax, int CH, int n_split, void* stream);
/* flash-form prefill attention (no workspace): q [M = B*S, Hq*D] (normed + roped), caches
 * already holding the S new tokens at *pos_dev .. +S-1; out [M, Hq*D]; D in {16, 32, 64, 128} */
int mtts_k_attention_prefill(const uint16_t* q, const uint16_t* kc, const uint16_t* vc, const uint8_t* mask,
                             const int32_t* pos_dev, uint16_t* out, int M, int S, int Hq, int Hkv, int D, int Cmax,
                             void* stream);
/* fused decode step of one layer's attention: q/k RMSNorm + RoPE of the new token (qkv
 * [B, (Hq+2Hkv)*D]), k/v appended to the cache at *pos_dev, attention over keys 0..pos
 * under mask [B, Cmax] (Cmax % 64 == 0), split over the context in 128-key blocks;
 * out [B, Hq*D].  workspace_dev: mtts_k_attn_decode_ws_bytes() bytes, zero-filled before
 * the first call (the kernel leaves its arrival counters at zero).
 * Replaces Qwen3Attention.forward for q_len == 1 (TF/models/qwen3/modeling_qwen3.py:241-280). */
size_t mtts_k_attn_decode_ws_bytes(int B, int Hq, int Hkv, int D, int Cmax);
int mtts_k_attn_decode(const uint16_t* qkv, const uint16_t* qn_w, const uint16_t* kn_w, const uint16_t* cos_t,
                       const uint16_t* sin_t, uint16_t* kc, uint16_t* vc, const uint8_t* mask, const int32_t* pos_dev,
                       uint16_t* out, void* workspace_dev, int B, int Hq, int Hkv, int D, int Cmax, float eps,
                       void* stream);
/* RoPE table exactly as the engine builds it: bf16 cos/sin [n_pos, D] on the host */
int mtts_rope_table(float theta, int D, int n_pos, uint16_t* cos_host, uint16_t* sin_host);
int mtts_k_fill_uniform(uint16_t* dst, size_t n, uint64_t seed, uint64_t tensor_id, float scale, float offset,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif
