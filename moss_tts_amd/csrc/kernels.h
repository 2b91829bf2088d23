// Kernel argument structs and launch entry points shared by the HIP kernels and the engine.
#pragma once
#include "common.h"

namespace mtts {

constexpr int64_t I64MAX = 0x7fffffffffffffffLL;

enum Epi { EPI_STORE = 0, EPI_RESADD = 1, EPI_SWIGLU = 2, EPI_LOGITS = 3 };

// PRO_NORM_PRE: PRO_NORM whose inputs fit one register load per thread ((B+1)*K <= 8192,
// K <= 4096), loaded before the first weight batch (gemv_body.h)
// PRO_ATTN_PRE: PRO_ATTN with one merged element per thread (B*Hq*D/8 <= threads) whose first
// two splits' partials load before the first weight batch; PRO_ATTN_PRE2: two per thread
// PRO_NORM_PREROW: PRO_NORM_PRE for K / 8 == threads (K 4096 at 8 waves): chunk j of a thread
// is row j (the norm weight after the B rows), one load each, B <= 5
// PRO_NORM_DMA: PRO_NORM whose inputs (x rows, norm weight, sums of squares; contiguous rows)
// go straight to LDS by LDS-DMA before the first weight batch (any B <= 16 whose staging fits)
enum Pro { PRO_NONE = 0, PRO_NORM = 1, PRO_ATTN = 2, PRO_NORM_PRE = 3, PRO_ATTN_PRE = 4, PRO_NORM_PREROW = 5,
           PRO_ATTN_PRE2 = 6, PRO_NORM_DMA = 7 };
// LDS of the PRO_NORM_DMA prologue: (B+1)*K bf16 + B*n_ss fp32, each region padded to whole
// 64-chunk (1 KiB) DMA wave-instructions
inline size_t norm_dma_lds_bytes(int B, int K, int n_ss) {
  const size_t cx = ((size_t)(B + 1) * K / 8 + 63) / 64 * 64, cs = ((size_t)B * n_ss / 4 + 63) / 64 * 64;
  return (cx + cs) * 16;
}
constexpr int PREROW_MAXB = 5;
// (B <= 8: the sums of squares of row b load in wave b % NW, two rows per wave at NW = 4)
inline bool norm_preload_fits(int B, int K) { return B <= 8 && (size_t)(B + 1) * K <= 8192 && K <= 4096; }

// decode-attention split partials as read by the o_proj prologue (PRO_ATTN)
constexpr int ATTN_PO_ALL = 1 << 30;  // po_max: every split publishes, the consumer merges

struct AttnPartView {
  const float* part;   // [B][Hkv][ns][G*(D+2)]: o[G][D], then (m, l) per head
  const int* pos;      // device: position of the new token
  int Hkv, G, D, ns, kb;  // kb = keys per attention block
  int po_max;             // contexts of more than po_max blocks were merged by the attention (read x)
};

struct GemvArgs {
  const bf16_t* w;     // packed tiles
  const bf16_t* x;     // [B, ldx] activations (bf16)
  bf16_t* y;           // [B, ldy] output
  const bf16_t* res;   // residual [B, ldres] (EPI_RESADD; may alias y)
  int ldx, ldy, ldres;
  int B;               // active rows of x / y
  int N;               // valid output columns
  int K;               // reduction length (multiple of 32)
  int KT;              // K / 32
  // EPI_LOGITS: columns n >= pad_start with (n - pad_start) % pad_period == pad_off -> -inf
  int pad_start, pad_period, pad_off;
  // fused Qwen3RMSNorm of x (TF/.../modeling_qwen3.py:59-64) when ss_in != nullptr:
  //   x' = bf16(nw[k] * bf16(x[b,k] * r_b)),  r_b = 1/sqrt(sum_t ss_in[b*ld_ss + t] / K + eps)
  // where ss_in holds per-16-column partial sums of squares of x (written by the producer)
  const float* ss_in;
  int ld_ss, n_ss;
  const bf16_t* nw;
  float eps;
  // EPI_RESADD: writes the partial sum of squares of its 16 new residual columns per row
  float* ss_out;       // [B, ld_ss_out] (nullptr: skip)
  int ld_ss_out;
  int force_nw;        // 0: automatic waves-per-block choice; 4/8/16: forced (tuning)
  int force_u;         // 0: automatic load-batch depth; 4/8 k-tiles per batch: forced (tuning)
  int tile0;           // first output row tile of this launch (row ranges of one matrix)
  const int* gate;     // device flag: the launch does nothing when *gate == 0 (nullptr: always on)
  int gate_tiles;      // gated launch: output tiles, walked block-stride by a capped grid (set by launch_nw)
  int n_row_tiles;     // packed 16-row weight tiles (set by the GEMM launcher)
  AttnPartView attn;   // PRO_ATTN (o_proj): x is merged from these partials; attn.part == nullptr: off
  float* ws;           // prefill GEMM split-K workspace (gemm_ex; nullptr: no split)
  size_t ws_floats;
  // 17-32 row decode (NB = 2): x / y in the fragment-packed layout (xpk_index) instead of [B, ld]
  int x_packed, y_packed;
  int pk_tiles;        // prefill GEMM (gemm2): token tiles T of the packed x / y (0: decode form, T = 2)
  // row gather (<= 16 rows, no prologue): x is an embedding table [rows, ldx] and row b of the
  // input is x + xtok[b * ld_xtok] * ldx -- the MossTTSLocal channel embedding read by the
  // next adapter's gate|up directly (no separate embed launch); nullptr: x rows are contiguous
  const int64_t* xtok;
  int ld_xtok;
  // prefill split-K residual GEMM (EPI_RESADD, packed): when pn_w != nullptr and the launch splits
  // K, its reduce also applies the NEXT op's input Qwen3RMSNorm (weight pn_w, eps pn_eps) to the
  // new residual rows and writes them packed (xpkT_index, pn_tiles token tiles) to pn_y, and sets
  // the host flag *pn_done = 1 (the caller then skips its rmsnorm_ss launch)
  const bf16_t* pn_w;
  bf16_t* pn_y;
  int pn_tiles;
  float pn_eps;
  int* pn_done;
  // prefill split-K q|k|v GEMM (EPI_STORE, D = 128): when qkr != nullptr (host pointer) and the
  // launch splits K, its reduce runs the q/k norm + RoPE + KV append of *qkr straight from the
  // partials (y is not written) and sets the host flag *qkr_done = 1
  const struct QKRopeArgs* qkr;
  int* qkr_done;
};

// Fragment-packed activations of the 17-32 row decode GEMVs: the MFMA B-operand order of
// v_mfma_f32_16x16x32_bf16 for 32 token slots -- [k tile][token half][lane][8 k] -- so a
// wave's x fragment of one k tile is ONE contiguous 1 KiB load (row-major x puts the 16
// tokens of a fragment 16 rows apart: 16 half-used cache lines per load).  u16 index of
// (token b < 32, column k); the buffer holds 32 * K elements.
// The prefill GEMM's form holds T token tiles of 16 (T = ceil(M / 16)); the decode form is T = 2.
__host__ __device__ inline size_t xpkT_index(int b, int k, int T) {
  return ((((size_t)(k >> 5) * T + (b >> 4)) * 64 + (b & 15) + 16 * ((k & 31) >> 3)) << 3) + (k & 7);
}
__host__ __device__ inline size_t xpk_index(int b, int k) { return xpkT_index(b, k, 2); }

inline GemvArgs gemv_args(const bf16_t* w, const bf16_t* x, int ldx, bf16_t* y, int ldy, int B, int N, int K) {
  GemvArgs a{};
  a.w = w; a.x = x; a.ldx = ldx; a.y = y; a.ldy = ldy; a.B = B; a.N = N; a.K = K; a.KT = K / 32;
  a.pad_period = 1;
  return a;
}

struct QKRopeArgs {
  const bf16_t* qkv;
  bf16_t* q_out;
  bf16_t* kc;
  bf16_t* vc;
  const bf16_t* qn_w;
  const bf16_t* kn_w;
  const bf16_t* cos_t;  // [max_pos, D]
  const bf16_t* sin_t;
  const int* pos_base;  // device: position of token s=0 (same for all rows)
  // device [rows] or null: RoPE position of row b's token = max(0, pos - rope_off[b]) (MossTTSLocal:
  // GenerationMixin's positions exclude a row's left pads); the cache slot stays pos
  const int* rope_off;
  int S;                // tokens per row
  int Hq, Hkv, D;
  int Cmax;
  float eps;
  int M;
};

struct AttnArgs {
  const bf16_t* q;       // [M, Hq*D]
  const bf16_t* kc;      // [Bmax][Hkv][Cmax][D]
  const bf16_t* vc;
  const uint8_t* mask;   // [Bmax][Cmax]
  const int* pos_base;   // device: absolute position of token s=0
  float* part_o;         // [M][n_split][Hq][D]
  float* part_ml;        // [M][n_split][Hq][2]
  bf16_t* out;           // [M, Hq*D]
  int S, Hq, Hkv, D, Cmax, CH, n_split, M;
  float scale;
  int out_tiles;         // > 0: out fragment-packed with this many 16-token tiles (xpkT_index)
};

// fused decode attention: one new token per row
struct DecAttnArgs {
  const bf16_t* qkv;    // [B, (Hq + 2 Hkv) * D]  output of the q|k|v GEMV
  const bf16_t* qn_w;
  const bf16_t* kn_w;
  const bf16_t* cos_t;  // [max_pos, D]
  const bf16_t* sin_t;
  bf16_t* kc;           // layer cache [Bmax][Hkv][Cmax][D]
  bf16_t* vc;
  const uint8_t* mask;  // [Bmax][Cmax]
  const int* pos;       // device: absolute position of the new token
  const int* rope_off;  // device [B] or null: the token's RoPE position is max(0, pos - rope_off[b])
  bf16_t* out;          // [B, Hq * D]
  float* part;          // split partials [B][Hkv][ns][G*(D+2)]
  int* cnt;             // arrival tickets [B][Hkv], zero between launches
  int Hq, Hkv, D, Cmax;
  int ns;               // splits per head (set by attn_decode)
  int nwv;              // waves per block (32 keys each; set by attn_decode)
  int nwv_force;        // 4 / 8 / 16: waves per block for this call (a self-combining form; 0: automatic)
  float eps, scale;
  int publish_only;     // 1: every block writes its (m, l, o) partial; the o_proj GEMV merges them
  int po_max;           // publish_only applies up to po_max blocks per head; longer contexts merge here
  int probe;            // timing probe (MTTS_ATTN_PROBE): 0 full; 1 exit after pos; 2 after loads + prologue; 3 no combine
  int out_packed;       // out in the fragment-packed layout (xpk_index; self-combining form, B <= 32)
};

constexpr int TOPK_CAP = 2048;  // largest sampler candidate set (topk.h); the host rejects top_k above it

// MossTTSLocal: one channel's processor set (moss_tts_local/modeling_moss_tts.py:356-368)
constexpr int LOCAL_MAXC = 64;
struct ChSampling {
  int sample;          // do_samples[i]: 0 = argmax of the raw logits
  float temp, top_p;   // TemperatureLogitsWarper / TopPLogitsWarper (1.0: absent)
  float pen;           // RepetitionPenaltyLogitsProcessor (1.0: absent; never on channel 0)
  int top_k;           // TopKLogitsWarper (<= 0: absent)
};

struct GenDev {
  // scalars
  int T0;          // prompt length
  int step;        // time_step of the logits being sampled
  int fwd_pos;     // absolute position of the token fed to the next forward
  int done_step;   // first step at which every row had stopped, -1 if none yet
  int need_text;   // some row samples the text channel freely at `step` (full text head needed)
  int text_head_steps;  // decode steps that evaluated the full text head (accounting)
  int B, n_vq, C, Ltot, Cmax;
  int vocab, audio_rows;  // text vocab, 1025
  int heads_ld;           // row stride of the logits buffer
  int P, part_len;        // text partitions
  // sampling
  float text_temp, text_top_p, audio_temp, audio_top_p, rep_penalty;
  int text_top_k, audio_top_k, text_sample, audio_sample;
  unsigned long long seed;
  MttsIds ids;
  int topk_overflow;  // a sampler cut threshold ties at TOPK_CAP (reported by poll)
  ChSampling lch[LOCAL_MAXC];  // MossTTSLocal: per-channel processors
};

struct GenBufs {
  GenDev* st;
  const bf16_t* logits;  // [B, heads_ld] bf16: text | audio_0 (1025) | audio_1 ...
  int* is_stopping;      // [B]
  int* is_audio;         // [B]
  int64_t* audio_len;    // [B]
  int64_t* delayed;      // [B]
  int64_t* cur_ids;      // [B, C]
  int64_t* gen_ids;      // [B, Ltot, C]
  uint8_t* mask;         // [B, Cmax]
  uint8_t* seen;         // [2, audio_rows] union of the audio history (ch 1 | ch >= 2)
  float* part_val;       // [B, P] greedy text slice argmax
  int* part_idx;
  int* text_cand;        // [B]
  int* audio_cand;       // [B, n_vq]
  const int* forced;     // [max_new] text override for sampled rows (-1 none) or nullptr
  int* wide_hist;        // [B, 65536] key bins of the wide text sampler (text_top_k <= 0 or > TOPK_CAP)
};

// gemv.hip
hipError_t gemv(const bf16_t* wpacked, const bf16_t* x, int ldx, bf16_t* y, int ldy, const bf16_t* res, int ldres,
                int B, int N, int K, int epi, int pad_start, int pad_period, int pad_off, hipStream_t s);
// full-control form (fused norm prologue / sum-of-squares epilogue); rows > 32 are chunked.
// The fused norm stages the B normalised rows + the norm weight in LDS: (B+1)*K*2 bytes
constexpr size_t NORM_LDS_MAX = 48 * 1024;
size_t norm_lds_bytes(int B, int K);
hipError_t gemv_ex(const GemvArgs& a, int epi, hipStream_t s);
// an o_proj (EPI_RESADD) of B rows x K over N outputs would preload decode-attention partials
bool gemv_attn_preload(int B, int K, int N, int force_nw);
// gemm.hip: prefill form of gemv_ex (B = tokens, any count; EPI_STORE / RESADD / SWIGLU;
// no fused norm prologue, no gate)
hipError_t gemm_ex(const GemvArgs& a, int epi, hipStream_t s);
hipError_t pack_weight(const bf16_t* src, bf16_t* dst, int rows, int K, int row_offset, int interleave, int which,
                       hipStream_t s);
// norm_rope.hip
// sum of the embeddings of channels 0..C-1 (channel 0 from emb_text, j >= 1 from table j-1 of
// emb_audio); ids row stride ld_ids (0: C)
hipError_t embed(const int64_t* ids, int C, const bf16_t* emb_text, const bf16_t* emb_audio, int audio_rows, int H,
                 bf16_t* h, int M, hipStream_t s, float* ss_out = nullptr, int ld_ss = 0, int ld_ids = 0);
hipError_t rmsnorm(const bf16_t* x, size_t x_off, size_t x_stride, const bf16_t* w, bf16_t* y, int M, int H, float eps,
                   hipStream_t s);
hipError_t rmsnorm_ss(const bf16_t* x, size_t x_off, size_t x_stride, const float* ss, size_t ss_off, size_t ss_stride,
                      const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s, int y_tiles = 0);
hipError_t qk_norm_rope(const QKRopeArgs& a, hipStream_t s);
// attention.hip
size_t attn_smem_bytes(int G, int D, int CH);
hipError_t attention(const AttnArgs& a, hipStream_t s);
// flash-form prefill attention (no workspace, no combine); D in {32, 64, 128}
hipError_t attention_prefill(const AttnArgs& a, hipStream_t s);
hipError_t attn_decode(const DecAttnArgs& a, int B, hipStream_t s);
int attn_decode_splits(int Cmax);
int attn_decode_keys_per_block();
int attn_decode_keys_per_block_nwv(int nwv);  // nwv 0: the default waves
int attn_publish_max_splits();
// workspace of attn_decode: ticket counters (zero-filled once by the owner) + partials
size_t attn_decode_ws_bytes(int B, int Hq, int Hkv, int D, int Cmax);
// splitk.hip: split-K decode GEMV with the residual epilogue (projections with few 16-row tiles):
// splits > 1 from gemv_splitk_splits; part: gemv_splitk_ws_floats fp32, cnt: n_tiles zeroed ints
int gemv_splitk_splits(int n_tiles, int KT, int B);
size_t gemv_splitk_ws_floats(int n_tiles, int S);
hipError_t gemv_splitk(const GemvArgs& a, int S, float* part, int* cnt, hipStream_t s);
// 17-32 packed rows: RT row tiles per workgroup, K split S ways (o_proj / down_proj at B = 32);
// part: gemv_splitk2_ws_floats(n_tiles, S), cnt: n_tiles / RT zeroed ints
bool gemv_splitk2_pick(int n_tiles, int KT, int B, int* RT, int* S);
size_t gemv_splitk2_ws_floats(int n_tiles, int S);
hipError_t gemv_splitk2(const GemvArgs& a, int RT, int S, float* part, int* cnt, hipStream_t s);

// pse.hip: the batch-1 decode stack as one persistent launch with a per-CU LDS-DMA weight ring
// running ahead of the data-tagged hand-offs (MossTTSDelay-8B shape, 256 CUs)
struct PseLayer {
  const bf16_t *qkv, *o, *gu, *down, *in_norm, *post_norm, *q_norm, *k_norm;
  bf16_t *kc, *vc;  // this layer's caches (row 0)
};
struct PseArgs {
  const PseLayer* L;  // device [layers]
  int layers;
  bf16_t* h;          // [H] residual stream: in = the embedding row, out = the stack's output
  float* ss;          // [H/16] its per-16-column sums of squares (in / out)
  const bf16_t *cos_t, *sin_t;
  const uint8_t* mask;  // [Cmax] (row 0)
  const int* pos;
  int Cmax;
  float eps, scale;
  // workspace (set by pse_decode): granules and words
  uint64_t *g_qkv, *g_att, *g_h[2], *g_ss[2], *g_act;
  uint64_t* g_part;   // long-context form: per-slice attention partials [q head][half][slice][66]
  uint32_t *err, *epoch, *exit_cnt;
  int* hcnt;        // PSE_HCNT / PSE4_HCNT: residual hand-off counters [layer][2], zero between launches
  uint32_t* go;     // ... = 2: release flags [layer][2][256 CUs], one 128-byte line each (epoch values)
  uint64_t* trace;  // nullptr, or [layers][PSE_TRACE_EV][256] s_memrealtime stamps
  int probe;        // timing probe (MTTS_PSE_PROBE; results invalid): 1 loader issues no DMA,
                    // 2 consumers skip the slot reads and MFMAs
};
constexpr int PSE_TRACE_EV = 28;
size_t pse_lds_bytes();
int pse_grid(int device);
bool pse_supported(int device, int B, int layers, int H, int Hq, int Hkv, int D, int I, int qkv_rows, int Cmax);
size_t pse_ws_bytes();  // zero-filled once by the owner
// coop: hipLaunchCooperativeKernel (the runtime checks the grid's co-residency at launch and
// refuses it with hipErrorCooperativeLaunchTooLarge) instead of a plain launch
// long_ctx: the all-CU attention form (every CU scores 1/32 of a KV head's cached keys, 64 merge
// units combine the slices) for contexts past the 2-CU-per-head form's range
hipError_t pse_decode(const PseArgs& a, void* ws, hipStream_t s, bool coop = false, bool long_ctx = false);
uint32_t* pse_err_word(void* ws);
// pse4.hip: the same for a decode batch of exactly 4 rows (configs[2]'s per-GPU share); PseArgs as
// above with h [4][H], ss [4][H/16], mask [4][Cmax] (rows 0-3), the caches' rows 0-3
size_t pse4_lds_bytes();
bool pse4_supported(int device, int layers, int H, int Hq, int Hkv, int D, int I, int qkv_rows, int Cmax);
size_t pse4_ws_bytes();  // zero-filled once by the owner
hipError_t pse4_decode(const PseArgs& a, void* ws, hipStream_t s, bool coop = false);
uint32_t* pse4_err_word(void* ws);
// lpse.hip: one MossTTSLocal channel's depth stage as one persistent launch -- the adapter into
// the depth stack, its layers, local_transformer.norm and the adapter out (the 1.7B depth shape:
// LH 1536, 16 / 8 heads x 128, I 8960, adapters F 2048 to H 2048; B <= 8 rows, 256 CUs)
constexpr int LPSE_MAXL = 6;
constexpr int LPSE_MAXB = 8;
// the attention stages the keys of at most this many earlier channel positions in LDS (lpse.hip
// AKEYS), so the launch serves frames of <= LPSE_MAX_CHANNELS channels (1 + n_vq <= 33); wider
// configs keep the per-op depth loop
constexpr int LPSE_MAX_CHANNELS = 33;
struct LpseLayer {
  const bf16_t *qkv, *o, *gu, *down, *in_norm, *post_norm, *q_norm, *k_norm;
};
struct LpseArgs {
  LpseLayer L[LPSE_MAXL];
  int layers;
  // the channel's input rows x_b = tok ? table + tok[b * ld_tok] * H : in + b * H (H = 2048)
  const bf16_t* in;
  const int64_t* tok;
  int ld_tok;
  const bf16_t *mi_gu, *mi_down, *norm, *mo_gu, *mo_down;  // packed adapters, local_transformer.norm
  // activations: h [B][LH] + ss [B][LH / 16] (the depth residual stream), qkvb [B][4096],
  // attnb [B][2048], act [B][I], actF [B][F], z [B][H] (the channel output)
  bf16_t *h, *qkvb, *attnb, *act, *actF, *z;
  float* ss;
  bf16_t *kc, *vc;   // depth KV caches [layer][Bmax][Hkv][64][D], V transposed [..][D][64]
  size_t layer_kv;   // elements per layer
  int B, pos;        // rows; the channel position (the new key's slot)
  float eps, scale;
  int* cnt;          // workspace (set by lpse_channel): hand-off counters (zero between launches),
  uint32_t* err;     // the error word, the launch epoch, the release flags
  uint32_t* epoch;
  uint32_t* go;
  uint64_t* trace;   // nullptr, or [layers][PSE_TRACE_EV][256] s_memrealtime stamps (lpse.hip)
};
size_t lpse_lds_bytes();
bool lpse_supported(int device, int B, int layers, int LH, int Hq, int Hkv, int D, int LI, int F, int H, int Cmax);
size_t lpse_ws_bytes();  // zero-filled once by the owner
hipError_t lpse_channel(const LpseArgs& a, void* ws, hipStream_t s);
uint32_t* lpse_err_word(void* ws);
// sample.hip
hipError_t gen_init(const GenBufs& g, const int64_t* ids, const uint8_t* mask, int B, int T, int C, hipStream_t s);
hipError_t sample_step(const GenBufs& g, int B, int n_vq, int P, hipStream_t s);
// local.hip (MossTTSLocal depth stage)
hipError_t moss_rmsnorm(const bf16_t* x, const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s);
hipError_t argmax_rows(const bf16_t* logits, int ld, int V, int64_t* out, int ld_out, int B, hipStream_t s);
// per-row count of masked (pad) columns among the first n of a [B][ld] key mask: the offset
// between a row's cache slots and its RoPE positions (kernels.h QKRopeArgs::rope_off)
hipError_t row_pad_count(const uint8_t* mask, int ld, int n, int B, int* out, int* bad, hipStream_t s);
hipError_t local_init(const int64_t* ids, const uint8_t* mask_in, int B, int T, int C, int64_t* gen_ids, int Ltot,
                      uint8_t* mask, int Cmax, int* finished, uint8_t* seen, int audio_rows, hipStream_t s);
hipError_t local_finalize(GenDev* st, int64_t* next, int* finished, int64_t* gen_ids, uint8_t* mask, uint8_t* seen,
                          int B, int C, int n_ch, int eos, int pad, hipStream_t s);
// channel token: argmax (greedy) or HF penalty/temperature/top-k/top-p + draw (sampled)
// wide_hist: [B][65536] ints of scratch (the key-bin walk of candidate sets past TOPK_CAP)
hipError_t local_pick(GenDev* st, const bf16_t* logits, int ld, int V, int ch, const uint8_t* seen, int64_t* next,
                      int C, int B, int* wide_hist, hipStream_t s);
// init.hip
hipError_t fill_uniform_bf16(bf16_t* dst, size_t n, unsigned long long seed, unsigned long long tensor_id, float scale,
                             float offset, hipStream_t s);

}  // namespace mtts
