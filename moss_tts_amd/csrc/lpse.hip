// MossTTSLocal: one channel of the per-frame depth stage as ONE persistent launch
// (moss_tts_local/modeling_moss_tts.py:390-423, channel i of `CustomMixin._sample`):
//
//   h_0 = speech_embedding_to_local_mlp(x)            x = the backbone state (channel 0) or the
//                                                     previous channel's token embedding  (:395, :421-423)
//   for each depth layer (Qwen3 decoder layer without RoPE, TF/.../modeling_qwen3.py:294-323):
//     input RMSNorm + q|k|v -> q/k RMSNorm, K/V append at the channel position, causal attention
//     over the channel positions -> o_proj + residual -> post-attention RMSNorm + gate|up + SwiGLU
//     -> down + residual
//   z = local_to_speech_embedding_mlps[i](local_transformer.norm(h))            (:402-406)
//
// The per-op form of this (local.cpp local_depth) is 27 dependent launches per channel, 5-12 us
// each, mostly latency: ~1 us of launch gap plus a cold start of every op's weight stream (the
// frame's 1,046 launches leave 958 us of gaps, profiles/r03_v_local_frame_timeline.txt).  Here
// every CU streams its share of ALL the channel's weights (460 MB) through an LDS ring from one
// loader wave, running ahead of the data, and the ops hand off through counters:
//
//  * CU roles.  96 "residual" CUs own one 16-column tile of the depth residual stream each (LH =
//    1536 = 96 tiles): o_proj and down_proj row tile c, the residual in registers, and the adapter
//    into the stack (mi down).  The 160 others run gate|up (pair c - 96 + 160 j in round j < 3);
//    the last 80 of the 560 gate/up tile pairs (round 3) run on residual CUs 0..79, ahead of their
//    down_proj, and the attention's units (one per row and KV head) on residual CUs 0..8B-1
//    (round 5: the 160 gate|up CUs were the frame's critical path -- 4 rounds of 6 slots each
//    after their input arrived, 19 us per layer -- and the attention units sat on them).
//    Every CU runs one q|k|v row tile (4096 rows = 256 tiles).  Per layer a residual CU streams
//    3 + 4 (+ 6) + 18 slots of 16 KiB, a gate|up CU 3 + 18.
//  * While a gate|up CU waits for its post-attention input (the attention and o_proj run
//    elsewhere) its consumer waves copy its first pair's 6 ring slots into registers as they land
//    (pse.hip's SlotCache), so the loader streams 6 slots further ahead through that wait.
//  * Hand-offs.  An op's producers store their outputs write-through (sc1), drain them
//    (s_waitcnt vmcnt(0)), then bump the op's counter (relaxed, agent scope); a consumer polls the
//    counter with sc1 loads and reads the data with sc1 loads (cdna_hip_programming.md Guideline
//    16, R1 -- the split-K GEMV's hand-off).  The last workgroup out zeroes the counters for the
//    next launch.  down_proj takes its input in four rounds as gate|up produces it (round j =
//    columns 2560 j .. +2560 = its k-tiles 80 j .. +80), straight into registers as MFMA B
//    fragments, so the 8 x 8,960 SwiGLU output is never gathered whole.
//  * Arithmetic as the per-op kernels: Qwen3RMSNorm bf16(w * bf16(x * r)) with r from the
//    producers' per-16-column sums of squares, v_mfma_f32_16x16x32_bf16 over packed weight tiles
//    (B operand = the rows), residual bf16(res + bf16(y)), SwiGLU bf16(bf16(silu(bf16 g)) * bf16 u),
//    attention scores in fp32 with the probabilities rounded to bf16 before P.V (the reference's
//    bf16 SDPA).  Accumulation orders differ from the per-op launches (parity: within the bf16
//    band of the oracle, tests/test_local_b8_gpu.py).
//  * Every wait is bounded: a timed-out wait sets the error word and drains the launch; the
//    engine then runs the per-op launches (local.cpp).
#include "kernels.h"

namespace mtts {

namespace {

constexpr int CW = 4;                   // consumer waves
constexpr int THREADS = (1 + CW) * 64;  // + the loader wave
#ifndef LPSE_INF
#define LPSE_INF 3  // ring slots in flight per loader (48 KiB: the batch-1 launch's measured optimum)
#endif
constexpr int NS = 7;                   // ring slots of 16 KiB
constexpr int INF = LPSE_INF;
static_assert(INF >= 1 && INF <= 3 && INF < NS, "vmcnt counts at most 63 loads");
constexpr int SLOT = 16 * 1024;
constexpr int NB = LPSE_MAXB;           // rows
constexpr int LH = 1536, H = 2048, F = 2048, LI = 8960, HQ = 16, HKV = 8, D = 128, QKVR = (HQ + 2 * HKV) * D;
constexpr int CMAX = 64;                // channel positions of the depth KV cache
constexpr int KT_LH = LH / 32, KT_H = H / 32, KT_F = F / 32, KT_LI = LI / 32, KT_AT = HQ * D / 32;
constexpr int NR = LH / 16;             // residual CUs (row tiles of the residual stream)
constexpr int P = 256;
constexpr int NM = P - NR;              // gate|up CUs
constexpr int GU_PAIRS = LI / 16, F_PAIRS = F / 16;
constexpr int ROUND_KT = NM * 16 / 32;  // down k-tiles per act round (80)
constexpr int R3_PAIRS = LI / 16 - 3 * NM;   // round 3's pairs (80), on residual CUs 0 .. 79
constexpr int R3_KT0 = 3 * ROUND_KT;         // their down k-tiles 240 .. 279
constexpr int DOWN_SLOTS_R3 = (KT_LI - R3_KT0 + 15) / 16;  // 3 (the last one half valid)
constexpr int TILE_E = 512;             // bf16 per 1 KiB weight tile
static_assert(QKVR / 16 == P && H / 16 == 128 && F_PAIRS == 128, "the 1.7B depth shape on 256 CUs");
static_assert(KT_LI == 3 * ROUND_KT + 40 && GU_PAIRS == 3 * NM + 80, "down's act rounds");

// hand-off counters
constexpr int C_MIGU = 0, C_MIDOWN = 1, C_MOGU_BASE = 2;
__device__ __forceinline__ int c_layer(int l, int k) { return 2 + 8 * l + k; }  // k: 0 q|k|v 1 att 2 o 3-6 gu rounds 7 down
constexpr int C_EXIT = 63;
constexpr int N_CNT = 64;

typedef __attribute__((address_space(1))) uint32_t g32;
typedef __attribute__((address_space(1))) int gi32;
typedef __attribute__((address_space(3))) void lvoid;

__device__ __forceinline__ void st32(void* p, uint32_t v) {
  __hip_atomic_store((g32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const void* p) {
  return __hip_atomic_load((g32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

struct Ctl {
  int full;       // ring slots whose DMA has landed
  int freed[CW];  // per consumer wave: ring slots it has read
  int bar;        // consumer barrier
  int abort;
};

constexpr uint32_t SPIN_LDS = 1u << 22;
constexpr uint32_t SPIN_MEM = 1u << 18;

// LDS layout (bytes)
constexpr int L_CTL = 0;
constexpr int L_PTR = 256;  // [layer][8] weight pointers (a runtime-indexed kernel-argument array would go to scratch)
constexpr int L_RING = 1024;
static_assert(L_PTR + LPSE_MAXL * 8 * 8 <= L_RING, "pointer table");
constexpr int L_X = L_RING + NS * SLOT;        // op input [k tile][row][32] bf16, K <= 2048: 32 KiB
constexpr int X_BYTES = KT_H * NB * 64;
constexpr int L_RED = L_X + X_BYTES;           // [CW][2][256] fp32
constexpr int L_MISC = L_RED + CW * 2 * 256 * 4;  // r_s[NB], sq[NB][16]
constexpr int L_END = L_MISC + (NB + NB * 16) * 4;
static_assert(L_END <= 160 * 1024, "LDS");
// attention scratch over the op-input region (the q|k|v input is consumed): the cached keys
// K [AKEYS][D] and values V^T [D][AKEYS] bf16 (prefetched while the q|k|v hand-off is awaited),
// qn [2][D], kn [D], vn [D], scores [2][CMAX], p [2][CMAX], l [2] (fp32)
constexpr int AKEYS = 32;  // channel positions before the newest (<= 33 channels per frame)
static_assert(AKEYS + 1 == LPSE_MAX_CHANNELS, "local.cpp gates the launch on 1 + n_vq <= LPSE_MAX_CHANNELS");
constexpr int L_AKC = L_X, L_AVC = L_AKC + AKEYS * D * 2;
constexpr int L_AQ = L_AVC + D * AKEYS * 2, L_AK = L_AQ + 2 * D * 4, L_AV = L_AK + D * 4, L_AS = L_AV + D * 4,
              L_AP = L_AS + 2 * CMAX * 4, L_AL = L_AP + 2 * CMAX * 4;
static_assert(L_AL + 16 <= L_X + X_BYTES, "attention scratch");

extern __shared__ __attribute__((aligned(16))) unsigned char lp_lds[];
#define LP_CTL (reinterpret_cast<Ctl*>(lp_lds + L_CTL))
// layer l's pointer k (LpseLayer order: qkv, o, gu, down, in_norm, post_norm, q_norm, k_norm)
enum { P_QKV = 0, P_O, P_GU, P_DOWN, P_INN, P_POSTN, P_QN, P_KN };
__device__ __forceinline__ const bf16_t* lptr(int l, int k) {
  return reinterpret_cast<const bf16_t* const*>(lp_lds + L_PTR)[l * 8 + k];
}

// trace (MTTS_PSE_TRACE=1 engines, scripts/lpse_trace.py): consumer wave 0 per layer -- 0 q|k|v input
// ready, 1 normed, 2 q|k|v done; attention units 3 start, 4 done; residual CUs 5 o input in, 6 o done,
// 11 round-3 pair done, 12-15 down round j input in, 16 down done; gate|up CUs 7 input normed, 8-10
// round j done
#define LP_STAMP(l, ev)                                                                          \
  do {                                                                                           \
    if (a.trace && x.w == 0 && x.lane == 0)                                                      \
      a.trace[((size_t)(l) * PSE_TRACE_EV + (ev)) * 256 + c] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)

struct Cx {
  uint32_t* err;
  float eps;
  int c, lane, w, tid, B;
  int bar_gen;
  int* cnt;        // hand-off counters
  uint32_t* go;    // LPSE_GO: per (counter, CU) release flags, one 128-byte line each
  uint32_t epoch;  // this launch's flag value
};

__device__ __forceinline__ bool failed() {
  return __hip_atomic_load(&LP_CTL->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
}
__device__ __forceinline__ void give_up(uint32_t* err, uint32_t code) {
  st32(err, code);
  __hip_atomic_store(&LP_CTL->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// consumer-only barrier (the loader never joins): a monotonic LDS counter
__device__ __forceinline__ void cbar(Cx& x) {
  x.bar_gen += CW;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (x.lane == 0) __hip_atomic_fetch_add(&LP_CTL->bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  for (uint32_t spins = 0;
       __hip_atomic_load(&LP_CTL->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < x.bar_gen; ++spins) {
    if (spins > SPIN_LDS || ((spins & 255) == 255 && failed())) {  // (after an abort the waves' counts may differ)
      give_up(x.err, 4);
      break;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Hand-off k is complete once `target` producers arrived.  LPSE_GO (default): the producer whose
// arrival completes it writes this launch's epoch into every consumer CU's own flag line, and a
// consumer polls only its line -- polled directly, the one counter line took the polls of all 1,024
// consumer waves (18 ms per frame against 8.4 for the per-op launches, profiles/r04_a_*); 0: poll
// the counter itself (A/B)
#ifndef LPSE_GO
#define LPSE_GO 1
#endif
constexpr int GO_STRIDE = 32;  // words: one 128-byte line per flag
__device__ __forceinline__ uint32_t* go_flag(const Cx& x, int k, int cu) { return x.go + ((size_t)k * P + cu) * GO_STRIDE; }

// wait until hand-off k is complete (sc1 polls); false on timeout / abort
struct NoPoll {
  __device__ void operator()() const {}
};
template <typename Poll = NoPoll>
__device__ __forceinline__ bool bwait(Cx& x, int k, int target, const Poll& each_poll = Poll()) {
  for (uint32_t spins = 0; LPSE_GO ? ld32(go_flag(x, k, x.c)) != x.epoch : (int)ld32(x.cnt + k) < target; ++spins) {
    if (spins > SPIN_MEM || ((spins & 255) == 255 && (failed() || ld32(x.err)))) {
      give_up(x.err, 2);
      return false;
    }
    each_poll();
    __builtin_amdgcn_s_sleep(1);
  }
  // every later read of the producers' data is an sc1 load: a wavefront-scope fence keeps the
  // compiler from hoisting them above the poll
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return !failed();
}

// LPSE_HTREE: a hand-off's arrivals (the producers: CUs lo .. hi - 1) counted in two levels -- a
// counter per group of 32 CUs (its own 128-byte line), whose completing arrival bumps the hand-off's
// counter -- instead of up to 256 agent-scope atomics queueing on one line (pse4.hip PSE4_HTREE)
#ifndef LPSE_HTREE
#define LPSE_HTREE 1
#endif
constexpr int AGRP = 32;                 // CUs per arrival group
constexpr int NGRP = P / AGRP;
constexpr int GC_STRIDE = 32;            // ints per group counter line
// workspace (bytes): counters [N_CNT] at 0, the error word and epoch behind them, the release flags
// from WS_GO, the group counters [N_CNT][NGRP] lines behind the flags
constexpr size_t WS_GO = 512;
constexpr size_t WS_GC = WS_GO + (size_t)N_CNT * P * GO_STRIDE * 4;
__device__ __forceinline__ int* grp_cnt(const Cx& x, int k, int g) {
  return x.cnt + WS_GC / 4 + ((size_t)k * NGRP + g) * GC_STRIDE;
}

// this workgroup's outputs of hand-off k are stored (write-through): drain, barrier, one arrival
// (producers: CUs lo .. hi - 1); the arrival that completes it releases every consumer CU's flag
__device__ __forceinline__ void arrive(Cx& x, int k, int lo, int hi) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  cbar(x);
  if (x.w == 0) {
    int t = 0, target = hi - lo;
    if (LPSE_HTREE && LPSE_GO) {
      const int g = x.c / AGRP;
      const int in_g = min(hi, (g + 1) * AGRP) - max(lo, g * AGRP);
      target = (hi - 1) / AGRP - lo / AGRP + 1;  // groups with producers
      if (x.lane == 0) {
        t = __hip_atomic_fetch_add((gi32*)grp_cnt(x, k, g), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        t = t == in_g - 1 ? __hip_atomic_fetch_add((gi32*)(x.cnt + k), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
      }
    } else if (x.lane == 0) {
      t = __hip_atomic_fetch_add((gi32*)(x.cnt + k), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    t = __shfl(t, 0, 64);
    if (LPSE_GO && t == target - 1)
#pragma unroll
      for (int i = 0; i < P / 64; ++i) st32(go_flag(x, k, x.lane + 64 * i), x.epoch);
  }
}

template <bool V>
struct RoleC {
  static constexpr bool value = V;
};

// ---- op input staging: rows [B][K] bf16 -> X [k tile][row][32] ----
// chunk i (8 columns) of the B x K input: row i / (K/8), columns 8 (i % (K/8)) ..
__device__ __forceinline__ int xidx(int b, int c8) { return ((c8 >> 2) * NB + b) * 4 + (c8 & 3); }

// plain rows (sc1 loads: written inside this launch, or before it); row b at src(b).  K = 2048:
// chunk j of every thread is row j (one uniform buffer resource per row)
template <int K, class Src>
__device__ __forceinline__ void stage_plain(Cx& x, const Src& src) {
  constexpr int C8 = K / 8;
  static_assert(C8 == CW * 64, "one chunk per thread per row");
  u32x4 v[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const bf16_t* row = src(b < x.B ? b : 0);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(row), 0, K * 2, 0x00020000);
    v[b] = __builtin_amdgcn_raw_buffer_load_b128(rs, b < x.B ? (uint32_t)x.tid * 16u : 0x7ffffff0u, 0, 16 /* sc1 */);
  }
  u32x4* X = reinterpret_cast<u32x4*>(lp_lds + L_X);
#pragma unroll
  for (int b = 0; b < NB; ++b) X[xidx(b, x.tid)] = v[b];
  cbar(x);
}

// Qwen3RMSNorm of the residual stream h [B][LH] (TF/.../modeling_qwen3.py:59-64):
// X = bf16(nw * bf16(h * r_b)), r_b = 1 / sqrt(sum_t ss[b][t] / LH + eps) -- the 96 per-16-column
// sums of squares summed as the GEMV prologue sums them (4 per lane, pairwise, then the wave)
__device__ __forceinline__ void stage_norm(Cx& x, const bf16_t* h, const float* ss, const bf16_t* nw) {
  constexpr int C8 = LH / 8, N = NB * C8 / (CW * 64);
  static_assert(NB * C8 % (CW * 64) == 0 && NR <= 4 * 64, "whole chunks per thread");
  constexpr uint32_t OOB = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(h), 0, NB * LH * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ss), 0, NB * NR * 4, 0x00020000);
  u32x4 hv[N], wv[N], sv[2];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int i = x.tid + j * CW * 64, b = i / C8, c8 = i - b * C8;
    hv[j] = __builtin_amdgcn_raw_buffer_load_b128(hrs, b < x.B ? (uint32_t)(b * LH + c8 * 8) * 2u : OOB, 0, 16);
    wv[j] = reinterpret_cast<const u32x4*>(nw)[c8];
  }
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int b = x.w + m * CW;
    sv[m] = __builtin_amdgcn_raw_buffer_load_b128(srs, (b < x.B && x.lane * 4 < NR) ? (uint32_t)(b * NR + x.lane * 4) * 4u : OOB,
                                                  0, 16);
  }
  float* r_s = reinterpret_cast<float*>(lp_lds + L_MISC);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const float s = wave_sum((__uint_as_float(sv[m][0]) + __uint_as_float(sv[m][1])) +
                             (__uint_as_float(sv[m][2]) + __uint_as_float(sv[m][3])));
    if (x.lane == 0) r_s[x.w + m * CW] = 1.0f / sqrtf(s / (float)LH + x.eps);
  }
  cbar(x);
  u32x4* X = reinterpret_cast<u32x4*>(lp_lds + L_X);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int i = x.tid + j * CW * 64, b = i / C8, c8 = i - b * C8;
    const float r = r_s[b];
    u32x4 o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x0 = __uint_as_float(hv[j][q] << 16), x1 = __uint_as_float(hv[j][q] & 0xffff0000u);
      const float w0 = __uint_as_float(wv[j][q] << 16), w1 = __uint_as_float(wv[j][q] & 0xffff0000u);
      o[q] = pack2(w0 * rbf(x0 * r), w1 * rbf(x1 * r));
    }
    X[xidx(b, c8)] = o;
  }
  cbar(x);
}

// ---- ring slots ----
// this consumer wave's 4 tiles of ring slot seq (then the slot is released to the loader)
__device__ __forceinline__ bool take4(Cx& x, int seq, u32x4 (&t)[4]) {
  for (uint32_t spins = 0;
       __hip_atomic_load(&LP_CTL->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= seq; ++spins) {
    if (spins > SPIN_LDS || failed()) {
      give_up(x.err, 3);
      return false;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const u32x4* sl = reinterpret_cast<const u32x4*>(lp_lds + L_RING + (seq % NS) * SLOT);
#pragma unroll
  for (int i = 0; i < 4; ++i) t[i] = sl[(x.w * 4 + i) * 64 + x.lane];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (x.lane == 0) __hip_atomic_store(&LP_CTL->freed[x.w], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  return true;
}

// B fragment of k tile kt from X: lane -> row (lane & 15) (zero past B), 8 columns at 8 (lane >> 4)
__device__ __forceinline__ u32x4 xfrag(const Cx& x, int kt) {
  const u32x4* X = reinterpret_cast<const u32x4*>(lp_lds + L_X);
  const int b = x.lane & 15;
  const u32x4 v = X[(kt * NB + (b & (NB - 1))) * 4 + (x.lane >> 4)];
  return b < x.B ? v : (u32x4){0u, 0u, 0u, 0u};
}

__device__ __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// NRT row tiles (a gate|up pair: 2) of KT k-tiles each, SPR ring slots per row tile, x from X
template <int NRT, int SPR, int KT>
__device__ __forceinline__ bool gemv_unit(Cx& x, int& seq, f32x4 (&acc)[NRT]) {
#pragma unroll
  for (int r = 0; r < NRT; ++r) {
    acc[r] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < SPR; ++s) {
      u32x4 t[4];
      if (!take4(x, seq++, t)) return false;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kt = s * 16 + x.w * 4 + i;
        if (kt < KT) acc[r] = mfma(t[i], xfrag(x, kt), acc[r]);
      }
    }
  }
  return true;
}

// ring slots drained into registers while the consumer waits for an input (pse.hip SlotCache):
// slots seq0 .. seq0 + RC - 1 in order, each released to the loader once copied
__device__ __forceinline__ bool slot_ready(int seq) {
  return __hip_atomic_load(&LP_CTL->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > seq;
}
#ifndef LPSE_RC
#define LPSE_RC 4  // a gate|up CU's ring slots drained into registers during the post-attention wait
#endif
template <int RC>
struct SlotCache {
  u32x4 rc[RC > 0 ? RC : 1][4];
  int nd = 0;
  __device__ __forceinline__ void drain(const Cx& x, int seq0) {
#pragma unroll
    for (int k = 0; k < RC; ++k)
      if (k == nd && slot_ready(seq0 + k)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const u32x4* sl = reinterpret_cast<const u32x4*>(lp_lds + L_RING + ((seq0 + k) % NS) * SLOT);
#pragma unroll
        for (int i = 0; i < 4; ++i) rc[k][i] = sl[(x.w * 4 + i) * 64 + x.lane];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (x.lane == 0)
          __hip_atomic_store(&LP_CTL->freed[x.w], seq0 + k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ++nd;
      }
  }
};
// a gate|up pair (2 row tiles x 3 slots) whose first RC slots may sit in a SlotCache (RC 6 spilled 19 VGPRs)
template <int RC>
__device__ __forceinline__ bool gu_pair_cached(Cx& x, int& seq, SlotCache<RC>& sc, f32x4 (&acc)[2]) {
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    acc[r] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 3; ++s) {
      const int k = r * 3 + s;
      u32x4 t[4];
      if (k < RC && k < sc.nd) {
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i] = sc.rc[k < RC ? k : 0][i];
        ++seq;
      } else if (!take4(x, seq++, t)) {
        return false;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[r] = mfma(t[i], xfrag(x, s * 16 + x.w * 4 + i), acc[r]);
    }
  }
  return true;
}

// fixed-order reduction of the CW waves' tiles: element t (< 256) of row tile r ->
// weight row n = 4 ((t >> 2) >> 4) + (t & 3), batch row b = (t >> 2) & 15
template <int NRT>
__device__ __forceinline__ void red_put(Cx& x, const f32x4 (&acc)[NRT]) {
  float* red = reinterpret_cast<float*>(lp_lds + L_RED);
#pragma unroll
  for (int r = 0; r < NRT; ++r)
#pragma unroll
    for (int i = 0; i < 4; ++i) red[(x.w * 2 + r) * 256 + x.lane * 4 + i] = acc[r][i];
  cbar(x);
}
__device__ __forceinline__ float red_get(const Cx& x, int r) {
  const float* red = reinterpret_cast<const float*>(lp_lds + L_RED);
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < CW; ++w) s += red[(w * 2 + r) * 256 + x.tid];
  return s;
}
__device__ __forceinline__ int el_n(int t) { return (((t >> 2) >> 4) << 2) + (t & 3); }
__device__ __forceinline__ int el_b(int t) { return (t >> 2) & 15; }

// write bf16 value v of element (b, col) -- pairs of neighbouring columns as one write-through
// dword (element t ^ 1 holds column col ^ 1 of the same row)
__device__ __forceinline__ void put_pair(const Cx& x, bf16_t* y, int ld, int col, float v) {
  const uint32_t me = f2bf(v);
  const uint32_t other = (uint32_t)__shfl_xor((int)me, 1, 64);
  const int b = el_b(x.tid);
  if (b < x.B && !(col & 1)) st32(y + (size_t)b * ld + col, me | (other << 16));
}

// residual epilogue: out = bf16(res + bf16(v)) (TF/.../modeling_qwen3.py:311, 322), res kept in
// the thread's register; h tile and its per-row sum of squares (16 columns summed in order, as
// the GEMV epilogue) go out write-through
__device__ __forceinline__ void resadd_out(Cx& x, float v, float& hres, bf16_t* h, float* ss, int tile) {
  const int n = el_n(x.tid), b = el_b(x.tid);
  const float out = bf2f(f2bf(hres + rbf(v)));
  hres = out;
  put_pair(x, h, LH, tile * 16 + n, out);
  float* sq = reinterpret_cast<float*>(lp_lds + L_MISC) + NB;
  if (b < NB) sq[b * 16 + n] = out * out;
  cbar(x);
  if (x.tid < x.B) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += sq[x.tid * 16 + i];
    st32(ss + (size_t)x.tid * NR + tile, __float_as_uint(s));
  }
}

__device__ __forceinline__ float swiglu(float g0, float u0) {
  const float g = rbf(g0), u = rbf(u0);
  return rbf(g / (1.0f + expf(-g))) * u;  // (TF/.../modeling_qwen3.py:81-83)
}

// ---- attention unit (row b, KV head g) of layer l at channel position pos ----
// q / k RMSNorm (no RoPE: MossTTSLocal's depth transformer, moss_tts_local/modeling_moss_tts.py:
// 126-176), K / V appended at pos (TF/cache_utils.py:127-145), softmax(q k^T / sqrt(D)) v over
// positions 0..pos (causal; every channel position is valid), probabilities rounded to bf16
// before P.V (the reference's bf16 SDPA).
// Round 5: the cached keys / values (positions < pos, written by earlier channels' launches) are
// loaded into registers BEFORE the q|k|v hand-off is awaited (att_prefetch) and land in LDS behind
// it; scores take 4 lanes per key (32 dims each) instead of one lane per key over all 128 dims.
struct KVPre {
  u32x4 k[2], v[2];
};
__device__ __forceinline__ bf16_t* att_kc(const LpseArgs& a, int l, int b, int g) {
  return a.kc + (size_t)l * a.layer_kv + (((size_t)b * HKV + g) * CMAX) * D;  // [CMAX][D]
}
__device__ __forceinline__ bf16_t* att_vc(const LpseArgs& a, int l, int b, int g) {
  return a.vc + (size_t)l * a.layer_kv + (((size_t)b * HKV + g) * D) * CMAX;  // [D][CMAX]
}
__device__ __forceinline__ KVPre att_prefetch(const Cx& x, const LpseArgs& a, int l, int b, int g) {
  const int pos = a.pos;
  constexpr uint32_t OOB = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(att_kc(a, l, b, g), 0, CMAX * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(att_vc(a, l, b, g), 0, CMAX * D * 2, 0x00020000);
  KVPre r;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int i = x.tid + m * CW * 64;  // 16-byte chunk i of K [AKEYS][D] / of V^T's first AKEYS columns
    const int key = i >> 4;             // K: 16 chunks per key
    r.k[m] = __builtin_amdgcn_raw_buffer_load_b128(krs, key < pos ? (uint32_t)i * 16u : OOB, 0, 0);
    const int d = i >> 2, q = i & 3;    // V^T: 4 chunks (32 keys) per dim
    r.v[m] = __builtin_amdgcn_raw_buffer_load_b128(vrs, q * 8 < pos ? (uint32_t)(d * CMAX + q * 8) * 2u : OOB, 0, 0);
  }
  return r;
}
__device__ __forceinline__ void attention(Cx& x, const LpseArgs& a, int l, int b, int g, const KVPre& pre) {
  const int pos = a.pos;
  bf16_t* Ks = reinterpret_cast<bf16_t*>(lp_lds + L_AKC);  // [AKEYS][D]
  bf16_t* Vs = reinterpret_cast<bf16_t*>(lp_lds + L_AVC);  // [D][AKEYS]
  float* qn = reinterpret_cast<float*>(lp_lds + L_AQ);
  float* kn = reinterpret_cast<float*>(lp_lds + L_AK);
  float* vn = reinterpret_cast<float*>(lp_lds + L_AV);
  float* sc = reinterpret_cast<float*>(lp_lds + L_AS);
  float* ps = reinterpret_cast<float*>(lp_lds + L_AP);
  float* ls = reinterpret_cast<float*>(lp_lds + L_AL);
  bf16_t* kc = att_kc(a, l, b, g);
  bf16_t* vc = att_vc(a, l, b, g);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int i = x.tid + m * CW * 64;
    reinterpret_cast<u32x4*>(Ks)[i] = pre.k[m];
    reinterpret_cast<u32x4*>(Vs)[(i >> 2) * (AKEYS / 8) + (i & 3)] = pre.v[m];
  }
  {
    // wave w: vector w (0, 1: q heads 2g, 2g + 1; 2: k; 3: v), two dims per lane
    const int hd = x.w < 2 ? g * 2 + x.w : (x.w == 2 ? HQ + g : HQ + HKV + g);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(a.qkvb + (size_t)b * QKVR + hd * D, 0, D * 2, 0x00020000);
    const uint32_t xv = __builtin_amdgcn_raw_buffer_load_b32(rs, (uint32_t)x.lane * 4u, 0, 16);
    const float x0 = __uint_as_float(xv << 16), x1 = __uint_as_float(xv & 0xffff0000u);
    if (x.w == 3) {
      vn[2 * x.lane] = x0;
      vn[2 * x.lane + 1] = x1;
      vc[(size_t)(2 * x.lane) * CMAX + pos] = f2bf(x0);
      vc[(size_t)(2 * x.lane + 1) * CMAX + pos] = f2bf(x1);
    } else {
      const uint32_t wv = reinterpret_cast<const uint32_t*>(lptr(l, x.w < 2 ? P_QN : P_KN))[x.lane];
      const float ss = wave_sum(x0 * x0 + x1 * x1);
      const float r = 1.0f / sqrtf(ss / (float)D + a.eps);
      const float n0 = rbf(__uint_as_float(wv << 16) * rbf(x0 * r));
      const float n1 = rbf(__uint_as_float(wv & 0xffff0000u) * rbf(x1 * r));
      float* dst = x.w < 2 ? qn + x.w * D : kn;
      dst[2 * x.lane] = n0;
      dst[2 * x.lane + 1] = n1;
      if (x.w == 2) *reinterpret_cast<uint32_t*>(kc + (size_t)pos * D + 2 * x.lane) = pack2(n0, n1);
    }
  }
  cbar(x);
  {
    // scores: thread -> head h = tid / 128, cached key j = (tid / 4) % 32, dims 32 (tid % 4) ..;
    // the new key (pos) by the first wave of each head
    const int h = x.tid >> 7, j = (x.tid >> 2) & (AKEYS - 1), qd = x.tid & 3;
    const float* q = qn + h * D + qd * 32;
    const u32x4* kr = reinterpret_cast<const u32x4*>(Ks + j * D + qd * 32);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const u32x4 kv = kr[c];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s += q[c * 8 + 2 * e] * __uint_as_float(kv[e] << 16);
        s += q[c * 8 + 2 * e + 1] * __uint_as_float(kv[e] & 0xffff0000u);
      }
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (qd == 0 && j < pos) sc[h * CMAX + j] = s * a.scale;
    if ((x.w & 1) == 0) {  // waves 0 / 2: the new key of head h
      const float sn = wave_sum(qn[h * D + 2 * x.lane] * kn[2 * x.lane] + qn[h * D + 2 * x.lane + 1] * kn[2 * x.lane + 1]);
      if (x.lane == 0) sc[h * CMAX + pos] = sn * a.scale;
    }
  }
  cbar(x);
  if (x.w < 2) {  // softmax of head w over keys 0..pos (lane = key)
    const int j = x.lane;
    const float sv = j <= pos ? sc[x.w * CMAX + j] : -INFINITY;
    const float m = wave_max(sv);
    const float p = j <= pos ? expf(sv - m) : 0.f;
    const float L = wave_sum(p);
    ps[x.w * CMAX + j] = rbf(p);
    if (x.lane == 0) ls[x.w] = L;
  }
  cbar(x);
  {
    // output (head h, dim d) per thread: sum over keys of bf16(p) * v, in key order
    const int h = x.tid >> 7, d = x.tid & (D - 1);
    const u32x4* vr = reinterpret_cast<const u32x4*>(Vs + d * AKEYS);
    float o = 0.f;
    for (int j0 = 0; j0 < pos; j0 += 8) {
      const u32x4 v8 = vr[j0 >> 3];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = j0 + 2 * e;
        if (j < pos) o += ps[h * CMAX + j] * __uint_as_float(v8[e] << 16);
        if (j + 1 < pos) o += ps[h * CMAX + j + 1] * __uint_as_float(v8[e] & 0xffff0000u);
      }
    }
    o += ps[h * CMAX + pos] * rbf(vn[d]);
    const float L = ls[h];
    const float out = L > 0.f ? o / L : 0.f;
    const uint32_t me = f2bf(out);
    const uint32_t other = (uint32_t)__shfl_xor((int)me, 1, 64);
    if (!(d & 1)) st32(a.attnb + (size_t)b * (HQ * D) + (2 * g + h) * D + d, me | (other << 16));
  }
}

}  // namespace

__global__ __launch_bounds__(THREADS) void lpse_kernel(LpseArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = blockIdx.x;
  if (threadIdx.x < 64) reinterpret_cast<int*>(lp_lds + L_CTL)[threadIdx.x] = 0;
  if (threadIdx.x == 64) {  // (constant indices only: no private copy of the argument array)
    const bf16_t** t = reinterpret_cast<const bf16_t**>(lp_lds + L_PTR);
#pragma unroll
    for (int l = 0; l < LPSE_MAXL; ++l) {
      const LpseLayer& q = a.L[l];
      t[l * 8 + P_QKV] = q.qkv; t[l * 8 + P_O] = q.o; t[l * 8 + P_GU] = q.gu; t[l * 8 + P_DOWN] = q.down;
      t[l * 8 + P_INN] = q.in_norm; t[l * 8 + P_POSTN] = q.post_norm; t[l * 8 + P_QN] = q.q_norm; t[l * 8 + P_KN] = q.k_norm;
    }
  }
  __syncthreads();
  const int L = a.layers;
  const bool resid = c < NR;
  const uint32_t epoch = ld32(a.epoch) + 1u;  // (the previous launch's last workgroup advanced it)

  if (wave == 0) {
    // =================== loader ===================
    // This CU's slots in consumption order; slot k of a segment = 16 weight tiles from its base.
    // Each slot goes global -> ring slot by LDS-DMA (16 wave-instructions of 1 KiB); the INF most
    // recent slots stay in flight, older ones are published in FULL.  `valid`: bytes of the matrix
    // from the segment base (a slot past it reads zeros: down_proj's half last slot of row tile 95)
    int issued = 0, pub = 0;
    bool dead = false;
    const uint32_t voff = (uint32_t)lane * 16u;
    auto publish = [&](int n) {
      if (n > pub) {
        pub = n;
        __hip_atomic_store(&LP_CTL->full, n, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    };
    auto seg = [&](const bf16_t* base, long long valid, int nslots) {
      for (int k = 0; k < nslots && !dead; ++k) {
        const int s = issued;
        if (s >= NS) {
          bool waited = false;
          for (uint32_t spins = 0;; ++spins) {  // ring slot s % NS is free once every consumer read slot s - NS
            int mn = 1 << 30;
#pragma unroll
            for (int w = 0; w < CW; ++w)
              mn = min(mn, __hip_atomic_load(&LP_CTL->freed[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (mn >= s - NS + 1) break;
            if (!waited) {  // nothing to issue: let every landed slot out first
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              publish(issued);
              waited = true;
            }
            if (spins > SPIN_LDS || __hip_atomic_load(&LP_CTL->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              dead = true;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
          if (dead) break;
        }
        const long long left = valid - (long long)k * SLOT;
        const int nrec = left <= 0 ? 0 : (left >= SLOT ? SLOT : (int)left);
        const uint64_t p = (uint64_t)(uintptr_t)(base + (size_t)k * 16 * TILE_E);
        const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, __builtin_amdgcn_readfirstlane(nrec), 0x00020000);
        unsigned char* dst = lp_lds + L_RING + (s % NS) * SLOT;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lvoid*)(dst + i * 1024), 16, voff + (uint32_t)i * 1024u, 0, 0, 0);
        issued = s + 1;
        // all but the INF - 1 newest slots have landed
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(16 * (INF - 1)) : "memory");
        publish(issued - (INF - 1));
      }
    };
    // the adapter into the stack: gate|up pairs on CUs NR .. NR + 127, down on the residual CUs
    if (!resid && c < NR + F_PAIRS) seg(a.mi_gu + (size_t)(c - NR) * 2 * KT_H * TILE_E, 1ll << 40, 2 * KT_H / 16);
    if (resid) seg(a.mi_down + (size_t)c * KT_F * TILE_E, 1ll << 40, KT_F / 16);
    for (int l = 0; l < L; ++l) {
      seg(lptr(l, P_QKV) + (size_t)c * KT_LH * TILE_E, 1ll << 40, KT_LH / 16);
      if (resid) {
        seg(lptr(l, P_O) + (size_t)c * KT_AT * TILE_E, 1ll << 40, KT_AT / 16);
        // round 3's gate|up pair, then down_proj: round 3's k-tiles (240 .. 279: 2.5 slots, the
        // last one half valid) first -- this CU group produces them -- then rounds 0-2 (0 .. 239)
        if (c < R3_PAIRS) seg(lptr(l, P_GU) + (size_t)(3 * NM + c) * 2 * KT_LH * TILE_E, 1ll << 40, 2 * KT_LH / 16);
        const bf16_t* dn = lptr(l, P_DOWN) + (size_t)c * KT_LI * TILE_E;
        seg(dn + (size_t)R3_KT0 * TILE_E, (long long)(KT_LI - R3_KT0) * 1024, DOWN_SLOTS_R3);
        seg(dn, (long long)R3_KT0 * 1024, R3_KT0 / 16);
      } else {
        for (int j = 0; j < 3; ++j) seg(lptr(l, P_GU) + (size_t)(c - NR + NM * j) * 2 * KT_LH * TILE_E, 1ll << 40, 2 * KT_LH / 16);
      }
    }
    // the adapter out: gate|up pairs on CUs 128 .., down row tiles on CUs .. 127
    if (c >= 128) seg(a.mo_gu + (size_t)(c - 128) * 2 * KT_LH * TILE_E, 1ll << 40, 2 * KT_LH / 16);
    else seg(a.mo_down + (size_t)c * KT_F * TILE_E, 1ll << 40, KT_F / 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (dead) st32(a.err, 1u);
    publish(issued);
  } else {
    // =================== consumers ===================
    Cx x{a.err, a.eps, c, lane, wave - 1, (int)threadIdx.x - 64, a.B, 0, a.cnt, a.go, epoch};
    int seq = 0;
    float hres = 0.f;  // residual CUs: element (el_b, el_n) of this CU's residual tile
    bool ok = true;
    // ---- speech_embedding_to_local_mlp (:395, :421-423): x -> gate|up (SwiGLU) -> down ----
    if (!resid && c < NR + F_PAIRS) {
      const int p = c - NR;
      stage_plain<H>(x, [&](int b) { return a.tok ? a.in + (size_t)a.tok[(size_t)b * a.ld_tok] * H : a.in + (size_t)b * H; });
      f32x4 acc[2];
      ok = gemv_unit<2, KT_H / 16, KT_H>(x, seq, acc);
      red_put<2>(x, acc);
      put_pair(x, a.actF, F, p * 16 + el_n(x.tid), swiglu(red_get(x, 0), red_get(x, 1)));
      arrive(x, C_MIGU, NR, NR + F_PAIRS);
    }
    if (resid && ok) {
      ok = bwait(x, C_MIGU, F_PAIRS);
      stage_plain<F>(x, [&](int b) { return a.actF + (size_t)b * F; });
      f32x4 acc[1];
      ok = ok && gemv_unit<1, KT_F / 16, KT_F>(x, seq, acc);
      red_put<1>(x, acc);
      resadd_out(x, red_get(x, 0), hres, a.h, a.ss, c);  // res = 0: bf16(0 + bf16(y)) = bf16(y)
      arrive(x, C_MIDOWN, 0, NR);
    }
    // the layer loop instantiated per role (residual / gate|up CU), so that one role's registers
    // (the gate|up CUs' drained slots, the residual CUs' down fragments) do not shape the other's
    // allocation; attention unit (row b, KV head g) on residual CU 8 b + g
    const bool att = resid && c < HKV * a.B;
    auto layers = [&](auto role) __attribute__((always_inline)) {
    constexpr bool R = decltype(role)::value;
    for (int l = 0; l < L && ok; ++l) {
      // ---- input RMSNorm + q|k|v: row tile c ----
      ok = bwait(x, l == 0 ? C_MIDOWN : c_layer(l - 1, 7), NR);
      LP_STAMP(l, 0);
      stage_norm(x, a.h, a.ss, lptr(l, P_INN));
      LP_STAMP(l, 1);
      {
        f32x4 acc[1];
        ok = ok && gemv_unit<1, KT_LH / 16, KT_LH>(x, seq, acc);
        red_put<1>(x, acc);
        put_pair(x, a.qkvb, QKVR, c * 16 + el_n(x.tid), rbf(red_get(x, 0)));
        arrive(x, c_layer(l, 0), 0, P);
        LP_STAMP(l, 2);
      }
      if constexpr (R) {
        // ---- attention (cached K / V loaded ahead of the q|k|v hand-off) ----
        if (att && ok) {
          const KVPre pre = att_prefetch(x, a, l, c >> 3, c & 7);
          ok = bwait(x, c_layer(l, 0), P);
          LP_STAMP(l, 3);
          if (ok) attention(x, a, l, c >> 3, c & 7, pre);
          arrive(x, c_layer(l, 1), 0, HKV * a.B);
          LP_STAMP(l, 4);
        }
        // ---- o_proj + residual: row tile c ----
        ok = ok && bwait(x, c_layer(l, 1), HKV * a.B);
        stage_plain<HQ * D>(x, [&](int b) { return a.attnb + (size_t)b * HQ * D; });
        LP_STAMP(l, 5);
        {
          f32x4 acc[1];
          ok = ok && gemv_unit<1, KT_AT / 16, KT_AT>(x, seq, acc);
          red_put<1>(x, acc);
          resadd_out(x, red_get(x, 0), hres, a.h, a.ss, c);
          arrive(x, c_layer(l, 2), 0, NR);
          LP_STAMP(l, 6);
        }
        // ---- round 3 of gate|up (pairs 480 + c, c < 80): post-attention RMSNorm + SwiGLU ----
        if (c < R3_PAIRS) {
          ok = ok && bwait(x, c_layer(l, 2), NR);
          stage_norm(x, a.h, a.ss, lptr(l, P_POSTN));
          f32x4 acc[2];
          ok = ok && gemv_unit<2, KT_LH / 16, KT_LH>(x, seq, acc);
          red_put<2>(x, acc);
          put_pair(x, a.act, LI, (3 * NM + c) * 16 + el_n(x.tid), swiglu(red_get(x, 0), red_get(x, 1)));
          arrive(x, c_layer(l, 6), 0, R3_PAIRS);
          LP_STAMP(l, 11);
        }
        // ---- down_proj + residual: row tile c, its input in rounds 3, 0, 1, 2 of gate|up output ----
        f32x4 dacc = (f32x4){0.f, 0.f, 0.f, 0.f};
        for (int jj = 0; jj < 4 && ok; ++jj) {
          const int j = jj == 0 ? 3 : jj - 1;
          ok = bwait(x, c_layer(l, 3 + j), j < 3 ? NM : R3_PAIRS);
          LP_STAMP(l, 12 + j);
          const int kt0 = j < 3 ? j * ROUND_KT : R3_KT0, nsl = j < 3 ? ROUND_KT / 16 : DOWN_SLOTS_R3;
          // this wave's B fragments of the round's (up to) 5 slots, straight from act (sc1)
          const int b = x.lane & 15;
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.act, 0, NB * LI * 2, 0x00020000);
          u32x4 fr[5][4];
#pragma unroll
          for (int s5 = 0; s5 < 5; ++s5)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const int kt = kt0 + s5 * 16 + x.w * 4 + i;
              fr[s5][i] = __builtin_amdgcn_raw_buffer_load_b128(
                  rs, (b < x.B && s5 < nsl && kt < KT_LI) ? (uint32_t)(b * LI + kt * 32 + 8 * (x.lane >> 4)) * 2u : 0x7ffffff0u,
                  0, 16);
            }
#pragma unroll
          for (int s5 = 0; s5 < 5; ++s5) {
            if (s5 >= nsl) break;
            u32x4 t[4];
            if (!take4(x, seq++, t)) {
              ok = false;
              break;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
              if (kt0 + s5 * 16 + x.w * 4 + i < KT_LI) dacc = mfma(t[i], fr[s5][i], dacc);
          }
        }
        f32x4 acc1[1] = {dacc};
        red_put<1>(x, acc1);
        resadd_out(x, red_get(x, 0), hres, a.h, a.ss, c);
        arrive(x, c_layer(l, 7), 0, NR);
        LP_STAMP(l, 16);
      } else {
        // ---- post-attention RMSNorm + gate|up + SwiGLU: pairs c - NR + 160 j (rounds 0-2) ----
        // (the first pair's 6 slots drain into registers through the wait)
        SlotCache<LPSE_RC> sc;
        const int seq0 = seq;
        ok = ok && bwait(x, c_layer(l, 2), NR, [&]() { sc.drain(x, seq0); });
        stage_norm(x, a.h, a.ss, lptr(l, P_POSTN));
        LP_STAMP(l, 7);
        for (int j = 0; j < 3 && ok; ++j) {
          const int p = c - NR + NM * j;
          f32x4 acc[2];
          ok = j == 0 ? gu_pair_cached(x, seq, sc, acc) : gemv_unit<2, KT_LH / 16, KT_LH>(x, seq, acc);
          red_put<2>(x, acc);
          put_pair(x, a.act, LI, p * 16 + el_n(x.tid), swiglu(red_get(x, 0), red_get(x, 1)));
          arrive(x, c_layer(l, 3 + j), NR, P);
          LP_STAMP(l, 8 + j);
        }
      }
    }
    };
    if (resid) layers(RoleC<true>{});
    else layers(RoleC<false>{});
    // ---- local_transformer.norm + local_to_speech_embedding_mlps[i] (:402-406) ----
    if (ok && c >= 128) {
      ok = bwait(x, c_layer(L - 1, 7), NR);
      stage_norm(x, a.h, a.ss, a.norm);
      f32x4 acc[2];
      ok = ok && gemv_unit<2, KT_LH / 16, KT_LH>(x, seq, acc);
      red_put<2>(x, acc);
      put_pair(x, a.actF, F, (c - 128) * 16 + el_n(x.tid), swiglu(red_get(x, 0), red_get(x, 1)));
      arrive(x, C_MOGU_BASE + 8 * L, 128, P);
    } else if (ok) {
      ok = bwait(x, C_MOGU_BASE + 8 * L, F_PAIRS);
      stage_plain<F>(x, [&](int b) { return a.actF + (size_t)b * F; });
      f32x4 acc[1];
      ok = ok && gemv_unit<1, KT_F / 16, KT_F>(x, seq, acc);
      red_put<1>(x, acc);
      put_pair(x, a.z, H, c * 16 + el_n(x.tid), rbf(red_get(x, 0)));
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    (void)ok;
  }
  // exit: the last workgroup out zeroes the counters for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add((gi32*)(a.cnt + C_EXIT), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == P - 1) {
      for (int k = 0; k < N_CNT; ++k) st32(a.cnt + k, 0u);
      for (int k = 0; k < N_CNT * NGRP; ++k) st32(a.cnt + WS_GC / 4 + (size_t)k * GC_STRIDE, 0u);
      st32(a.epoch, epoch);
    }
  }
}

// ---------------------------------------------------------------------------
size_t lpse_lds_bytes() { return (size_t)L_END; }

bool lpse_supported(int device, int B, int layers, int LH_, int Hq, int Hkv, int D_, int LI_, int F_, int H_, int Cmax) {
  if (B < 1 || B > NB || layers < 1 || layers > LPSE_MAXL || 2 + 8 * layers + 1 > C_EXIT) return false;
  if (LH_ != LH || Hq != HQ || Hkv != HKV || D_ != D || LI_ != LI || F_ != F || H_ != H || Cmax != CMAX) return false;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess || p.multiProcessorCount != P) return false;
  if (hipFuncSetAttribute((const void*)lpse_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lpse_lds_bytes()) !=
      hipSuccess)
    return false;
  int per_cu = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, lpse_kernel, THREADS, lpse_lds_bytes()) == hipSuccess &&
         per_cu >= 1;
}

// counters [N_CNT], error word, epoch, then the release flags [N_CNT][P] lines
size_t lpse_ws_bytes() { return WS_GC + (size_t)N_CNT * NGRP * GC_STRIDE * 4; }

hipError_t lpse_channel(const LpseArgs& a0, void* ws, hipStream_t s) {
  if (a0.layers < 1 || a0.layers > LPSE_MAXL || a0.B < 1 || a0.B > NB || a0.pos < 0 || a0.pos >= CMAX)
    return hipErrorInvalidValue;
  LpseArgs a = a0;
  unsigned char* w = reinterpret_cast<unsigned char*>(ws);
  a.cnt = reinterpret_cast<int*>(w);
  a.err = reinterpret_cast<uint32_t*>(w + N_CNT * 4);
  a.epoch = a.err + 1;
  a.go = reinterpret_cast<uint32_t*>(w + WS_GO);
  hipLaunchKernelGGL(lpse_kernel, dim3(P), dim3(THREADS), lpse_lds_bytes(), s, a);
  return hipGetLastError();
}

uint32_t* lpse_err_word(void* ws) { return reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ws) + N_CNT * 4); }

}  // namespace mtts
