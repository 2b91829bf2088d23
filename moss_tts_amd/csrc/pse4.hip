// Persistent streaming engine for BATCH 4 (configs[2]'s per-GPU share): the decode step's decoder
// stack for 4 rows as ONE launch -- the batch-1 engine of pse.hip (read its header first) with
// every op input, hand-off and epilogue carried for 4 rows.  Per layer, as there:
//   input RMSNorm + q|k|v  ->  attention (q/k norm, RoPE, KV append)  ->  o_proj + residual
//   ->  post-attention RMSNorm + gate|up + SwiGLU  ->  down + residual
// (TF/models/qwen3/modeling_qwen3.py:294-323, :241-280, :81-83).
//
// What changes with 4 rows:
//  * The weight stream is the batch-1 one (same slots, same split); each MFMA's B operand holds the
//    4 rows in columns 0-3 (v_mfma_f32_16x16x32_bf16 computes 16 columns anyway: 4 rows cost no
//    more MFMAs than one), and the epilogues keep columns 0-3.
//  * Op inputs in LDS are [k tile][row][32] bf16: 32 KiB for a 4096-column op.  down_proj's
//    12,288-column input (96 KiB) never sits in LDS whole: the gate|up rounds' SwiGLU columns come
//    in three 32 KiB gathers that alternate between two regions, each gathered while the slots of
//    the previous region run (the batch-1 engine's act pipelining).  Op input = 64 KiB, which
//    leaves a 5-slot ring (80 KiB) besides the loader's 3 register-staged slots.
//  * Hand-offs: the same 8-byte {payload, tag} granules, 4x as many (h: 9,216 per gather).  Every
//    gather ends in a consumer barrier (no per-wave column ownership as in pse.hip).
//  * Attention: 32 units, one per (row, KV head), each the head's 4 q heads over every cached key
//    of its row (each row has its own cache and mask); the units' CUs pause their loaders while the
//    attention runs, their k|v half tile goes to the neighbour CU (as in pse.hip).
#include "kernels.h"
#include "pse_chunk.h"

namespace mtts {

namespace {

constexpr int NB = 4;                   // rows
constexpr int CW = 4;                   // consumer waves
constexpr int LW = 1;                   // loader wave
constexpr int THREADS = (LW + CW) * 64;
#ifndef PSE4_NS
#define PSE4_NS 5
#endif
#ifndef PSE4_RC
#define PSE4_RC 2  // ring slots a plain CU's consumer waves drain into registers during the attention wait
#endif
// PSE4_LC: after those, ring slots drained into region B (free from the previous layer's down_proj
// until this layer's SwiGLU rounds: 2 slots of 16 KiB), so the loader runs RC + LC slots further
// ahead through the attention wait (a register drain past 2 slots spills: 16 / 27 VGPRs at 3 / 4)
#ifndef PSE4_LC
#define PSE4_LC 0
#endif
static_assert(PSE4_LC >= 0 && PSE4_LC <= 2, "region B holds two slots");
// PSE4_HCNT: the residual hand-offs (h after o_proj / down, 9,216 tagged granules per consumer CU)
// as counter + bulk load -- producers store the bf16 rows write-through and bump a per-layer counter,
// consumers poll it and then load the 32 KiB of rows + sums of squares in one round of 16-byte sc1
// loads (lpse.hip's hand-off form; half the bytes and a quarter of the load instructions of a sweep)
#ifndef PSE4_HCNT
#define PSE4_HCNT 2
#endif
// PSE4_ATTF: the attention output hand-off (8,192 granules per consumer CU) in the same release-flag
// form (with PSE4_HCNT 2)
// PSE4_APAUSE: the attention CUs pause their loader through the attention (1, until round 6) or keep it streaming
// (0: 3.036-3.041 -> 3.023-3.029 ms/step same box; pse.hip PSE_APAUSE)
#ifndef PSE4_APAUSE
#define PSE4_APAUSE 0
#endif
#ifndef PSE4_ADB
#define PSE4_ADB 0  // attention: double-buffered chunk loads (A/B)
#endif
#ifndef PSE4_ATTF
#define PSE4_ATTF 0
#endif
#define P4_AFLAG (PSE4_HCNT == 2 && PSE4_ATTF)
// PSE4_HTREE: the 256 arrivals of a residual hand-off counted in two levels -- 8 group counters
// (CUs 32 g .. 32 g + 31, each on its own 128-byte line), whose completing arrival bumps the
// hand-off's counter (8 arrivals) -- instead of 256 agent-scope atomics queueing on one line
#ifndef PSE4_HTREE
#define PSE4_HTREE 1
#endif
constexpr int HGRP = 8;                              // arrival groups
constexpr int GCNT_STRIDE = 32;                      // ints: one 128-byte line per group counter
constexpr int NS = PSE4_NS;
constexpr int SLOT_KB = 16;
constexpr int H_ = 4096, HQ_ = 32, HKV_ = 8, D_ = 128, I_ = 12288, QKVR_ = 6144;
constexpr int G_ = HQ_ / HKV_;
enum { OP_QKV = 0, OP_ATT = 1, OP_O = 2, OP_GU = 3, OP_DOWN = 4 };

typedef __attribute__((address_space(1))) uint64_t g64;
typedef __attribute__((address_space(1))) uint32_t g32;

__device__ __forceinline__ void st64(void* p, uint64_t v) {
  __hip_atomic_store((g64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32(const void* p) {
  return __hip_atomic_load((g32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32(void* p, uint32_t v) {
  __hip_atomic_store((g32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// trace (MTTS_PSE_TRACE=1, scripts/pse4_trace.py): consumer wave 1 per layer -- 0 start, 1 q|k|v input
// normed, 2 q|k|v done, 3 attention done (attention CUs), 4 o input, 5 o done, 6 gate|up input normed,
// 7 gate|up rounds 0-1 done, 8 act round 0 in (+ round 2), 9 round 1 in (+ down 0-7), 10 round 2 in
// (+ down 8-15), 11 down done; loader 12-15 first q|k|v / o / gate|up / down slot issued
#define P4_STAMP(l, ev)                                                                         \
  do {                                                                                          \
    if (a.trace && lane == 0) a.trace[((size_t)(l) * PSE_TRACE_EV + (ev)) * 256 + c] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
__device__ __forceinline__ uint64_t gran(uint32_t payload, uint32_t tag) { return (uint64_t)tag << 32 | payload; }
__device__ __forceinline__ uint32_t tagof(uint32_t epoch, int l, int op) { return epoch << 8 | (uint32_t)(l * 5 + op); }

// granule counts per hand-off (all 4 rows)
constexpr int NG_H = NB * H_ / 2;              // residual: [k tile][row][16]
constexpr int NG_SS = NB * (H_ / 16);          // its sums of squares: [row][256], right behind
constexpr int NG_QKV_ROW = (QKVR_ / 16) * 2 * 16;  // q|k|v K-half partials of one row (768 units x 16)
constexpr int NG_ATT = NB * HQ_ * D_ / 2;      // attention output: [k tile][row][16]
constexpr int NG_ACT = NB * I_ / 2;            // SwiGLU output: [k tile][row][16]
constexpr int NG_ACT_ROUND = NG_ACT / 3;

// same unit / slot map as pse.hip (q|k|v units, o_proj row tile c, gate|up pairs c + 256 j, down
// row tile c), with this launch's attention CUs
__device__ __forceinline__ void qkv_unit(int c, int j, int* t, int* half) {
  const int o = j == 3 ? c + 1 : c;
  *t = j < 2 ? c : HQ_ * D_ / 16 + (o >> 1);
  *half = j < 2 ? j : (o & 1);
}
__device__ __forceinline__ int gu_pair(int c, int j) { return c + 256 * j; }

}  // namespace

// PSE4_KS (round 6): attention units per (row, KV head), splitting its cached keys (pse.hip PSE_KSPLIT):
// unit k takes the 32-key chunks of share k for the head's 4 q heads; units 1 .. KS-1 publish their
// unnormalised rows and (max, sum) per head, unit 0 folds them in with the new key.  1: one unit.
#ifndef PSE4_KS
#define PSE4_KS 1
#endif
static_assert(PSE4_KS == 1 || PSE4_KS == 2, "1 or 2 units per (row, KV head)");
constexpr int AUS = PSE4_KS == 1 ? 7 : 3;  // CU spacing of the units (every XCD under round-robin placement)
// (PSE4_KS 2) a (row, KV head)'s partner part: rows [G][D] fp32, then (max, sum) per head
constexpr int KS_ROWS = G_ * D_, KS_N = (PSE4_KS - 1) * (G_ * D_ + 2 * G_);
// attention units: unit u = (row * 8 + head) * KS + k on CU P - 1 - AUS u
__host__ __device__ inline int pse4_att_unit(int c, int P) {
  const int d = P - 1 - c;
  return (d >= 0 && d % AUS == 0 && d / AUS < HKV_ * NB * PSE4_KS) ? d / AUS : -1;
}
__host__ __device__ inline int pse4_nq(int c, int P) {
  return pse4_att_unit(c, P) >= 0 ? 2 : (pse4_att_unit(c + 1, P) >= 0 ? 4 : 3);
}

namespace {

__device__ __forceinline__ const bf16_t* slot_src(const bf16_t* const* wp, int c, int nq, int s) {
  const int spl = 4 * nq + 80, l = s / spl, r = s - l * spl, rq = 4 * nq;
  if (r < rq) {
    int t, half;
    qkv_unit(c, r / 4, &t, &half);
    return wp[l * 4 + 0] + ((size_t)t * 128 + half * 64 + (r % 4) * 16) * 512;
  } else if (r < rq + 8) {
    return wp[l * 4 + 1] + ((size_t)c * 128 + (r - rq) * 16) * 512;
  } else if (r < rq + 56) {
    const int q = r - rq - 8, pr = gu_pair(c, q / 16), rt = 2 * pr + (q % 16) / 8;
    return wp[l * 4 + 2] + ((size_t)rt * 128 + (q % 8) * 16) * 512;
  }
  return wp[l * 4 + 3] + ((size_t)c * 384 + (r - rq - 56) * 16) * 512;
}

struct Ctl {
  int full;
  int freed[CW];
  int bar;
  int abort;
  int apause;
};

constexpr uint32_t SPIN_LDS = 1u << 22;
constexpr uint32_t SPIN_MEM = 1u << 18;

// LDS layout (bytes)
constexpr int XR = NB * H_ * 2;                        // one 4096-column op input: 32 KiB
constexpr int L_CTL = 0;
constexpr int L_RING = 256;
constexpr int L_XA = L_RING + NS * SLOT_KB * 1024;     // region A: normed inputs, o_proj input, act rounds 1
constexpr int L_XB = L_XA + XR;                        // region B: act rounds 0 and 2
constexpr int L_RED = L_XB + XR;                       // [CW][2][NB][16] fp32
constexpr int L_MISC = L_RED + CW * 2 * NB * 16 * 4;   // [NB][256] gathered sums of squares
constexpr int PSE_MAXL = 64;
constexpr int L_PTR = L_MISC + NB * 256 * 4;
constexpr int L_END = L_PTR + PSE_MAXL * 4 * 8;
static_assert(L_END <= 160 * 1024, "LDS");
// attention CUs' scratch over region A (q|k|v's input is consumed, o_proj's gather comes after):
// gathered q|k|v partials [48 tiles][2][16] fp32, q_s [16][D] bf16, k_s / v_s [D] fp32,
// p_s [CW][16][32] bf16, ml_s [CW][G][2], acc_s [CW][G][D]
constexpr int L_GRAW = L_XA;
constexpr int L_ATT = L_GRAW + 1536 * 4;
static_assert(L_ATT + 16 * D_ * 2 + 2 * D_ * 4 + CW * 16 * 32 * 2 + CW * G_ * 2 * 4 + CW * G_ * D_ * 4 <= L_XA + 2 * XR,
              "attention scratch fits the op input regions");

extern __shared__ __attribute__((aligned(16))) unsigned char p4_lds[];
#define P4_CTL (reinterpret_cast<Ctl*>(p4_lds + L_CTL))

struct Ctx {
  uint32_t* err;
  float eps;
  int c, lane, wave, tid;
  uint32_t epoch;
  int bar_gen;
};

__device__ __forceinline__ bool failed(const Ctx& x) {
  return __hip_atomic_load(&P4_CTL->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;
}
__device__ __forceinline__ void give_up(Ctx& x, uint32_t code) {
  st32(x.err, code);
  __hip_atomic_store(&P4_CTL->abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void cbar(Ctx& x) {
  x.bar_gen += CW;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (x.lane == 0) __hip_atomic_fetch_add(&P4_CTL->bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  uint32_t spins = 0;
  while (__hip_atomic_load(&P4_CTL->bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < x.bar_gen) {
    if (++spins > SPIN_LDS) {
      give_up(x, 4);
      break;
    }
    __builtin_amdgcn_s_sleep(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct NoHook {
  __device__ void operator()() const {}
};
template <bool B>
struct BoolC4 {
  static constexpr bool value = B;
};
template <int V>
struct IntC4 {
  static constexpr int value = V;
};
// Gather granules g[0..n) carrying tag t into LDS words (the first n0 to dst0, the rest to dst1):
// every consumer thread takes granules tid + 256 k in ONE sweep loop (pse.hip `gather`), then a
// consumer barrier.  `after_first_issue` runs behind the first sweep (work independent of the
// granules), `each_poll` after every sweep's results are in.
template <int MAXP, typename Hook = NoHook, typename Poll = NoHook>
__device__ __forceinline__ bool gather(Ctx& x, const uint64_t* g, int n, uint32_t t, uint32_t* dst0, int n0,
                                       uint32_t* dst1 = nullptr, const Hook& after_first_issue = Hook(),
                                       const Poll& each_poll = Poll()) {
  constexpr uint32_t OOB = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(g), 0, n * 8, 0x00020000);
  uint64_t pend = 0;
#pragma unroll
  for (int i = 0; i < MAXP; ++i)
    if (x.tid + i * CW * 64 < n) pend |= 1ull << i;
  __builtin_amdgcn_s_setprio(3);
  bool ok = true;
  uint32_t lo[MAXP], hi[MAXP];
  // one lane offset (tid * 8) for every granule i: i's 2 KiB stride rides in the SGPR offset, so a
  // gather site keeps no per-granule offset registers live across the layer loop (MAXP = 36 of
  // them spilled the consumers' registers)
  const uint32_t vo = (uint32_t)x.tid * 8u;
  auto issue = [&]() {
#pragma unroll
    for (int i = 0; i < MAXP; ++i) {
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (pend >> i & 1ull) ? vo : OOB, i * CW * 64 * 8, 16 /* sc1 */);
      lo[i] = v[0];
      hi[i] = v[1];
    }
  };
  // (n0 % 256 == 0: granule i of every thread goes to the same destination)
  auto take = [&]() {
#pragma unroll
    for (int i = 0; i < MAXP; ++i)
      if ((pend >> i & 1ull) && hi[i] == t) {
        if (i * CW * 64 < n0) dst0[x.tid + i * CW * 64] = lo[i];
        else dst1[x.tid + i * CW * 64 - n0] = lo[i];
        pend &= ~(1ull << i);
      }
  };
  issue();
  after_first_issue();
  take();
  each_poll();
  for (uint32_t spins = 1; __any(pend != 0); ++spins) {
    if (spins > SPIN_MEM || ((spins & 255) == 255 && (failed(x) || ld32(x.err)))) {
      give_up(x, 2);
      ok = false;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    issue();
    take();
    each_poll();
  }
  __builtin_amdgcn_s_setprio(0);
  cbar(x);
  return ok && !failed(x);
}

// PSE4_HCNT: wait for hand-off k (counter hcnt[k] at `target`, or with PSE4_HCNT 2 this CU's own
// release flag), then bulk-load 4 rows (bf16 [4][H] at hb) into region A as [k tile][row][16 words]
// and, with hs, their sums of squares (fp32 [4][256]) into ss32; `hook` runs before the poll (loads
// independent of it), `each_poll` after every poll (the ring slot drain)
template <typename Hook, typename Poll = NoHook>
__device__ __forceinline__ bool hgather(Ctx& x, const int* hcnt, const uint32_t* go, int k, int target, const bf16_t* hb,
                                        const float* hs, uint32_t* xa32, uint32_t* ss32, const Hook& hook,
                                        const Poll& each_poll = Poll()) {
  hook();
  __builtin_amdgcn_s_setprio(3);
  // (PSE4_HCNT 2: this CU's own release flag line; 1: the counter line every consumer wave polls)
  for (uint32_t spins = 0; PSE4_HCNT == 2 ? ld32(go + ((size_t)k * 256 + x.c) * 32) != x.epoch : (int)ld32(hcnt + k) < target;
       ++spins) {
    if (spins > SPIN_MEM || ((spins & 255) == 255 && (failed(x) || ld32(x.err)))) {
      give_up(x, 2);
      __builtin_amdgcn_s_setprio(0);
      return false;
    }
    each_poll();
    __builtin_amdgcn_s_sleep(1);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (every read below is an sc1 load)
  constexpr int CPR = H_ / 8;  // 16-byte chunks per row
  const __amdgpu_buffer_rsrc_t hrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(hb), 0, NB * H_ * 2, 0x00020000);
  u32x4 v[NB * CPR / (CW * 64)];
#pragma unroll
  for (int j = 0; j < NB * CPR / (CW * 64); ++j) {
    const int b = j / (CPR / (CW * 64)), c8 = x.tid + (CW * 64) * (j % (CPR / (CW * 64)));
    v[j] = __builtin_amdgcn_raw_buffer_load_b128(hrs, (uint32_t)(b * H_ + c8 * 8) * 2u, 0, 16 /* sc1 */);
  }
  u32x4 sv = (u32x4){0u, 0u, 0u, 0u};
  if (hs) {
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(hs), 0, NB * (H_ / 16) * 4, 0x00020000);
    sv = __builtin_amdgcn_raw_buffer_load_b128(srs, (uint32_t)x.tid * 16u, 0, 16);
  }
  u32x4* xa = reinterpret_cast<u32x4*>(xa32);
#pragma unroll
  for (int j = 0; j < NB * CPR / (CW * 64); ++j) {
    const int b = j / (CPR / (CW * 64)), c8 = x.tid + (CW * 64) * (j % (CPR / (CW * 64)));
    xa[((c8 >> 2) * NB + b) * 4 + (c8 & 3)] = v[j];
  }
  if (hs) reinterpret_cast<u32x4*>(ss32)[x.tid] = sv;
  __builtin_amdgcn_s_setprio(0);
  cbar(x);
  return !failed(x);
}
// one arrival at hand-off k after this CU's stores of it drained (by every storing wave); the
// arrival that completes it (target) releases every consumer CU's flag line (PSE4_HCNT 2)
__device__ __forceinline__ void harrive(const Ctx& x, int* hcnt, uint32_t* go, int k, int target) {
  typedef __attribute__((address_space(1))) int gi;
  int t = 0;
  if (PSE4_HTREE && target == 256) {
    // group counter g = c / 32 (its line: hcnt + 3 PSE_MAXL + (k HGRP + g) GCNT_STRIDE); the group's
    // 32nd arrival is the one arrival at the hand-off's counter
    int* gc = hcnt + 3 * PSE_MAXL + ((size_t)k * HGRP + x.c / (256 / HGRP)) * GCNT_STRIDE;
    if (x.lane == 0) {
      t = __hip_atomic_fetch_add((gi*)gc, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = t == 256 / HGRP - 1 ? __hip_atomic_fetch_add((gi*)(hcnt + k), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : -1;
    }
    t = __shfl(t, 0, 64);
    target = HGRP;
  } else {
    if (x.lane == 0) t = __hip_atomic_fetch_add((gi*)(hcnt + k), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t = __shfl(t, 0, 64);
  }
  if (PSE4_HCNT == 2 && t == target - 1)
#pragma unroll
    for (int i = 0; i < 4; ++i) st32(go + ((size_t)k * 256 + x.lane + 64 * i) * 32, x.epoch);
}
static_assert(NB * (H_ / 16) == 4 * CW * 64, "one 16-byte sums-of-squares chunk per consumer thread");

// q|k|v partial granules of row b, grouped by KV head (pse.hip qkv_gran) -- unit (b, g) gathers
// one contiguous range
__device__ __forceinline__ int qkv_gran(int t) {
  constexpr int TPH = D_ / 16, G = HQ_ / HKV_, GT = (G + 2) * TPH;
  int g, o;
  if (t < HQ_ * TPH) { g = t / (G * TPH); o = t - g * G * TPH; }
  else if (t < (HQ_ + HKV_) * TPH) { g = (t - HQ_ * TPH) / TPH; o = G * TPH + (t - HQ_ * TPH - g * TPH); }
  else { g = (t - (HQ_ + HKV_) * TPH) / TPH; o = (G + 1) * TPH + (t - (HQ_ + HKV_) * TPH - g * TPH); }
  return (g * GT + o) * 32;
}

// an op input's granule / LDS word of (row b, column pair starting at even column k):
// [k tile][row][16 words]
__device__ __forceinline__ int xword(int b, int k) { return ((k >> 5) * NB + b) * 16 + ((k & 31) >> 1); }

// Qwen3RMSNorm of the gathered 4096-column rows in region A, in place: thread t normalises column
// groups t and t + 256 (8 columns each) of all 4 rows; r_b from row b's 256 per-16-column sums of
// squares (summed as pse.hip / the GEMV prologue sum them).  nw: this thread's 2 weight groups.
struct NormW {
  u32x4 a, b;
};
__device__ __forceinline__ NormW norm_w(const Ctx& x, const bf16_t* w) {
  const u32x4* wv = reinterpret_cast<const u32x4*>(w);
  return NormW{wv[x.tid], wv[x.tid + 256]};
}
__device__ __forceinline__ void norm_stage(Ctx& x, NormW nw) {
  const float* ss = reinterpret_cast<const float*>(p4_lds + L_MISC);
  float r[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const float* sb = ss + b * 256;
    float s = (sb[4 * x.lane] + sb[4 * x.lane + 1]) + (sb[4 * x.lane + 2] + sb[4 * x.lane + 3]);
    s = wave_sum(s);
    r[b] = 1.0f / sqrtf(s / (float)H_ + x.eps);
  }
  u32x4* xv = reinterpret_cast<u32x4*>(p4_lds + L_XA);
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cg = x.tid + 256 * j;  // column group: columns 8 cg .. 8 cg + 7
    const u32x4 nv = j ? nw.b : nw.a;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      const int i = ((cg >> 2) * NB + b) * 4 + (cg & 3);
      const u32x4 hv = xv[i];
      u32x4 o;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float h0 = __uint_as_float(hv[q] << 16), h1 = __uint_as_float(hv[q] & 0xffff0000u);
        const float w0 = __uint_as_float(nv[q] << 16), w1 = __uint_as_float(nv[q] & 0xffff0000u);
        o[q] = pack2(w0 * rbf(h0 * r[b]), w1 * rbf(h1 * r[b]));
      }
      xv[i] = o;
    }
  }
  cbar(x);
}

// This consumer wave's 4 tiles of ring slot `seq` times the input region at byte offset `reg`,
// k tiles kt0 + 4 w .. (B operand: lane l holds row l & 3 -- columns 4-15 repeat rows 0-3 and are
// never kept)
__device__ __forceinline__ void consume_slot(Ctx& x, int seq, int reg, int kt0, f32x4& acc) {
  for (uint32_t spins = 0; __hip_atomic_load(&P4_CTL->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) <= seq;
       ++spins) {
    if (spins > SPIN_LDS || failed(x)) {
      give_up(x, 3);
      return;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  const u32x4* sl = reinterpret_cast<const u32x4*>(p4_lds + L_RING + (seq % NS) * SLOT_KB * 1024);
  const u32x4* xv = reinterpret_cast<const u32x4*>(p4_lds + reg);
  const int w = x.wave - LW;
  u32x4 wt[4], xb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = w * 4 + i;
    wt[i] = sl[t * 64 + x.lane];
    xb[i] = xv[((kt0 + t) * NB + (x.lane & (NB - 1))) * 4 + (x.lane >> 4)];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (x.lane == 0) __hip_atomic_store(&P4_CTL->freed[w], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
  for (int i = 0; i < 4; ++i)
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wt[i]), __builtin_bit_cast(bf16x8, xb[i]),
                                                  acc, 0, 0, 0);
}

// ring slot drain into registers during the attention wait (pse.hip SlotCache)
__device__ __forceinline__ bool slot_ready(int seq) {
  return __hip_atomic_load(&P4_CTL->full, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) > seq;
}
template <int RC, int LC = 0>
struct SlotCache {
  u32x4 rc[RC > 0 ? RC : 1][4];
  int nd = 0;
  __device__ __forceinline__ void drain(Ctx& x, int seq) {
#pragma unroll
    for (int k = 0; k < RC + LC; ++k)
      if (k == nd && slot_ready(seq + k)) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const u32x4* sl = reinterpret_cast<const u32x4*>(p4_lds + L_RING + ((seq + k) % NS) * SLOT_KB * 1024);
        const int w = x.wave - LW;
        if (k < RC) {
#pragma unroll
          for (int i = 0; i < 4; ++i) rc[k < RC ? k : 0][i] = sl[(w * 4 + i) * 64 + x.lane];
        } else {  // this wave's 4 tiles -> region B slot k - RC (same tile layout as a ring slot)
          u32x4* lb = reinterpret_cast<u32x4*>(p4_lds + L_XB + (k - RC) * SLOT_KB * 1024);
          u32x4 t[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) t[i] = sl[(w * 4 + i) * 64 + x.lane];
#pragma unroll
          for (int i = 0; i < 4; ++i) lb[(w * 4 + i) * 64 + x.lane] = t[i];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (x.lane == 0)
          __hip_atomic_store(&P4_CTL->freed[w], seq + k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        ++nd;
      }
  }
  // slot i (RC <= i < RC + LC) from region B, else the ring
  __device__ __forceinline__ void take_lds(Ctx& x, int& seq, int i, int reg, int kt0, f32x4& acc) {
    if (i < nd) {
      const u32x4* lb = reinterpret_cast<const u32x4*>(p4_lds + L_XB + (i - RC) * SLOT_KB * 1024);
      const u32x4* xv = reinterpret_cast<const u32x4*>(p4_lds + reg);
      const int w = x.wave - LW;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 wt = lb[(w * 4 + q) * 64 + x.lane];
        const u32x4 xb = xv[((kt0 + w * 4 + q) * NB + (x.lane & (NB - 1))) * 4 + (x.lane >> 4)];
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wt), __builtin_bit_cast(bf16x8, xb), acc,
                                                      0, 0, 0);
      }
      ++seq;
    } else {
      consume_slot(x, seq++, reg, kt0, acc);
    }
  }
  __device__ __forceinline__ void take(Ctx& x, int& seq, int i, int reg, int kt0, f32x4& acc) {
    if (i < RC && i < nd) {
      const u32x4* xv = reinterpret_cast<const u32x4*>(p4_lds + reg);
      const int w = x.wave - LW;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const u32x4 xb = xv[((kt0 + w * 4 + q) * NB + (x.lane & (NB - 1))) * 4 + (x.lane >> 4)];
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, rc[i < RC ? i : 0][q]),
                                                      __builtin_bit_cast(bf16x8, xb), acc, 0, 0, 0);
      }
      ++seq;
    } else {
      consume_slot(x, seq++, reg, kt0, acc);
    }
  }
};

// fixed-order reduction of the CW waves' partial tiles: columns 0..NB-1 (MFMA D: lane l holds
// rows 4 (l >> 4) + i of column l & 15)
__device__ __forceinline__ void red_put(Ctx& x, int r, const f32x4& acc) {
  if ((x.lane & 15) >= NB) return;
  float* p = reinterpret_cast<float*>(p4_lds + L_RED) + (((x.wave - LW) * 2 + r) * NB + (x.lane & 15)) * 16 +
             (x.lane >> 4) * 4;
  p[0] = acc[0]; p[1] = acc[1]; p[2] = acc[2]; p[3] = acc[3];
}
__device__ __forceinline__ float red_get(int r, int col, int row) {
  const float* red = reinterpret_cast<const float*>(p4_lds + L_RED);
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < CW; ++w) s += red[((w * 2 + r) * NB + col) * 16 + row];
  return s;
}

// ---------------------------------------------------------------------------
// Attention unit (row b, KV head g): the head's 4 q heads over every cached key of row b (pse.hip
// attention() with one unit per head, HU = 4): q / k RMSNorm + RoPE, K / V appended at pos,
// softmax(q k^T / sqrt(D)) v with bf16 probabilities before P.V, per-wave online softmax over
// 32-key chunks run while the new token's k / v are gathered, the wave partials and the new key
// merged in a fixed order, the 4 x D outputs published as granules.  Not inlined (its chunk
// state would push the layer loop's allocation past the budget).  Returns the barrier count, -1
// on a failed wait.
// (KU: the unit's role with PSE4_KS 2, one callee per role; 0 without the key split)
template <int KU>
__device__ __attribute__((noinline)) int attention(const PseLayer* Lp, const int* pos_p, const uint8_t* mask_all,
                                                   const bf16_t* cos_t, const bf16_t* sin_t, uint64_t* g_qkv,
                                                   uint64_t* g_att, uint64_t* g_pp, int* hcnt, uint32_t* go, uint32_t* err,
                                                   uint64_t* trace,
                                                   float eps, float scale, int Cmax,
                                                   uint32_t epoch, int bar_gen, int l, int unit, uint32_t tq) {
  Ctx x{err, eps, (int)blockIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6), (int)threadIdx.x - LW * 64,
        epoch, bar_gen};
  constexpr int D = D_, G = G_, KW = 32, QS = D / 32, DT = D / 16, HU = G_;
  const int pair = unit / PSE4_KS, kk = unit % PSE4_KS;
  const int b = pair / HKV_, g = pair % HKV_;
  const float* graw = reinterpret_cast<const float*>(p4_lds + L_GRAW);
  uint32_t* graw32 = reinterpret_cast<uint32_t*>(p4_lds + L_GRAW);
  const PseLayer& Lw = *Lp;
  const int pos = *pos_p;
  const int lane = x.lane, w = x.wave - LW, g4 = lane >> 4, c16 = lane & 15;
  bf16_t* kcache = Lw.kc + ((size_t)b * HKV_ + g) * Cmax * D;  // [Cmax][D]
  bf16_t* vcache = Lw.vc + ((size_t)b * HKV_ + g) * D * Cmax;  // [D][Cmax]
  const uint8_t* mask = mask_all + (size_t)b * Cmax;
  bf16_t* q_s = reinterpret_cast<bf16_t*>(p4_lds + L_ATT);
  float* k_s = reinterpret_cast<float*>(q_s + 16 * D);
  float* v_s = k_s + D;
  bf16_t* p_s = reinterpret_cast<bf16_t*>(v_s + D);
  float* ml_s = reinterpret_cast<float*>(p_s + CW * 16 * KW);
  float* acc_s = ml_s + CW * G * 2;
  constexpr uint32_t OOBA = 0x7ffffff0u;
  const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(kcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(vcache, 0, Cmax * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t mrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(mask), 0, Cmax, 0x00020000);
  const int nchunk = pos / KW + 1;
  const int cb = kk * nchunk / PSE4_KS, ce = (kk + 1) * nchunk / PSE4_KS;  // this unit's chunks
  auto load_chunk = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], uint32_t (&mk)[2]) {
    const int k0 = ch * KW;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int key = k0 + t * 16 + c16;
#pragma unroll
      for (int s2 = 0; s2 < QS; ++s2)
        kt[t][s2] = __builtin_amdgcn_raw_buffer_load_b128(
            krs, key < pos ? (uint32_t)(key * D + s2 * 32 + 8 * g4) * 2u : OOBA, 0, 0);
      mk[t] = __builtin_amdgcn_raw_buffer_load_b32(mrs, (k0 + t * 16 <= pos) ? (uint32_t)(k0 + t * 16 + g4 * 4) : OOBA,
                                                   0, 0);
    }
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int kb = k0 + 8 * g4;
      vt[dt] = __builtin_amdgcn_raw_buffer_load_b128(
          vrs, kb < pos ? (uint32_t)((dt * 16 + c16) * Cmax + kb) * 2u : OOBA, 0, 0);
    }
  };
  u32x4 ktA[2][QS], vtA[DT];
  uint32_t mkA[2];
  const int ch0 = cb + w;
  uint32_t qnw = 0, knw = 0, pcs = 0, psn = 0, mnew = 0;
  auto prefetch = [&]() {
    load_chunk(ch0, ktA, vtA, mkA);
    qnw = reinterpret_cast<const uint32_t*>(Lw.q_norm)[lane];
    knw = reinterpret_cast<const uint32_t*>(Lw.k_norm)[lane];
    pcs = reinterpret_cast<const uint32_t*>(cos_t + (size_t)pos * D)[lane];
    psn = reinterpret_cast<const uint32_t*>(sin_t + (size_t)pos * D)[lane];
    mnew = mask[pos];
  };
  auto val = [&](int base_tile, int i) {
    const float* p = graw + (base_tile + i / 16) * 32 + i % 16;
    return rbf(p[0] + p[16]);
  };
  auto norm_rope = [&](float x0, float x1, uint32_t nw, float& o0, float& o1) {
    const float ss = wave_sum(x0 * x0 + x1 * x1);
    const float r = 1.0f / sqrtf(ss / (float)D + eps);
    const float n0 = rbf(__uint_as_float(nw << 16) * rbf(x0 * r)), n1 = rbf(__uint_as_float(nw & 0xffff0000u) * rbf(x1 * r));
    constexpr int q4 = D / 4;
    const bool lo = 2 * lane < D / 2;
    const int partner = lo ? lane + q4 : lane - q4;
    const float p0 = __shfl(n0, partner, 64), p1 = __shfl(n1, partner, 64);
    const float sg = lo ? -1.f : 1.f;
    const float c0 = __uint_as_float(pcs << 16), c1 = __uint_as_float(pcs & 0xffff0000u);
    const float s0 = __uint_as_float(psn << 16), s1 = __uint_as_float(psn & 0xffff0000u);
    o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
    o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
  };
  if (PSE4_APAUSE && x.tid == 0) __hip_atomic_store(&P4_CTL->apause, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  // ---- 1. q (this row's q tiles of the head's 4 q heads, complete two thirds into q|k|v) ----
  constexpr int NG = (G_ + 2) * (D_ / 16) * 32;
  constexpr int NQ = HU * (D_ / 16) * 32, NKV = 2 * (D_ / 16) * 32;
  uint64_t* gq = g_qkv + (size_t)b * NG_QKV_ROW + (size_t)g * NG;
#define P4_ASTAMP(ev)                                                                                 \
  do {                                                                                                \
    if (trace && w == 0 && lane == 0)                                                                 \
      trace[((size_t)l * PSE_TRACE_EV + (ev)) * 256 + x.c] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
  if (!gather<(NQ + CW * 64 - 1) / (CW * 64)>(x, gq, NQ, tq, graw32, NQ, nullptr, prefetch)) return -1;
  P4_ASTAMP(16);
  if (w < HU) {
    const int bt = w * (D / 16);
    float o0, o1;
    norm_rope(val(bt, 2 * lane), val(bt, 2 * lane + 1), qnw, o0, o1);
    q_s[w * D + 2 * lane] = f2bf(o0);
    q_s[w * D + 2 * lane + 1] = f2bf(o1);
  }
  for (int i = x.tid; i < 16 * D; i += CW * 64)
    if (i / D >= HU) q_s[i] = 0;
  cbar(x);
  // ---- 2. the cached keys ----
  float m_run = -INFINITY, l_run = 0.f;
  float* o_s = acc_s + w * HU * D + c16;  // the running output (pse_chunk.h)
  pse_chunk_init<HU, D>(g4, o_s);
  auto compute = [&](int ch, u32x4 (&kt)[2][QS], u32x4 (&vt)[DT], const uint32_t (&mk)[2]) {
    pse_chunk_step<HU, D>(ch * KW, pos, g4, c16, kt, vt, mk, q_s, p_s + w * 16 * KW, o_s, scale, m_run, l_run);
  };
  auto chunks = [&]() {
#if PSE4_ADB
    // two chunks in flight per wave: the next chunk's K / V^T load while this one computes
    u32x4 ktB[2][QS], vtB[DT];
    uint32_t mkB[2];
    int ch = ch0;
    if (ch + CW < nchunk) load_chunk(ch + CW, ktB, vtB, mkB);
    while (ch < nchunk) {
      compute(ch, ktA, vtA, mkA);
      ch += CW;
      if (ch >= nchunk) break;
      if (ch + CW < nchunk) load_chunk(ch + CW, ktA, vtA, mkA);
      compute(ch, ktB, vtB, mkB);
      ch += CW;
      if (ch >= nchunk) break;
      if (ch + CW < nchunk) load_chunk(ch + CW, ktB, vtB, mkB);
    }
#else
    for (int ch = ch0; ch < ce; ch += CW) {
      if (ch != ch0) load_chunk(ch, ktA, vtA, mkA);
      compute(ch, ktA, vtA, mkA);
    }
#endif
  };
  if (KU == 1) {  // (only unit 0 takes the new token's k / v)
    chunks();
    if (failed(x)) return -1;
  } else if (!gather<(NKV + CW * 64 - 1) / (CW * 64)>(x, gq + G * (D_ / 16) * 32, NKV, tq, graw32 + G * (D_ / 16) * 32,
                                                      NKV, nullptr, chunks)) {
    return -1;
  }
  P4_ASTAMP(17);
  // ---- 3. k (wave 0) and v (wave 1), appended at pos ----
  if (KU == 1) {
  } else if (w == 0) {
    float o0, o1;
    norm_rope(val(G * (D / 16), 2 * lane), val(G * (D / 16), 2 * lane + 1), knw, o0, o1);
    k_s[2 * lane] = o0;
    k_s[2 * lane + 1] = o1;
    *reinterpret_cast<uint32_t*>(kcache + (size_t)pos * D + 2 * lane) = pack2(o0, o1);
  } else if (w == 1) {
    const float x0 = val((G + 1) * (D / 16), 2 * lane), x1 = val((G + 1) * (D / 16), 2 * lane + 1);
    v_s[2 * lane] = x0;
    v_s[2 * lane + 1] = x1;
    vcache[(size_t)(2 * lane) * Cmax + pos] = f2bf(x0);
    vcache[(size_t)(2 * lane + 1) * Cmax + pos] = f2bf(x1);
  }
  if (lane < HU) {
    ml_s[(w * HU + lane) * 2] = m_run;
    ml_s[(w * HU + lane) * 2 + 1] = l_run;
  }
  cbar(x);
  // (PSE4_KS 2) unit 0: the partner's rows -> graw (q / k / v are in q_s / k_s / v_s), its (max, sum)
  // per head -> the sums-of-squares scratch (free through the attention)
  const float* pp = graw;
  const float* pml = reinterpret_cast<const float*>(p4_lds + L_MISC);
  if constexpr (PSE4_KS > 1 && KU == 0) {
    if (!gather<(KS_N + CW * 64 - 1) / (CW * 64)>(x, g_pp + (size_t)pair * KS_N, KS_N, tagof(x.epoch, l, OP_ATT), graw32,
                                                  (PSE4_KS - 1) * KS_ROWS, reinterpret_cast<uint32_t*>(p4_lds + L_MISC)))
      return -1;
  }
  // ---- 4. merge (thread e / 2: 2 dims of local head e / D) and publish ----
  const int e = 2 * x.tid, h = e / D, d = e % D;
  {
    float M = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) M = fmaxf(M, ml_s[(ww * HU + h) * 2]);
    const float sn = wave_sum(bf2f(q_s[h * D + d]) * k_s[d] + bf2f(q_s[h * D + d + 1]) * k_s[d + 1]) * scale;
    const bool nv = mnew != 0u && KU == 0;
    if (nv) M = fmaxf(M, sn);
    float L = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int ww = 0; ww < CW; ++ww) {
      const float mw = ml_s[(ww * HU + h) * 2];
      const float f = (mw == -INFINITY) ? 0.f : expf(mw - M);
      L += f * ml_s[(ww * HU + h) * 2 + 1];
      o0 += f * acc_s[(ww * HU + h) * D + d];
      o1 += f * acc_s[(ww * HU + h) * D + d + 1];
    }
    if (nv) {
      const float f = expf(sn - M);
      L += f;
      o0 += f * v_s[d];
      o1 += f * v_s[d + 1];
    }
    if (KU == 1) {  // this unit's part, unnormalised, against its own max
      const uint32_t ta = tagof(x.epoch, l, OP_ATT);
      uint64_t* q = g_pp + (size_t)pair * KS_N;
      const int pi = kk - 1;
      st64(q + pi * KS_ROWS + h * D + d, gran(__float_as_uint(o0), ta));
      st64(q + pi * KS_ROWS + h * D + d + 1, gran(__float_as_uint(o1), ta));
      if (d == 0) {
        st64(q + (PSE4_KS - 1) * KS_ROWS + pi * 2 * G + 2 * h, gran(__float_as_uint(M), ta));
        st64(q + (PSE4_KS - 1) * KS_ROWS + pi * 2 * G + 2 * h + 1, gran(__float_as_uint(L), ta));
      }
    } else {
      if (PSE4_KS > 1) {  // the partners' parts, in unit order, rescaled to the joint max
        float Mj = M;
#pragma unroll
        for (int pi = 0; pi < PSE4_KS - 1; ++pi) Mj = fmaxf(Mj, pml[pi * 2 * G + 2 * h]);
        const float f0 = (M == -INFINITY) ? 0.f : expf(M - Mj);
        L *= f0;
        o0 *= f0;
        o1 *= f0;
#pragma unroll
        for (int pi = 0; pi < PSE4_KS - 1; ++pi) {
          const float mp = pml[pi * 2 * G + 2 * h];
          const float fp = (mp == -INFINITY) ? 0.f : expf(mp - Mj);
          L += fp * pml[pi * 2 * G + 2 * h + 1];
          o0 += fp * pp[pi * KS_ROWS + h * D + d];
          o1 += fp * pp[pi * KS_ROWS + h * D + d + 1];
        }
      }
      if (P4_AFLAG)  // rows bf16 [4][4096] over the granule region; one arrival below
        st32(reinterpret_cast<bf16_t*>(g_att) + (size_t)b * HQ_ * D_ + (g * G + h) * D + d, L > 0.f ? pack2(o0 / L, o1 / L) : 0u);
      else
        st64(g_att + xword(b, (g * G + h) * D + d), gran(L > 0.f ? pack2(o0 / L, o1 / L) : 0u, tagof(x.epoch, l, OP_ATT)));
    }
  }
  if (P4_AFLAG) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  cbar(x);
  P4_ASTAMP(18);
  if (P4_AFLAG && w == 0 && KU == 0) harrive(x, hcnt, go, 2 * PSE_MAXL + l, HKV_ * NB);
  return x.bar_gen;
}

}  // namespace

// ---------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void pse4_kernel(PseArgs a) {
  unsigned char* const lds = p4_lds;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x, P = gridDim.x;
  Ctl* ctl = reinterpret_cast<Ctl*>(lds + L_CTL);
  static_assert(sizeof(Ctl) <= 256, "control words");
  if (threadIdx.x < 64) reinterpret_cast<int*>(lds + L_CTL)[threadIdx.x] = 0;
  const bf16_t** wp = reinterpret_cast<const bf16_t**>(lds + L_PTR);
  for (int i = threadIdx.x; i < a.layers * 4; i += THREADS) {
    const PseLayer& q = a.L[i / 4];
    wp[i] = (i & 3) == 0 ? q.qkv : ((i & 3) == 1 ? q.o : ((i & 3) == 2 ? q.gu : q.down));
  }
  __syncthreads();
  const uint32_t epoch = (ld32(a.epoch) + 1u) & 0xffffffu;
  const int nq = pse4_nq(c, P), spl = 4 * nq + 80;
  const int total = a.layers * spl;

  if (wave < LW) {
    // =================== loader (pse.hip's register-staged loader) ===================
    u32x4 bA[SLOT_KB], bB[SLOT_KB], bC[SLOT_KB];
    bool dead = false;
    const uint32_t voff = (uint32_t)lane * 16u;
    typedef __attribute__((address_space(3))) void lvoid;
    const uint32_t ring0 = (uint32_t)(uintptr_t)(lvoid*)(lds + L_RING) + voff;
    auto src_of = [&](int s0) -> const void* {
      const int s = min(s0, total - 1);
      if (a.trace && lane == 0 && s0 < total) {
        const int l = s / spl, r = s - l * spl, rq = 4 * nq;
        const int ev = r == 0 ? 12 : (r == rq ? 13 : (r == rq + 8 ? 14 : (r == rq + 56 ? 15 : -1)));
        if (ev >= 0) a.trace[((size_t)l * PSE_TRACE_EV + ev) * 256 + c] = __builtin_amdgcn_s_memrealtime();
      }
      if (s0 < total)  // this CU's attention is gathering its inputs: no new loads
        for (uint32_t spins = 0; __hip_atomic_load(&ctl->apause, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                                 !__hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) &&
                                 spins < SPIN_LDS;
             ++spins)
          __builtin_amdgcn_s_sleep(1);
      const uint64_t p = (uint64_t)(uintptr_t)slot_src(wp, c, nq, s);
      const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)p), hi = __builtin_amdgcn_readfirstlane((uint32_t)(p >> 32));
      return (const void*)(((uint64_t)hi << 32) | lo);
    };
#define P4_RL_OPS                                                                                   \
  [b0] "+v"(b[0]), [b1] "+v"(b[1]), [b2] "+v"(b[2]), [b3] "+v"(b[3]), [b4] "+v"(b[4]), [b5] "+v"(b[5]), \
      [b6] "+v"(b[6]), [b7] "+v"(b[7]), [b8] "+v"(b[8]), [b9] "+v"(b[9]), [b10] "+v"(b[10]),          \
      [b11] "+v"(b[11]), [b12] "+v"(b[12]), [b13] "+v"(b[13]), [b14] "+v"(b[14]), [b15] "+v"(b[15])
// (s_nop 4: the base SGPRs come fresh from v_readfirstlane -- pse.hip PSE_RL_LOADS)
#define P4_RL_LOADS                                                                                 \
  "s_nop 4\n\t"                                                                                    \
  "global_load_dwordx4 %[b0], %[o0], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b1], %[o0], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b2], %[o0], %[g] offset:2048 nt\n\t"                                     \
  "global_load_dwordx4 %[b3], %[o0], %[g] offset:3072 nt\n\t"                                     \
  "global_load_dwordx4 %[b4], %[o1], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b5], %[o1], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b6], %[o1], %[g] offset:2048 nt\n\t"                                     \
  "global_load_dwordx4 %[b7], %[o1], %[g] offset:3072 nt\n\t"                                     \
  "global_load_dwordx4 %[b8], %[o2], %[g] offset:0 nt\n\t"                                        \
  "global_load_dwordx4 %[b9], %[o2], %[g] offset:1024 nt\n\t"                                     \
  "global_load_dwordx4 %[b10], %[o2], %[g] offset:2048 nt\n\t"                                    \
  "global_load_dwordx4 %[b11], %[o2], %[g] offset:3072 nt\n\t"                                    \
  "global_load_dwordx4 %[b12], %[o3], %[g] offset:0 nt\n\t"                                       \
  "global_load_dwordx4 %[b13], %[o3], %[g] offset:1024 nt\n\t"                                    \
  "global_load_dwordx4 %[b14], %[o3], %[g] offset:2048 nt\n\t"                                    \
  "global_load_dwordx4 %[b15], %[o3], %[g] offset:3072 nt\n\t"
    auto load = [&](u32x4 (&b)[SLOT_KB], int s_issue) {
      const void* g = src_of(s_issue);
      asm volatile(P4_RL_LOADS
                   : P4_RL_OPS
                   : [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u), [o3] "v"(voff + 12288u)
                   : "memory");
    };
    auto copy_load = [&](u32x4 (&b)[SLOT_KB], int s, int s_issue) {
      if (s >= NS && !dead)
        for (uint32_t spins = 0;; ++spins) {
          int mn = 1 << 30;
#pragma unroll
          for (int w = 0; w < CW; ++w)
            mn = min(mn, __hip_atomic_load(&ctl->freed[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          if (mn >= s - NS + 1) break;
          if (spins > SPIN_LDS || __hip_atomic_load(&ctl->abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
            dead = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      const void* g = src_of(s_issue);
      const uint32_t dst = ring0 + (uint32_t)(s % NS) * (SLOT_KB * 1024u);
      asm volatile("s_waitcnt vmcnt(32)\n\t"
                   "ds_write_b128 %[d], %[b0] offset:0\n\t"
                   "ds_write_b128 %[d], %[b1] offset:1024\n\t"
                   "ds_write_b128 %[d], %[b2] offset:2048\n\t"
                   "ds_write_b128 %[d], %[b3] offset:3072\n\t"
                   "ds_write_b128 %[d], %[b4] offset:4096\n\t"
                   "ds_write_b128 %[d], %[b5] offset:5120\n\t"
                   "ds_write_b128 %[d], %[b6] offset:6144\n\t"
                   "ds_write_b128 %[d], %[b7] offset:7168\n\t"
                   "ds_write_b128 %[d], %[b8] offset:8192\n\t"
                   "ds_write_b128 %[d], %[b9] offset:9216\n\t"
                   "ds_write_b128 %[d], %[b10] offset:10240\n\t"
                   "ds_write_b128 %[d], %[b11] offset:11264\n\t"
                   "ds_write_b128 %[d], %[b12] offset:12288\n\t"
                   "ds_write_b128 %[d], %[b13] offset:13312\n\t"
                   "ds_write_b128 %[d], %[b14] offset:14336\n\t"
                   "ds_write_b128 %[d], %[b15] offset:15360\n\t"
                   "s_waitcnt lgkmcnt(0)\n\t" P4_RL_LOADS
                   : P4_RL_OPS
                   : [d] "v"(dst), [g] "s"(g), [o0] "v"(voff), [o1] "v"(voff + 4096u), [o2] "v"(voff + 8192u),
                     [o3] "v"(voff + 12288u)
                   : "memory");
      if (!dead && s < total) __hip_atomic_store(&ctl->full, s + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    load(bA, 0);
    load(bB, 1);
    load(bC, 2);
    for (int s = 0; s < total && !dead; s += 3) {
      copy_load(bA, s, s + 3);
      if (s + 1 >= total) break;
      copy_load(bB, s + 1, s + 4);
      if (s + 2 >= total) break;
      copy_load(bC, s + 2, s + 5);
    }
    {
      u32x4(&b)[SLOT_KB] = bA;
      asm volatile("s_waitcnt vmcnt(0)" : P4_RL_OPS::"memory");
    }
    {
      u32x4(&b)[SLOT_KB] = bB;
      asm volatile("" : P4_RL_OPS::"memory");
    }
    {
      u32x4(&b)[SLOT_KB] = bC;
      asm volatile("" : P4_RL_OPS::"memory");
    }
#undef P4_RL_OPS
#undef P4_RL_LOADS
    if (dead) st32(a.err, 1u);
    __hip_atomic_store(&ctl->full, dead ? 0 : total, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  } else {
    // =================== consumers ===================
    Ctx x{a.err, a.eps, c, lane, wave, (wave - LW) * 64 + lane, epoch, 0};
    uint32_t* xa32 = reinterpret_cast<uint32_t*>(lds + L_XA);
    uint32_t* xb32 = reinterpret_cast<uint32_t*>(lds + L_XB);
    uint32_t* ss32 = reinterpret_cast<uint32_t*>(lds + L_MISC);
    constexpr int NT = H_ / 16;
    const int att_u = pse4_att_unit(c, P);
    auto run = [&](auto att_c) __attribute__((always_inline)) {
      constexpr bool ATT = decltype(att_c)::value;
      // residual columns 16c .. 16c+15 of the 4 rows: wave 1, lane l = (row l >> 4, column l & 15)
      const int ecol = lane >> 4, erow = lane & 15;
      float hres = wave == LW ? bf2f(a.h[(size_t)ecol * H_ + c * 16 + erow]) : 0.f;
      float hsq = 0.f;
      int seq = 0;
      // hidden = residual + bf16(o) (TF/.../modeling_qwen3.py:311,322), published with each row's
      // sum of squares over the 16 columns in column order
      auto emit_h = [&](uint64_t* gh, uint32_t t, float o, int k) {
        if (wave != LW) return;
        const float hv = rbf(hres + rbf(o));
        hres = hv;
        const float sq = hv * hv;
        float s16 = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) s16 += __shfl(sq, (lane & 48) + i, 64);
        hsq = s16;
        const float hn = __shfl_down(hv, 1, 64);
        if constexpr (PSE4_HCNT) {
          // rows bf16 [4][H] over the granule region's first 32 KiB, sums of squares fp32 [4][256] behind
          // them; drained, then one arrival
          bf16_t* hb = reinterpret_cast<bf16_t*>(gh);
          float* hs = reinterpret_cast<float*>(gh + NG_H);
          if ((erow & 1) == 0) st32(hb + (size_t)ecol * H_ + c * 16 + erow, pack2(hv, hn));
          if (erow == 0) st32(hs + ecol * NT + c, __float_as_uint(s16));
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          harrive(x, a.hcnt, a.go, k, 256);
        } else {
          if ((erow & 1) == 0) st64(gh + xword(ecol, c * 16 + erow), gran(pack2(hv, hn), t));
          if (erow == 0) st64(gh + NG_H + ecol * NT + c, gran(__float_as_uint(s16), t));
        }
      };
      for (int l = 0; l < a.layers && !failed(x); ++l) {
        const PseLayer& Lw = a.L[l];
        constexpr int RC = ATT ? 0 : PSE4_RC;
        NormW nw;
        if (wave == LW) P4_STAMP(l, 0);
        // ---------------- q|k|v (input RMSNorm fused) ----------------
        if (l == 0) {  // the embedding rows and their sums of squares (previous launch)
          nw = norm_w(x, Lw.in_norm);
          for (int i = x.tid; i < NB * H_ / 2; i += CW * 64) {
            const int b = i / (H_ / 2), k = (i - b * (H_ / 2)) * 2;
            xa32[xword(b, k)] = reinterpret_cast<const uint32_t*>(a.h)[i];
          }
          for (int i = x.tid; i < NB * NT; i += CW * 64) ss32[i] = __float_as_uint(a.ss[i]);
          cbar(x);
        } else if (PSE4_HCNT) {
          if (!hgather(x, a.hcnt, a.go, (l - 1) * 2 + 1, 256, reinterpret_cast<const bf16_t*>(a.g_h[1]),
                       reinterpret_cast<const float*>(a.g_h[1] + NG_H), xa32, ss32, [&]() { nw = norm_w(x, Lw.in_norm); }))
            break;
        } else if (!gather<36>(x, a.g_h[1], NG_H + NG_SS, tagof(epoch, l - 1, OP_DOWN), xa32, NG_H, ss32,
                               [&]() { nw = norm_w(x, Lw.in_norm); })) {
          break;
        }
        norm_stage(x, nw);
        if (wave == LW) P4_STAMP(l, 1);
        const uint32_t tq = tagof(epoch, l, OP_QKV);
#pragma unroll 1
        for (int j = 0; j < (ATT ? 2 : nq); ++j) {
          int tile, half;
          qkv_unit(c, j, &tile, &half);
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
          for (int k = 0; k < 4; ++k) consume_slot(x, seq++, L_XA, half * 64 + k * 16, acc);
          __builtin_amdgcn_s_setprio(3);
          red_put(x, 0, acc);
          cbar(x);
          if (wave == LW)
            st64(a.g_qkv + (size_t)ecol * NG_QKV_ROW + qkv_gran(tile) + half * 16 + erow,
                 gran(__float_as_uint(red_get(0, ecol, erow)), tq));
          cbar(x);
          __builtin_amdgcn_s_setprio(0);
        }
        if (wave == LW) P4_STAMP(l, 2);
        // ---------------- attention (32 units: one per row and KV head) ----------------
        if constexpr (ATT) {
          auto att = [&](auto ku_c) {
            return attention<decltype(ku_c)::value>(a.L + l, a.pos, a.mask, a.cos_t, a.sin_t, a.g_qkv, a.g_att, a.g_part,
                                                    a.hcnt, a.go, a.err, a.trace, a.eps, a.scale, a.Cmax, epoch, x.bar_gen,
                                                    l, att_u, tq);
          };
          // (key split: role 0 = unit 0 of its (row, KV head), 1 = its partner; PSE4_KS 1: role 0 only)
          const int bg = att_u % PSE4_KS == 0 ? att(IntC4<0>{}) : att(IntC4<1>{});
          const bool att_ok = bg >= 0;
          if (att_ok) x.bar_gen = bg;
          if (x.tid == 0) __hip_atomic_store(&P4_CTL->apause, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (!att_ok) break;
          if (wave == LW) P4_STAMP(l, 3);
        }
        // ---------------- o_proj (+ residual) ----------------
        constexpr int LC = ATT ? 0 : PSE4_LC;
        SlotCache<RC, LC> co;
        if (P4_AFLAG) {
          if (!hgather(x, a.hcnt, a.go, 2 * PSE_MAXL + l, HKV_ * NB, reinterpret_cast<const bf16_t*>(a.g_att), nullptr, xa32,
                       nullptr, NoHook(), [&]() { co.drain(x, seq); }))
            break;
        } else if (!gather<32>(x, a.g_att, NG_ATT, tagof(epoch, l, OP_ATT), xa32, NG_ATT, nullptr, NoHook(),
                               [&]() { co.drain(x, seq); })) {
          break;
        }
        if (wave == LW) P4_STAMP(l, 4);
        {
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int k = 0; k < RC; ++k) co.take(x, seq, k, L_XA, k * 16, acc);
#pragma unroll
          for (int k = RC; k < RC + LC; ++k) co.take_lds(x, seq, k, L_XA, k * 16, acc);
#pragma unroll 1
          for (int k = RC + LC; k < 8; ++k) consume_slot(x, seq++, L_XA, k * 16, acc);
          __builtin_amdgcn_s_setprio(3);
          red_put(x, 0, acc);
          cbar(x);
          emit_h(a.g_h[0], tagof(epoch, l, OP_O), red_get(0, ecol, erow), l * 2);
          cbar(x);
          __builtin_amdgcn_s_setprio(0);
        }
        if (wave == LW) P4_STAMP(l, 5);
        // ---------------- gate|up (post-attention RMSNorm fused, SwiGLU) ----------------
        if (PSE4_HCNT) {
          if (!hgather(x, a.hcnt, a.go, l * 2, 256, reinterpret_cast<const bf16_t*>(a.g_h[0]),
                       reinterpret_cast<const float*>(a.g_h[0] + NG_H), xa32, ss32, [&]() { nw = norm_w(x, Lw.post_norm); }))
            break;
        } else if (!gather<36>(x, a.g_h[0], NG_H + NG_SS, tagof(epoch, l, OP_O), xa32, NG_H, ss32,
                               [&]() { nw = norm_w(x, Lw.post_norm); })) {
          break;
        }
        norm_stage(x, nw);
        if (wave == LW) P4_STAMP(l, 6);
        const uint32_t tg = tagof(epoch, l, OP_GU);
        auto gu_round = [&](int j) {
          f32x4 ag = (f32x4){0.f, 0.f, 0.f, 0.f}, au = ag;
#pragma unroll 1
          for (int k = 0; k < 8; ++k) consume_slot(x, seq++, L_XA, k * 16, ag);
#pragma unroll 1
          for (int k = 0; k < 8; ++k) consume_slot(x, seq++, L_XA, k * 16, au);
          __builtin_amdgcn_s_setprio(3);
          red_put(x, 0, ag);
          red_put(x, 1, au);
          cbar(x);
          if (wave == LW) {
            // bf16(bf16(silu(bf16 g)) * bf16 u)   (TF/.../modeling_qwen3.py:81-83)
            const float gg = rbf(red_get(0, ecol, erow)), uu = rbf(red_get(1, ecol, erow));
            const float o = rbf(rbf(gg / (1.0f + expf(-gg))) * uu);
            const float on = __shfl_down(o, 1, 64);
            if ((erow & 1) == 0) st64(a.g_act + xword(ecol, gu_pair(c, j) * 16 + erow), gran(pack2(o, on), tg));
          }
          cbar(x);
          __builtin_amdgcn_s_setprio(0);
        };
        gu_round(0);
        gu_round(1);
        if (wave == LW) P4_STAMP(l, 7);
        // round 0's columns -> region B while round 2 runs on region A's normed input
        if (!gather<32>(x, a.g_act, NG_ACT_ROUND, tg, xb32, NG_ACT_ROUND, nullptr, [&]() {
              __builtin_amdgcn_s_setprio(0);
              gu_round(2);
              __builtin_amdgcn_s_setprio(3);
            }))
          break;
        if (wave == LW) P4_STAMP(l, 8);
        // ---------------- down (+ residual) ----------------
        {
          f32x4 acc = (f32x4){0.f, 0.f, 0.f, 0.f};
          auto slots = [&](int k0, int reg) {
            __builtin_amdgcn_s_setprio(0);
#pragma unroll 1
            for (int k = k0; k < k0 + 8; ++k) consume_slot(x, seq++, reg, (k - k0) * 16, acc);
            __builtin_amdgcn_s_setprio(3);
          };
          // round 1 -> region A (its normed input is dead) while slots 0-7 read round 0 in B;
          // round 2 -> region B while slots 8-15 read round 1 in A; slots 16-23 then read B
          if (!gather<32>(x, a.g_act + NG_ACT_ROUND, NG_ACT_ROUND, tg, xa32, NG_ACT_ROUND, nullptr,
                          [&]() { slots(0, L_XB); }))
            break;
          if (wave == LW) P4_STAMP(l, 9);
          if (!gather<32>(x, a.g_act + 2 * NG_ACT_ROUND, NG_ACT_ROUND, tg, xb32, NG_ACT_ROUND, nullptr,
                          [&]() { slots(8, L_XA); }))
            break;
          if (wave == LW) P4_STAMP(l, 10);
#pragma unroll 1
          for (int k = 16; k < 24; ++k) consume_slot(x, seq++, L_XB, (k - 16) * 16, acc);
          __builtin_amdgcn_s_setprio(3);
          red_put(x, 0, acc);
          cbar(x);
          emit_h(a.g_h[1], tagof(epoch, l, OP_DOWN), red_get(0, ecol, erow), l * 2 + 1);
          cbar(x);
          __builtin_amdgcn_s_setprio(0);
        }
        if (wave == LW) P4_STAMP(l, 11);
      }
      // the final residual rows and their sums of squares for the heads (plain stores: the next launch)
      if (wave == LW) a.h[(size_t)ecol * H_ + c * 16 + erow] = f2bf(hres);
      if (wave == LW && erow == 0) a.ss[(size_t)ecol * NT + c] = hsq;
    };
    if (att_u >= 0) run(BoolC4<true>{});
    else run(BoolC4<false>{});
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add((g32*)a.exit_cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (uint32_t)P - 1) {
      if (PSE4_HCNT) {
        for (int k = 0; k < 2 * a.layers; ++k) st32(a.hcnt + k, 0u);
        for (int k = 0; k < a.layers; ++k) st32(a.hcnt + 2 * PSE_MAXL + k, 0u);
        for (int k = 0; k < 2 * a.layers * HGRP; ++k) st32(a.hcnt + 3 * PSE_MAXL + (size_t)k * GCNT_STRIDE, 0u);
      }
      st32(a.exit_cnt, 0u);
      st32(a.epoch, epoch);
    }
  }
}

// ---------------------------------------------------------------------------
size_t pse4_lds_bytes() { return (size_t)L_END; }

bool pse4_supported(int device, int layers, int H, int Hq, int Hkv, int D, int I, int qkv_rows, int Cmax) {
  if (H != H_ || Hq != HQ_ || Hkv != HKV_ || D != D_ || I != I_ || qkv_rows != QKVR_ || Cmax % 64) return false;
  if (layers < 1 || layers > PSE_MAXL || layers * 5 > 256) return false;
  hipDeviceProp_t p;
  if (hipGetDeviceProperties(&p, device) != hipSuccess || p.multiProcessorCount != 256) return false;
  if (hipFuncSetAttribute((const void*)pse4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)pse4_lds_bytes()) !=
      hipSuccess)
    return false;
  int per_cu = 0;
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)pse4_kernel, THREADS, pse4_lds_bytes()) ==
             hipSuccess &&
         per_cu >= 1;
}

// counters: [3 PSE_MAXL] hand-off counters, then the group counters of the residual hand-offs
// [2 PSE_MAXL][HGRP] one 128-byte line each (PSE4_HTREE), then the release flags
constexpr size_t HCNT_BYTES = ((size_t)3 * PSE_MAXL + (size_t)2 * PSE_MAXL * HGRP * GCNT_STRIDE) * 4;
size_t pse4_ws_bytes() {
  return (size_t)(NB * NG_QKV_ROW + NG_ATT + 2 * (NG_H + NG_SS) + NG_ACT + NB * HKV_ * KS_N) * 8 + HCNT_BYTES +
         (PSE4_HCNT == 2 ? (size_t)3 * PSE_MAXL * 256 * 128 : 0) + 64;
}

hipError_t pse4_decode(const PseArgs& a0, void* ws, hipStream_t s, bool coop) {
  if (a0.layers < 1 || a0.layers > PSE_MAXL || a0.layers * 5 > 256 || a0.Cmax % 64) return hipErrorInvalidValue;
  PseArgs a = a0;
  uint64_t* g = reinterpret_cast<uint64_t*>(ws);
  a.g_qkv = g; g += NB * NG_QKV_ROW;
  a.g_att = g; g += NG_ATT;
  a.g_h[0] = g; g += NG_H + NG_SS;  // h granules, then its sums of squares: one gather range
  a.g_ss[0] = a.g_h[0] + NG_H;
  a.g_h[1] = g; g += NG_H + NG_SS;
  a.g_ss[1] = a.g_h[1] + NG_H;
  a.g_act = g; g += NG_ACT;
  a.g_part = g; g += NB * HKV_ * KS_N;  // (PSE4_KS 2) the partner parts
  a.hcnt = reinterpret_cast<int*>(g);
  a.go = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(g) + HCNT_BYTES);
  uint32_t* w = reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ws) + pse4_ws_bytes() - 64);
  a.err = w; a.epoch = w + 1; a.exit_cnt = w + 2;
  if (coop) {
    void* args[] = {&a};
    return hipLaunchCooperativeKernel((const void*)pse4_kernel, dim3(256), dim3(THREADS), args, (unsigned)pse4_lds_bytes(), s);
  }
  hipLaunchKernelGGL(pse4_kernel, dim3(256), dim3(THREADS), pse4_lds_bytes(), s, a);
  return hipGetLastError();
}

uint32_t* pse4_err_word(void* ws) {
  return reinterpret_cast<uint32_t*>(reinterpret_cast<unsigned char*>(ws) + pse4_ws_bytes() - 64);
}

}  // namespace mtts
