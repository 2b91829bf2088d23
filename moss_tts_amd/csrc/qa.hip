// One launch for a decoder layer's q|k|v projection (input RMSNorm fused) and its decode
// attention (B <= QA_MAXB rows, one new token each):
//   TF/models/qwen3/modeling_qwen3.py:59-64 input_layernorm, :252-254 q/k/v_proj + q/k_norm,
//   :148-170 RoPE, TF/cache_utils.py:127-145 cache append, TF/integrations/sdpa_attention.py.
//
//   workgroups [0, n_gemv) are the q|k|v GEMV's 16-row output tiles (gemv_body, PRO_NORM,
//   EPI_STORE, write-through stores); each drains and counts itself into an XCD-sharded counter.
//   Workgroups >= n_gemv are attention units (split, KV head, row): they issue their K / V^T /
//   mask loads at once -- those do not depend on the projection -- then wait for every GEMV
//   tile (relaxed polls, one agent-scope acquire) and run attn_decode_body from the prologue on,
//   publishing (m, l, o) partials for the o_proj GEMV's prologue (publish-only, as attn_decode).
// Roles by blockIdx, the waiting units last: the host launches this only when the whole grid
// is co-resident (qkv_attn_supported), and every wait is bounded (error word, no hang).
// Per-block role tickets were tried first: ~1,200 same-address atomics per launch serialise
// at ~12 ns each (MI355X_MICROARCH.md fanin) and cost more than the fusion saves.
// What the fusion removes from the chain: the attention launch's dependent-launch boundary and
// grid fill, and the latency of its K / V reads (hidden under the weight stream).  The last
// attention unit to leave resets the counters (graph replay).
#include "attn_body.h"
#include "gemv_body.h"

namespace mtts {

namespace {
constexpr int QA_NW = 8;  // waves per workgroup for both roles (GEMV K split 8 ways; attention 8 x 32 keys)
}

template <int G, int D>
__global__ __launch_bounds__(QA_NW * 64) void qkv_attn_kernel(GemvArgs gq, DecAttnArgs da, int* sync, int n_gemv,
                                                              int n_att) {
  const int t = threadIdx.x, bid = blockIdx.x;
  if (bid < n_gemv) {
    // write-through (sc1) output stores, drained, then a relaxed count into this block's XCD
    // shard (bid % 8): no per-block release fence (an agent-scope release writes back the
    // XCD's L2) and no single hot counter (~12 ns per same-address atomic, serialised)
    gemv_body<1, 1, EPI_STORE, PRO_NORM, QA_NW, false, NoWait, true>(gq, bid, NoWait{});
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) __hip_atomic_fetch_add(&sync[bid & 7], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  auto wait = [&] {
    if (t == 0) {
      for (int spins = 0;; ++spins) {
        bool done = true;
#pragma unroll
        for (int x = 0; x < 8; ++x)
          done = done && __hip_atomic_load(&sync[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (n_gemv - x + 7) / 8;
        if (done) break;
        if (spins > (1 << 22)) {  // bounded: report a stuck producer instead of hanging
          sync[9] = 1;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  };
  const int u = bid - n_gemv;
  const int sp = u % da.ns, rest = u / da.ns;
  attn_decode_body<G, D, QA_NW, false>(da, sp, rest % da.Hkv, rest / da.Hkv, wait);
  __syncthreads();
  if (t == 0) {
    // the last attention block resets the counters for the next launch: every GEMV block has
    // counted (all attention blocks that waited saw it) and every waiting block is past its wait
    const int done = __hip_atomic_fetch_add(&sync[8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (done == n_att - 1)
      for (int x = 0; x < 9; ++x) __hip_atomic_store(&sync[x], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

bool qkv_attn_supported(const GemvArgs& g, const DecAttnArgs& da, int B) {
  const int G = da.Hkv > 0 ? da.Hq / da.Hkv : 0;
  // co-residency of the whole grid (the attention units spin): at most 2 workgroups per CU
  // (LDS, registers) on 256 CUs, with margin
  const int n_blocks = g.N / 16 + attn_decode_splits(da.Cmax) * (da.Hkv > 0 ? da.Hkv : 1) * B;
  return n_blocks <= 448 && B >= 1 && B <= QA_MAXB && g.ss_in && g.B == B && g.K % 32 == 0 && g.N % 16 == 0 && da.Hq % da.Hkv == 0 &&
         (G == 1 || G == 2 || G == 4 || G == 8) && (da.D == 128 || da.D == 64) && da.Cmax % 64 == 0 &&
         norm_lds_bytes(B, g.K) <= NORM_LDS_MAX && attn_decode_keys_per_block() == QA_NW * DEC_KW &&
         attn_decode_splits(da.Cmax) <= DEC_MAXS;
}

template <int D>
static hipError_t qa_launch(const GemvArgs& g, const DecAttnArgs& da, int* sync, int n_gemv, int n_att, int G,
                            hipStream_t s) {
  const size_t lds = norm_lds_bytes(g.B, g.K);
  const dim3 grid(n_gemv + n_att), blk(QA_NW * 64);
  switch (G) {
    case 1: hipLaunchKernelGGL((qkv_attn_kernel<1, D>), grid, blk, lds, s, g, da, sync, n_gemv, n_att); break;
    case 2: hipLaunchKernelGGL((qkv_attn_kernel<2, D>), grid, blk, lds, s, g, da, sync, n_gemv, n_att); break;
    case 4: hipLaunchKernelGGL((qkv_attn_kernel<4, D>), grid, blk, lds, s, g, da, sync, n_gemv, n_att); break;
    case 8: hipLaunchKernelGGL((qkv_attn_kernel<8, D>), grid, blk, lds, s, g, da, sync, n_gemv, n_att); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t qkv_attn(const GemvArgs& g0, const DecAttnArgs& da0, int* sync, int B, hipStream_t s) {
  if (!sync || !qkv_attn_supported(g0, da0, B)) return hipErrorInvalidValue;
  GemvArgs g = g0;
  g.KT = g.K / 32;
  g.pad_period = 1;
  g.tile0 = 0;
  g.gate = nullptr;
  DecAttnArgs da = da0;
  // the same split geometry as attn_decode's publish-only form (the o_proj prologue's view)
  da.nwv = QA_NW;
  da.ns = attn_decode_splits(da.Cmax);
  da.publish_only = 1;
  da.po_max = ATTN_PO_ALL;  // the o_proj GEMV merges every split (engine: g.attn.po_max)
  da.probe = 0;
  const int n_gemv = g.N / 16;
  const int n_att = da.ns * da.Hkv * B;
  const int G = da.Hq / da.Hkv;
  return da.D == 128 ? qa_launch<128>(g, da, sync, n_gemv, n_att, G, s) : qa_launch<64>(g, da, sync, n_gemv, n_att, G, s);
}

}  // namespace mtts
