// One wave's 32-key chunk of the persistent launches' decode attention (pse.hip attention() /
// attention_slice(), pse4.hip attention()): S = K q^T on the MFMA, masked online softmax, P.V
// accumulated into the running output.  Reference semantics: TF/integrations/sdpa_attention.py:79-166
// (softmax over the cached keys 0 .. pos-1 whose mask byte is set; the new key joins in the caller's
// merge).
//
// Register shape: K tiles kt[2][QS] (MFMA A operands, key = c16 of tile t), V^T fragments vt[DT] (B
// operands, 8 keys per lane), q rows from LDS (q_s [16][D], rows >= HU zero).  The running output of
// the HU real q rows lives in LDS (o_s: this wave's rows of acc_s, [HU][D]; lanes g4 == 0 own them)
// rather than in DT x HU VGPRs: the attention bodies are noinline callees, and every VGPR past v39
// they touch at their peak is a callee-saved stripe written to scratch and read back per call, on
// every CU and layer.  p is taken against the running max mn, so the MFMA accumulates straight into
// the rescaled output (o = alpha o + P.V, no per-tile temporaries).
#pragma once
#include "common.h"

namespace mtts {

template <int HU, int D, int KW = 32>
__device__ __forceinline__ void pse_chunk_step(int k0, int pos, int g4, int c16, u32x4 (&kt)[2][D / 32],
                                               u32x4 (&vt)[D / 16], const uint32_t (&mk)[2], const bf16_t* q_s,
                                               bf16_t* p_w, float* o_s, float scale, float& m_run, float& l_run) {
  constexpr int QS = D / 32, DT = D / 16;
  {
    // the V^T fragment holding pos also read keys pos .. kb+7: cache rows never written (or stale
    // after a capacity change).  Their p is 0, but 0 * NaN / Inf in the P.V MFMA is NaN: zero those
    // 16-bit lanes (as attn_body.h's per-op attention does)
    const int nv = pos - (k0 + 8 * g4);
    uint32_t vm[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vm[q] = (2 * q < nv ? 0x0000ffffu : 0u) | (2 * q + 1 < nv ? 0xffff0000u : 0u);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int q = 0; q < 4; ++q) vt[dt][q] &= vm[q];
  }
  f32x4 sacc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    sacc[t] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s2 = 0; s2 < QS; ++s2)
      sacc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kt[t][s2]),
                                                       *reinterpret_cast<const bf16x8*>(&q_s[c16 * D + s2 * 32 + 8 * g4]),
                                                       sacc[t], 0, 0, 0);
  }
  // lane (g4, c16): q row c16, keys k0 + 16 t + 4 g4 + r
  float sv[2][4], mc = -INFINITY;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int key = k0 + t * 16 + g4 * 4 + r;
      const bool valid = key < pos && ((mk[t] >> (8 * r)) & 0xffu);
      sv[t][r] = valid ? sacc[t][r] * scale : -INFINITY;
      mc = fmaxf(mc, sv[t][r]);
    }
  mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
  mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
  const float mn = fmaxf(m_run, mc);
  const float alpha = (m_run == -INFINITY) ? 0.f : expf(m_run - mn);
  float lc = 0.f;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float pr4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float p = (mn == -INFINITY || sv[t][r] == -INFINITY) ? 0.f : expf(sv[t][r] - mn);
      lc += p;
      pr4[r] = p;
    }
    uint2 pk;
    pk.x = pack2(pr4[0], pr4[1]);
    pk.y = pack2(pr4[2], pr4[3]);
    *reinterpret_cast<uint2*>(&p_w[c16 * KW + t * 16 + g4 * 4]) = pk;
  }
  lc += __shfl_xor(lc, 16, 64);
  lc += __shfl_xor(lc, 32, 64);
  l_run = l_run * alpha + lc;
  m_run = mn;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  // P as the A operand (row = q row c16, keys 8 g4 ..), V^T as B: D rows 4 g4 + r = q rows, so the
  // HU real rows sit in lanes g4 == 0
  const bf16x8 pf = *reinterpret_cast<const bf16x8*>(&p_w[c16 * KW + 8 * g4]);
  float al[HU];
#pragma unroll
  for (int r = 0; r < HU; ++r) al[r] = __shfl(alpha, r, 64);
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) {
    f32x4 o4 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < HU; ++r) o4[r] = o_s[r * D + dt * 16] * al[r];
    o4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, __builtin_bit_cast(bf16x8, vt[dt]), o4, 0, 0, 0);
    if (g4 == 0)
#pragma unroll
      for (int r = 0; r < HU; ++r) o_s[r * D + dt * 16] = o4[r];
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// zero this wave's running output rows (lanes g4 == 0 own them)
template <int HU, int D>
__device__ __forceinline__ void pse_chunk_init(int g4, float* o_s) {
  if (g4 == 0)
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
      for (int r = 0; r < HU; ++r) o_s[r * D + dt * 16] = 0.f;
}

}  // namespace mtts
