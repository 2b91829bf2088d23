// q/k RMSNorm + RoPE + KV-cache append of one (token, head) item at D = 128, shared by the q|k|v
// prefill path's per-item kernel (norm_rope.hip) and the split-K q|k|v reduce (gemm.hip).
// TF/models/qwen3/modeling_qwen3.py:252-254 (q_norm / k_norm), :148-170 (RoPE in bf16),
// TF/cache_utils.py:127-145 (the cache append, in place at the token's position).
#pragma once
#include "kernels.h"

namespace mtts {

// one (token m, head hd) item of 16 lanes (l16: dims 8 l16 .. 8 l16 + 7, x its bf16 q|k|v values):
// q / k heads normed, rotated and stored (q_out / K cache), V heads into the transposed cache.
// No FMA contraction (the file including it may allow it): both callers give identical bits.
__device__ __forceinline__ void qk_item_d128(const QKRopeArgs& a, int m, int hd, int l16, const float (&x)[8], bool live) {
#pragma clang fp contract(off)
  constexpr int D = 128;
  const int b = m / a.S, s = m % a.S;
  const int pos = *a.pos_base + s;
  const int rpos = a.rope_off ? max(0, pos - a.rope_off[b]) : pos;
  if (hd >= a.Hq + a.Hkv) {  // V head (short prompts): into the transposed cache
    if (!live) return;
    bf16_t* dst = a.vc + ((size_t)b * a.Hkv + (hd - a.Hq - a.Hkv)) * D * a.Cmax + pos;
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[(size_t)(8 * l16 + i) * a.Cmax] = f2bf(x[i]);
    return;
  }
  const bool isq = hd < a.Hq;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) ss += x[i] * x[i];
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) ss += __shfl_xor(ss, o, 64);
  const float r = 1.0f / sqrtf(ss / (float)D + a.eps);
  float w[8], c[8], sn[8], n[8];
  unpack8(*reinterpret_cast<const uint4*>((isq ? a.qn_w : a.kn_w) + 8 * l16), w);
  unpack8(*reinterpret_cast<const uint4*>(a.cos_t + (size_t)rpos * D + 8 * l16), c);
  unpack8(*reinterpret_cast<const uint4*>(a.sin_t + (size_t)rpos * D + 8 * l16), sn);
#pragma unroll
  for (int i = 0; i < 8; ++i) n[i] = rbf(w[i] * rbf(x[i] * r));
  uint4 nq;
  nq.x = pack2(n[0], n[1]); nq.y = pack2(n[2], n[3]); nq.z = pack2(n[4], n[5]); nq.w = pack2(n[6], n[7]);
  uint4 pq;
  pq.x = __shfl_xor(nq.x, 8, 64); pq.y = __shfl_xor(nq.y, 8, 64);
  pq.z = __shfl_xor(nq.z, 8, 64); pq.w = __shfl_xor(nq.w, 8, 64);
  float p[8];
  unpack8(pq, p);
  const float sg = l16 < 8 ? -1.f : 1.f;
  float o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = rbf(rbf(n[i] * c[i]) + rbf(sg * p[i] * sn[i]));
  if (!live) return;
  uint4 ov;
  ov.x = pack2(o[0], o[1]); ov.y = pack2(o[2], o[3]); ov.z = pack2(o[4], o[5]); ov.w = pack2(o[6], o[7]);
  bf16_t* dst = isq ? a.q_out + (size_t)m * a.Hq * D + (size_t)hd * D
                    : a.kc + (((size_t)b * a.Hkv + (hd - a.Hq)) * a.Cmax + pos) * D;
  *reinterpret_cast<uint4*>(dst + 8 * l16) = ov;
}

}  // namespace mtts
