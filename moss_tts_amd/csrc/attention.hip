// KV-cached grouped-query attention (decode and prefill), split over the context.
//
// Replaces sdpa_attention_forward (TF/integrations/sdpa_attention.py:79-166) with the
// causal + padding mask of TF/masking_utils.py: query token at absolute position p
// attends key j iff j <= p and mask[b][j].  Scores and softmax statistics are fp32;
// the un-normalised probabilities exp(s - max) are rounded to bf16 before P.V, as the
// reference's flash kernels do for bf16 (oracle/moss_delay.py attention()).
//
// Grid (n_split, Hkv, M): one block = one context chunk of CH keys for the G = Hq/Hkv
// query heads sharing one KV head (GQA), so each K/V row is read once per token.
// K/V rows (D*2 bytes) are read as 16-byte lane chunks, LPK = D/8 lanes per key.
// Partials (max, sum, unnormalised o) go to a workspace; attn_combine merges them.
#include "kernels.h"

namespace mtts {


template <int G>
__global__ __launch_bounds__(256) void attn_kernel(AttnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int split = blockIdx.x, kvh = blockIdx.y, m = blockIdx.z;
  const int b = m / a.S, s = m % a.S;
  const int pos = *a.pos_base + s;
  const int ctx = pos + 1;
  const int c0 = split * a.CH;
  if (c0 >= ctx) return;
  const int c1 = min(ctx, c0 + a.CH);
  const int n = c1 - c0;
  const int D = a.D;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float* q_s = smem;                 // [G][D]
  float* s_s = q_s + G * D;          // [G][CH]
  float* ml_s = s_s + G * a.CH;      // [G][2]
  float* red = smem + ((G * D + G * a.CH + 2 * G + 2 + 3) & ~3);  // [slots][G*D], 16B aligned (attn_smem_bytes)

  // q for the G heads of this KV head
  for (int e = t; e < G * D; e += 256) {
    const int h = e / D, d = e % D;
    q_s[e] = bf2f(a.q[(size_t)m * a.Hq * D + (size_t)(kvh * G + h) * D + d]);
  }
  __syncthreads();

  const int LPK = D >> 3;        // lanes per key
  const int KPW = 64 / LPK;      // keys per wave pass
  const int dl = (lane % LPK) * 8;
  const bf16_t* kbase = a.kc + ((size_t)b * a.Hkv + kvh) * a.Cmax * D;
  const bf16_t* vbase = a.vc + ((size_t)b * a.Hkv + kvh) * a.Cmax * D;
  const uint8_t* mrow = a.mask + (size_t)b * a.Cmax;
  for (int kb = c0 + wave * KPW; kb < c1; kb += 4 * KPW) {
    const int key = kb + lane / LPK;
    const bool inr = key < c1;
    float kv[8];
    if (inr) unpack8(*reinterpret_cast<const uint4*>(kbase + (size_t)key * D + dl), kv);
    else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kv[i] = 0.f;
    }
    const bool valid = inr && mrow[key];
#pragma unroll
    for (int h = 0; h < G; ++h) {
      float pd = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) pd += q_s[h * D + dl + i] * kv[i];
      for (int o = 1; o < LPK; o <<= 1) pd += __shfl_xor(pd, o, 64);
      if (inr && (lane % LPK) == 0) s_s[h * a.CH + (key - c0)] = valid ? pd * a.scale : -INFINITY;
    }
  }
  __syncthreads();

  // softmax statistics per head (one wave per head)
  for (int h = wave; h < G; h += 4) {
    float mx = -INFINITY;
    for (int i = lane; i < n; i += 64) mx = fmaxf(mx, s_s[h * a.CH + i]);
    mx = wave_max(mx);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = (mx == -INFINITY) ? 0.f : expf(s_s[h * a.CH + i] - mx);
      l += p;
      s_s[h * a.CH + i] = rbf(p);
    }
    l = wave_sum(l);
    if (lane == 0) {
      ml_s[2 * h] = mx;
      ml_s[2 * h + 1] = l;
    }
  }
  __syncthreads();

  // P.V: slot = key lane group, 8 dims per thread
  const int slots = 256 / LPK;
  const int slot = t / LPK;
  const int dd = (t % LPK) * 8;
  float acc[G][8];
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[h][i] = 0.f;
  for (int key = c0 + slot; key < c1; key += slots) {
    float vv[8];
    unpack8(*reinterpret_cast<const uint4*>(vbase + (size_t)key * D + dd), vv);
#pragma unroll
    for (int h = 0; h < G; ++h) {
      const float p = s_s[h * a.CH + (key - c0)];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[h][i] += p * vv[i];
    }
  }
#pragma unroll
  for (int h = 0; h < G; ++h)
#pragma unroll
    for (int i = 0; i < 8; ++i) red[(size_t)slot * G * D + h * D + dd + i] = acc[h][i];
  __syncthreads();
  for (int e = t; e < G * D; e += 256) {
    float o = 0.f;
    for (int sl = 0; sl < slots; ++sl) o += red[(size_t)sl * G * D + e];
    const int h = e / D, d = e % D;
    const int hq = kvh * G + h;
    const size_t pidx = ((size_t)m * a.n_split + split) * a.Hq + hq;
    a.part_o[pidx * D + d] = o;
    if (d == 0) {
      a.part_ml[pidx * 2] = ml_s[2 * h];
      a.part_ml[pidx * 2 + 1] = ml_s[2 * h + 1];
    }
  }
}

// merge the context chunks of one (token, q-head): one wave, lanes over D
__global__ __launch_bounds__(256) void attn_combine_kernel(AttnArgs a) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (gw >= a.M * a.Hq) return;
  const int m = gw / a.Hq, hq = gw % a.Hq;
  const int s = m % a.S;
  const int ctx = *a.pos_base + s + 1;
  const int nu = min(a.n_split, (ctx + a.CH - 1) / a.CH);
  float M = -INFINITY;
  for (int sp = 0; sp < nu; ++sp) M = fmaxf(M, a.part_ml[(((size_t)m * a.n_split + sp) * a.Hq + hq) * 2]);
  float L = 0.f;
  float o0 = 0.f, o1 = 0.f;
  const int D = a.D;
  for (int sp = 0; sp < nu; ++sp) {
    const size_t pidx = ((size_t)m * a.n_split + sp) * a.Hq + hq;
    const float ms = a.part_ml[pidx * 2];
    const float w = (ms == -INFINITY) ? 0.f : expf(ms - M);
    L += w * a.part_ml[pidx * 2 + 1];
    if (2 * lane < D) {
      o0 += w * a.part_o[pidx * D + 2 * lane];
      o1 += w * a.part_o[pidx * D + 2 * lane + 1];
    }
  }
  const float inv = L > 0.f ? 1.0f / L : 0.f;
  if (2 * lane < D) {
    bf16_t* dst = a.out + (size_t)m * a.Hq * D + (size_t)hq * D + 2 * lane;
    *reinterpret_cast<uint32_t*>(dst) = pack2(o0 * inv, o1 * inv);
  }
}

size_t attn_smem_bytes(int G, int D, int CH) {
  const int LPK = D / 8;
  const int slots = 256 / LPK;
  size_t f = (size_t)G * D + (size_t)G * CH + 2 * G + 2;
  f = (f + 3) & ~(size_t)3;
  return (f + (size_t)slots * G * D) * sizeof(float);
}

hipError_t attention(const AttnArgs& a0, hipStream_t st) {
  AttnArgs a = a0;
  const int G = a.Hq / a.Hkv;
  if (a.Hq % a.Hkv || a.D % 8 || a.D > 128 || a.CH % 64) return hipErrorInvalidValue;
  // red must start 16B aligned: attn_smem_bytes rounds the prefix; mirror it in the kernel
  const size_t sm = attn_smem_bytes(G, a.D, a.CH);
  dim3 grid(a.n_split, a.Hkv, a.M);
  switch (G) {
    case 1: hipLaunchKernelGGL(attn_kernel<1>, grid, dim3(256), sm, st, a); break;
    case 2: hipLaunchKernelGGL(attn_kernel<2>, grid, dim3(256), sm, st, a); break;
    case 4: hipLaunchKernelGGL(attn_kernel<4>, grid, dim3(256), sm, st, a); break;
    case 8: hipLaunchKernelGGL(attn_kernel<8>, grid, dim3(256), sm, st, a); break;
    default: return hipErrorInvalidValue;
  }
  const int waves = a.M * a.Hq;
  hipLaunchKernelGGL(attn_combine_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, a);
  return hipGetLastError();
}

}  // namespace mtts
