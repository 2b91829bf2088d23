// Codec decoder kernels (MOSS-Audio-Tokenizer decode side, codec.cpp):
//   rvq_dequant   residual-vector dequantisation: x[m] = sum_q table_q[code[m][q]]
//                 (each quantizer's output projection folded into its table), fp32 sum
//                 in quantizer order, one bf16 rounding, plus the per-16-column sums of
//                 squares the first decoder layer's fused RMSNorm reads
//   sumsq16       those sums for a tensor produced by a plain GEMM (the upsampling
//                 projection between stages)
//   patch_out     the last stage's tokens -> fp32 waveform patches (x . W^T, W stored
//                 transposed so a block's threads read consecutive samples of one k)
//   fill_int      a device int (stage positions) set from a kernel argument
#include "kernels.h"

namespace mtts {

// one block per token row, one thread per 8 columns (D <= 2048)
// token row m = b * F + t reads codes[b * ld_b + t * ld_codes + q]
__global__ __launch_bounds__(256) void rvq_dequant_kernel(const int64_t* __restrict__ codes, int ld_codes, size_t ld_b,
                                                          int F, int n_q, const bf16_t* __restrict__ tables, int cb,
                                                          int D, bf16_t* __restrict__ x, float* __restrict__ ss) {
  const int m = blockIdx.x, c = threadIdx.x;
  const int b = m / F, t = m - b * F;
  const int C8 = D / 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C8) {
    const int64_t* cm = codes + (size_t)b * ld_b + (size_t)t * ld_codes;
    for (int q = 0; q < n_q; ++q) {
      int64_t code = cm[q];
      code = code < 0 ? 0 : (code >= cb ? cb - 1 : code);
      const uint4 v = *reinterpret_cast<const uint4*>(tables + ((size_t)q * cb + code) * D + c * 8);
      float f[8];
      unpack8(v, f);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += f[i];
    }
  }
  float sq = 0.f;
  uint4 o;
  o.x = pack2(acc[0], acc[1]); o.y = pack2(acc[2], acc[3]); o.z = pack2(acc[4], acc[5]); o.w = pack2(acc[6], acc[7]);
  if (c < C8) {
    float r[8];
    unpack8(o, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) sq += r[i] * r[i];
    *reinterpret_cast<uint4*>(x + (size_t)m * D + c * 8) = o;
  }
  sq += __shfl_xor(sq, 1, 64);  // the two 8-column halves of a 16-column tile
  if (c < C8 && !(c & 1)) ss[(size_t)m * (D / 16) + c / 2] = sq;
}

__global__ __launch_bounds__(256) void sumsq16_kernel(const bf16_t* __restrict__ x, int H, int M, float* __restrict__ ss) {
  const int NT = H / 16;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (size_t)M * NT) return;
  const size_t m = i / NT, t = i % NT;
  const uint4* p = reinterpret_cast<const uint4*>(x + m * H + t * 16);
  float f[8], s = 0.f;
  unpack8(p[0], f);
#pragma unroll
  for (int k = 0; k < 8; ++k) s += f[k] * f[k];
  unpack8(p[1], f);
#pragma unroll
  for (int k = 0; k < 8; ++k) s += f[k] * f[k];
  ss[i] = s;
}

// PT token rows per block staged in LDS; thread p < patch accumulates PT outputs over k
constexpr int PATCH_PT = 8;
__global__ __launch_bounds__(256) void patch_out_kernel(const bf16_t* __restrict__ x, int M, int K,
                                                        const bf16_t* __restrict__ wt, int patch, float* __restrict__ wav,
                                                        int S, size_t ld_wav, size_t off0) {
  extern __shared__ float xs_f[];  // [PATCH_PT][K]
  const int m0 = blockIdx.x * PATCH_PT;
  for (int i = threadIdx.x; i < PATCH_PT * K; i += 256) {
    const int r = i / K, k = i - r * K;
    xs_f[i] = m0 + r < M ? bf2f(x[(size_t)(m0 + r) * K + k]) : 0.f;
  }
  __syncthreads();
  for (int p = threadIdx.x; p < patch; p += 256) {
    float acc[PATCH_PT];
#pragma unroll
    for (int r = 0; r < PATCH_PT; ++r) acc[r] = 0.f;
    for (int k = 0; k < K; ++k) {
      const float w = bf2f(wt[(size_t)k * patch + p]);
#pragma unroll
      for (int r = 0; r < PATCH_PT; ++r) acc[r] = fmaf(xs_f[r * K + k], w, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < PATCH_PT; ++r) {
      const int m = m0 + r;
      if (m >= M) break;
      const int b = m / S, n = m - b * S;
      wav[(size_t)b * ld_wav + off0 + (size_t)n * patch + p] = acc[r];
    }
  }
}

__global__ void fill_int_kernel(int* p, int v) { *p = v; }

hipError_t rvq_dequant(const int64_t* codes, int ld_codes, size_t ld_b, int F, int n_q, const bf16_t* tables, int cb,
                       int D, bf16_t* x, float* ss, int M, hipStream_t s) {
  if (D % 16 || D / 8 > 256 || M <= 0 || n_q <= 0 || F <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rvq_dequant_kernel, dim3(M), dim3(256), 0, s, codes, ld_codes, ld_b, F, n_q, tables, cb, D, x, ss);
  return hipGetLastError();
}

hipError_t sumsq16(const bf16_t* x, int H, int M, float* ss, hipStream_t s) {
  if (H % 16 || M <= 0) return hipErrorInvalidValue;
  const size_t n = (size_t)M * (H / 16);
  hipLaunchKernelGGL(sumsq16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, H, M, ss);
  return hipGetLastError();
}

hipError_t patch_out(const bf16_t* x, int M, int K, const bf16_t* wt, int patch, float* wav, int S, size_t ld_wav,
                     size_t off0, hipStream_t s) {
  const size_t lds = (size_t)PATCH_PT * K * sizeof(float);
  if (M <= 0 || S <= 0 || lds > 64 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(patch_out_kernel, dim3((M + PATCH_PT - 1) / PATCH_PT), dim3(256), lds, s, x, M, K, wt, patch, wav, S,
                     ld_wav, off0);
  return hipGetLastError();
}

hipError_t fill_int(int* p, int v, hipStream_t s) {
  hipLaunchKernelGGL(fill_int_kernel, dim3(1), dim3(1), 0, s, p, v);
  return hipGetLastError();
}

}  // namespace mtts
