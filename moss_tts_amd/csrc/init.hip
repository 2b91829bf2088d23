// Deterministic weight fill (benchmarks / tests): the device twin of oracle/prng.py.
//   z = splitmix64(seed * GOLDEN + (tensor_id << 40) + i);  u = (z >> 40) * 2^-24
//   val = bf16(offset + scale * (2u - 1))      (two fp32 roundings, no FMA contraction)
#include "kernels.h"

namespace mtts {

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long x) {
  unsigned long long z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_uniform_kernel(bf16_t* dst, size_t n, unsigned long long seed, unsigned long long tid, float scale,
                                    float offset) {
  const unsigned long long base = seed * 0x9E3779B97F4A7C15ull + (tid << 40);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const unsigned long long z = splitmix64(base + i);
    const float u = (float)(z >> 40) * (1.0f / 16777216.0f);
    const float t = __fmul_rn(scale, __fsub_rn(__fmul_rn(2.0f, u), 1.0f));
    dst[i] = f2bf(__fadd_rn(offset, t));
  }
}

hipError_t fill_uniform_bf16(bf16_t* dst, size_t n, unsigned long long seed, unsigned long long tensor_id, float scale,
                             float offset, hipStream_t s) {
  const int blocks = (int)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(fill_uniform_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, dst, n, seed, tensor_id,
                     scale, offset);
  return hipGetLastError();
}

}  // namespace mtts
