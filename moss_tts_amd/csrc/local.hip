// Device kernels of the MossTTSLocal depth stage (moss_tts_local/modeling_moss_tts.py):
// MossTTSRMSNorm in bf16, greedy channel argmax, and the per-frame stop/append state machine
// of CustomMixin._sample (:377-456).  The projections and the depth transformer reuse the
// GEMV / decode-attention kernels of the backbone.
#include "kernels.h"

namespace mtts {

// MossTTSRMSNorm (:34-44) WITHOUT the fp32 upcast of Qwen3RMSNorm: every torch op rounds to
// bf16.  norm = mean(bf16(x*x)) (fp32 accumulation, rounded), r = bf16(rsqrt(bf16(norm+eps))),
// y = bf16(bf16(x*r) * w).  One block per row, 16-byte chunks.
__global__ __launch_bounds__(256) void moss_rmsnorm_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w,
                                                           bf16_t* __restrict__ y, int H, float eps) {
  __shared__ float red[4];
  const int m = blockIdx.x, t = threadIdx.x;
  const bf16_t* xr = x + (size_t)m * H;
  float s = 0.f;
  for (int c = t; c < (H >> 3); c += 256) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += rbf(v[i] * v[i]);
  }
  s = wave_sum(s);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  const float tot = (red[0] + red[1]) + (red[2] + red[3]);
  const float norm = rbf(tot / (float)H);
  const float r = rbf(1.0f / sqrtf(rbf(norm + eps)));
  for (int c = t; c < (H >> 3); c += 256) {
    float v[8], g[8], q[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
    unpack8(*reinterpret_cast<const uint4*>(w + c * 8), g);
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = rbf(v[i] * r) * g[i];
    uint4 o;
    o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
    *reinterpret_cast<uint4*>(y + (size_t)m * H + c * 8) = o;
  }
}

hipError_t moss_rmsnorm(const bf16_t* x, const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s) {
  if (H % 8 || M <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(moss_rmsnorm_kernel, dim3(M), dim3(256), 0, s, x, w, y, H, eps);
  return hipGetLastError();
}

// torch.argmax over one logits row (first index among equal maxima), one block per row
__global__ __launch_bounds__(1024) void argmax_rows_kernel(const bf16_t* __restrict__ logits, int ld, int V,
                                                           int64_t* __restrict__ out, int ld_out) {
  __shared__ ArgMax sh[16];
  const int b = blockIdx.x, t = threadIdx.x;
  const bf16_t* row = logits + (size_t)b * ld;
  ArgMax a{-INFINITY, 0x7fffffff};
  const int nv = V >> 3;
  if ((ld & 7) == 0) {
    for (int c = t; c < nv; c += 1024) {
      float v[8];
      unpack8(*reinterpret_cast<const uint4*>(row + c * 8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) a = am_better(a, ArgMax{v[i], c * 8 + i});
    }
    for (int i = nv * 8 + t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
  } else {
    for (int i = t; i < V; i += 1024) a = am_better(a, ArgMax{bf2f(row[i]), i});
  }
  a = wave_argmax(a);
  if ((t & 63) == 0) sh[t >> 6] = a;
  __syncthreads();
  if (t == 0) {
    ArgMax r = sh[0];
    for (int i = 1; i < 16; ++i) r = am_better(r, sh[i]);
    out[(size_t)b * ld_out] = r.i == 0x7fffffff ? 0 : r.i;
  }
}

hipError_t argmax_rows(const bf16_t* logits, int ld, int V, int64_t* out, int ld_out, int B, hipStream_t s) {
  if (B <= 0 || V <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(argmax_rows_kernel, dim3(B), dim3(1024), 0, s, logits, ld, V, out, ld_out);
  return hipGetLastError();
}

// prompt rows into the generation buffer and the backbone key mask; rows start unfinished
__global__ void local_init_kernel(const int64_t* __restrict__ ids, const uint8_t* __restrict__ mask_in, int T, int C,
                                  int64_t* __restrict__ gen_ids, int Ltot, uint8_t* __restrict__ mask, int Cmax,
                                  int* __restrict__ finished) {
  const int b = blockIdx.x;
  for (int i = threadIdx.x; i < T * C; i += blockDim.x)
    gen_ids[(size_t)b * Ltot * C + i] = ids[(size_t)b * T * C + i];
  for (int t = threadIdx.x; t < Cmax; t += blockDim.x)
    mask[(size_t)b * Cmax + t] = t < T ? (mask_in ? mask_in[(size_t)b * T + t] : (uint8_t)1) : (uint8_t)0;
  if (threadIdx.x == 0) finished[b] = 0;
}

hipError_t local_init(const int64_t* ids, const uint8_t* mask_in, int B, int T, int C, int64_t* gen_ids, int Ltot,
                      uint8_t* mask, int Cmax, int* finished, hipStream_t s) {
  hipLaunchKernelGGL(local_init_kernel, dim3(B), dim3(256), 0, s, ids, mask_in, T, C, gen_ids, Ltot, mask, Cmax, finished);
  return hipGetLastError();
}

// End of a frame (:425-446): channels >= n_ch are 0; finished rows emit eos / pad; the frame
// is appended at column T0 + step and unmasked for the next forward; a row finishes on eos
// in channel 0.  One block, a thread per row.
__global__ __launch_bounds__(256) void local_finalize_kernel(GenDev* st, int64_t* __restrict__ next, int* __restrict__ finished,
                                                             int64_t* __restrict__ gen_ids, uint8_t* __restrict__ mask,
                                                             int B, int C, int n_ch, int eos, int pad) {
  __shared__ int alive;
  const int b = threadIdx.x;
  if (b == 0) alive = 0;
  __syncthreads();
  const int step = st->step, col = st->T0 + step;
  if (b < B) {
    const int fin = finished[b];
    int64_t* row = next + (size_t)b * C;
    int64_t* g = gen_ids + ((size_t)b * st->Ltot + col) * C;
    for (int i = 0; i < C; ++i) {
      int64_t v = i < n_ch ? row[i] : 0;
      if (fin) v = i == 0 ? eos : pad;
      row[i] = v;
      g[i] = v;
    }
    mask[(size_t)b * st->Cmax + col] = 1;
    const int f = fin | (row[0] == eos);
    finished[b] = f;
    if (!f) atomicOr(&alive, 1);
  }
  __syncthreads();
  if (b == 0) {
    if (!alive && st->done_step < 0) st->done_step = step;
    st->fwd_pos = col;
    st->step = step + 1;
  }
}

hipError_t local_finalize(GenDev* st, int64_t* next, int* finished, int64_t* gen_ids, uint8_t* mask, int B, int C,
                          int n_ch, int eos, int pad, hipStream_t s) {
  if (B <= 0 || B > 256) return hipErrorInvalidValue;
  hipLaunchKernelGGL(local_finalize_kernel, dim3(1), dim3(256), 0, s, st, next, finished, gen_ids, mask, B, C, n_ch, eos,
                     pad);
  return hipGetLastError();
}

}  // namespace mtts
