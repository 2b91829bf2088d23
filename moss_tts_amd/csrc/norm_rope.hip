// Embedding sum, RMSNorm, q/k-norm + RoPE + KV-cache append.
#include "kernels.h"

namespace mtts {

// ---------------------------------------------------------------------------
// h[m, :] = E_text[ids[m,0]] + E_0[ids[m,1]] + ... + E_{n-1}[ids[m,n]], each add rounded to
// bf16 left to right (moss_tts_delay/modeling_moss_tts.py:196-213).
// Grid (M, H/256): a block gathers the C embedding slices of its 256 columns into LDS with
// every 16-byte load in flight at once, then each thread sums one column in channel order.
// It also emits the sum of squares of every 16-column tile for the next RMSNorm.
constexpr int EMB_COLS = 256, EMB_MAXC = 64;
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, int C, const bf16_t* __restrict__ emb_text,
                                                    const bf16_t* __restrict__ emb_audio, int audio_rows, int H,
                                                    bf16_t* __restrict__ h, float* __restrict__ ss_out, int ld_ss,
                                                    int ld_ids) {
  constexpr int LPT = (EMB_MAXC * EMB_COLS / 8 + 255) / 256;  // 16-byte loads per thread (max)
  __shared__ __attribute__((aligned(16))) bf16_t rows_s[EMB_MAXC][EMB_COLS];
  __shared__ int64_t id_s[EMB_MAXC];
  const int m = blockIdx.x, c0 = blockIdx.y * EMB_COLS, t = threadIdx.x;
  if (t < C) id_s[t] = ids[(size_t)m * ld_ids + t];
  __syncthreads();
  const int ncols = min(EMB_COLS, H - c0);
  const int cpr = ncols >> 3;
  const int n = C * cpr;
  uint4 v[LPT];
#pragma unroll
  for (int u = 0; u < LPT; ++u) {
    const int i = t + u * 256;
    if (i < n) {
      const int j = i / cpr, cc = i - j * cpr;
      const bf16_t* src = j == 0 ? emb_text + (size_t)id_s[0] * H : emb_audio + ((size_t)(j - 1) * audio_rows + id_s[j]) * H;
      v[u] = *reinterpret_cast<const uint4*>(src + c0 + cc * 8);
    }
  }
#pragma unroll
  for (int u = 0; u < LPT; ++u) {
    const int i = t + u * 256;
    if (i < n) {
      const int j = i / cpr, cc = i - j * cpr;
      *reinterpret_cast<uint4*>(&rows_s[j][cc * 8]) = v[u];
    }
  }
  __syncthreads();
  float e = 0.f;
  if (t < ncols) {
    e = bf2f(rows_s[0][t]);
    for (int j = 1; j < C; ++j) e = rbf(e + bf2f(rows_s[j][t]));
    h[(size_t)m * H + c0 + t] = f2bf(e);
  }
  float ss = e * e;
  ss += __shfl_xor(ss, 1, 64);
  ss += __shfl_xor(ss, 2, 64);
  ss += __shfl_xor(ss, 4, 64);
  ss += __shfl_xor(ss, 8, 64);
  if (ss_out && t < ncols && (t & 15) == 0) ss_out[(size_t)m * ld_ss + ((c0 + t) >> 4)] = ss;
}

// ---------------------------------------------------------------------------
// Qwen3RMSNorm (TF/models/qwen3/modeling_qwen3.py:59-64): fp32 statistics,
// y = bf16(w * bf16(x * rsqrt(mean(x^2) + eps))).  One block per row.
// Row m of the input is x + x_off + m * x_stride (lets the heads pick the last token).
__global__ __launch_bounds__(256) void rmsnorm_kernel(const bf16_t* __restrict__ x, size_t x_off, size_t x_stride,
                                                      const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int H,
                                                      float eps) {
  const int m = blockIdx.x;
  const bf16_t* xr = x + x_off + (size_t)m * x_stride;
  const int nchunk = H >> 3;
  float ss = 0.f;
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float v[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) ss += v[i] * v[i];
  }
  __shared__ float part[4];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = ss;
  __syncthreads();
  const float tot = ((part[0] + part[1]) + part[2]) + part[3];
  const float r = 1.0f / sqrtf(tot / (float)H + eps);
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    float v[8], g[8];
    unpack8(*reinterpret_cast<const uint4*>(xr + c * 8), v);
    unpack8(*reinterpret_cast<const uint4*>(w + c * 8), g);
    uint4 o;
    float q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = rbf(g[i] * rbf(v[i] * r));
    o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
    *reinterpret_cast<uint4*>(y + (size_t)m * H + c * 8) = o;
  }
}

// ---------------------------------------------------------------------------
// Single-pass Qwen3RMSNorm from the producer's per-16-column sums of squares (written by
// the residual-add GEMV epilogue or the embedding kernel): every wave reduces the row's
// H/16 partials itself (one float4 per lane), so there is no block-wide reduction and x
// is read once.  Block = H/8 threads (one 16-byte chunk each), one block per row.
__global__ __launch_bounds__(512) void rmsnorm_ss_kernel(const bf16_t* __restrict__ x, size_t x_off, size_t x_stride,
                                                         const float* __restrict__ ss, size_t ss_off, size_t ss_stride,
                                                         const bf16_t* __restrict__ w, bf16_t* __restrict__ y, int H,
                                                         float eps, int y_tiles) {
  const int m = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int c = threadIdx.x;
  const bf16_t* xr = x + x_off + (size_t)m * x_stride;
  uint4 xv = make_uint4(0, 0, 0, 0), wv = make_uint4(0, 0, 0, 0);
  const bool ok = c < (H >> 3);
  if (ok) {
    xv = *reinterpret_cast<const uint4*>(xr + c * 8);
    wv = *reinterpret_cast<const uint4*>(w + c * 8);
  }
  const float* sp = ss + ss_off + (size_t)m * ss_stride;
  float s = 0.f;
  for (int t4 = lane * 4; t4 < (H >> 4); t4 += 256) {
    const float4 v = *reinterpret_cast<const float4*>(sp + t4);
    s += (v.x + v.y) + (v.z + v.w);
  }
  s = wave_sum(s);
  const float r = 1.0f / sqrtf(s / (float)H + eps);
  if (!ok) return;
  float v[8], g[8], q[8];
  unpack8(xv, v);
  unpack8(wv, g);
#pragma unroll
  for (int i = 0; i < 8; ++i) q[i] = g[i] * rbf(v[i] * r);
  uint4 o;
  o.x = pack2(q[0], q[1]); o.y = pack2(q[2], q[3]); o.z = pack2(q[4], q[5]); o.w = pack2(q[6], q[7]);
  *reinterpret_cast<uint4*>(y + (y_tiles ? xpkT_index(m, c * 8, y_tiles) : (size_t)m * H + c * 8)) = o;
}

hipError_t rmsnorm_ss(const bf16_t* x, size_t x_off, size_t x_stride, const float* ss, size_t ss_off, size_t ss_stride,
                      const bf16_t* w, bf16_t* y, int M, int H, float eps, hipStream_t s, int y_tiles) {
  if (H % 16 || H > 4096) return hipErrorInvalidValue;  // one 16-byte chunk per thread, <= 512 threads
  if (y_tiles && (M > 16 * y_tiles || H % 32)) return hipErrorInvalidValue;
  const int threads = ((H / 8 + 63) / 64) * 64;
  hipLaunchKernelGGL(rmsnorm_ss_kernel, dim3(M), dim3(threads < 64 ? 64 : threads), 0, s, x, x_off, x_stride, ss,
                     ss_off, ss_stride, w, y, H, eps, y_tiles);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-head q_norm / k_norm (TF/.../modeling_qwen3.py:252-254), RoPE in bf16
// (:148-170, cos/sin from a bf16 table computed in fp32, :126-137) and the KV
// cache append (DynamicLayer.update, TF/cache_utils.py:127-145) as an in-place
// write at the token's absolute position.
//
// qkv   [M, (Hq + 2 Hkv) * D] (bf16, output of the fused q|k|v GEMV)
// q_out [M, Hq * D]
// cache k/v: [Bmax][Hkv][Cmax][D] per layer; token m = b*S + s sits at position pos0[b?] + s
// One wave per (token, head); D <= 128, each lane holds dims 2l, 2l+1.

__global__ __launch_bounds__(256) void qk_norm_rope_kernel(QKRopeArgs a) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);  // global wave = (token, head)
  const int heads = a.Hq + 2 * a.Hkv;
  if (gw >= a.M * heads) return;
  const int m = gw / heads;
  const int hd = gw % heads;
  const int b = m / a.S, s = m % a.S;
  const int pos = *a.pos_base + s;
  const int rpos = a.rope_off ? max(0, pos - a.rope_off[b]) : pos;  // RoPE position (cache slot: pos)
  const int D = a.D;
  const bool act = 2 * lane < D;
  const bf16_t* src = a.qkv + (size_t)m * heads * D + (size_t)hd * D;
  float x0 = 0.f, x1 = 0.f;
  if (act) {
    const uint32_t pr = *reinterpret_cast<const uint32_t*>(src + 2 * lane);
    x0 = __uint_as_float(pr << 16);
    x1 = __uint_as_float(pr & 0xffff0000u);
  }
  if (hd >= a.Hq + a.Hkv) {  // V head: copy into the cache
    const int kvh = hd - a.Hq - a.Hkv;
    if (act) {  // V cache is stored transposed: [Hkv][D][Cmax]
      bf16_t* dst = a.vc + ((size_t)b * a.Hkv + kvh) * D * a.Cmax + pos;
      dst[(size_t)(2 * lane) * a.Cmax] = f2bf(x0);
      dst[(size_t)(2 * lane + 1) * a.Cmax] = f2bf(x1);
    }
    return;
  }
  const bool isq = hd < a.Hq;
  const bf16_t* nw = isq ? a.qn_w : a.kn_w;
  // RMSNorm over D in fp32
  float ss = wave_sum(x0 * x0 + x1 * x1);
  const float r = 1.0f / sqrtf(ss / (float)D + a.eps);
  float w0 = 0.f, w1 = 0.f;
  if (act) {
    const uint32_t pw = *reinterpret_cast<const uint32_t*>(nw + 2 * lane);
    w0 = __uint_as_float(pw << 16);
    w1 = __uint_as_float(pw & 0xffff0000u);
  }
  const float n0 = rbf(w0 * rbf(x0 * r));
  const float n1 = rbf(w1 * rbf(x1 * r));
  // rotate_half: dims d < D/2 take -x[d + D/2], dims >= D/2 take x[d - D/2]; partner lane = lane +- D/4
  const int q4 = D >> 2;
  const int partner = (2 * lane < D / 2) ? lane + q4 : lane - q4;
  const float p0 = __shfl(n0, partner, 64);
  const float p1 = __shfl(n1, partner, 64);
  const float sg = (2 * lane < D / 2) ? -1.f : 1.f;
  float c0 = 0.f, c1 = 0.f, s0 = 0.f, s1 = 0.f;
  if (act) {
    const uint32_t pc = *reinterpret_cast<const uint32_t*>(a.cos_t + (size_t)rpos * D + 2 * lane);
    const uint32_t ps = *reinterpret_cast<const uint32_t*>(a.sin_t + (size_t)rpos * D + 2 * lane);
    c0 = __uint_as_float(pc << 16); c1 = __uint_as_float(pc & 0xffff0000u);
    s0 = __uint_as_float(ps << 16); s1 = __uint_as_float(ps & 0xffff0000u);
  }
  const float o0 = rbf(rbf(n0 * c0) + rbf(sg * p0 * s0));
  const float o1 = rbf(rbf(n1 * c1) + rbf(sg * p1 * s1));
  if (!act) return;
  if (isq) {
    bf16_t* dst = a.q_out + (size_t)m * a.Hq * D + (size_t)hd * D;
    *reinterpret_cast<uint32_t*>(dst + 2 * lane) = pack2(o0, o1);
  } else {
    const int kvh = hd - a.Hq;
    bf16_t* dst = a.kc + (((size_t)b * a.Hkv + kvh) * a.Cmax + pos) * D;
    *reinterpret_cast<uint32_t*>(dst + 2 * lane) = pack2(o0, o1);
  }
}

hipError_t embed(const int64_t* ids, int C, const bf16_t* emb_text, const bf16_t* emb_audio, int audio_rows, int H,
                 bf16_t* h, int M, hipStream_t s, float* ss_out, int ld_ss, int ld_ids) {
  if (H % 16 || C < 1 || C > EMB_MAXC) return hipErrorInvalidValue;
  if (ld_ids <= 0) ld_ids = C;
  hipLaunchKernelGGL(embed_kernel, dim3(M, (H + EMB_COLS - 1) / EMB_COLS), dim3(256), 0, s, ids, C, emb_text, emb_audio,
                     audio_rows, H, h, ss_out, ld_ss, ld_ids);
  return hipGetLastError();
}

hipError_t rmsnorm(const bf16_t* x, size_t x_off, size_t x_stride, const bf16_t* w, bf16_t* y, int M, int H, float eps,
                   hipStream_t s) {
  if (H % 8) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rmsnorm_kernel, dim3(M), dim3(256), 0, s, x, x_off, x_stride, w, y, H, eps);
  return hipGetLastError();
}

hipError_t qk_norm_rope(const QKRopeArgs& a, hipStream_t s) {
  if (a.D > 128 || a.D % 4) return hipErrorInvalidValue;
  const int waves = a.M * (a.Hq + 2 * a.Hkv);
  hipLaunchKernelGGL(qk_norm_rope_kernel, dim3((waves + 3) / 4), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace mtts
